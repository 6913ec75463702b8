// tools/pll_runs.cpp — how often does the stereo PLL's trigArg move once trigOffset has stuck at
// 2^24 (src/filter.cpp:165-166), and in what runs?  The reference's step (filter.cpp:157-171,
// glibc double atan2 / cos / sin, float state) over a carrier file (the oracle's carrier
// band-pass output, float32), counting after `skip` steps: the fraction of steps whose trigArg
// differs from the previous one, and the histogram of the distances between such steps.
// pll_sat.hip's design (batch-parallel pairs, refresh on a move) rests on these numbers.
//
//   g++ -O2 -ffp-contract=off -o /tmp/pll_runs tools/pll_runs.cpp
//   pll_runs <carrier.f32> <skip>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: pll_runs carrier.f32 skip\n");
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<float> x;
    float buf[4096];
    size_t n;
    while ((n = std::fread(buf, 4, 4096, f)) > 0) x.insert(x.end(), buf, buf + n);
    std::fclose(f);
    const long skip = std::atol(argv[2]);
    // project.cpp:166 PLL(carrier, 19000, 240000, 2, 0, 0.01, ...): Kp, Ki as filter.cpp:141-144
    const float nb = 0.01f;
    const float Kp = nb * (float)2.666, Ki = nb * nb * (float)3.555;
    const double w = 2 * 3.14159265358979323846 * (double)(19000.0f / 240000.0f);
    float integ = 0, phase = 0, fbI = 1, fbQ = 0, trig = 0, prev = NAN;
    long changes = 0, last = 0;
    std::vector<long> hist(65, 0);
    for (size_t i = 0; i < x.size(); i++) {
        const float eI = x[i] * fbI, eQ = x[i] * (-fbQ);
        const float e = (float)std::atan2((double)eQ, (double)eI);
        integ = integ + Ki * e;
        phase = phase + ((Kp * e) + integ);
        trig = trig + 1.0f;
        const float arg = (float)(w * (double)trig + (double)phase);
        if ((long)i >= skip && arg != prev) {
            changes++;
            const long L = (long)i - last;
            hist[L < 64 ? L : 64]++;
            last = (long)i;
        }
        if ((long)i < skip) last = (long)i;
        prev = arg;
        fbI = (float)std::cos((double)arg);
        fbQ = (float)std::sin((double)arg);
    }
    const long counted = (long)x.size() > skip ? (long)x.size() - skip : 0;
    std::printf("steps_counted %ld moves %ld fraction %.4f\nrun length: count (cumulative fraction)\n", counted,
                changes, counted ? (double)changes / counted : 0.0);
    long acc = 0;
    for (int L = 1; L <= 64; L++) {
        acc += hist[L];
        if (hist[L]) std::printf("%s%d: %ld (%.3f)\n", L == 64 ? ">=" : "", L, hist[L], (double)acc / changes);
    }
    return 0;
}
