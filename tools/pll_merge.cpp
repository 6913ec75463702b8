// tools/pll_merge.cpp — can one stream's PLL (src/filter.cpp:136-174) be run in parallel in
// time?  A time-parallel exact scheme would start segment k speculatively W steps early, at
// t_k - W, from a guessed state, and keep its output once its float state bit-merges with the
// true trajectory.  This measures whether and where such restarts merge, on the reference's
// own arithmetic (float state, glibc double atan2 / cos / sin, filter.cpp:157-171).
//
//   pll_merge <carrier.f32> <freq> <fs> <restarts> <max_steps> <saturated 0|1>
//
// saturated = 1 starts the true run with trigOffset = 2^24 (where the reference's float
// trigOffset sticks: from 69.9 s of signal on at 240 kS/s), so the regime after saturation is
// measured without 70 s of input.  For each of `restarts` start points t (spread over the
// input) and each guess -- zero state (integ = phase = 0, fb = (1, 0)), stale state (the true
// state one window earlier, the previous segment's estimate), and the true state with the
// phase 1 ulp off -- the guessed run is stepped next to the truth for up to max_steps and the
// first step at which (integ, phase, fbI, fbQ) are bit-identical is recorded.  Prints one JSON
// line: per guess, the merge count within 10^3, 10^4, 10^5 and max_steps, and the integrator /
// phase gaps left at the end of the unmerged runs.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

struct St {
    float integ, phase, fbI, fbQ, trig;
};

// one step of filter.cpp:157-171, the reference's types and promotions (PI as a double)
inline void step(St& s, float v, float Ki, float Kp, double w) {
    const float eI = v * s.fbI, eQ = v * (-s.fbQ);
    const float e = (float)std::atan2((double)eQ, (double)eI);
    s.integ = s.integ + Ki * e;
    s.phase = s.phase + ((Kp * e) + s.integ);
    s.trig = s.trig + 1.0f;
    const float arg = (float)(w * (double)s.trig + (double)s.phase);
    s.fbI = (float)std::cos((double)arg);
    s.fbQ = (float)std::sin((double)arg);
}

inline bool same(const St& a, const St& b) {
    return std::memcmp(&a, &b, sizeof(St)) == 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: pll_merge carrier.f32 freq fs restarts max_steps saturated\n");
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<float> x;
    float buf[4096];
    size_t n;
    while ((n = std::fread(buf, 4, 4096, f)) > 0) x.insert(x.end(), buf, buf + n);
    std::fclose(f);
    const float freq = (float)std::atof(argv[2]), fs = (float)std::atof(argv[3]);
    const int restarts = std::atoi(argv[4]);
    const long max_steps = std::atol(argv[5]);
    const bool sat = std::atoi(argv[6]) != 0;
    // project.cpp:166 PLL(carrier, 19000, if_fs, 2, 0, 0.01, ...): Kp, Ki as filter.cpp:141-144
    const float nb = 0.01f;
    const float Kp = nb * (float)2.666, Ki = nb * nb * (float)3.555;
    const double w = 2 * 3.14159265358979323846 * (double)(freq / fs);
    const size_t N = x.size();
    // the true trajectory: state after every step
    std::vector<St> tr(N + 1);
    tr[0] = St{0.0f, 0.0f, 1.0f, 0.0f, sat ? 16777216.0f : 0.0f};
    for (size_t i = 0; i < N; i++) {
        tr[i + 1] = tr[i];
        step(tr[i + 1], x[i], Ki, Kp, w);
    }
    const char* names[3] = {"zero", "stale", "phase_1ulp"};
    const long marks[4] = {1000, 10000, 100000, max_steps};
    std::printf("{\"input_steps\": %zu, \"saturated_trigOffset\": %s, \"restarts\": %d, \"max_steps\": %ld",
                N, sat ? "true" : "false", restarts, max_steps);
    for (int g = 0; g < 3; g++) {
        long merged[4] = {0, 0, 0, 0};
        double gap_i = 0, gap_p = 0;
        int unmerged = 0;
        long first_sum = 0;
        int first_n = 0;
        for (int r = 0; r < restarts; r++) {
            // start points spread over [max_steps, N - max_steps): a window of history in front
            const size_t span = N > (size_t)(2 * max_steps) ? N - 2 * (size_t)max_steps : 1;
            const size_t t = (size_t)max_steps + span * (size_t)r / (size_t)restarts;
            St s = tr[t];
            if (g == 0) {
                s.integ = 0.0f;
                s.phase = 0.0f;
                s.fbI = 1.0f;
                s.fbQ = 0.0f;
            } else if (g == 1) {
                const St old = tr[t - (size_t)max_steps / 2];
                s.integ = old.integ;
                s.phase = old.phase;
                s.fbI = old.fbI;
                s.fbQ = old.fbQ;
            } else {
                s.phase = std::nextafterf(s.phase, INFINITY);
            }
            long k = 0;
            bool ok = false;
            for (; k < max_steps && t + (size_t)k < N; k++) {
                if (same(s, tr[t + (size_t)k])) {
                    ok = true;
                    break;
                }
                step(s, x[t + (size_t)k], Ki, Kp, w);
            }
            if (!ok && t + (size_t)k <= N && same(s, tr[t + (size_t)k])) ok = true;
            if (ok) {
                for (int m = 0; m < 4; m++)
                    if (k <= marks[m]) merged[m]++;
                first_sum += k;
                first_n++;
            } else {
                const St& tt = tr[t + (size_t)k];
                gap_i += std::fabs((double)s.integ - (double)tt.integ);
                gap_p += std::fabs(std::remainder((double)s.phase - (double)tt.phase, 2 * M_PI));
                unmerged++;
            }
        }
        std::printf(", \"%s\": {\"merged_within_1e3\": %ld, \"merged_within_1e4\": %ld, \"merged_within_1e5\": %ld, "
                    "\"merged_within_max\": %ld, \"mean_merge_step\": %.1f, \"unmerged\": %d, "
                    "\"mean_integ_gap_unmerged\": %.3g, \"mean_phase_gap_unmerged_mod_2pi\": %.3g}",
                    names[g], merged[0], merged[1], merged[2], merged[3],
                    first_n ? (double)first_sum / first_n : -1.0, unmerged, unmerged ? gap_i / unmerged : 0.0,
                    unmerged ? gap_p / unmerged : 0.0);
    }
    std::printf("}\n");
    return 0;
}
