// tools/pll_predict.cpp — can the unsaturated PLL's trigArg be predicted ahead of the serial
// chain?  The reference's step (src/filter.cpp:157-171: float state, glibc double atan2 / cos /
// sin) over a carrier file (the carrier band-pass output, float32), for every step before
// trigOffset sticks at 2^24:
//
//   trigArg_j = float(P_j + phase_j),  P_j = 2 pi (f/Fs) trigOffset_j in double.
//
// A candidate for trigArg_j formed from an EARLIER phase, float(P_j + phase_s) with s the last
// step of the previous batch (batches of B steps), is off by k_j float ulps; if |k_j| <= 1 for
// nearly every step, lanes could evaluate the feedback (sin, cos, atan2 offset) of the 3
// candidates of every step of a batch in parallel and the serial step would only select
// (pll_sat.hip's pattern for the stuck trigOffset).  Prints, per range of j and batch size, the
// fraction of steps with |k| = 0, <= 1, <= 2, and the fraction of batches whose every step has
// |k| <= 1 (B = 1: the previous step's phase).  A lookback of lb batches takes the phase at the
// end of batch b - lb instead (lb = 2: batch b + 1's candidates can be evaluated during batch b).
//
//   g++ -O2 -ffp-contract=off -o /tmp/pll_predict tools/pll_predict.cpp
//   pll_predict <carrier.f32> [lookback]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

static long ulps_between(float a, float b) {  // signed distance in floats, a and b same sign region
    if (a == b) return 0;
    long n = 0;
    float t = a;
    const float dir = b > a ? INFINITY : -INFINITY;
    while (t != b && n < 1000) {
        t = std::nextafter(t, dir);
        n++;
    }
    return b > a ? n : -n;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: pll_predict carrier.f32\n");
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<float> x;
    float buf[4096];
    size_t n;
    while ((n = std::fread(buf, 4, 4096, f)) > 0) x.insert(x.end(), buf, buf + n);
    std::fclose(f);
    const float nb = 0.01f;
    const float Kp = nb * (float)2.666, Ki = nb * nb * (float)3.555;
    const double w = 2 * 3.14159265358979323846 * (double)(19000.0f / 240000.0f);
    const size_t N = x.size();  // steps from 2^24 on: trigOffset stuck (pll_sat.hip's regime)
    std::vector<float> phase(N), arg(N), integs(N);
    float integ = 0, ph = 0, fbI = 1, fbQ = 0, trig = 0;
    for (size_t i = 0; i < N; i++) {
        const float eI = x[i] * fbI, eQ = x[i] * (-fbQ);
        const float e = (float)std::atan2((double)eQ, (double)eI);
        integ = integ + Ki * e;
        ph = ph + ((Kp * e) + integ);
        trig = trig + 1.0f;
        const float a = (float)(w * (double)trig + (double)ph);
        phase[i] = ph;
        integs[i] = integ;
        arg[i] = a;
        fbI = (float)std::cos((double)a);
        fbQ = (float)std::sin((double)a);
    }
    // ranges of j (step index = trigOffset - 1)
    const size_t edges[] = {0, 1u << 16, 1u << 20, 1u << 21, 1u << 22, 1u << 23, 1u << 24, N};
    const int batches[] = {1, 4, 8, 16, 32, 64, 128};
    // lookback: the candidate's phase is the one at the end of batch b - lb (lb = 1: the
    // previous batch; lb = 2 lets the candidates of batch b + 1 be evaluated during batch b)
    const int lb = argc > 2 ? std::atoi(argv[2]) : 1;
    std::printf("steps %zu (of %zu in the file), lookback %d batch(es)\n", N, x.size(), lb);
    float pmin = 1e30f, pmax = -1e30f;
    for (size_t i = 0; i < N; i++) {
        pmin = std::fmin(pmin, phase[i]);
        pmax = std::fmax(pmax, phase[i]);
    }
    std::printf("phase range [%g, %g]\n", pmin, pmax);
    std::printf("%-22s %5s %9s %9s %9s %9s %12s %12s\n", "j range", "B", "k=0", "|k|<=1", "|k|<=2", "|k|>2",
                "batch|k|<=1", "batch|k|<=2");
    for (int r = 0; r + 1 < 8; r++) {
        const size_t j0 = edges[r], j1 = std::min(edges[r + 1], N);
        if (j0 >= j1) continue;
        for (int B : batches) {
            long k0 = 0, k1 = 0, k2 = 0, kx = 0, nb_all = 0, nb_ok = 0, nb_ok2 = 0;
            for (size_t b0 = (j0 / B) * B; b0 < j1; b0 += B) {
                const size_t back = (size_t)(lb - 1) * B + 1;  // the last step of batch b - lb
                const float p0 = b0 >= back ? phase[b0 - back] : 0.0f;
                bool ok = true, ok2 = true;
                for (size_t j = b0; j < b0 + B && j < j1; j++) {
                    if (j < j0) continue;
                    const float cand = (float)(w * (double)std::min((float)(j + 1), 16777216.0f) + (double)p0);
                    const long k = std::labs(ulps_between(cand, arg[j]));
                    if (k == 0) k0++;
                    if (k <= 1) k1++;
                    if (k <= 2) k2++;
                    else kx++;
                    ok = ok && k <= 1;
                    ok2 = ok2 && k <= 2;
                }
                nb_all++;
                nb_ok += ok;
                nb_ok2 += ok2;
            }
            const double tot = (double)(j1 - j0);
            std::printf("[2^%-4.1f, 2^%-4.1f)     %5d %9.4f %9.4f %9.4f %9.4f %12.4f %12.4f\n",
                        j0 ? std::log2((double)j0) : 0.0, std::log2((double)j1), B, k0 / tot, k1 / tot, k2 / tot,
                        kx / tot, (double)nb_ok / nb_all, (double)nb_ok2 / nb_all);
        }
    }
    // two candidates: c0 and its neighbour on the side of the exact sum P + phase_ref (the
    // rounding's direction), batches of B with lookback lb
    std::printf("two candidates (c0 and the neighbour towards P + phase_ref):\n");
    for (int r = 2; r + 1 < 8; r++) {
        const size_t j0 = edges[r], j1 = std::min(edges[r + 1], N);
        if (j0 >= j1) continue;
        for (int B : {8, 16, 32, 64}) {
            long hit = 0, nb_all = 0, nb_ok = 0;
            for (size_t b0 = (j0 / B) * B; b0 < j1; b0 += B) {
                const size_t back = (size_t)(lb - 1) * B + 1;
                const float p0 = b0 >= back ? phase[b0 - back] : 0.0f;
                bool ok = true;
                for (size_t j = b0; j < b0 + B && j < j1; j++) {
                    const double sum = w * (double)std::min((float)(j + 1), 16777216.0f) + (double)p0;
                    const float c0 = (float)sum;
                    const float c1 = std::nextafter(c0, sum > (double)c0 ? INFINITY : -INFINITY);
                    const bool h = arg[j] == c0 || arg[j] == c1;
                    hit += h;
                    ok = ok && h;
                }
                nb_all++;
                nb_ok += ok;
            }
            std::printf("[2^%-4.1f, 2^%-4.1f)     %5d  step hit %.4f  batch hit %.4f\n", std::log2((double)j0),
                        std::log2((double)j1), B, (double)hit / (double)(j1 - j0), (double)nb_ok / nb_all);
        }
    }
    // the candidates centred on an extrapolated phase: phase_ref + integ_ref (j - s) (the phase
    // moves by about integ a step, filter.cpp:161-162), s the step of the reference state; the
    // fraction of B-step batches whose every step is within m floats of that centre
    std::printf("B-step batches within m floats of the extrapolated centre, lookback %d:\n", lb);
    const int mx[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 12, 16};
    std::printf("%-22s %s\n", "j range", "m = 0 1 2 3 4 5 6 7 8 12 16");
    for (int B : {16, 32, 64})
    for (int e = 17; e < 25; e++) {
        const size_t j0 = (size_t)1 << e, j1 = std::min(e == 24 ? N : ((size_t)1 << (e + 1)), N);
        if (j0 >= j1) continue;
        long nb_all = 0, ok[11] = {}, okc[11] = {};
        for (size_t b0 = j0; b0 + B <= j1; b0 += B) {
            const size_t back = (size_t)(lb - 1) * B + 1;
            const size_t sref = b0 - back;
            const float p0 = phase[sref], i0 = integs[sref];
            long kmax = 0, kmaxc = 0;
            for (size_t j = b0; j < b0 + B; j++) {
                const double pr = w * (double)std::min((float)(j + 1), 16777216.0f);
                const float cand = (float)(pr + (double)p0 + (double)i0 * (double)(j - sref));
                kmax = std::max(kmax, std::labs(ulps_between(cand, arg[j])));
                const float cand0 = (float)(pr + (double)p0);
                kmaxc = std::max(kmaxc, std::labs(ulps_between(cand0, arg[j])));
            }
            nb_all++;
            for (int q = 0; q < 11; q++) {
                ok[q] += kmax <= mx[q];
                okc[q] += kmaxc <= mx[q];
            }
        }
        std::printf("[2^%d, 2^%d)  B=%-3d extrap", e, e + 1, B);
        for (int q = 0; q < 11; q++) std::printf(" %.4f", (double)ok[q] / nb_all);
        std::printf("\n                    plain ");
        for (int q = 0; q < 11; q++) std::printf(" %.4f", (double)okc[q] / nb_all);
        std::printf("\n");
    }
    // past the stick (trigOffset 2^24: one constant P, trigArg on a 1-rad grid): the fraction of
    // B-step batches whose trigArgs are all one float (one candidate for the whole batch), and the
    // mean run of one trigArg
    if (N > (1u << 24) + 4096) {
        std::printf("past the stick: B-step batches with one trigArg throughout\n");
        for (int B : {8, 16, 32, 64, 128, 256}) {
            long nb_all = 0, one = 0;
            for (size_t b0 = (size_t)1 << 24; b0 + B <= N; b0 += B) {
                bool same = true;
                for (size_t j = b0 + 1; j < b0 + B; j++) same = same && arg[j] == arg[b0];
                nb_all++;
                one += same;
            }
            std::printf("  B=%-4d %.4f of %ld\n", B, (double)one / nb_all, nb_all);
        }
        long runs = 0;
        for (size_t j = ((size_t)1 << 24) + 1; j < N; j++) runs += arg[j] != arg[j - 1];
        std::printf("  trigArg changes %ld in %zu steps: mean run %.1f steps\n", runs, N - ((size_t)1 << 24),
                    (double)(N - ((size_t)1 << 24)) / (double)(runs + 1));
    }
    // below 2^22: fraction of B-step batches whose every step is within m floats of c0 (2m + 1
    // candidates), per octave of j -- how many candidates a chain would need there
    const int ms[] = {1, 2, 3, 4, 6, 8, 12, 16, 24, 31};
    std::printf("B-step batches within m floats of c0 (2m + 1 candidates), lookback %d:\n", lb);
    std::printf("%-22s %s\n", "j range", "m = 1 2 3 4 6 8 12 16 24 31");
    for (int B : {8, 16, 32, 64})
    for (int e = 14; e < 22; e++) {
        const size_t j0 = (size_t)1 << e, j1 = std::min((size_t)1 << (e + 1), N);
        if (j0 >= j1) continue;
        long nb_all = 0, ok[10] = {};
        for (size_t b0 = j0; b0 + B <= j1; b0 += B) {
            const size_t back = (size_t)(lb - 1) * B + 1;
            const float p0 = phase[b0 - back];
            long kmax = 0;
            for (size_t j = b0; j < b0 + B; j++) {
                const float cand = (float)(w * (double)(float)(j + 1) + (double)p0);
                kmax = std::max(kmax, std::labs(ulps_between(cand, arg[j])));
            }
            nb_all++;
            for (int q = 0; q < 10; q++) ok[q] += kmax <= ms[q];
        }
        std::printf("[2^%d, 2^%d)  B=%-3d     ", e, e + 1, B);
        for (int q = 0; q < 10; q++) std::printf(" %.4f", (double)ok[q] / nb_all);
        std::printf("\n");
    }
    return 0;
}
