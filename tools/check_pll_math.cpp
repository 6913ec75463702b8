// tools/check_pll_math.cpp — validate csrc/pll_math.h against glibc on the host.
//
// For every tested argument where the fast path claims a certain float result, that result
// must equal float(glibc(x)) — the value the reference's PLL uses (src/filter.cpp:161-170).
// Modes:
//   sincos <lo> <hi> <stride>   every `stride`-th float in [lo, hi] (both signs)
//   atan2  <n> <seed>           n random float pairs from several distributions
//   rot    <n> <seed>           the PLL's rotation atan2 (rot_atan2_f): n random (trigArg x,
//                               sample v) pairs, context from sincos_ctx_f(x), fb = glibc's
//                               float cos/sin of x, checked against glibc atan2(eQ, eI)
// Prints counts: checked, fast-path hits, fallbacks, MISMATCHES (must be 0).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../software-defined-radio-course-project_amd/csrc/pll_math.h"

static float bits2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static uint32_t f2bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

struct Count { unsigned long long n = 0, fast = 0, fb = 0, fb2 = 0, bad = 0; };

static uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage\n"); return 2; }
    const int T = std::thread::hardware_concurrency() ? (int)std::thread::hardware_concurrency() : 4;
    std::vector<Count> cnt(T);
    std::vector<std::thread> th;
    if (!std::strcmp(argv[1], "sincos")) {
        const float lo = std::atof(argv[2]), hi = std::atof(argv[3]);
        const uint32_t stride = (uint32_t)std::atoll(argv[4]);
        const uint32_t b0 = f2bits(lo), b1 = f2bits(hi);
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                Count& c = cnt[t];
                for (uint64_t b = b0 + (uint64_t)t * stride; b <= b1; b += (uint64_t)T * stride) {
                    for (int sg = 0; sg < 2; sg++) {
                        const float x = sg ? -bits2f((uint32_t)b) : bits2f((uint32_t)b);
                        float s, co;
                        c.n++;
                        if (fmrx::fast_sincos_f(x, &s, &co)) {
                            c.fast++;
                            const float gs = (float)std::sin((double)x), gc = (float)std::cos((double)x);
                            if (f2bits(s) != f2bits(gs) || f2bits(co) != f2bits(gc)) {
                                if (c.bad < 5) std::printf("MISMATCH sincos x=%.9g fast=(%.9g,%.9g) glibc=(%.9g,%.9g)\n", x, s, co, gs, gc);
                                c.bad++;
                            }
                        } else {
                            c.fb++;
                        }
                        // the cosine alone (fast_cos_f, the NCO): certified => glibc's float
                        float c1;
                        if (fmrx::fast_cos_f(x, &c1) && f2bits(c1) != f2bits((float)std::cos((double)x))) {
                            if (c.bad < 5) std::printf("MISMATCH cos x=%.9g fast=%.9g\n", x, c1);
                            c.bad++;
                        }
                        // the PLL's own path (context-producing sincos, integer certification)
                        fmrx::PllCtx ctx{};
                        float s2, c2;
                        if (fmrx::sincos_ctx_f(x, &s2, &c2, &ctx)) {
                            const float gs = (float)std::sin((double)x), gc = (float)std::cos((double)x);
                            if (f2bits(s2) != f2bits(gs) || f2bits(c2) != f2bits(gc)) {
                                if (c.bad < 5) std::printf("MISMATCH sincos_ctx x=%.9g fast=(%.9g,%.9g) glibc=(%.9g,%.9g)\n", x, s2, c2, gs, gc);
                                c.bad++;
                            }
                        } else {
                            c.fb2++;
                        }
                    }
                }
            });
    } else if (!std::strcmp(argv[1], "rot")) {
        const unsigned long long n = std::atoll(argv[2]);
        const uint64_t seed = std::atoll(argv[3]);
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                Count& c = cnt[t];
                for (unsigned long long i = t; i < n; i += T) {
                    const uint64_t h = sm64(seed * 0x7654321ull + i), h2 = sm64(h);
                    float x;
                    switch (h % 4) {
                        case 0: x = (float)((int32_t)h) * 4.0e-3f; break;                      // |x| < 8.6e6
                        case 1: x = (float)((int32_t)h) * 1.0e-9f; break;                      // |x| < 2.2
                        case 2: x = (float)((double)((int32_t)(h >> 8) >> 8) * 1.5707963267948966 +
                                             (double)((int32_t)h2) * 1e-14); break;            // near k pi/2
                        default: x = bits2f((uint32_t)(h >> 32) & 0x4EFFFFFFu) * ((h & 8) ? -1.0f : 1.0f); break;
                    }
                    float v;
                    switch (h2 % 3) {
                        case 0: v = (float)((int32_t)(h2 >> 16)) * 2.3e-11f; break;
                        case 1: v = (float)((int32_t)(h2 >> 16)) * 1.7e-3f; break;
                        default: v = bits2f((uint32_t)(h2 >> 32)); break;                     // any bits
                    }
                    if (std::isnan(v) || std::isinf(v)) continue;
                    fmrx::PllCtx ctx{};
                    float s2, c2;
                    fmrx::sincos_ctx_f(x, &s2, &c2, &ctx);
                    const float fbI = (float)std::cos((double)x), fbQ = (float)std::sin((double)x);
                    const float eI = v * fbI, eQ = v * (-fbQ);
                    float a;
                    c.n++;
                    if (fmrx::rot_atan2_f(eQ, eI, ctx, &a)) {
                        c.fast++;
                        const float g = (float)std::atan2((double)eQ, (double)eI);
                        if (f2bits(a) != f2bits(g)) {
                            if (c.bad < 5) std::printf("MISMATCH rot x=%.9g v=%.9g fast=%.9g glibc=%.9g\n", x, v, a, g);
                            c.bad++;
                        }
                    } else {
                        c.fb++;
                    }
                }
            });
    } else {
        const unsigned long long n = std::atoll(argv[2]);
        const uint64_t seed = std::atoll(argv[3]);
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                Count& c = cnt[t];
                for (unsigned long long i = t; i < n; i += T) {
                    const uint64_t h = sm64(seed * 0x1234567ull + i);
                    float y, x;
                    switch (h % 4) {
                        case 0: y = bits2f((uint32_t)h); x = bits2f((uint32_t)(h >> 32)); break;  // any bits
                        case 1: y = (float)((int32_t)h) * 1e-9f; x = (float)((int32_t)(h >> 32)) * 1e-9f; break;
                        case 2: { // PLL-like: v * fb, v small, |fb| <= 1
                            const float v = (float)((int32_t)h) * 2.3e-11f;
                            const float ph = (float)((h >> 32) & 0xFFFFFF) * 3.7e-7f;
                            y = v * -(float)std::sin(ph); x = v * (float)std::cos(ph); break; }
                        default: y = (float)((int32_t)h) * 1e-3f; x = (float)(h >> 40) * 1e-20f; break;  // near-axis
                    }
                    if (std::isnan(y) || std::isnan(x)) continue;
                    float a;
                    c.n++;
                    if (fmrx::fast_atan2_f(y, x, &a)) {
                        c.fast++;
                        const float g = (float)std::atan2((double)y, (double)x);
                        if (f2bits(a) != f2bits(g)) {
                            if (c.bad < 5) std::printf("MISMATCH atan2 y=%.9g x=%.9g fast=%.9g glibc=%.9g\n", y, x, a, g);
                            c.bad++;
                        }
                    } else {
                        c.fb++;
                    }
                }
            });
    }
    for (auto& t : th) t.join();
    Count s;
    for (auto& c : cnt) { s.n += c.n; s.fast += c.fast; s.fb += c.fb; s.fb2 += c.fb2; s.bad += c.bad; }
    std::printf("%s checked=%llu fast=%llu fallback=%llu ctx_fallback=%llu mismatches=%llu\n", argv[1], s.n, s.fast,
                s.fb, s.fb2, s.bad);
    return s.bad ? 1 : 0;
}
