// tools/check_pll_run.cpp — run the whole PLL recurrence (src/filter.cpp:136-174) two ways on
// the host and require bit-identical output: (a) the reference's arithmetic with glibc's
// double atan2/cos/sin, (b) csrc/pll_math.h's pll_step (certified fast paths + glibc
// fallbacks), (c) pll_kernel's schedule: side data per chunk (pll_side, as pll_prep_kernel),
// 16-sample pll_batch_fast batches, a batch redone with pll_step when it cannot be certified,
// the tail with pll_step -- the GPU's arithmetic.
// Usage: check_pll_run <carrier.f32> <freq> <fs> [chunk] [split=1]   (state carried across chunks)
#include <cmath>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../software-defined-radio-course-project_amd/csrc/pll_math.h"

struct GlibcLib {
    float atan2f_(float y, float x) const {
        float e;
        if (fmrx::fast_atan2_f(y, x, &e)) return e;
        return (float)std::atan2((double)y, (double)x);
    }
    void sincosf_(float a, float* s, float* c) const {
        *s = (float)std::sin((double)a);
        *c = (float)std::cos((double)a);
    }
};

int main(int argc, char** argv) {
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<float> x;
    float buf[4096];
    size_t n;
    while ((n = std::fread(buf, 4, 4096, f)) > 0) x.insert(x.end(), buf, buf + n);
    std::fclose(f);
    const float freq = std::atof(argv[2]), fs = std::atof(argv[3]);
    const size_t chunk = argc > 4 ? std::atol(argv[4]) : x.size();
    // the GPU runs the split sin/cos form up to 4 streams per wave, the fdlibm form beyond
    const bool split = argc > 5 ? std::atoi(argv[5]) != 0 : true;
    const float Kp = 0.01f * (float)2.666, Ki = (0.01f * 0.01f) * (float)3.555;
    const double step = (2.0 * 3.14159265358979323846) * (double)(freq / fs);
    // (a) reference arithmetic
    float integ = 0, phase = 0, fbI = 1, fbQ = 0, trig = 0;
    std::vector<float> ref(x.size());
    for (size_t i = 0; i < x.size(); i++) {
        const float eI = x[i] * fbI, eQ = x[i] * (-fbQ);
        const float e = (float)std::atan2((double)eQ, (double)eI);
        integ = integ + Ki * e;
        phase = phase + ((Kp * e) + integ);
        trig = trig + 1.0f;
        const float arg = (float)(step * (double)trig + (double)phase);
        fbI = (float)std::cos((double)arg);
        fbQ = (float)std::sin((double)arg);
        ref[i] = (float)std::cos((double)(arg * 2.0f + 0.0f));
    }
    // (b) pll_step, context reset at every chunk boundary like a new GPU call
    fmrx::PllState p{0, 0, 1, 0, 0};
    GlibcLib lib;
    size_t bad = 0;
    for (size_t c0 = 0; c0 < x.size(); c0 += chunk) {
        fmrx::PllCtx ctx{};
        ctx.valid = false;
        for (size_t i = c0; i < std::min(x.size(), c0 + chunk); i++) {
            const float arg = fmrx::pll_step(p, ctx, x[i], Ki, Kp, step, lib);
            const float nco = (float)std::cos((double)(arg * 2.0f + 0.0f));
            if (std::memcmp(&nco, &ref[i], 4) != 0) {
                if (bad < 5) std::printf("MISMATCH at %zu: %.9g vs %.9g\n", i, nco, ref[i]);
                bad++;
            }
        }
    }
    bool state_ok = p.integ == integ && p.phase == phase && p.fbI == fbI && p.fbQ == fbQ && p.trig == trig;
    // (c) batches as in pll_kernel
    constexpr int NB = 16;
    fmrx::PllState pb{0, 0, 1, 0, 0};
    size_t bad_c = 0, batches = 0, redone = 0;
    for (size_t c0 = 0; c0 < x.size(); c0 += chunk) {
        fmrx::PllCtx ctx{};
        ctx.valid = false;
        const size_t c1 = std::min(x.size(), c0 + chunk);
        std::vector<float> out(c1 - c0);
        size_t i = c0;
        // side data of the chunk, as pll_prep_kernel computes it from the entering trigOffset
        std::vector<double> iv(c1 - c0), pr(c1 - c0);
        for (size_t k = c0; k < c1; k++)
            fmrx::pll_side(x[k], pb.trig, (long long)(k - c0), step, &iv[k - c0], &pr[k - c0]);
        for (; i + NB <= c1; i += NB) {
            float v[NB], o[NB];
            double bi[NB], bp[NB];
            std::memcpy(v, &x[i], sizeof v);
            std::memcpy(bi, &iv[i - c0], sizeof bi);
            std::memcpy(bp, &pr[i - c0], sizeof bp);
            const fmrx::PllState p0 = pb;
            const fmrx::PllCtx ctx0 = ctx;
            batches++;
            if (!(split ? fmrx::pll_batch_fast<NB, true>(pb, ctx, v, bi, bp, o, Ki, Kp, [](int) {})
                        : fmrx::pll_batch_fast<NB, false>(pb, ctx, v, bi, bp, o, Ki, Kp, [](int) {}))) {
                redone++;
                pb = p0;
                ctx = ctx0;
                for (int j = 0; j < NB; j++) o[j] = fmrx::pll_step(pb, ctx, v[j], Ki, Kp, step, lib);
            }
            std::memcpy(&out[i - c0], o, sizeof o);
        }
        for (; i < c1; i++) out[i - c0] = fmrx::pll_step(pb, ctx, x[i], Ki, Kp, step, lib);
        for (size_t k = c0; k < c1; k++) {
            const float nco = (float)std::cos((double)(out[k - c0] * 2.0f + 0.0f));
            if (std::memcmp(&nco, &ref[k], 4) != 0) {
                if (bad_c < 5) std::printf("MISMATCH (batch) at %zu: %.9g vs %.9g\n", k, nco, ref[k]);
                bad_c++;
            }
        }
    }
    state_ok = state_ok && pb.integ == integ && pb.phase == phase && pb.fbI == fbI && pb.fbQ == fbQ && pb.trig == trig;
    std::printf("batches=%zu redone=%zu\n", batches, redone);
    std::printf("samples=%zu mismatches=%zu state_equal=%d\n", x.size(), bad + bad_c, (int)state_ok);
    return (bad || bad_c || !state_ok) ? 1 : 0;
}
