// tools/check_pll_run.cpp — run the whole PLL recurrence (src/filter.cpp:136-174) two ways on
// the host and require bit-identical output: (a) the reference's arithmetic with glibc's
// double atan2/cos/sin, (b) csrc/pll_math.h's pll_step (certified fast paths + the device's
// pll_cr.h fallbacks), (c) pll_kernel's schedule: side data per chunk (pll_side, as pll_prep_kernel),
// 16-sample pll_batch_fast batches, a batch redone with pll_step when it cannot be certified,
// the tail with pll_step -- the GPU's arithmetic.
// Usage: check_pll_run <carrier.f32> <freq> <fs> [chunk] [split=1]   (state carried across chunks)
#include <cmath>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../software-defined-radio-course-project_amd/csrc/pll_cr.h"
#include "../software-defined-radio-course-project_amd/csrc/pll_math.h"

// the fallbacks exactly as the device's DeviceLib (csrc/stereo.hip): fdlibm atan2, then the
// double-double pll_cr.h evaluations; glibc only beyond the cr domain (as the device's ocml)
struct GlibcLib {
    float atan2f_(float y, float x) const {
        float e;
        if (fmrx::fast_atan2_f(y, x, &e)) return e;
        return fmrx::cr::atan2_f(y, x);
    }
    void sincosf_(float a, float* s, float* c) const {
        if (!fmrx::cr::sincos_domain(a)) {
            *s = (float)std::sin((double)a);
            *c = (float)std::cos((double)a);
            return;
        }
        fmrx::cr::sincos_f(a, s, c);
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
    // (d) the speculative launch (stereo.hip pll_spec_kernel / pll_check_kernel / pll_kernel
    // with fail): the runner's uncertified batches with their (integ, phase) records, every
    // batch rechecked with pll_step from the record before it, the certified path resumed at
    // the first batch that differs, then the tail
    fmrx::PllState ps{0, 0, 1, 0, 0};
    size_t bad_d = 0, chunks = 0, chunks_failed = 0, batches_resumed = 0;
    for (size_t c0 = 0; c0 < x.size(); c0 += chunk) {
        const size_t c1 = std::min(x.size(), c0 + chunk), m = c1 - c0, nb = m / NB;
        std::vector<double> iv(m), pr(m);
        for (size_t k = c0; k < c1; k++) fmrx::pll_side(x[k], ps.trig, (long long)(k - c0), step, &iv[k - c0], &pr[k - c0]);
        std::vector<float> out(m);
        std::vector<std::pair<float, float>> rec(nb);
        const fmrx::PllState s0 = ps;
        {  // runner
            fmrx::PllState p = s0;
            fmrx::PllCtx ctx{};
            ctx.valid = false;
            if (nb > 0) {  // batch 0 exactly
                for (int j = 0; j < NB; j++) out[j] = fmrx::pll_step(p, ctx, x[c0 + j], Ki, Kp, step, lib);
                rec[0] = {p.integ, p.phase};
            }
            for (size_t b = 1; b < nb; b++) {
                float v[NB], o[NB];
                double bi[NB], bp[NB];
                std::memcpy(v, &x[c0 + b * NB], sizeof v);
                std::memcpy(bi, &iv[b * NB], sizeof bi);
                std::memcpy(bp, &pr[b * NB], sizeof bp);
                double hh[NB];  // the pre-pass's half turns
                for (int j = 0; j < NB; j++) hh[j] = bi[j] < 0.0 ? 0.5 : 0.0;
                if (split) fmrx::pll_batch_fast<NB, true, true>(p, ctx, v, bi, bp, o, Ki, Kp, [](int) {}, {}, hh);
                else fmrx::pll_batch_fast<NB, false, true>(p, ctx, v, bi, bp, o, Ki, Kp, [](int) {}, {}, hh);
                std::memcpy(&out[b * NB], o, sizeof o);
                rec[b] = {p.integ, p.phase};
            }
        }
        size_t fail = nb;  // checker
        for (size_t b = 0; b < nb; b++) {
            fmrx::PllState p = s0;
            fmrx::PllCtx ctx{};
            ctx.valid = false;
            if (!fmrx::pll_trig_domain(s0.trig)) { fail = 0; break; }
            if (b > 0) fmrx::pll_state_at(p, ctx, rec[b - 1].first, rec[b - 1].second, s0.trig, (long long)(b * NB), out[b * NB - 1], lib);
            bool same = true;
            for (int j = 0; j < NB; j++) {
                const float a = fmrx::pll_step(p, ctx, x[c0 + b * NB + j], Ki, Kp, step, lib);
                same = same && std::memcmp(&a, &out[b * NB + j], 4) == 0;
            }
            same = same && std::memcmp(&p.integ, &rec[b].first, 4) == 0 && std::memcmp(&p.phase, &rec[b].second, 4) == 0;
            if (!same) {
                if (std::getenv("PLL_SPEC_VERBOSE")) std::printf("chunk at %zu: batch %zu of %zu differs\n", c0, b, nb);
                fail = b;
                break;
            }
        }
        chunks++;
        if (fail < nb) chunks_failed++;
        batches_resumed += nb - fail;
        {  // fix-up from batch `fail` on the certified path
            fmrx::PllState p = s0;
            fmrx::PllCtx ctx{};
            ctx.valid = false;
            if (fail > 0) fmrx::pll_state_at(p, ctx, rec[fail - 1].first, rec[fail - 1].second, s0.trig, (long long)(fail * NB), out[fail * NB - 1], lib);
            size_t i = fail * NB;
            for (; i + NB <= m; i += NB) {
                float v[NB], o[NB];
                double bi[NB], bp[NB];
                std::memcpy(v, &x[c0 + i], sizeof v);
                std::memcpy(bi, &iv[i], sizeof bi);
                std::memcpy(bp, &pr[i], sizeof bp);
                const fmrx::PllState p0 = p;
                const fmrx::PllCtx ctx0 = ctx;
                if (!(split ? fmrx::pll_batch_fast<NB, true>(p, ctx, v, bi, bp, o, Ki, Kp, [](int) {})
                            : fmrx::pll_batch_fast<NB, false>(p, ctx, v, bi, bp, o, Ki, Kp, [](int) {}))) {
                    p = p0;
                    ctx = ctx0;
                    for (int j = 0; j < NB; j++) o[j] = fmrx::pll_step(p, ctx, v[j], Ki, Kp, step, lib);
                }
                std::memcpy(&out[i], o, sizeof o);
            }
            for (; i < m; i++) out[i] = fmrx::pll_step(p, ctx, x[c0 + i], Ki, Kp, step, lib);
            ps = p;
        }
        for (size_t k = c0; k < c1; k++) {
            const float nco = (float)std::cos((double)(out[k - c0] * 2.0f + 0.0f));
            if (std::memcmp(&nco, &ref[k], 4) != 0) {
                if (bad_d < 5) std::printf("MISMATCH (speculative) at %zu: %.9g vs %.9g\n", k, nco, ref[k]);
                bad_d++;
            }
        }
    }
    state_ok = state_ok && ps.integ == integ && ps.phase == phase && ps.fbI == fbI && ps.fbQ == fbQ && ps.trig == trig;
    std::printf("speculative: chunks=%zu failed=%zu batches_resumed=%zu\n", chunks, chunks_failed, batches_resumed);
    bad_c += bad_d;
    std::printf("batches=%zu redone=%zu\n", batches, redone);
    std::printf("samples=%zu mismatches=%zu state_equal=%d\n", x.size(), bad + bad_c, (int)state_ok);
    return (bad || bad_c || !state_ok) ? 1 : 0;
}
