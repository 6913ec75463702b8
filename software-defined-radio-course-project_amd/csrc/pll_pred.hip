// pll_pred.hip — the speculative PLL runner with predicted trigArgs (src/filter.cpp:157-171) for
// segments from trigOffset 2^20 on, the 2^24 stick included; streams by 16-lane row (spw <= 4),
// like pll_spec_lane_kernel.
//
// trigArg_j = float(P_j + phase_j) with P_j = 2 pi (f/Fs) trigOffset_j in double (pll_side's pr).
// From 2^20 steps on, P_j's float grid is 2^-5 rad or coarser (2^-2 from 2^22, 1 once trigOffset
// has stuck) while the phase moves by |Kp e + integ| < 0.05 rad a step and stays within a few
// radians: a candidate formed ahead of the chain from an EARLIER phase, c0 = float(P_j +
// phase_ref), is within one float of the true trigArg on 99 % of the steps below 2^22 and on
// every step of the bench stream from there on (tools/pll_predict.cpp, phase_ref from two batches
// back).  So the feedback of a step -- sin, cos and the atan2 offset of trigArg_j,
// which the NEXT step's error e needs -- need not wait for the serial chain.
//
// Two waves per workgroup (one group of spw streams; the two land on different SIMDs of the CU,
// tools/ubench_wgsimd.hip, profiles/r03/ubench_wgsimd.txt):
//   wave 1 (the evaluator) computes, for every step l of batch b + 1, the next step's error e for
//     the three candidates c0 - 1, c0, c0 + 1 ulp (lane l of a row; phase_ref = the phase at the
//     start of batch b; with one stream the four rows split the three candidates and the rest),
//     and stores them, the thresholds float(S) >= c of two candidates as doubles (thr_of) and P_l
//     in LDS;
//   wave 0 (the chain) runs batch b from LDS: per step the candidate of trigArg_{j-1}, chosen by
//     comparing the double sum S_{j-1} = P + phase (before its rounding to float) with the two
//     thresholds, (Ki e, Kp e), integ += Ki e, phase += Kp e + integ, S_j = P_j + phase; trigArg
//     = float(S_j) off the chain.
// One barrier per batch; the chain's wave issues nothing else, so its step is the dependency
// chain itself.  A step whose trigArg is not a candidate sets the batch's miss flag: the chain
// redoes the batch from its start, evaluating such steps' e directly (uniform loads of the step's
// input, sin and cos in every lane).  The arithmetic of e is pll_spec_lane_kernel's (e =
// float(fma(Y, 1/v, B)), the same sin/cos polynomials and offsets), and the output -- trigArgs and
// the per-batch (integ, phase) records -- is checked by pll_check_kernel like every runner's, so
// the result is the certified path's bit for bit whatever was predicted.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "dsp_device.h"
#include "fmrx_internal.h"
#include "pll_device.h"
#include "pll_math.h"

namespace fmrx {

#ifdef FMRX_AB_PROF
// A/B build only (Makefile `ab`, AB=-DFMRX_AB_PROF): shader-clock cycles of the two waves, body vs
// barrier wait, summed over every batch and workgroup, printed at exit
__device__ unsigned long long g_pred_prof[6];
#define PROF_T() __builtin_amdgcn_s_memtime()
#else
#define PROF_T() 0ull
#endif

namespace {

// e of a step (input v, 1/v = iv, half turn h = 0.5 [v < 0]) whose previous trigArg is a:
// pll_spec_lane_kernel's step with both sin and cos in this lane.
__device__ inline float pred_e(float a, float v, double iv) {
    const double x = (double)a;
    const double nd = rint(x * kInvPio2);
    const double r = fma(-nd, kPio2Lo, fma(-nd, kPio2Hi, x));
    const double z = r * r;
    const double sn = r * split_w_horner(z, split_coef(false));
    const double cs = split_w_horner(z, split_coef(true));
    const float fc = (float)cs, nfs = -(float)sn;
    const float2v ab = float2v{fc, nfs} * v;
    const double Y = fma((double)ab.x, sn, (double)ab.y * cs);
    const double h = iv < 0.0 ? 0.5 : 0.0;
    const double B = pll_offset_h(x, h);
    return (float)fma(Y, iv, B);
}

// The smallest double S with float(S) >= c, for a positive float c given by its bits cb: the
// midpoint of c and its predecessor (exact in double), or the double just above it when the
// tie rounds down (ties to even: an odd c loses it).  trigArg = float(S) with S = P + phase in
// double, so float(S) >= c is S >= thr_of(c): the chain selects a candidate by comparing the
// double sum it forms anyway, without waiting for its rounding to float.
__device__ inline double thr_of(uint32_t cb) {
    const double m = 0.5 * ((double)__builtin_bit_cast(float, cb - 1u) + (double)__builtin_bit_cast(float, cb));
    return (cb & 1u) ? __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, m) + 1ull) : m;
}

template <int NB>
__global__ void __launch_bounds__(128) pll_pred_kernel(const float* io, int n, int n_streams, int spw, size_t stride,
                                                      const double* side, size_t seg, double step, float norm_bw,
                                                      const float* st, float* out_base, size_t ostride, int* fail,
                                                      float2* rec, size_t rb, int inject, int sat_ok) {
    // per step of the batch, double-buffered by batch parity: (e_m, e_0, e_p, bits of c0 - 1 ulp),
    // the thresholds (thr_of(c0), thr_of(c0 + 1 ulp)) and P
    __shared__ float4 cand[2][4][NB];
    __shared__ double2 thr[2][4][NB];
    __shared__ double prs_l[2][4][NB];
    __shared__ float ph[2][4];  // the phase at the start of batch k, slot k & 1
    const int t = threadIdx.x & 63;
    const bool chain = threadIdx.x < 64;
    const int q = (t >> 4) & (spw - 1);  // the row's stream in the group
    const int s_lane = blockIdx.x * spw + q;
    const bool owner = chain && (t & 15) == 0 && (t >> 4) < spw && s_lane < n_streams;
    const int s = s_lane < n_streams ? s_lane : n_streams - 1;
    const int l = t & 15;
    const float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    const float* S = st + 8 * (size_t)s;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    PllState p{S[0], S[1], S[2], S[3], S[5]};
    // both waves alike: the lane runner's waves, or the saturated runner's when it is launched
    if (!pll_pred_wave(p.trig, step) || (sat_ok && pll_sat_segment(spw, p.trig, step))) return;
    const int nb = n / NB;
    if (nb < 2) {  // batch 0 alone, exactly (no barrier is reached)
        if (chain) {
            if (owner) fail[s] = nb;
            if (nb > 0) {
                PllCtx ctx{};
                ctx.valid = false;
                const PllPair r = pll_redo(p, ctx, x, out, NB, Ki, Kp, step, s_lane < n_streams);
                if (owner) rec[(size_t)s * rb] = make_float2(r.p.integ, r.p.phase);
            }
        }
        return;
    }
    // side data, stream-major (pll_prep_major_kernel): 1/v and pr planes
    const double* ivs = side + (size_t)s * seg;
    const double* prs = side + seg * (size_t)n_streams + (size_t)s * seg;

    if (!chain) {
        // ---- the evaluator: batch b + 1's candidates during the chain's batch b
        // this lane's data for batch b: pr of step l, the input of step l + 1 (the step its e is
        // for; the segment's last sample stands in past the end)
        auto ld = [&](int b, float& v, double& iv, double& pr) {
            const int jn = min(b * NB + l + 1, n - 1);
            v = x[jn];
            iv = ivs[jn];
            pr = prs[b * NB + l];
        };
        auto put = [&](int b, float phase_ref, float v, double iv, double pr) {
            const float c0 = (float)(pr + (double)phase_ref);
            const uint32_t cb = __builtin_bit_cast(uint32_t, c0);
            // a candidate that is not a positive finite float: every trigArg misses it
            const uint32_t cmb = (c0 > 0.0f && c0 < 3.0e38f) ? cb - 1u : 0xFFFFFFFFu;
            if (spw == 1) {
                // one stream: its four rows share the work -- rows 0-2 the e of candidates
                // c0 - 1, c0, c0 + 1 ulp, row 3 the miss bits, thresholds and P
                const int r = t >> 4;
                float* slot = reinterpret_cast<float*>(&cand[b & 1][0][l]);
                if (r < 3) {
                    slot[r] = pred_e(__builtin_bit_cast(float, cb + (uint32_t)(r - 1)), v, iv);
                } else {
                    slot[3] = __builtin_bit_cast(float, cmb);
                    thr[b & 1][0][l] = make_double2(thr_of(cb), thr_of(cb + 1u));
                    prs_l[b & 1][0][l] = pr;
                }
                return;
            }
            const float em = pred_e(__builtin_bit_cast(float, cb - 1u), v, iv);
            const float e0 = pred_e(c0, v, iv);
            const float ep = pred_e(__builtin_bit_cast(float, cb + 1u), v, iv);
            if ((t >> 4) < spw) {
                cand[b & 1][q][l] = make_float4(em, e0, ep, __builtin_bit_cast(float, cmb));
                thr[b & 1][q][l] = make_double2(thr_of(cb), thr_of(cb + 1u));
                prs_l[b & 1][q][l] = pr;
            }
        };
        // ring of 4 batches of step data: batch k in slot k & 3, refilled right after its use,
        // so each load has ~3 batches to land
        float vq[4];
        double ivq[4], prq[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k = 1 + u;  // batches 1..4 in slots 1, 2, 3, 0
            ld(k < nb ? k : nb - 1, vq[k & 3], ivq[k & 3], prq[k & 3]);
        }
        // batch 1 from the phase at the start of batch 0: the initial state
        put(1, p.phase, vq[1], ivq[1], prq[1]);
        ld(5 < nb ? 5 : nb - 1, vq[1], ivq[1], prq[1]);
        __syncthreads();  // (prologue)
        unsigned long long ev_body = 0, ev_wait = 0;
        // iteration b: batch b + 1's candidates from the phase at the start of batch b; groups
        // of four iterations from b0 = 1 (mod 4), so the ring slots are compile-time
        for (int b0 = 1; b0 < nb; b0 += 4) {
            unroll_ic(
                [&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    constexpr int sl = (2 + u) & 3;  // slot of batch b + 1 = (b0 + u + 1) & 3
                    const int b = b0 + u;
                    if (b < nb) {
                        const unsigned long long p0 = PROF_T();
                        if (b + 1 < nb) {
                            put(b + 1, ph[b & 1][q], vq[sl], ivq[sl], prq[sl]);
                            const int bq = b + 5 < nb ? b + 5 : nb - 1;
                            ld(bq, vq[sl], ivq[sl], prq[sl]);
                        }
                        const unsigned long long p1 = PROF_T();
                        __syncthreads();
                        ev_body += p1 - p0;
                        ev_wait += PROF_T() - p1;
                    }
                },
                std::make_integer_sequence<int, 4>{});
        }
#ifdef FMRX_AB_PROF
        if (t == 0) {
            atomicAdd(&g_pred_prof[2], ev_body);
            atomicAdd(&g_pred_prof[3], ev_wait);
        }
#endif
        (void)ev_body;
        (void)ev_wait;
        return;
    }

    // ---- the chain
    if (owner) fail[s] = nb;
    PllCtx ctx{};
    ctx.valid = false;
    {  // batch 0 on the exact path (see pll_spec_kernel)
        const PllPair r = pll_redo(p, ctx, x, out, NB, Ki, Kp, step, s_lane < n_streams);
        p = r.p;
        ctx = r.ctx;
        if (owner) rec[(size_t)s * rb] = make_float2(p.integ, p.phase);
    }
    float integ = p.integ, phase = p.phase;
    // Sd: the double sum P + phase of the last step done (trigArg = float(Sd)); batch 0's last
    // trigArg comes from the exact path, where only its float is known -- the carry's three
    // slots are alike, so the selection does not depend on Sd there
    double Sd = ctx.x;
    float4 carry_a;
    double2 carry_d;
    {
        const float e = pred_e((float)ctx.x, x[NB], ivs[NB]);
        carry_a = make_float4(e, e, e, __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, (float)ctx.x) - 1u));
        carry_d = make_double2(0.0, 0.0);
    }
    if (l == 0) ph[1][q] = phase;  // the start of batch 1, for the evaluator's batch 2
    __syncthreads();               // (prologue)
    unsigned long long ch_body = 0, ch_wait = 0;
    for (int b = 1; b < nb; b++) {
        const unsigned long long p0 = PROF_T();
        const int bp = b & 1;
        const float integ0 = integ, phase0 = phase;
        const double Sd0 = Sd;
        // step J: the e of candidate float(S_{J-1}) among those of trigArg_{J-1} (batch b - 1's
        // last step for J = 0: the carry), chosen by comparing S_{J-1} with their thresholds
        auto cand_of = [&](auto jc, float4& a, double2& d) {
            constexpr int J = decltype(jc)::value;
            if constexpr (J == 0) {
                a = carry_a;
                d = carry_d;
            } else {
                a = cand[bp][q][J - 1];
                d = thr[bp][q][J - 1];
            }
        };
        float o[NB];
        // max over the steps of bits(trigArg) - bits(c0 - 1 ulp): > 2 is a miss.  It starts with
        // the previous batch's last trigArg against the carry: a miss there (also left by that
        // batch's redo, which does not reach the step after it) is this batch's step 0
        uint32_t dmax = __builtin_bit_cast(uint32_t, (float)Sd0) - __builtin_bit_cast(uint32_t, carry_a.w);
        unroll_ic(
            [&](auto jc) {
                constexpr int J = decltype(jc)::value;
                float4 a;
                double2 d;
                cand_of(jc, a, d);
                const float e = Sd >= d.y ? a.z : (Sd >= d.x ? a.y : a.x);
                const float2v k = float2v{Ki, Kp} * e;
                integ = integ + k.x;
                phase = phase + (k.y + integ);
                Sd = prs_l[bp][q][J] + (double)phase;
                const float arg = (float)Sd;
                o[J] = arg;
                dmax = max(dmax, __builtin_bit_cast(uint32_t, arg) - __builtin_bit_cast(uint32_t, cand[bp][q][J].w));
            },
            std::make_integer_sequence<int, NB>{});
        if (__builtin_expect(dmax > 2u, 0)) {
            // a trigArg outside its candidates: redo the batch, evaluating the e of a step that
            // follows a miss directly (rows without a miss are masked off here)
            integ = integ0;
            phase = phase0;
            Sd = Sd0;
            const int j0 = b * NB;
            unroll_ic(
                [&](auto jc) {
                    constexpr int J = decltype(jc)::value;
                    float4 a;
                    double2 d;
                    cand_of(jc, a, d);
                    float e = Sd >= d.y ? a.z : (Sd >= d.x ? a.y : a.x);
                    const float ta = (float)Sd;
                    if (__builtin_bit_cast(uint32_t, ta) - __builtin_bit_cast(uint32_t, a.w) > 2u)
                        e = pred_e(ta, x[j0 + J], ivs[j0 + J]);
                    const float2v k = float2v{Ki, Kp} * e;
                    integ = integ + k.x;
                    phase = phase + (k.y + integ);
                    Sd = prs_l[bp][q][J] + (double)phase;
                    o[J] = (float)Sd;
                },
                std::make_integer_sequence<int, NB>{});
        }
        phase += (inject >= 0 && b == 1 + (inject + s) % (nb - 1)) ? 1.0e-3f : 0.0f;  // test hook
        if (inject >= 0) Sd = prs_l[bp][q][NB - 1] + (double)phase;
        // every lane stores: the rows of a stream hold the same values, and rows past the last
        // stream recompute it bit for bit (their evaluator rows too), so the writes agree
        float* ob = out + b * NB;
#pragma unroll
        for (int qq = 0; qq < NB / 4; qq++)
            reinterpret_cast<float4*>(ob)[qq] = *reinterpret_cast<const float4*>(&o[4 * qq]);
        rec[(size_t)s * rb + b] = make_float2(integ, phase);
        carry_a = cand[bp][q][NB - 1];  // the candidates of step 15: step 0 of batch b + 1
        carry_d = thr[bp][q][NB - 1];
        if (l == 0) ph[(b + 1) & 1][q] = phase;
        const unsigned long long p1 = PROF_T();
        __syncthreads();
        ch_body += p1 - p0;
        ch_wait += PROF_T() - p1;
    }
#ifdef FMRX_AB_PROF
    if (t == 0) {
        atomicAdd(&g_pred_prof[0], ch_body);
        atomicAdd(&g_pred_prof[1], ch_wait);
        atomicAdd(&g_pred_prof[4], (unsigned long long)(nb - 1));
    }
#endif
    (void)ch_body;
    (void)ch_wait;
}

}  // namespace

#ifdef FMRX_AB_PROF
static void print_pred_prof() {
    unsigned long long h[6] = {};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pred_prof), sizeof h) == hipSuccess && h[4])
        std::fprintf(stderr, "pll_pred prof: batches %llu chain body %.1f wait %.1f, evaluator body %.1f wait %.1f "
                     "(shader cycles per batch)\n", h[4], (double)h[0] / h[4], (double)h[1] / h[4],
                     (double)h[2] / h[4], (double)h[3] / h[4]);
}
#endif

void launch_pll_pred(int waves, hipStream_t s, const float* io, int n, int n_streams, int spw, size_t stride,
                     const double* side, size_t seg, double step, float norm_bw, const float* st, float* out,
                     size_t ostride, int* fail, float2* rec, size_t rb, int inject, int sat_ok) {
#ifdef FMRX_AB_PROF
    static const bool reg = [] { return std::atexit(print_pred_prof) == 0; }();
    (void)reg;
#endif
    hipLaunchKernelGGL(pll_pred_kernel<kPllBatch>, dim3(waves), dim3(128), 0, s, io, n, n_streams, spw, stride, side,
                       seg, step, norm_bw, st, out, ostride, fail, rec, rb, inject, sat_ok);
}

}  // namespace fmrx
