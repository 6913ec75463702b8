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

#include <climits>
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
__device__ unsigned long long g_pipe_prof[6];
__device__ unsigned long long g_pipe_prof_w2[4];  // wave 2's body / barrier wait / put / check
__device__ unsigned long long g_miss_reason[3];   // pll_pipe_kernel's missed steps by reason
__device__ unsigned long long g_idx_prof[6];
__device__ unsigned long long g_cnt_prof[6];
// redos per stream (blockIdx.x) and form: pipe 16-step, pipe 64-step five, pipe three, index
constexpr int kProfStreams = 4096;
__device__ unsigned int g_redo_stream[4][kProfStreams];
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

// Adjacent floats, across zero too (the phase may sit near it).
__device__ inline float f_up(float x) {
    const uint32_t u = __builtin_bit_cast(uint32_t, x);
    return __builtin_bit_cast(float, (u & 0x80000000u) ? (u == 0x80000000u ? 1u : u - 1u) : u + 1u);
}
__device__ inline float f_down(float x) {
    const uint32_t u = __builtin_bit_cast(uint32_t, x);
    return __builtin_bit_cast(float, (u & 0x80000000u) ? u + 1u : (u == 0u ? 0x80000001u : u - 1u));
}

// trigArg = float(P + phase) in double (filter.cpp:165) is monotone in the float phase, so
// "trigArg >= c" is "phase >= T" for a float threshold T: the smallest phase whose trigArg
// reaches c.  The chain then selects its candidate with float compares of the phase it has just
// formed, before the double sum and its roundings.  T lies within an ulp of float(m - P), m the
// boundary of c's rounding interval (the midpoint with its predecessor, the tie rounding to
// even): the first of its two lower neighbours, itself and its upper neighbour that reaches c,
// checked by the double sum itself, exactly; -inf flags a T outside that window (the caller
// poisons the step's candidates, so the chain takes it as a miss).
__device__ inline bool reaches(double P, float ph, float c) { return (float)(P + (double)ph) >= c; }
__device__ inline float phase_thr(double P, uint32_t cb) {
    const float c = __builtin_bit_cast(float, cb);
    const double m = 0.5 * ((double)__builtin_bit_cast(float, cb - 1u) + (double)c);
    const float f0 = (float)(m - P), fm = f_down(f0), fmm = f_down(fm), fp = f_up(f0);
    const bool rp = reaches(P, fp, c), r0 = reaches(P, f0, c), rm = reaches(P, fm, c), rmm = reaches(P, fmm, c);
    const float T = rm ? fm : (r0 ? f0 : fp);
    return (rp && !rmm) ? T : -__builtin_inff();
}

// The chain's candidate choice, e of trigArg_{j-1} from the phase: a = (T0, T1, e(c0 - 1),
// e(c0)), ep = e(c0 + 1); phase >= T1 -> c0 + 1, >= T0 -> c0, else c0 - 1.  One asm block: two
// compares into SGPR masks, then the two v_cndmask, with the two wait states a VALU-written lane
// mask needs before a VALU reads it (the s_nop and the first v_cndmask stand between each compare
// and its reader).  Left to itself the compiler writes VCC twice, each with its own wait states;
// as separate statements it pads each one (tools/ubench_chain.hip, modes 6 and 9).
__device__ inline float pick(float phase, float4 a, float ep) {
    float e;
    uint64_t m0, m1;
    asm("v_cmp_ge_f32_e64 %1, %3, %4\n"
        "v_cmp_ge_f32_e64 %2, %3, %5\n"
        "s_nop 0\n"
        "v_cndmask_b32_e64 %0, %6, %7, %1\n"
        "v_cndmask_b32_e64 %0, %0, %8, %2"
        : "=&v"(e), "=&s"(m0), "=&s"(m1)
        : "v"(phase), "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(ep));
    return e;
}

// The same with five candidates: T = (T(c0 - 1), T(c0), T(c0 + 1), T(c0 + 2)), E = (e(c0 - 2) ..
// e(c0 + 1)), e2 = e(c0 + 2).  Four compares into SGPR masks, then four v_cndmask, each reading a
// mask written four VALU earlier (no wait state needed).
__device__ inline float pick5(float phase, float4 T, float4 E, float e2) {
    float e;
    uint64_t m0, m1, m2, m3;
    asm("v_cmp_ge_f32_e64 %1, %5, %6\n"
        "v_cmp_ge_f32_e64 %2, %5, %7\n"
        "v_cmp_ge_f32_e64 %3, %5, %8\n"
        "v_cmp_ge_f32_e64 %4, %5, %9\n"
        "v_cndmask_b32_e64 %0, %10, %11, %1\n"
        "v_cndmask_b32_e64 %0, %0, %12, %2\n"
        "v_cndmask_b32_e64 %0, %0, %13, %3\n"
        "v_cndmask_b32_e64 %0, %0, %14, %4"
        : "=&v"(e), "=&s"(m0), "=&s"(m1), "=&s"(m2), "=&s"(m3)
        : "v"(phase), "v"(T.x), "v"(T.y), "v"(T.z), "v"(T.w), "v"(E.x), "v"(E.y), "v"(E.z), "v"(E.w), "v"(e2));
    return e;
}

// Four of pll_pipe_kernel's chain steps in one asm block: per step the candidate choice (pick /
// pick5), (Ki e, Kp e) as one v_pk_mul_f32 with (Ki, Kp) in an SGPR pair (kk: Ki low, Kp high),
// and the three float updates integ += Ki e, phase += Kp e + integ (filter.cpp:161-162), each
// product and sum rounded on its own as there.  9 instructions a step with three candidates, 12
// with five.  Compiled step by step, the same chain issued 11 and 14: the compiler puts a wait
// state after every asm statement whose result a VALU reads (it cannot see the statement's last
// instruction), and another after a v_pk_mul_f32 reading (Ki, Kp) from VGPRs; here one wait
// state follows each block of four (tools/ubench_chain.hip modes 9 and 20).  e and the two
// products live in v252-v255, clobbered.  ph[k] = the phase after step k.
#define FMRX_CHAIN_TAIL(P, Q)                                    \
    "v_pk_mul_f32 v[254:255], v[252:253], %[kk] op_sel_hi:[0,1]\n" \
    "v_add_f32 %[ig], %[ig], v254\n"                             \
    "v_add_f32 v255, v255, %[ig]\n"                              \
    "v_add_f32 " Q ", " P ", v255\n"
#define FMRX_CHAIN_STEP3(P, Q, K)                                      \
    "v_cmp_ge_f32_e64 %[m0], " P ", %[ta" #K "]\n"                       \
    "v_cmp_ge_f32_e64 %[m1], " P ", %[tb" #K "]\n"                       \
    "s_nop 0\n"                                                        \
    "v_cndmask_b32_e64 v252, %[ea" #K "], %[eb" #K "], %[m0]\n"          \
    "v_cndmask_b32_e64 v252, v252, %[ec" #K "], %[m1]\n" FMRX_CHAIN_TAIL(P, Q)
#define FMRX_CHAIN_STEP5(P, Q, K)                                      \
    "v_cmp_ge_f32_e64 %[m0], " P ", %[ta" #K "]\n"                       \
    "v_cmp_ge_f32_e64 %[m1], " P ", %[tb" #K "]\n"                       \
    "v_cmp_ge_f32_e64 %[m2], " P ", %[tc" #K "]\n"                       \
    "v_cmp_ge_f32_e64 %[m3], " P ", %[td" #K "]\n"                       \
    "v_cndmask_b32_e64 v252, %[ea" #K "], %[eb" #K "], %[m0]\n"          \
    "v_cndmask_b32_e64 v252, v252, %[ec" #K "], %[m1]\n"                 \
    "v_cndmask_b32_e64 v252, v252, %[ed" #K "], %[m2]\n"                 \
    "v_cndmask_b32_e64 v252, v252, %[ee" #K "], %[m3]\n" FMRX_CHAIN_TAIL(P, Q)
#define FMRX_CHAIN_OUTS \
    [q0] "=&v"(ph[0]), [q1] "=&v"(ph[1]), [q2] "=&v"(ph[2]), [q3] "=&v"(ph[3]), [ig] "+v"(integ)

// a[k] = (T0, T1, e(c0 - 1), e(c0)), ep[k] = e(c0 + 1) of step k (pick's arguments)
__device__ inline void chain4_3(float phase, float& integ, uint64_t kk, const float4 (&a)[4], const float (&ep)[4],
                                float (&ph)[4]) {
    uint64_t m0, m1;
    asm volatile(FMRX_CHAIN_STEP3("%[p]", "%[q0]", 0) FMRX_CHAIN_STEP3("%[q0]", "%[q1]", 1)
                     FMRX_CHAIN_STEP3("%[q1]", "%[q2]", 2) FMRX_CHAIN_STEP3("%[q2]", "%[q3]", 3)
                 : FMRX_CHAIN_OUTS, [m0] "=&s"(m0), [m1] "=&s"(m1)
                 : [p] "v"(phase), [kk] "s"(kk),
                   [ta0] "v"(a[0].x), [tb0] "v"(a[0].y), [ea0] "v"(a[0].z), [eb0] "v"(a[0].w), [ec0] "v"(ep[0]),
                   [ta1] "v"(a[1].x), [tb1] "v"(a[1].y), [ea1] "v"(a[1].z), [eb1] "v"(a[1].w), [ec1] "v"(ep[1]),
                   [ta2] "v"(a[2].x), [tb2] "v"(a[2].y), [ea2] "v"(a[2].z), [eb2] "v"(a[2].w), [ec2] "v"(ep[2]),
                   [ta3] "v"(a[3].x), [tb3] "v"(a[3].y), [ea3] "v"(a[3].z), [eb3] "v"(a[3].w), [ec3] "v"(ep[3])
                 : "v252", "v253", "v254", "v255");
}

// T[k], E[k], e2[k]: pick5's arguments of step k
__device__ inline void chain4_5(float phase, float& integ, uint64_t kk, const float4 (&T)[4], const float4 (&E)[4],
                                const float (&e2)[4], float (&ph)[4]) {
    uint64_t m0, m1, m2, m3;
    asm volatile(FMRX_CHAIN_STEP5("%[p]", "%[q0]", 0) FMRX_CHAIN_STEP5("%[q0]", "%[q1]", 1)
                     FMRX_CHAIN_STEP5("%[q1]", "%[q2]", 2) FMRX_CHAIN_STEP5("%[q2]", "%[q3]", 3)
                 : FMRX_CHAIN_OUTS, [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3)
                 : [p] "v"(phase), [kk] "s"(kk),
                   [ta0] "v"(T[0].x), [tb0] "v"(T[0].y), [tc0] "v"(T[0].z), [td0] "v"(T[0].w),
                   [ea0] "v"(E[0].x), [eb0] "v"(E[0].y), [ec0] "v"(E[0].z), [ed0] "v"(E[0].w), [ee0] "v"(e2[0]),
                   [ta1] "v"(T[1].x), [tb1] "v"(T[1].y), [tc1] "v"(T[1].z), [td1] "v"(T[1].w),
                   [ea1] "v"(E[1].x), [eb1] "v"(E[1].y), [ec1] "v"(E[1].z), [ed1] "v"(E[1].w), [ee1] "v"(e2[1]),
                   [ta2] "v"(T[2].x), [tb2] "v"(T[2].y), [tc2] "v"(T[2].z), [td2] "v"(T[2].w),
                   [ea2] "v"(E[2].x), [eb2] "v"(E[2].y), [ec2] "v"(E[2].z), [ed2] "v"(E[2].w), [ee2] "v"(e2[2]),
                   [ta3] "v"(T[3].x), [tb3] "v"(T[3].y), [tc3] "v"(T[3].z), [td3] "v"(T[3].w),
                   [ea3] "v"(E[3].x), [eb3] "v"(E[3].y), [ec3] "v"(E[3].z), [ed3] "v"(E[3].w), [ee3] "v"(e2[3])
                 : "v252", "v253", "v254", "v255");
}
#undef FMRX_CHAIN_OUTS
#undef FMRX_CHAIN_STEP5
#undef FMRX_CHAIN_STEP3
#undef FMRX_CHAIN_TAIL

template <int NB>
__global__ void __launch_bounds__(128) pll_pred_kernel(const float* io, int n, int n_streams, int spw, size_t stride,
                                                      const double* side, size_t seg, double step, float norm_bw,
                                                      const float* st, float* out_base, size_t ostride, int* fail,
                                                      float2* rec, size_t rb, int inject, int sat_ok,
                                                      int pipe_on) {
    // per step of the batch, double-buffered by batch parity: the phase thresholds of c0 and
    // c0 + 1 ulp, the bits of c0 - 1 ulp and the next step's e for c0 - 1 ulp (sa); its e for c0
    // and c0 + 1 ulp and P (sb: e_0, e_p, P as two words).  Two 16-B reads a step: the chain
    // loads a whole batch into registers before its first step.
    __shared__ float4 sa[2][4][NB];
    __shared__ float4 sb[2][4][NB];
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
    if (!pll_pred_wave(p.trig, step) || (sat_ok && pll_sat_segment(spw, p.trig, step)) ||
        (pipe_on && pll_pipe_stream(p.trig, step)))
        return;
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
            const uint2 prw = __builtin_bit_cast(uint2, pr);
            if (spw == 1) {
                // one stream: its four rows share the work -- rows 0-2 the e of candidates
                // c0 - 1, c0, c0 + 1 ulp, row 3 the thresholds, the miss bits and P
                const int r = t >> 4;
                float* a = reinterpret_cast<float*>(&sa[b & 1][0][l]);
                float* bb = reinterpret_cast<float*>(&sb[b & 1][0][l]);
                if (r < 3) {
                    const float e = pred_e(__builtin_bit_cast(float, cb + (uint32_t)(r - 1)), v, iv);
                    if (r == 0) a[3] = e;
                    else bb[r - 1] = e;
                } else {
                    const float T0 = phase_thr(pr, cb), T1 = phase_thr(pr, cb + 1u);
                    // a candidate that is not a positive finite float or a threshold outside its
                    // window: every trigArg misses the step's candidates
                    const bool ok = c0 > 0.0f && c0 < 3.0e38f && T0 > -__builtin_inff() && T1 > -__builtin_inff();
                    a[0] = T0;
                    a[1] = T1;
                    a[2] = __builtin_bit_cast(float, ok ? cb - 1u : 0xFFFFFFFFu);
                    bb[2] = __builtin_bit_cast(float, prw.x);
                    bb[3] = __builtin_bit_cast(float, prw.y);
                }
                return;
            }
            const float em = pred_e(__builtin_bit_cast(float, cb - 1u), v, iv);
            const float e0 = pred_e(c0, v, iv);
            const float ep = pred_e(__builtin_bit_cast(float, cb + 1u), v, iv);
            const float T0 = phase_thr(pr, cb), T1 = phase_thr(pr, cb + 1u);
            const bool ok = c0 > 0.0f && c0 < 3.0e38f && T0 > -__builtin_inff() && T1 > -__builtin_inff();
            if ((t >> 4) < spw) {
                sa[b & 1][q][l] = make_float4(T0, T1, __builtin_bit_cast(float, ok ? cb - 1u : 0xFFFFFFFFu), em);
                sb[b & 1][q][l] = make_float4(e0, ep, __builtin_bit_cast(float, prw.x), __builtin_bit_cast(float, prw.y));
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
    float tlast = (float)ctx.x;  // the last trigArg done
    // the carry: the candidates of the previous batch's last trigArg -- after the exact batch 0
    // its e directly (all three slots alike, so the thresholds do not matter)
    float4 carry_a, carry_b;
    {
        const float e = pred_e(tlast, x[NB], ivs[NB]);
        carry_a = make_float4(0.0f, 0.0f, __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, tlast) - 1u), e);
        carry_b = make_float4(e, e, 0.0f, 0.0f);
    }
    if (l == 0) ph[1][q] = phase;  // the start of batch 1, for the evaluator's batch 2
    __syncthreads();               // (prologue)
    unsigned long long ch_body = 0, ch_wait = 0;
    for (int b = 1; b < nb; b++) {
        const unsigned long long p0 = PROF_T();
        const int bp = b & 1;
        const float integ0 = integ, phase0 = phase, tlast0 = tlast;
        // the whole batch's data into registers first (32 reads), so no step waits on LDS
        float4 A[NB], Bv[NB];
#pragma unroll
        for (int J = 0; J < NB; J++) {
            A[J] = sa[bp][q][J];
            Bv[J] = sb[bp][q][J];
        }
        __builtin_amdgcn_sched_barrier(0);
        auto P_of = [&](int J) {
            return __builtin_bit_cast(double, make_uint2(__builtin_bit_cast(uint32_t, Bv[J].z),
                                                         __builtin_bit_cast(uint32_t, Bv[J].w)));
        };
        // step J's selection data: those of trigArg_{J-1} (the carry for J = 0)
        auto sel_of = [&](auto jc, float4& a, float4& bb) {
            constexpr int J = decltype(jc)::value;
            if constexpr (J == 0) {
                a = carry_a;
                bb = carry_b;
            } else {
                a = A[J - 1];
                bb = Bv[J - 1];
            }
        };
        float o[NB];
        // max over the steps of bits(trigArg) - bits(c0 - 1 ulp): > 2 is a miss.  It starts with
        // the previous batch's last trigArg against the carry: a miss there (also left by that
        // batch's redo, which does not reach the step after it) is this batch's step 0
        uint32_t dmax = __builtin_bit_cast(uint32_t, tlast) - __builtin_bit_cast(uint32_t, carry_a.z);
        unroll_ic(
            [&](auto jc) {
                constexpr int J = decltype(jc)::value;
                float4 a, bb;
                sel_of(jc, a, bb);
                // the chain: two compares of the phase, e, (Ki e, Kp e), the three float updates
                const float e = pick(phase, make_float4(a.x, a.y, a.w, bb.x), bb.y);
                const float2v k = float2v{Ki, Kp} * e;
                integ = integ + k.x;
                phase = phase + (k.y + integ);
                // off the chain: trigArg (filter.cpp:165) and its candidate check
                const float arg = (float)(P_of(J) + (double)phase);
                o[J] = arg;
                dmax = max(dmax, __builtin_bit_cast(uint32_t, arg) - __builtin_bit_cast(uint32_t, A[J].z));
            },
            std::make_integer_sequence<int, NB>{});
        tlast = o[NB - 1];
        if (__builtin_expect(dmax > 2u, 0)) {
            // a trigArg outside its candidates: redo the batch, evaluating the e of a step that
            // follows a miss directly (rows without a miss are masked off here)
            integ = integ0;
            phase = phase0;
            float tprev = tlast0;
            const int j0 = b * NB;
            unroll_ic(
                [&](auto jc) {
                    constexpr int J = decltype(jc)::value;
                    float4 a, bb;
                    sel_of(jc, a, bb);
                    float e = pick(phase, make_float4(a.x, a.y, a.w, bb.x), bb.y);
                    if (__builtin_bit_cast(uint32_t, tprev) - __builtin_bit_cast(uint32_t, a.z) > 2u)
                        e = pred_e(tprev, x[j0 + J], ivs[j0 + J]);
                    const float2v k = float2v{Ki, Kp} * e;
                    integ = integ + k.x;
                    phase = phase + (k.y + integ);
                    tprev = (float)(P_of(J) + (double)phase);
                    o[J] = tprev;
                },
                std::make_integer_sequence<int, NB>{});
            tlast = o[NB - 1];
        }
        if (inject >= 0 && b == 1 + (inject + s) % (nb - 1)) {  // test hook: a wrong batch
            phase += 1.0e-3f;
            tlast = (float)(P_of(NB - 1) + (double)phase);
        }
        // every lane stores: the rows of a stream hold the same values, and rows past the last
        // stream recompute it bit for bit (their evaluator rows too), so the writes agree
        float* ob = out + b * NB;
#pragma unroll
        for (int qq = 0; qq < NB / 4; qq++)
            reinterpret_cast<float4*>(ob)[qq] = *reinterpret_cast<const float4*>(&o[4 * qq]);
        rec[(size_t)s * rb + b] = make_float2(integ, phase);
        carry_a = A[NB - 1];  // the candidates of step 15: step 0 of batch b + 1
        carry_b = Bv[NB - 1];
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


// ---- pll_pipe_kernel: one stream a workgroup of three waves, trigOffset from 2^20 on ----------
//
// pll_pred_kernel's chain wave issues ~16 VALU a step (the candidate choice, the updates, trigArg
// and its check), and one wave issues a VALU per ~4 cycles, dependent or not (tools/ubench_dep.hip,
// profiles/r03/ubench_dep.txt): its step costs its instruction count, wait states included.  Here
// the chain keeps only the recurrence -- the candidate choice (compares of the phase into SGPR
// masks, v_cndmask), (Ki e, Kp e), the three float updates: 9 instructions a step with NC = 3
// candidates, 12 with 5, four steps an asm block (chain4_3 / chain4_5) -- and hands one state a
// batch, (integ, phase) after its last step, to the other waves:
//   wave 1: interval k + 1's e for the NC candidates c0 - NC/2 .. c0 + NC/2 of every step, each
//           with its certification (pred_e_cert: the float roundings of the candidate's sin/cos
//           and of atan2 proven as in pll_batch_fast);
//   wave 2: interval k + 1's NC - 1 phase thresholds a step, c0's bits and P; and interval
//           k - 1 replayed batch by batch from those states, one lane group a batch (the chain's
//           arithmetic on the same data, so the same phases), its trigArgs float(P + phase)
//           (filter.cpp:165), their check against the candidates AND the certification of the
//           candidate each step took, and the output stores.
// So the runner is exact by construction: every e the chain used is the exact path's e (a
// certified candidate that is the true trigArg), every state it carries is the exact path's.  No
// pll_check_kernel, no resume kernel, no pre-pass (1/v and P = step x trigOffset are formed
// inline, pll_side's arithmetic): one launch runs a form's whole range of the call, however long,
// and leaves the exact end state in st.
// The candidates of interval k + 1 come from the phase at the start of interval k
// (tools/pll_predict.cpp, lookback 2).  NC = 3 with 64-step intervals from 2^22 (every interval
// of the bench stream hit), NC = 5 with 64-step intervals in [2^21, 2^22) (99.97 %) and with
// 16-step ones in [2^20, 2^21) (99.7 %).  The chain reads an interval's data in bursts before
// their steps (spread over the steps the reads stall it more: tools/ubench_chain.hip,
// profiles/r03/ubench_chain.txt).  A missed interval (a trigArg outside its candidates, or taken
// from an uncertified one) -- wave 2 flags it in the interval after the chain ran it, the chain
// reads the flag at the end of the next one -- is redone on the exact path with the two after it
// (pll_redo from the state at the interval's start, kept in the LDS ring); every wave takes two
// more barriers around that redo, and the evaluators redo the next interval from the corrected
// phase.

// pred_e with pll_batch_fast's certification of one step: the float roundings of the
// candidate's cos and sin (16-ulp margin), |r| >= kPllMinR, |a| < kPllMaxX, [th - E, th + E]
// within one float (E = kPllEBatch: d = Y iv with the rcp-Newton 1/v), |d| < kPllMaxD, |B| <=
// kPllMaxB, a finite iv.  ok: e is then the exact path's e (pll_step, glibc's atan2 rounded) for
// a step with input v after trigArg a, bit for bit.
__device__ inline float pred_e_cert(float a, float v, double iv, bool& ok) {
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
    const double d = Y * iv;
    const double th = d + B;
    const float lo = (float)(th - kPllEBatch), hi = (float)(th + kPllEBatch);
    ok = (int)(fabs(x) < kPllMaxX) & (int)(pll_margin16x8(cs) > 256u) & (int)(pll_margin16x8(sn) > 256u) &
         (int)(fabs(r) >= kPllMinR) & (int)(lo == hi) & (int)(fabs(d) < kPllMaxD) & (int)(fabs(B) <= kPllMaxB);
    return lo;
}

// 1 / v as the check kernel forms it (reciprocal + one Newton step, ~2^-46 relative, within the
// batch bound kPllEBatch); NaN outside [kPllMinV, 1e300) (pll_side)
__device__ inline double pll_iv(float v) {
    const double vd = (double)v;
    const double r0 = __builtin_amdgcn_rcp(vd);
    const double r1 = fma(r0, fma(-vd, r0, 1.0), r0);
    return (fabs(vd) >= (double)kPllMinV && fabs(vd) < 1.0e300) ? r1 : (double)NAN;
}

// The exact path's e of a step with input v whose previous trigArg is a (pll_step's first half
// from the state after that trigArg: its sin/cos certified or from the library, then the
// rotation atan2 certified or from the library).  Used where the chain continues after an exact
// stretch, by the chain and by wave 2's replay alike.
__device__ __noinline__ float exact_e(float a, float v) {
    const DeviceLib lib;
    PllCtx c{};
    float sv, cv;
    if (!sincos_ctx_f(a, &sv, &cv, &c)) lib.sincosf_(a, &sv, &cv);
    const float eI = v * cv;
    const float eQ = v * (-sv);
    float e;
    if (!rot_atan2_f(eQ, eI, c, &e)) e = lib.atan2f_(eQ, eI);
    return e;
}

// The e of a range's first step from the state it starts with (pll_step's first half with the
// state's own feedback, no sincos context: the library atan2, as pll_redo's first step).
__device__ __noinline__ float exact_e_fb(float fbI, float fbQ, float v) {
    const DeviceLib lib;
    const float eI = v * fbI;
    const float eQ = v * (-fbQ);
    return lib.atan2f_(eQ, eI);
}

// One wave a SIMD (amdgpu_waves_per_eu): the register budget is the chain's, so the scheduler
// keeps each burst of reads whole instead of threading it through the steps for occupancy.
// io / out: the stream's input and trigArg rows from the range's first sample (stride / ostride
// floats a stream), n samples; st: the state (read at the start, the exact end state written).
// WIDE (the short-call form, launch_pll_pipe form 24): the 16-step five-candidate form from 2^20 on,
// across the later forms' ranges and the stick (five candidates cover what three do there)
template <int NB, int BPI, int RD, int NC, bool STK = false, bool WIDE = false>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(1, 1))) pll_pipe_kernel(const float* io, int n, int n_streams, size_t stride,
                                                      double step, float norm_bw, float* st, float* out_base,
                                                      size_t ostride, int inject, int miss,
                                                      unsigned long long* stats, unsigned* redos) {
    constexpr int NI = NB * BPI;
    static_assert(NI == 16 || NI == 32 || NI == 64 || (BPI > 1 && (NI == 128 || NI == 256)),
                  "the evaluators' lane map: 64 / NI lanes a step, or NI / 64 steps a lane");
    static_assert(NC == 3 || NC == 5, "three or five candidates");
    // STK: the stuck trigOffset (2^24, filter.cpp:165-166: 69.9 s into a stream).  Every step's
    // P is then the same, so c0 = float(P + phase_ref) and the two thresholds are the interval's
    // constants: wave 2 forms them once (sthr) and the e of the three candidates sit three floats a
    // step (sek) -- 0.75 16-byte reads a step for the chain instead of 1.25
    static_assert(!STK || (NC == 3 && BPI > 1), "the stick form is the three-candidate replay form");
    constexpr int NIL = NI > 64 ? 64 : NI;  // the evaluators' lane map: step l + NIL sp on lane l
    constexpr int SPL = NI / NIL;          // steps a lane (128-step intervals: two)
    constexpr int LPS = 64 / NIL;          // evaluator lanes a step
    constexpr int HC = NC / 2;    // candidates c0 - HC .. c0 + HC
    // the chain's steps a burst of reads (its registers hold a burst's data)
#ifndef FMRX_CHM
#define FMRX_CHM 32
#endif
    constexpr int CHM = FMRX_CHM;
    constexpr int CH = NC == 5 ? 16 : (NI < CHM ? NI : CHM);
    // rings of four intervals (interval k in slot k & 3; slot 0 holds the range's start state), per step: NC = 3:
    // the thresholds of c0 and c0 + 1 ulp and the e of c0 - 1 and c0 (sel), the e of c0 + 1
    // (sep); NC = 5: the thresholds of c0 - 1 .. c0 + 2 (sel), the e of c0 - 2 .. c0 + 1 (sel2),
    // of c0 + 2 (sep); bits(c0) - HC (scb), P (spr); the certification of each candidate's e
    // (scert, byte r for c0 - HC + r); the chain's (integ, phase) at the end of each batch (sst);
    // per interval the check's verdict (smiss) and "redone exactly" (sexact)
    __shared__ float4 sel[STK ? 1 : 4][STK ? 1 : NI];  // (the stick form: sthr and sek instead)
    __shared__ float4 sel2[NC == 5 ? 4 : 1][NC == 5 ? NI : 1];
    __shared__ float sep[STK ? 1 : 4][STK ? 1 : NI];
    __shared__ uint32_t scb[4][NI];
    __shared__ double spr[4][NI];
    __shared__ uint8_t scert[4][NI][8];
    __shared__ float2 sst[4][BPI];
    // one batch an interval (the 16-step form): the replay below would be as long as the chain's
    // own interval, so the chain hands over every phase instead (sph) and wave 2 checks those
    constexpr bool REPLAY = BPI > 1;
    __shared__ float sph[REPLAY ? 1 : 4][REPLAY ? 1 : NI];
    __shared__ int smiss[4], sexact[4];
    __shared__ int sdemote;  // the chain demoted the stream (pll_demote) at its redo
    __shared__ __attribute__((aligned(16))) float sek[STK ? 4 : 1][STK ? 3 * NI : 4];
    __shared__ float2 sthr[4];
    // the candidate data the chain and the replay select from at step J of ring slot sl: (T0, T1,
    // e(c0 - 1), e(c0)) and e(c0 + 1)
    auto cand = [&](int sl, int J) {
        if constexpr (STK) {
            const float2 T = sthr[sl];
            return make_float4(T.x, T.y, sek[STK ? sl : 0][STK ? 3 * J : 0], sek[STK ? sl : 0][STK ? 3 * J + 1 : 0]);
        } else {
            return sel[sl][J];
        }
    };
    auto cand_ep = [&](int sl, int J) {
        if constexpr (STK) return sek[STK ? sl : 0][STK ? 3 * J + 2 : 0];
        else return sep[sl][J];
    };
    // the wave (readfirstlane: uniform, so the waves' branches and loops are scalar)
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63, l = t & (NIL - 1), h = t / NIL;
    const int s = blockIdx.x;  // grid = n_streams
    const float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    float* S = st + 8 * (size_t)s;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    // the stream's state, uniform over the group (readfirstlane): the domain test below and every
    // branch and loop after it stay scalar
    auto uni = [](float v) { return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v))); };
    PllState p{uni(S[0]), uni(S[1]), uni(S[2]), uni(S[3]), uni(S[5])};
    // demoted by an earlier runner launch of this call (pll_demote; state slot 6: the steps it left
    // to pll_demoted_kernel, int bits): this range is theirs too -- add it and leave (uniform)
    if (const int rem = __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, S[6])); rem > 0) {
        if (threadIdx.x == 0) {
            S[6] = __builtin_bit_cast(float, rem + n);
            if (redos) atomicAdd(&redos[kPllRedoSlots * (size_t)s + 4 + pll_redo_range(p.trig)], (unsigned)n);
        }
        return;
    }
    // the variant's domain (uniform over the group): NC = 3 from 2^22; NC = 5 with 64-step
    // intervals in [2^21, 2^22), with 16-step ones in [2^20, 2^21)
    static_assert(!WIDE || (NC == 5 && BPI == 1 && !STK), "the wide form is the 16-step five-candidate one");
    const bool in_domain = STK ? pll_pipe_stream(p.trig, step, kPllTrigStick)
                         : WIDE ? pll_pipe_stream(p.trig, step, kPllPipeMinLow)
                         : NC == 3 ? pll_pipe_stream(p.trig, step, kPllPipeMin)
                                   : NI >= 64 ? pll_pipe_stream(p.trig, step, kPllPipeMin5, kPllPipeMin - 1.0f)
                                              : pll_pipe_stream(p.trig, step, kPllPipeMinLow, kPllPipeMin5 - 1.0f);
    const float trig0 = p.trig;
    const double t0d = (double)trig0;
    // pll_side's P of step j (trigOffset after the step's increment, stuck at 2^24)
    auto pr_at = [&](long long j) {
        return step * (double)(float)fmin(t0d + (double)(j + 1), (double)kPllTrigStick);
    };
    const int nb = n / NB;
    const int ni = nb / BPI;  // intervals 1 .. ni from the range's first step (the first predicted too)
    // test hook: a miss on interval 1 + (inject + s) % ni of this stream (the exact redo runs)
    const int inj = inject >= 0 && ni > 0 ? 1 + (inject + s) % ni : -1;
    // steps [j0, j1) exactly from state q (c): outputs
    auto exact = [&](PllState& q, PllCtx& c, long long j0, long long j1) {
        if (j1 > j0) {
            const PllPair z = pll_redo(q, c, x + j0, out + j0, (int)(j1 - j0), Ki, Kp, step, true);
            q = z.p;
            c = z.ctx;
        }
    };
    // a short range, or a stream outside the form's domain (the host's trigOffset bounds were
    // wrong: costs speed, never bits): every step exactly (no barrier is reached)
    if (ni < 2 || !in_domain) {
        if (w == 0) {
            PllCtx c{};
            c.valid = false;
            exact(p, c, 0, n);
            if (t == 0) {
                S[0] = p.integ; S[1] = p.phase; S[2] = p.fbI; S[3] = p.fbQ; S[5] = p.trig;
                S[6] = 0.0f;  // not demoted (pll_demoted_kernel)
                if (stats) {  // outside the domain: the whole range "resumed" on the exact path
                    if (!in_domain) atomicAdd(stats, (unsigned long long)nb);
                    atomicAdd(stats + 1, (unsigned long long)nb);
                }
            }
        }
        return;
    }
    auto j0 = [](int k) { return (k - 1) * NI; };  // interval k's first step (k >= 1)

    if (w > 0) {
        // ring of RD intervals of step inputs, interval k in slot k % RD, loaded RD - 1 ahead
        float vq[RD][SPL];
        auto ld = [&](int k, float (&v)[SPL]) {
#pragma unroll
            for (int sp = 0; sp < SPL; sp++) {
                const int j = j0(k <= ni ? k : ni) + l + NIL * sp;
                v[sp] = x[min(j + 1, n - 1)];  // the step the e is for
            }
        };
        // interval k's candidate data from phase_ref, the phase at the start of interval k - 1:
        // E1 lane (h, l) the e (and its certification) of candidates c0 - HC + r of step l, r = h,
        // h + LPS, ... < NC; E2 lane (h, l) the thresholds of c0 - HC + 1 + r, r = h, h + LPS,
        // ... < NC - 1, lanes h = 0 also c0's bits and P
        auto put = [&](int k, float phase_ref, const float (&vs)[SPL]) {
#pragma unroll
          for (int sp = 0; sp < SPL; sp++) {
            const int ls = l + NIL * sp;  // this lane's step
            const float v = vs[sp];
            const int j = j0(k <= ni ? k : ni) + ls;
            const double pr = pr_at(j);
            const float c0 = (float)(pr + (double)phase_ref);
            const uint32_t cb = __builtin_bit_cast(uint32_t, c0);
            const int sl = k & 3;
            if (w == 1) {
                const double iv = pll_iv(v);
                // one candidate at a time (unrolled, the five certified evaluations interleave and
                // spill the kernel's registers)
#pragma unroll 1
                for (int r = h; r < NC; r += LPS) {
                    bool ok;
                    const float e = pred_e_cert(__builtin_bit_cast(float, cb + (uint32_t)(r - HC)), v, iv, ok);
                    scert[sl][ls][r] = ok ? 1 : 0;
                    if (STK) sek[STK ? sl : 0][STK ? 3 * ls + r : 0] = e;
                    else if (r == NC - 1) sep[sl][ls] = e;
                    else if (NC == 3) reinterpret_cast<float*>(&sel[sl][ls])[2 + r] = e;
                    else reinterpret_cast<float*>(&sel2[NC == 5 ? sl : 0][NC == 5 ? ls : 0])[r] = e;
                }
                // the stick form's two thresholds, the interval's constants (every step's P and c0
                // are the same): here, where the evaluations leave time, not in wave 2 -- its check
                // sets the stick form's pace (profiles/r05/rprof_w2/)
                if (STK && t == 0 && sp == 0)
                    sthr[sl] = make_float2(phase_thr(pr, cb + (uint32_t)(1 - HC)), phase_thr(pr, cb + (uint32_t)(2 - HC)));
            } else {
                if (!STK) {
                    for (int r = h; r < NC - 1; r += LPS)
                        reinterpret_cast<float*>(&sel[sl][ls])[r] = phase_thr(pr, cb + (uint32_t)(r + 1 - HC));
                }
                if (h == 0) {
                    scb[sl][ls] = cb - (uint32_t)HC;
                    spr[sl][ls] = pr;
                }
            }
          }
        };
        // E2: interval k's check.  Lane group g = t / NB replays batch g of the interval (BPI
        // batches) from the chain's state before it -- the chain's steps on the same candidate data,
        // so the same phases -- forms each step's trigArg float(P + phase) (filter.cpp:165) and
        // checks it against the step's candidates and that candidate's certification; lane l of
        // the group stores step l's.  A candidate that is not a positive finite float, a
        // threshold outside its window (-inf), an uncertified e or a state out of pll_batch_fast's
        // range counts as a miss.  (The chain hands over one state a batch instead of every phase:
        // an LDS store of four phases cost it ~20 cycles.)
        auto verdict = [&](int sl, int J, float a) {
            const uint32_t cm = scb[sl][J];
            const float4 tt = cand(sl, J);
            const float c0 = __builtin_bit_cast(float, cm + (uint32_t)HC);
            const bool thr_ok = tt.x > -__builtin_inff() && tt.y > -__builtin_inff() &&
                                (NC == 3 || (tt.z > -__builtin_inff() && tt.w > -__builtin_inff()));
            const uint32_t idx = __builtin_bit_cast(uint32_t, a) - cm;
            const bool cert = idx < (uint32_t)NC && scert[sl][J][idx < (uint32_t)NC ? idx : 0] != 0;
#ifdef FMRX_AB_PROF
            // why a step misses: its trigArg outside the candidates / its e uncertified / a threshold
            // outside its window
            if (idx >= (uint32_t)NC) atomicAdd(&g_miss_reason[0], 1ull);
            else if (!cert) atomicAdd(&g_miss_reason[1], 1ull);
            if (!thr_ok) atomicAdd(&g_miss_reason[2], 1ull);
#endif
            return !cert || !thr_ok || !(c0 > 0.0f && c0 < 3.0e38f);
        };
        auto check = [&](int k) {
            if (w != 2) return;
            const int sl = k & 3;
            if (sexact[sl]) {  // redone exactly: the chain stored it
                if (t == 0) smiss[sl] = 0;
                return;
            }
            if constexpr (!REPLAY) {  // the chain's phases, lanes h = 0
                const float ph = sph[REPLAY ? 0 : sl][REPLAY ? 0 : l];
                const float a = (float)(spr[sl][l] + (double)ph);
                if (h == 0) out[j0(k) + l] = a;
                // pll_batch_fast's range test, on the state at the batch's start
                const float2 r0 = sst[(k - 1) & 3][BPI - 1];
                const bool bad = verdict(sl, l, a) || !(fabsf(r0.y) < kPllMaxPhase && fabsf(r0.x) < kPllMaxInteg);
                const bool any = __builtin_amdgcn_ballot_w64(h == 0 && bad) != 0 || pll_hook_miss(k, miss, ni);
                // test hooks: a forced miss (the redo path); inject's is counted as resumed
                if (t == 0) smiss[sl] = k == inj ? 2 : any ? 1 : 0;
                return;
            }
            // 64 / NB lane groups a wave, so BPI > 64 / NB batches (128-step intervals) take rounds
            constexpr int GPW = 64 / NB, RND = (BPI + GPW - 1) / GPW;
            const int g0 = t / NB, lg = t & (NB - 1);
            bool anybad = false;
#pragma unroll 1
            for (int rd = 0; rd < RND; rd++) {
                const int g = g0 + GPW * rd;
                const bool act = g < BPI;
                const int gb = act ? g : 0;  // the groups past the interval's batches replay batch 0
                const float2 r0 = gb > 0 ? sst[sl][gb - 1] : sst[(k - 1) & 3][BPI - 1];
                float ig = r0.x, ph = r0.y;
                // step 0's candidate data: those of the trigArg before it (after an exactly redone
                // interval that trigArg's exact e in every slot, as the chain's carry)
                float4 ca, ca2;
                float cep;
                if (gb > 0) {
                    ca = cand(sl, NB * gb - 1);
                    cep = cand_ep(sl, NB * gb - 1);
                    ca2 = sel2[NC == 5 ? sl : 0][NC == 5 ? NB * gb - 1 : 0];
                } else if (sexact[(k - 1) & 3]) {
                    const int j = j0(k);
                    // (interval 1: the range's first step, from the state's own feedback)
                    const float e = k == 1 ? exact_e_fb(p.fbI, p.fbQ, x[0])
                                           : exact_e((float)(pr_at(j - 1) + (double)ph), x[min(j, n - 1)]);
                    ca = NC == 3 ? make_float4(0.0f, 0.0f, e, e) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    ca2 = make_float4(e, e, e, e);
                    cep = e;
                } else {
                    ca = cand((k - 1) & 3, NI - 1);
                    cep = cand_ep((k - 1) & 3, NI - 1);
                    ca2 = sel2[NC == 5 ? (k - 1) & 3 : 0][NC == 5 ? NI - 1 : 0];
                }
                // the batch's candidate data, read before the steps (the step loop then never waits on
                // LDS); lane l keeps the phase of step l and checks its own trigArg afterwards
                float4 da[NB], da2[NC == 5 ? NB : 1];
                float dep[NB];
                if constexpr (STK) {  // the batch's three e a step as 16-byte reads, the thresholds once
                    const float2 T = sthr[sl];
                    float ek[3 * NB];
#pragma unroll
                    for (int q = 0; q < 3 * NB / 4; q++)
                        *reinterpret_cast<float4*>(&ek[4 * q]) =
                            reinterpret_cast<const float4*>(&sek[STK ? sl : 0][STK ? 3 * NB * gb : 0])[q];
#pragma unroll
                    for (int j = 0; j < NB - 1; j++) {
                        da[j] = make_float4(T.x, T.y, ek[3 * j], ek[3 * j + 1]);
                        dep[j] = ek[3 * j + 2];
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < NB - 1; j++) {
                        da[j] = cand(sl, NB * gb + j);
                        dep[j] = cand_ep(sl, NB * gb + j);
                        if constexpr (NC == 5) da2[j] = sel2[NC == 5 ? sl : 0][NC == 5 ? NB * gb + j : 0];
                    }
                }
                // pll_batch_fast's range test, on the state at the batch's start
                const bool range_ok = fabsf(r0.y) < kPllMaxPhase && fabsf(r0.x) < kPllMaxInteg;
                float mine = 0.0f;
#pragma unroll
                for (int j = 0; j < NB; j++) {
                    const float e = NC == 3 ? pick(ph, j == 0 ? ca : da[j > 0 ? j - 1 : 0], j == 0 ? cep : dep[j > 0 ? j - 1 : 0])
                                            : pick5(ph, j == 0 ? ca : da[j > 0 ? j - 1 : 0], j == 0 ? ca2 : da2[NC == 5 && j > 0 ? j - 1 : 0],
                                                    j == 0 ? cep : dep[j > 0 ? j - 1 : 0]);
                    const float2v kv = float2v{Ki, Kp} * e;
                    ig = ig + kv.x;
                    ph = ph + (kv.y + ig);
                    if (j == lg) mine = ph;
                }
                const int J = NB * gb + lg;  // this lane's step
                const float a = (float)(spr[sl][J] + (double)mine);
                const bool bad = verdict(sl, J, a) || !range_ok;
                if (act) out[j0(k) + J] = a;
                anybad = anybad || (act && bad);
            }
            const bool any = __builtin_amdgcn_ballot_w64(anybad) != 0 || pll_hook_miss(k, miss, ni);
            // test hooks: a forced miss (the redo path); inject's is counted as resumed
            if (t == 0) smiss[sl] = k == inj ? 2 : any ? 1 : 0;
        };
#pragma unroll
        for (int u = 0; u < RD; u++) ld(1 + u, vq[(1 + u) % RD]);
        put(1, p.phase, vq[1 % RD]);  // interval 1 from the initial phase
        ld(1 + RD, vq[1 % RD]);
        __syncthreads();  // (prologue)
        unsigned long long ev_body = 0, ev_wait = 0, ev_put = 0, ev_check = 0;
        // the chain demoted the stream at a redo (pll_demote): it runs the rest of the range alone
        bool demoted = false;
        // interval i: interval i + 1's data, interval i - 1's check; groups of RD intervals from
        // i0 = 1 (mod RD), so the ring slots are compile-time
        for (int i0 = 1; i0 <= ni && !demoted; i0 += RD) {
            unroll_ic(
                [&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    constexpr int sl = (2 + u) % RD;  // slot of interval i + 1
                    const int i = i0 + u;
                    if (i <= ni && !demoted) {
                        const unsigned long long p0 = PROF_T();
                        if (i + 1 <= ni) {
                            put(i + 1, sst[(i - 1) & 3][BPI - 1].y, vq[sl]);
                            ld(i + 1 + RD, vq[sl]);
                        }
                        const unsigned long long pa = PROF_T();
                        check(i - 1);
                        ev_put += pa - p0;
                        ev_check += PROF_T() - pa;
                        const int redo = __builtin_amdgcn_readfirstlane(smiss[(i - 2) & 3]);
                        if (redo) {
                            // the chain redoes interval i - 2 exactly, then runs i - 1 again on
                            // its candidates (from the phase at i - 2's start, which was right)
                            // and i on candidates predicted anew here from the corrected phase
                            __syncthreads();  // B1: the chain's exact redo of i - 2 follows
                            __syncthreads();  // B1.5: i - 2's exact end state is in the ring
                            if (__builtin_amdgcn_readfirstlane(sdemote)) {  // set before B1.5
                                demoted = true;
                                return;
                            }
                            {
                                float v[SPL];
                                ld(i, v);
                                put(i, sst[(i - 2) & 3][BPI - 1].y, v);
                            }
                            __syncthreads();  // B2: the chain ran i - 1 again
                            check(i - 1);
                            if (i + 1 <= ni) {  // interval i + 1 from the phase at i's start
                                float v[SPL];
                                ld(i + 1, v);
                                put(i + 1, sst[(i - 1) & 3][BPI - 1].y, v);
                            }
                            __syncthreads();  // B3: the chain ran i again
                        }
                        const unsigned long long p1 = PROF_T();
                        __syncthreads();
                        ev_body += p1 - p0;
                        ev_wait += PROF_T() - p1;
                    }
                },
                std::make_integer_sequence<int, RD>{});
        }
        if (!demoted) {
            check(ni);
            __syncthreads();  // the chain reads the last two verdicts
        }
#ifdef FMRX_AB_PROF
        if (t == 0 && w == 1) {
            atomicAdd(&g_pipe_prof[2], ev_body);
            atomicAdd(&g_pipe_prof[3], ev_wait);
        }
        if (t == 0 && w == 2) {
            atomicAdd(&g_pipe_prof_w2[0], ev_body);
            atomicAdd(&g_pipe_prof_w2[1], ev_wait);
            atomicAdd(&g_pipe_prof_w2[2], ev_put);
            atomicAdd(&g_pipe_prof_w2[3], ev_check);
        }
#endif
        (void)ev_body;
        (void)ev_wait;
        (void)ev_put;
        (void)ev_check;
        return;
    }

    // ---- the chain
    // interval 1 starts at the range's first step, predicted from the start phase like every other
    // (until round 6 its first batch ran on the exact path: 16 steps at ~400 ns, ~6 us a launch)
    float integ = p.integ, phase = p.phase;
    // (Ki, Kp) as an SGPR pair for the chain's v_pk_mul_f32 (uniform: readfirstlane)
    const uint64_t kk = (uint64_t)__builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, Ki)) |
                        ((uint64_t)__builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, Kp)) << 32);
    // the carry: step 0's candidate data (those of the previous interval's last trigArg); after
    // an exact stretch that trigArg's exact e in every slot
    float4 carry, carry2;
    float carry_ep;
    auto carry_exact = [&](float a, int k) {
        const float e = exact_e(a, x[min(j0(k), n - 1)]);
        carry = NC == 3 ? make_float4(0.0f, 0.0f, e, e) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        carry2 = make_float4(e, e, e, e);
        carry_ep = e;
    };
    {  // step 0's e from the state's feedback (the exact path's first step)
        const float e = exact_e_fb(p.fbI, p.fbQ, x[0]);
        carry = NC == 3 ? make_float4(0.0f, 0.0f, e, e) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        carry2 = make_float4(e, e, e, e);
        carry_ep = e;
    }
    if (t == 0) {
        sst[0][BPI - 1] = make_float2(integ, phase);  // the start of interval 1 (the evaluators' interval 2)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            smiss[k] = 0;
            sexact[k] = k == 0;
        }
        sdemote = 0;
    }
    __syncthreads();  // (prologue)
    unsigned long long ch_body = 0, ch_wait = 0, n_redo = 0, n_inj = 0, n_dem = 0;
    uint32_t hist = 0;  // the last 32 verdicts (pll_demote)
    bool demoted = false;
    PllState qd;        // demoted: the exact state at the end of the redone interval, and its step
    PllCtx cd{};
    long long jd = 0;
    // the exact state before interval f from the ring (its trigArg's sin / cos recomputed); before
    // interval 1 the range's start state as given (its feedback may not be that sin / cos: a state
    // set by the caller)
    auto state_before = [&](int f, PllState& q, PllCtx& c) {
        if (f <= 1) {
            q = p;
            c = PllCtx{};
            c.valid = false;
            return;
        }
        const float2 r0 = sst[(f - 1) & 3][BPI - 1];
        const float a = (float)(pr_at(j0(f) - 1) + (double)r0.y);  // the trigArg before it
        pll_state_at(q, c, r0.x, r0.y, trig0, (long long)j0(f), a, DeviceLib{});
    };
    // interval i on the fast chain from (integ, phase) and the carry, its data in ring slot i & 3
    auto run = [&](int i) {
        const int is = i & 3;
        // in bursts of CH steps: the data, 1.25 CH (NC = 5: 2.25 CH) 16-byte reads at once in the
        // order the steps need them (spread over the steps they stall the chain more,
        // tools/ubench_chain.hip), then the steps, then the batch states
        float4 A[CH], A2[NC == 5 ? CH : 1];
        float EP[CH];
        unroll_ic(
            [&](auto hc) {
                constexpr int H = decltype(hc)::value;
                if constexpr (STK) {  // three 16-byte reads a group of four steps, the thresholds once
                    const float2 T = sthr[is];
#pragma unroll
                    for (int q = 0; q < CH / 4; q++) {
                        float ek[12];
#pragma unroll
                        for (int u = 0; u < 3; u++)
                            *reinterpret_cast<float4*>(&ek[4 * u]) =
                                reinterpret_cast<const float4*>(&sek[STK ? is : 0][STK ? 3 * H * CH : 0])[3 * q + u];
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            A[4 * q + u] = make_float4(T.x, T.y, ek[3 * u], ek[3 * u + 1]);
                            EP[4 * q + u] = ek[3 * u + 2];
                        }
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < CH / 4; q++) {
                        *reinterpret_cast<float4*>(&EP[4 * q]) = reinterpret_cast<const float4*>(&sep[is][H * CH])[q];
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            A[4 * q + u] = sel[is][H * CH + 4 * q + u];
                            if constexpr (NC == 5) A2[4 * q + u] = sel2[NC == 5 ? is : 0][NC == 5 ? H * CH + 4 * q + u : 0];
                        }
                    }
                }
                float2 brec[CH / NB];  // (integ, phase) at the end of each batch of the burst
                float PH[REPLAY ? 1 : CH];  // (the 16-step form) the burst's phases
                unroll_ic(
                    [&](auto gc) {
                        constexpr int J = 4 * decltype(gc)::value;  // steps J .. J + 3
                        float4 a[4], a2[4];
                        float ep[4];
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            a[u] = J + u == 0 ? carry : A[J + u > 0 ? J + u - 1 : 0];
                            ep[u] = J + u == 0 ? carry_ep : EP[J + u > 0 ? J + u - 1 : 0];
                            if constexpr (NC == 5) a2[u] = J + u == 0 ? carry2 : A2[J + u > 0 ? J + u - 1 : 0];
                        }
                        float q[4];
                        if constexpr (NC == 3)
                            chain4_3(phase, integ, kk, a, ep, q);
                        else
                            chain4_5(phase, integ, kk, a, a2, ep, q);
                        phase = q[3];
                        if constexpr (!REPLAY) {
#pragma unroll
                            for (int u = 0; u < 4; u++) PH[REPLAY ? 0 : J + u] = q[u];
                        }
                        if constexpr ((J + 3) % NB == NB - 1) brec[(J + 3) / NB] = make_float2(integ, phase);
                    },
                    std::make_integer_sequence<int, CH / 4>{});
                // Every read of the burst has landed by now (the steps used them), but the waitcnt
                // pass cannot tell: after the stores' exec-masked branch it would wait for the
                // stores too (lgkmcnt(0)) before the next burst's first use.  Waiting here is free.
                // (sched_barrier: the wait stays after the steps; the scheduler moves a bare
                // s_waitcnt up among the burst's first steps)
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
                __builtin_amdgcn_sched_barrier(0);
                // every lane stores (the chain's values are uniform: the same LDS words, the same
                // arithmetic), so no lane test on the chain -- its lane id was spilled to scratch
                // and reloaded at every burst
                if constexpr (!REPLAY) {
#pragma unroll
                    for (int q = 0; q < CH / 4; q++)
                        reinterpret_cast<float4*>(&sph[REPLAY ? 0 : is][REPLAY ? 0 : H * CH])[q] =
                            *reinterpret_cast<const float4*>(&PH[REPLAY ? 0 : 4 * q]);
                }
#pragma unroll
                for (int q = 0; q < CH / NB; q++) sst[is][H * (CH / NB) + q] = brec[q];
                carry = A[CH - 1];
                if constexpr (NC == 5) carry2 = A2[CH - 1];
                carry_ep = EP[CH - 1];
            },
            std::make_integer_sequence<int, NI / CH>{});
        sexact[is] = 0;
    };
    for (int i = 1; i <= ni; i++) {
        const unsigned long long p0 = PROF_T();
        const int flag = smiss[(i - 2) & 3];  // the verdict on interval i - 2 (slot 3 is clear at i = 1)
        run(i);
        const bool over = pll_demote(hist, __builtin_amdgcn_readfirstlane(flag) != 0);
        if (__builtin_amdgcn_readfirstlane(flag)) {
            n_redo++;
            n_inj += inj == i - 2 ? 1 : 0;  // the inject hook's interval, redone exactly
            __syncthreads();  // B1: E2's stores of interval i - 1 happen before the redo's
            // interval i - 2 (missed) exactly, from the state at its start (the end of interval
            // i - 3 in the ring; interval 1: the range's own start state, slot 0)
            const int f = i - 2;
            PllState q;
            PllCtx c{};
            state_before(f, q, c);
            exact(q, c, j0(f), j0(f) + NI);
            if (t == 0) {
                sst[f & 3][BPI - 1] = make_float2(q.integ, q.phase);
                sexact[f & 3] = 1;
                smiss[(i - 1) & 3] = 0;  // E2's verdict on the wrong interval i - 1
            }
            integ = q.integ;
            phase = q.phase;
            if (over && n >= kPllDemoteMinIntervals * NI &&  // demoted: the evaluators leave after B1.5,
                __builtin_amdgcn_ballot_w64(fabsf(q.phase) < kPllMaxPhase && fabsf(q.integ) < kPllMaxInteg) != 0) {
                                                               // pll_demoted_kernel runs the rest
                sdemote = 1;
                __syncthreads();  // B1.5
                demoted = true;
                qd = q;
                cd = c;
                jd = j0(f) + NI;
                break;
            }
            carry_exact((float)c.x, f + 1);
            __syncthreads();  // B1.5: the evaluators predict interval i anew from i - 2's end
            // interval i - 1 again on the fast chain: its candidates came from the phase at the
            // start of i - 2, which was right; E2 checks it again after B2
            run(i - 1);
            __syncthreads();  // B2: interval i's new candidates are in; E2 checks i - 1, the
                              // evaluators predict i + 1 from i - 1's end
            run(i);
            __syncthreads();  // B3
        }
        const unsigned long long p1 = PROF_T();
        __syncthreads();
        ch_body += p1 - p0;
        ch_wait += PROF_T() - p1;
    }
    PllState q;
    PllCtx c{};
    int f;  // the first interval the tail below runs exactly
    if (demoted) {  // the redone interval's exact end: pll_demoted_kernel runs the rest
        q = qd;
        c = cd;
        f = (int)(jd / NI) + 1;
        n_dem = (unsigned long long)(n - jd);
    } else {
        __syncthreads();  // E2's checks of the last two intervals
        // a miss in them: from the first missed interval on exactly; then the steps past the last
        // interval exactly, from the state at the end of the last good interval
        f = smiss[(ni - 1) & 3] ? ni - 1 : (smiss[ni & 3] ? ni : ni + 1);
        state_before(f, q, c);
        exact(q, c, j0(f), n);
    }
    if (t == 0) {
        S[0] = q.integ; S[1] = q.phase; S[2] = q.fbI; S[3] = q.fbQ; S[5] = q.trig;
        S[6] = __builtin_bit_cast(float, demoted ? (int)(n - jd) : 0);  // the steps left to pll_demoted_kernel, or 0
        // fmrx_debug_pll_stats: batches run; "resumed" only for the inject hook's forced redos
        // (the runner is exact by construction: its own redos of missed intervals are internal)
        if (stats) {
            const int fin = inj >= f ? 1 : 0;  // the hook's interval redone after the loop
            atomicAdd(stats, (n_inj + (unsigned long long)fin) * 3 * BPI);
            atomicAdd(stats + 1, (unsigned long long)nb);
        }
        // fmrx_debug_pll_redos: this stream's redone intervals and demoted steps
        if (redos) {  // by the range's trigOffset at its start (the wide 16-step form runs in any
                      // range from 2^20: launch_pll's short calls and long forms' tails)
            const int rg = pll_redo_range(trig0);
            atomicAdd(&redos[kPllRedoSlots * (size_t)s + rg], (unsigned)n_redo);
            atomicAdd(&redos[kPllRedoSlots * (size_t)s + 4 + rg], (unsigned)n_dem);
        }
    }
#ifdef FMRX_AB_PROF
    if (t == 0) {
        atomicAdd(&g_pipe_prof[0], ch_body);
        atomicAdd(&g_pipe_prof[1], ch_wait);
        atomicAdd(&g_pipe_prof[4], (unsigned long long)ni);
        atomicAdd(&g_pipe_prof[5], n_redo);
        if (s < kProfStreams) atomicAdd(&g_redo_stream[NI == 16 ? 0 : NC == 5 ? 1 : 2][s], (unsigned int)n_redo);
    }
#endif
    (void)ch_body;
    (void)ch_wait;
    (void)n_redo;
    (void)n_inj;
}


// A/B build only (make ab AB=-DFMRX_AB_NODEMOTE): the index and count runners without pll_demote's
// checks (timing of the locked path; an unlocked stream then redoes every interval)
#ifdef FMRX_AB_NODEMOTE
constexpr bool kAbNoDemote = true;
#else
constexpr bool kAbNoDemote = false;
#endif

// ---- pll_idx_kernel: one stream a workgroup of 1 + NW waves, trigOffset in [2^17, 2^20) ---------
//
// Below 2^20 trigArg's float grid (2^-8 .. 2^-5 rad) is finer than the phase moves in the two
// intervals between a prediction and its use, so three or five candidates miss; 16 to 64 do not
// (tools/pll_predict.cpp, profiles/r04/pll_predict_below_2_20.txt: 16-step intervals from the
// phase one interval back hit with 64 candidates on 0.9999+ of them in [2^17, 2^18), with 32 in
// [2^18, 2^19), with 16 in [2^19, 2^20); the [2^17, 2^18) form runs 32 (~0.99 of intervals hit,
// the misses redone: faster than 64 evaluations a step, profiles/r04/ab_idx17_nc32/)).  Compares
// against NC - 1 thresholds would cost the chain 2 (NC - 1) instructions a step, so here the chain forms the step's trigArg itself --
// float(P + (double)phase), filter.cpp:165, three instructions -- and turns it into a lane index:
// the NC candidates of a step c0 - NC/2 .. c0 + NC/2 - 1 sit in NC consecutive lanes of one VGPR
// row (64 / NC steps a row), so e = v_readlane(row, bits(trigArg) - base) with
// base = bits(c0) - NC/2 - the step's lane offset:
//   the chain (wave 0), per step: e from the previous trigArg's lane (v_readlane), (Ki e, Kp e),
//     the three float updates (filter.cpp:161-162), trigArg (cvt, add_f64, cvt), its lane index
//     (sub, v_readfirstlane), the index recorded in lane J of a row (v_writelane) -- 11 VALU a
//     step whatever NC is.  After the interval it tests the row (every index inside its step's
//     NC lanes) and the phase (not NaN: an uncertified candidate's e is NaN, so a chain that took
//     one carries NaN from there); a miss is redone on the exact path at once, from the state at
//     the interval's start (in registers), so it costs 16 exact steps and no pipeline restart: the
//     evaluators' next interval was predicted from the phase before the missed one, still right;
//   the evaluators (waves 1 .. NW, one SIMD each), per interval k: interval k + 1's candidate
//     rows (pred_e_cert for each lane's candidate, NaN where uncertified), P and base of each
//     step, from the phase at interval k's start; wave 1 also stores interval k - 1's trigArgs
//     (base + index: the candidate IS the trigArg) unless the chain redid it.
// So the runner is exact by construction, as pll_pipe_kernel: every e the chain used is a
// certified candidate's that is the true trigArg.  One launch runs a form's whole range of the
// call and leaves the exact end state in st.
template <int NC, int NW>
__global__ void __launch_bounds__(64 * (1 + NW)) __attribute__((amdgpu_waves_per_eu(1, 1)))
pll_idx_kernel(const float* io, int n, int n_streams, size_t stride, double step, float norm_bw, float* st,
               float* out_base, size_t ostride, int inject, int miss, float lo, float hi, unsigned long long* stats,
               unsigned* redos) {
    constexpr int NI = 16;          // steps an interval
    constexpr int SPP = 64 / NC;    // steps a candidate row
    constexpr int NR = NI / SPP;    // candidate rows an interval
    constexpr int HC = NC / 2;      // candidates c0 - HC .. c0 + HC - 1
    constexpr int RD = 4;           // intervals of step inputs in flight
    constexpr int NP = (NR + NW - 1) / NW;  // rows an evaluator wave computes
    static_assert(NC == 16 || NC == 32 || NC == 64, "a power of two dividing the wave");
    // rings of four intervals (interval k in slot k & 3): per step (P lo, P hi, base, -) (sp), the
    // candidate rows (se), the chain's lane index of each step's trigArg (srow), its (integ,
    // phase) at the interval's end (sst), "redone exactly" (sexact)
    __shared__ float4 sp[4][NI];
    __shared__ float se[4][NR][64];
    __shared__ int srow[4][NI];
    __shared__ float4 sst[4];  // (integ, phase, the verdict "redone exactly" as int bits, -)
    __shared__ int sexact[4];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    const int s = blockIdx.x;  // grid = n_streams
    const float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    float* S = st + 8 * (size_t)s;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    auto uni = [](float v) { return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v))); };
    PllState p{uni(S[0]), uni(S[1]), uni(S[2]), uni(S[3]), uni(S[5])};
    // demoted by an earlier runner launch of this call (pll_demote; state slot 6: the steps it left
    // to pll_demoted_kernel, int bits): this range is theirs too -- add it and leave (uniform)
    if (const int rem = __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, S[6])); rem > 0) {
        if (threadIdx.x == 0) {
            S[6] = __builtin_bit_cast(float, rem + n);
            if (redos) atomicAdd(&redos[kPllRedoSlots * (size_t)s + 4 + pll_redo_range(p.trig)], (unsigned)n);
        }
        return;
    }
    const bool in_domain = pll_pipe_stream(p.trig, step, lo, hi);
    const float trig0 = p.trig;
    const double t0d = (double)trig0;
    auto pr_at = [&](long long j) {
        return step * (double)(float)fmin(t0d + (double)(j + 1), (double)kPllTrigStick);
    };
    const int nb = n / NI;
    const int ni = nb;  // intervals 1 .. nb from the range's first step (the first predicted too)
    // test hook: a forced miss on interval 1 + (inject + s) % ni (counted as resumed)
    const int inj = inject >= 0 && ni > 0 ? 1 + (inject + s) % ni : -1;
    auto exact = [&](PllState& q, PllCtx& c, long long j0, long long j1) {
        if (j1 > j0) {
            const PllPair z = pll_redo(q, c, x + j0, out + j0, (int)(j1 - j0), Ki, Kp, step, true);
            q = z.p;
            c = z.ctx;
        }
    };
    if (ni < 2 || !in_domain) {
        if (w == 0) {
            PllCtx c{};
            c.valid = false;
            exact(p, c, 0, n);
            if (t == 0) {
                S[0] = p.integ; S[1] = p.phase; S[2] = p.fbI; S[3] = p.fbQ; S[5] = p.trig;
                S[6] = 0.0f;  // not demoted (pll_demoted_kernel)
                if (stats) {
                    if (!in_domain) atomicAdd(stats, (unsigned long long)nb);
                    atomicAdd(stats + 1, (unsigned long long)nb);
                }
            }
        }
        return;
    }
    auto j0 = [](int k) { return NI * (k - 1); };  // interval k's first step (k >= 1)

    if (w > 0) {
        // this wave's rows r = w - 1 + NW q; lane t: step J = r SPP + t / NC, candidate t % NC
        float vq[RD][NP];
        auto ld = [&](int k, float (&v)[NP]) {
            const int kk = k <= ni ? k : ni;
#pragma unroll
            for (int q = 0; q < NP; q++) {
                const int r = min(w - 1 + NW * q, NR - 1);
                const int j = j0(kk) + r * SPP + t / NC;
                v[q] = x[min(j + 1, n - 1)];  // the step the e is for
            }
        };
        auto put = [&](int k, float phase_ref, const float (&v)[NP]) {
            const int sl = k & 3;
#pragma unroll
            for (int q = 0; q < NP; q++) {
                const int r = w - 1 + NW * q;
                if (NP * NW > NR && r >= NR) break;
                const int J = r * SPP + t / NC, kc = t % NC;
                const int j = j0(k) + J;
                const double pr = pr_at(j);
                const uint32_t cb = __builtin_bit_cast(uint32_t, (float)(pr + (double)phase_ref));
                bool ok;
                const float e = pred_e_cert(__builtin_bit_cast(float, cb - (uint32_t)HC + (uint32_t)kc), v[q],
                                            pll_iv(v[q]), ok);
                // a candidate that is not a positive finite float never certifies: c0 < 2^126
                const bool fin = cb > (uint32_t)HC && cb < 0x7F000000u;
                se[sl][r][t] = ok && fin ? e : __builtin_nanf("");
                if (kc == 0) {
                    const uint64_t pb = __builtin_bit_cast(uint64_t, pr);
                    sp[sl][J] = make_float4(__builtin_bit_cast(float, (uint32_t)pb),
                                            __builtin_bit_cast(float, (uint32_t)(pb >> 32)),
                                            __builtin_bit_cast(float, cb - (uint32_t)HC - (uint32_t)(NC * (J % SPP))),
                                            0.0f);
                }
            }
        };
        // test hook pll_pipe_miss = -m (m >= 2): every interval from m - 1 on misses -- its step-0
        // base moved off the candidates, so the chain's lane index leaves the row (wave 1, lane 0)
        auto hook_poison = [&](int k) {
            if (miss <= -2 && k >= -miss - 1 && w == 1 && t == 0)
                reinterpret_cast<uint32_t*>(&sp[k & 3][0])[2] += 0x40000000u;
        };
        // wave 1: interval k's trigArgs, base + the chain's lane index (the chain stored a redone
        // interval itself)
        auto store = [&](int k) {
            if (w != 1) return;
            const int sl = k & 3;
            if (sexact[sl]) return;
            const int J = t & (NI - 1);
            const float a = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, sp[sl][J].z) + (uint32_t)srow[sl][J]);
            if (t < NI) out[j0(k) + J] = a;
        };
#pragma unroll
        for (int u = 0; u < RD; u++) ld(1 + u, vq[(1 + u) % RD]);
        put(1, p.phase, vq[1 % RD]);  // interval 1 from the start phase (its own start)
        hook_poison(1);
        ld(1 + RD, vq[1 % RD]);
        __syncthreads();  // (prologue)
        unsigned long long ev_body = 0, ev_wait = 0;
        // pll_demote is the chain's (its verdicts are at hand there, a few scalar ops an interval):
        // it may leave only after the last interval of one of these groups of RD, saying so in
        // that interval's state word (w); the evaluators look once a group, store that interval's
        // trigArgs and leave too, without another barrier (a test per interval cost the index forms
        // ~3 ns a step: the evaluators set their pace)
        bool left = false;
        for (int i0 = 1; i0 <= ni; i0 += RD) {
            unroll_ic(
                [&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    constexpr int sl = (2 + u) % RD;  // slot of interval i + 1
                    const int i = i0 + u;
                    if (i <= ni) {
                        const unsigned long long p0 = PROF_T();
                        // the chain's state at interval i's start
                        const float4 rs = sst[(i - 1) & 3];
                        if (i + 1 <= ni) {
                            put(i + 1, rs.y, vq[sl]);  // from the phase at interval i's start
                            hook_poison(i + 1);
                            ld(i + 1 + RD, vq[sl]);
                        }
                        store(i - 1);
                        const unsigned long long p1 = PROF_T();
                        __syncthreads();
                        ev_body += p1 - p0;
                        ev_wait += PROF_T() - p1;
                    }
                },
                std::make_integer_sequence<int, RD>{});
            // (at the group's end, not its start: a test skipped on the first group made LLVM peel
            // a whole group)
            if (!kAbNoDemote &&
                __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, sst[(i0 + RD - 1) & 3].w)) != 0) {
                store(i0 + RD - 1);
                left = true;
                break;
            }
        }
        if (!left) store(ni);
#ifdef FMRX_AB_PROF
        if (t == 0 && w == 1) {
            atomicAdd(&g_idx_prof[2], ev_body);
            atomicAdd(&g_idx_prof[3], ev_wait);
        }
#endif
        (void)ev_body;
        (void)ev_wait;
        return;
    }

    // ---- the chain
    // interval 1 starts at the range's first step, predicted from the start phase like every other
    // (until round 6 a whole interval ran first on the exact path, at ~400 ns a step)
    float integ = p.integ, phase = p.phase;
    // the carry: the candidate row value of the previous trigArg and its lane (SGPR); after an
    // exact stretch that trigArg's exact e in every lane
    float cE;
    uint32_t cL = 0;
    auto carry_exact = [&](float a, int k) {
        cE = exact_e(a, x[min(j0(k), n - 1)]);
        cL = 0;
    };
    cE = exact_e_fb(p.fbI, p.fbQ, x[0]);  // step 0's e from the state's feedback (every lane)
    if (t == 0) {
        // the start state; its verdict (z) reads as a hit (no prediction pll_demote counts), and
        // no i >= 2 test in the evaluators' loop (LLVM peels a whole unrolled iteration for one)
        sst[0] = make_float4(integ, phase, 0.0f, 0.0f);
        sexact[0] = 1;
    }
    __syncthreads();  // (prologue)
    // pll_demote: the chain's verdicts of its last 32 intervals (SGPR bits); past kPllDemoteMisses
    // misses it leaves after the interval (dem_i) and the demoted kernel runs the rest
    int dem_i = 0;
    uint32_t hist = 0;
    unsigned long long n_redo = 0, n_inj = 0, ch_body = 0, ch_wait = 0;
    const uint32_t off = (uint32_t)(NC * ((t & (NI - 1)) % SPP));  // lane t's step's lane offset
    // the last interval's verdict (SGPR); the start values are 0 but not constants to the compiler
    // (constants there made LLVM peel the first interval: a second copy of the chain loop)
    uint32_t prev_bad = n < 0 ? 1u : 0u;
    hist = n < 0 ? 1u : 0u;
    for (int i = 1; i <= ni; i++) {
        const unsigned long long p0 = PROF_T();
        const int is = i & 3;
        const float integ0 = integ, phase0 = phase;
        // the verdicts up to interval i - 1 decide whether the chain leaves after this one: scalar
        // work at the interval's start, off the chain's path (at its end it delayed the barrier)
        hist = (hist << 1) | prev_bad;
        // (and only from a state the demoted kernel's fast batches take: beyond their range every
        // interval misses for that reason alone, and the exact path is what runs either way; the
        // range test only then, the common path SALU work only)
        bool leave = false;
        if (!kAbNoDemote && i % RD == 0 && i < ni && n >= kPllDemoteMinIntervals * NI &&
            __builtin_popcount(hist) >= kPllDemoteMissesIdx)  // (scalar, nearly always false: a branch
            leave = __builtin_amdgcn_ballot_w64(fabsf(phase) < kPllMaxPhase && fabsf(integ) < kPllMaxInteg) != 0;
        // the interval's data before its steps (NI 16-byte broadcasts, NR row reads)
        float4 D[NI];
        float E[NR];
#pragma unroll
        for (int J = 0; J < NI; J++) D[J] = sp[is][J];
#pragma unroll
        for (int r = 0; r < NR; r++) E[r] = se[is][r][t];
        __builtin_amdgcn_sched_barrier(0);
        int row = 0;
        unroll_ic(
            [&](auto jc) {
                constexpr int J = decltype(jc)::value;
                // step J: e from the previous trigArg's candidate lane, filter.cpp:161-162
                const float e = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cE), cL));
                const float2v kv = float2v{Ki, Kp} * e;
                integ = integ + kv.x;
                phase = phase + (kv.y + integ);
                // trigArg (filter.cpp:165) and its lane in step J's candidate row
                const double P = __builtin_bit_cast(double, make_uint2(__builtin_bit_cast(uint32_t, D[J].x),
                                                                       __builtin_bit_cast(uint32_t, D[J].y)));
                const float a = (float)(P + (double)phase);
                cL = __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, a) - __builtin_bit_cast(uint32_t, D[J].z));
                cE = E[J / SPP];
                int rw = row;  // (a local: clang rejects a captured variable as an asm operand here)
                const uint32_t sl = cL;
                asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(rw) : "s"(sl), "i"(J));
                row = rw;
            },
            std::make_integer_sequence<int, NI>{});
        // the interval's verdict: every trigArg's lane inside its step's candidates, no NaN e
        // taken (the phase), the start state in pll_batch_fast's range; test hooks force misses
        const bool lane_bad = t < NI && (uint32_t)row - off >= (uint32_t)NC;
        // (one ballot over the lane test and the uniform ones: provably uniform, an SGPR -- the redo
        // branch scalar and pll_demote's history SALU work, no readfirstlane round trip)
        const bool bad = __builtin_amdgcn_ballot_w64(lane_bad || !(phase == phase) ||
                                                     !(fabsf(phase0) < kPllMaxPhase && fabsf(integ0) < kPllMaxInteg)) != 0 ||
                         i == min(miss, ni) || i == inj;
        if (bad) {  // uniform: redo the interval exactly from its start (the chain stores it)
            n_redo++;
            n_inj += i == inj ? 1 : 0;
            PllState q = p;  // interval 1: the range's start state as given
            PllCtx c{};
            c.valid = false;
            if (i > 1) {
                const float a = (float)(pr_at(j0(i) - 1) + (double)phase0);  // the trigArg before it
                pll_state_at(q, c, integ0, phase0, trig0, (long long)j0(i), a, DeviceLib{});
            }
            exact(q, c, j0(i), j0(i) + NI);
            integ = q.integ;
            phase = q.phase;
            carry_exact((float)c.x, i + 1);
        }
        if (t < NI) srow[is][t] = row;
        prev_bad = bad ? 1u : 0u;
        sst[is] = make_float4(integ, phase, __builtin_bit_cast(float, bad ? 1 : 0), __builtin_bit_cast(float, leave ? 1 : 0));
        sexact[is] = bad ? 1 : 0;
        const unsigned long long p1 = PROF_T();
        __syncthreads();
        ch_body += p1 - p0;
        ch_wait += PROF_T() - p1;
        if (leave) {  // (the evaluators leave after this interval's barrier too)
            dem_i = i;
            break;
        }
    }
#ifdef FMRX_AB_PROF
    if (t == 0) {
        atomicAdd(&g_idx_prof[0], ch_body);
        atomicAdd(&g_idx_prof[1], ch_wait);
        atomicAdd(&g_idx_prof[4], (unsigned long long)ni);
        atomicAdd(&g_idx_prof[5], n_redo);
        if (s < kProfStreams) atomicAdd(&g_redo_stream[3][s], (unsigned int)n_redo);
    }
#endif
    (void)ch_body;
    (void)ch_wait;
    // the steps past the last interval the chain ran exactly, from the end state -- or, demoted, the
    // exact state at jf and its step for pll_demoted_kernel (pll_demote.hip), which runs the rest
    const long long jf = j0((dem_i ? dem_i : ni) + 1);
    const unsigned long long n_dem = dem_i ? (unsigned long long)(n - jf) : 0ull;
    const float a = (float)(pr_at(jf - 1) + (double)phase);
    PllState q;
    PllCtx c{};
    pll_state_at(q, c, integ, phase, trig0, jf, a, DeviceLib{});
    if (n_dem == 0) exact(q, c, jf, n);
    if (t == 0) {
        S[0] = q.integ; S[1] = q.phase; S[2] = q.fbI; S[3] = q.fbQ; S[5] = q.trig;
        S[6] = __builtin_bit_cast(float, n_dem ? (int)(n - jf) : 0);  // the steps left to pll_demoted_kernel, or 0
        if (stats) {
            atomicAdd(stats, n_inj);  // "resumed": the inject hook's forced redos only
            atomicAdd(stats + 1, (unsigned long long)nb);
        }
        if (redos) {  // fmrx_debug_pll_redos: slot 0, [2^17, 2^20)
            atomicAdd(&redos[kPllRedoSlots * (size_t)s], (unsigned)n_redo);
            atomicAdd(&redos[kPllRedoSlots * (size_t)s + 4], (unsigned)n_dem);
        }
    }
}


// ---- pll_cnt_kernel: one stream a workgroup of 1 + NW waves; the chain picks e by a count --------
//
// The exact phase threshold of every candidate (phase_thr_exact: "trigArg >= c" is "phase >=
// T(c)", trigArg = float(P + (double)phase) being monotone in the float phase, filter.cpp:165)
// turns the candidate choice into ONE compare of the phase against a row of thresholds: lane l of
// step J's T row holds T(c_base + l) (l <= NC; +inf beyond), so the bits of the compare's mask
// are a prefix and their count is the trigArg's place in the window, plus one.  Lane l of the E
// row holds the e of candidate c_base + l - 1 (certified, NaN where not; lanes 0 and NC + 1 NaN:
// a trigArg below or above the window), so e = v_readlane(E, count) -- a compare, s_bcnt1 and a
// v_readlane whatever NC is (tools/ubench_cnt.hip mode 3: 60 cycles a step with the data in
// registers, against 91 for the index runner's f64 trigArg and lane index, mode 0).  So the
// window can be wide enough that a trigArg outside it is rare even for 64-step intervals
// predicted 64 to 128 steps ahead (tools/pll_predict.cpp, profiles/r04/g5/predict.txt).
//   the chain (wave 0), per step: e, (Ki e, Kp e), the three float updates (filter.cpp:161-162),
//     the compare and count, the count recorded in lane J of a row.  After the interval: a NaN
//     phase or carry e (a trigArg outside its window, an uncertified candidate) or a start state
//     out of the certified range redoes the interval on the exact path at once, from the state at
//     its start (the evaluators' next interval came from that state: no restart);
//   the evaluators (waves 1 .. NW), per interval k: interval k + 1's T and E rows from the phase
//     at interval k's start (c0 = float(P + phase_ref), c_base = c0 - NC / 2), items spread over
//     all their lanes; wave 1 also stores interval k - 1's trigArgs (c_base + count - 1: the
//     candidate IS the trigArg) unless the chain redid it.
// Exact by construction as pll_pipe_kernel / pll_idx_kernel.

// The smallest float phase f with float(P + (double)f) >= c (phase_thr's T), always found: when
// phase_thr's window of four neighbours does not hold it (rare), a bisection over the ordered
// float line (32 halvings; "reaches" is monotone in f).
__device__ inline uint32_t fkey(float f) {
    const uint32_t b = __builtin_bit_cast(uint32_t, f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ inline float fkey_inv(uint32_t k) {
    return __builtin_bit_cast(float, (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ inline float phase_thr_exact(double P, uint32_t cb) {
    const float T = phase_thr(P, cb);
    if (T > -__builtin_inff()) return T;
    const float c = __builtin_bit_cast(float, cb);
    uint32_t lo = fkey(-__builtin_inff()), hi = fkey(__builtin_inff());  // reaches(lo) false, (hi) true
    for (int it = 0; it < 34 && hi - lo > 1u; it++) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (reaches(P, fkey_inv(mid), c)) hi = mid;
        else lo = mid;
    }
    return fkey_inv(hi);
}

template <int NI, int NC, int NW>
__global__ void __launch_bounds__(64 * (1 + NW)) __attribute__((amdgpu_waves_per_eu(1, 1)))
pll_cnt_kernel(const float* io, int n, int n_streams, size_t stride, double step, float norm_bw, float* st,
               float* out_base, size_t ostride, int inject, int miss, float lo, float hi, unsigned long long* stats,
               unsigned* redos) {
    constexpr int NP = NC + 2;  // row slots: T(c_base + l) l <= NC, +inf | NaN, e(c_base + l - 1), NaN
    constexpr int HC = NC / 2;  // candidates c0 - HC .. c0 + HC
    constexpr int RD = 4;       // intervals of step inputs in flight
    constexpr int EV = 64 * NW;                    // evaluator lanes
    constexpr int NE = (NI * NC + EV - 1) / EV;    // e items a lane an interval
    constexpr int NT = (NI * (NC + 1) + EV - 1) / EV;  // threshold items a lane an interval
    constexpr int CH = NI < 16 ? NI : 16;          // the chain's steps a burst of reads
    static_assert(NC % 2 == 1 && NP <= 64, "an odd window within a wave");
    static_assert(NI == 16 || NI == 32 || NI == 64 || NI == 128, "the counts in one or two VGPR rows");
    constexpr int NRW = NI > 64 ? 2 : 1;  // rows of counts: step J in lane J & 63 of row J >> 6
    // rings of four intervals (interval k in slot k & 3): the T and E rows of each pair of steps
    // interleaved by row slot (sR[.][p][l] = T_2p(l), E_2p(l), T_2p+1(l), E_2p+1(l): one 16-byte
    // read a lane gives the chain two steps' rows), bits(c_base) - 1 of each step (the trigArg
    // store), the chain's count of each step, its (integ, phase) at the interval's end, "redone
    // exactly"
    __shared__ float4 sR[4][NI / 2][NP];
    auto sT = [&](int sl, int J, int l) -> float& { return reinterpret_cast<float*>(&sR[sl][J >> 1][l])[2 * (J & 1)]; };
    auto sE = [&](int sl, int J, int l) -> float& { return reinterpret_cast<float*>(&sR[sl][J >> 1][l])[2 * (J & 1) + 1]; };
    __shared__ uint32_t sbase[4][NI];
    __shared__ int srow[4][NI];
    __shared__ float4 sst[4];  // (integ, phase, the verdict "redone exactly" as int bits, -)
    __shared__ int sexact[4];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    const int s = blockIdx.x;  // grid = n_streams
    const float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    float* S = st + 8 * (size_t)s;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    auto uni = [](float v) { return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v))); };
    PllState p{uni(S[0]), uni(S[1]), uni(S[2]), uni(S[3]), uni(S[5])};
    // demoted by an earlier runner launch of this call (pll_demote; state slot 6: the steps it left
    // to pll_demoted_kernel, int bits): this range is theirs too -- add it and leave (uniform)
    if (const int rem = __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, S[6])); rem > 0) {
        if (threadIdx.x == 0) {
            S[6] = __builtin_bit_cast(float, rem + n);
            if (redos) atomicAdd(&redos[kPllRedoSlots * (size_t)s + 4 + pll_redo_range(p.trig)], (unsigned)n);
        }
        return;
    }
    const bool in_domain = pll_pipe_stream(p.trig, step, lo, hi);
    const float trig0 = p.trig;
    const double t0d = (double)trig0;
    auto pr_at = [&](long long j) {
        return step * (double)(float)fmin(t0d + (double)(j + 1), (double)kPllTrigStick);
    };
    const int nb = n / NI;
    const int ni = nb;  // intervals 1 .. nb from the range's first step (the first predicted too)
    // test hook: a forced miss on interval 1 + (inject + s) % ni (counted as resumed)
    const int inj = inject >= 0 && ni > 0 ? 1 + (inject + s) % ni : -1;
    auto exact = [&](PllState& q, PllCtx& c, long long j0, long long j1) {
        if (j1 > j0) {
            const PllPair z = pll_redo(q, c, x + j0, out + j0, (int)(j1 - j0), Ki, Kp, step, true);
            q = z.p;
            c = z.ctx;
        }
    };
    if (ni < 2 || !in_domain) {
        if (w == 0) {
            PllCtx c{};
            c.valid = false;
            exact(p, c, 0, n);
            if (t == 0) {
                S[0] = p.integ; S[1] = p.phase; S[2] = p.fbI; S[3] = p.fbQ; S[5] = p.trig;
                S[6] = 0.0f;  // not demoted (pll_demoted_kernel)
                if (stats) {  // in 16-step batches, as every runner counts
                    if (!in_domain) atomicAdd(stats, (unsigned long long)(n / kPllBatch));
                    atomicAdd(stats + 1, (unsigned long long)(n / kPllBatch));
                }
            }
        }
        return;
    }
    auto j0 = [](int k) { return NI * (k - 1); };  // interval k's first step (k >= 1)
    // the rows' constant slots, once: T slot NC + 1 = +inf (never counted), E slots 0 and NC + 1 NaN
    for (int q = threadIdx.x; q < 4 * NI; q += 64 * (1 + NW)) {
        sT(q / NI, q % NI, NC + 1) = __builtin_inff();
        sE(q / NI, q % NI, 0) = __builtin_nanf("");
        sE(q / NI, q % NI, NC + 1) = __builtin_nanf("");
    }

    if (w > 0) {
        const int el = (w - 1) * 64 + t;  // evaluator lane
        // item q of interval k: e item (J, kc) = (q / NC, q % NC), q = el + EV u (u < NE)
        float vq[RD][NE];
        auto ld = [&](int k, float (&v)[NE]) __attribute__((always_inline)) {
            const int kk = k <= ni ? k : ni;
#pragma unroll
            for (int u = 0; u < NE; u++) {
                const int q = min(el + EV * u, NI * NC - 1);
                v[u] = x[min(j0(kk) + q / NC + 1, n - 1)];  // the step the e is for
            }
        };
        auto put = [&](int k, float phase_ref, const float (&v)[NE]) __attribute__((always_inline)) {
            const int sl = k & 3;
#pragma unroll
            for (int u = 0; u < NE; u++) {
                const int q = el + EV * u;
                if (NE * EV > NI * NC && q >= NI * NC) break;
                const int J = q / NC, kc = q % NC;
                const double pr = pr_at(j0(k) + J);
                const uint32_t cb = __builtin_bit_cast(uint32_t, (float)(pr + (double)phase_ref));
                bool ok;
                const float e = pred_e_cert(__builtin_bit_cast(float, cb - (uint32_t)HC + (uint32_t)kc), v[u],
                                            pll_iv(v[u]), ok);
                // a window that is not of positive finite floats never certifies: c0 < 2^126
                const bool fin = cb > (uint32_t)HC && cb < 0x7F000000u;
                sE(sl, J, kc + 1) = ok && fin ? e : __builtin_nanf("");
            }
#pragma unroll
            for (int u = 0; u < NT; u++) {
                const int q = el + EV * u;
                if (NT * EV > NI * (NC + 1) && q >= NI * (NC + 1)) break;
                const int J = q / (NC + 1), kc = q % (NC + 1);
                const double pr = pr_at(j0(k) + J);
                const uint32_t cb = __builtin_bit_cast(uint32_t, (float)(pr + (double)phase_ref));
                sT(sl, J, kc) = phase_thr_exact(pr, cb - (uint32_t)HC + (uint32_t)kc);
                if (kc == 0) sbase[sl][J] = cb - (uint32_t)HC - 1u;
            }
        };
        // test hook pll_pipe_miss = -m (m >= 2): every interval from m - 1 on misses -- step 0's E row
        // NaN (the lanes of wave 1 that wrote it in put)
        auto hook_poison = [&](int k) {
            if (miss <= -2 && k >= -miss - 1 && w == 1 && t < NC) sE(k & 3, 0, t + 1) = __builtin_nanf("");
        };
        // wave 1: interval k's trigArgs, bits(c_base) - 1 + the chain's count (the chain stored a
        // redone interval itself)
        auto store = [&](int k) {
            if (w != 1) return;
            const int sl = k & 3;
            if (sexact[sl]) return;
#pragma unroll
            for (int r = 0; r < NRW; r++) {
                const int J = t + 64 * r;
                if (J < NI) out[j0(k) + J] = __builtin_bit_cast(float, sbase[sl][J] + (uint32_t)srow[sl][J]);
            }
        };
#pragma unroll
        for (int u = 0; u < RD; u++) ld(1 + u, vq[(1 + u) % RD]);
        put(1, p.phase, vq[1 % RD]);  // interval 1 from the start phase (its own start)
        hook_poison(1);
        ld(1 + RD, vq[1 % RD]);
        __syncthreads();  // (prologue)
        unsigned long long ev_body = 0, ev_wait = 0;
        // pll_demote is the chain's (its verdicts are at hand there, a few scalar ops an interval):
        // it may leave only after the last interval of one of these groups of RD, saying so in
        // that interval's state word (w); the evaluators look once a group, store that interval's
        // trigArgs and leave too, without another barrier (a test per interval cost the index forms
        // ~3 ns a step: the evaluators set their pace)
        bool left = false;
        for (int i0 = 1; i0 <= ni; i0 += RD) {
            unroll_ic(
                [&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    constexpr int sl = (2 + u) % RD;  // slot of interval i + 1
                    const int i = i0 + u;
                    if (i <= ni) {
                        const unsigned long long p0 = PROF_T();
                        // the chain's state at interval i's start
                        const float4 rs = sst[(i - 1) & 3];
                        if (i + 1 <= ni) {
                            put(i + 1, rs.y, vq[sl]);  // from the phase at interval i's start
                            hook_poison(i + 1);
                            ld(i + 1 + RD, vq[sl]);
                        }
                        store(i - 1);
                        const unsigned long long p1 = PROF_T();
                        __syncthreads();
                        ev_body += p1 - p0;
                        ev_wait += PROF_T() - p1;
                    }
                },
                std::make_integer_sequence<int, RD>{});
            // (at the group's end, not its start: a test skipped on the first group made LLVM peel
            // a whole group)
            if (!kAbNoDemote &&
                __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, sst[(i0 + RD - 1) & 3].w)) != 0) {
                store(i0 + RD - 1);
                left = true;
                break;
            }
        }
        if (!left) store(ni);
#ifdef FMRX_AB_PROF
        if (t == 0 && w == 1) {
            atomicAdd(&g_cnt_prof[2], ev_body);
            atomicAdd(&g_cnt_prof[3], ev_wait);
        }
#endif
        (void)ev_body;
        (void)ev_wait;
        return;
    }

    // ---- the chain
    // interval 1 starts at the range's first step, predicted from the start phase like every other
    // (until round 6 a whole interval ran first on the exact path, at ~400 ns a step)
    float integ = p.integ, phase = p.phase;
    // the carry: the E row of the previous trigArg and its count (SGPR); after an exact stretch
    // that trigArg's exact e in every lane
    float cE;
    uint32_t cC = 1;
    auto carry_exact = [&](float a, int k) {
        cE = exact_e(a, x[min(j0(k), n - 1)]);
        cC = 1;
    };
    cE = exact_e_fb(p.fbI, p.fbQ, x[0]);  // step 0's e from the state's feedback (every lane)
    if (t == 0) {
        // the start state; its verdict (z) reads as a hit (no prediction pll_demote counts), and
        // no i >= 2 test in the evaluators' loop (LLVM peels a whole unrolled iteration for one)
        sst[0] = make_float4(integ, phase, 0.0f, 0.0f);
        sexact[0] = 1;
    }
    __syncthreads();  // (prologue)
    // pll_demote: the chain's verdicts of its last 32 intervals (SGPR bits); past kPllDemoteMisses
    // misses it leaves after the interval (dem_i) and the demoted kernel runs the rest
    int dem_i = 0;
    uint32_t hist = 0;
    unsigned long long n_redo = 0, n_inj = 0, ch_body = 0, ch_wait = 0;
    const int ls = t < NP ? t : NP - 1;  // this lane's row slot (lanes past the row read its last)
    // the last interval's verdict (SGPR); the start values are 0 but not constants to the compiler
    // (constants there made LLVM peel the first interval: a second copy of the chain loop)
    uint32_t prev_bad = n < 0 ? 1u : 0u;
    hist = n < 0 ? 1u : 0u;
    for (int i = 1; i <= ni && dem_i == 0; i++) {
        const unsigned long long p0 = PROF_T();
        const int is = i & 3;
        const float integ0 = integ, phase0 = phase;
        // the verdicts up to interval i - 1 decide whether the chain leaves after this one: scalar
        // work at the interval's start, off the chain's path (at its end it delayed the barrier)
        hist = (hist << 1) | prev_bad;
        // (and only from a state the demoted kernel's fast batches take: beyond their range every
        // interval misses for that reason alone, and the exact path is what runs either way; the
        // range test only then, the common path SALU work only)
        bool leave = false;
        if (!kAbNoDemote && i % RD == 0 && i < ni && n >= kPllDemoteMinIntervals * NI &&
            __builtin_popcount(hist) >= kPllDemoteMisses)  // (scalar, nearly always false: a branch
            leave = __builtin_amdgcn_ballot_w64(fabsf(phase) < kPllMaxPhase && fabsf(integ) < kPllMaxInteg) != 0;
        int row[NRW] = {};
        unroll_ic(
            [&](auto hc) {
                constexpr int H = decltype(hc)::value;
                // the burst's rows before its steps
                float T[CH], E[CH];
#pragma unroll
                for (int J = 0; J < CH; J += 2) {
                    const float4 r = sR[is][(H * CH + J) / 2][ls];
                    T[J] = r.x;
                    E[J] = r.y;
                    T[J + 1] = r.z;
                    E[J + 1] = r.w;
                }
                __builtin_amdgcn_sched_barrier(0);
                unroll_ic(
                    [&](auto jc) {
                        constexpr int J = decltype(jc)::value;
                        // step H CH + J: e of the previous trigArg (filter.cpp:161-162)
                        const float e = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cE), cC));
                        const float2v kv = float2v{Ki, Kp} * e;
                        integ = integ + kv.x;
                        phase = phase + (kv.y + integ);
                        // the count of thresholds the phase reaches: trigArg's place in the window + 1
                        cC = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(phase >= T[J]));
                        cE = E[J];
                        int rw = row[(H * CH + J) >> 6];
                        const uint32_t sc = cC;
                        asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(rw) : "s"(sc), "i"((H * CH + J) & 63));
                        row[(H * CH + J) >> 6] = rw;
                    },
                    std::make_integer_sequence<int, CH>{});
            },
            std::make_integer_sequence<int, NI / CH>{});
        // the interval's verdict: no NaN e taken (the phase) or carried (the last trigArg's), the
        // start state in pll_batch_fast's range; test hooks force misses
        const float ce = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cE), cC));
        // (one ballot: provably uniform, an SGPR -- the redo branch scalar, pll_demote's history SALU)
        const bool bad = __builtin_amdgcn_ballot_w64(!(phase == phase) || !(ce == ce) ||
                                                     !(fabsf(phase0) < kPllMaxPhase && fabsf(integ0) < kPllMaxInteg)) != 0 ||
                         i == min(miss, ni) || i == inj;
        if (bad) {  // uniform: redo the interval exactly from its start (the chain stores it)
            n_redo++;
            n_inj += i == inj ? 1 : 0;
            PllState q = p;  // interval 1: the range's start state as given
            PllCtx c{};
            c.valid = false;
            if (i > 1) {
                const float a = (float)(pr_at(j0(i) - 1) + (double)phase0);  // the trigArg before it
                pll_state_at(q, c, integ0, phase0, trig0, (long long)j0(i), a, DeviceLib{});
            }
            exact(q, c, j0(i), j0(i) + NI);
            integ = q.integ;
            phase = q.phase;
            carry_exact((float)c.x, i + 1);
        }
#pragma unroll
        for (int r = 0; r < NRW; r++)
            if (t + 64 * r < NI) srow[is][t + 64 * r] = row[r];
        prev_bad = bad ? 1u : 0u;
        sst[is] = make_float4(integ, phase, __builtin_bit_cast(float, bad ? 1 : 0), __builtin_bit_cast(float, leave ? 1 : 0));
        sexact[is] = bad ? 1 : 0;
        const unsigned long long p1 = PROF_T();
        __syncthreads();
        ch_body += p1 - p0;
        ch_wait += PROF_T() - p1;
        if (leave) dem_i = i;  // (the evaluators leave after this interval's barrier too)
    }
#ifdef FMRX_AB_PROF
    if (t == 0) {
        atomicAdd(&g_cnt_prof[0], ch_body);
        atomicAdd(&g_cnt_prof[1], ch_wait);
        atomicAdd(&g_cnt_prof[4], (unsigned long long)ni);
        atomicAdd(&g_cnt_prof[5], n_redo);
    }
#endif
    (void)ch_body;
    (void)ch_wait;
    // the steps past the last interval the chain ran exactly, from the end state -- or, demoted, the
    // exact state at jf and its step for pll_demoted_kernel (pll_demote.hip), which runs the rest
    const long long jf = j0((dem_i ? dem_i : ni) + 1);
    const unsigned long long n_dem = dem_i ? (unsigned long long)(n - jf) : 0ull;
    const float a = (float)(pr_at(jf - 1) + (double)phase);
    PllState q;
    PllCtx c{};
    pll_state_at(q, c, integ, phase, trig0, jf, a, DeviceLib{});
    if (n_dem == 0) exact(q, c, jf, n);
    if (t == 0) {
        S[0] = q.integ; S[1] = q.phase; S[2] = q.fbI; S[3] = q.fbQ; S[5] = q.trig;
        S[6] = __builtin_bit_cast(float, n_dem ? (int)(n - jf) : 0);  // the steps left to pll_demoted_kernel, or 0
        if (stats) {  // in 16-step batches, as every runner counts
            atomicAdd(stats, n_inj * (NI / kPllBatch));  // "resumed": the inject hook's forced redos only
            atomicAdd(stats + 1, (unsigned long long)(n / kPllBatch));
        }
        if (redos) {  // fmrx_debug_pll_redos, by the range's trigOffset
            atomicAdd(&redos[kPllRedoSlots * (size_t)s + pll_redo_range(lo)], (unsigned)n_redo);
            atomicAdd(&redos[kPllRedoSlots * (size_t)s + 4 + pll_redo_range(lo)], (unsigned)n_dem);
        }
    }
}

}  // namespace

#ifdef FMRX_AB_PROF
static void print_pred_prof();
static void reg_pred_prof() {
    static const bool reg = [] { return std::atexit(print_pred_prof) == 0; }();
    (void)reg;
}
static void print_pred_prof() {
    unsigned long long h[6] = {};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pred_prof), sizeof h) == hipSuccess && h[4])
        std::fprintf(stderr, "pll_pred prof: batches %llu chain body %.1f wait %.1f, evaluator body %.1f wait %.1f "
                     "(shader cycles per batch)\n", h[4], (double)h[0] / h[4], (double)h[1] / h[4],
                     (double)h[2] / h[4], (double)h[3] / h[4]);
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_cnt_prof), sizeof h) == hipSuccess && h[4])
        std::fprintf(stderr, "pll_cnt prof: intervals %llu chain body %.1f wait %.1f, evaluator body %.1f wait %.1f "
                     "(shader cycles per interval), %llu redos\n", h[4], (double)h[0] / h[4], (double)h[1] / h[4],
                     (double)h[2] / h[4], (double)h[3] / h[4], h[5]);
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_idx_prof), sizeof h) == hipSuccess && h[4])
        std::fprintf(stderr, "pll_idx prof: intervals %llu chain body %.1f wait %.1f, evaluator body %.1f wait %.1f "
                     "(shader cycles per interval), %llu redos\n", h[4], (double)h[0] / h[4], (double)h[1] / h[4],
                     (double)h[2] / h[4], (double)h[3] / h[4], h[5]);
    static unsigned int rs[4][kProfStreams];
    if (hipMemcpyFromSymbol(rs, HIP_SYMBOL(g_redo_stream), sizeof rs) == hipSuccess) {
        const char* names[4] = {"pipe 16-step", "pipe 64-step five", "pipe three", "index"};
        for (int f = 0; f < 4; f++) {
            unsigned long long tot = 0;
            unsigned int mx = 0;
            int n = 0, arg = -1;
            for (int k = 0; k < kProfStreams; k++) {
                tot += rs[f][k];
                if (rs[f][k]) n++;
                if (rs[f][k] > mx) { mx = rs[f][k]; arg = k; }
            }
            if (tot)
                std::fprintf(stderr, "redos per stream, %s: total %llu over %d streams, max %u (stream %d)\n", names[f],
                             tot, n, mx, arg);
        }
    }
    unsigned long long mr[3] = {};
    if (hipMemcpyFromSymbol(mr, HIP_SYMBOL(g_miss_reason), sizeof mr) == hipSuccess && (mr[0] | mr[1] | mr[2]))
        std::fprintf(stderr, "pll_pipe missed steps: trigArg outside the candidates %llu, e uncertified %llu, "
                     "threshold outside its window %llu\n", mr[0], mr[1], mr[2]);
    unsigned long long h2[4] = {};
    (void)hipMemcpyFromSymbol(h2, HIP_SYMBOL(g_pipe_prof_w2), sizeof h2);
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pipe_prof), sizeof h) == hipSuccess && h[4])
        std::fprintf(stderr, "pll_pipe prof: wave 2 body %.1f wait %.1f, of the body its data %.1f and its check %.1f "
                     "(shader cycles per interval)\n", (double)h2[0] / h[4], (double)h2[1] / h[4], (double)h2[2] / h[4],
                     (double)h2[3] / h[4]);
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pipe_prof), sizeof h) == hipSuccess && h[4])
        std::fprintf(stderr, "pll_pipe prof: intervals %llu chain body %.1f wait %.1f, evaluator body %.1f wait %.1f "
                     "(shader cycles per interval), %llu redos\n", h[4], (double)h[0] / h[4], (double)h[1] / h[4],
                     (double)h[2] / h[4], (double)h[3] / h[4], h[5]);
}
#endif

void launch_pll_pred(int waves, hipStream_t s, const float* io, int n, int n_streams, int spw, size_t stride,
                     const double* side, size_t seg, double step, float norm_bw, const float* st, float* out,
                     size_t ostride, int* fail, float2* rec, size_t rb, int inject, int sat_ok, int pipe_on) {
#ifdef FMRX_AB_PROF
    reg_pred_prof();
#endif
    hipLaunchKernelGGL(pll_pred_kernel<kPllBatch>, dim3(waves), dim3(128), 0, s, io, n, n_streams, spw, stride, side,
                       seg, step, norm_bw, st, out, ostride, fail, rec, rb, inject, sat_ok, pipe_on);
}

#ifndef FMRX_STICK_BPI
#define FMRX_STICK_BPI 16  // batches an interval of the stick form: 256-step intervals (8: 128, 4: 64)
#endif
#ifndef FMRX_PIPE22_BPI
#define FMRX_PIPE22_BPI 16  // batches an interval of the three-candidate form below the stick (256 steps)
#endif
#ifndef FMRX_PIPE21_BPI
#define FMRX_PIPE21_BPI 8  // batches an interval of the five-candidate [2^21, 2^22) form (128 steps)
#endif
#ifndef FMRX_PIPE_RD
#define FMRX_PIPE_RD 8  // intervals of step inputs in flight (the evaluators' loop is unrolled by it)
#endif
void launch_pll_pipe(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step, float norm_bw,
                     float* st, float* out, size_t ostride, int inject, int miss, int form,
                     unsigned long long* stats, unsigned* redos) {
#ifdef FMRX_AB_PROF
    reg_pred_prof();
#endif
    if (n <= 0) return;
    if (form == 25)  // short calls from 2^22: three candidates in 128-step intervals (640 = 5 of them)
        hipLaunchKernelGGL((pll_pipe_kernel<kPllBatch, 8, FMRX_PIPE_RD, 3>), dim3(n_streams), dim3(192), 0, s, io, n,
                           n_streams, stride, step, norm_bw, st, out, ostride, inject, miss, stats, redos);
    else if (form == 24)  // the short-call form: any trigOffset from 2^20, 16-step intervals
        hipLaunchKernelGGL((pll_pipe_kernel<kPllBatch, 1, FMRX_PIPE_RD, 5, false, true>), dim3(n_streams), dim3(192), 0, s,
                           io, n, n_streams, stride, step, norm_bw, st, out, ostride, inject, miss, stats, redos);
    else if (form == 23)
        hipLaunchKernelGGL((pll_pipe_kernel<kPllBatch, FMRX_STICK_BPI, FMRX_PIPE_RD, 3, true>), dim3(n_streams), dim3(192), 0, s, io, n,
                           n_streams, stride, step, norm_bw, st, out, ostride, inject, miss, stats, redos);
    else if (form == 22)
        hipLaunchKernelGGL((pll_pipe_kernel<kPllBatch, FMRX_PIPE22_BPI, FMRX_PIPE_RD, 3>), dim3(n_streams), dim3(192), 0, s, io, n, n_streams,
                           stride, step, norm_bw, st, out, ostride, inject, miss, stats, redos);
    else if (form == 21)
        hipLaunchKernelGGL((pll_pipe_kernel<kPllBatch, FMRX_PIPE21_BPI, FMRX_PIPE_RD, 5>), dim3(n_streams), dim3(192), 0, s, io, n, n_streams,
                           stride, step, norm_bw, st, out, ostride, inject, miss, stats, redos);
    else
        hipLaunchKernelGGL((pll_pipe_kernel<kPllBatch, 1, FMRX_PIPE_RD, 5>), dim3(n_streams), dim3(192), 0, s, io, n, n_streams,
                           stride, step, norm_bw, st, out, ostride, inject, miss, stats, redos);
}

#ifndef FMRX_IDX17_NC
#define FMRX_IDX17_NC 32
#endif
#ifndef FMRX_IDX18_NC
#define FMRX_IDX18_NC 32
#endif
#ifndef FMRX_IDX_NW
#define FMRX_IDX_NW 4  // evaluator waves of the 32-candidate forms: two rows of candidates each
                       // (three waves: three rows, evaluator-bound; profiles/r04/ab_idx_nw4/)
#endif

// A form's workgroup must be resident on one CU for its waves to run side by side (the chain
// spins on barriers with its evaluators): checked once per kernel against the compiled register
// and LDS use, so a build that outgrows it fails loudly instead of serialising.
template <int NC, int NW>
static int idx_launch(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step,
                      float norm_bw, float* st, float* out, size_t ostride, int inject, int miss, float lo, float hi,
                      unsigned long long* stats, unsigned* redos) {
    constexpr int threads = 64 * (1 + NW);
    static const int resident = [] {
        int nb = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pll_idx_kernel<NC, NW>, threads, 0) == hipSuccess
                   ? nb : 0;
    }();
    if (resident < 1) return -1;
    hipLaunchKernelGGL((pll_idx_kernel<NC, NW>), dim3(n_streams), dim3(threads), 0, s, io, n, n_streams, stride, step,
                       norm_bw, st, out, ostride, inject, miss, lo, hi, stats, redos);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_pll_idx(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step, float norm_bw,
                   float* st, float* out, size_t ostride, int inject, int miss, int form, unsigned long long* stats,
                   unsigned* redos) {
#ifdef FMRX_AB_PROF
    reg_pred_prof();
#endif
    if (n <= 0) return 0;
    if (form == 17)
        return idx_launch<FMRX_IDX17_NC, FMRX_IDX_NW>(s, io, n, n_streams, stride, step, norm_bw, st, out, ostride,
                                                      inject, miss, 131072.0f, 262143.0f, stats, redos);
    if (form == 18)
        return idx_launch<FMRX_IDX18_NC, FMRX_IDX_NW>(s, io, n, n_streams, stride, step, norm_bw, st, out, ostride,
                                                      inject, miss, 262144.0f, 524287.0f, stats, redos);
    return idx_launch<16, 3>(s, io, n, n_streams, stride, step, norm_bw, st, out, ostride, inject, miss, 524288.0f,
                             1048575.0f, stats, redos);
}

// The count runner's forms (form: the trigOffset range as launch_pll numbers it), one stream a
// workgroup of 1 + NW waves (a CU), residency checked like idx_launch.
template <int NI, int NC, int NW>
static int cnt_launch(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step,
                      float norm_bw, float* st, float* out, size_t ostride, int inject, int miss, float lo, float hi,
                      unsigned long long* stats, unsigned* redos) {
    constexpr int threads = 64 * (1 + NW);
    static const int resident = [] {
        int nb = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pll_cnt_kernel<NI, NC, NW>, threads, 0) == hipSuccess
                   ? nb : 0;
    }();
    if (resident < 1) return -1;
    hipLaunchKernelGGL((pll_cnt_kernel<NI, NC, NW>), dim3(n_streams), dim3(threads), 0, s, io, n, n_streams, stride,
                       step, norm_bw, st, out, ostride, inject, miss, lo, hi, stats, redos);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

#ifndef FMRX_CNT19_NI
#define FMRX_CNT19_NI 64  // steps an interval of the [2^19, 2^20) count form
#endif
#ifndef FMRX_CNT20_NI
#define FMRX_CNT20_NI 128  // steps an interval of the [2^20, 2^21) count form (two rows of counts)
#endif
#ifndef FMRX_CNT_NW
#define FMRX_CNT_NW 4  // evaluator waves of the [2^19, 2^21) count forms
#endif
#ifndef FMRX_CNT17_NI
#define FMRX_CNT17_NI 16  // steps an interval of the [2^17, 2^19) count forms (off by default)
#endif
#ifndef FMRX_CNT17_NW
#define FMRX_CNT17_NW 4  // their evaluator waves
#endif
int pll_form_interval(int form, bool cnt) {
    if (cnt) return form <= 18 ? FMRX_CNT17_NI : form == 19 ? FMRX_CNT19_NI : form == 20 ? FMRX_CNT20_NI : 64;
    if (form < 20) return 16;  // the index runner
    if (form == 25) return kPllBatch * 8;
    return form == 20 || form == 24 ? kPllBatch : form == 21 ? kPllBatch * FMRX_PIPE21_BPI
         : form == 22 ? kPllBatch * FMRX_PIPE22_BPI : kPllBatch * FMRX_STICK_BPI;
}

int launch_pll_cnt(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step, float norm_bw,
                   float* st, float* out, size_t ostride, int inject, int miss, int form, unsigned long long* stats,
                   unsigned* redos) {
#ifdef FMRX_AB_PROF
    reg_pred_prof();
#endif
    if (n <= 0) return 0;
    switch (form) {
        case 17:
            return cnt_launch<FMRX_CNT17_NI, 31, FMRX_CNT17_NW>(s, io, n, n_streams, stride, step, norm_bw, st, out, ostride, inject, miss,
                                         131072.0f, 262143.0f, stats, redos);
        case 18:
            return cnt_launch<FMRX_CNT17_NI, 31, FMRX_CNT17_NW>(s, io, n, n_streams, stride, step, norm_bw, st, out, ostride, inject, miss,
                                         262144.0f, 524287.0f, stats, redos);
        case 19:
            return cnt_launch<FMRX_CNT19_NI, 15, FMRX_CNT_NW>(s, io, n, n_streams, stride, step, norm_bw, st, out, ostride, inject, miss,
                                         524288.0f, 1048575.0f, stats, redos);
        case 20:
            return cnt_launch<FMRX_CNT20_NI, 15, FMRX_CNT_NW>(s, io, n, n_streams, stride, step, norm_bw, st, out, ostride, inject, miss,
                                         kPllPipeMinLow, kPllPipeMin5 - 1.0f, stats, redos);
        default:  // three waves a stream, as the three-wave runner it would replace
            return cnt_launch<64, 7, 2>(s, io, n, n_streams, stride, step, norm_bw, st, out, ostride, inject, miss,
                                        kPllPipeMin5, kPllPipeMin - 1.0f, stats, redos);
    }
}

}  // namespace fmrx
