// pll_pred.hip — the speculative PLL runner with predicted trigArgs (src/filter.cpp:157-171), for
// segments from trigOffset 2^20 up to the 2^24 stick; streams by 16-lane row (spw <= 4), like
// pll_spec_lane_kernel.
//
// trigArg_j = float(P_j + phase_j) with P_j = 2 pi (f/Fs) trigOffset_j in double (pll_side's pr).
// From 2^20 steps on, P_j's float grid is 2^-5 rad or coarser (2^-2 from 2^22) while the phase
// moves by |Kp e + integ| < 0.05 rad a step and stays within a few radians: a candidate formed
// ahead of the chain from an EARLIER phase, c0 = float(P_j + phase_ref), is within one float of
// the true trigArg on 99 % of the steps below 2^22 and on every step of the bench stream above
// (tools/pll_predict.cpp, phase_ref two batches back).  So the feedback of each
// step -- sin, cos and the atan2 offset of trigArg_j, which the NEXT step's error needs --
// does not have to wait for the serial chain: lane l of a row evaluates, for step l of a batch,
// the next step's (Ki e, Kp e) for the three candidates c0 - 1, c0, c0 + 1 ulp, in parallel over
// the row, one batch ahead of the chain (the phase at the start of batch b is phase_ref for
// batch b + 1, so the evaluation interleaves with batch b's steps).  The serial step is then:
//   row broadcasts of lane j-1's three pairs and c0 (off the chain), d = bits(trigArg) - bits(c0),
//   the pair of candidate d (two selects), integ += Ki e, phase += Kp e + integ,
//   trigArg = float(P_j + phase).
// A step whose trigArg is not a candidate (|d| > 1) sets the batch's miss flag; the batch is then
// redone from its start with the same steps, each miss evaluating its pair directly (uniform loads
// of the step's input, sin and cos in every lane).  The per-step arithmetic is
// pll_spec_lane_kernel's (e = float(fma(Y, 1/v, B)), the same sin/cos polynomials and offsets),
// and the output -- trigArgs and the per-batch (integ, phase) records -- is checked by
// pll_check_kernel exactly like every runner's, so the result is the certified path's bit for bit
// whatever was predicted.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "dsp_device.h"
#include "fmrx_internal.h"
#include "pll_device.h"
#include "pll_math.h"

namespace fmrx {

namespace {

template <int L>
__device__ inline uint32_t row_bcast32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + L, 0xF, 0xF, false);
}

// (Ki e, Kp e) of a step (input v, 1/v = iv, half turn h = 0.5 [v < 0]) whose previous trigArg is
// a: pll_spec_lane_kernel's step with both sin and cos in this lane.  Returned as a double's bits.
__device__ inline double pred_ke(float a, float v, double iv, float Ki, float Kp) {
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
    const float e = (float)fma(Y, iv, B);
    return __builtin_bit_cast(double, float2v{Ki, Kp} * e);
}

// the three candidates of one step's trigArg and the next step's pair for each
struct Cand {
    double pm, p0, pp;  // pairs for trigArg = c0 - 1 ulp, c0, c0 + 1 ulp
    uint32_t cb;        // bits of c0
};

__device__ inline Cand pred_eval(float phase_ref, double pr, float v, double iv, float Ki, float Kp) {
    const float c0 = (float)(pr + (double)phase_ref);
    const uint32_t cb = __builtin_bit_cast(uint32_t, c0);
    Cand c;
    c.pm = pred_ke(__builtin_bit_cast(float, cb - 1u), v, iv, Ki, Kp);
    c.p0 = pred_ke(c0, v, iv, Ki, Kp);
    c.pp = pred_ke(__builtin_bit_cast(float, cb + 1u), v, iv, Ki, Kp);
    c.cb = cb;
    return c;
}

template <int NB>
__global__ void __launch_bounds__(256) pll_pred_kernel(const float* io, int n, int n_streams, int spw, size_t stride,
                                                      const double* side, size_t seg, double step, float norm_bw,
                                                      const float* st, float* out_base, size_t ostride, int* fail,
                                                      float2* rec, size_t rb, int inject) {
    const int t = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int s_lane = wave * spw + ((t >> 4) & (spw - 1));
    const bool owner = (t & 15) == 0 && (t >> 4) < spw && s_lane < n_streams;
    const int s = s_lane < n_streams ? s_lane : n_streams - 1;
    const int l = t & 15;
    const float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    const float* S = st + 8 * (size_t)s;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    PllState p{S[0], S[1], S[2], S[3], S[5]};
    if (!pll_pred_wave(p.trig, step)) return;  // pll_spec_lane_kernel's (or pll_sat_kernel's)
    const int nb = n / NB;
    if (owner) fail[s] = nb;
    PllCtx ctx{};
    ctx.valid = false;
    if (nb > 0) {  // batch 0 on the exact path (see pll_spec_kernel)
        const PllPair r = pll_redo(p, ctx, x, out, NB, Ki, Kp, step, s_lane < n_streams);
        p = r.p;
        ctx = r.ctx;
        if (owner) rec[(size_t)s * rb] = make_float2(p.integ, p.phase);
    }
    if (nb < 2) return;
    // side data, stream-major (pll_prep_major_kernel): 1/v and pr planes
    const double* ivs = side + (size_t)s * seg;
    const double* prs = side + seg * (size_t)n_streams + (size_t)s * seg;
    float integ = p.integ, phase = p.phase;
    uint32_t tb = __builtin_bit_cast(uint32_t, (float)ctx.x);  // trigArg of the last step done
    // step 0 of batch 1: its pair from the known trigArg (all three slots alike)
    Cand carry;
    carry.p0 = pred_ke((float)ctx.x, x[NB], ivs[NB], Ki, Kp);
    carry.pm = carry.pp = carry.p0;
    carry.cb = tb;
    // this lane's data for batch b: pr of step l, and the input of step l + 1 (the step its
    // candidates' pairs are for; the segment's last sample stands in past the end)
    auto ld = [&](int b, float& v, double& iv, double& pr) {
        const int jn = min(b * NB + l + 1, n - 1);
        v = x[jn];
        iv = ivs[jn];
        pr = prs[b * NB + l];
    };
    float v1, v2;
    double iv1, iv2, pr1, pr2;
    ld(1, v1, iv1, pr1);
    ld(2 < nb ? 2 : nb - 1, v2, iv2, pr2);
    Cand cur = pred_eval(phase, pr1, v1, iv1, Ki, Kp);  // batch 1 from the phase after batch 0
    double prc = pr1;                                    // pr of step l of the current batch
    float vn = v2;
    double ivn = iv2, prn = pr2;
    for (int b = 1; b < nb; b++) {
        // batch b + 1's candidates from the phase at the start of batch b (two batches back)
        const Cand nxt = pred_eval(phase, prn, vn, ivn, Ki, Kp);
        const double prnx = prn;
        {  // refill for batch b + 2 (its candidates are evaluated during batch b + 1)
            const int bq = b + 2 < nb ? b + 2 : nb - 1;
            ld(bq, vn, ivn, prn);
        }
        const float integ0 = integ, phase0 = phase;
        const uint32_t tb0 = tb;
        float o[NB];
        uint32_t miss = 0;
        // step J: the pair of candidate bits(trigArg_{J-1}) - c0 of lane J - 1 (batch b - 1's
        // lane 15: the carry, for J = 0)
        unroll_ic(
            [&](auto jc) {
                constexpr int J = decltype(jc)::value;
                double pm, p0, pp;
                uint32_t cb;
                if constexpr (J == 0) {
                    pm = carry.pm;
                    p0 = carry.p0;
                    pp = carry.pp;
                    cb = carry.cb;
                } else {
                    pm = row_bcast<J - 1>(cur.pm);
                    p0 = row_bcast<J - 1>(cur.p0);
                    pp = row_bcast<J - 1>(cur.pp);
                    cb = row_bcast32<J - 1>(cur.cb);
                }
                const double prj = row_bcast<J>(prc);
                const int d = (int)(tb - cb);
                const double pk = d == 0 ? p0 : (d < 0 ? pm : pp);
                miss |= (uint32_t)(d + 1) > 2u ? 1u : 0u;
                const float2v k = __builtin_bit_cast(float2v, pk);
                integ = integ + k.x;
                phase = phase + (k.y + integ);
                const float arg = (float)(prj + (double)phase);
                o[J] = arg;
                tb = __builtin_bit_cast(uint32_t, arg);
            },
            std::make_integer_sequence<int, NB>{});
        if (__builtin_expect(miss != 0, 0)) {
            // a trigArg outside its candidates: redo the batch, evaluating such steps' pairs
            // directly (rows without a miss are masked off here)
            integ = integ0;
            phase = phase0;
            tb = tb0;
            const int j0 = b * NB;
            unroll_ic(
                [&](auto jc) {
                    constexpr int J = decltype(jc)::value;
                    double pm, p0, pp;
                    uint32_t cb;
                    if constexpr (J == 0) {
                        pm = carry.pm;
                        p0 = carry.p0;
                        pp = carry.pp;
                        cb = carry.cb;
                    } else {
                        pm = row_bcast<J - 1>(cur.pm);
                        p0 = row_bcast<J - 1>(cur.p0);
                        pp = row_bcast<J - 1>(cur.pp);
                        cb = row_bcast32<J - 1>(cur.cb);
                    }
                    const double prj = row_bcast<J>(prc);
                    const int d = (int)(tb - cb);
                    double pk = d == 0 ? p0 : (d < 0 ? pm : pp);
                    if ((uint32_t)(d + 1) > 2u)
                        pk = pred_ke(__builtin_bit_cast(float, tb), x[j0 + J], ivs[j0 + J], Ki, Kp);
                    const float2v k = __builtin_bit_cast(float2v, pk);
                    integ = integ + k.x;
                    phase = phase + (k.y + integ);
                    const float arg = (float)(prj + (double)phase);
                    o[J] = arg;
                    tb = __builtin_bit_cast(uint32_t, arg);
                },
                std::make_integer_sequence<int, NB>{});
        }
        phase += (inject >= 0 && b == 1 + (inject + s) % (nb - 1)) ? 1.0e-3f : 0.0f;  // test hook
        // every lane stores (rows of one stream hold the same values; see pll_spec_lane_kernel)
        float* ob = out + b * NB;
#pragma unroll
        for (int q = 0; q < NB / 4; q++)
            reinterpret_cast<float4*>(ob)[q] = *reinterpret_cast<const float4*>(&o[4 * q]);
        rec[(size_t)s * rb + b] = make_float2(integ, phase);
        // lane 15's candidates are those of step 0 of batch b + 1
        carry.pm = row_bcast<NB - 1>(cur.pm);
        carry.p0 = row_bcast<NB - 1>(cur.p0);
        carry.pp = row_bcast<NB - 1>(cur.pp);
        carry.cb = row_bcast32<NB - 1>(cur.cb);
        cur = nxt;
        prc = prnx;
    }
}

}  // namespace

void launch_pll_pred(dim3 grid, dim3 block, hipStream_t s, const float* io, int n, int n_streams, int spw,
                     size_t stride, const double* side, size_t seg, double step, float norm_bw, const float* st,
                     float* out, size_t ostride, int* fail, float2* rec, size_t rb, int inject) {
    hipLaunchKernelGGL(pll_pred_kernel<kPllBatch>, grid, block, 0, s, io, n, n_streams, spw, stride, side, seg, step,
                       norm_bw, st, out, ostride, fail, rec, rb, inject);
}

}  // namespace fmrx
