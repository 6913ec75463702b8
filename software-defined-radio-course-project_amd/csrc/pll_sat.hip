// pll_sat.hip — the speculative PLL runner for saturated segments (src/filter.cpp:157-171 once
// trigOffset has stuck at 2^24, filter.cpp:165-166), one stream a wave.
//
// From 2^24 samples on (69.9 s at 240 kS/s) the reference's float trigOffset no longer moves,
// so trigArg = float(step 2^24 + phase) only changes when the phase crosses its grid: on ~7 %
// of steps of the bench stream, half of the moves 1-2 steps apart, the rest after 9-64 repeats
// (tools/pll_runs.cpp, profiles/r02/pll_sat_runs.txt).  While trigArg repeats, the feedback
// (fc, nfs, sn, cs) and the two atan2 offsets -B(x, 0), -B(x, 1/2) stay fixed, so a step's
// error e_j = float(Y(v_j) / v_j - B(x, h_j)) does not depend on the loop state: lane l of the
// 16-lane row computes (Ki e, Kp e) of step l of a batch for all 16 steps at once, and the
// serial chain per step is one row broadcast of that pair, the three float updates, trigArg
// and the repeat test.  When trigArg moves, the sin/cos and offsets are refreshed (lanes 0/1
// sin/cos, lanes 2/3 the offsets, pll_spec_lane_kernel's shared reduction) and the pairs of the
// batch recomputed.  Half turn h_j = 1/2 [iv_j < 0]: iv's sign bit.  The output (trigArgs and
// batch records) is checked by pll_check_kernel exactly like the other runners'.
//
// Its own translation unit: built without the SLP vectorizer (Makefile), which would pair the
// float updates of neighbouring steps into packed ops (each read back after a wait state, with
// register moves around them) -- while the other kernels of stereo.hip gain from it.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "dsp_device.h"
#include "fmrx_internal.h"
#include "pll_device.h"
#include "pll_math.h"

namespace fmrx {

namespace {

template <int NB>
__global__ void __launch_bounds__(256) pll_sat_kernel(const float* io, int n, int n_streams, int spw, size_t stride,
                                                     const double* side, size_t seg, double step, float norm_bw,
                                                     const float* st, float* out_base, size_t ostride, int* fail,
                                                     float2* rec, size_t rb, int inject) {
    const int t = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int s_lane = wave * spw + ((t >> 4) & (spw - 1));
    const bool owner = (t & 15) == 0 && (t >> 4) < spw && s_lane < n_streams;
    const SplitCoef sc = split_coef((t & 1) != 0);
    const int s = s_lane < n_streams ? s_lane : n_streams - 1;
    const float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    const float* S = st + 8 * (size_t)s;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    PllState p{S[0], S[1], S[2], S[3], S[5]};
    if (!pll_sat_segment(spw, p.trig, step)) return;  // pll_spec_lane_kernel's
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
    const double prd = step * (double)kPllTrigStick;  // pll_side's step x trigOffset, stuck
    const int l = t & 15;
    const bool off = l == 2 || l == 3;
    const double C1 = off ? kInv2Pi : kInvPio2;
    const double Chi = off ? k2PiHi : kPio2Hi;
    const double Clo = off ? k2PiLo : kPio2Lo;
    const double Hc = l == 2 ? 0.5 : 0.0;  // lane 2 -B(x, 1/2), lane 3 -B(x, 0)
    const double* ivs = side + (size_t)s * seg;
    const int q0 = ctx.q;
    const float u0 = (q0 & 1) ? p.fbQ : p.fbI, w0 = (q0 & 1) ? p.fbI : -p.fbQ;
    float fc = (q0 & 2) ? -u0 : u0, nfs = (q0 & 2) ? -w0 : w0;
    double sn = ctx.sn, cs = ctx.cs;
    double nB0 = -pll_offset_h(ctx.x, 0.0), nB1 = -pll_offset_h(ctx.x, 0.5);
    float integ = p.integ, phase = p.phase;
    uint32_t prev = __builtin_bit_cast(uint32_t, (float)ctx.x);
    // (Ki e, Kp e) of this lane's step from the current feedback
    auto ke_of = [&](float vl, double ivl) -> double {
        const float2v ab = float2v{fc, nfs} * vl;
        const double Y = fma((double)ab.x, sn, (double)ab.y * cs);
        const uint64_t ib = __builtin_bit_cast(uint64_t, ivl);
        const uint64_t m = (uint64_t)(uint32_t)((int)(uint32_t)(ib >> 32) >> 31) * 0x100000001ull;
        const double nB = __builtin_bit_cast(double, (m & __builtin_bit_cast(uint64_t, nB1)) |
                                                         (~m & __builtin_bit_cast(uint64_t, nB0)));
        const float e = (float)fma(Y, ivl, -nB);
        return __builtin_bit_cast(double, float2v{Ki, Kp} * e);
    };
    // fresh feedback and offsets from trigArg a (lanes 0/1 sin/cos, lanes 2/3 the offsets)
    auto refresh = [&](uint32_t a_bits) {
        const double xa = (double)__builtin_bit_cast(float, a_bits);
        const double tq = rint(fma(xa, C1, Hc)) - Hc;
        const double w = fma(-tq, Clo, fma(-tq, Chi, xa));
        nB1 = row_bcast<2>(w);
        nB0 = row_bcast<3>(w);
        const double W = split_w_horner(w * w, sc);
        sn = row_bcast<0>(w * W);
        cs = row_bcast<1>(W);
        fc = (float)cs;
        nfs = -(float)sn;
    };
    // the moved flag of the last step computed, tested with the next pair (see below)
    uint64_t moved = 0;
    // one batch; vb, ivb: this lane's step data (step l of the batch)
    auto batch = [&](int b, float vb, double ivb) __attribute__((always_inline)) {
        double ke = ke_of(vb, ivb);
        float o[NB];
        // step J from (integ, phase, trigArg bits) i0, p0, a0: the new state and the moved flag
        auto step_at = [&](auto jc, float i0, float p0, uint32_t a0, float& i1, float& p1, uint32_t& a1,
                           uint64_t& m1) {
            constexpr int J = decltype(jc)::value;
            // integ + Ki e, then phase + (Kp e + integ) (filter.cpp:162-164)
            const float2v k = __builtin_bit_cast(float2v, row_bcast<J>(ke));
            i1 = i0 + k.x;
            p1 = p0 + (k.y + i1);
            const float arg = (float)(prd + (double)p1);
            o[J] = arg;
            a1 = __builtin_bit_cast(uint32_t, arg);
            m1 = __builtin_amdgcn_ballot_w64(a1 != a0);
        };
        // Steps in pairs (e, o) = (2k, 2k + 1); after each pair, one branch on the moved
        // flags of steps e - 1 and e (made at least a step earlier: a branch on a compare
        // just made waits ~40 cycles for it).  A move at e - 1 leaves e and o computed with
        // the old pairs, a move at e leaves o: both are redone after the refresh; the flag
        // of o goes to the next pair's test.
        unroll_ic(
            [&](auto kc) {
                constexpr int e = 2 * decltype(kc)::value;
                const std::integral_constant<int, e> ec{};
                const std::integral_constant<int, e + 1> oc{};
                const float iP = integ, pP = phase;
                const uint32_t aP = prev;
                float iQ, pQ;
                uint32_t aQ;
                uint64_t mQ;
                step_at(ec, iP, pP, aP, iQ, pQ, aQ, mQ);
                uint64_t mR;
                step_at(oc, iQ, pQ, aQ, integ, phase, prev, mR);
                if (__builtin_expect((moved | mQ) != 0, 0)) {
                    if (moved != 0) {  // trigArg moved at e - 1: e and o are stale
                        refresh(aP);
                        ke = ke_of(vb, ivb);
                        step_at(ec, iP, pP, aP, iQ, pQ, aQ, mQ);
                    }
                    if (mQ != 0) {  // moved at e: o is stale
                        refresh(aQ);
                        ke = ke_of(vb, ivb);
                    }
                    step_at(oc, iQ, pQ, aQ, integ, phase, prev, mR);
                }
                moved = mR;
            },
            std::make_integer_sequence<int, NB / 2>{});
        phase += (inject >= 0 && b == 1 + (inject + s) % (nb - 1)) ? 1.0e-3f : 0.0f;  // test hook
        float* ob = out + b * NB;
#pragma unroll
        for (int q = 0; q < NB / 4; q++)
            reinterpret_cast<float4*>(ob)[q] = *reinterpret_cast<const float4*>(&o[4 * q]);
        rec[(size_t)s * rb + b] = make_float2(integ, phase);
    };
    // The lane's step data is loaded about three batches ahead (a batch here is ~800
    // cycles, shorter than a load from HBM): ring slot u serves batches 1 + u (mod 4) and is
    // refilled at the end of its batch, after its last read, so the load lands in place.
    float vq[4];
    double ivq[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int bq = 1 + u < nb ? 1 + u : nb - 1;
        vq[u] = x[bq * NB + l];
        ivq[u] = ivs[bq * NB + l];
    }
    // landed before the loop: the loop top then waits only for the slot it reads (a load
    // issued last here would make the waitcnt pass wait for every load at each iteration)
    __builtin_amdgcn_s_waitcnt(0);
    int b0 = 1;
    for (; b0 + 3 < nb; b0 += 4) {
        unroll_ic(
            [&](auto uc) {
                constexpr int u = decltype(uc)::value;
                batch(b0 + u, vq[u], ivq[u]);
                const int bq = b0 + u + 4 < nb ? b0 + u + 4 : nb - 1;
                vq[u] = x[bq * NB + l];
                ivq[u] = ivs[bq * NB + l];
            },
            std::make_integer_sequence<int, 4>{});
    }
    for (; b0 < nb; b0++) batch(b0, x[b0 * NB + l], ivs[b0 * NB + l]);
}

}  // namespace

void launch_pll_sat(dim3 grid, dim3 block, hipStream_t s, const float* io, int n, int n_streams, int spw,
                    size_t stride, const double* side, size_t seg, double step, float norm_bw, const float* st,
                    float* out, size_t ostride, int* fail, float2* rec, size_t rb, int inject) {
    hipLaunchKernelGGL(pll_sat_kernel<kPllBatch>, grid, block, 0, s, io, n, n_streams, spw, stride, side, seg, step,
                       norm_bw, st, out, ostride, fail, rec, rb, inject);
}

}  // namespace fmrx
