// pll_demote.hip — the PLL (src/filter.cpp:157-171) of a stream a self-certifying runner demoted.
//
// The runners of pll_pred.hip select each step's e among candidates predicted from the phase one
// or two intervals back.  On an unlocked loop (no pilot, heavy noise, random bytes; the PLL of
// modes 2 and 3, which the reference hands the upsampled if_fs, project.cpp:166,348,357) the phase
// moves many candidate cells an interval, nearly every interval misses and is redone on the exact
// path: ~400 ns a step (profiles/r06/unlocked.json, before this kernel).  pll_demote (pll_device.h)
// makes a runner leave the rest of its range to this kernel once 24 of its last 32 intervals
// missed; the runner writes the exact state at that step to st and the step to st slot 6.
//
// One stream a workgroup of four waves:
//   the chain (wave 0) runs the recurrence speculatively with pll_spec_lane_kernel's step (sin and
//     cos as one polynomial on lane pairs, the atan2 offset on lane 2 of each 16-lane row, no
//     certification: ~37 VALU a step), sub-segment after sub-segment of kDemSB batches, storing
//     every trigArg (out, and the LDS ring) and the (integ, phase) at the end of every batch;
//   the checkers (waves 1-3), one sub-segment behind, recompute each batch of the sub-segment the
//     chain ran last exactly -- one lane a batch, from the state the chain recorded before it,
//     pll_batch_fast certified or pll_step -- and compare the trigArgs and the end state bit for
//     bit (pll_check_kernel's test); two sub-segments ahead they form the chain's side data (1/v
//     as reciprocal + Newton, P = step x trigOffset) into a ring of four.
// A batch that does not verify: the chain recomputes its sub-segment exactly from that batch on
// (the first failing batch's start state was verified) and runs the sub-segment after it again.
// So the output is the exact path's bit for bit, and the chain runs at the speculative runner's
// pace instead of the certified step's.  Two barriers a sub-segment: A (the checkers' verdicts
// are in) and B (the chain's orders for the next sub-segment are in).
#include <hip/hip_runtime.h>

#include <climits>

#include "dsp_device.h"
#include "fmrx_internal.h"
#include "pll_device.h"
#include "pll_math.h"

namespace fmrx {
namespace {

// the helpers inlined (466 VGPRs, the runners' 16 B of scratch; unlocked streams 70-78 ns a step
// against 76-78 out of line, profiles/r06/demote_probe/r06v_*) -- or, A/B build FMRX_AB_DEM_NOINLINE,
// out of line (their frames on the stack: 528 B of scratch a lane)
#ifdef FMRX_AB_DEM_NOINLINE
#define FMRX_DEM_FN __device__ __noinline__
#else
#define FMRX_DEM_FN __device__ __attribute__((always_inline))
#endif
constexpr int kDemNB = kPllBatch;       // steps a batch (verified as one)
constexpr int kDemSB = 16;              // batches a sub-segment
constexpr int kDemL = kDemNB * kDemSB;  // steps a sub-segment
#ifndef FMRX_DEM_W
#define FMRX_DEM_W 2  // (4 until the r06 A/B: the same speed; half the CU to wait for at dispatch)
#endif
constexpr int kDemW = FMRX_DEM_W;       // waves: the chain and the checkers

__device__ inline double dem_iv(float v) {  // pll_check_kernel's 1/v (pll_side's NaN outside the range)
    const double vd = (double)v;
    const double r0 = __builtin_amdgcn_rcp(vd);
    const double r1 = fma(r0, fma(-vd, r0, 1.0), r0);
    return (fabs(vd) >= (double)kPllMinV && fabs(vd) < 1.0e300) ? r1 : (double)NAN;
}

// n exact steps from (p, ctx): certified kDemNB-step batches with the side data formed inline, a
// batch that does not certify redone with pll_step (pll_redo) from its start.  Every lane of the
// wave runs this stream (the chain), lane parity picking sin or cos.  Outside the trigOffset domain
// pll_side assumes (integer-valued, <= 2^24): pll_redo throughout.
FMRX_DEM_FN PllPair pll_run_fast(PllState p, PllCtx ctx, const float* xb, float* ob, int n, float Ki,
                                             float Kp, double step) {
    constexpr int NB = kDemNB;
    const SplitCoef sc = split_coef((threadIdx.x & 1) != 0);
    int j = 0;
    if (pll_trig_domain(p.trig)) {
#pragma unroll 1
        for (; j + NB <= n; j += NB) {
            float v[NB], o[NB];
            double iv[NB], pr[NB];
            const double t0d = (double)p.trig;
#pragma unroll
            for (int u = 0; u < NB; u++) {
                v[u] = xb[j + u];
                iv[u] = dem_iv(v[u]);
                pr[u] = step * fmin(t0d + (double)(u + 1), (double)kPllTrigStick);
            }
            const PllState p0 = p;
            const PllCtx c0 = ctx;
            if (fabs(pr[NB - 1]) < kPllMaxPr && pll_batch_fast<NB, true>(p, ctx, v, iv, pr, o, Ki, Kp, [](int) {}, sc)) {
#pragma unroll
                for (int u = 0; u < NB; u++) ob[j + u] = o[u];
            } else {
                const PllPair r = pll_redo(p0, c0, xb + j, ob + j, NB, Ki, Kp, step, true);
                p = r.p;
                ctx = r.ctx;
            }
        }
    }
    if (j < n) {
        const PllPair r = pll_redo(p, ctx, xb + j, ob + j, n - j, Ki, Kp, step, true);
        p = r.p;
        ctx = r.ctx;
    }
    return PllPair{p, ctx};
}

// the state before step k of the range from (integ, phase) after step k - 1 and that step's
// trigArg a (pll_state_at: fbI, fbQ and the context from the exact sin/cos of a)
FMRX_DEM_FN PllPair dem_state(float integ, float phase, float t0, int k, float a) {
    PllPair r;
    r.ctx = PllCtx{};
    pll_state_at(r.p, r.ctx, integ, phase, t0, (long long)k, a, DeviceLib{});
    return r;
}

// One checker lane: batch b of a sub-segment whose first step is J0, from (integ, phase, a) before
// it; tg: the chain's trigArgs of the batch, (ei, ep) its end state.  True when they are exact.
FMRX_DEM_FN bool dem_verify(const float* x, int J, float integ, float phase, float a, float t0, double step,
                                       float Ki, float Kp, const float* tg, float ei, float ep) {
    constexpr int NB = kDemNB;
    PllPair z = dem_state(integ, phase, t0, J, a);
    PllState p = z.p;
    PllCtx c = z.ctx;
    float v[NB], o[NB];
    double iv[NB], pr[NB];
    const double t0d = (double)t0;
#pragma unroll
    for (int u = 0; u < NB; u++) {
        v[u] = x[J + u];
        iv[u] = dem_iv(v[u]);
        pr[u] = step * fmin(t0d + (double)(J + u + 1), (double)kPllTrigStick);
    }
    bool same = true;
    const PllState p0 = p;
    const PllCtx c0 = c;
    if (fabs(pr[NB - 1]) < kPllMaxPr && pll_batch_fast<NB, false>(p, c, v, iv, pr, o, Ki, Kp, [](int) {})) {
#pragma unroll
        for (int u = 0; u < NB; u++) same &= __float_as_uint(o[u]) == __float_as_uint(tg[u]);
    } else {
        p = p0;
        c = c0;
        const DeviceLib lib;
        for (int u = 0; u < NB; u++) {
            const float aa = pll_step(p, c, v[u], Ki, Kp, step, lib);
            same &= __float_as_uint(aa) == __float_as_uint(tg[u]);
        }
    }
    return same && __float_as_uint(p.integ) == __float_as_uint(ei) && __float_as_uint(p.phase) == __float_as_uint(ep);
}

#ifndef FMRX_DEM_WPE
#define FMRX_DEM_WPE 1  // waves a SIMD the register budget allows (A/B: 2 = 256 VGPRs, co-resident with stage kernels)
#endif
__global__ void __launch_bounds__(64 * kDemW) __attribute__((amdgpu_waves_per_eu(FMRX_DEM_WPE, FMRX_DEM_WPE)))
pll_demoted_kernel(const float* io, int n, size_t stride, double step, float norm_bw, float* st, float* out_base,
                   size_t ostride, int inject, unsigned long long* stats) {
    constexpr int NB = kDemNB, SB = kDemSB, L = kDemL;
    const int s = blockIdx.x;
    // the steps the call's runner launches left to this kernel, up to the end of its range (state
    // slot 6, int bits; 0 none): launch_pll queues it once, after them, over the call's runner ranges
    const int rem = __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, st[8 * (size_t)s + 6]));
    if (rem <= 0 || rem >= n) return;  // not demoted (uniform: no barrier reached)
    const int j0 = n - rem;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    const float* x = io + (size_t)s * stride + j0;  // the demoted rest of the range: steps [0, m)
    float* out = out_base + (size_t)s * ostride + j0;
    float* S = st + 8 * (size_t)s;
    const int m = n - j0;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    auto uni = [](float v) { return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v))); };
    const float t0 = uni(S[5]);  // trigOffset after the step before the range
    const double t0d = (double)t0;
    const int nbt = m / NB;                      // whole batches (the rest: exact, at the end)
    const int nsub = (nbt + SB - 1) / SB;        // sub-segments
    auto nbat = [&](int g) { return min(SB, nbt - g * SB); };
    // side data ring (sub-segment g in slot g & 3), the chain's trigArgs and batch end states
    // (sub-segment g in slot g & 1) and its start (integ, phase, the trigArg before it)
    // (side data of step u: v, 1/v, P, and the half turn 0.5 [v < 0] in groups (h_u, h_u+1, 0, 0) of
    // two steps -- lane 2 of each row reads the pair, the row's other lanes the zeros beside it)
    __shared__ __attribute__((aligned(16))) float sv[4][L];
    __shared__ double siv[4][L], spr[4][L], shz[4][2 * L];
    __shared__ __attribute__((aligned(16))) float starg[2][L];
    __shared__ float2 srec[2][SB];
    __shared__ float4 sstart[2];
    __shared__ int sfail[2];
    __shared__ int sctl[5];  // orders: run, verify, side (sub-segments, -1 none), done, a second side (prologue)

    if (w > 0) {
        const int cl = (w - 1) * 64 + t;  // checker lane
        auto side = [&](int g) {
            if (g < 0) return;
            for (int u = cl; u < L; u += 64 * (kDemW - 1)) {
                const int j = g * L + u;
                const bool in = j < m;
                const float v = in ? x[j] : 0.0f;
                const double iv = in ? dem_iv(v) : 0.0;
                sv[g & 3][u] = v;
                siv[g & 3][u] = iv;
                spr[g & 3][u] = in ? step * fmin(t0d + (double)(j + 1), (double)kPllTrigStick) : 0.0;
                shz[g & 3][4 * (u >> 1) + (u & 1)] = iv < 0.0 ? 0.5 : 0.0;
                shz[g & 3][4 * (u >> 1) + 2 + (u & 1)] = 0.0;
            }
        };
        auto verify = [&](int g) {
            if (g < 0 || cl >= nbat(g)) return;
            const int b = cl, sl = g & 1;
            float integ, phase, a;
            if (b == 0) {
                const float4 z = sstart[sl];
                integ = z.x;
                phase = z.y;
                a = z.z;
            } else {
                const float2 z = srec[sl][b - 1];
                integ = z.x;
                phase = z.y;
                a = starg[sl][b * NB - 1];
            }
            float tg[NB];
#pragma unroll
            for (int u = 0; u < NB; u++) tg[u] = starg[sl][b * NB + u];
            const float2 e = srec[sl][b];
            const int J = g * L + b * NB;
            if (dem_verify(x, J, integ, phase, a, t0, step, Ki, Kp, tg, e.x, e.y)) {
                // the output (a batch after a failed one is rewritten by the chain after barrier A)
#pragma unroll
                for (int u = 0; u < NB; u++) out[J + u] = tg[u];
            } else {
                atomicMin(&sfail[sl], b);
            }
        };
        __syncthreads();  // B (prologue): the first orders
        side(sctl[2]);
        side(sctl[4]);
        __syncthreads();  // A
#pragma unroll 1
        for (;;) {
            __syncthreads();  // B: this sub-segment's orders
            const int run = __builtin_amdgcn_readfirstlane(sctl[0]);
            const int ver = __builtin_amdgcn_readfirstlane(sctl[1]);
            const int sd = __builtin_amdgcn_readfirstlane(sctl[2]);
            if (__builtin_amdgcn_readfirstlane(sctl[3])) return;
            (void)run;
            side(sd);
            verify(ver);
            __syncthreads();  // A: the verdicts are in
        }
    }

    // ---- the chain
    const bool b_lane = (t & 15) == 2;
    const SplitCoef sc = split_coef((t & 1) != 0);
    const double C1 = b_lane ? kInv2Pi : kInvPio2;
    const double Chi = b_lane ? k2PiHi : kPio2Hi;
    const double Clo = b_lane ? k2PiLo : kPio2Lo;
    // the exact state at the range's start (the runner's), its trigArg a = float(P + phase)
    float integ = uni(S[0]), phase = uni(S[1]);
    float a_prev = (float)(step * t0d + (double)phase);
    PllState pe{integ, phase, uni(S[2]), uni(S[3]), t0};
    PllCtx ce{};
    {
        float sv, cv;
        if (!sincos_ctx_f(a_prev, &sv, &cv, &ce)) DeviceLib{}.sincosf_(a_prev, &sv, &cv);
    }
    bool init = true;  // the chain's registers from (pe, ce) before its next sub-segment
    float fc = 0.0f, nfs = 0.0f;
    double sn = 0.0, cs = 0.0, nB = 0.0;
    bool injected = inject < 0;  // test hook (knob pll_inject): one wrong batch, then a rollback
    const int inj_b = inject >= 0 && nbt > 1 ? 1 + inject % (nbt - 1) : -1;
    unsigned long long n_roll = 0;
    if (t == 0) {
        sctl[0] = -1;
        sctl[1] = -1;
        sctl[2] = 0;
        sctl[3] = 0;
        sctl[4] = nsub > 1 ? 1 : -1;
    }
    __syncthreads();  // B (prologue)
    __syncthreads();  // A
    int r = 0, vp = -1;
    // the step data of one batch in registers (pll_spec_lane_kernel's one register set, refilled
    // with the next batch's right after each step consumed its own)
    float v[NB];
    double iv[NB], pr[NB], hz[NB];
    const int hoff = b_lane ? 0 : 2;  // lane 2 reads the half turns, the others the zeros beside them
    auto ld_v = [&](int s4, int u, int q) {
        *reinterpret_cast<float4*>(&v[4 * q]) = reinterpret_cast<const float4*>(&sv[s4][u])[q];
    };
    auto ld_d = [&](int s4, int u, int q) {
        *reinterpret_cast<double2*>(&iv[2 * q]) = reinterpret_cast<const double2*>(&siv[s4][u])[q];
        *reinterpret_cast<double2*>(&pr[2 * q]) = reinterpret_cast<const double2*>(&spr[s4][u])[q];
        *reinterpret_cast<double2*>(&hz[2 * q]) = *reinterpret_cast<const double2*>(&shz[s4][2 * u + 4 * q + hoff]);
    };
    auto ld_batch = [&](int g, int b) {
        const int s4 = g & 3, u = b * NB;
#pragma unroll
        for (int q = 0; q < NB / 4; q++) ld_v(s4, u, q);
#pragma unroll
        for (int q = 0; q < NB / 2; q++) ld_d(s4, u, q);
    };
    int loaded = -1;  // the sub-segment whose batch 0 is in the registers
    auto run_sub = [&](int g) {
        const int sl = g & 1, nbg = nbat(g);
        if (loaded != g) ld_batch(g, 0);
        if (init) {
            const int q0 = ce.q;
            const float u0 = (q0 & 1) ? pe.fbQ : pe.fbI, w0 = (q0 & 1) ? pe.fbI : -pe.fbQ;
            fc = (q0 & 2) ? -u0 : u0;
            nfs = (q0 & 2) ? -w0 : w0;
            sn = ce.sn;
            cs = ce.cs;
            nB = -pll_offset_h(ce.x, iv[0] < 0.0 ? 0.5 : 0.0);
            integ = pe.integ;
            phase = pe.phase;
            init = false;
        }
        sstart[sl] = make_float4(integ, phase, a_prev, 0.0f);
#pragma unroll 1
        for (int b = 0; b < nbg; b++) {
            // the next batch: this sub-segment's, or the first of the next (formed two ahead)
            const int gn = b + 1 < nbg ? g : g + 1, un = b + 1 < nbg ? (b + 1) * NB : 0, s4n = gn & 3;
            float o[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const float2v ab = float2v{fc, nfs} * v[j];
                const double Y = fma((double)ab.x, sn, (double)ab.y * cs);
                const float e = (float)fma(Y, iv[j], -nB);
                const float ki_e = Ki * e;
                const float kp_e = Kp * e;
                integ = integ + ki_e;
                phase = phase + (kp_e + integ);
                const float arg = (float)(pr[j] + (double)phase);
                o[j] = arg;
                const double xa = (double)arg;
                const double H = hz[(j + 1) % NB];  // the next step's half turn on lane 2, else 0
                const double tq = rint(fma(xa, C1, H)) - H;
                const double wv = fma(-tq, Clo, fma(-tq, Chi, xa));  // r, or -B on lane 2
                nB = row_bcast<2>(wv);
                const double W = split_w_horner(wv * wv, sc);
                sn = row_bcast<0>(wv * W);
                cs = row_bcast<1>(W);
                fc = (float)cs;
                nfs = -(float)sn;
                // refill after step j: v[j], iv[j], pr[j] and hz[j] (read at step j - 1) are dead
                if (j % 4 == 3) ld_v(s4n, un, j / 4);
                if (j % 2 == 1) ld_d(s4n, un, j / 2);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (!injected && g * SB + b == inj_b) {  // test hook: a wrong batch (its check fails)
                phase += 1.0e-3f;
                injected = true;
            }
#pragma unroll
            for (int q = 0; q < NB / 4; q++)
                reinterpret_cast<float4*>(&starg[sl][b * NB])[q] = *reinterpret_cast<const float4*>(&o[4 * q]);
            srec[sl][b] = make_float2(integ, phase);
            a_prev = o[NB - 1];
        }
        loaded = g + 1;
    };
#pragma unroll 1
    for (;;) {
        const int run = r < nsub ? r : -1;
        const int ver = vp;
        if (run < 0 && ver < 0) break;
        if (t == 0) {
            sctl[0] = run;
            sctl[1] = ver;
            sctl[2] = run >= 0 && run + 2 < nsub ? run + 2 : -1;
            if (run >= 0) sfail[run & 1] = INT_MAX;
        }
        __syncthreads();  // B
        if (run >= 0) run_sub(run);
        __syncthreads();  // A
        const int f = ver >= 0 ? __builtin_amdgcn_readfirstlane(sfail[ver & 1]) : INT_MAX;
        if (f != INT_MAX) {
            // batch f of sub-segment ver did not verify (the batches before it did): that
            // sub-segment from batch f exactly, then the one after it again from its exact end
            const int sl = ver & 1, J = ver * L + f * NB, Je = ver * L + nbat(ver) * NB;
            float ig, ph, a;
            if (f == 0) {
                const float4 z = sstart[sl];
                ig = z.x;
                ph = z.y;
                a = z.z;
            } else {
                const float2 z = srec[sl][f - 1];
                ig = z.x;
                ph = z.y;
                a = starg[sl][f * NB - 1];
            }
            PllPair zz = dem_state(ig, ph, t0, J, a);
            zz = pll_run_fast(zz.p, zz.ctx, x + J, out + J, Je - J, Ki, Kp, step);
            pe = zz.p;
            ce = zz.ctx;
            a_prev = (float)ce.x;
            integ = pe.integ;
            phase = pe.phase;
            init = true;
            loaded = -1;
            n_roll += (unsigned long long)(nbat(ver) - f);
            r = ver + 1;
            vp = -1;
            continue;
        }
        vp = run;
        if (run >= 0) r = run + 1;
    }
    if (t == 0) sctl[3] = 1;
    __syncthreads();  // B: the checkers leave
    // the state after the last whole batch, then the steps past it exactly
    PllPair z = dem_state(integ, phase, t0, nbt * NB, a_prev);
    if (nbt == 0) z = PllPair{pe, ce};
    z = pll_run_fast(z.p, z.ctx, x + nbt * NB, out + nbt * NB, m - nbt * NB, Ki, Kp, step);
    if (t == 0) {
        S[0] = z.p.integ; S[1] = z.p.phase; S[2] = z.p.fbI; S[3] = z.p.fbQ; S[5] = z.p.trig;
        S[6] = 0.0f;
        if (stats && n_roll) atomicAdd(stats, n_roll);  // "resumed": batches redone after a failed check
    }
}

}  // namespace

int launch_pll_demoted(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step,
                       float norm_bw, float* st, float* out, size_t ostride, int inject,
                       unsigned long long* stats) {
    if (n <= 0) return 0;
    static const int resident = [] {
        int nb = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pll_demoted_kernel, 64 * kDemW, 0) == hipSuccess
                   ? nb : 0;
    }();
    if (resident < 1) return -1;
    hipLaunchKernelGGL(pll_demoted_kernel, dim3(n_streams), dim3(64 * kDemW), 0, s, io, n, stride, step, norm_bw, st,
                       out, ostride, inject, stats);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace fmrx
