// stereo.hip — the stereo half of the receive chain (src/project.cpp:152-193):
// channel + carrier band-pass, pilot PLL, mixer, the audio LPF with the reference's SHARED
// audio_state, the mono delay line, L/R matrix and the R,L S16 quantiser.
//
// REF_EXACT semantics: in project.cpp the mono and stereo resample calls of
// one block share one history vector (project.cpp:114,146,172), so
//   * mono   of block b uses as history the last samples of block b-1's MIXER output;
//   * stereo of block b uses as history the last samples of block b's own DEMOD input.
// Both are reproduced exactly at the reference's block boundaries; this is the only
// place where the reference block size (SURVEY table M) changes the numbers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "dsp_device.h"
#include "fmrx_internal.h"
#include "pll_cr.h"
#include "pll_device.h"
#include "pll_math.h"

namespace fmrx {

namespace {

constexpr int kBpMax = 64;

struct BpTaps {
    float2 c[kBpMax];  // (channel, carrier) tap k, interleaved: one SGPR pair per packed product
};

// Channel (22-54 kHz) and carrier (18.5-19.5 kHz) band-pass FIRs share their input, so they
// run as ONE packed FIR: (acc_ch, acc_ca) += (h_ch[k], h_ca[k]) * x, two exact f32 lanes per
// v_pk op, each a sequential ascending-k sum (filter.cpp:84-92, up = down = 1).
template <int BT>
__global__ void __launch_bounds__(256) bpf_pair_kernel(StereoLaunch L, BpTaps t) {
    const int s = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= L.n_if) return;
    const float* x = L.demod + (size_t)s * L.demod_stride + L.hist + j;
    float2v acc = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < BT; k++) {
        const float xv = x[-k];
        const float2v p = float2v{t.c[k].x, t.c[k].y} * xv;
        acc = acc + p;
    }
    L.channel[(size_t)s * L.out_stride + j] = acc.x;
    L.carrier[(size_t)s * L.out_stride + j] = acc.y;
}

// The same FIR pair tiled through LDS: a workgroup stages kBpTile outputs' demod samples plus
// BT-1 of history once (coalesced), each thread keeps the window of its kBpR consecutive
// outputs in registers (one ds_read_b128 per 4 samples, lane stride 16 B: conflict-free) and
// the interleaved (h_ch, h_ca) taps are kernel arguments (SGPR pairs in the packed products).  Each output is
// still the ascending-k sequential sum of separately rounded products (filter.cpp:84-92).
// Replaces one global load per tap per output (51 VMEM instructions an output): 19.4 -> 15.1
// ms per call at 1,024 streams x 10 s.  Measured and dropped: workgroups walking 8 tiles with
// the next tile's loads in flight, and 8 outputs a thread (the taps then spill from SGPRs).
constexpr int kBpR = 4, kBpThreads = 256, kBpTile = kBpR * kBpThreads;  // (the pin below names 4)
template <int BT, bool SRC>
__global__ void __launch_bounds__(kBpThreads) bpf_pair_tile_kernel(StereoLaunch L, BpTaps t) {
    constexpr int W = kBpR + BT - 1;  // a thread's window: samples 4 tid .. 4 tid + W - 1 of the tile
    constexpr int WV = (W + 1) / 2;   // float4 reads (two duplicated samples each)
    // xs2[i] = (x, x), x = demod sample j0 - (BT - 1) + i: the packed product (h_ch, h_ca) * (x, x)
    // needs no splat; the L.hist >= BT - 1 history samples sit in front of the call's demod
    __shared__ float4 xs4[(kBpTile + BT - 1 + 1) / 2 + WV];
    float2* xs2 = reinterpret_cast<float2*>(xs4);
    const int s = blockIdx.y, tid = threadIdx.x;
    const long long j0 = (long long)blockIdx.x * kBpTile;
    const float* x = L.demod + (size_t)s * L.demod_stride + L.hist + j0 - (BT - 1);
    const long long avail = (long long)L.n_if - j0 + (BT - 1);  // samples of this stream from x on
    if constexpr (SRC) {  // the new samples from L.src (this tile's own ones also stored behind the history)
        // every load issued before any store (src may be host memory: one round trip, not one per
        // pass; src and demod could alias as far as the compiler knows)
        constexpr int kPass = (kBpTile + BT - 1 + kBpThreads - 1) / kBpThreads;
        const float* src = L.src + (size_t)s * L.n_if + j0 - (BT - 1);
        float* dst = const_cast<float*>(x);
        float v[kPass];
#pragma unroll
        for (int r = 0; r < kPass; r++) {
            const int i = tid + kBpThreads * r;
            const long long g = j0 - (BT - 1) + i;  // call index of sample i (< 0: history)
            v[r] = i < kBpTile + BT - 1 && i < avail ? (g < 0 ? x[i] : src[i]) : 0.0f;
        }
#pragma unroll
        for (int r = 0; r < kPass; r++) {
            const int i = tid + kBpThreads * r;
            if (i >= kBpTile + BT - 1) break;
            if (i >= BT - 1 && i < avail) dst[i] = v[r];
            xs2[i] = make_float2(v[r], v[r]);
        }
    } else {
        for (int i = tid; i < kBpTile + BT - 1; i += kBpThreads) {
            const float v = i < avail ? x[i] : 0.0f;
            xs2[i] = make_float2(v, v);
        }
    }
    __syncthreads();
    float2v win[2 * WV];
#pragma unroll
    for (int q = 0; q < WV; q++) {  // lane stride 32 B
        const float4 w = xs4[2 * tid + q];
        win[2 * q] = float2v{w.x, w.y};
        win[2 * q + 1] = float2v{w.z, w.w};
    }
    float2v acc[kBpR];
#pragma unroll
    for (int r = 0; r < kBpR; r++) acc[r] = float2v{0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < BT; k++) {
        float2v pv[kBpR];  // the products first, then the sums: no sum reads the product just made
#pragma unroll
        for (int r = 0; r < kBpR; r++) pv[r] = float2v{t.c[k].x, t.c[k].y} * win[r + BT - 1 - k];  // output j0 + 4 tid + r, tap k
#pragma unroll
        for (int r = 0; r < kBpR; r++) acc[r] = acc[r] + pv[r];
        // tap-outer order kept (the accumulators pinned tap by tap, or LLVM sinks each output's
        // chain whole to its store): the kBpR chains interleave, so no packed result is read by
        // the next instruction (that costs a wait state on gfx950)
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]));
    }
    const long long j = j0 + (long long)kBpR * tid;
#pragma unroll
    for (int r = 0; r < kBpR; r++) {
        if (j + r < L.n_if) {
            L.channel[(size_t)s * L.out_stride + j + r] = acc[r].x;
            L.carrier[(size_t)s * L.out_stride + j + r] = acc[r].y;
        }
    }
}

__global__ void bpf_pair_generic(StereoLaunch L, BpTaps t) {
    const int s = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= L.n_if) return;
    const float* x = L.demod + (size_t)s * L.demod_stride + L.hist + j;
    float a = 0.0f, b = 0.0f;
    for (int k = 0; k < L.bp_taps; k++) {
        const float pa = t.c[k].x * x[-k];
        const float pb = t.c[k].y * x[-k];
        a = a + pa;
        b = b + pb;
    }
    L.channel[(size_t)s * L.out_stride + j] = a;
    L.carrier[(size_t)s * L.out_stride + j] = b;
}

// Side data of one PLL segment (pll_math.h pll_side): iv, pr for every sample, in
// parallel, from the trigOffset the segment starts with.  Two arrays of seg x n_streams
// doubles, sample pairs stream-minor: element (j, s) at (j/2 * n_streams + s) * 2 + j%2, so
// the PLL wave's lanes (one stream each) read consecutive 16-B pairs -- coalesced.

// One workgroup per tile of kPrepS streams x kPrepJ samples, transposed through LDS: rows of
// the stream-major input are read coalesced, the stream-minor pairs written coalesced.
constexpr int kPrepS = 16, kPrepJ = 64;
__global__ void __launch_bounds__(256) pll_prep_kernel(const float* io, int m, int n_streams, size_t stride,
                                                       double* side, size_t seg, const float* st, double step,
                                                       int* fail) {
    __shared__ double2 t_iv[kPrepJ / 2][kPrepS], t_pr[kPrepJ / 2][kPrepS], t_h[kPrepJ / 2][kPrepS];
    const int j0 = blockIdx.x * kPrepJ, s0 = blockIdx.y * kPrepS;
    // fail[] sentinel: 0 (= resume the whole segment exactly) until a runner claims the stream
    if (fail && blockIdx.x == 0 && threadIdx.x < kPrepS && s0 + (int)threadIdx.x < n_streams) fail[s0 + threadIdx.x] = 0;
    for (int e = threadIdx.x; e < kPrepS * kPrepJ; e += blockDim.x) {
        const int r = e / kPrepJ, c = e % kPrepJ, s = s0 + r, j = j0 + c;
        double iv = 0.0, pr = 0.0;
        if (s < n_streams && j < m) pll_side(io[(size_t)s * stride + j], st[8 * (size_t)s + 5], j, step, &iv, &pr);
        double* a = reinterpret_cast<double*>(&t_iv[c >> 1][r]);
        double* b = reinterpret_cast<double*>(&t_pr[c >> 1][r]);
        double* h = reinterpret_cast<double*>(&t_h[c >> 1][r]);
        a[c & 1] = iv;
        b[c & 1] = pr;
        h[c & 1] = iv < 0.0 ? 0.5 : 0.0;  // pll_batch_fast's half turn (SPEC)
    }
    __syncthreads();
    double2* siv = reinterpret_cast<double2*>(side);
    double2* spr = siv + seg * (size_t)n_streams / 2;
    double2* sh = spr + seg * (size_t)n_streams / 2;
    for (int e = threadIdx.x; e < kPrepS * kPrepJ / 2; e += blockDim.x) {
        const int jp = e / kPrepS, r = e % kPrepS, s = s0 + r;
        if (s < n_streams && j0 + 2 * jp < m) {
            const size_t a = (size_t)(j0 / 2 + jp) * n_streams + s;
            siv[a] = t_iv[jp][r];
            spr[a] = t_pr[jp][r];
            sh[a] = t_h[jp][r];
        }
    }
}

// The same side data stream-major (element (j, s) at s seg + j: each stream's samples
// contiguous; the half turns with zero gaps, 2 seg per stream), for the split kernels: a wave there works on at most 4 streams, so stream-minor
// rows would put every 16-B load of a wave on its own page (rows n_streams x 16 B apart).
// One thread per sample pair.
// with_h = 0: no half-turn plane (only pll_spec_lane_kernel reads it; the host passes 0 when that
// runner is not launched for the segment): 16 B a sample written instead of 32.
__global__ void __launch_bounds__(256) pll_prep_major_kernel(const float* io, int m, int n_streams, size_t stride,
                                                             double* side, size_t seg, const float* st, double step,
                                                             int with_h, int* fail) {
    const int s = blockIdx.y;
    const int jp = blockIdx.x * blockDim.x + threadIdx.x;
    // fail[] sentinel: 0 = pll_kernel resumes the whole segment on the certified path.  Every
    // runner that takes stream s overwrites it (fail[s] = nb, then the check's atomicMin), so a
    // stream no launched runner took -- a wrong trigOffset hint -- costs speed, never bits.
    if (fail && jp == 0) fail[s] = 0;
    if (2 * jp >= m) return;
    const float t0 = st[8 * (size_t)s + 5];
    double2 iv, pr, h;
    pll_side(io[(size_t)s * stride + 2 * jp], t0, 2 * jp, step, &iv.x, &pr.x);
    if (2 * jp + 1 < m) pll_side(io[(size_t)s * stride + 2 * jp + 1], t0, 2 * jp + 1, step, &iv.y, &pr.y);
    else iv.y = pr.y = 0.0;
    h.x = iv.x < 0.0 ? 0.5 : 0.0;
    h.y = iv.y < 0.0 ? 0.5 : 0.0;
    double2* siv = reinterpret_cast<double2*>(side);
    const size_t plane = seg * (size_t)n_streams / 2, a = (size_t)s * (seg / 2) + jp;
    siv[a] = iv;
    siv[plane + a] = pr;
    if (!with_h) return;
    // half turns in 32-B groups (h_2jp, h_2jp+1, 0, 0): pll_spec_lane_kernel's lane 2 reads the
    // first 16 B, the row's other lanes the zeros beside them (same cache line, no mask op)
    double2* sh = siv + 2 * plane + (size_t)s * seg + 2 * (size_t)jp;
    sh[0] = h;
    sh[1] = make_double2(0.0, 0.0);
}

// pll_math.h pll_state_at for the start of batch b (b NB steps into the segment), out of line.
__device__ __noinline__ PllPair pll_state_at_batch(float2 rec, float t0, int b, int nbatch, float a) {
    PllPair r;
    pll_state_at(r.p, r.ctx, rec.x, rec.y, t0, (long long)b * nbatch, a, DeviceLib{});
    return r;
}

// Streams per wave (spw, a power of two <= 64): lane t works on stream blockIdx.x spw + t % spw,
// and only lanes t < spw store.  The other lanes recompute their stream in lockstep (identical
// values): a wave with every lane active runs the serial chain ~15 % faster than one with a
// single live lane (one stream alone paid ~64 cycles a step of dependency stalls, a full wave
// none), and up to one wave per SIMD the streams run side by side at that single-wave speed.
//
// SPLIT (spw <= 4): streams by 16-lane row (lane t: stream blockIdx.x spw + (t / 16) % spw), so
// the batch's sin and cos can be one polynomial per lane, even lanes sin, odd lanes cos, shared
// by row broadcasts (pll_sincos_split); lane 0 of the stream's first row stores.
//
// The exact PLL (and, after pll_spec_kernel / pll_check_kernel, the fix-up): trigArg of step j
// goes to out[j] (out == io in place for the plain launch).  With `fail` (the first batch of
// each stream whose speculative result did not verify, nb when all did), the wave starts at
// the smallest such batch b0 of its streams, from the state recorded at the end of batch
// b0 - 1 -- exact for every stream of the wave, since none failed before b0 -- so a segment
// that verified costs only the tail.
template <int NB, bool SPLIT>
__global__ void __launch_bounds__(256) pll_kernel(float* io, int n, int n_streams, int spw, size_t stride,
                                                 const double* side, size_t seg, double step, float norm_bw,
                                                 float* st, float* out_base, size_t ostride, const int* fail,
                                                 const float2* rec, size_t rb, unsigned long long* stats) {
    const int t = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int s_lane = wave * spw + (SPLIT ? ((t >> 4) & (spw - 1)) : (t & (spw - 1)));
    const bool owner = (SPLIT ? ((t & 15) == 0 && (t >> 4) < spw) : t < spw) && s_lane < n_streams;
    const SplitCoef sc = split_coef((t & 1) != 0);
    const int s = s_lane < n_streams ? s_lane : n_streams - 1;
    float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    // pair q of batch b of this stream: element (b NB/2 + q) n_streams + s of a row of double2
    // (uniform base + lane offset: global loads with an SGPR base, no per-load address VALU)
    const double2* siv = reinterpret_cast<const double2*>(side);
    const double2* spr = siv + seg * (size_t)n_streams / 2;
    float* S = st + 8 * (size_t)s;
    const float Cp = static_cast<float>(2.666);
    const float Ci = static_cast<float>(3.555);
    const float Kp = norm_bw * Cp;
    const float Ki = (norm_bw * norm_bw) * Ci;
    PllState p{S[0], S[1], S[2], S[3], S[5]};
    PllCtx ctx{};
    ctx.valid = false;
    int i = 0;
    int b0 = 0;
    if (fail) {  // after the speculative runner: x is aligned (the host checked)
        int m = fail[s];
        if (stats && owner) {  // diagnostic counters (fmrx_debug_pll_stats), one atomic per stream
            const int nbs = n / NB;
            atomicAdd(stats, (unsigned long long)(nbs - m));
            atomicAdd(stats + 1, (unsigned long long)nbs);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
        b0 = m;
        if (b0 > 0) {
            const PllPair r = pll_state_at_batch(rec[(size_t)s * rb + b0 - 1], p.trig, b0, NB, out[b0 * NB - 1]);
            p = r.p;
            ctx = r.ctx;
        }
    }
    if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        // Batches of NB samples + side data (v, iv, pr: 20 B a sample) in ONE register set:
        // step j of batch b reloads the elements it has just consumed with batch b+1's (16-B
        // loads; see pll_batch_fast's refill), so every load has a whole batch to land and no
        // second set is needed (two sets overflow the 256 addressable VGPRs into AGPRs).
        float v[NB];
        double iv[NB], pr[NB];
        const int nb = n / NB;
        auto ld_v = [&](int b, int q) {  // floats 4q..4q+3
            *reinterpret_cast<float4*>(&v[4 * q]) = reinterpret_cast<const float4*>(x + b * NB)[q];
        };
        auto ld_d = [&](double (&dst)[NB], const double2* row, int b, int q) {  // doubles 2q, 2q+1
            *reinterpret_cast<double2*>(&dst[2 * q]) = SPLIT ? row[(size_t)s * (seg / 2) + b * (NB / 2) + q]
                                                        : (row + (size_t)(b * (NB / 2) + q) * n_streams)[s];
        };
        if (b0 < nb) {
#pragma unroll
            for (int q = 0; q < NB / 4; q++) ld_v(b0, q);
#pragma unroll
            for (int q = 0; q < NB / 2; q++) {
                ld_d(iv, siv, b0, q);
                ld_d(pr, spr, b0, q);
            }
        }
        for (int b = b0; b < nb; b++) {
            const int bn = b + 1 < nb ? b + 1 : b;  // the last batch reloads itself (no branch)
            // after step j: v[j], pr[j] are dead, and iv[j] (its sign was read at step j-1)
            auto refill = [&](int j) {
                if (j % 4 == 3) ld_v(bn, j / 4);
                if (j % 2 == 1) {
                    ld_d(iv, siv, bn, j / 2);
                    ld_d(pr, spr, bn, j / 2);
                }
            };
            // Optimistic batch: the 16 steps run straight-line on the certified fast paths
            // (pll_batch_fast: no per-step branch, no quadrant bookkeeping, no reciprocal);
            // only if some step of this stream could not be certified (~1e-4 per step) is the
            // batch redone from the saved state on the exact path with the library fallbacks,
            // from the inputs still in memory.  Bit-identical either way.
            const PllState p0 = p;
            const PllCtx ctx0 = ctx;
            float o[NB];
            float* xb = x + b * NB;
            float* ob = out + b * NB;
            if (pll_batch_fast<NB, SPLIT>(p, ctx, v, iv, pr, o, Ki, Kp, refill, sc)) {
                if (owner) {
#pragma unroll
                    for (int q = 0; q < NB / 4; q++)
                        reinterpret_cast<float4*>(ob)[q] = *reinterpret_cast<const float4*>(&o[4 * q]);
                }
            } else {  // rare: redo from the saved state on the exact path (duplicate rows of a
                      // wave write in lockstep, identical values; padding waves do not write)
                const PllPair r = pll_redo(p0, ctx0, xb, ob, NB, Ki, Kp, step, s_lane < n_streams);
                p = r.p;
                ctx = r.ctx;
            }
        }
        i = nb * NB;
    }
    if (i < n) {  // tail (and unaligned streams): exact steps
        const PllPair r = pll_redo(p, ctx, x + i, out + i, n - i, Ki, Kp, step, s_lane < n_streams);
        p = r.p;
    }
    if (owner) {
        S[0] = p.integ; S[1] = p.phase; S[2] = p.fbI; S[3] = p.fbQ; S[5] = p.trig;
    }
}

// ---- speculative PLL: runner + parallel exact check + fix-up ---------------------------------
//
// The certification inside pll_batch_fast is ~20 % of the serial step.  pll_spec_kernel runs
// the recurrence WITHOUT it (pll_batch_fast<SPEC>): trigArg to out, and (integ, phase) at the
// end of every batch to rec.  pll_check_kernel then recomputes every batch of every stream in
// parallel, one thread each, exactly (the certified batch, pll_step where it cannot certify)
// from the state the runner recorded at the end of the previous batch (batch 0: the true
// initial state st), and compares the 16 trigArgs and the end state bit for bit; fail[s] =
// the first batch that differs.  By
// induction every batch before fail[s] is exact.  pll_kernel (with `fail`) resumes from there
// on the certified path and runs the tail, so the result equals the plain launch bit for bit
// whatever the runner did; when everything verified it only runs the tail.
template <int NB>
__global__ void __launch_bounds__(256) pll_spec_kernel(const float* io, int n, int n_streams, int spw, size_t stride,
                                                      const double* side, size_t seg, double step, float norm_bw,
                                                      const float* st, float* out_base, size_t ostride, int* fail,
                                                      float2* rec, size_t rb, int inject) {
    const int t = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int s_lane = wave * spw + (t & (spw - 1));
    const bool owner = t < spw && s_lane < n_streams;
    const int s = s_lane < n_streams ? s_lane : n_streams - 1;
    const float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    const double2* siv = reinterpret_cast<const double2*>(side);
    const double2* spr = siv + seg * (size_t)n_streams / 2;
    const double2* sh = spr + seg * (size_t)n_streams / 2;
    const float* S = st + 8 * (size_t)s;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    PllState p{S[0], S[1], S[2], S[3], S[5]};
    const int nb = n / NB;
    if (owner) fail[s] = nb;
    // batch 0 on the exact path, as pll_kernel starts (a stream's first samples are often
    // exact zeros, where the uncertified rotation is NaN), which also sets the context
    PllCtx ctx{};
    ctx.valid = false;
    if (nb > 0) {
        const PllPair r = pll_redo(p, ctx, x, out, NB, Ki, Kp, step, s_lane < n_streams);
        p = r.p;
        ctx = r.ctx;
        if (owner) rec[(size_t)s * rb] = make_float2(p.integ, p.phase);
    }
    float v[NB];
    double iv[NB], pr[NB], hh[NB];
    auto ld_v = [&](int b, int q) {
        *reinterpret_cast<float4*>(&v[4 * q]) = reinterpret_cast<const float4*>(x + b * NB)[q];
    };
    auto ld_d = [&](double (&dst)[NB], const double2* row, int b, int q) {
        *reinterpret_cast<double2*>(&dst[2 * q]) = (row + (size_t)(b * (NB / 2) + q) * n_streams)[s];
    };
    if (nb > 1) {
#pragma unroll
        for (int q = 0; q < NB / 4; q++) ld_v(1, q);
#pragma unroll
        for (int q = 0; q < NB / 2; q++) {
            ld_d(iv, siv, 1, q);
            ld_d(pr, spr, 1, q);
            ld_d(hh, sh, 1, q);
        }
    }
    for (int b = 1; b < nb; b++) {
        const int bn = b + 1 < nb ? b + 1 : b;
        auto refill = [&](int j) {
            if (j % 4 == 3) ld_v(bn, j / 4);
            if (j % 2 == 1) {
                ld_d(iv, siv, bn, j / 2);
                ld_d(pr, spr, bn, j / 2);
                ld_d(hh, sh, bn, j / 2);
            }
            __builtin_amdgcn_sched_barrier(0);  // see pll_spec_lane_kernel
        };
        float o[NB];
        (void)pll_batch_fast<NB, false, true>(p, ctx, v, iv, pr, o, Ki, Kp, refill, SplitCoef{}, hh);
        if (inject >= 0 && b == 1 + (inject + s) % (nb - 1)) p.phase += 1.0e-3f;  // test hook: a wrong batch
        if (owner) {
            float* ob = out + b * NB;
#pragma unroll
            for (int q = 0; q < NB / 4; q++)
                reinterpret_cast<float4*>(ob)[q] = *reinterpret_cast<const float4*>(&o[4 * q]);
            rec[(size_t)s * rb + b] = make_float2(p.integ, p.phase);
        }
    }
}

// ---- the speculative runner with lane roles (split layout, 16-lane rows; spw <= 4) ------------
//
// pll_spec_kernel's recurrence with the lanes of a row (one stream) doing different work:
// sin and cos are one polynomial on even / odd lanes (pll_sincos_split), and lane 2 takes a
// third job.  The two reductions of a step's trigArg
// x -- r = x - nd pi/2 for sin/cos and the atan2 offset B = (m - h) 2 pi - x of the NEXT step
// (pll_offset_h) -- are the same five operations with different constants,
//     t = rint(fma(x, C1, H)) - H,   w = fma(-t, Clo, fma(-t, Chi, x)),
// (C1, Chi, Clo, H) = (2/pi, pi/2 hi, pi/2 lo, 0) on the sin/cos lanes (w = r, bit for bit:
// fma(x, C1, +0) is the rounded product) and (1/(2 pi), 2 pi hi, 2 pi lo, half turn) on lane 2
// of the row (w = -B, bit for bit: fma is odd under negating an operand pair), so lane 2
// computes the offset while the others compute r, and a third row broadcast hands -B to every
// lane.  The half turns reach lane 2 only: the other lanes load the zeros stored beside them.
// The batch state (fc, nfs, sn, cs, -B) stays in registers from batch to batch; nothing on
// the serial chain is a packed op but the first product (a packed f32 result read by the next
// instruction costs a wait state on gfx950).  ~36 VALU a step, 82 % of the wave's cycles issuing VALU
// (profiles/r02/runner/).  The result is checked by pll_check_kernel like pll_spec_kernel's.
template <int NB>
__global__ void __launch_bounds__(256) pll_spec_lane_kernel(const float* io, int n, int n_streams, int spw,
                                                           size_t stride, const double* side, size_t seg, double step,
                                                           float norm_bw, const float* st, float* out_base,
                                                           size_t ostride, int* fail, float2* rec, size_t rb,
                                                           int inject, int sat_ok, int pred_ok) {
    const int t = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int s_lane = wave * spw + ((t >> 4) & (spw - 1));
    const bool owner = (t & 15) == 0 && (t >> 4) < spw && s_lane < n_streams;
    const bool b_lane = (t & 15) == 2;
    const SplitCoef sc = split_coef((t & 1) != 0);
    const int s = s_lane < n_streams ? s_lane : n_streams - 1;
    const float* x = io + (size_t)s * stride;
    float* out = out_base + (size_t)s * ostride;
    const double2* siv = reinterpret_cast<const double2*>(side) + (size_t)s * (seg / 2);
    const double2* spr = reinterpret_cast<const double2*>(side) + seg * (size_t)n_streams / 2 + (size_t)s * (seg / 2);
    const float* S = st + 8 * (size_t)s;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    PllState p{S[0], S[1], S[2], S[3], S[5]};
    if (sat_ok && pll_sat_segment(spw, p.trig, step)) return;  // pll_sat_kernel's (pll_sat.hip)
    if (pred_ok && pll_pred_wave(p.trig, step)) return;        // pll_pred_kernel's (pll_pred.hip)
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
    // reduction constants: 2 pi on the offset lane (lane 2), pi/2 on the sin/cos lanes
    const double C1 = b_lane ? kInv2Pi : kInvPio2;
    const double Chi = b_lane ? k2PiHi : kPio2Hi;
    const double Clo = b_lane ? k2PiLo : kPio2Lo;
    // half turns: lane 2 reads (h_j, h_j+1), the other lanes the zero pair beside it
    const double2* shl =
        reinterpret_cast<const double2*>(side) + seg * (size_t)n_streams + (size_t)s * seg + (b_lane ? 0 : 1);
    float v[NB];
    double iv[NB], pr[NB], hz[NB];
    auto ld_v = [&](int b, int q) {
        *reinterpret_cast<float4*>(&v[4 * q]) = reinterpret_cast<const float4*>(x + b * NB)[q];
    };
    auto ld_d = [&](double (&dst)[NB], const double2* row, int b, int q) {
        *reinterpret_cast<double2*>(&dst[2 * q]) = row[b * (NB / 2) + q];
    };
    auto ld_h = [&](int b, int q) {
        *reinterpret_cast<double2*>(&hz[2 * q]) = shl[2 * (b * (NB / 2) + q)];
    };
#pragma unroll
    for (int q = 0; q < NB / 4; q++) ld_v(1, q);
#pragma unroll
    for (int q = 0; q < NB / 2; q++) {
        ld_d(iv, siv, 1, q);
        ld_d(pr, spr, 1, q);
        ld_h(1, q);
    }
    // land batch 1 before the loop: the loop's back edge then carries the only loads in flight
    // at its top (a load issued last here would otherwise make every batch start with a full
    // wait, the waitcnt pass merging both edges)
    __builtin_amdgcn_s_waitcnt(0);
    // the state of batch 1's first step, as pll_batch_fast starts (every lane alike)
    const int q0 = ctx.q;
    const float u0 = (q0 & 1) ? p.fbQ : p.fbI, w0 = (q0 & 1) ? p.fbI : -p.fbQ;
    float fc = (q0 & 2) ? -u0 : u0, nfs = (q0 & 2) ? -w0 : w0;
    double sn = ctx.sn, cs = ctx.cs;
    double nB = -pll_offset_h(ctx.x, iv[0] < 0.0 ? 0.5 : 0.0);
    float integ = p.integ, phase = p.phase;
    // the rotation's Y = a sn + b cs of a sample from the current feedback (fc, nfs, sn, cs); the
    // one packed op on the chain: one instruction for both products, its wait state often filled
    // by scalar work (measured 0.4 % faster than two v_mul_f32)
    auto y_of = [&](float vv) -> double {
        const float2v ab = float2v{fc, nfs} * vv;
        return fma((double)ab.x, sn, (double)ab.y * cs);
    };
    for (int b = 1; b < nb; b++) {
        const int bn = b + 1 < nb ? b + 1 : b;
        float o[NB];
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const float e = (float)fma(y_of(v[j]), iv[j], -nB);
            const float ki_e = Ki * e;
            const float kp_e = Kp * e;
            integ = integ + ki_e;
            phase = phase + (kp_e + integ);
            const float arg = (float)(pr[j] + (double)phase);
            o[j] = arg;
            const double xa = (double)arg;
            const double H = hz[(j + 1) % NB];  // the next step's half turn on lane 2, else 0
            const double tq = rint(fma(xa, C1, H)) - H;
            const double w = fma(-tq, Clo, fma(-tq, Chi, xa));  // r, or -B on lane 2
            nB = row_bcast<2>(w);
            // sin/cos of r on the sin/cos lanes from the reduction's w
            const double W = split_w_horner(w * w, sc);
            sn = row_bcast<0>(w * W);
            cs = row_bcast<1>(W);
            fc = (float)cs;
            nfs = -(float)sn;
            // refill after step j: v[j], iv[j], pr[j] and hz[j] (read at step j - 1) are dead
            if (j % 4 == 3) ld_v(bn, j / 4);
            if (j % 2 == 1) {
                ld_d(iv, siv, bn, j / 2);
                ld_d(pr, spr, bn, j / 2);
                ld_h(bn, j / 2);
            }
            // keep each refill after the step that consumed its registers: hoisted loads
            // would overlap the old values and cost a register copy per element a batch
            __builtin_amdgcn_sched_barrier(0);
        }
        // test hook (a wrong batch), branch-free
        phase += (inject >= 0 && b == 1 + (inject + s) % (nb - 1)) ? 1.0e-3f : 0.0f;
        // every lane stores: the lanes of a row hold the same values, and rows past the last
        // stream recompute it bit for bit, so the writes agree; with no branch around them
        // the loads in flight across the loop's back edge need no full wait at its top
        float* ob = out + b * NB;
#pragma unroll
        for (int q = 0; q < NB / 4; q++)
            reinterpret_cast<float4*>(ob)[q] = *reinterpret_cast<const float4*>(&o[4 * q]);
        rec[(size_t)s * rb + b] = make_float2(integ, phase);
    }
}

// One thread per (batch, stream): NB exact steps from the recorded start, compared bit for
// bit.  The batch's side data (1/v, step x trigOffset) is recomputed, not read back: the kernel
// then reads only the input, the runner's trigArgs and records (125 vs 210 us a segment at
// 1,024 streams).
template <int NB>
__global__ void __launch_bounds__(64) pll_check_kernel(const float* io, int n, size_t stride, double step,
                                                       float norm_bw, const float* st, const float* out_base,
                                                       size_t ostride, int* fail, const float2* rec, size_t rb) {
    const int s = blockIdx.y;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    const int nb = n / NB;
    if (b >= nb) return;
    const float* S = st + 8 * (size_t)s;
    const float t0 = S[5];
    if (!pll_trig_domain(t0)) {  // pll_state_at's trigOffset needs it: the whole segment exactly
        if (b == 0) atomicMin(fail + s, 0);
        return;
    }
    const float* x = io + (size_t)s * stride + (size_t)b * NB;
    const float* o = out_base + (size_t)s * ostride + (size_t)b * NB;
    const float Kp = norm_bw * static_cast<float>(2.666);
    const float Ki = (norm_bw * norm_bw) * static_cast<float>(3.555);
    PllState p{S[0], S[1], S[2], S[3], t0};
    PllCtx ctx{};
    ctx.valid = false;
    const DeviceLib lib;
    if (b > 0) {  // inline: no call, no scratch frame for the returned state
        const float2 rb1 = rec[(size_t)s * rb + b - 1];
        pll_state_at(p, ctx, rb1.x, rb1.y, t0, (long long)b * NB, o[-1], lib);
    }
    bool same = true;
    bool done = false;
    // pr_j = step trig_j exactly as pll_side forms it (trig_j = min(t0 + j + 1, 2^24), integer-
    // valued t0 checked above), recomputed instead of read back: it rises with j, so the batch's
    // last value decides whether any is out of the fast path's range (pll_side's NaN)
    const double t0d = (double)t0;
    const double pr_last = step * fmin(t0d + (double)((long long)b * NB + NB), (double)kPllTrigStick);
    if (ctx.valid && fabs(pr_last) < kPllMaxPr) {  // the certified fast path (~2.5x cheaper than 16 pll_step)
        float v[NB], c[NB];
        double iv[NB], pr[NB];
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const size_t jj = (size_t)b * NB + j;
            v[j] = x[j];
            // 1/v recomputed too (reciprocal + one Newton step, ~2^-46 relative; pll_side's NaN
            // outside [kPllMinV, 1e300)): the batch's bound takes |Y/v| (|delta| + |eta|) with
            // |Y/v| <= 2^-23, so eta = 2^-46 adds ~2^-69 to kPllEBatch's 2e-14 (pll_math.h)
            const double vd = (double)v[j];
            const double r0 = __builtin_amdgcn_rcp(vd);
            const double r1 = fma(r0, fma(-vd, r0, 1.0), r0);
            iv[j] = (fabs(vd) >= (double)kPllMinV && fabs(vd) < 1.0e300) ? r1 : (double)NAN;
            pr[j] = step * fmin(t0d + (double)(jj + 1), (double)kPllTrigStick);
        }
        const PllState p0 = p;
        const PllCtx c0 = ctx;
        if (pll_batch_fast<NB, false>(p, ctx, v, iv, pr, c, Ki, Kp, [](int) {})) {
#pragma unroll
            for (int j = 0; j < NB; j++) same &= __float_as_uint(c[j]) == __float_as_uint(o[j]);
            done = true;
        } else {
            p = p0;
            ctx = c0;
        }
    }
    if (!done) {
        for (int j = 0; j < NB; j++) {
            const float a = pll_step(p, ctx, x[j], Ki, Kp, step, lib);
            same &= __float_as_uint(a) == __float_as_uint(o[j]);
        }
    }
    const float2 e = rec[(size_t)s * rb + b];
    same &= __float_as_uint(p.integ) == __float_as_uint(e.x) && __float_as_uint(p.phase) == __float_as_uint(e.y);
    if (!same) atomicMin(fail + s, b);
}

// filter.cpp:170: ncoOut[i] = cos(trigArg * nocoScale + phaseAdjust), float arithmetic inside,
// double cos, float result; also the ncoOut_state carry (filter.cpp:173).
__global__ void pll_nco_kernel(float* io, int n, size_t stride, const float* args, size_t astride,
                               float nco_scale, float phase_adjust, float* st) {
    const int s = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float* x = io + (size_t)s * stride;
    const float a = args[(size_t)s * astride + i] * nco_scale + phase_adjust;
    float cv;
#ifdef FMRX_AB_NCO_COS
    if (!fast_cos_f(a, &cv)) cv = sincos_lib(a).y;  // A/B: only the cosine certified
#else
    float sv;
    if (!fast_sincos_f(a, &sv, &cv)) cv = sincos_lib(a).y;
#endif
    x[i] = cv;
    if (i == n - 1) st[8 * (size_t)s + 4] = cv;
}

// Test hook (fmrx_test_pll_fallback): the PLL's out-of-line fallbacks on given arguments.
// kind 0: sincos_lib(a) -> out[2i] = sin, out[2i + 1] = cos; kind 1: atan2_lib(a = y, b = x);
// kind 2: the NCO's cos (pll_nco_kernel: fast_sincos_f, else the fallback).
__global__ void pll_fallback_test_kernel(int kind, const float* a, const float* b, size_t n, float* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (kind == 0) {
        const float2 r = sincos_lib(a[i]);
        out[2 * i] = r.x;
        out[2 * i + 1] = r.y;
    } else if (kind == 1) {
        out[i] = atan2_lib(a[i], b[i]);
    } else {
        float sv, cv;
        if (!fast_sincos_f(a[i], &sv, &cv)) cv = sincos_lib(a[i]).y;
        out[i] = cv;
    }
}

// ---- audio stage -------------------------------------------------------------------------
struct AudioView {
    const float* d;    // demod of block b (index 0 = first sample of block b)
    const float* ch;   // channel of block b
    const float* nco;  // nco of block b
};

__device__ inline float mixer_at(const AudioView& v, int i) { return 2.0f * (v.ch[i] * v.nco[i]); }

// mono of block b, frame m (project.cpp:146): history = previous block's mixer tail
// (or the carried tail for the first block of a call).
// Output m of the resampler: phase k0 = (m down) mod up, base input j0 = floor(m down / up);
// taps k = k0 + i up (i ascending = k ascending, filter.cpp:84-92) against input j0 - i: one
// division per output, none per tap.  The prototype stays in its own order: at tap step i the
// lanes of a wave read inside one up-wide window (coalesced), where a phase-major table would
// scatter them over up rows.
struct Phase {
    long long j0;
    const float* c;  // c[i * up] = coeff[k0 + i up]
    int cnt;
};
__device__ inline Phase phase_of(const AudioLaunch& L, int m) {
    const long long nd = (long long)m * L.down;
    Phase p;
    p.j0 = nd / L.up;
    const int k0 = (int)(nd - p.j0 * L.up);
    p.cnt = (L.at - k0 + L.up - 1) / L.up;
    p.c = L.audio_c + k0;
    return p;
}

__device__ inline float mono_at(const AudioLaunch& L, const AudioView& cur, const AudioView& prv,
                                bool has_prev, const float* tail, int tl, int m) {
    const Phase ph = phase_of(L, m);
    float acc = 0.0f;
    for (int i = 0; i < ph.cnt; i++) {
        const long long j = ph.j0 - i;
        float x;
        if (j >= 0) x = cur.d[j];
        else x = has_prev ? mixer_at(prv, L.if_per_block + (int)j) : tail[tl + j];
        const float p = ph.c[i * L.up] * x;
        acc = acc + p;
    }
    return acc;
}

// stereo of block b, frame m (project.cpp:172): history = the same block's demod tail.
__device__ inline float stereo_at(const AudioLaunch& L, const AudioView& cur, int m) {
    const Phase ph = phase_of(L, m);
    float acc = 0.0f;
    for (int i = 0; i < ph.cnt; i++) {
        const long long j = ph.j0 - i;
        const float x = j >= 0 ? mixer_at(cur, (int)j) : cur.d[L.if_per_block + j];
        const float p = ph.c[i * L.up] * x;
        acc = acc + p;
    }
    return acc;
}

__device__ inline AudioView view(const AudioLaunch& L, int s, int b) {
    const size_t nif = (size_t)L.n_blocks * L.if_per_block;
    AudioView v;
    v.d = L.demod + (size_t)s * L.demod_stride + L.hist + (size_t)b * L.if_per_block;
    v.ch = L.channel + (size_t)s * nif + (size_t)b * L.if_per_block;
    v.nco = L.nco + (size_t)s * nif + (size_t)b * L.if_per_block;
    return v;
}

constexpr int kTail = 64;  // mixer tail kept across calls (>= ceil((at-1)/up) + 1)

__global__ void stereo_audio_kernel(AudioLaunch L, int b0) {
    // grid.x = blocks x frame tiles (no 65,535 limit on the block count), grid.y = streams;
    // blocks b0, b0 + 1, ... of the call
    const int ft = (L.frames_per_block + (int)blockDim.x - 1) / (int)blockDim.x;
    const int s = blockIdx.y;
    const int bl = blockIdx.x / ft;
    const int b = b0 + bl;
    const int m = (blockIdx.x - bl * ft) * blockDim.x + threadIdx.x;
    if (m >= L.frames_per_block) return;
    const AudioView cur = view(L, s, b);
    const AudioView prv = b > 0 ? view(L, s, b - 1) : cur;
    const float* tail = L.mix_tail + (size_t)s * kTail;
    const float mono = mono_at(L, cur, prv, b > 0, tail, kTail, m);
    float shift;  // project.cpp:152-159, 5-sample delay line
    if (m >= kMonoDelay) {
        shift = mono_at(L, cur, prv, b > 0, tail, kTail, m - kMonoDelay);
    } else if (b > 0) {
        const AudioView pp = b > 1 ? view(L, s, b - 2) : prv;
        shift = mono_at(L, prv, pp, b > 1, tail, kTail, L.frames_per_block - kMonoDelay + m);
    } else {
        shift = L.mono_state[(size_t)s * 8 + m];
    }
    const float st = stereo_at(L, cur, m);
    const float left = half_of(shift + st);    // filter.cpp:196
    const float right = half_of(shift - st);   // filter.cpp:197
    const size_t o = ((size_t)s * L.n_blocks + b) * (size_t)L.frames_per_block + m;
    L.pcm[2 * o] = quantize_s16(right);        // project.cpp:184-187 (R first)
    L.pcm[2 * o + 1] = quantize_s16(left);
    if (L.mono_out) L.mono_out[o] = mono;
}

// Modes 0/1 (up = 1): one workgroup per (block, stream).  The block's (demod, mixer) pairs sit in
// LDS behind the histories of both resamplers -- (previous block's mixer, own demod tail), the
// shared-audio_state quirk of project.cpp:146/172 -- so the mono and stereo LPF of a frame are
// ONE packed FIR over one float2 array (v_pk_mul/v_pk_add, each lane an ascending-tap
// sequential sum as filter.cpp:84-92), and the mono of each frame is computed once: the 5-frame
// delay line reads it back from LDS.  Same arithmetic as stereo_audio_kernel.
constexpr int kTileIf = 1024, kTileFrames = 256, kTileTaps = 64;

// carry (the small kernel's last block): the state carry from this tile's LDS instead of
// audio_state_carry's global re-reads -- MO holds the block's monos (mono_at's sums, same
// order) and X[H + i].y its mixer samples.
__device__ void audio_tile(const AudioLaunch& L, int s, int b, bool carry = false) {
    constexpr int kPer = kTileFrames / 128;    // frames per thread
    __shared__ float2 X[kTileTaps + kTileIf];  // X[H + j]: (mono input, stereo input) at IF index j
    __shared__ float C[kTileTaps], MO[kTileFrames];
    const int ipb = L.if_per_block, fpb = L.frames_per_block, at = L.at, H = at - 1;
    const AudioView cur = view(L, s, b);
    for (int i = threadIdx.x; i < ipb; i += blockDim.x) X[H + i] = make_float2(cur.d[i], mixer_at(cur, i));
    if (b > 0) {
        const AudioView prv = view(L, s, b - 1);
        for (int i = threadIdx.x; i < H; i += blockDim.x)
            X[i] = make_float2(mixer_at(prv, ipb - H + i), cur.d[ipb - H + i]);
    } else {
        for (int i = threadIdx.x; i < H; i += blockDim.x)
            X[i] = make_float2(L.mix_tail[(size_t)s * kTail + kTail - H + i], cur.d[ipb - H + i]);
    }
    for (int i = threadIdx.x; i < at; i += blockDim.x) C[i] = L.audio_c[i];
    __syncthreads();
    float st[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const int m = threadIdx.x + 128 * k;
        st[k] = 0.0f;
        if (m < fpb) {
            const float2* x = X + H + m * L.down;
            float2v acc = {0.0f, 0.0f};
            for (int i = 0; i < at; i++) {
                const float2 v = x[-i];
                const float2v p = float2v{v.x, v.y} * C[i];
                acc = acc + p;
            }
            MO[m] = acc.x;
            st[k] = acc.y;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const int m = threadIdx.x + 128 * k;
        if (m >= fpb) continue;
        float shift;  // project.cpp:152-159, 5-sample delay line
        if (m >= kMonoDelay) {
            shift = MO[m - kMonoDelay];
        } else if (b > 0) {  // the previous block's last frames read only its own demod (host-checked)
            const float* d = view(L, s, b - 1).d + (fpb - kMonoDelay + m) * L.down;
            float a = 0.0f;
            for (int i = 0; i < at; i++) {
                const float p = C[i] * d[-i];
                a = a + p;
            }
            shift = a;
        } else {
            shift = L.mono_state[(size_t)s * 8 + m];
        }
        const float left = half_of(shift + st[k]);   // filter.cpp:196
        const float right = half_of(shift - st[k]);  // filter.cpp:197
        const size_t o = ((size_t)s * L.n_blocks + b) * (size_t)fpb + m;
        L.pcm[2 * o] = quantize_s16(right);          // project.cpp:184-187 (R first)
        L.pcm[2 * o + 1] = quantize_s16(left);
        if (L.mono_out) L.mono_out[o] = MO[m];
    }
    if (!carry) return;
    __syncthreads();  // every read of the old mono_state / mix_tail happened above
    const int i = threadIdx.x;
    if (i < kMonoDelay) L.mono_state[(size_t)s * 8 + i] = MO[fpb - kMonoDelay + i];
    if (i < kTail) L.mix_tail[(size_t)s * kTail + i] = X[H + ipb - kTail + i].y;
}

__global__ void __launch_bounds__(128) stereo_audio_tile_kernel(AudioLaunch L, int b0) {
    audio_tile(L, blockIdx.y, b0 + (int)blockIdx.x);  // block b of the call, stream blockIdx.y
}

// Carry the audio state of the LAST block of this call into the next call (thread i of stream s).
__device__ void audio_state_carry(const AudioLaunch& L, int s, int i) {
    const int b = L.n_blocks - 1;
    const AudioView cur = view(L, s, b);
    const AudioView prv = b > 0 ? view(L, s, b - 1) : cur;
    const float* tail = L.mix_tail + (size_t)s * kTail;
    float mono = 0.0f, mix = 0.0f;
    if (i < kMonoDelay)
        mono = mono_at(L, cur, prv, b > 0, tail, kTail, L.frames_per_block - kMonoDelay + i);
    if (i < kTail) mix = mixer_at(cur, L.if_per_block - kTail + i);
    __syncthreads();  // every read of the old tail happens before it is overwritten
    if (i < kMonoDelay) L.mono_state[(size_t)s * 8 + i] = mono;
    if (i < kTail) L.mix_tail[(size_t)s * kTail + i] = mix;
}

__global__ void stereo_state_kernel(AudioLaunch L) { audio_state_carry(L, blockIdx.x, threadIdx.x); }

// A few blocks a stream (the reference's per-block seam, fmrx_audio_block with one block): the
// NCO (pll_nco_kernel's arithmetic, from the PLL's trigArgs), every block's audio in order
// (audio_tile), the state carry (stereo_state_kernel) and the demod history for the next call
// (the last kDemodHist samples to the front) in ONE launch, one workgroup a stream -- four
// launches fewer than the parallel path, which costs each of them ~4-7 us at this size
// (profiles/r06/seam: kernel trace of the seam).
__global__ void __launch_bounds__(128) stereo_audio_small_kernel(AudioLaunch L, const float* args, size_t astride,
                                                                 float nco_scale, float phase_adjust, float* pll_st,
                                                                 int demod_hist) {
    const int s = blockIdx.x;
    const int nif = L.n_blocks * L.if_per_block;
    float* nco = const_cast<float*>(L.nco) + (size_t)s * nif;
    for (int i = threadIdx.x; i < nif; i += blockDim.x) {  // filter.cpp:170 (pll_nco_kernel)
        const float a = args[(size_t)s * astride + i] * nco_scale + phase_adjust;
        float sv, cv;
        if (!fast_sincos_f(a, &sv, &cv)) cv = sincos_lib(a).y;
        nco[i] = cv;
        if (i == nif - 1) pll_st[8 * (size_t)s + 4] = cv;
    }
    __syncthreads();
    for (int b = 0; b < L.n_blocks; b++) {
        audio_tile(L, s, b, b == L.n_blocks - 1);  // the last block carries the state
        __syncthreads();
    }
    float* d = const_cast<float*>(L.demod) + (size_t)s * L.demod_stride;
    for (int i = threadIdx.x; i < demod_hist; i += blockDim.x) d[i] = d[nif + i];
}

inline int ok() { return hipGetLastError() == hipSuccess ? 0 : -2; }

}  // namespace

int launch_bpf_pair(const StereoLaunch& L, int n_streams, hipStream_t s, bool tiled) {
    if (L.n_if <= 0) return 0;
    if (L.bp_taps > kBpMax) return -1;
    BpTaps t{};
    for (int k = 0; k < L.bp_taps; k++) t.c[k] = make_float2(L.ch_c[k], L.ca_c[k]);
    const dim3 grid((L.n_if + 255) / 256, n_streams), block(256);
    const bool tile = L.bp_taps == 51 && L.hist >= 50 && tiled;
    if (L.src && !tile &&  // the per-output kernels read the new samples from demod: copy them there
        hipMemcpy2DAsync(const_cast<float*>(L.demod) + L.hist, L.demod_stride * sizeof(float), L.src,
                         (size_t)L.n_if * sizeof(float), (size_t)L.n_if * sizeof(float), n_streams,
                         hipMemcpyDefault, s) != hipSuccess)
        return -1;
    if (tile && L.src)
        hipLaunchKernelGGL((bpf_pair_tile_kernel<51, true>), dim3((L.n_if + kBpTile - 1) / kBpTile, n_streams),
                           dim3(kBpThreads), 0, s, L, t);
    else if (tile)
        hipLaunchKernelGGL((bpf_pair_tile_kernel<51, false>), dim3((L.n_if + kBpTile - 1) / kBpTile, n_streams),
                           dim3(kBpThreads), 0, s, L, t);
    else if (L.bp_taps == 51)
        hipLaunchKernelGGL(bpf_pair_kernel<51>, grid, block, 0, s, L, t);
    else
        hipLaunchKernelGGL(bpf_pair_generic, grid, block, 0, s, L, t);
    return ok();
}

// The scratch of a launch_pll call, in doubles: one segment's side data (iv, pr, half turns:
// 3 seg, plus seg as slack for the stream-minor layout), the call's trigArgs (n floats a stream:
// every runner writes its steps' trigArgs there, the NCO reads them once at the end), the
// speculative runners' batch records (seg / 16 float2 a stream) and fail[] (ints).
// Segment length (the lane / two-wave / saturated runners, checked by pll_check_kernel): kPllSeg
// samples up to 32 streams, then shorter so that segment x streams stays ~2^23 (down to 2^14): a
// batch the runner got wrong (~3e-9 of steps) costs the rest of its segment on the certified
// path, serially, so the expected cost per segment grows with segment^2 x streams.  The
// three-wave runner certifies itself and needs no segments (pll_pipe_kernel).
static size_t pll_seg_len(int n, int n_streams) {
    size_t cap = kPllSeg;
    while (cap > ((size_t)1 << 14) && cap * (size_t)std::max(n_streams, 1) > ((size_t)1 << 23)) cap >>= 1;
    return std::min<size_t>(((size_t)std::max(n, 0) + 15) / 16 * 16, cap);
}
size_t pll_side_doubles(int n, int n_streams) {
    const size_t seg = pll_seg_len(n, n_streams), ns = (size_t)n_streams;
    return 4 * seg * ns + ((size_t)std::max(n, 0) * ns + 1) / 2 + (seg / kPllBatch) * ns + (ns + 1) / 2;
}

// The PLL over n samples of n_streams streams, then the NCO of every sample in parallel
// (filter.cpp:136-174).  With the host's trigOffset bounds known and equal for every stream
// (every context's streams advance together) and a SIMD for each of the three-wave runner's
// waves, the samples from trigOffset 2^20 on run on it: one self-certifying launch per form
// (pll_pipe_kernel; 2^20 / 2^21 / 2^22), no per-segment kernels.  The samples before, or all of
// them otherwise, run in segments (pll_seg_len): side data of the segment (parallel), the
// speculative runner (pll_spec_lane_kernel, pll_pred_kernel or pll_sat_kernel by regime,
// pll_spec_kernel beyond 4 streams a wave), pll_check_kernel, then pll_kernel resuming at the
// first batch that did not verify; the state carries in st between launches, so the segments
// chain exactly like one launch.  FMRX_PLL_SPEC=0 (or rows not 16-byte aligned): the plain
// certified pll_kernel in place.
int launch_pll(float* io, int n, int n_streams, size_t stride, float freq, float fs,
               float nco_scale, float phase_adjust, float norm_bw, float* st, double* side, hipStream_t s,
               const PllHint& hint, unsigned long long* spec_stats, bool nco) {
    if (n <= 0) return 0;
    const size_t seg = pll_seg_len(n, n_streams);
    const size_t rb = seg / kPllBatch;
    float* args = reinterpret_cast<float*>(side + 4 * seg * (size_t)n_streams);  // n per stream
    float2* rec = reinterpret_cast<float2*>(side + 4 * seg * (size_t)n_streams +
                                            ((size_t)n * n_streams + 1) / 2);  // rb per stream
    int* fail = reinterpret_cast<int*>(rec + rb * (size_t)n_streams);
    // one stream per wave while the waves fit one per SIMD, then more streams per wave
    const int n_simd = hint.n_simd;
    const PllKnobs& kn = hint.knobs;  // the context's switches (fmrx_debug_set_knob)
    const bool spec_env = kn.spec != 0;
    // test hook (tests/test_gpu_parity.py, knob pll_inject): the runners corrupt batch
    // 1 + (k + s) % (nb - 1) of stream s (the self-certifying runners: a forced miss on one
    // interval), so the check and the fix-up from that batch (the exact redo) run on every stream
    const int inject = kn.inject;
    const bool spec = spec_env && (reinterpret_cast<uintptr_t>(io) & 15) == 0 && stride % 4 == 0;
    // pll_sat = 0 / pll_pred = 0 (measurements, tests): saturated segments / segments from 2^20
    // steps on the ordinary runner too (pll_pred = 2, tests: the two-wave runner even where its
    // waves share SIMDs)
    const int sat_ok = kn.sat != 0 ? 1 : 0;
    const int pred_ok = kn.pred == 0 ? 0 : kn.pred == 2 ? 2 : 1;
    int spw = 1;
    while (spw < 64 && (long long)spw * n_simd < n_streams) spw *= 2;
    // Waves of 64 lanes; past 256 waves, workgroups of 4 waves, one per SIMD of a CU: 64-lane
    // workgroups alone were placed two to a SIMD at 1,024 waves (half speed for both)
    const int waves = (n_streams + spw - 1) / spw;
    const int wpg = waves > n_simd / 4 ? 4 : 1;
    const dim3 grid((waves + wpg - 1) / wpg), block(64 * wpg);

    // pll_pipe = 0 (measurements, tests): no three-wave runner; pll_pipe_miss = k (test hook): the
    // self-certifying runners report a miss on interval k of every launch, so the redo path runs
    const int pipe_env = kn.pipe != 0 ? 1 : 0;
    const int pipe_miss = kn.pipe_miss;
    // pll_hint_skew = d (test hook): the host's trigOffset bounds shifted by d samples, so the
    // runners launched are the wrong ones.  A segment stream no runner takes keeps the pre-pass's
    // fail[] sentinel 0 and is resumed whole on the certified path; a self-certifying launch outside
    // its domain runs its range exactly (same bits either way)
    const double skew = kn.skew;
    // filter.cpp:163: 2*PI*(freq/Fs) in double from the float quotient (host == device IEEE)
    const double step = (2.0 * 3.14159265358979323846) * static_cast<double>(freq / fs);  // dy4.h:14 PI
    const bool step_ok = std::fabs(step * (double)kPllTrigStick) < kPllMaxPr;
    const double hlo = std::max(hint.trig_lo + skew, 0.0), hhi = std::max(hint.trig_hi + skew, 0.0);
    const bool k = hint.known && step_ok;
    StageTimer* tm = hint.timer;
    auto timed = [&](int kind, double steps, auto&& launch) {
        const int t = tm ? tm->begin(s) : -1;
        launch();
        if (tm) tm->end(t, kind, steps, s);
    };
    // the three-wave runner: every stream at the same known trigOffset t, a SIMD per wave (one
    // stream a workgroup of three); it takes the samples from trigOffset 2^20 on
    const bool pipe = spec && pred_ok && pipe_env && spw == 1 && 3 * n_streams <= n_simd && k && hlo == hhi;
    // the index runner in [2^17, 2^20) wants a CU a stream (pll_idx = 0: not launched; 1: from
    // 2^18 only, the lane runner keeping [2^17, 2^18))
    const int idx_env = kn.idx == 0 ? 0 : kn.idx == 1 ? 1 : 2;
    const bool idx = pipe && idx_env && kPllIdxSimds * n_streams <= n_simd;
    const double fast_min = idx ? (double)(idx_env == 2 ? kPllIdxMin64 : kPllIdxMin) : (double)kPllPipeMinLow;
    size_t n_seg = (size_t)n;  // samples through the segment loop
    if (pipe) n_seg = hlo >= fast_min ? 0 : std::min((size_t)n, (size_t)(fast_min - hlo));

    for (size_t off = 0; off < n_seg; off += seg) {
        // the runners a segment can need (pll_sat_segment / pll_pred_wave take their streams, the
        // lane kernel the rest): with known trigOffset bounds the others are not launched
        const double lo = std::min(hlo + (double)off, (double)kPllTrigStick);
        const double hi = std::min(hhi + (double)off, (double)kPllTrigStick);
        // the two-wave runner too wants a SIMD per wave (two of its waves on one SIMD ran slower
        // than the lane runner: 1,024 streams x 10 s 0.291 vs 0.279 s, 2,048 0.405 vs 0.371 s)
        const bool pred_fit = pred_ok && (2 * waves <= n_simd || pred_ok == 2);
        const bool sat_all = k && sat_ok && spw == 1 && lo >= (double)kPllTrigStick;
        const bool run_lane = !(k && lo >= (double)kPllPredMin && (pred_fit || sat_all));
        const bool run_sat = sat_ok && spw == 1 && (!k || hi >= (double)kPllTrigStick);
        const bool run_pred = pred_fit && (!k || hi >= (double)kPllPredMin) && !sat_all;
        const int m = (int)std::min(seg, n_seg - off);
        float* x = io + off;
        float* out = spec ? args + off : x;
        const size_t ostride = spec ? (size_t)n : stride;
        // a runner's steps count toward its regime only when it is the segment's one runner
        const bool lane_on = spec && spw <= 4 && run_lane, sat_on = spec && spw <= 4 && run_sat,
                   pred_on = spec && spw <= 4 && run_pred;
        const double one = (int)lane_on + sat_on + pred_on == 1 ? (double)m : 0.0;
        timed(kStPrep, 0.0, [&] {
            if (spw <= 4)  // the split kernels read stream-major side data
                hipLaunchKernelGGL(pll_prep_major_kernel, dim3(((m + 1) / 2 + 255) / 256, n_streams), dim3(256), 0, s,
                                   x, m, n_streams, stride, side, seg, st, step, (spec && run_lane) ? 1 : 0,
                                   spec ? fail : nullptr);
            else
                hipLaunchKernelGGL(pll_prep_kernel, dim3((m + kPrepJ - 1) / kPrepJ, (n_streams + kPrepS - 1) / kPrepS),
                                   dim3(256), 0, s, x, m, n_streams, stride, side, seg, st, step, spec ? fail : nullptr);
        });
        if (spec) {
            if (spw <= 4) {
                if (run_lane)
                    timed(kStLane, one, [&] {
                        hipLaunchKernelGGL(pll_spec_lane_kernel<kPllBatch>, grid, block, 0, s, x, m, n_streams, spw,
                                           stride, side, seg, step, norm_bw, st, out, ostride, fail, rec, rb, inject,
                                           run_sat ? 1 : 0, run_pred ? 1 : 0);  // it leaves waves only to those launched
                    });
                // saturated streams (pll_sat_segment), which the lane kernel leaves to it
                if (run_sat)
                    timed(kStSat, one, [&] {
                        launch_pll_sat(grid, block, s, x, m, n_streams, spw, stride, side, seg, step, norm_bw, st,
                                       out, ostride, fail, rec, rb, inject);
                    });
                // waves from trigOffset 2^20 below the stick (pll_pred_wave)
                if (run_pred)
                    timed(kStPred, one, [&] {
                        launch_pll_pred(waves, s, x, m, n_streams, spw, stride, side, seg, step, norm_bw, st, out,
                                        ostride, fail, rec, rb, inject, run_sat ? 1 : 0, 0);
                    });
            } else
                timed(kStLane, (double)m, [&] {
                    hipLaunchKernelGGL(pll_spec_kernel<kPllBatch>, grid, block, 0, s, x, m, n_streams, spw, stride,
                                       side, seg, step, norm_bw, st, out, ostride, fail, rec, rb, inject);
                });
            const int nb = m / kPllBatch;
            if (nb > 0)
                timed(kStCheck, 0.0, [&] {
                    hipLaunchKernelGGL(pll_check_kernel<kPllBatch>, dim3((nb + 63) / 64, n_streams), dim3(64), 0, s, x,
                                       m, stride, step, norm_bw, st, out, ostride, fail, rec, rb);
                });
        }
        timed(kStTail, 0.0, [&] {
            if (spw <= 4)
                hipLaunchKernelGGL((pll_kernel<kPllBatch, true>), grid, block, 0, s, x, m, n_streams, spw, stride,
                                   side, seg, step, norm_bw, st, out, ostride, spec ? fail : nullptr, rec, rb,
                                   spec_stats);
            else
                hipLaunchKernelGGL((pll_kernel<kPllBatch, false>), grid, block, 0, s, x, m, n_streams, spw, stride,
                                   side, seg, step, norm_bw, st, out, ostride, spec ? fail : nullptr, rec, rb,
                                   spec_stats);
        });
    }
    // the self-certifying runners' ranges: the index runner's [2^17, 2^18) / [2^18, 2^19) /
    // [2^19, 2^20) forms (64 / 32 / 16 candidates), then the three-wave runner's [2^20, 2^21)
    // 16-step five-candidate form, [2^21, 2^22) the 64-step one, from 2^22 (the stick included)
    // three candidates
    int idx_rc = 0;
    // A range of fewer than kPllShortIntervals of its form's long intervals runs on the 16-step
    // forms (the index runner below 2^20, the wide three-wave form 24 from 2^20: in a short call to
    // the call's end); a long form's steps past its last whole interval go to the 16-step form too
    // (on the exact path they cost ~400 ns a step).  The first interval of every form is predicted,
    // so a long form pays nothing extra for a short call: the per-block seam's 640 steps are 10
    // count-form intervals in [2^19, 2^20), 5 in [2^20, 2^22), 2 + a 128-step tail past 2^22.
    const bool short_call = (size_t)n < kPllShortCall;
    // pll_demoted_kernel after each runner range that may demote, or with hint.demote_once ONCE a
    // call after its runner launches (a demoted stream's later launches only add their steps to its
    // hand-off): beside the pipelined engine's stage kernels each launch of it waited for CUs, ~11 ms
    // of configs[4] at one a range (profiles/r06/demote_probe/)
    size_t dem_from = (size_t)n;
    auto run = [&](int form, bool cnt, size_t j, size_t e) {
        const int kind = cnt ? kStCnt17 + (form - 17)
                       : form == 17 ? kStIdx17 : form == 18 ? kStIdx18 : form == 19 ? kStIdx19
                       : form == 20 || form == 24 ? kStPipe20 : form == 21 ? kStPipe21 : form == 22 || form == 25 ? kStPipe22
                       : kStStick;
        timed(kind, (double)(e - j), [&] {
            if (cnt)
                idx_rc |= launch_pll_cnt(s, io + j, (int)(e - j), n_streams, stride, step, norm_bw, st, args + j,
                                         (size_t)n, inject, pipe_miss, form, spec_stats, hint.redos);
            else if (form < 20)
                idx_rc |= launch_pll_idx(s, io + j, (int)(e - j), n_streams, stride, step, norm_bw, st, args + j,
                                         (size_t)n, inject, pipe_miss, form, spec_stats, hint.redos);
            else
                launch_pll_pipe(s, io + j, (int)(e - j), n_streams, stride, step, norm_bw, st, args + j, (size_t)n,
                                inject, pipe_miss, form, spec_stats, hint.redos);
            // a launch that may demote a stream (kPllDemoteMinIntervals, the runner's own rule): the
            // demoted kernel runs the rest of its range right after it, or (demote_once) follows the
            // call's last runner launch, from the first such launch on
            if ((e - j) >= (size_t)kPllDemoteMinIntervals * (size_t)pll_form_interval(form, cnt)) {
                if (hint.demote_once)
                    dem_from = std::min(dem_from, j);
#ifndef FMRX_AB_NO_DEMOTED_LAUNCH
                else
                    idx_rc |= launch_pll_demoted(s, io + j, (int)(e - j), n_streams, stride, step, norm_bw, st,
                                                 args + j, (size_t)n, inject, spec_stats);
#endif
            }
        });
    };
    for (size_t j = n_seg; pipe && j < (size_t)n;) {
        const double t = std::min(hlo + (double)j, (double)kPllTrigStick);
        // form 23 (the stuck trigOffset, 2^24): the three-candidate runner's stick form (pll_stick)
        const bool stick = kn.stick != 0;
        int form = t < 262144.0 ? 17 : t < 524288.0 ? 18 : t < (double)kPllPipeMinLow ? 19
                       : t < (double)kPllPipeMin5 ? 20 : t < (double)kPllPipeMin ? 21
                       : (!stick || t < (double)kPllTrigStick) ? 22 : 23;
        const double edge = form == 17 ? 262144.0 : form == 18 ? 524288.0 : form == 19 ? (double)kPllPipeMinLow
                          : form == 20 ? (double)kPllPipeMin5 : form == 21 ? (double)kPllPipeMin
                          : form == 22 && stick ? (double)kPllTrigStick : 0.0;
        size_t e = edge == 0.0 ? (size_t)n : std::min((size_t)(edge - hlo), (size_t)n);
        const bool cnt = form < 22 && ((kn.cnt >> (form - 17)) & 1) && kPllIdxSimds * n_streams <= n_simd;
        // a short call from 2^22 on the three-candidate form in 128-step intervals (launch form 25):
        // the per-block seam's 640 steps are 5 of them, of 256-step ones 2 and a tail
        if (short_call && form >= 22) {
            form = 25;
            e = (size_t)n;
        }
        const size_t len = e - j, ni = (size_t)pll_form_interval(form, cnt);
        // the 16-step forms (the index runner below 2^20, the wide three-wave form 24 from 2^20 to the
        // end of a short call) for a short call and for a range of few long intervals
        if (ni > 16 && len < kPllShortIntervals * ni) {
            if (form >= 20 && short_call) e = (size_t)n;
            run(form >= 20 ? 24 : form, false, j, e);
            j = e;
            continue;
        }
        // a long form: its whole intervals, then the tail on the 16-step form (when it is long enough
        // for one: below, it runs exactly in the long launch)
        size_t body = len;
#ifdef FMRX_AB_NO_TAIL_SPLIT  // A/B: the long form's tail on its own exact path
        if (false) {
#else
        if (ni > 16) {
#endif
            body = len / ni * ni;
            if (len - body < kPllShortTail) body = len;
        }
        run(form, cnt, j, j + body);
        if (body < len) run(form >= 20 ? 24 : form, false, j + body, e);
        j = e;
    }
#ifndef FMRX_AB_NO_DEMOTED_LAUNCH  // A/B timing only (a demoted stream's range would stay unrun)
    if (dem_from < (size_t)n)
        timed(kStTail, 0.0, [&] {
            idx_rc |= launch_pll_demoted(s, io + dem_from, (int)((size_t)n - dem_from), n_streams, stride, step, norm_bw,
                                         st, args + dem_from, (size_t)n, inject, spec_stats);
        });
#endif
    // the NCO of every sample from its trigArg (filter.cpp:170), in parallel, over the input in place
    if (nco)
        timed(kStNco, 0.0, [&] {
            hipLaunchKernelGGL(pll_nco_kernel, dim3((n + 255) / 256, n_streams), dim3(256), 0, s, io, n, stride,
                               spec ? args : io, spec ? (size_t)n : stride, nco_scale, phase_adjust, st);
        });
    else if (!spec)  // the trigArgs are in io itself: launch_pll_nco reads them from `side`
        (void)hipMemcpy2DAsync(reinterpret_cast<float*>(side + 4 * seg * (size_t)n_streams), (size_t)n * sizeof(float),
                               io, stride * sizeof(float), (size_t)n * sizeof(float), n_streams,
                               hipMemcpyDeviceToDevice, s);
    return idx_rc ? -2 : ok();
}

int launch_pll_nco(float* io, int n, int n_streams, size_t stride, float nco_scale, float phase_adjust, float* st,
                   const double* side, hipStream_t s) {
    if (n <= 0) return 0;
    const size_t seg = pll_seg_len(n, n_streams);
    const float* args = reinterpret_cast<const float*>(side + 4 * seg * (size_t)n_streams);  // n per stream
#ifdef FMRX_AB_NO_NCO
    return 0;  // A/B build only (timing: what the NCO beside the chains costs them; output wrong)
#endif
    hipLaunchKernelGGL(pll_nco_kernel, dim3((n + 255) / 256, n_streams), dim3(256), 0, s, io, n, stride, args,
                       (size_t)n, nco_scale, phase_adjust, st);
    return ok();
}

int launch_stereo_audio_range(const AudioLaunch& L, int b0, int b1, bool last, int n_streams, hipStream_t s) {
    if (L.n_blocks <= 0 || b0 < 0 || b1 > L.n_blocks || b0 > b1) return 0;
    const int H = L.at - 1;
    if (b1 > b0) {
        if (L.up == 1 && L.if_per_block <= kTileIf && L.frames_per_block <= kTileFrames && L.at <= kTileTaps &&
            L.frames_per_block * L.down <= L.if_per_block && (L.frames_per_block - kMonoDelay) * L.down >= H) {
            hipLaunchKernelGGL(stereo_audio_tile_kernel, dim3(b1 - b0, n_streams), dim3(128), 0, s, L, b0);
        } else {
            const dim3 grid(((L.frames_per_block + 127) / 128) * (b1 - b0), n_streams);
            hipLaunchKernelGGL(stereo_audio_kernel, grid, dim3(128), 0, s, L, b0);
        }
    }
    if (last) hipLaunchKernelGGL(stereo_state_kernel, dim3(n_streams), dim3(kTail), 0, s, L);
    return ok();
}

const float* pll_trig_args(const double* side, int n, int n_streams) {
    return reinterpret_cast<const float*>(side + 4 * pll_seg_len(n, n_streams) * (size_t)n_streams);
}

int launch_stereo_audio_small(const AudioLaunch& L, int n_streams, const float* args, size_t astride, float nco_scale,
                              float phase_adjust, float* pll_st, int demod_hist, hipStream_t s) {
    if (L.up != 1 || L.if_per_block > kTileIf || L.frames_per_block > kTileFrames || L.at > kTileTaps ||
        L.if_per_block < kTail || L.n_blocks < 1 || demod_hist > L.n_blocks * L.if_per_block)
        return -1;
    hipLaunchKernelGGL(stereo_audio_small_kernel, dim3(n_streams), dim3(128), 0, s, L, args, astride, nco_scale,
                       phase_adjust, pll_st, demod_hist);
    return ok();
}

int launch_stereo_audio(const AudioLaunch& L, int n_streams, hipStream_t s) {
    return launch_stereo_audio_range(L, 0, L.n_blocks, true, n_streams, s);
}

int launch_pll_fallback_test(int kind, const float* a, const float* b, size_t n, float* out, hipStream_t s) {
    if (n == 0) return 0;
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(pll_fallback_test_kernel, dim3(grid), dim3(256), 0, s, kind, a, b, n, out);
    return hipGetLastError() != hipSuccess;
}

}  // namespace fmrx
