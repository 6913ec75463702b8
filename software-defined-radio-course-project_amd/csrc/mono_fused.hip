// mono_fused.hip — the hot path: u8 I/Q -> RF LPF + decimate -> FM demod -> audio LPF
// (+decimate) -> S16, one launch, inputs and outputs in HBM, every intermediate on chip.
//
// Reference path:
//   readStdinBlockData + deinterleave   src/iofunc.cpp:62-69, src/project.cpp:56-62
//   resample(I), resample(Q) (RF LPF)   src/filter.cpp:67-103 via project.cpp:65-66
//   FMDemod                             src/filter.cpp:106-133 via project.cpp:69
//   resample (mono audio LPF)           src/filter.cpp:67-103 via project.cpp:146
//   S16 quantiser                       src/project.cpp:185-191
//
// Decomposition.  A stream's IF samples are cut into chunks of CIF = NT*R samples; one
// workgroup owns a contiguous run of chunks (a "segment") and walks it in order, carrying
// the overlap-save state from chunk to chunk exactly like the reference carries it from
// block to block: the last T-1 normalised I/Q pairs (RF history, filter.cpp:94-102), the
// last I/Q output (FMDemod prev_i/prev_q) and the last 50 demod samples (audio history).
// A segment starts with one "pre-roll" chunk whose outputs are discarded: it rebuilds that
// state from the raw bytes in front of the segment, so segments (and calls) are independent
// and the result equals the reference's sequential block loop bit for bit.
//
// Per chunk:
//   stage : coalesced 16-B loads of u8 I/Q (prefetched one chunk ahead into registers),
//           u8 -> float conversion, written to LDS as float2 (I,Q) pairs;
//   RF    : thread t computes R consecutive decimated outputs j = R t .. R t + R-1 from a
//           window of D(R-1)+T pairs; I and Q advance together in PACKED f32 ops
//           (v_pk_mul_f32 / v_pk_add_f32 with a broadcast tap: 2 f32 results per lane-op,
//           twice the scalar f32 rate on gfx950) and each output is a sequential sum in
//           ascending tap order with separately rounded mul and add (no FMA), as
//           filter.cpp:84-92;
//   demod : neighbour I/Q by a DPP wave shift (LDS for multi-wave workgroups), FMDemod in the
//           reference's mixed float/double precision;
//   audio : 51-tap decimating LPF over the demod window in LDS, quantise, store S16.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "dsp_device.h"
#include "mono_launch.h"

namespace fmrx {

namespace {

constexpr int kAudioTaps = 51;  // src/project.cpp:319 (modes 0 and 1: audio_interp = 1)
constexpr int kAH = kAudioTaps - 1;

template <int T, int D, int AD, int NT, int R>
struct MonoCfg {
    static constexpr int S = R * D;                     // pairs between adjacent threads
    static constexpr int G = (S % 4 == 2) ? 0 : 2;      // LDS pad pairs per S (bank spread)
    static constexpr int CIF = NT * R;                  // IF samples per chunk
    static constexpr int P = CIF * D;                   // I/Q pairs per chunk
    static constexpr int H = T - 1;                     // RF history pairs
    static constexpr int WH = T - 1 + D * (R - 1);      // highest window offset of a thread
    // LDS slot of buffer pair b (b = H + chunk-relative pair).  Pads of G pairs every S pairs
    // make the lane stride (S+G) pairs bank-conflict free for ds_read_b128, and (even b, b+1)
    // groups never straddle a pad, so every pair group is one aligned 16-B access.
    static constexpr int slot(int b) { return b + G * (b / S); }
    static constexpr int XB = slot(H + P + 2) + 4;      // LDS pairs
    static constexpr int NLD = (P / 2 + NT - 1) / NT;   // 4-B (2-pair) loads per thread/chunk
    static constexpr int LH0 = ((P - H) / 2) / NT;      // first load index holding history pairs
    static constexpr int CAmax = (CIF + AD - 1) / AD;   // max audio outputs in one chunk
    static constexpr int NG = (T + 1) / 2;              // tap groups: {0}, {1,2}, {3,4}, ...
    // Audio window (modes 0/1): GA consecutive chunks of demod are gathered before the audio
    // FIR runs once over them, two outputs per lane in packed ops: lane t owns window outputs
    // t and t + NA, whose samples are DX = AD NA apart.  The window (50 history samples + GA
    // chunks) is stored as DX + 50 float2 (sample s, sample s + DX), so one ds_read_b64 gives
    // a tap's two samples.  GA is the largest count (<= 3) whose outputs fit two per lane.
    static constexpr int na_for(int g) { return ((g * CIF + AD - 1) / AD + 1) / 2; }
    static constexpr int GA = na_for(3) <= NT ? 3 : na_for(2) <= NT ? 2 : 1;
    static constexpr int NA = na_for(GA);
    static constexpr int DX = AD * NA;
    static constexpr int DWI = DX + 50;  // float2 entries: sample s in .x (s < DX + 50), in .y (s >= DX)
    static_assert(2 * DX >= GA * CIF, "every window sample has a slot");
    static_assert(T % 2 == 1, "odd tap count");
    static_assert(S % 2 == 0 && H % 2 == 0, "pair groups must stay 16-B aligned");
    static_assert(P % 2 == 0, "chunk must be whole dwords");
    static_assert(CAmax <= NT, "one audio output per thread per chunk");
};

// 4 bytes (two I/Q pairs) of the virtual stream (halo ++ data ++ 0x80 padding) at byte
// offset `off` (a multiple of 4).  Bytes past the end read as 128, i.e. x = 0.0.
__device__ inline uint32_t load4(const uint8_t* in, const uint8_t* halo, long long off,
                                 long long total, long long halo_bytes) {
    if (off >= 0) {
        if (off + 4 <= total) return *reinterpret_cast<const uint32_t*>(in + off);
        return 0x80808080u;
    }
    return *reinterpret_cast<const uint32_t*>(halo + (halo_bytes + off));
}

// Signed sample of byte k of w after w ^= 0x80808080: s = u - 128 as an exact float.  One
// SDWA v_cvt_f32_i32 with sign extension per sample.  The FIR runs on s (the reference's
// x = s / 128): fl(c*s) * 2^-7 == fl(c*x) and every partial sum scales exactly too (all
// values stay far from the subnormal range), so the 2^-7 is applied once per output.
template <int K>
__device__ inline float sbyte(uint32_t w) {
    float f;
    if constexpr (K == 0)
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0" : "=v"(f) : "v"(w));
    else if constexpr (K == 1)
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(f) : "v"(w));
    else if constexpr (K == 2)
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2" : "=v"(f) : "v"(w));
    else
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3" : "=v"(f) : "v"(w));
    return f;
}

// The workgroup's LDS hand-offs.  A single-wave workgroup (NT = 64) needs no s_barrier and no
// drain: a wave's LDS instructions execute in issue order, so a read issued after a write (any
// lanes) sees it, and every value read into registers is waited for by its own s_waitcnt.
// Wavefront-scope fences around a wave barrier keep the compiler from moving LDS accesses
// across the hand-off, without the lgkmcnt(0) a workgroup fence emits.  Larger workgroups take
// __syncthreads().
template <int NT>
__device__ inline void chunk_sync() {
    if constexpr (NT == 64) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

// Workgroup -> (stream, chunk range).  Uniform: segment blockIdx % segs of stream
// blockIdx / segs.  With L.older_share (> 0, in 1/1024; even segs): the grid is two waves per
// SIMD, and the hardware dispatches workgroup w into the first wave slot of its SIMD and
// w + grid/2 into the second; the first-dispatched wave wins VALU arbitration (measured on
// MI355X: in 1,024 of 1,024 SIMD pairs it finished first, ~410 vs ~571 us with equal shares,
// profiles/r02/mono_stamps_*.json).  So w and w + grid/2 split one span of one stream, w
// taking older_share/1024 of it, and both finish together.  Every chunk is still covered
// exactly once and each range starts with its own pre-roll, so the output is unchanged.
__device__ inline void mono_share(const MonoLaunch& L, int w, int n_chunks, int* stream, int* c0, int* c1) {
    if (L.older_share > 0) {
        const int half = L.segs / 2;              // span pairs per stream
        const int H = (int)gridDim.x / 2;         // = n_streams * half
        const int p = w < H ? w : w - H;          // pair index
        const int s = p / half, q = p - s * half;
        const int p0 = (int)((long long)q * n_chunks / half), p1 = (int)((long long)(q + 1) * n_chunks / half);
        const int cut = p0 + (int)(((long long)(p1 - p0) * L.older_share) >> 10);
        *stream = s;
        *c0 = w < H ? p0 : cut;
        *c1 = w < H ? cut : p1;
        return;
    }
    *stream = w / L.segs;
    const int seg = w - *stream * L.segs;
    *c0 = (int)((long long)seg * n_chunks / L.segs);
    *c1 = (int)((long long)(seg + 1) * n_chunks / L.segs);
}

// ABL (timing ablations only, never selected in production): bit 1 skips the RF FIR, 2 the
// audio FIR, 4 the demod, 8 the byte conversion of the staging, 16 the global loads, 32 the
// staging writes.
// TR = 1 keeps the RF taps in VGPRs for the whole launch (the kernel is LDS-capped at two
// waves per SIMD, which leaves the register file room for them) instead of re-reading them
// from LDS once per chunk.  Single-wave workgroups (NT = 64) take the demod's neighbour I/Q
// by a DPP wave shift, larger ones through LDS.
// Measured and dropped: prefetching two chunks ahead, the audio stage once per
// two chunks in packed ops, a single-buffered demod window with R = 2 for three waves per
// SIMD, the audio FIR pipelined into the RF tap loop, staggered workgroup starts.
// AU > 1: the audio stage is the rational resampler of modes 2/3 (up AU, down AD; 51 taps
// per output phase of a 51*AU-tap prototype read from L.audio_coeff).
// Z0 (bit 1: RF, bit 2: the windowed audio FIR): tap 0 of the context's designed filter is
// +-0 (filter.cpp:33's window sin(0)^2 = 0 zeroes h[0] of every design), so its products are
// +-0 and the reference's sum 0.0f + (+-0) leaves +0 -- the state the accumulator starts in: the
// tap is skipped, bit for bit (inputs are finite: u8 samples, demod quotients).  The host
// selects it only after checking h[0] == +-0.
template <int T, int D, int AD, int NT, int R, int PD, int ABL = 0, int TR = 0, int AU = 1, int Z0 = 0>
__global__ void __launch_bounds__(NT) mono_fused_kernel(MonoLaunch L, MonoTaps taps) {
    using C = MonoCfg<T, D, AD, NT, R>;
    constexpr int CIF = C::CIF, P = C::P, H = C::H, S = C::S, G = C::G, NLD = C::NLD;
    constexpr int WH = C::WH, NG = C::NG;
    constexpr bool kShfl = NT == 64;
    static_assert(AU == 1 || ((long long)CIF * AU + AD - 1) / AD + 1 <= NT, "one audio output per thread");

    constexpr bool kWin = AU == 1;               // windowed packed audio stage (modes 0/1)
    constexpr int GA = C::GA;
    __shared__ float4 xb4[C::XB / 2 + 1];        // scaled (I,Q) pairs, two per float4
    // demod: modes 0/1 the paired audio window (50 history + GA chunks); modes 2/3 two
    // alternating 50 + chunk windows
    __shared__ float2 dwi[kWin ? C::DWI : 1];
    __shared__ float dbuf[kWin ? 1 : 2][kWin ? 1 : kAH + CIF];
    __shared__ float2v pbuf[kShfl ? 1 : 2][kShfl ? 1 : NT + 1];  // last RF output per thread
    __shared__ float2 ctab2[TR ? 1 : NG + 1];    // (c[2j-1], c[2j]); c[-1] = 0 (TR = 0 only)
    __shared__ float4 atab4[(kAudioTaps + 3) / 4];  // audio taps, 16-B aligned for broadcast ds_read_b128
    float* atab = reinterpret_cast<float*>(atab4);
    float* ctab = reinterpret_cast<float*>(ctab2);
    // window sample s (0..49 history, 50.. the GA chunks)
    auto wput = [&](int s, float v) {
        if (s < C::DWI) dwi[s].x = v;
        if (s >= C::DX) dwi[s - C::DX].y = v;
    };

    const int tid = threadIdx.x;
    const long long n_if = L.n_if;
    // chunk indices fit 32 bits for any HBM-resident stream (n_if / CIF < 2^31); positions
    // in the stream stay 64-bit
    const int n_chunks = (int)((n_if + CIF - 1) / CIF);
    // the next call's halo (halo_kernel's copy, fused): every workgroup moves a few 16-B words
    // of the streams' tails; nothing in this launch reads halo_next
    if (L.halo_next) {
        const size_t words = L.halo_bytes / 16, total = words * (size_t)(gridDim.x / L.segs);
        for (size_t i = (size_t)blockIdx.x * NT + tid; i < total; i += (size_t)gridDim.x * NT) {
            const size_t s = i / words, j = i - s * words, v = L.stream_bytes + 16 * j;  // into halo ++ iq
            const uint4 w = v < L.halo_bytes ? *reinterpret_cast<const uint4*>(L.halo + s * L.halo_stride + v)
                                             : *reinterpret_cast<const uint4*>(L.iq + s * L.iq_stride + (v - L.halo_bytes));
            *reinterpret_cast<uint4*>(L.halo_next + s * L.halo_bytes + 16 * j) = w;
        }
    }
    int stream, c0, c1;
    mono_share(L, (int)blockIdx.x, n_chunks, &stream, &c0, &c1);
    const int c_full = (int)(L.stream_bytes / (2 * P));  // chunks lying wholly in the data
    const int c_tail = n_if >= kAH ? (int)((n_if - kAH) / CIF) : -2;  // chunks holding the last 50
    if (c0 >= c1) return;
    // ABL & 64 (diagnostic build, results unchanged): shader-clock and 100 MHz stamps around
    // the workgroup's work, written only to L.stamps (nothing in the kernel reads them)
    unsigned long long st_t0 = 0, st_r0 = 0;
    if constexpr ((ABL & 64) != 0) {
        st_t0 = __builtin_amdgcn_s_memtime();
        st_r0 = __builtin_amdgcn_s_memrealtime();
    }
    const long long n_audio = n_if * AU / AD;

    const uint8_t* in = L.iq + (size_t)stream * L.iq_stride;
    const uint8_t* halo = L.halo + (size_t)stream * L.halo_stride;
    const long long total = (long long)L.stream_bytes;
    const long long hb = (long long)L.halo_bytes;

    if constexpr (TR == 0)
        for (int i = tid; i < 2 * (NG + 1); i += NT) ctab[i] = (i >= 1 && i <= T) ? taps.rf[i - 1] : 0.0f;
    for (int i = tid; i < kAudioTaps; i += NT) atab[i] = taps.audio[i];

    // ---- prologue: RF history in front of the pre-roll chunk (pairs [(c0-1)P - H, (c0-1)P))
    for (int i = tid; i < H / 2; i += NT) {
        const uint32_t w = load4(in, halo, ((long long)(c0 - 1) * P - H + 2 * i) * 2, total, hb) ^ 0x80808080u;
        xb4[C::slot(2 * i) / 2] = make_float4(sbyte<0>(w), sbyte<1>(w), sbyte<2>(w), sbyte<3>(w));
    }
    // Input prefetch, one chunk ahead.  It is always the same coalesced dword loads, from a
    // base clamped into the stream so that they never leave it; the few chunks that touch
    // the halo or run past the end (c outside [0, c_full)) are rebuilt at staging time.  One
    // load path keeps the loads asynchronous: with a second path the compiler merges the two
    // register sets right after issue, behind an s_waitcnt that exposes the HBM latency.
    uint32_t pf[NLD];
    auto fetch = [&](int cc) {
        if constexpr ((ABL & 16) != 0) {  // ablation: no global loads
#pragma unroll
            for (int l = 0; l < NLD; l++) pf[l] = (uint32_t)(cc * 77 + l * 77 + tid);
            return;
        }
        if (c_full == 0) return;  // stream shorter than a chunk: every chunk is rebuilt
        const int cl = cc < 0 ? 0 : (cc < c_full ? cc : c_full - 1);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(in + (size_t)cl * (2 * P)) + tid;
#pragma unroll
        for (int l = 0; l < NLD; l++)
            if ((P / 2) % NT == 0 || tid + l * NT < P / 2) pf[l] = src[l * NT];
    };
    fetch(c0 - 1);

    float2 creg[TR ? NG : 1];
    if constexpr (TR != 0) {  // straight from the kernel arguments (scalar loads)
#pragma unroll
        for (int j = 0; j < NG; j++) creg[j] = make_float2(j == 0 ? 0.0f : taps.rf[2 * j - 1], taps.rf[2 * j]);
    }
    int cur = 0;
    // (c0-1) CIF = AD aq + ar; for c0 = 0 this is (-(CIF/AD), -(CIF%AD)), which the first
    // increment turns into (0, 0), and ar is only read for c >= c0.
    long long aq = (long long)(c0 - 1) * CIF / AD;
    int ar = (int)((long long)(c0 - 1) * CIF - aq * AD);
    float2v carry = {0.0f, 0.0f};  // NT = 64: last RF output of the previous chunk
    float4 hist[NLD - C::LH0];     // staged groups of the chunk's last H pairs (loads l >= LH0)
    int slot = -1;                 // audio window slot of chunk c (-1: the pre-roll chunk)
    // modes 2/3: lane t's resampler offset t AD = au_qt AU + au_rt
    const int au_qt = AU > 1 ? tid * AD / AU : 0;
    const int au_rt = AU > 1 ? tid * AD - au_qt * AU : 0;
    long long wm0 = 0;             // first audio output of the current window
    int woff0 = 0;                 // its IF offset from the window start
    for (int c = c0 - 1; c < c1; c++) {
        // ---- stage chunk c: lane u writes pairs H+2u, H+2u+1 as one float4; consecutive
        // lanes write consecutive 16-B slots (conflict-free ds_write_b128).
        if ((ABL & 16) == 0 && !(c >= 0 && c < c_full)) {
            // rare (one uniform branch): rebuild this chunk's words from the halo / padding
#pragma unroll
            for (int l = 0; l < NLD; l++) {
                const int u = tid + l * NT;
                if ((P / 2) % NT == 0 || u < P / 2) pf[l] = load4(in, halo, (long long)c * (2 * P) + 4LL * u, total, hb);
            }
        }
#pragma unroll
        for (int l = 0; l < NLD; l++) {
            const int u = tid + l * NT;
            if ((P / 2) % NT == 0 || u < P / 2) {
                const uint32_t w = pf[l] ^ 0x80808080u;
                if constexpr ((ABL & 32) != 0) {  // ablation: no staging writes
                    asm volatile("" ::"v"(w));
                    continue;
                }
                const float4 f = (ABL & 8) != 0 ? make_float4(__uint_as_float(w), 0.f, 0.f, 0.f)
                                                : make_float4(sbyte<0>(w), sbyte<1>(w), sbyte<2>(w), sbyte<3>(w));
                xb4[C::slot(H + 2 * u) / 2] = f;
                if (l >= C::LH0) hist[l - C::LH0] = f;  // the chunk's last H pairs: next chunk's history
            }
        }
        chunk_sync<NT>();  // (A) chunk c staged, carry from c-1 in place
        if (c + 1 < c1) fetch(c + 1);

        // ---- RF LPF + decimate.  Thread t owns outputs j = R t + r, r < R, whose samples are
        // window offsets o = D r + T-1-k (window base pair S t).  Tap-outer order: at tap k all
        // R outputs take their k-th term, so each output is still an ascending-k sequential
        // sum, while samples slide through a register window (each LDS pair read once per
        // thread).  Group 0 = tap 0, group j = taps 2j-1, 2j; group j's new samples are the
        // pair (T-1-2j, T-2j); loads run PD groups ahead of use.
        if constexpr (TR != 0) {
            // Opaque per chunk, so LICM cannot hoist 101 loop-invariant (c, c) splats out of
            // the chunk loop; the products then broadcast a tap with op_sel instead.
#pragma unroll
            for (int j = 0; j < NG; j++) asm volatile("" : "+v"(creg[j]));
        }
        float2v acc[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = float2v{0.0f, 0.0f};
        int zero;  // opaque 0: keeps the tap reads as one base VGPR + immediate offsets
        asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
        const float2* cb = ctab2 + zero;
        float2v X[WH + 3];  // X[o] = window pair o, o in [0, WH+1]
        float2 cc[NG];
        const float4* wb = xb4 + ((S + G) / 2) * tid;
        auto ld = [&](int o) {  // o even: pairs (o, o+1), one ds_read_b128
            const float4 q = wb[(o + G * (o / S)) / 2];
            X[o] = float2v{q.x, q.y};
            X[o + 1] = float2v{q.z, q.w};
        };
        auto ldg = [&](int j) {  // loads of group j
            if (j < NG) {
                if constexpr (TR == 0) cc[j] = cb[j];
                if (j >= 1) ld(T - 1 - 2 * j);
            }
        };
#pragma unroll
        for (int o = T - 1; o <= WH; o += 2) ld(o);
#pragma unroll
        for (int j = 0; j < PD; j++) ldg(j);
#pragma unroll
        for (int j = 0; j < NG; j++) {
            if constexpr ((ABL & 1) != 0) break;
            ldg(j + PD);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int k = 2 * j - 1 + h;
                if (k >= ((Z0 & 1) ? 1 : 0)) {
                    const float2 cj = TR ? creg[TR ? j : 0] : cc[j];
                    const float ck = h == 0 ? cj.x : cj.y;
#pragma unroll
                    for (int r = 0; r < R; r++) {
                        const float2v p = X[T - 1 - k + D * r] * ck;
                        acc[r] = acc[r] + p;
                    }
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr ((ABL & 1) != 0) {
#pragma unroll
            for (int r = 0; r < R; r++) acc[r] = X[T - 1 + D * r] * (TR ? creg[0].y : cc[0].y);
        }
        // Pin the accumulators here: without it LLVM sinks the pure-register FIR chains past
        // the barrier to their first use (demod), keeping the whole sample window live.
        // The accumulators stay scaled by 2^7: FMDemod is invariant under an exact power-of-2
        // scaling of every I/Q (num and den scale by 2^14, every rounding with them; all
        // values are far from the subnormal and overflow ranges), and nothing else reads them.
#pragma unroll
        for (int r = 0; r < R; r++) asm volatile("" ::"v"(acc[r]));
        if constexpr (!kShfl) pbuf[cur][tid + 1] = acc[R - 1];
        chunk_sync<NT>();  // (B) all RF reads of xb done, pbuf visible

        // ---- carries for chunk c+1: RF history (the chunk's pairs [P - H, P) -> [0, H)) as
        // aligned 16-B pair groups (P and H are even, so groups never straddle a pad), written
        // from the staging registers (no LDS read and wait), last I/Q
#pragma unroll
        for (int l = C::LH0; l < NLD; l++) {
            const int i = tid + l * NT - (P - H) / 2;  // history group of staging lane u = tid + l NT
            if (i >= 0 && ((P / 2) % NT == 0 || tid + l * NT < P / 2)) xb4[C::slot(2 * i) / 2] = hist[l - C::LH0];
        }
        float2v prev;  // FM demod's previous I/Q: the neighbouring thread's / previous chunk's
        if constexpr (!kShfl) {
            if (tid == 0) pbuf[cur ^ 1][0] = pbuf[cur][NT];
            prev = pbuf[cur][tid];
        } else {
            // lane t - 1's last output by a DPP wave shift (wave_shr:1, one v_mov_b32_dpp a
            // component, no LDS round trip); lane 0 has no source lane and keeps `old`, the
            // previous chunk's carry
            prev.x = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(carry.x), __float_as_int(acc[R - 1].x),
                                                                0x138, 0xF, 0xF, false));
            prev.y = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(carry.y), __float_as_int(acc[R - 1].y),
                                                                0x138, 0xF, 0xF, false));
            carry.x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc[R - 1].x), NT - 1));
            carry.y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc[R - 1].y), NT - 1));
        }
        float d[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const float2v pv = r == 0 ? prev : acc[r - 1];
            if constexpr ((ABL & 4) != 0)
                d[r] = acc[r].x - pv.y;
            else
                d[r] = fm_demod_one(acc[r].x, acc[r].y, pv.x, pv.y);
        }
        const long long g0 = (long long)c * CIF + R * tid;  // IF index of d[0]
        if constexpr (kWin) {
            // window slot `slot` of the audio window; the pre-roll chunk (slot -1) leaves only
            // its last 50 samples, as the first window's history
            if (L.audio) {
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int jl = R * tid + r;
                    if (slot >= 0)
                        wput(kAH + slot * CIF + jl, d[r]);
                    else if (jl >= CIF - kAH)
                        wput(jl - (CIF - kAH), d[r]);
                }
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int jl = R * tid + r;
                dbuf[cur][kAH + jl] = d[r];
                if (jl >= CIF - kAH) dbuf[cur ^ 1][jl - (CIF - kAH)] = d[r];
            }
        }
        // Demod to global only for the split API / the chunk holding the stream's last 50
        // samples (one scalar test per chunk; the fused mono path skips it otherwise).
        if (c >= c0 && (L.demod || (L.demod_tail && c >= c_tail))) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                const long long g = g0 + r;
                if (g < n_if) {
                    if (L.demod)
                        L.demod[(size_t)stream * L.demod_stride + L.demod_hist + g] = d[r];
                    if (L.demod_tail && g >= n_if - kAH)
                        L.demod_tail[(size_t)stream * L.demod_tail_stride + (g - (n_if - kAH))] = d[r];
                }
            }
        }
        chunk_sync<NT>();  // (C) demod window complete
        // (c+1) CIF = AD aq1 + ar1
        long long aq1 = aq + CIF / AD;
        int ar1 = ar + CIF % AD;
        if (ar1 >= AD) { ar1 -= AD; aq1++; }

        // ---- audio LPF + decimate + quantise: outputs m with AD*m in this chunk.  Chunk c
        // starts at IF index pos = c CIF = AD aq + ar (tracked incrementally); its first audio
        // output is m0 = aq + (ar > 0), at chunk offset off0 = AD m0 - pos.
        if constexpr (AU > 1) {
            // rational resampler (project.cpp:146 with up = AU, down = AD): output m has phase
            // k0 = (m AD) mod AU and base j0 = floor(m AD / AU); it reads demod j0 - i, i < 51,
            // against coeff[k0 + i AU] (i ascending = k ascending, filter.cpp:84-92), and
            // belongs to the chunk that holds j0 (its 50 predecessors are the window history)
            // Lane t takes output mlo + t: with t AD = qt AU + rt (per lane, once) and
            // mlo AD = qb AU + rb (per chunk, scalar), j0 and k0 follow without a division.
            // The output's 51 taps are row k0 of L.audio_rows, read as 16-B vectors.
            if (L.audio && c >= c0) {
                const long long mlo = ((long long)c * CIF * AU + AD - 1) / AD;
                const long long mhi = ((long long)(c + 1) * CIF * AU + AD - 1) / AD;
                const long long m = mlo + tid;
                if (m < mhi && m < n_audio) {
                    const long long nb = mlo * AD;
                    const long long qb = nb / AU;
                    const int rb = (int)(nb - qb * AU);
                    const int rr = rb + au_rt;
                    const int wrap = rr >= AU ? 1 : 0;
                    const int k0 = rr - wrap * AU;
                    const int jl = (int)(qb - (long long)c * CIF) + au_qt + wrap;  // j0 - c CIF
                    const float* dw = &dbuf[cur][kAH + jl];
                    const float4* row = reinterpret_cast<const float4*>(L.audio_rows + (size_t)k0 * kAudioRow);
                    // every load first -- the row's 13 16-B vectors (L2-resident) and the 51
                    // window samples -- then the sequential sum: one exposed latency per output
                    // instead of one per few taps (the FIR's registers are free here)
                    float4 cq[kAudioRow / 4];
                    float xv[kAudioTaps];
#pragma unroll
                    for (int i4 = 0; i4 < kAudioRow / 4; i4++) cq[i4] = row[i4];
#pragma unroll
                    for (int i = 0; i < kAudioTaps; i++) xv[i] = dw[-i];
                    __builtin_amdgcn_sched_barrier(0);
                    float a = 0.0f;
#pragma unroll
                    for (int i4 = 0; i4 < kAudioRow / 4; i4++) {
                        const float cv[4] = {cq[i4].x, cq[i4].y, cq[i4].z, cq[i4].w};
#pragma unroll
                        for (int e = 0; e < 4; e++) {
                            const int i = 4 * i4 + e;
                            if (i < kAudioTaps) {
                                const float p = cv[e] * xv[i];
                                a = a + p;
                            }
                        }
                    }
                    const size_t oi = (size_t)stream * (size_t)n_audio + (size_t)m;
                    L.pcm[oi] = quantize_s16(a);
                    if (L.mono) L.mono[oi] = a;
                }
            }
        } else if (L.audio && slot >= 0) {
            // mono audio LPF + decimate (project.cpp:146, up = 1) over the window of chunks
            // c - slot .. c, run once the window is full (or the segment ends).  Lane t owns
            // window outputs t and t + NA and advances them together in packed ops: each is
            // still an ascending-tap sequential sum of separately rounded products
            // (filter.cpp:84-92).
            if (slot == 0) {  // first output of the window and its offset in the window
                wm0 = aq + (ar > 0);
                woff0 = ar > 0 ? AD - ar : 0;
            }
            if (slot == GA - 1 || c == c1 - 1) {
                long long mend = aq1 + (ar1 > 0);  // first output of the next window
                if (mend > n_audio) mend = n_audio;
                const long long nw = mend - wm0;
                if (tid < C::NA && tid < nw) {
                    // base[kAH - k] = (sample o_a - k, sample o_a + DX - k), o_a = woff0 + AD t
                    const float2* base = dwi + woff0 + AD * tid;
                    float2v a2 = {0.0f, 0.0f};
                    // The taps first (13 broadcast ds_read_b128 from one base + immediates), then
                    // the window samples kAP taps ahead of their products: the FIR's registers
                    // are free here, so the loop waits on LDS once instead of every few taps.
                    constexpr int k0 = (Z0 & 2) ? 1 : 0, k1 = (ABL & 2) != 0 ? 1 : kAudioTaps, kAP = 16;
                    int zero_a;  // opaque 0: one base VGPR + immediate offsets
                    asm volatile("v_mov_b32 %0, 0" : "=v"(zero_a));
                    const float4* at4 = atab4 + zero_a;
                    float4 tq[(kAudioTaps + 3) / 4];
#pragma unroll
                    for (int q = 0; q < (kAudioTaps + 3) / 4; q++) tq[q] = at4[q];
                    float2 xs[kAudioTaps];
#pragma unroll
                    for (int k = k0; k < k1 && k < k0 + kAP; k++) xs[k] = base[kAH - k];
#pragma unroll
                    for (int k = k0; k < k1; k++) {
                        if (k + kAP < k1) xs[k + kAP] = base[kAH - k - kAP];
                        const float4 t4 = tq[k / 4];
                        const float tk = (k & 3) == 0 ? t4.x : (k & 3) == 1 ? t4.y : (k & 3) == 2 ? t4.z : t4.w;
                        const float2v p = float2v{xs[k].x, xs[k].y} * tk;
                        a2 = a2 + p;
                    }
                    const size_t oi = (size_t)stream * (size_t)n_audio + (size_t)(wm0 + tid);
                    L.pcm[oi] = quantize_s16(a2.x);
                    if (L.mono) L.mono[oi] = a2.x;
                    if (tid + C::NA < nw) {
                        L.pcm[oi + C::NA] = quantize_s16(a2.y);
                        if (L.mono) L.mono[oi + C::NA] = a2.y;
                    }
                }
                if (slot == GA - 1) {
                    chunk_sync<NT>();  // window reads done: its last 50 samples become history,
                    // written from this chunk's demod registers (window sample GA CIF + i is
                    // chunk output jl = CIF - 50 + i) instead of read back from the window
#pragma unroll
                    for (int r = 0; r < R; r++) {
                        const int jl = R * tid + r;
                        if (jl >= CIF - kAH) wput(jl - (CIF - kAH), d[r]);
                    }
                }
            }
        }
        cur ^= 1;
        aq = aq1;
        ar = ar1;
        if constexpr (kWin) slot = slot + 1 == GA ? 0 : slot + 1;
    }
    if constexpr ((ABL & 64) != 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_ID: SIMD, CU, SE
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
        if (tid == 0 && L.stamps) {  // per-lane address: a plain vector store
            unsigned long long* o = L.stamps + 6 * ((size_t)blockIdx.x + tid);
            o[0] = st_t0;
            o[1] = t1;
            o[2] = st_r0;
            o[3] = r1;
            o[4] = hw;
            o[5] = xcc;
        }
    }
}

template <int T, int D, int AD, int NT, int R, int PD, int TR = 0, int AU = 1, int Z0 = 0>
int launch_variant(const MonoLaunch& L, int n_streams, const MonoTaps& taps, hipStream_t s) {
    hipLaunchKernelGGL((mono_fused_kernel<T, D, AD, NT, R, PD, 0, TR, AU, Z0>), dim3(n_streams * L.segs), dim3(NT), 0,
                       s, L, taps);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// h[0] == +-0 (Z0 above)
bool tap0_zero(float h0) { return (__builtin_bit_cast(uint32_t, h0) & 0x7FFFFFFFu) == 0; }

// Tunables.  The default was picked by measurement on MI355X (tools/tune_list.py); the other
// variants stay compiled for the tuning sweep (FMRX_MONO_VARIANT=<index>).
struct Variant {
    int nt, r, pd, tr, wg_per_cu;  // wg_per_cu: resident workgroups per CU (LDS-limited)
};
constexpr Variant kVariants[] = {{256, 3, 3, 0, 2}, {128, 3, 3, 0, 4}, {64, 3, 3, 0, 8}, {128, 5, 3, 0, 3},
                                 {256, 3, 5, 0, 2}, {64, 3, 3, 1, 8}, {64, 3, 4, 1, 8}};
constexpr int kDefaultVariant = 6;  // one wave per workgroup, taps in VGPRs, 4 groups of prefetch

int variant_index() {  // FMRX_MONO_VARIANT: tuning sweeps only
    static int v = [] {
        const char* e = getenv("FMRX_MONO_VARIANT");
        const int i = e ? atoi(e) : kDefaultVariant;
        return (i >= 0 && i < (int)(sizeof kVariants / sizeof kVariants[0])) ? i : kDefaultVariant;
    }();
    return v;
}

}  // namespace

size_t mono_halo_bytes(int rf_taps, int rf_decim, int /*audio_down*/) {
    size_t pairs = 0;  // the largest pre-roll chunk over all variants + RF history
    for (const Variant& v : kVariants) pairs = std::max(pairs, (size_t)v.nt * v.r * rf_decim);
    pairs += (size_t)(rf_taps - 1);
    return ((2 * pairs + 15) / 16) * 16 + 16;
}

long long mono_chunks(long long n_if, int /*rf_taps*/, int rf_decim, int /*audio_down*/) {
    const Variant v = kVariants[variant_index()];
    const long long cif = rf_decim == 9 ? 64 * 2 : (long long)v.nt * v.r;
    return (n_if + cif - 1) / cif;
}

int mono_wg_per_cu(int rf_decim) { return rf_decim == 9 ? 8 : kVariants[variant_index()].wg_per_cu; }

#ifdef FMRX_AB_ABLATE
// A/B build only (Makefile `ab`, AB=-DFMRX_AB_ABLATE; tools/gpu_ablate.sh): the stage-removal
// bitmask from the environment -- timing experiments, results wrong by design, so never in the
// product library
int ablation() {
    static int a = [] {
        const char* e = getenv("FMRX_ABLATE");
        return e ? atoi(e) : 0;
    }();
    return a;
}
#endif

template <int ABL>
int launch_ablation(const MonoLaunch& L, int n_streams, const MonoTaps& taps, hipStream_t s) {
    hipLaunchKernelGGL((mono_fused_kernel<101, 10, 5, 64, 3, 4, ABL, 1>), dim3(n_streams * L.segs), dim3(64), 0,
                       s, L, taps);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_mono_fused(const MonoLaunch& L, int n_streams, int rf_taps, int rf_decim,
                      int audio_up, int audio_down, const MonoTaps& taps, hipStream_t s) {
    const int vi = variant_index();
    if (audio_up > 1 && L.audio) {
        // modes 2/3 with the rational resampler fused (the default kernel shape; mode 3's odd
        // decimation keeps R = 2)
        if (rf_decim == 10 && audio_up == 147 && audio_down == 800) {
            const bool z = tap0_zero(taps.rf[0]);
            if (rf_taps == 51 && z) return launch_variant<51, 10, 800, 64, 3, 4, 1, 147, 1>(L, n_streams, taps, s);
            if (rf_taps == 101 && z) return launch_variant<101, 10, 800, 64, 3, 4, 1, 147, 1>(L, n_streams, taps, s);
            if (rf_taps == 51) return launch_variant<51, 10, 800, 64, 3, 4, 1, 147>(L, n_streams, taps, s);
            if (rf_taps == 101) return launch_variant<101, 10, 800, 64, 3, 4, 1, 147>(L, n_streams, taps, s);
        }
        if (rf_decim == 9 && audio_up == 441 && audio_down == 2560) {
            if (rf_taps == 51) return launch_variant<51, 9, 2560, 64, 2, 3, 0, 441>(L, n_streams, taps, s);
            if (rf_taps == 101) return launch_variant<101, 9, 2560, 64, 2, 3, 0, 441>(L, n_streams, taps, s);
        }
        return -1;
    }
    if (audio_up > 1) audio_down = 5;  // RF + demod only (stereo engine, split API): any compiled AD
    // clock / occupancy stamps (fmrx_debug_mono_stamps): the default kernel plus stamps
    if (L.stamps && rf_taps == 101 && rf_decim == 10 && audio_down == 5 && vi == kDefaultVariant)
        return launch_ablation<64>(L, n_streams, taps, s);
#ifdef FMRX_AB_ABLATE
    if (const int a = ablation(); a != 0 && rf_taps == 101 && rf_decim == 10) {
        switch (a) {
            case 1: return launch_ablation<1>(L, n_streams, taps, s);
            case 2: return launch_ablation<2>(L, n_streams, taps, s);
            case 4: return launch_ablation<4>(L, n_streams, taps, s);
            case 6: return launch_ablation<6>(L, n_streams, taps, s);
            case 8: return launch_ablation<8>(L, n_streams, taps, s);
            case 14: return launch_ablation<14>(L, n_streams, taps, s);
            case 15: return launch_ablation<15>(L, n_streams, taps, s);
            case 16: return launch_ablation<16>(L, n_streams, taps, s);
            case 30: return launch_ablation<30>(L, n_streams, taps, s);
            case 32: return launch_ablation<32>(L, n_streams, taps, s);
            case 31: return launch_ablation<31>(L, n_streams, taps, s);
            case 62: return launch_ablation<62>(L, n_streams, taps, s);
            case 63: return launch_ablation<63>(L, n_streams, taps, s);
            case 64: return launch_ablation<64>(L, n_streams, taps, s);
            default: break;
        }
    }
#endif
    // the default variant skips tap 0 (Z0) when the designs have h[0] = +-0 (always, for the
    // context's own taps; both FIRs then), the sweep variants keep it
    const bool z0 = tap0_zero(taps.rf[0]) && (!L.audio || tap0_zero(taps.audio[0]));
#define FMRX_V(T_, D_, AD_, I_, NT_, R_, PD_, TR_)                                              \
    if (rf_taps == T_ && rf_decim == D_ && audio_down == AD_ && vi == I_) {                     \
        if (I_ == kDefaultVariant && z0)                                                        \
            return launch_variant<T_, D_, AD_, NT_, R_, PD_, TR_, 1, (I_ == kDefaultVariant ? 3 : 0)>(L, n_streams, \
                                                                                                      taps, s);  \
        return launch_variant<T_, D_, AD_, NT_, R_, PD_, TR_>(L, n_streams, taps, s);           \
    }
#define FMRX_ALL(T_, D_, AD_)              \
    FMRX_V(T_, D_, AD_, 0, 256, 3, 3, 0)   \
    FMRX_V(T_, D_, AD_, 1, 128, 3, 3, 0)   \
    FMRX_V(T_, D_, AD_, 2, 64, 3, 3, 0)    \
    FMRX_V(T_, D_, AD_, 3, 128, 5, 3, 0)   \
    FMRX_V(T_, D_, AD_, 4, 256, 3, 5, 0)   \
    FMRX_V(T_, D_, AD_, 5, 64, 3, 3, 1)    \
    FMRX_V(T_, D_, AD_, 6, 64, 3, 4, 1)
    FMRX_ALL(51, 10, 5)    // mode 0 (and mode 2's RF stage), reference taps
    FMRX_ALL(101, 10, 5)   // mode 0, 101-tap RF (BASELINE configs[1])
    FMRX_ALL(51, 4, 6)     // mode 1
    FMRX_ALL(101, 4, 6)
    // mode 3 (odd decimation 9): R = 2 keeps the per-thread stride S = 18 even; the
    // polyphase 441/2560 audio stage runs separately, so AD is a placeholder here
    if (rf_decim == 9 && rf_taps == 51) return launch_variant<51, 9, 5, 64, 2, 3>(L, n_streams, taps, s);
    if (rf_decim == 9 && rf_taps == 101) return launch_variant<101, 9, 5, 64, 2, 3>(L, n_streams, taps, s);
#undef FMRX_ALL
#undef FMRX_V
    return -1;
}

}  // namespace fmrx
