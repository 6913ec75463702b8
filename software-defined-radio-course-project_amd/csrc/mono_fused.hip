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
//   demod : neighbour I/Q via LDS, FMDemod in the reference's mixed float/double precision;
//   audio : 51-tap decimating LPF over the demod window in LDS, quantise, store S16.
#include <hip/hip_runtime.h>

#include "dsp_device.h"
#include "fmrx_internal.h"

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
    // LDS slot of buffer pair b (b = H + chunk-relative pair).  The +1 shift and the pad
    // placement make every (odd o, o+1) window pair one aligned 16-B ds_read_b128 that never
    // straddles a pad, and make the lane stride (S+G) pairs bank-conflict free.
    static constexpr int pad(int b) { return b + G * ((b + 1) / S); }
    static constexpr int slot(int b) { return pad(b) + 1; }
    static constexpr int XB = slot(H + P + 2) + 2;      // LDS pairs
    static constexpr int NL = (2 * P / 16 + NT - 1) / NT;  // 16-B loads per thread per chunk
    static constexpr int CAmax = (CIF + AD - 1) / AD + 1;  // audio outputs per chunk (bound)
    static_assert(T % 2 == 1, "odd tap count (window pairs align on odd offsets)");
    static_assert(D % 2 == 0 && S % 2 == 0, "even decimation keeps pair groups aligned");
    static_assert((2 * P) % 16 == 0, "chunk must be a whole number of 16-B loads");
    static_assert(CAmax <= NT, "one audio output per thread per chunk");
};

// 16 bytes of the virtual stream (halo ++ data ++ 0x80 padding) at byte offset `off`
// (a multiple of 16).  Bytes past the end read as 128, i.e. x = 0.0.
__device__ inline uint4 load16(const uint8_t* in, const uint8_t* halo, long long off,
                               long long total, long long halo_bytes) {
    if (off >= 0) {
        if (off + 16 <= total) return *reinterpret_cast<const uint4*>(in + off);
        return make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
    }
    return *reinterpret_cast<const uint4*>(halo + (halo_bytes + off));
}

__device__ inline uint32_t load_pair(const uint8_t* in, const uint8_t* halo, long long pair,
                                     long long total, long long halo_bytes) {
    const long long off = 2 * pair;
    const uint8_t* p;
    if (off >= 0) {
        if (off + 2 > total) return 0x8080u;
        p = in + off;
    } else {
        p = halo + (halo_bytes + off);
    }
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8);
}

__device__ inline float2v byte_pair(uint32_t w) {
    return float2v{u8_to_sample(w & 0xFFu), u8_to_sample((w >> 8) & 0xFFu)};
}

template <int T, int D, int AD, int NT, int R>
__global__ void __launch_bounds__(NT) mono_fused_kernel(MonoLaunch L, MonoTaps taps) {
    using C = MonoCfg<T, D, AD, NT, R>;
    constexpr int CIF = C::CIF, P = C::P, H = C::H, S = C::S, G = C::G, NL = C::NL;
    constexpr int WH = C::WH;

    __shared__ float4 xb4[C::XB / 2 + 1];        // (I,Q) pairs, two per float4
    __shared__ float dbuf[2][kAH + CIF];         // demod window: 50 history + chunk
    __shared__ float2v pbuf[2][NT + 1];          // last RF output of each thread (+carry)
    __shared__ float4 ctab4[(T + 3) / 4 + 1];    // RF taps (broadcast reads)
    __shared__ float atab[kAudioTaps + 1];       // audio taps
    float2v* xb = reinterpret_cast<float2v*>(xb4);
    float* ctab = reinterpret_cast<float*>(ctab4);

    const int tid = threadIdx.x;
    const int stream = blockIdx.x / L.segs;
    const int seg = blockIdx.x - stream * L.segs;
    const long long n_if = L.n_if;
    const long long n_chunks = (n_if + CIF - 1) / CIF;
    const long long c0 = seg * n_chunks / L.segs;
    const long long c1 = (seg + 1) * n_chunks / L.segs;
    if (c0 >= c1) return;
    const long long n_audio = n_if / AD;

    const uint8_t* in = L.iq + (size_t)stream * L.stream_bytes;
    const uint8_t* halo = L.halo + (size_t)stream * L.halo_bytes;
    const long long total = (long long)L.stream_bytes;
    const long long hb = (long long)L.halo_bytes;

    for (int i = tid; i < 4 * ((T + 3) / 4 + 1); i += NT) ctab[i] = i < T ? taps.rf[i] : 0.0f;
    for (int i = tid; i < kAudioTaps; i += NT) atab[i] = taps.audio[i];

    // ---- prologue: RF history in front of the pre-roll chunk (pairs [(c0-1)P - H, (c0-1)P))
    {
        const long long p0 = (c0 - 1) * (long long)P - H;
        for (int i = tid; i < H; i += NT) xb[C::slot(i)] = byte_pair(load_pair(in, halo, p0 + i, total, hb));
    }
    uint4 pf[NL];
#pragma unroll
    for (int l = 0; l < NL; l++) {
        const int u = tid + l * NT;
        if (u < 2 * P / 16) pf[l] = load16(in, halo, (c0 - 1) * 2LL * P + 16LL * u, total, hb);
    }

    int cur = 0;
    for (long long c = c0 - 1; c < c1; c++) {
        // ---- stage chunk c: 16 B = 8 pairs b0..b0+7 (b0 = H + 8u even) -> LDS slots.
        // slot(b) is odd for even b, so the group is written as b0 | b0+1..b0+6 | b0+7.
#pragma unroll
        for (int l = 0; l < NL; l++) {
            const int u = tid + l * NT;
            if (u < 2 * P / 16) {
                const int b0 = H + 8 * u;
                const uint32_t w[4] = {pf[l].x, pf[l].y, pf[l].z, pf[l].w};
                float v[16];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    v[4 * q + 0] = u8_to_sample(w[q] & 0xFFu);
                    v[4 * q + 1] = u8_to_sample((w[q] >> 8) & 0xFFu);
                    v[4 * q + 2] = u8_to_sample((w[q] >> 16) & 0xFFu);
                    v[4 * q + 3] = u8_to_sample(w[q] >> 24);
                }
                xb[C::slot(b0)] = float2v{v[0], v[1]};
#pragma unroll
                for (int q = 0; q < 3; q++)
                    xb4[C::slot(b0 + 1 + 2 * q) / 2] =
                        make_float4(v[2 + 4 * q], v[3 + 4 * q], v[4 + 4 * q], v[5 + 4 * q]);
                xb[C::slot(b0 + 7)] = float2v{v[14], v[15]};
            }
        }
        __syncthreads();  // (A) chunk c staged, carry from c-1 in place
        if (c + 1 < c1) {
#pragma unroll
            for (int l = 0; l < NL; l++) {
                const int u = tid + l * NT;
                if (u < 2 * P / 16) pf[l] = load16(in, halo, (c + 1) * 2LL * P + 16LL * u, total, hb);
            }
        }

        // ---- RF LPF + decimate.  Thread t owns outputs j = R t + r, r < R, whose samples are
        // window offsets o = D r + T-1-k (window base pair S t).  Tap-outer order: at tap k all
        // R outputs take their k-th term, so each output is still an ascending-k sequential
        // sum, while the samples slide through a register window (each LDS pair read once) and
        // each tap is one broadcast LDS value.
        float2v acc[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = float2v{0.0f, 0.0f};
        int zero;  // opaque 0: keeps the tap reads as one base VGPR + immediate offsets
        asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
        const float* cbase = ctab + zero;
        float2v X[WH + 2];  // X[o + 1] = window pair o, o in [-1, WH]
        // slot(S t + o) = (S+G) t + o + 1 + G*((o+1)/S): a per-thread base plus a compile-time
        // offset, so every read is ds_read_b128 base, offset:imm.
        const float4* wb = xb4 + ((S + G) / 2) * tid;
        auto ld = [&](int o) {  // o odd: pairs (o, o+1) in one ds_read_b128
            const float4 q = wb[(o + 1 + G * ((o + 1) / S)) / 2];
            X[o + 1] = float2v{q.x, q.y};
            X[o + 2] = float2v{q.z, q.w};
        };
#pragma unroll
        for (int o = WH - 1; o >= T; o -= 2) ld(o);
        ld(T - 2);
        ld(T - 4);
#pragma unroll
        for (int k = 0; k < T; k += 2) {
            if (T - 6 - k >= -1) ld(T - 6 - k);  // two steps of prefetch distance
            const float2 cc = *reinterpret_cast<const float2*>(&cbase[k]);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if (k + h < T) {
                    const float ck = h == 0 ? cc.x : cc.y;
#pragma unroll
                    for (int r = 0; r < R; r++) {
                        const float2v p = X[T - 1 - (k + h) + D * r + 1] * ck;
                        acc[r] = acc[r] + p;
                    }
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // Pin the accumulators here: without it LLVM sinks the pure-register FIR chains past
        // the barrier to their first use (demod), keeping the whole sample window live.
#pragma unroll
        for (int r = 0; r < R; r++) asm volatile("" ::"v"(acc[r]));
        pbuf[cur][tid + 1] = acc[R - 1];
        __syncthreads();  // (B) all RF reads of xb done, pbuf visible

        // ---- carries for chunk c+1: RF history (pairs [P, P+H) -> [0, H)), last I/Q
        for (int i = tid; i < H; i += NT) xb[C::slot(i)] = xb[C::slot(P + i)];
        if (tid == 0) pbuf[cur ^ 1][0] = pbuf[cur][NT];

        // ---- FM demod (prev from the neighbouring thread / previous chunk)
        const float2v prev = pbuf[cur][tid];
        float d[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const float2v pv = r == 0 ? prev : acc[r - 1];
            d[r] = fm_demod_one(acc[r].x, acc[r].y, pv.x, pv.y);
        }
        const long long g0 = c * CIF + R * tid;  // IF index of d[0]
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int jl = R * tid + r;
            dbuf[cur][kAH + jl] = d[r];
            if (jl >= CIF - kAH) dbuf[cur ^ 1][jl - (CIF - kAH)] = d[r];
        }
        if (c >= c0) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                const long long g = g0 + r;
                if (g < n_if) {
                    if (L.demod)
                        L.demod[(size_t)stream * L.demod_stride + L.demod_hist + g] = d[r];
                    if (L.demod_tail && g >= n_if - kAH)
                        L.demod_tail[(size_t)stream * kAH + (g - (n_if - kAH))] = d[r];
                }
            }
        }
        __syncthreads();  // (C) demod window complete

        // ---- audio LPF + decimate + quantise: outputs m with AD*m in this chunk
        if (L.audio && c >= c0) {
            const long long m0 = (c * CIF + AD - 1) / AD;
            const long long m = m0 + tid;
            if (tid < C::CAmax && AD * m < (c + 1) * CIF && m < n_audio) {
                const float* dw = &dbuf[cur][AD * m - c * CIF + kAH];
                float a = 0.0f;
#pragma unroll
                for (int k = 0; k < kAudioTaps; k++) {
                    const float p = atab[k] * dw[-k];
                    a = a + p;
                }
                const size_t oi = (size_t)stream * (size_t)n_audio + (size_t)m;
                L.pcm[oi] = quantize_s16(a);
                if (L.mono) L.mono[oi] = a;
            }
        }
        cur ^= 1;
    }
}

template <int T, int D, int AD, int NT, int R>
int launch_variant(const MonoLaunch& L, int n_streams, const MonoTaps& taps, hipStream_t s) {
    const dim3 grid(n_streams * L.segs), block(NT);
    hipLaunchKernelGGL((mono_fused_kernel<T, D, AD, NT, R>), grid, block, 0, s, L, taps);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Tunables per (decim, audio_down) family.
constexpr int kNT = 256;
constexpr int kR = 3;

}  // namespace

size_t mono_halo_bytes(int rf_taps, int rf_decim, int /*audio_down*/) {
    const size_t pairs = (size_t)kNT * kR * rf_decim + (size_t)(rf_taps - 1);
    return ((2 * pairs + 15) / 16) * 16 + 16;
}

long long mono_chunks(long long n_if, int /*rf_taps*/, int /*rf_decim*/, int /*audio_down*/) {
    const long long cif = (long long)kNT * kR;
    return (n_if + cif - 1) / cif;
}

int launch_mono_fused(const MonoLaunch& L, int n_streams, int rf_taps, int rf_decim,
                      int audio_down, const MonoTaps& taps, hipStream_t s) {
#define FMRX_VARIANT(T_, D_, AD_)                                                  \
    if (rf_taps == T_ && rf_decim == D_ && audio_down == AD_)                      \
        return launch_variant<T_, D_, AD_, kNT, kR>(L, n_streams, taps, s);
    FMRX_VARIANT(51, 10, 5)    // mode 0, reference taps
    FMRX_VARIANT(101, 10, 5)   // mode 0, 101-tap RF (BASELINE config 2)
    FMRX_VARIANT(51, 4, 6)     // mode 1
    FMRX_VARIANT(101, 4, 6)
#undef FMRX_VARIANT
    return -1;
}

}  // namespace fmrx
