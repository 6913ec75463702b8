// prims.hip — the reference's filter.h primitives as standalone device kernels (one
// launch per call, device buffers), plus the small bookkeeping kernels of the runtime.
// These back the per-primitive C ABI (fmrx_resample, fmrx_fm_demod, ...) that mirrors
// include/filter.h:15-27 one function for one function.  The fused hot path does not use
// them; they exist so a caller of the reference API can swap any single stage.
#include <hip/hip_runtime.h>

#include "dsp_device.h"
#include "fmrx_internal.h"

namespace fmrx {

namespace {

inline int blocks_for(size_t n, int bs) { return (int)((n + bs - 1) / bs); }

// src/filter.cpp:67-103 resample: one thread per output; input index j < 0 reads the
// carried state (taps-1 floats).  Ascending-k sequential sum, separate mul and add.
__global__ void resample_kernel(float* __restrict__ out, const float* __restrict__ state,
                                const float* __restrict__ in, const float* __restrict__ coeff,
                                int taps, int up, int down, int n_out) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_out) return;
    const long long nd = (long long)n * down;
    float acc = 0.0f;
    for (int k = (int)(nd % up); k < taps; k += up) {
        const long long j = (nd - k) / up;
        const float x = j >= 0 ? in[j] : state[(taps - 1) + j];
        const float p = coeff[k] * x;
        acc = acc + p;
    }
    out[n] = acc;
}

// The same resample for the rational audio resamplers (project.cpp:146; 147/800 and
// 441/2560 in modes 2/3): output n has phase k0 = (n down) mod up and base input j0 =
// floor(n down / up); its taps are coeff[k0 + i up] against in[j0 - i], i ascending (= k
// ascending, as filter.cpp:84-92).  One division per output instead of one per tap; the
// prototype keeps its order, so at tap step i a wave's lanes read inside one up-wide window.
// All streams in one launch (grid.y = stream); the S16 quantiser (project.cpp:185-191) is
// fused, the float output is written only when the caller asks for it (out != nullptr).
__global__ void polyphase_kernel(PolyStreams P) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = blockIdx.y;
    if (n >= P.n_out) return;
    const float* in = P.in + (size_t)s * P.in_stride;
    const float* state = P.state + (size_t)s * P.state_stride;
    const int taps = P.taps, up = P.up;
    const long long nd = (long long)n * P.down;
    const long long j0 = nd / up;
    const int k0 = (int)(nd - j0 * up);
    const int cnt = (taps - k0 + up - 1) / up;  // taps of this phase: k0 + i up < taps
    const float* c = P.coeff + k0;
    float acc = 0.0f;
    if (cnt == 51 && j0 >= 50) {
        // every phase of the modes 2/3 prototypes (7497 = 51 x 147, 22491 = 51 x 441): a
        // fixed trip count unrolls, so all 102 loads are in flight before the sum starts
        const float* x = in + j0;
#pragma unroll
        for (int i = 0; i < 51; i++) {
            const float p = c[i * up] * x[-i];
            acc = acc + p;
        }
    } else if (j0 >= cnt - 1) {  // the whole window lies in this call's input
        const float* x = in + j0;
        for (int i = 0; i < cnt; i++) {
            const float p = c[i * up] * x[-i];
            acc = acc + p;
        }
    } else {
        for (int i = 0; i < cnt; i++) {
            const long long j = j0 - i;
            const float x = j >= 0 ? in[j] : state[(taps - 1) + j];
            const float p = c[i * up] * x;
            acc = acc + p;
        }
    }
    if (P.out) P.out[(size_t)s * P.out_stride + n] = acc;
    P.pcm[(size_t)s * P.pcm_stride + n] = quantize_s16(acc);
}

// dst[s][i] = src[s][i], i < n, every stream in one launch (grid.y = stream).  dst and src
// may share a buffer (the demod history move) as long as the ranges do not overlap.
__global__ void copy_streams_kernel(float* __restrict__ dst, size_t dst_stride, const float* __restrict__ src,
                                    size_t src_stride, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = blockIdx.y;
    if (i < n) dst[(size_t)s * dst_stride + i] = src[(size_t)s * src_stride + i];
}

__global__ void copy_kernel(float* __restrict__ dst, const float* __restrict__ src, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

// src/filter.cpp:106-133 FMDemod, one thread per sample; prev of sample 0 is the carried
// {prev_i, prev_q}.  The carry itself is advanced by demod_prev_kernel afterwards.
__global__ void fm_demod_kernel(float* __restrict__ out, const float* __restrict__ prev,
                                const float* __restrict__ i_ds, const float* __restrict__ q_ds,
                                int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float pi = k > 0 ? i_ds[k - 1] : prev[0];
    const float pq = k > 0 ? q_ds[k - 1] : prev[1];
    out[k] = fm_demod_one(i_ds[k], q_ds[k], pi, pq);
}

__global__ void demod_prev_kernel(float* prev, const float* i_ds, const float* q_ds, int n) {
    if (threadIdx.x == 0 && n > 0) {
        prev[0] = i_ds[n - 1];
        prev[1] = q_ds[n - 1];
    }
}

// src/filter.cpp:176-184
__global__ void mixer_kernel(float* out, const float* a, const float* b, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = 2.0f * (a[i] * b[i]);
}

// src/filter.cpp:186-199
__global__ void lr_kernel(float* l, float* r, const float* m, const float* s, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        l[i] = half_of(m[i] + s[i]);
        r[i] = half_of(m[i] - s[i]);
    }
}

// src/iofunc.cpp:67 + src/project.cpp:56-62
__global__ void normalize_kernel(const uint8_t* iq, size_t n_pairs, float* i_out, float* q_out) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n_pairs) {
        i_out[k] = u8_to_sample(iq[2 * k]);
        q_out[k] = u8_to_sample(iq[2 * k + 1]);
    }
}

// src/project.cpp:185-191
__global__ void quantize_kernel(const float* x, size_t n, int16_t* out) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) out[k] = quantize_s16(x[k]);
}

// new_halo = last hb bytes of (old_halo ++ in), per stream.
__global__ void halo_kernel(const uint8_t* in, size_t sb, const uint8_t* old_halo,
                            uint8_t* new_halo, size_t hb) {
    const int s = blockIdx.y;
    const uint8_t* src = in + (size_t)s * sb;
    const uint8_t* oh = old_halo + (size_t)s * hb;
    uint8_t* nh = new_halo + (size_t)s * hb;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < hb;
         i += (size_t)gridDim.x * blockDim.x) {
        // virtual index into old_halo ++ in: hb + sb - hb + i = sb + i
        const size_t v = sb + i;
        nh[i] = v < hb ? oh[v] : src[v - hb];
    }
}

__global__ void synth_kernel(SynthParams p, const int16_t* __restrict__ tab, uint64_t first,
                             size_t n, uint8_t* __restrict__ out) {
    __shared__ int16_t lt[kSinSize];
    for (int i = threadIdx.x; i < kSinSize; i += blockDim.x) lt[i] = tab[i];
    __syncthreads();
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (size_t)gridDim.x * blockDim.x) {
        uint8_t iq[2];
        synth_pair(p, lt, first + k, iq);
        reinterpret_cast<uint16_t*>(out)[k] = (uint16_t)iq[0] | ((uint16_t)iq[1] << 8);
    }
}

// One launch for a (stream, sample) grid: blockIdx.y = stream, its parameters from d_params
// (the generator is position-addressable, so every workgroup fills its own slice).
__global__ void synth_streams_kernel(const SynthParams* __restrict__ ps, const int16_t* __restrict__ tab,
                                     uint64_t first, size_t n, uint8_t* __restrict__ out, size_t stride) {
    __shared__ int16_t lt[kSinSize];
    for (int i = threadIdx.x; i < kSinSize; i += blockDim.x) lt[i] = tab[i];
    const SynthParams p = ps[blockIdx.y];
    uint16_t* o = reinterpret_cast<uint16_t*>(out + (size_t)blockIdx.y * stride);
    __syncthreads();
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (size_t)gridDim.x * blockDim.x) {
        uint8_t iq[2];
        synth_pair(p, lt, first + k, iq);
        o[k] = (uint16_t)iq[0] | ((uint16_t)iq[1] << 8);
    }
}

inline int ok() { return hipGetLastError() == hipSuccess ? 0 : -2; }

}  // namespace

int launch_resample(float* out, const float* state, const float* in, int n_in,
                    const float* coeff, int taps, int up, int down, int n_out, hipStream_t s) {
    (void)n_in;
    if (n_out <= 0) return 0;
    hipLaunchKernelGGL(resample_kernel, dim3(blocks_for(n_out, 256)), dim3(256), 0, s, out, state,
                       in, coeff, taps, up, down, n_out);
    return ok();
}

int launch_polyphase(const PolyStreams& P, int n_streams, hipStream_t s) {
    if (P.n_out <= 0 || n_streams <= 0) return 0;
    hipLaunchKernelGGL(polyphase_kernel, dim3(blocks_for(P.n_out, 256), n_streams), dim3(256), 0, s, P);
    return ok();
}

int launch_copy_streams(float* dst, size_t dst_stride, const float* src, size_t src_stride, int n, int n_streams,
                        hipStream_t s) {
    if (n <= 0 || n_streams <= 0) return 0;
    hipLaunchKernelGGL(copy_streams_kernel, dim3(blocks_for(n, 256), n_streams), dim3(256), 0, s, dst, dst_stride,
                       src, src_stride, n);
    return ok();
}

int launch_tail_copy(float* dst, const float* src, int n, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(copy_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, dst, src, n);
    return ok();
}

int launch_fm_demod(float* out, float* prev, const float* i, const float* q, int n, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(fm_demod_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, out, prev, i, q,
                       n);
    hipLaunchKernelGGL(demod_prev_kernel, dim3(1), dim3(64), 0, s, prev, i, q, n);
    return ok();
}

int launch_mixer(float* out, const float* a, const float* b, int n, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(mixer_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, out, a, b, n);
    return ok();
}

int launch_lr(float* l, float* r, const float* m, const float* st, int n, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(lr_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, l, r, m, st, n);
    return ok();
}

int launch_normalize(const uint8_t* iq, size_t n_pairs, float* i, float* q, hipStream_t s) {
    if (n_pairs == 0) return 0;
    hipLaunchKernelGGL(normalize_kernel, dim3(blocks_for(n_pairs, 256)), dim3(256), 0, s, iq,
                       n_pairs, i, q);
    return ok();
}

int launch_quantize(const float* x, size_t n, int16_t* out, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(quantize_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, x, n, out);
    return ok();
}

int launch_halo_update(const uint8_t* iq, size_t stream_bytes, const uint8_t* old_halo,
                       uint8_t* new_halo, size_t halo_bytes, int n_streams, hipStream_t s) {
    const int bx = blocks_for(halo_bytes, 256) > 64 ? 64 : blocks_for(halo_bytes, 256);
    hipLaunchKernelGGL(halo_kernel, dim3(bx, n_streams), dim3(256), 0, s, iq, stream_bytes,
                       old_halo, new_halo, halo_bytes);
    return ok();
}

int launch_synth(const SynthParams& p, const int16_t* d_sintab, uint64_t first, size_t n,
                 uint8_t* out, hipStream_t s) {
    if (n == 0) return 0;
    int blocks = blocks_for(n, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(synth_kernel, dim3(blocks), dim3(256), 0, s, p, d_sintab, first, n, out);
    return ok();
}

int launch_synth_streams(const SynthParams* d_params, int n_streams, const int16_t* d_sintab,
                         uint64_t first, size_t n, uint8_t* out, size_t stride, hipStream_t s) {
    if (n == 0 || n_streams <= 0) return 0;
    int bx = blocks_for(n, 256);
    const int cap = std::max(1, 8192 / n_streams);  // ~8k workgroups in all: every CU busy, LDS table loads amortised
    if (bx > cap) bx = cap;
    hipLaunchKernelGGL(synth_streams_kernel, dim3(bx, n_streams), dim3(256), 0, s, d_params, d_sintab, first, n,
                       out, stride);
    return ok();
}

}  // namespace fmrx
