// spectrum.hip — SURVEY §8f rank 4: the arctan FM demodulator of the Python models and the
// PSD estimate of the reference's spectrum tooling.  Both are floating-point diagnostics off
// the C++ output path; parity is to a stated tolerance (tests/test_gpu_parity.py), not bits.
//
//   demod_arctan_kernel  fmDemodArctan (model/fmSupportLib.py:34-63): per sample
//                        wrap(atan2(Q,I) - previous phase) into [-pi, pi] with np.unwrap's
//                        rule, in double, one thread per sample (the model's loop carries the
//                        unwrapped phase; a principal value is equivalent mod 2 pi).
//   psd_segment_kernel   estimatePSD (src/fourier.cpp:35-117, fmSupportLib.py:83-157): one
//                        workgroup per segment, float Hann-windowed samples, radix-2 FFT in
//                        double in LDS, 10 log10(4/(Fs N) |X|^2) for the positive bins.
//   psd_mean_kernel      the average over segments in segment order (float, as fourier.cpp).
#include <hip/hip_runtime.h>

#include "fmrx_internal.h"

namespace fmrx {

namespace {

constexpr double kPiD = 3.141592653589793;

__device__ inline double wrap_phase(double dd) {
    if (fabs(dd) < kPiD) return dd;
    // numpy: mod(dd + pi, 2 pi) - pi (floored mod), and +pi for the -pi boundary when dd > 0
    double m = fmod(dd + kPiD, 2.0 * kPiD);
    if (m != 0.0 && m < 0.0) m += 2.0 * kPiD;
    double r = m - kPiD;
    if (r == -kPiD && dd > 0.0) r = kPiD;
    return r;
}

__global__ void demod_arctan_kernel(float* __restrict__ out, const double* __restrict__ prev,
                                    const float* __restrict__ i_in, const float* __restrict__ q_in,
                                    int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double cur = atan2((double)q_in[k], (double)i_in[k]);
    const double pv = k > 0 ? atan2((double)q_in[k - 1], (double)i_in[k - 1]) : prev[0];
    out[k] = (float)wrap_phase(cur - pv);
}

__global__ void demod_arctan_state_kernel(double* prev, const float* i_in, const float* q_in, int n) {
    if (threadIdx.x == 0) prev[0] = atan2((double)q_in[n - 1], (double)i_in[n - 1]);
}

// Dynamic LDS: N complex doubles.  256 threads; N a power of two in [2, kPsdMaxBins].
__global__ void __launch_bounds__(256) psd_segment_kernel(const float* __restrict__ x, int N, int log2n,
                                                          const float* __restrict__ hann, double scale,
                                                          float* __restrict__ seg_db) {
    extern __shared__ double2 buf[];
    const int tid = threadIdx.x;
    const float* base = x + (size_t)blockIdx.x * N;
    for (int i = tid; i < N; i += blockDim.x) {
        const unsigned r = __brev((unsigned)i) >> (32 - log2n);
        const float w = base[i] * hann[i];  // fourier.cpp:90-92, float
        buf[r] = make_double2((double)w, 0.0);
    }
    __syncthreads();
    for (int s = 1; s <= log2n; s++) {
        const int half = 1 << (s - 1);
        for (int j = tid; j < N / 2; j += blockDim.x) {
            const int pos = j & (half - 1);
            const int a = ((j >> (s - 1)) << s) + pos;
            const int b = a + half;
            double sw, cw;
            sincospi(-(double)pos / (double)half, &sw, &cw);  // exp(-2 pi i pos / 2^s)
            const double2 u = buf[a], v = buf[b];
            const double tr = cw * v.x - sw * v.y, ti = cw * v.y + sw * v.x;
            buf[a] = make_double2(u.x + tr, u.y + ti);
            buf[b] = make_double2(u.x - tr, u.y - ti);
        }
        __syncthreads();
    }
    float* out = seg_db + (size_t)blockIdx.x * (N / 2);
    for (int k = tid; k < N / 2; k += blockDim.x) {
        const double2 X = buf[k];
        out[k] = (float)(10.0 * log10(scale * (X.x * X.x + X.y * X.y)));
    }
}

__global__ void psd_mean_kernel(const float* __restrict__ seg_db, int nseg, int half, float* __restrict__ psd) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= half) return;
    float acc = 0.0f;
    for (int l = 0; l < nseg; l++) acc += seg_db[(size_t)l * half + k];
    psd[k] = acc / (float)nseg;
}

}  // namespace

int launch_demod_arctan(float* out, double* prev, const float* i, const float* q, int n, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(demod_arctan_kernel, dim3((n + 255) / 256), dim3(256), 0, s, out, prev, i, q, n);
    hipLaunchKernelGGL(demod_arctan_state_kernel, dim3(1), dim3(64), 0, s, prev, i, q, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_psd(const float* x, int nseg, int N, const float* hann, double scale, float* seg_db, float* psd,
               hipStream_t s) {
    int log2n = 0;
    while ((1 << log2n) < N) log2n++;
    if ((1 << log2n) != N || N < 2 || N > kPsdMaxBins || nseg < 1) return -1;
    const size_t lds = sizeof(double2) * (size_t)N;
    // > 64 KiB of dynamic LDS for the largest transforms (set per call: per current device)
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&psd_segment_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)(sizeof(double2) * kPsdMaxBins)) != hipSuccess)
        return -2;
    hipLaunchKernelGGL(psd_segment_kernel, dim3(nseg), dim3(256), lds, s, x, N, log2n, hann, scale, seg_db);
    hipLaunchKernelGGL(psd_mean_kernel, dim3((N / 2 + 255) / 256), dim3(256), 0, s, seg_db, nseg, N / 2, psd);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace fmrx
