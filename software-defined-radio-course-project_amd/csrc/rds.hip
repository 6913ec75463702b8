// rds.hip — RDS front half: the rds_thread body of src/project.cpp:200-271,
// which the reference defines but never launches (:380-382).  Per stream and IF sample n:
//
//   channel[n] = sum_k ex[k] demod[n-k]          BPF 54-60 kHz        (:211, :247)
//   sq[n]      = channel[n] * channel[n]                               (:250-254)
//   carrier[n] = sum_k ca[k] sq[n-k]              BPF 113.5-114.5 kHz (:217, :257)
//   nco        = PLL(carrier, 114 kHz, bp_fs, ncoScale 0.5, 0, 0.01)   (:259)
//   rds[n]     = 2 * (nco[n] * channel[n-5])      delay 5 + mixer     (:262-271)
//
// Every FIR output is the reference's sequential ascending-tap sum with separately rounded
// products (filter.cpp:84-92).  All stages are block-size invariant, so one call may cover
// any number of blocks.  rds_front_kernel fuses both FIRs and the square: a workgroup stages
// its demod tile plus 100 samples of history in LDS, computes the channel for the tile and
// the 50 samples before it (the second FIR's history, recomputed rather than carried: the
// same inputs give the same floats), squares it in LDS, and runs the carrier FIR.  The PLL is
// the stereo engine's (one lane per stream, certified fast trig); rds_mix_kernel applies the
// 5-sample delay and the mixer.
#include <hip/hip_runtime.h>

#include "fmrx_internal.h"

namespace fmrx {

namespace {

constexpr int kT = kRdsTaps;
constexpr int kH = kT - 1;
constexpr int kTile = 256;

__global__ void __launch_bounds__(kTile) rds_front_kernel(RdsLaunch L) {
    __shared__ float xs[kTile + 2 * kH];  // demod [n0 - 100, n0 + kTile)
    __shared__ float sq[kTile + kH];      // channel^2 [n0 - 50, n0 + kTile)
    __shared__ float ex[kT], ca[kT];
    const int tid = threadIdx.x;
    const int s = blockIdx.y;
    const int n0 = blockIdx.x * kTile;
    const float* d = L.demod + (size_t)s * L.demod_stride;
    const float* h = L.dhist + (size_t)s * kRdsDemodHist;  // the 100 samples before d[0]
    float* chan = L.chan + (size_t)s * L.chan_stride + kRdsChanHist;
    float* car = L.carrier + (size_t)s * L.car_stride;
    for (int i = tid; i < kT; i += kTile) {
        ex[i] = L.ex[i];
        ca[i] = L.ca[i];
    }
    for (int i = tid; i < kTile + 2 * kH; i += kTile) {
        const int m = n0 - 2 * kH + i;
        xs[i] = m < 0 ? h[kRdsDemodHist + m] : (m < L.n_if ? d[m] : 0.0f);
    }
    __syncthreads();
    for (int i = tid; i < kTile + kH; i += kTile) {
        const int m = n0 - kH + i;  // channel sample; xs index of demod[m - k] is i + kH - k
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < kT; k++) {
            const float p = ex[k] * xs[i + kH - k];
            acc = acc + p;
        }
        sq[i] = acc * acc;
        if (i >= kH && m < L.n_if) chan[m] = acc;
    }
    __syncthreads();
    const int n = n0 + tid;
    if (n < L.n_if) {
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < kT; k++) {
            const float p = ca[k] * sq[tid + kH - k];
            acc = acc + p;
        }
        car[n] = acc;
    }
}

// rds[n] = 2 * (nco[n] * channel[n - 5]); channel[-5..-1] is the previous call's tail.
__global__ void rds_mix_kernel(RdsLaunch L) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = blockIdx.y;
    if (n >= L.n_if) return;
    const float* chan = L.chan + (size_t)s * L.chan_stride + kRdsChanHist;
    const float nco = L.carrier[(size_t)s * L.car_stride + n];
    const float v = nco * chan[n - kRdsDelay];
    L.out[(size_t)s * L.out_stride + n] = 2.0f * v;
}

// Carry for the next call: the last 100 demod samples and the last kRdsChanHist channel
// samples (the delay needs 5) move in front.  One workgroup per stream.
__global__ void rds_state_kernel(RdsLaunch L) {
    const int s = blockIdx.x;
    const int t = threadIdx.x;
    const float* d = L.demod + (size_t)s * L.demod_stride;
    float* h = L.dhist + (size_t)s * kRdsDemodHist;
    float* chan = L.chan + (size_t)s * L.chan_stride;
    // n_if >= 100 is guaranteed by the caller (whole blocks of >= 640 samples)
    float dv = 0.0f, cv = 0.0f;
    if (t < kRdsDemodHist) dv = d[L.n_if - kRdsDemodHist + t];
    if (t < kRdsChanHist) cv = chan[L.n_if + t];  // = channel[n_if - kRdsChanHist + t]
    __syncthreads();
    if (t < kRdsDemodHist) h[t] = dv;
    if (t < kRdsChanHist) chan[t] = cv;
}

}  // namespace

int launch_rds(const RdsLaunch& L, int n_streams, hipStream_t s) {
    if (L.n_if <= 0) return 0;
    if (L.n_if < kRdsDemodHist) return -1;
    hipLaunchKernelGGL(rds_front_kernel, dim3((L.n_if + kTile - 1) / kTile, n_streams), dim3(kTile), 0, s, L);
    // project.cpp:259: PLL(carrier_data, 114000, bp_fs, 0.5, 0, 0.01, ...), in place -> NCO
    if (launch_pll(L.carrier, L.n_if, n_streams, L.car_stride, 114000.0f, L.bp_fs, 0.5f, 0.0f, 0.01f,
                   L.pll, L.pll_side, s, L.hint))
        return -2;
    hipLaunchKernelGGL(rds_mix_kernel, dim3((L.n_if + 255) / 256, n_streams), dim3(256), 0, s, L);
    hipLaunchKernelGGL(rds_state_kernel, dim3(n_streams), dim3(128), 0, s, L);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace fmrx
