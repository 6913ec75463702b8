// tools/ubench_dpp.hip — one wave: does a 64-bit row-broadcast DPP result cost extra latency
// before a dependent VALU read?  Chains of (DPP, dependent f64 fma) vs (plain move, fma), with
// the 2 wait states a DPP needs after the VALU write of its source as explicit nops in both.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X X X X X X X X

__global__ void dpp_chain(double* out, long long* cyc, int n) {
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8("v_fma_f64 %0, %0, 1.0, 0.5\n s_nop 1\n v_mov_b64_dpp %0, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf\n")
                     : "+v"(a));
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void mov_chain(double* out, long long* cyc, int n) {
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8("v_fma_f64 %0, %0, 1.0, 0.5\n s_nop 1\n v_mov_b64 %0, %0\n") : "+v"(a));
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void dpp_cvt_chain(float* out, long long* cyc, int n) {  // dpp -> cvt -> fma-ish loop
    double a = threadIdx.x;
    float f = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8("v_mov_b64_dpp %0, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf\n v_cvt_f32_f64 %1, %0\n v_cvt_f64_f32 %0, %1\n s_nop 1\n")
                     : "+v"(a), "+v"(f));
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = f;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void mov_cvt_chain(float* out, long long* cyc, int n) {
    double a = threadIdx.x;
    float f = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8("v_mov_b64 %0, %0\n v_cvt_f32_f64 %1, %0\n v_cvt_f64_f32 %0, %1\n s_nop 1\n") : "+v"(a), "+v"(f));
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = f;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <class K, class T>
void run(const char* name, K k) {
    T* out;
    long long* cyc;
    hipMalloc(&out, 64 * sizeof(T));
    hipMalloc(&cyc, 8);
    const int n = 2048;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 16);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, n);
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-36s %7.2f cycles per group\n", name, (double)c / (n * 8.0));
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run<decltype(dpp_chain), double>("fma, nop1, dpp64 (dependent)", dpp_chain);
    run<decltype(mov_chain), double>("fma, nop1, mov64 (dependent)", mov_chain);
    run<decltype(dpp_cvt_chain), float>("dpp64, cvt, cvt, nop1", dpp_cvt_chain);
    run<decltype(mov_cvt_chain), float>("mov64, cvt, cvt, nop1", mov_cvt_chain);
    return 0;
}
