// tools/ubench_lat3.hip — one wave, 64 ops per loop iteration (loop overhead amortised):
// cycles per op of a dependent chain vs independent ops, f64 fma and f32 add, and a dependent
// chain whose ops alternate with one independent op.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X X X X X X X X
#define R64(X) R8(R8(X))
#define R2_(X) X X

__global__ void dep_f64(double* out, long long* cyc, int n) {
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) asm volatile(R64("v_fma_f64 %0, %0, 1.0, 0.5\n") : "+v"(a));
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void ind_f64(double* out, long long* cyc, int n) {
    double a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8(R2_("v_fma_f64 %0, %0, 1.0, 0.5\n v_fma_f64 %1, %1, 1.0, 0.5\n v_fma_f64 %2, %2, 1.0, 0.5\n v_fma_f64 %3, %3, 1.0, 0.5\n"))
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void dep_f32(float* out, long long* cyc, int n) {
    float a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) asm volatile(R64("v_add_f32 %0, 1.0, %0\n") : "+v"(a));
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void dep_cvt(float* out, long long* cyc, int n) {
    float a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8(R2_("v_cvt_f64_f32 v[40:41], %0\n v_cvt_f32_f64 %0, v[40:41]\n v_cvt_f64_f32 v[40:41], %0\n v_cvt_f32_f64 %0, v[40:41]\n")) : "+v"(a) :: "v40", "v41");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void dep_mixed(double* out, long long* cyc, int n) {  // f32 add -> cvt -> f64 fma -> cvt
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8(R2_("v_cvt_f32_f64 v40, %0\n v_add_f32 v40, 1.0, v40\n v_cvt_f64_f32 %0, v40\n v_fma_f64 %0, %0, 1.0, 0.5\n")) : "+v"(a) :: "v40");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <class K, class T>
void run(const char* name, K k, int ops_per_iter) {
    T* out;
    long long* cyc;
    hipMalloc(&out, 64 * sizeof(T));
    hipMalloc(&cyc, 8);
    const int n = 2048;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 16);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, n);
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-28s %6.2f cycles per op\n", name, (double)c / ((double)n * ops_per_iter));
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run<decltype(dep_f64), double>("dependent v_fma_f64", dep_f64, 64);
    run<decltype(ind_f64), double>("4 independent v_fma_f64", ind_f64, 64);
    run<decltype(dep_f32), float>("dependent v_add_f32", dep_f32, 64);
    run<decltype(dep_cvt), float>("dependent cvt f32<->f64", dep_cvt, 64);
    run<decltype(dep_mixed), double>("dependent cvt/add/cvt/fma", dep_mixed, 64);
    return 0;
}
