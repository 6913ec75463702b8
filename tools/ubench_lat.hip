// tools/ubench_lat.hip — dependent-chain latency (cycles) of the ops on the PLL's critical
// path, one wave on an otherwise idle GPU, measured with s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN(NAME, T, INIT, ASM)                                                        \
    __global__ void NAME(T* out, long long* cyc, int n) {                                \
        T a = INIT;                                                                      \
        long long t0 = __builtin_amdgcn_s_memtime();                                     \
        for (int i = 0; i < n; i++) {                                                    \
            asm volatile(ASM "\n" ASM "\n" ASM "\n" ASM "\n" ASM "\n" ASM "\n" ASM "\n" ASM \
                         : "+v"(a));                                                      \
        }                                                                                \
        long long t1 = __builtin_amdgcn_s_memtime();                                     \
        out[threadIdx.x] = a;                                                            \
        if (threadIdx.x == 0) *cyc = t1 - t0;                                            \
    }

CHAIN(k_add_f32, float, 1.0f, "v_add_f32 %0, 1.0, %0")
CHAIN(k_mul_f32, float, 1.0f, "v_mul_f32 %0, 1.0, %0")
CHAIN(k_fma_f64, double, 1.0, "v_fma_f64 %0, %0, 1.0, 0.5")
CHAIN(k_add_f64, double, 1.0, "v_add_f64 %0, %0, 0.5")
CHAIN(k_mul_f64, double, 1.0, "v_mul_f64 %0, %0, 1.0")
CHAIN(k_rcp_f64, double, 1.0, "v_rcp_f64 %0, %0")
CHAIN(k_rndne_f64, double, 1.0, "v_rndne_f64 %0, %0")
CHAIN(k_cvt_rt, float, 1.0f, "v_cvt_f64_f32 v[40:41], %0\n v_cvt_f32_f64 %0, v[40:41]")
typedef float f2v __attribute__((ext_vector_type(2)));
CHAIN(k_pk_add, f2v, f2v(1.0f), "v_pk_add_f32 %0, %0, %0")


// issue rate of independent ops from one wave: 4 interleaved chains
#define INDEP(NAME, T, INIT, OP)                                                          \
    __global__ void NAME(T* out, long long* cyc, int n) {                                \
        T a = INIT, b = INIT, c = INIT, d = INIT;                                        \
        long long t0 = __builtin_amdgcn_s_memtime();                                     \
        for (int i = 0; i < n; i++) {                                                    \
            asm volatile(OP(0) "\n" OP(1) "\n" OP(2) "\n" OP(3) "\n" OP(0) "\n" OP(1) "\n" OP(2) "\n" OP(3) \
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));                          \
        }                                                                                \
        long long t1 = __builtin_amdgcn_s_memtime();                                     \
        out[threadIdx.x] = a + b + c + d;                                                \
        if (threadIdx.x == 0) *cyc = t1 - t0;                                            \
    }
#define OPF64(k) "v_fma_f64 %" #k ", %" #k ", 1.0, 0.5"
#define OPF32(k) "v_mul_f32 %" #k ", 1.0, %" #k
#define OPRCP(k) "v_rcp_f64 %" #k ", %" #k
#define OPCVT(k) "v_cvt_f64_f32 v[40:41], %" #k "\n v_cvt_f32_f64 %" #k ", v[40:41]"
INDEP(i_fma_f64, double, 1.0, OPF64)
INDEP(i_mul_f32, float, 1.0f, OPF32)
INDEP(i_rcp_f64, double, 1.0, OPRCP)
INDEP(i_cvt, float, 1.0f, OPCVT)

template <class K, class T>
void run(const char* name, K k, int asm_ops) {
    T* out; long long* cyc;
    hipMalloc(&out, 64 * sizeof(T)); hipMalloc(&cyc, 8);
    const int n = 4096;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 16);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, n);
    long long c = 0; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // s_memtime ticks = shader clock
    printf("%-12s %6.2f cycles per dependent op\n", name, (double)c / (n * 8.0 * asm_ops));
    hipFree(out); hipFree(cyc);
}

int main() {
    run<decltype(k_add_f32), float>("add_f32", k_add_f32, 1);
    run<decltype(k_mul_f32), float>("mul_f32", k_mul_f32, 1);
    run<decltype(k_fma_f64), double>("fma_f64", k_fma_f64, 1);
    run<decltype(k_add_f64), double>("add_f64", k_add_f64, 1);
    run<decltype(k_mul_f64), double>("mul_f64", k_mul_f64, 1);
    run<decltype(k_rcp_f64), double>("rcp_f64", k_rcp_f64, 1);
    run<decltype(k_rndne_f64), double>("rndne_f64", k_rndne_f64, 1);
    run<decltype(k_cvt_rt), float>("cvt f32<->f64 pair", k_cvt_rt, 2);
    run<decltype(k_pk_add), f2v>("pk_add_f32", k_pk_add, 1);
    run<decltype(i_fma_f64), double>("indep4 fma_f64", i_fma_f64, 1);
    run<decltype(i_mul_f32), float>("indep4 mul_f32", i_mul_f32, 1);
    run<decltype(i_rcp_f64), double>("indep4 rcp_f64", i_rcp_f64, 1);
    run<decltype(i_cvt), float>("indep4 cvt pair", i_cvt, 2);
    return 0;
}
