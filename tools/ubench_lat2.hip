// tools/ubench_lat2.hip — more dependent-chain latencies for the PLL runner's step (one wave,
// otherwise idle GPU, s_memtime = shader clock): conversions one way, DPP 64-bit row
// broadcasts, packed f32, and whether a chain runs faster with only 16 or 1 lanes enabled.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN(NAME, T, INIT, ASM, LANES)                                                 \
    __global__ void NAME(T* out, long long* cyc, int n) {                                \
        T a = INIT;                                                                      \
        long long t0 = 0, t1 = 0;                                                        \
        if ((int)threadIdx.x < LANES) {                                                  \
            t0 = __builtin_amdgcn_s_memtime();                                           \
            for (int i = 0; i < n; i++) {                                                \
                asm volatile(ASM "\n" ASM "\n" ASM "\n" ASM "\n" ASM "\n" ASM "\n" ASM "\n" ASM \
                             : "+v"(a));                                                  \
            }                                                                            \
            t1 = __builtin_amdgcn_s_memtime();                                           \
        }                                                                                \
        out[threadIdx.x] = a;                                                            \
        if (threadIdx.x == 0) *cyc = t1 - t0;                                            \
    }

typedef float f2v __attribute__((ext_vector_type(2)));
CHAIN(k_fma_f64_64, double, 1.0, "v_fma_f64 %0, %0, 1.0, 0.5", 64)
CHAIN(k_fma_f64_16, double, 1.0, "v_fma_f64 %0, %0, 1.0, 0.5", 16)
CHAIN(k_fma_f64_1, double, 1.0, "v_fma_f64 %0, %0, 1.0, 0.5", 1)
CHAIN(k_add_f32_16, float, 1.0f, "v_add_f32 %0, 1.0, %0", 16)
CHAIN(k_cvt64_32, float, 1.0f, "v_cvt_f64_f32 v[40:41], %0\n v_mov_b32 %0, v40", 64)
CHAIN(k_mov32, float, 1.0f, "v_mov_b32 v40, %0\n v_mov_b32 %0, v40", 64)
CHAIN(k_dpp64, double, 1.0, "v_mov_b64_dpp %0, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf\n s_nop 1", 64)
CHAIN(k_nop1, double, 1.0, "s_nop 1", 64)
CHAIN(k_pk_mul, f2v, f2v(1.0f), "v_pk_mul_f32 %0, %0, %0", 64)
CHAIN(k_f64_f32_mix, double, 1.0,
      "v_cvt_f32_f64 v40, %0\n v_add_f32 v40, 1.0, v40\n v_cvt_f64_f32 %0, v40", 64)
CHAIN(k_fma_dpp, double, 1.0,
      "v_fma_f64 %0, %0, 1.0, 0.5\n s_nop 1\n v_mov_b64_dpp %0, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf", 64)
CHAIN(k_fma_nop, double, 1.0, "v_fma_f64 %0, %0, 1.0, 0.5\n s_nop 1", 64)

template <class K, class T>
void run(const char* name, K k, int asm_ops) {
    T* out;
    long long* cyc;
    hipMalloc(&out, 64 * sizeof(T));
    hipMalloc(&cyc, 8);
    const int n = 4096;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 16);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, n);
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-22s %6.2f cycles per group\n", name, (double)c / (n * 8.0 * asm_ops));
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run<decltype(k_fma_f64_64), double>("fma_f64 64 lanes", k_fma_f64_64, 1);
    run<decltype(k_fma_f64_16), double>("fma_f64 16 lanes", k_fma_f64_16, 1);
    run<decltype(k_fma_f64_1), double>("fma_f64 1 lane", k_fma_f64_1, 1);
    run<decltype(k_add_f32_16), float>("add_f32 16 lanes", k_add_f32_16, 1);
    run<decltype(k_cvt64_32), float>("cvt_f64_f32+mov", k_cvt64_32, 1);
    run<decltype(k_mov32), float>("mov+mov", k_mov32, 1);
    run<decltype(k_dpp64), double>("dpp64+nop1", k_dpp64, 1);
    run<decltype(k_nop1), double>("s_nop 1", k_nop1, 1);
    run<decltype(k_pk_mul), f2v>("pk_mul_f32", k_pk_mul, 1);
    run<decltype(k_f64_f32_mix), double>("cvt,add32,cvt", k_f64_f32_mix, 1);
    run<decltype(k_fma_dpp), double>("fma,nop1,dpp64", k_fma_dpp, 1);
    run<decltype(k_fma_nop), double>("fma,nop1", k_fma_nop, 1);
    return 0;
}
