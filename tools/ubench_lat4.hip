// tools/ubench_lat4.hip — one wave: cycles per group of the saturated runner's serial pieces
// (s_memtime ticks; the clock ratio to the 100 MHz s_memrealtime is printed too).
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X X X X X X X X

#define KERNEL(NAME, BODY, ...)                                                      \
    __global__ void NAME(float* out, long long* cyc, int n) {                        \
        float a = threadIdx.x, b = a + 1.0f;                                         \
        double d = a, e = b;                                                         \
        long long t0 = __builtin_amdgcn_s_memtime();                                 \
        long long r0 = __builtin_amdgcn_s_memrealtime();                             \
        for (int i = 0; i < n; i++) asm volatile(R8(BODY) : "+v"(a), "+v"(b), "+v"(d), "+v"(e)::"vcc"); \
        long long t1 = __builtin_amdgcn_s_memtime();                                 \
        long long r1 = __builtin_amdgcn_s_memrealtime();                             \
        out[threadIdx.x] = a + b + (float)d + (float)e;                              \
        if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }                \
    }

KERNEL(k_add32, "v_add_f32 %0, %0, %1\n")
KERNEL(k_add32x3, "v_add_f32 %0, %0, %1\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %0, %1\n")
KERNEL(k_add64, "v_add_f64 %2, %2, %3\n")
KERNEL(k_fma64, "v_fma_f64 %2, %2, %3, %3\n")
KERNEL(k_cvt_pair, "v_cvt_f64_f32 %2, %0\n v_cvt_f32_f64 %0, %2\n")
KERNEL(k_arg, "v_cvt_f64_f32 %2, %0\n v_add_f64 %2, %3, %2\n v_cvt_f32_f64 %0, %2\n")
KERNEL(k_cmp_br, "v_add_f32 %0, %0, %1\n v_cmp_ne_u32 vcc, %0, %1\n s_cbranch_vccnz 0\n")
KERNEL(k_cmp_only, "v_add_f32 %0, %0, %1\n v_cmp_ne_u32 vcc, %0, %1\n")
KERNEL(k_step, "v_add_f32 %0, %0, %1\n v_add_f32 %1, %1, %0\n v_add_f32 %0, %0, %1\n v_cvt_f64_f32 %2, %0\n v_add_f64 %2, %3, %2\n v_cvt_f32_f64 %1, %2\n v_cmp_ne_u32 vcc, %0, %1\n s_cbranch_vccnz 0\n")
KERNEL(k_step_nobr, "v_add_f32 %0, %0, %1\n v_add_f32 %1, %1, %0\n v_add_f32 %0, %0, %1\n v_cvt_f64_f32 %2, %0\n v_add_f64 %2, %3, %2\n v_cvt_f32_f64 %1, %2\n v_cmp_ne_u32 vcc, %0, %1\n")
KERNEL(k_dpp_add, "v_mov_b64_dpp %2, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_add_f64 %3, %3, %2\n")

template <class K>
void run(const char* name, K k, int per_group) {
    float* out;
    long long* cyc;
    hipMalloc(&out, 64 * sizeof(float));
    hipMalloc(&cyc, 16);
    const int n = 4096;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 16);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, n);
    long long c[2] = {0, 0};
    hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
    const double groups = n * 8.0;
    printf("%-44s %7.2f ticks/group (%5.2f per instr), %6.2f ns/group, tick %.2f GHz\n", name, c[0] / groups,
           c[0] / groups / per_group, c[1] * 10.0 / groups, (double)c[0] / (c[1] * 10.0));
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run("add_f32 dependent", k_add32, 1);
    run("3 add_f32 dependent", k_add32x3, 3);
    run("add_f64 dependent", k_add64, 1);
    run("fma_f64 dependent", k_fma64, 1);
    run("cvt f32->f64->f32", k_cvt_pair, 2);
    run("cvt, add_f64, cvt (trigArg)", k_arg, 3);
    run("add, cmp vcc, cbranch_vccnz (not taken)", k_cmp_br, 3);
    run("add, cmp vcc", k_cmp_only, 2);
    run("SAT2 step (3 add, arg, cmp, branch)", k_step, 8);
    run("SAT2 step without the branch", k_step_nobr, 7);
    run("dpp64, dependent add_f64", k_dpp_add, 2);
    return 0;
}
