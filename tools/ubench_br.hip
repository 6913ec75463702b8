// tools/ubench_br.hip — one wave: cost of VALU ops issued with EXEC = 0, and of a uniform
// s_cbranch_vccnz per 16 ops, taken or not.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X X X X X X X X
#define R64(X) R8(R8(X))

__global__ void fma_exec0(double* out, long long* cyc, int n) {
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b64 exec, 0\n" R64("v_fma_f64 %0, %0, 1.0, 0.5\n") "s_mov_b64 exec, s[40:41]\n"
                     : "+v"(a) :: "s40", "s41");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void fma_exec1(double* out, long long* cyc, int n) {
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b64 exec, s[40:41]\n" R64("v_fma_f64 %0, %0, 1.0, 0.5\n") "s_mov_b64 exec, s[40:41]\n"
                     : "+v"(a) :: "s40", "s41");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
// 16 fmas, then v_cmp + s_cbranch_vccnz over 0 instructions (falls through either way)
#define BLK_NT "v_fma_f64 %0, %0, 1.0, 0.5\n" R8("v_fma_f64 %0, %0, 1.0, 0.5\n") "v_fma_f64 %0, %0, 1.0, 0.5\n v_fma_f64 %0, %0, 1.0, 0.5\n v_fma_f64 %0, %0, 1.0, 0.5\n v_fma_f64 %0, %0, 1.0, 0.5\n v_fma_f64 %0, %0, 1.0, 0.5\n v_fma_f64 %0, %0, 1.0, 0.5\n v_fma_f64 %0, %0, 1.0, 0.5\n"
__global__ void br_not_taken(double* out, long long* cyc, int n) {
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8(BLK_NT "v_cmp_gt_f64 vcc, 0, %0\n s_nop 1\n s_cbranch_vccnz 1\n s_nop 0\n") : "+v"(a) :: "vcc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void br_taken(double* out, long long* cyc, int n) {
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8(BLK_NT "v_cmp_le_f64 vcc, 0, %0\n s_nop 1\n s_cbranch_vccnz 1\n s_nop 0\n") : "+v"(a) :: "vcc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void no_br(double* out, long long* cyc, int n) {
    double a = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++)
        asm volatile(R8(BLK_NT "v_cmp_le_f64 vcc, 0, %0\n s_nop 1\n s_nop 0\n s_nop 0\n") : "+v"(a) :: "vcc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <class K>
void run(const char* name, K k, double per) {
    double* out;
    long long* cyc;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, 8);
    const int n = 2048;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 16);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, n);
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-34s %8.2f cycles per unit\n", name, (double)c / ((double)n * per));
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run("64 fma with EXEC=0 (per fma)", fma_exec0, 64);
    run("64 fma with EXEC=all (per fma)", fma_exec1, 64);
    run("16 fma + cmp + branch not taken", br_not_taken, 8);
    run("16 fma + cmp + branch taken (+1)", br_taken, 8);
    run("16 fma + cmp + nops, no branch", no_br, 8);
    return 0;
}
