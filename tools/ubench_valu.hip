// tools/ubench_valu.hip — VALU issue-rate probe on gfx950 for the instruction mixes the
// FIR kernels can use under the no-FMA bit-exactness contract:
//   scalar : v_mul_f32 + v_add_f32
//   packed : v_pk_mul_f32 + v_pk_add_f32  (two lanes-worth of f32 per instruction)
//   mix    : v_fma_mix_f32 (f16 operand, f32 product) + v_add_f32
// Prints lane-ops (f32 results) per second for each.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int KIND>
__global__ void __launch_bounds__(256) probe(float* out, int iters, float c) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
          a6 = a0 + 6, a7 = a0 + 7;
    float b0 = a0 * 0.5f, b1 = a1 * 0.5f, b2 = a2 * 0.5f, b3 = a3 * 0.5f, b4 = a4 * 0.5f,
          b5 = a5 * 0.5f, b6 = a6 * 0.5f, b7 = a7 * 0.5f;
    for (int i = 0; i < iters; i++) {
        if constexpr (KIND == 0) {
            // 16 instructions, 16 f32 results
            asm volatile(
                "v_mul_f32 %0, %8, %0\n v_mul_f32 %1, %8, %1\n v_mul_f32 %2, %8, %2\n v_mul_f32 %3, %8, %3\n"
                "v_mul_f32 %4, %8, %4\n v_mul_f32 %5, %8, %5\n v_mul_f32 %6, %8, %6\n v_mul_f32 %7, %8, %7\n"
                "v_add_f32 %0, %8, %0\n v_add_f32 %1, %8, %1\n v_add_f32 %2, %8, %2\n v_add_f32 %3, %8, %3\n"
                "v_add_f32 %4, %8, %4\n v_add_f32 %5, %8, %5\n v_add_f32 %6, %8, %6\n v_add_f32 %7, %8, %7\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "s"(c));
        } else if constexpr (KIND == 1) {
            // 8 packed instructions on 4 register pairs each mul/add -> 16 f32 results
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
            f2 q0 = {b0, b1}, q1 = {b2, b3}, q2 = {b4, b5}, q3 = {b6, b7};
            asm volatile(
                "v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %5\n v_pk_mul_f32 %2, %2, %6\n v_pk_mul_f32 %3, %3, %7\n"
                "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %5\n v_pk_add_f32 %2, %2, %6\n v_pk_add_f32 %3, %3, %7\n"
                : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)
                : "v"(q0), "v"(q1), "v"(q2), "v"(q3));
            a0 = p0.x; a1 = p0.y; a2 = p1.x; a3 = p1.y; a4 = p2.x; a5 = p2.y; a6 = p3.x; a7 = p3.y;
        } else if constexpr (KIND == 2) {
            // v_fma_mix_f32: f32 = c * f16(lo of b) + 0 ; then v_add_f32
            asm volatile(
                "v_fma_mix_f32 %0, %8, %9, 0 op_sel_hi:[0,1,0]\n v_fma_mix_f32 %1, %8, %9, 0 op_sel_hi:[0,1,0]\n"
                "v_fma_mix_f32 %2, %8, %9, 0 op_sel_hi:[0,1,0]\n v_fma_mix_f32 %3, %8, %9, 0 op_sel_hi:[0,1,0]\n"
                "v_fma_mix_f32 %4, %8, %9, 0 op_sel_hi:[0,1,0]\n v_fma_mix_f32 %5, %8, %9, 0 op_sel_hi:[0,1,0]\n"
                "v_fma_mix_f32 %6, %8, %9, 0 op_sel_hi:[0,1,0]\n v_fma_mix_f32 %7, %8, %9, 0 op_sel_hi:[0,1,0]\n"
                "v_add_f32 %0, %8, %0\n v_add_f32 %1, %8, %1\n v_add_f32 %2, %8, %2\n v_add_f32 %3, %8, %3\n"
                "v_add_f32 %4, %8, %4\n v_add_f32 %5, %8, %5\n v_add_f32 %6, %8, %6\n v_add_f32 %7, %8, %7\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(c), "v"(b0));
        } else if constexpr (KIND == 3) {
            // dependent chain of v_add_f32 (latency probe): 16 adds on one register
            asm volatile(
                "v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n"
                "v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n"
                "v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n"
                "v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0\n"
                : "+v"(a0) : "s"(c));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int KIND>
int run(const char* name, int blocks, double results_per_iter_per_lane) {
    float* out;
    CHECK(hipMalloc(&out, sizeof(float) * blocks * 256));
    const int iters = 20000;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    probe<KIND><<<blocks, 256>>>(out, 100, 1.0f);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    probe<KIND><<<blocks, 256>>>(out, iters, 1.0000001f);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    double lane_ops = (double)blocks * 256 * iters * results_per_iter_per_lane;
    printf("%-28s blocks=%6d  %8.3f ms  %8.2f T f32-results/s\n", name, blocks, ms,
           lane_ops / (ms * 1e-3) / 1e12);
    CHECK(hipFree(out));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
    for (int wpc : {4, 8, 16, 32}) {
        int blocks = p.multiProcessorCount * wpc / 4;
        char n[64];
        snprintf(n, 64, "scalar mul+add (%d w/CU)", wpc); run<0>(n, blocks, 16);
        snprintf(n, 64, "packed mul+add (%d w/CU)", wpc); run<1>(n, blocks, 16);
        snprintf(n, 64, "fma_mix+add    (%d w/CU)", wpc); run<2>(n, blocks, 16);
        snprintf(n, 64, "dep add chain  (%d w/CU)", wpc); run<3>(n, blocks, 16);
    }
    return 0;
}
