// tools/ubench_pk.hip — issue/latency model of packed f32 on gfx950 for FIR-shaped streams.
//   A: dependent v_pk_add_f32 chains, C independent chains per wave (latency probe)
//   B: FIR step pattern: per step C x (pk_mul from registers, pk_add into chain)
// Run with 1, 2, 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef float f2 __attribute__((ext_vector_type(2)));

template <int C, int KIND>
__global__ void __launch_bounds__(256) probe(float* out, int iters) {
    f2 acc[C], x[C];
#pragma unroll
    for (int i = 0; i < C; i++) { acc[i] = f2{(float)threadIdx.x, 1.0f}; x[i] = f2{1e-7f * i, 2e-7f}; }
    f2 c = f2{1.0000001f, 0.9999999f};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int rep = 0; rep < 16; rep++) {
            if constexpr (KIND == 0) {
#pragma unroll
                for (int i = 0; i < C; i++) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(x[i]));
            } else {
#pragma unroll
                for (int i = 0; i < C; i++) {
                    f2 p;
                    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "v"(c), "v"(x[i]));
                    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(p));
                }
            }
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < C; i++) s += acc[i].x + acc[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int C, int KIND>
int run(int wps) {
    float* out;
    int blocks = 256 * wps;  // 256-thread blocks = 4 waves = 1 per SIMD
    CHECK(hipMalloc(&out, sizeof(float) * blocks * 256));
    const int iters = 2000;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    probe<C, KIND><<<blocks, 256>>>(out, 10);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    probe<C, KIND><<<blocks, 256>>>(out, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    double instr_per_wave = (double)iters * 16 * C * (KIND == 0 ? 1 : 2);
    // cycles per wave-instruction per SIMD, assuming 2.1 GHz
    double cyc = ms * 1e-3 * 2.1e9 / (instr_per_wave * wps);
    printf("%s C=%2d waves/SIMD=%d : %.3f ms  %.2f cyc per wave-instr per SIMD\n",
           KIND == 0 ? "dep pk_add chains" : "fir mul+add      ", C, wps, ms, cyc);
    CHECK(hipFree(out));
    return 0;
}

int main() {
    for (int w : {1, 2, 4}) {
        run<1, 0>(w); run<2, 0>(w); run<4, 0>(w); run<8, 0>(w);
        run<2, 1>(w); run<3, 1>(w); run<4, 1>(w); run<6, 1>(w); run<8, 1>(w);
    }
    return 0;
}
