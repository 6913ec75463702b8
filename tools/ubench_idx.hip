// tools/ubench_idx.hip — the cost of an "index" PLL chain step (a candidate runner for trigOffset
// below 2^20, where trigArg's float grid is finer than a step's phase move and three or five
// candidates miss; tools/pll_predict.cpp, profiles/r04/pll_predict_below_2_20.txt).  The chain
// forms the step's trigArg exactly as the reference does (float(P + (double)phase),
// filter.cpp:165), turns its bits into a lane index (bits(trigArg) - bits(c0) + 32) and reads the
// step's e from that lane of a VGPR whose 64 lanes hold the e of candidates c0 - 32 .. c0 + 31
// (v_readfirstlane + v_readlane), then (Ki e, Kp e) and the three float updates -- ~10 VALU a
// step for 64 candidates, against 2 (NC - 1) + 4 for the compare-and-select chains.
//   mode 0: step data (P, base, e row) in registers, the same every batch,
//   mode 1: the batch's data read from LDS before its steps (16 x 16-B broadcast + 16 x b32),
//   mode 2: mode 1 + the step's lane index written into lane J of a row (v_writelane), the row
//           stored to LDS after the batch,
//   mode 3: mode 1 + every step's trigArg stored to global memory (all lanes, one address),
//   mode 4: mode 1 + the range test: OR of the lane indices (SALU), tested after the batch,
//   mode 5: mode 4 + mode 2's writelane,
//   mode 6: mode 5 with three waves (the evaluators' SIMDs) busy on f64 FMAs,
//   mode 7: mode 5 with 32-step batches (two bursts of reads).
// Prints shader cycles per step.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_idx tools/ubench_idx.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <utility>

typedef float float2v __attribute__((ext_vector_type(2)));

template <class F, int... J>
__device__ inline void unroll_ic(F&& f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}

constexpr int NBMAX = 32;

template <int MODE>
__global__ void __launch_bounds__(256) chain(float* out, long long* cyc, int nb, int busy) {
    constexpr int NB = MODE == 7 ? 32 : 16;
    __shared__ float4 sp[2][NBMAX];   // (P lo, P hi, base, -) per step
    __shared__ float se[2][NBMAX][64];  // lane c: e of candidate c0 - 32 + c
    __shared__ int srow[2][64];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    const int nw = blockDim.x >> 6;
    // P near 2^18 steps' worth of phase, the candidates around float(P + 0.01)
    for (int e = threadIdx.x; e < 2 * NBMAX; e += blockDim.x) {
        const int k = e % NBMAX;
        const double P = 130000.0 + 0.079 * k;
        const float c0 = (float)(P + 0.01);
        const double2 pd = make_double2(P, 0.0);
        sp[e / NBMAX][k] = make_float4(__builtin_bit_cast(float, (uint32_t)__builtin_bit_cast(uint64_t, P)),
                                       __builtin_bit_cast(float, (uint32_t)(__builtin_bit_cast(uint64_t, P) >> 32)),
                                       __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, c0) - 32u), 0.0f);
        (void)pd;
    }
    for (int e = threadIdx.x; e < 2 * NBMAX * 64; e += blockDim.x)
        (&se[0][0][0])[e] = 1e-4f * ((e & 63) - 32) + 1e-6f * (e >> 6);
    __syncthreads();
    if (w > 0) {
        double acc = t * 1e-9;
        for (int b = 0; b < nb; b++) {
            if (busy)
                for (int i = 0; i < 48; i++) acc = fma(acc, 0.999999, 1e-7);
            __syncthreads();
        }
        out[threadIdx.x] = (float)acc;
        return;
    }
    const float Ki = 1e-4f, Kp = 2.6e-2f;
    float integ = 0.0f, phase = 0.01f;
    float4 R0[NB];
    float E0[NB];
#pragma unroll
    for (int J = 0; J < NB; J++) {
        R0[J] = sp[0][J];
        E0[J] = se[0][J][t];
    }
    float acc = 0.0f;
    uint32_t orr = 0;
    int bad = 0;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    for (int b = 0; b < nb; b++) {
        float4 R[NB];
        float E[NB];
        if constexpr (MODE == 0) {
#pragma unroll
            for (int J = 0; J < NB; J++) {
                R[J] = R0[J];
                E[J] = E0[J];
            }
        } else {
#pragma unroll
            for (int J = 0; J < NB; J++) {
                R[J] = sp[b & 1][J];
                E[J] = se[b & 1][J][t];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        int row = 0;
        unroll_ic(
            [&](auto jc) {
                constexpr int J = decltype(jc)::value;
                const double P = __builtin_bit_cast(double, make_uint2(__builtin_bit_cast(uint32_t, R[J].x),
                                                                       __builtin_bit_cast(uint32_t, R[J].y)));
                const float a = (float)(P + (double)phase);
                const uint32_t i = __builtin_bit_cast(uint32_t, a) - __builtin_bit_cast(uint32_t, R[J].z);
                const uint32_t si = __builtin_amdgcn_readfirstlane(i);
                const float e = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, E[J]), si));
                const float2v k = float2v{Ki, Kp} * e;
                integ = integ + k.x;
                phase = phase + (k.y + integ);
                if constexpr (MODE == 4 || MODE == 5 || MODE == 6 || MODE == 7) orr |= si;
                if constexpr (MODE == 2 || MODE == 5 || MODE == 6 || MODE == 7)
                    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(row) : "s"(si), "i"(J));
                if constexpr (MODE == 3) out[256 + (b & 1) * NB + J] = a;
                acc += (MODE == 0 || MODE == 1) ? a * 0.0f : 0.0f;
            },
            std::make_integer_sequence<int, NB>{});
        if constexpr (MODE == 2 || MODE == 5 || MODE == 6 || MODE == 7) srow[b & 1][t] = row;
        if constexpr (MODE >= 4) bad |= (orr >> 6) != 0;
        phase = phase * 0.5f;
        if (nw > 1) __syncthreads();
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const long long t1 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    out[t] = acc + integ + phase + (float)bad + (float)srow[0][t];
    if (t == 0) cyc[0] = t1 - t0;
    (void)NBMAX;
}

template <int MODE>
static void run(int waves, int busy, float* d_out, long long* d_cyc) {
    const int nb = 4096;
    constexpr int NB = MODE == 7 ? 32 : 16;
    long long best = 1LL << 60;
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(chain<MODE>, dim3(1), dim3(64 * waves), 0, 0, d_out, d_cyc, nb, busy);
        long long c;
        (void)hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
        if (c < best) best = c;
    }
    std::printf("mode %d  waves %d  others %-5s  %7.1f cycles/step\n", MODE, waves, busy ? "busy" : "idle",
                (double)best / ((double)nb * NB));
}

int main() {
    float* d_out;
    long long* d_cyc;
    (void)hipMalloc(&d_out, 1024 * 4);
    (void)hipMalloc(&d_cyc, 8);
    for (int waves : {1, 4}) {
        run<0>(waves, 0, d_out, d_cyc);
        run<1>(waves, 0, d_out, d_cyc);
        run<2>(waves, 0, d_out, d_cyc);
        run<3>(waves, 0, d_out, d_cyc);
        run<4>(waves, 0, d_out, d_cyc);
        run<5>(waves, 0, d_out, d_cyc);
        run<7>(waves, 0, d_out, d_cyc);
    }
    run<6>(4, 1, d_out, d_cyc);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return 0;
}
