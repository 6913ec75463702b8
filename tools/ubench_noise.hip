// tools/ubench_noise.hip — what slows the serial PLL chain when other work shares its CU (the
// stage kernels beside the runners in configs[4]).  One workgroup: wave 0 runs the stick form's
// chain (the four-step asm block of pll_pred.hip, its e from LDS in 16-byte bursts, as
// tools/ubench_stick.hip mode 1) for a fixed number of 16-step batches; waves 1 .. K run one kind
// of noise until the chain is done:
//   kind 0: none (the K waves exit at once),
//   kind 1: FP32 VALU (independent v_fma chains in registers),
//   kind 2: LDS reads (ds_read_b128, distinct addresses a lane, conflict-free),
//   kind 3: LDS writes (ds_write_b128),
//   kind 4: global loads streaming from HBM (global_load_dwordx4, 64 MiB),
//   kind 5: f64 VALU (v_fma_f64 chains: what the evaluators run).
// The LDS kinds again with the chain wave at s_setprio 3.
// K = 3: one noise wave on each other SIMD; K = 7: two a SIMD, one beside the chain.  Prints the
// chain's shader cycles (s_memtime) a step.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench_noise tools/ubench_noise.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int NB = 16;
typedef float f4 __attribute__((ext_vector_type(4)));

#define ST_TAIL(P, Q)                                            \
    "v_pk_mul_f32 v[254:255], v[252:253], %[kk] op_sel_hi:[0,1]\n" \
    "v_add_f32 %[ig], %[ig], v254\n"                             \
    "v_add_f32 v255, v255, %[ig]\n"                              \
    "v_add_f32 " Q ", " P ", v255\n"
#define ST_STEP(P, Q, K)                                      \
    "v_cmp_ge_f32_e64 %[m0], " P ", %[ta]\n"                    \
    "v_cmp_ge_f32_e64 %[m1], " P ", %[tb]\n"                    \
    "s_nop 0\n"                                               \
    "v_cndmask_b32_e64 v252, %[ea" #K "], %[eb" #K "], %[m0]\n" \
    "v_cndmask_b32_e64 v252, v252, %[ec" #K "], %[m1]\n" ST_TAIL(P, Q)

__device__ inline void chain4(float& phase, float& integ, uint64_t kk, float ta, float tb, const float* e) {
    float p1, p2, p3, p4;
    uint64_t m0, m1;
    asm volatile(ST_STEP("%[p]", "%[q1]", 0) ST_STEP("%[q1]", "%[q2]", 1) ST_STEP("%[q2]", "%[q3]", 2)
                     ST_STEP("%[q3]", "%[q4]", 3)
                 : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ),
                   [m0] "=&s"(m0), [m1] "=&s"(m1)
                 : [p] "v"(phase), [kk] "s"(kk), [ta] "v"(ta), [tb] "v"(tb), [ea0] "v"(e[0]), [eb0] "v"(e[1]),
                   [ec0] "v"(e[2]), [ea1] "v"(e[3]), [eb1] "v"(e[4]), [ec1] "v"(e[5]), [ea2] "v"(e[6]),
                   [eb2] "v"(e[7]), [ec2] "v"(e[8]), [ea3] "v"(e[9]), [eb3] "v"(e[10]), [ec3] "v"(e[11])
                 : "v252", "v253", "v254", "v255");
    phase = p4;
}

template <int KIND, bool PRIO = false>
__global__ void __launch_bounds__(512) noise(const float* __restrict__ g, const float4* __restrict__ big, size_t nbig,
                                             float* out, long long* cyc, int nb) {
    __shared__ __attribute__((aligned(16))) float se[4][3 * NB];
    __shared__ __attribute__((aligned(16))) float4 sn[8][1024];  // the noise waves' LDS traffic
    __shared__ int done;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    for (int q = threadIdx.x; q < 4 * 3 * NB; q += blockDim.x) se[q / (3 * NB)][q % (3 * NB)] = g[q];
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    if (w > 0) {
        if (KIND == 0) return;
        float a0 = t * 1e-3f, a1 = a0 + 1.0f, a2 = a0 + 2.0f, a3 = a0 + 3.0f;
        double d0 = a0, d1 = a1;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        size_t gi = ((size_t)w * 64 + t) % nbig;
        int it = 0;
        while (__builtin_amdgcn_readfirstlane(__atomic_load_n(&done, __ATOMIC_RELAXED)) == 0) {
            for (int r = 0; r < 64; r++) {
                if constexpr (KIND == 1) {
                    a0 = fmaf(a0, 0.9999f, 1e-4f);
                    a1 = fmaf(a1, 0.9999f, 1e-4f);
                    a2 = fmaf(a2, 0.9999f, 1e-4f);
                    a3 = fmaf(a3, 0.9999f, 1e-4f);
                } else if constexpr (KIND == 2) {
                    f4 v;
                    const uint32_t ad = (uint32_t)(uintptr_t)&sn[w][(t + 64 * ((r + it) & 15)) & 1023];
                    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ad) : "memory");
                    acc.x += v.x;
                } else if constexpr (KIND == 3) {
                    const f4 v = {a0, a1, a2, (float)r};
                    const uint32_t ad = (uint32_t)(uintptr_t)&sn[w][(t + 64 * ((r + it) & 15)) & 1023];
                    asm volatile("ds_write_b128 %0, %1" : : "v"(ad), "v"(v) : "memory");
                } else if constexpr (KIND == 4) {
                    const float4 v = big[gi];
                    gi = (gi + 64 * 8) % nbig;
                    acc.x += v.x;
                } else {
                    d0 = fma(d0, 0.9999, 1e-4);
                    d1 = fma(d1, 0.9999, 1e-4);
                }
            }
            it++;
        }
        out[256 + threadIdx.x] = a0 + a1 + a2 + a3 + acc.x + (float)(d0 + d1) + (float)it;
        return;
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
    const float Ki = 1e-4f, Kp = 2.6e-2f;
    const uint64_t kk = (uint64_t)__builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, Ki)) |
                        ((uint64_t)__builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, Kp)) << 32);
    const float ta = 0.0f, tb = 0.5f;
    float integ = 0.0f, phase = 0.01f;
    float e[3 * NB];
    __builtin_amdgcn_s_waitcnt(0);
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < nb; b++) {
#pragma unroll
        for (int q = 0; q < 3 * NB / 4; q++)
            *reinterpret_cast<float4*>(&e[4 * q]) = reinterpret_cast<const float4*>(&se[b & 3][0])[q];
#pragma unroll
        for (int q = 0; q < NB / 4; q++) chain4(phase, integ, kk, ta, tb, &e[12 * q]);
    }
    __builtin_amdgcn_s_waitcnt(0);
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (t == 0) {
        cyc[0] = t1 - t0;
        __atomic_store_n(&done, 1, __ATOMIC_RELAXED);
    }
    out[t] = phase + integ;
}

template <int KIND, bool PRIO = false>
static void run(const float* g, const float4* big, size_t nbig, float* out, long long* cyc, int nb, int k) {
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL((noise<KIND, PRIO>), dim3(1), dim3(64 * (1 + k)), 0, 0, g, big, nbig, out, cyc, nb);
        (void)hipDeviceSynchronize();
    }
    long long c = 0;
    (void)hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    std::printf("kind %d  noise waves %d  chain%s %.1f cycles/step\n", KIND, k, PRIO ? " at s_setprio 3" : "",
                (double)c / ((double)nb * NB));
}

int main() {
    const int nb = 20000;
    float h[4 * 3 * NB];
    for (int i = 0; i < 4 * 3 * NB; i++) h[i] = 0.1f + 1e-3f * (float)(i % 17);
    float *g, *out;
    float4* big;
    long long* cyc;
    const size_t nbig = (64u << 20) / sizeof(float4);
    (void)hipMalloc(&g, sizeof h);
    (void)hipMalloc(&big, nbig * sizeof(float4));
    (void)hipMemset(big, 0, nbig * sizeof(float4));
    (void)hipMalloc(&out, 1024 * sizeof(float));
    (void)hipMalloc(&cyc, sizeof(long long));
    (void)hipMemcpy(g, h, sizeof h, hipMemcpyHostToDevice);
    for (int k : {3, 7}) {
        run<0>(g, big, nbig, out, cyc, nb, k);
        run<1>(g, big, nbig, out, cyc, nb, k);
        run<2>(g, big, nbig, out, cyc, nb, k);
        run<3>(g, big, nbig, out, cyc, nb, k);
        run<4>(g, big, nbig, out, cyc, nb, k);
        run<5>(g, big, nbig, out, cyc, nb, k);
        run<2, true>(g, big, nbig, out, cyc, nb, k);
        run<3, true>(g, big, nbig, out, cyc, nb, k);
    }
    return 0;
}
