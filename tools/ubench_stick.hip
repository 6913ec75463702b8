// tools/ubench_stick.hip — where the stick form's chain (pll_pred.hip pll_pipe_kernel<..., STK>)
// gets its three e a step from, and what that costs the one wave that runs the chain.  Wave 0
// runs batches of 16 steps of the three-candidate four-step asm block (chain4_3, the two
// thresholds constant) with the 48 floats of a batch's e from:
//   mode 0: registers (the same every batch: the floor with no reads),
//   mode 1: LDS, 12 ds_read_b128 of one address for all lanes at the batch start (the kernel's
//           burst; the compiler waits for each read at its first use),
//   mode 2: LDS as mode 1 but one batch ahead (the next batch's 12 reads issued before this
//           batch's steps; all waited for after them),
//   mode 3: global memory, 12 global_load_dwordx4 of one address for all lanes, one batch ahead,
//   mode 4: mode 3 with the loads bypassing the vector L1 (sc0 sc1: what data another wave just
//           wrote would need),
//   mode 5: global memory, 3 s_load_dwordx16 a batch one batch ahead into SGPRs and 48 v_mov_b32
//           to VGPRs (the e a v_cndmask reads must be VGPRs),
//   mode 6: the pipe form's two thresholds a step (not the stick's constants) as SGPR operands of
//           the compares, from a uniform read-only address (s_load) one batch ahead, the e from
//           LDS as mode 1,
//   mode 8: mode 6 with the thresholds loaded at the batch start,
//   mode 7: the pipe form as the kernel has it: (T0, T1, e(c0 - 1), e(c0)) and e(c0 + 1) from LDS,
//           20 ds_read_b128 a batch,
// the other waves of the workgroup (0 or 2) idle at one barrier a batch.  Prints shader cycles
// (s_memtime) a step.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench_stick tools/ubench_stick.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int NB = 16;

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

#define ST_STEPT(P, Q, K)                                     \
    "v_cmp_ge_f32_e64 %[m0], " P ", %[ta" #K "]\n"               \
    "v_cmp_ge_f32_e64 %[m1], " P ", %[tb" #K "]\n"               \
    "s_nop 0\n"                                               \
    "v_cndmask_b32_e64 v252, %[ea" #K "], %[eb" #K "], %[m0]\n" \
    "v_cndmask_b32_e64 v252, v252, %[ec" #K "], %[m1]\n" ST_TAIL(P, Q)
#define ST_OPS_E                                                                                      \
    [ea0] "v"(e[0]), [eb0] "v"(e[1]), [ec0] "v"(e[2]), [ea1] "v"(e[3]), [eb1] "v"(e[4]), [ec1] "v"(e[5]), \
        [ea2] "v"(e[6]), [eb2] "v"(e[7]), [ec2] "v"(e[8]), [ea3] "v"(e[9]), [eb3] "v"(e[10]), [ec3] "v"(e[11])
// per-step thresholds T[2k], T[2k + 1] of step k: SGPR operands (SG) or VGPRs
template <bool SG>
__device__ inline void chain4t(float& phase, float& integ, uint64_t kk, const float* T, const float* e) {
    float p1, p2, p3, p4;
    uint64_t m0, m1;
    if constexpr (SG)
        asm volatile(ST_STEPT("%[p]", "%[q1]", 0) ST_STEPT("%[q1]", "%[q2]", 1) ST_STEPT("%[q2]", "%[q3]", 2)
                         ST_STEPT("%[q3]", "%[q4]", 3)
                     : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ),
                       [m0] "=&s"(m0), [m1] "=&s"(m1)
                     : [p] "v"(phase), [kk] "s"(kk), [ta0] "s"(T[0]), [tb0] "s"(T[1]), [ta1] "s"(T[2]),
                       [tb1] "s"(T[3]), [ta2] "s"(T[4]), [tb2] "s"(T[5]), [ta3] "s"(T[6]), [tb3] "s"(T[7]), ST_OPS_E
                     : "v252", "v253", "v254", "v255");
    else
        asm volatile(ST_STEPT("%[p]", "%[q1]", 0) ST_STEPT("%[q1]", "%[q2]", 1) ST_STEPT("%[q2]", "%[q3]", 2)
                         ST_STEPT("%[q3]", "%[q4]", 3)
                     : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ),
                       [m0] "=&s"(m0), [m1] "=&s"(m1)
                     : [p] "v"(phase), [kk] "s"(kk), [ta0] "v"(T[0]), [tb0] "v"(T[1]), [ta1] "v"(T[2]),
                       [tb1] "v"(T[3]), [ta2] "v"(T[4]), [tb2] "v"(T[5]), [ta3] "v"(T[6]), [tb3] "v"(T[7]), ST_OPS_E
                     : "v252", "v253", "v254", "v255");
    phase = p4;
}

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

template <int MODE>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(1, 1)))
stick(const float* __restrict__ g, float* __restrict__ out, long long* __restrict__ cyc, int nb) {
    __shared__ __attribute__((aligned(16))) float se[4][3 * NB];
    __shared__ __attribute__((aligned(16))) float st[4][4 * NB];
    __shared__ __attribute__((aligned(16))) float sp[4][NB];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    for (int q = threadIdx.x; q < 4 * 3 * NB; q += blockDim.x) se[q / (3 * NB)][q % (3 * NB)] = g[q];
    for (int q = threadIdx.x; q < 4 * 4 * NB; q += blockDim.x) st[q / (4 * NB)][q % (4 * NB)] = g[q % (4 * 3 * NB)];
    for (int q = threadIdx.x; q < 4 * NB; q += blockDim.x) sp[q / NB][q % NB] = g[q];
    __syncthreads();
    if (w > 0) {
        for (int b = 0; b < nb; b++) __syncthreads();
        return;
    }
    const float Ki = 1e-4f, Kp = 2.6e-2f;
    const uint64_t kk = (uint64_t)__builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, Ki)) |
                        ((uint64_t)__builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, Kp)) << 32);
    const float ta = 0.0f, tb = 0.5f;
    float integ = 0.0f, phase = 0.01f;
    float e[3 * NB], en[3 * NB];
#pragma unroll
    for (int i = 0; i < 3 * NB; i++) e[i] = en[i] = g[i] * (1.0f + 1e-7f * t);
    auto load_lds = [&](int slot, float (&d)[3 * NB]) {
#pragma unroll
        for (int q = 0; q < 3 * NB / 4; q++)
            *reinterpret_cast<float4*>(&d[4 * q]) = reinterpret_cast<const float4*>(&se[slot][0])[q];
    };
    auto load_glb = [&](int slot, float (&d)[3 * NB]) {
        const float4* p = reinterpret_cast<const float4*>(g + 3 * NB * slot);
#pragma unroll
        for (int q = 0; q < 3 * NB / 4; q++) {
            if constexpr (MODE == 4) {
                float4 v;
                asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p + q));
                *reinterpret_cast<float4*>(&d[4 * q]) = v;
            } else if constexpr (MODE == 3) {
                float4 v;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p + q));
                *reinterpret_cast<float4*>(&d[4 * q]) = v;
            } else {
                *reinterpret_cast<float4*>(&d[4 * q]) = p[q];
            }
        }
    };
    float Tn[2 * NB];
#pragma unroll
    for (int i = 0; i < 2 * NB; i++) Tn[i] = g[4 * 3 * NB + i];
    __builtin_amdgcn_s_waitcnt(0);
    const long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0);
    for (int b = 0; b < nb; b++) {
        if constexpr (MODE == 1) {
            load_lds(b & 3, e);
        } else if constexpr (MODE == 2) {
            load_lds((b + 1) & 3, en);
        } else if constexpr (MODE >= 3 && MODE <= 5) {
            load_glb((b + 1) & 3, en);  // mode 5: plain C on a uniform read-only address (s_load)
        }
        if constexpr (MODE >= 6) {
            // the pipe form's step data: two thresholds a step beside the three e
            float T[2 * NB];
            if constexpr (MODE == 6 || MODE == 8) {  // thresholds by s_load, e from LDS
                // mode 6: this batch's thresholds were loaded during the last one (Tn)
                const float* __restrict__ pt = g + 4 * 3 * NB + 2 * NB * ((b + (MODE == 6 ? 1 : 0)) & 3);
#pragma unroll
                for (int i = 0; i < 2 * NB; i++) {
                    if constexpr (MODE == 6) {
                        T[i] = Tn[i];
                        Tn[i] = pt[i];
                    } else {
                        T[i] = pt[i];
                    }
                }
                load_lds(b & 3, e);
            } else {  // the kernel's layout: (T0, T1, ea, eb) and ec, 20 16-byte reads a batch
#pragma unroll
                for (int J = 0; J < NB; J++) {
                    const float4 r = reinterpret_cast<const float4*>(&st[b & 3][0])[J];
                    T[2 * J] = r.x;
                    T[2 * J + 1] = r.y;
                    e[3 * J] = r.z;
                    e[3 * J + 1] = r.w;
                }
#pragma unroll
                for (int q = 0; q < NB / 4; q++) {
                    const float4 r = reinterpret_cast<const float4*>(&sp[b & 3][0])[q];
                    e[3 * (4 * q) + 2] = r.x;
                    e[3 * (4 * q + 1) + 2] = r.y;
                    e[3 * (4 * q + 2) + 2] = r.z;
                    e[3 * (4 * q + 3) + 2] = r.w;
                }
            }
#pragma unroll
            for (int q = 0; q < NB / 4; q++) chain4t<MODE != 7>(phase, integ, kk, &T[8 * q], &e[12 * q]);
        } else {
#pragma unroll
            for (int q = 0; q < NB / 4; q++) chain4(phase, integ, kk, ta, tb, &e[12 * q]);
        }
        if constexpr (MODE >= 2 && MODE <= 5) {
#pragma unroll
            for (int i = 0; i < 3 * NB; i++) e[i] = en[i];
        }
        __syncthreads();
    }
    __builtin_amdgcn_s_waitcnt(0);
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (t == 0) cyc[0] = t1 - t0;
    out[t] = phase + integ;
}

template <int MODE>
static void run(const float* g, float* out, long long* cyc, int nb, int waves) {
    hipLaunchKernelGGL(stick<MODE>, dim3(1), dim3(64 * waves), 0, 0, g, out, cyc, nb);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(stick<MODE>, dim3(1), dim3(64 * waves), 0, 0, g, out, cyc, nb);
    (void)hipDeviceSynchronize();
    long long c = 0;
    (void)hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    std::printf("mode %d  waves %d  %.1f cycles/step\n", MODE, waves, (double)c / ((double)nb * NB));
}

int main() {
    const int nb = 20000;
    float h[4 * 3 * NB + 4 * 2 * NB];
    for (int i = 0; i < 4 * 3 * NB + 4 * 2 * NB; i++) h[i] = 0.1f + 1e-3f * (float)(i % 17);
    float *g, *out;
    long long* cyc;
    (void)hipMalloc(&g, sizeof h);
    (void)hipMalloc(&out, 256 * sizeof(float));
    (void)hipMalloc(&cyc, sizeof(long long));
    (void)hipMemcpy(g, h, sizeof h, hipMemcpyHostToDevice);
    for (int waves : {1, 3}) {
        run<0>(g, out, cyc, nb, waves);
        run<1>(g, out, cyc, nb, waves);
        run<2>(g, out, cyc, nb, waves);
        run<3>(g, out, cyc, nb, waves);
        run<4>(g, out, cyc, nb, waves);
        run<5>(g, out, cyc, nb, waves);
        run<6>(g, out, cyc, nb, waves);
        run<7>(g, out, cyc, nb, waves);
        run<8>(g, out, cyc, nb, waves);
    }
    return 0;
}
