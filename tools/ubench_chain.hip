// tools/ubench_chain.hip — what does the three-wave PLL runner's chain step cost (pll_pred.hip
// pll_pipe_kernel)?  One workgroup; wave 0 runs batches of 16 chain steps (two sign masks, two
// bitfield inserts, (Ki e, Kp e), three float updates) with the candidate data
//   mode 0: in registers (the same every batch),
//   mode 1: read from LDS at the batch start (20 x 16-B broadcast reads, then wait),
//   mode 2: read from LDS one 16-B read a step, for the next batch,
//   mode 3: mode 2 with only lanes 0-15 active in the chain,
//   mode 4: mode 1 with only lane 0 reading (EXEC = 1 around the reads, in asm; the other lanes
//           run the chain on stale data),
//   mode 5: mode 4 with all lanes reading (the asm control),
//   mode 6: mode 0 with the choice (subs, shifts, inserts) in one asm block (no wait states),
//   mode 7: mode 1 with mode 6's asm block (pll_pipe_kernel's chain),
//   mode 8: mode 7 with only lane 0 reading (an exec-masked branch around the reads),
//   mode 9: mode 6 with the choice by two compares to SGPR masks and two v_cndmask,
//   mode 10: mode 6 with the whole step in one asm block (choice, v_pk_mul, the three adds),
//   mode 11: mode 10 with mode 9's choice,
//   mode 12: mode 9 + the phases stored to LDS after the batch from lane 0 (exec-masked branch),
//   mode 13: mode 9 + each group of 4 phases stored as soon as made, every lane to one address,
//   mode 14: mode 9 + each group of 4 phases stored as soon as made, lane 0 only (exec in asm),
// and the other waves (0, 1 or 2 of them) either idle at the barrier or busy with f64 FMAs
// (`busy`); one barrier per batch when there are other waves.  Prints shader cycles per step.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_chain tools/ubench_chain.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <utility>

typedef float float2v __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// 4 x 16-B LDS reads at addr, +16, +32, +48 with EXEC = lane 0 only (ONE) or all lanes, waited for
template <bool ONE>
__device__ inline void rd4(unsigned addr, f4& a, f4& b, f4& c, f4& d) {
    if constexpr (ONE)
        asm volatile(
            "s_mov_b64 s[40:41], exec\n s_mov_b64 exec, 1\n"
            " ds_read_b128 %0, %4\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n"
            " ds_read_b128 %3, %4 offset:48\n s_waitcnt lgkmcnt(0)\n s_mov_b64 exec, s[40:41]"
            : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
            : "v"(addr)
            : "s40", "s41", "memory");
    else
        asm volatile(
            " ds_read_b128 %0, %4\n ds_read_b128 %1, %4 offset:16\n ds_read_b128 %2, %4 offset:32\n"
            " ds_read_b128 %3, %4 offset:48\n s_waitcnt lgkmcnt(0)"
            : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
            : "v"(addr)
            : "memory");
}

__device__ inline uint32_t sign_mask(float x) {
    uint32_t m;
    asm("v_ashrrev_i32 %0, 31, %1" : "=v"(m) : "v"(x));
    return m;
}
__device__ inline float bfi(uint32_t m, float a, float b) {
    float d;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(d) : "v"(m), "v"(a), "v"(b));
    return d;
}
template <class F, int... J>
__device__ inline void unroll_ic(F&& f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}

constexpr int NB = 16;

template <int MODE>
__global__ void __launch_bounds__(192) chain(float* out, long long* cyc, int nb, int busy) {
    __shared__ float4 sel[2][NB];
    __shared__ float sep[2][NB];
    __shared__ float4 sph[2][NB / 4];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    const int nw = blockDim.x >> 6;
    if (threadIdx.x < 2 * NB) {
        const int k = threadIdx.x & (NB - 1);
        // thresholds around the phase's range, distinct e's: the choice varies step to step
        sel[threadIdx.x / NB][k] = make_float4(-0.3f + 0.01f * k, 0.2f - 0.01f * k, 1e-3f * (k + 1), -2e-3f * (k + 1));
        sep[threadIdx.x / NB][k] = 5e-4f * (k - 7);
    }
    __syncthreads();
    if (w > 0) {
        double acc = t * 1e-9;
        for (int b = 0; b < nb; b++) {
            if (busy)
                for (int i = 0; i < 64; i++) acc = fma(acc, 0.999999, 1e-7);
            __syncthreads();
        }
        out[threadIdx.x] = (float)acc;
        return;
    }
    const float Ki = 1e-4f, Kp = 2.6e-2f;
    float integ = 1e-5f * t, phase = 0.01f;
    float4 A0[NB], A1[NB];
    float E0[NB], E1[NB];
#pragma unroll
    for (int J = 0; J < NB; J++) {
        A0[J] = sel[0][J];
        E0[J] = sep[0][J];
    }
    float acc = 0.0f;
    auto run = [&](int b, float4(&A)[NB], float(&EP)[NB], float4(&NA)[NB], float(&NEP)[NB]) {
        if constexpr (MODE == 4 || MODE == 5) {
            const unsigned as = (unsigned)(uintptr_t)&sel[b & 1][0], ae = (unsigned)(uintptr_t)&sep[b & 1][0];
            f4 v[20];
#pragma unroll
            for (int q = 0; q < 4; q++) rd4<MODE == 4>(as + 64 * q, v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
            rd4<MODE == 4>(ae, v[16], v[17], v[18], v[19]);
#pragma unroll
            for (int J = 0; J < NB; J++) A[J] = make_float4(v[J].x, v[J].y, v[J].z, v[J].w);
#pragma unroll
            for (int J = 0; J < NB; J++) EP[J] = v[16 + J / 4][J % 4];
        }
        if constexpr (MODE == 8) {
            if (t == 0) {
#pragma unroll
                for (int J = 0; J < NB; J++) A[J] = sel[b & 1][J];
#pragma unroll
                for (int J = 0; J < NB / 4; J++)
                    *reinterpret_cast<float4*>(&EP[4 * J]) = reinterpret_cast<const float4*>(sep[b & 1])[J];
            }
        }
        if constexpr (MODE == 1 || MODE == 7) {
#pragma unroll
            for (int J = 0; J < NB; J++) A[J] = sel[b & 1][J];
#pragma unroll
            for (int J = 0; J < NB / 4; J++)
                *reinterpret_cast<float4*>(&EP[4 * J]) = reinterpret_cast<const float4*>(sep[b & 1])[J];
        }
        float PH[NB] = {};
        if (MODE != 3 || t < 16)  // mode 3: lanes 16-63 sit out
        unroll_ic(
            [&](auto jc) {
                constexpr int J = decltype(jc)::value;
                if constexpr (MODE == 2 || MODE == 3) {
                    NA[J] = sel[(b + 1) & 1][J];
                    if constexpr (J % 4 == 0)
                        *reinterpret_cast<float4*>(&NEP[J]) = reinterpret_cast<const float4*>(sep[(b + 1) & 1])[J / 4];
                }
                const float4 a = (MODE == 0 || MODE == 6 || MODE >= 9) ? A0[J] : A[J];
                const float ep = (MODE == 0 || MODE == 6 || MODE >= 9) ? E0[J] : EP[J];
                (void)0;
                float e;
                if constexpr (MODE == 10 || MODE == 11) {
                    uint32_t d0, d1;
                    float k1;
                    if constexpr (MODE == 10)
                        asm volatile(
                            "v_sub_f32 %1, %3, %6\n v_sub_f32 %2, %3, %7\n v_ashrrev_i32 %1, 31, %1\n"
                            " v_ashrrev_i32 %2, 31, %2\n v_bfi_b32 %1, %1, %8, %9\n v_bfi_b32 %1, %2, %1, %10\n"
                            " v_mul_f32 %5, %11, %1\n v_mul_f32 %2, %12, %1\n"
                            " v_add_f32 %4, %4, %5\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %2"
                            : "=&v"(e), "=&v"(d0), "=&v"(d1), "+v"(phase), "+v"(integ), "=&v"(k1)
                            : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(ep), "v"(Ki), "v"(Kp));
                    else
                        asm volatile(
                            "v_cmp_ge_f32_e64 s[40:41], %3, %6\n v_cmp_ge_f32_e64 s[42:43], %3, %7\n s_nop 0\n"
                            " v_cndmask_b32_e64 %1, %8, %9, s[40:41]\n v_cndmask_b32_e64 %1, %1, %10, s[42:43]\n"
                            " v_mul_f32 %5, %11, %1\n v_mul_f32 %2, %12, %1\n"
                            " v_add_f32 %4, %4, %5\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %2"
                            : "=&v"(e), "=&v"(d0), "=&v"(d1), "+v"(phase), "+v"(integ), "=&v"(k1)
                            : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(ep), "v"(Ki), "v"(Kp)
                            : "s40", "s41", "s42", "s43");
                    PH[J] = phase;
                    (void)e;
                } else if constexpr (MODE == 9 || MODE >= 12) {
                    asm volatile(
                        "v_cmp_ge_f32_e64 s[40:41], %1, %2\n v_cmp_ge_f32_e64 s[42:43], %1, %3\n s_nop 0\n"
                        " v_cndmask_b32_e64 %0, %4, %5, s[40:41]\n v_cndmask_b32_e64 %0, %0, %6, s[42:43]"
                        : "=&v"(e)
                        : "v"(phase), "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(ep)
                        : "s40", "s41", "s42", "s43");
                } else if constexpr (MODE == 6 || MODE == 7 || MODE == 8) {
                    uint32_t d0, d1;
                    asm("v_sub_f32 %1, %3, %4\n v_sub_f32 %2, %3, %5\n v_ashrrev_i32 %1, 31, %1\n"
                        " v_ashrrev_i32 %2, 31, %2\n v_bfi_b32 %1, %1, %6, %7\n v_bfi_b32 %0, %2, %1, %8"
                        : "=&v"(e), "=&v"(d0), "=&v"(d1)
                        : "v"(phase), "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(ep));
                } else {
                    const uint32_t m0 = sign_mask(phase - a.x), m1 = sign_mask(phase - a.y);
                    e = bfi(m1, bfi(m0, a.z, a.w), ep);
                }
                if constexpr (MODE != 10 && MODE != 11) {
                    const float2v k = float2v{Ki, Kp} * e;
                    integ = integ + k.x;
                    phase = phase + (k.y + integ);
                    PH[J] = phase;
                }
                if constexpr ((MODE == 13 || MODE == 14) && J % 4 == 3) {
                    const float4 v4 = make_float4(PH[J - 3], PH[J - 2], PH[J - 1], PH[J]);
                    if constexpr (MODE == 13) {
                        sph[b & 1][J / 4] = v4;
                    } else {
                        f4 v = {v4.x, v4.y, v4.z, v4.w};
                        const unsigned a = (unsigned)(uintptr_t)&sph[b & 1][J / 4];
                        asm volatile("s_mov_b64 s[44:45], exec\n s_mov_b64 exec, 1\n ds_write_b128 %0, %1\n"
                                     " s_mov_b64 exec, s[44:45]" ::"v"(a), "v"(v) : "s44", "s45", "memory");
                    }
                }
                if constexpr (MODE == 2 || MODE == 3) __builtin_amdgcn_sched_barrier(0);
            },
            std::make_integer_sequence<int, NB>{});
        if constexpr (MODE == 12) {
            if (t == 0) {
#pragma unroll
                for (int q = 0; q < NB / 4; q++)
                    sph[b & 1][q] = make_float4(PH[4 * q], PH[4 * q + 1], PH[4 * q + 2], PH[4 * q + 3]);
            }
        }
#pragma unroll
        for (int J = 0; J < NB; J++) acc += PH[J];
        phase = phase * 0.5f;  // keep it in range
        if (nw > 1) __syncthreads();
    };
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    for (int b = 0; b < nb; b += 2) {
        run(b, A0, E0, A1, E1);
        run(b + 1, A1, E1, A0, E0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const long long t1 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    out[t] = acc + integ;
    if (t == 0) cyc[0] = t1 - t0;
}

template <int MODE>
static void run(int waves, int busy, float* d_out, long long* d_cyc) {
    const int nb = 4096;
    long long best = 1LL << 60;
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(chain<MODE>, dim3(1), dim3(64 * waves), 0, 0, d_out, d_cyc, nb, busy);
        long long c;
        (void)hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
        if (c < best) best = c;
    }
    std::printf("mode %d  waves %d  others %-5s  %7.1f cycles/step\n", MODE, waves, busy ? "busy" : "idle",
                (double)best / (nb * NB));
}

int main() {
    float* d_out;
    long long* d_cyc;
    (void)hipMalloc(&d_out, 256 * 4);
    (void)hipMalloc(&d_cyc, 8);
    for (int waves : {1, 3}) {
        for (int busy : {0, 1}) {
            if (waves == 1 && busy) continue;
            run<0>(waves, busy, d_out, d_cyc);
            run<1>(waves, busy, d_out, d_cyc);
            run<2>(waves, busy, d_out, d_cyc);
            run<3>(waves, busy, d_out, d_cyc);
            run<4>(waves, busy, d_out, d_cyc);
            run<5>(waves, busy, d_out, d_cyc);
            run<6>(waves, busy, d_out, d_cyc);
            run<7>(waves, busy, d_out, d_cyc);
            run<8>(waves, busy, d_out, d_cyc);
            run<9>(waves, busy, d_out, d_cyc);
            run<10>(waves, busy, d_out, d_cyc);
            run<11>(waves, busy, d_out, d_cyc);
            run<12>(waves, busy, d_out, d_cyc);
            run<13>(waves, busy, d_out, d_cyc);
            run<14>(waves, busy, d_out, d_cyc);
        }
    }
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return 0;
}
