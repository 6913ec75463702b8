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
//   mode 15: mode 9 with the choice in C (ternaries; the compiler places the wait states),
//   mode 16: mode 15 + the next batch's data read during the steps, one read placed by
//            sched_group_barrier in each wait-state slot (between the compares and the selects,
//            and before the multiply),
//   mode 17: mode 9 with (Ki e, Kp e) as two v_mul_f32 instead of v_pk_mul_f32,
//   mode 18: mode 9 with the next batch's 16-B reads inside the choice's asm block in place of
//            its s_nop (timing only: the compiler does not know those registers are in flight),
//   mode 19: mode 17 + mode 2's reads (one a step, compiler-placed),
//   mode 20: the whole step in one asm block with fresh outputs (compares, s_nop, selects, two
//            v_mul_f32, three adds: 10 instructions, no copies),
//   mode 21: mode 20 with the next batch's 16-B read in the s_nop's place, its ep reads every
//            fourth step and the phases stored to LDS four at a time (lane 0 to the ring, the
//            other lanes to a scratch row: no exec mask, no branch),
//   mode 22: mode 21 with EXEC = lane 0 over the batch's steps (set and restored in asm),
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
    __shared__ float4 sdum[64 + NB / 2];
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
        if constexpr (MODE == 18 || MODE >= 21) __builtin_amdgcn_s_waitcnt(0xC07F);  // the asm's reads (previous batch)
        if constexpr (MODE == 22) asm volatile("s_mov_b64 s[44:45], exec\n s_mov_b64 exec, 1" ::: "s44", "s45");
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
                if constexpr (MODE == 19) {
                    NA[J] = sel[(b + 1) & 1][J];
                    if constexpr (J % 4 == 0)
                        *reinterpret_cast<float4*>(&NEP[J]) = reinterpret_cast<const float4*>(sep[(b + 1) & 1])[J / 4];
                }
                const bool regs = MODE == 0 || MODE == 6 || (MODE >= 9 && MODE != 16 && MODE != 18 && MODE != 19 && MODE != 21 && MODE != 22);
                const float4 a = regs ? A0[J] : A[J];
                const float ep = regs ? E0[J] : EP[J];
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
                } else if constexpr (MODE == 15 || MODE == 16) {
                    if constexpr (MODE == 16) {
                        NA[J] = sel[(b + 1) & 1][J];
                        if constexpr (J % 4 == 0)
                            *reinterpret_cast<float4*>(&NEP[J]) = reinterpret_cast<const float4*>(sep[(b + 1) & 1])[J / 4];
                    }
                    const bool m0 = phase >= a.x, m1 = phase >= a.y;
                    e = m1 ? ep : (m0 ? a.w : a.z);
                } else if constexpr (MODE == 18) {
                    const unsigned na = (unsigned)(uintptr_t)&sel[(b + 1) & 1][J];
                    f4 v;
                    asm volatile(
                        "v_cmp_ge_f32_e64 s[40:41], %2, %3\n v_cmp_ge_f32_e64 s[42:43], %2, %4\n ds_read_b128 %1, %8\n"
                        " v_cndmask_b32_e64 %0, %5, %6, s[40:41]\n v_cndmask_b32_e64 %0, %0, %7, s[42:43]"
                        : "=&v"(e), "=&v"(v)
                        : "v"(phase), "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(ep), "v"(na)
                        : "s40", "s41", "s42", "s43");
                    NA[J] = make_float4(v.x, v.y, v.z, v.w);
                    if constexpr (J % 4 == 0)
                        *reinterpret_cast<float4*>(&NEP[J]) = reinterpret_cast<const float4*>(sep[(b + 1) & 1])[J / 4];
                } else if constexpr (MODE == 20 || MODE == 21 || MODE == 22) {
                    float e, ka, kb, ig, ph;
                    uint64_t m0, m1;
                    f4 nx;
                    if constexpr (MODE == 20)
                        asm volatile(
                            "v_cmp_ge_f32_e64 %[m0], %[p], %[t0]\n v_cmp_ge_f32_e64 %[m1], %[p], %[t1]\n s_nop 0\n"
                            " v_cndmask_b32_e64 %[e], %[em], %[e0], %[m0]\n v_cndmask_b32_e64 %[e], %[e], %[ep], %[m1]\n"
                            " v_mul_f32 %[ka], %[ki], %[e]\n v_mul_f32 %[kb], %[kp], %[e]\n"
                            " v_add_f32 %[ig], %[ii], %[ka]\n v_add_f32 %[kb], %[kb], %[ig]\n v_add_f32 %[ph], %[p], %[kb]"
                            : [e] "=&v"(e), [ka] "=&v"(ka), [kb] "=&v"(kb), [ig] "=&v"(ig), [ph] "=&v"(ph),
                              [m0] "=&s"(m0), [m1] "=&s"(m1)
                            : [p] "v"(phase), [ii] "v"(integ), [t0] "v"(a.x), [t1] "v"(a.y), [em] "v"(a.z),
                              [e0] "v"(a.w), [ep] "v"(ep), [ki] "v"(Ki), [kp] "v"(Kp));
                    else
                        asm volatile(
                            "v_cmp_ge_f32_e64 %[m0], %[p], %[t0]\n v_cmp_ge_f32_e64 %[m1], %[p], %[t1]\n"
                            " ds_read_b128 %[nx], %[ra] offset:%[ro]\n"
                            " v_cndmask_b32_e64 %[e], %[em], %[e0], %[m0]\n v_cndmask_b32_e64 %[e], %[e], %[ep], %[m1]\n"
                            " v_mul_f32 %[ka], %[ki], %[e]\n v_mul_f32 %[kb], %[kp], %[e]\n"
                            " v_add_f32 %[ig], %[ii], %[ka]\n v_add_f32 %[kb], %[kb], %[ig]\n v_add_f32 %[ph], %[p], %[kb]"
                            : [e] "=&v"(e), [ka] "=&v"(ka), [kb] "=&v"(kb), [ig] "=&v"(ig), [ph] "=&v"(ph),
                              [m0] "=&s"(m0), [m1] "=&s"(m1), [nx] "=&v"(nx)
                            : [p] "v"(phase), [ii] "v"(integ), [t0] "v"(a.x), [t1] "v"(a.y), [em] "v"(a.z),
                              [e0] "v"(a.w), [ep] "v"(ep), [ki] "v"(Ki), [kp] "v"(Kp),
                              [ra] "v"((unsigned)(uintptr_t)&sel[(b + 1) & 1][0]), [ro] "i"(16 * J));
                    if constexpr (MODE >= 21) {
                        NA[J] = make_float4(nx.x, nx.y, nx.z, nx.w);
                        if constexpr (J % 4 == 0) {
                            f4 ne;
                            asm volatile("ds_read_b128 %0, %1 offset:%2"
                                         : "=v"(ne) : "v"((unsigned)(uintptr_t)&sep[(b + 1) & 1][0]), "i"(4 * J));
                            NEP[J] = ne.x; NEP[J + 1] = ne.y; NEP[J + 2] = ne.z; NEP[J + 3] = ne.w;
                        }
                    }
                    integ = ig;
                    phase = ph;
                    PH[J] = phase;
                    e = 0.0f;
                    (void)e;
                    if constexpr (MODE >= 21 && J % 4 == 3) {
                        const unsigned wa = t == 0 ? (unsigned)(uintptr_t)&sph[b & 1][0]
                                                   : (unsigned)(uintptr_t)&sdum[t];
                        const f4 v = {PH[J - 3], PH[J - 2], PH[J - 1], PH[J]};
                        asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(wa), "v"(v), "i"(4 * (J - 3)) : "memory");
                    }
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
                if constexpr (MODE == 17 || MODE == 19) {
                    float k1 = Ki * e;
                    asm("" : "+v"(k1));  // keeps the two products apart (no v_pk_mul_f32)
                    const float k2 = Kp * e;
                    integ = integ + k1;
                    phase = phase + (k2 + integ);
                    PH[J] = phase;
                } else if constexpr (MODE != 10 && MODE != 11 && MODE != 20 && MODE != 21 && MODE != 22) {
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
                if constexpr (MODE == 16) {
                    // cmp, cmp | read | cndmask, cndmask | read (every 4th step) | pk_mul | adds
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, J);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, J);
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, J);
                    if constexpr (J % 4 == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, J);
                    __builtin_amdgcn_sched_group_barrier(0x002, 4, J);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if constexpr (MODE == 2 || MODE == 3 || MODE == 18 || MODE == 19) __builtin_amdgcn_sched_barrier(0);
            },
            std::make_integer_sequence<int, NB>{});
        if constexpr (MODE == 22) asm volatile("s_mov_b64 exec, s[44:45]" ::: "memory");
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
            run<15>(waves, busy, d_out, d_cyc);
            run<16>(waves, busy, d_out, d_cyc);
            run<17>(waves, busy, d_out, d_cyc);
            run<18>(waves, busy, d_out, d_cyc);
            run<19>(waves, busy, d_out, d_cyc);
            run<20>(waves, busy, d_out, d_cyc);
            run<21>(waves, busy, d_out, d_cyc);
            run<22>(waves, busy, d_out, d_cyc);
        }
    }
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return 0;
}
