// tools/ubench_cnt.hip — the dependent latency of the PLL chain forms, measured per form and per
// piece (round 4's verdict: "report the chain's measured dependent latency beside the instruction
// count").  One workgroup; wave 0 runs batches of 16 chain steps with the step data in registers
// (the same every batch), the other waves idle at one barrier a batch or busy with f64 FMAs.
//   mode 0: pll_idx_kernel's step (pll_pred.hip): e = v_readlane(row, s) with s from the previous
//           step's v_readfirstlane, (Ki e, Kp e), the three float updates, trigArg =
//           float(P + (double)phase) (cvt, add_f64, cvt), its lane index (sub, readfirstlane);
//   mode 1: mode 0 without the f64 trigArg: the index from the float phase's bits (sub only);
//   mode 2: mode 0 without the SGPR round trip: e = E[J] (no readlane), the index kept in a VGPR
//           and folded into e by a v_cndmask on (idx < 64) -- the f64 trigArg still on the chain;
//   mode 3: the "count" step: one v_cmp_ge_f32 of the phase against a row of thresholds (lane l:
//           T(c_base + l)) into an SGPR pair, s_bcnt1 of the mask, e = v_readlane(E, count),
//           (Ki e, Kp e) with e an SGPR operand, the three updates (C, compiler-scheduled);
//   mode 4: mode 3 as one asm block of four steps (no compiler padding, VCC-free);
//   mode 5: mode 4 with the compare into VCC (v_cmp_ge_f32_e32);
//   mode 6: the tail alone: e = v_readlane(E, const SGPR), (Ki e, Kp e), three updates;
//   mode 7: pll_pipe_kernel's three-candidate step (two compares, two v_cndmask, pk_mul, three
//           updates; ubench_chain mode 9);
//   mode 8: mode 4 with the pk_mul replaced by two v_mul_f32 with the SGPR e;
//   mode 9: the bare VALU tail: e = E[J] (VGPR), pk_mul, three updates (the arithmetic floor);
//   mode 10: mode 4 with (Ki e, Kp e) precomputed (two rows, two v_readlane, no multiply);
//   mode 11: mode 7 with (Ki e, Kp e) precomputed (four v_cndmask, no multiply);
//   mode 12: the "exec" step: v_cmpx_ge_f32 of the phase against a row of thresholds in
//            descending lane order (EXEC = the lanes whose threshold the phase reaches, a
//            suffix), e = v_readfirstlane(E) (the lowest active lane holds the chosen e),
//            EXEC restored, (Ki e, Kp e) with e an SGPR, three updates; s_nop 4 after the cmpx;
//   mode 13: mode 12 with s_nop 0 after the cmpx (timing only if the hazard needs more);
//   mode 14: mode 12 with (Ki e, Kp e) precomputed (two v_readfirstlane, no multiply);
//   mode 15: pll_pipe_kernel's five-candidate step as its four-step asm block (chain4_5: four
//            compares into SGPR masks, four v_cndmask, v_pk_mul_f32 with (Ki, Kp) in SGPRs, three
//            updates);
//   mode 16: the three-candidate step as its four-step asm block (chain4_3).
// Prints shader cycles (s_memtime) per step.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench_cnt tools/ubench_cnt.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <utility>

typedef float float2v __attribute__((ext_vector_type(2)));

template <class F, int... J>
__device__ inline void unroll_ic(F&& f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}

constexpr int NB = 16;

// one count step: phase vs the row of thresholds T, e = E[count], (Ki e, Kp e), three updates
#define CNT_STEP(P, Q, K)                                      \
    "v_cmp_ge_f32_e64 s[40:41], " P ", %[t" #K "]\n"             \
    "s_bcnt1_i32_b64 s42, s[40:41]\n"                          \
    "v_readlane_b32 s44, %[e" #K "], s42\n"                      \
    "s_nop 1\n"                                                 \
    "v_pk_mul_f32 v[254:255], s[44:45], %[kk] op_sel_hi:[0,1]\n" \
    "v_add_f32 %[ig], %[ig], v254\n"                           \
    "v_add_f32 v255, v255, %[ig]\n"                            \
    "v_add_f32 " Q ", " P ", v255\n"
#define CNT_STEP_VCC(P, Q, K)                                  \
    "v_cmp_ge_f32_e32 vcc, " P ", %[t" #K "]\n"                  \
    "s_bcnt1_i32_b64 s42, vcc\n"                               \
    "v_readlane_b32 s44, %[e" #K "], s42\n"                      \
    "s_nop 1\n"                                                 \
    "v_pk_mul_f32 v[254:255], s[44:45], %[kk] op_sel_hi:[0,1]\n" \
    "v_add_f32 %[ig], %[ig], v254\n"                           \
    "v_add_f32 v255, v255, %[ig]\n"                            \
    "v_add_f32 " Q ", " P ", v255\n"
#define CNT_STEP_2MUL(P, Q, K)                                 \
    "v_cmp_ge_f32_e64 s[40:41], " P ", %[t" #K "]\n"             \
    "s_bcnt1_i32_b64 s42, s[40:41]\n"                          \
    "v_readlane_b32 s44, %[e" #K "], s42\n"                      \
    "s_nop 1\n"                                                 \
    "v_mul_f32 v254, s44, %[ki]\n"                             \
    "v_mul_f32 v255, s44, %[kp]\n"                             \
    "v_add_f32 %[ig], %[ig], v254\n"                           \
    "v_add_f32 v255, v255, %[ig]\n"                            \
    "v_add_f32 " Q ", " P ", v255\n"

#define CNT_STEP_PRE(P, Q, K)                                  \
    "v_cmp_ge_f32_e64 s[40:41], " P ", %[t" #K "]\n"             \
    "s_bcnt1_i32_b64 s42, s[40:41]\n"                          \
    "v_readlane_b32 s44, %[e" #K "], s42\n"                      \
    "v_readlane_b32 s45, %[f" #K "], s42\n"                      \
    "s_nop 0\n"                                                 \
    "v_add_f32 %[ig], %[ig], s44\n"                            \
    "v_add_f32 v255, s45, %[ig]\n"                             \
    "v_add_f32 " Q ", " P ", v255\n"
#define EXEC_STEP(P, Q, K, NOP)                                 \
    "v_cmpx_ge_f32_e64 s[40:41], " P ", %[t" #K "]\n"            \
    "s_nop " #NOP "\n"                                          \
    "v_readfirstlane_b32 s44, %[e" #K "]\n"                     \
    "s_mov_b64 exec, -1\n"                                     \
    "s_nop 1\n"                                                 \
    "v_pk_mul_f32 v[254:255], s[44:45], %[kk] op_sel_hi:[0,1]\n" \
    "v_add_f32 %[ig], %[ig], v254\n"                           \
    "v_add_f32 v255, v255, %[ig]\n"                            \
    "v_add_f32 " Q ", " P ", v255\n"
#define EXEC_STEP_PRE(P, Q, K)                                  \
    "v_cmpx_ge_f32_e64 s[40:41], " P ", %[t" #K "]\n"            \
    "s_nop 4\n"                                                 \
    "v_readfirstlane_b32 s44, %[e" #K "]\n"                     \
    "v_readfirstlane_b32 s45, %[f" #K "]\n"                     \
    "s_mov_b64 exec, -1\n"                                     \
    "s_nop 0\n"                                                 \
    "v_add_f32 %[ig], %[ig], s44\n"                            \
    "v_add_f32 v255, s45, %[ig]\n"                             \
    "v_add_f32 " Q ", " P ", v255\n"

#define ASM4(STEP, ...)                                                                                  \
    asm volatile(STEP("%[p]", "%[q1]", 0 __VA_ARGS__) STEP("%[q1]", "%[q2]", 1 __VA_ARGS__)            \
                     STEP("%[q2]", "%[q3]", 2 __VA_ARGS__) STEP("%[q3]", "%[q4]", 3 __VA_ARGS__)       \
                 : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ)      \
                 : [p] "v"(phase), [kk] "v"(kk), [t0] "v"(T[q]), [t1] "v"(T[q + 1]), [t2] "v"(T[q + 2]), \
                   [t3] "v"(T[q + 3]), [e0] "v"(E[q]), [e1] "v"(E[q + 1]), [e2] "v"(E[q + 2]),           \
                   [e3] "v"(E[q + 3]), [f0] "v"(F[q]), [f1] "v"(F[q + 1]), [f2] "v"(F[q + 2]),           \
                   [f3] "v"(F[q + 3])                                                                     \
                 : "s40", "s41", "s42", "s44", "s45", "v254", "v255", "exec")

// pll_pred.hip's chain blocks (FMRX_CHAIN_STEP3 / STEP5), verbatim
#define PT_TAIL(P, Q)                                            \
    "v_pk_mul_f32 v[254:255], v[252:253], %[kk] op_sel_hi:[0,1]\n" \
    "v_add_f32 %[ig], %[ig], v254\n"                             \
    "v_add_f32 v255, v255, %[ig]\n"                              \
    "v_add_f32 " Q ", " P ", v255\n"
#define PT_STEP3(P, Q, K)                                  \
    "v_cmp_ge_f32_e64 %[m0], " P ", %[ta" #K "]\n"           \
    "v_cmp_ge_f32_e64 %[m1], " P ", %[tb" #K "]\n"           \
    "s_nop 0\n"                                            \
    "v_cndmask_b32_e64 v252, %[ea" #K "], %[eb" #K "], %[m0]\n" \
    "v_cndmask_b32_e64 v252, v252, %[ec" #K "], %[m1]\n" PT_TAIL(P, Q)
#define PT_STEP5(P, Q, K)                                  \
    "v_cmp_ge_f32_e64 %[m0], " P ", %[ta" #K "]\n"           \
    "v_cmp_ge_f32_e64 %[m1], " P ", %[tb" #K "]\n"           \
    "v_cmp_ge_f32_e64 %[m2], " P ", %[tc" #K "]\n"           \
    "v_cmp_ge_f32_e64 %[m3], " P ", %[td" #K "]\n"           \
    "v_cndmask_b32_e64 v252, %[ea" #K "], %[eb" #K "], %[m0]\n" \
    "v_cndmask_b32_e64 v252, v252, %[ec" #K "], %[m1]\n"     \
    "v_cndmask_b32_e64 v252, v252, %[ed" #K "], %[m2]\n"     \
    "v_cndmask_b32_e64 v252, v252, %[ee" #K "], %[m3]\n" PT_TAIL(P, Q)

template <int MODE>
__global__ void __launch_bounds__(256) chain(float* out, long long* cyc, int nb, int busy) {
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
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
    // step data: P near 2^18 steps' worth of phase, thresholds around the phase, e values
    float4 R[NB];
    float E[NB], T[NB], F[NB];
#pragma unroll
    for (int J = 0; J < NB; J++) {
        const double P = 130000.0 + 0.079 * J;
        const float c0 = (float)(P + 0.01);
        const uint64_t pb = __builtin_bit_cast(uint64_t, P);
        R[J] = make_float4(__builtin_bit_cast(float, (uint32_t)pb), __builtin_bit_cast(float, (uint32_t)(pb >> 32)),
                           __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, c0) - 32u), 0.0f);
        E[J] = 1e-4f * (t - 32) + 1e-6f * J;
        F[J] = 2e-4f * (t - 32) + 3e-6f * J;
        T[J] = 0.01f + 1e-3f * (t - 32) + 1e-7f * J;
    }
    float acc = 0.0f;
    uint32_t cL = 0;
    float cE = E[0];
    const float2v kk{Ki, Kp};
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    for (int b = 0; b < nb; b++) {
        if constexpr (MODE == 10 || MODE == 12 || MODE == 13 || MODE == 14) {
#pragma unroll
            for (int q = 0; q < NB; q += 4) {
                float p1, p2, p3, p4;
                if constexpr (MODE == 10)
                    ASM4(CNT_STEP_PRE);
                else if constexpr (MODE == 12)
                    ASM4(EXEC_STEP, , 4);
                else if constexpr (MODE == 13)
                    ASM4(EXEC_STEP, , 0);
                else
                    ASM4(EXEC_STEP_PRE);
                phase = p4;
                (void)p1;
                (void)p2;
                (void)p3;
            }
        } else if constexpr (MODE == 15 || MODE == 16) {
            const uint64_t skk = (uint64_t)__builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, Ki)) |
                                 ((uint64_t)__builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, Kp)) << 32);
#pragma unroll
            for (int q = 0; q < NB; q += 4) {
                float p1, p2, p3, p4;
                uint64_t m0, m1, m2, m3;
                auto Tq = [&](int u, int d) { return T[(q + u + d) % NB]; };
                auto Eq = [&](int u, int d) { return E[(q + u + d) % NB]; };
                if constexpr (MODE == 15)
                    asm volatile(PT_STEP5("%[p]", "%[q1]", 0) PT_STEP5("%[q1]", "%[q2]", 1) PT_STEP5("%[q2]", "%[q3]", 2)
                                     PT_STEP5("%[q3]", "%[q4]", 3)
                                 : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ),
                                   [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3)
                                 : [p] "v"(phase), [kk] "s"(skk),
                                   [ta0] "v"(Tq(0, 0)), [tb0] "v"(Tq(0, 1)), [tc0] "v"(Tq(0, 2)), [td0] "v"(Tq(0, 3)),
                                   [ea0] "v"(Eq(0, 0)), [eb0] "v"(Eq(0, 1)), [ec0] "v"(Eq(0, 2)), [ed0] "v"(Eq(0, 3)), [ee0] "v"(Eq(0, 4)),
                                   [ta1] "v"(Tq(1, 0)), [tb1] "v"(Tq(1, 1)), [tc1] "v"(Tq(1, 2)), [td1] "v"(Tq(1, 3)),
                                   [ea1] "v"(Eq(1, 0)), [eb1] "v"(Eq(1, 1)), [ec1] "v"(Eq(1, 2)), [ed1] "v"(Eq(1, 3)), [ee1] "v"(Eq(1, 4)),
                                   [ta2] "v"(Tq(2, 0)), [tb2] "v"(Tq(2, 1)), [tc2] "v"(Tq(2, 2)), [td2] "v"(Tq(2, 3)),
                                   [ea2] "v"(Eq(2, 0)), [eb2] "v"(Eq(2, 1)), [ec2] "v"(Eq(2, 2)), [ed2] "v"(Eq(2, 3)), [ee2] "v"(Eq(2, 4)),
                                   [ta3] "v"(Tq(3, 0)), [tb3] "v"(Tq(3, 1)), [tc3] "v"(Tq(3, 2)), [td3] "v"(Tq(3, 3)),
                                   [ea3] "v"(Eq(3, 0)), [eb3] "v"(Eq(3, 1)), [ec3] "v"(Eq(3, 2)), [ed3] "v"(Eq(3, 3)), [ee3] "v"(Eq(3, 4))
                                 : "v252", "v253", "v254", "v255");
                else
                    asm volatile(PT_STEP3("%[p]", "%[q1]", 0) PT_STEP3("%[q1]", "%[q2]", 1) PT_STEP3("%[q2]", "%[q3]", 2)
                                     PT_STEP3("%[q3]", "%[q4]", 3)
                                 : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ),
                                   [m0] "=&s"(m0), [m1] "=&s"(m1)
                                 : [p] "v"(phase), [kk] "s"(skk),
                                   [ta0] "v"(Tq(0, 0)), [tb0] "v"(Tq(0, 1)), [ea0] "v"(Eq(0, 0)), [eb0] "v"(Eq(0, 1)), [ec0] "v"(Eq(0, 2)),
                                   [ta1] "v"(Tq(1, 0)), [tb1] "v"(Tq(1, 1)), [ea1] "v"(Eq(1, 0)), [eb1] "v"(Eq(1, 1)), [ec1] "v"(Eq(1, 2)),
                                   [ta2] "v"(Tq(2, 0)), [tb2] "v"(Tq(2, 1)), [ea2] "v"(Eq(2, 0)), [eb2] "v"(Eq(2, 1)), [ec2] "v"(Eq(2, 2)),
                                   [ta3] "v"(Tq(3, 0)), [tb3] "v"(Tq(3, 1)), [ea3] "v"(Eq(3, 0)), [eb3] "v"(Eq(3, 1)), [ec3] "v"(Eq(3, 2))
                                 : "v252", "v253", "v254", "v255");
                phase = p4;
                (void)m2;
                (void)m3;
                (void)p1;
                (void)p2;
                (void)p3;
            }
        } else if constexpr (MODE == 11) {
#pragma unroll
            for (int J = 0; J < NB; J++) {
                float a, b;
                uint64_t m0, m1;
                asm volatile(
                    "v_cmp_ge_f32_e64 %2, %4, %5\n"
                    "v_cmp_ge_f32_e64 %3, %4, %6\n"
                    "s_nop 0\n"
                    "v_cndmask_b32_e64 %0, %7, %8, %2\n"
                    "v_cndmask_b32_e64 %1, %10, %11, %2\n"
                    "v_cndmask_b32_e64 %0, %0, %9, %3\n"
                    "v_cndmask_b32_e64 %1, %1, %12, %3"
                    : "=&v"(a), "=&v"(b), "=&s"(m0), "=&s"(m1)
                    : "v"(phase), "v"(T[J]), "v"(T[(J + 1) % NB]), "v"(E[J]), "v"(E[(J + 1) % NB]),
                      "v"(E[(J + 2) % NB]), "v"(F[J]), "v"(F[(J + 1) % NB]), "v"(F[(J + 2) % NB]));
                integ = integ + a;
                phase = phase + (b + integ);
            }
        } else if constexpr (MODE == 4 || MODE == 5 || MODE == 8) {
#pragma unroll
            for (int q = 0; q < NB; q += 4) {
                float p1, p2, p3, p4;
                if constexpr (MODE == 4)
                    asm volatile(CNT_STEP("%[p]", "%[q1]", 0) CNT_STEP("%[q1]", "%[q2]", 1) CNT_STEP("%[q2]", "%[q3]", 2)
                                     CNT_STEP("%[q3]", "%[q4]", 3)
                                 : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ)
                                 : [p] "v"(phase), [kk] "v"(kk), [t0] "v"(T[q]), [t1] "v"(T[q + 1]),
                                   [t2] "v"(T[q + 2]), [t3] "v"(T[q + 3]), [e0] "v"(E[q]), [e1] "v"(E[q + 1]),
                                   [e2] "v"(E[q + 2]), [e3] "v"(E[q + 3])
                                 : "s40", "s41", "s42", "s44", "s45", "v254", "v255");
                else if constexpr (MODE == 5)
                    asm volatile(CNT_STEP_VCC("%[p]", "%[q1]", 0) CNT_STEP_VCC("%[q1]", "%[q2]", 1)
                                     CNT_STEP_VCC("%[q2]", "%[q3]", 2) CNT_STEP_VCC("%[q3]", "%[q4]", 3)
                                 : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ)
                                 : [p] "v"(phase), [kk] "v"(kk), [t0] "v"(T[q]), [t1] "v"(T[q + 1]),
                                   [t2] "v"(T[q + 2]), [t3] "v"(T[q + 3]), [e0] "v"(E[q]), [e1] "v"(E[q + 1]),
                                   [e2] "v"(E[q + 2]), [e3] "v"(E[q + 3])
                                 : "vcc", "s42", "s44", "s45", "v254", "v255");
                else
                    asm volatile(CNT_STEP_2MUL("%[p]", "%[q1]", 0) CNT_STEP_2MUL("%[q1]", "%[q2]", 1)
                                     CNT_STEP_2MUL("%[q2]", "%[q3]", 2) CNT_STEP_2MUL("%[q3]", "%[q4]", 3)
                                 : [q1] "=&v"(p1), [q2] "=&v"(p2), [q3] "=&v"(p3), [q4] "=&v"(p4), [ig] "+v"(integ)
                                 : [p] "v"(phase), [ki] "v"(Ki), [kp] "v"(Kp), [t0] "v"(T[q]), [t1] "v"(T[q + 1]),
                                   [t2] "v"(T[q + 2]), [t3] "v"(T[q + 3]), [e0] "v"(E[q]), [e1] "v"(E[q + 1]),
                                   [e2] "v"(E[q + 2]), [e3] "v"(E[q + 3])
                                 : "s40", "s41", "s42", "s44", "s45", "v254", "v255");
                phase = p4;
                (void)p1;
                (void)p2;
                (void)p3;
            }
        } else if constexpr (MODE == 7) {
#pragma unroll
            for (int J = 0; J < NB; J++) {
                float e;
                uint64_t m0, m1;
                asm volatile(
                    "v_cmp_ge_f32_e64 %1, %3, %4\n"
                    "v_cmp_ge_f32_e64 %2, %3, %5\n"
                    "s_nop 0\n"
                    "v_cndmask_b32_e64 %0, %6, %7, %1\n"
                    "v_cndmask_b32_e64 %0, %0, %8, %2"
                    : "=&v"(e), "=&s"(m0), "=&s"(m1)
                    : "v"(phase), "v"(T[J]), "v"(T[(J + 1) % NB]), "v"(E[J]), "v"(E[(J + 1) % NB]),
                      "v"(E[(J + 2) % NB]));
                const float2v k = kk * e;
                integ = integ + k.x;
                phase = phase + (k.y + integ);
            }
        } else {
            unroll_ic(
                [&](auto jc) {
                    constexpr int J = decltype(jc)::value;
                    float e;
                    if constexpr (MODE == 0 || MODE == 1) {
                        e = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cE), cL));
                    } else if constexpr (MODE == 2) {
                        e = (cL < 64u) ? cE : 0.0f;
                    } else if constexpr (MODE == 3) {
                        const uint64_t m = __builtin_amdgcn_ballot_w64(phase >= T[J]);
                        const uint32_t c = (uint32_t)__builtin_popcountll(m);
                        e = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, E[J]), c));
                    } else if constexpr (MODE == 6) {
                        e = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, E[J]), J));
                    } else {
                        e = E[J];
                    }
                    const float2v k = kk * e;
                    integ = integ + k.x;
                    phase = phase + (k.y + integ);
                    if constexpr (MODE <= 2) {
                        const double P = __builtin_bit_cast(double, make_uint2(__builtin_bit_cast(uint32_t, R[J].x),
                                                                               __builtin_bit_cast(uint32_t, R[J].y)));
                        const float a = MODE == 1 ? phase : (float)(P + (double)phase);
                        const uint32_t i = __builtin_bit_cast(uint32_t, a) - __builtin_bit_cast(uint32_t, R[J].z);
                        cL = MODE == 2 ? i : __builtin_amdgcn_readfirstlane(i);
                        cE = E[J];
                    }
                },
                std::make_integer_sequence<int, NB>{});
        }
        phase = phase * 0.5f;
        if (blockDim.x > 64) __syncthreads();
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const long long t1 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    out[t] = acc + integ + phase + (float)cL;
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
                (double)best / ((double)nb * NB));
}

template <int... M>
static void run_all(int waves, int busy, float* d_out, long long* d_cyc, std::integer_sequence<int, M...>) {
    (run<M>(waves, busy, d_out, d_cyc), ...);
}

int main() {
    float* d_out;
    long long* d_cyc;
    (void)hipMalloc(&d_out, 1024 * 4);
    (void)hipMalloc(&d_cyc, 8);
    run_all(1, 0, d_out, d_cyc, std::make_integer_sequence<int, 17>{});
    run_all(4, 0, d_out, d_cyc, std::make_integer_sequence<int, 17>{});
    run_all(4, 1, d_out, d_cyc, std::make_integer_sequence<int, 17>{});
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return 0;
}
