// tools/ubench_dep.hip — cycles per instruction of dependent VALU chains on one wave (gfx950).
// The predicted PLL runner (pll_pred.hip) is a serial chain of a few VALU ops per step; this
// measures what each link costs: a dependent add, a compare feeding v_cndmask through VCC, the
// sub / shift / bitfield-insert select that needs no VCC, packed multiply, f64 add and the
// float -> double -> float round trip.  One wave, s_memtime around 64 x 32 chained ops.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/ubench_dep tools/ubench_dep.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(x) x x x x x x x x
#define R32(x) R8(x) R8(x) R8(x) R8(x)

template <int K>
__global__ void chain(float* out, long long* cyc, float a, float b) {
    float x = a + threadIdx.x * 1e-7f, y = b, z = b * 0.5f, w = b * 0.25f;
    float x1 = x + 1.0f, x2 = x + 2.0f, x3 = x + 3.0f;
    double d = x, dd = y;
    float m = 0.0f;
    long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0);
    for (int it = 0; it < 64; it++) {
        if constexpr (K == 0) {  // dependent f32 add
            asm volatile(R32("v_add_f32 %0, %0, %1\n") : "+v"(x) : "v"(y));
        } else if constexpr (K == 1) {  // four independent f32 add chains (issue rate)
            asm volatile(R8("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4\n")
                         : "+v"(x), "+v"(x1), "+v"(x2), "+v"(x3)
                         : "v"(y));
        } else if constexpr (K == 2) {  // compare -> VCC -> cndmask -> next compare (one link = 2 ops)
            asm volatile(R32("v_cmp_ge_f32 vcc, %0, %1\n s_nop 1\n v_cndmask_b32 %0, %2, %3, vcc\n")
                         : "+v"(x)
                         : "v"(y), "v"(z), "v"(w)
                         : "vcc");
        } else if constexpr (K == 3) {  // sub -> sign mask -> bfi (one link = 3 ops, no VCC)
            asm volatile(R32("v_sub_f32 %1, %0, %2\n v_ashrrev_i32 %1, 31, %1\n v_bfi_b32 %0, %1, %3, %4\n")
                         : "+v"(x), "=&v"(m)
                         : "v"(y), "v"(z), "v"(w));
        } else if constexpr (K == 4) {  // dependent packed f32 multiply
            asm volatile(R32("v_pk_mul_f32 %0, %0, %1\n") : "+v"(d) : "v"(dd));
        } else if constexpr (K == 5) {  // dependent f64 add
            asm volatile(R32("v_add_f64 %0, %0, %1\n") : "+v"(d) : "v"(dd));
        } else if constexpr (K == 6) {  // float -> double, add, -> float (one link = 3 ops)
            asm volatile(R32("v_cvt_f64_f32 %1, %0\n v_add_f64 %1, %1, %2\n v_cvt_f32_f64 %0, %1\n")
                         : "+v"(x), "=&v"(d)
                         : "v"(dd));
        } else if constexpr (K == 7) {  // med3 chain (a select-like op with no mask)
            asm volatile(R32("v_med3_f32 %0, %0, %1, %2\n") : "+v"(x) : "v"(y), "v"(z));
        } else if constexpr (K == 8) {  // compare to an SGPR pair (e64) -> cndmask
            asm volatile(R32("v_cmp_ge_f32_e64 s[8:9], %0, %1\n s_nop 1\n v_cndmask_b32_e64 %0, %2, %3, s[8:9]\n")
                         : "+v"(x)
                         : "v"(y), "v"(z), "v"(w)
                         : "s8", "s9");
        } else if constexpr (K == 9) {  // the same compare/cndmask without the s_nop
            asm volatile(R32("v_cmp_ge_f32 vcc, %0, %1\n v_cndmask_b32 %0, %2, %3, vcc\n")
                         : "+v"(x)
                         : "v"(y), "v"(z), "v"(w)
                         : "vcc");
        } else if constexpr (K == 10) {  // dependent f32 fma-free mul+add pair
            asm volatile(R32("v_mul_f32 %0, %0, %1\n v_add_f32 %0, %0, %2\n") : "+v"(x) : "v"(y), "v"(z));
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    long long t1 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0);
    out[threadIdx.x] = x + x1 + x2 + x3 + (float)d + m;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int K>
static void run(const char* what, int ops_per_link, float* d_out, long long* d_cyc) {
    long long best = 1LL << 60;
    for (int r = 0; r < 5; r++) {
        hipLaunchKernelGGL(chain<K>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, 1.0f, 0.5f);
        long long c;
        hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
        if (c < best) best = c;
    }
    const double links = 64.0 * 32.0;
    std::printf("%-52s %6.2f cycles/link  %5.2f cycles/op\n", what, best / links, best / links / ops_per_link);
}

int main() {
    float* d_out;
    long long* d_cyc;
    hipMalloc(&d_out, 64 * 4);
    hipMalloc(&d_cyc, 8);
    run<0>("dependent v_add_f32", 1, d_out, d_cyc);
    run<1>("4 independent v_add_f32 (per 4 ops)", 4, d_out, d_cyc);
    run<2>("v_cmp vcc; s_nop 1; v_cndmask (dependent)", 2, d_out, d_cyc);
    run<9>("v_cmp vcc; v_cndmask (no s_nop)", 2, d_out, d_cyc);
    run<8>("v_cmp_e64 sgpr; s_nop 1; v_cndmask_e64", 2, d_out, d_cyc);
    run<3>("v_sub_f32; v_ashrrev; v_bfi (dependent)", 3, d_out, d_cyc);
    run<4>("dependent v_pk_mul_f32", 1, d_out, d_cyc);
    run<5>("dependent v_add_f64", 1, d_out, d_cyc);
    run<6>("v_cvt_f64_f32; v_add_f64; v_cvt_f32_f64", 3, d_out, d_cyc);
    run<7>("dependent v_med3_f32", 1, d_out, d_cyc);
    run<10>("dependent v_mul_f32; v_add_f32", 2, d_out, d_cyc);
    hipFree(d_out);
    hipFree(d_cyc);
    return 0;
}
