// tools/ubench_mfma_add.hip — can the matrix pipe take part of the mono RF FIR's additions?
//
// The FIR (filter.cpp:84-92) needs, per tap and output, fl(c * s) then acc + that product, each
// separately rounded; no two outputs share a product.  f32 MFMA is an fmaf chain (MI355X_MICROARCH
// "Matrix cores"), so v_mfma_f32_4x4x1_16b_f32 with B one-hot (B_b[0] = 1, B_b[1..3] = 0) adds
// lane (4b + i)'s A value to D_b[i][0] with one rounding -- v_add_f32 -- and leaves the other 12
// entries of the block as they were (fma(a, 0, c) = c).  A takes one value a lane, so one such
// instruction does at most 64 useful (unshared) additions.  This probe measures what that buys
// beside the FIR's own packed VALU stream:
//   mode 0  FIR stream: per step C x (v_pk_mul_f32, v_pk_add_f32) -- 2 useful adds a lane per add
//   mode 1  the same stream with one 4x4x1 MFMA every G steps and the VALU multiplies its adds
//           need (one v_pk_mul_f32 every second MFMA): 64 more taps an MFMA
//   mode 2  4x4x1 MFMAs back to back (independent accumulators), no VALU
//   mode 3  16x16x4 f32 MFMAs back to back (the dense f32 rate, for reference)
// plus an exactness check: MFMA-one-hot sums == v_add_f32 sums bit for bit on random data.
// Output: FIR taps (a multiply and its add, for one of I or Q) per SIMD cycle (s_memtime) for
// modes 0/1, MFMA additions per SIMD cycle for 2/3; 1 and 2 waves a SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE, int C, int G>
__global__ void __launch_bounds__(256) probe(float* out, unsigned long long* cyc, int iters) {
    f2 acc[C], x[C];
    f4 d[4];
#pragma unroll
    for (int i = 0; i < C; i++) { acc[i] = f2{(float)threadIdx.x, 1.0f}; x[i] = f2{1e-7f * i, 2e-7f}; }
#pragma unroll
    for (int i = 0; i < 4; i++) d[i] = f4{1.0f * i, 2.0f, 3.0f, 4.0f};
    const float bsel = (threadIdx.x & 3) == 0 ? 1.0f : 0.0f;  // B one-hot: column 0 of each block
    f2 c = f2{1.0000001f, 0.9999999f};
    float a = 1e-3f * (float)threadIdx.x;
    f2 am = f2{a, a};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int rep = 0; rep < 16; rep++) {
            if constexpr (MODE == 0 || MODE == 1) {
#pragma unroll
                for (int i = 0; i < C; i++) {
                    f2 p;
                    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "v"(c), "v"(x[i]));
                    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(p));
                }
                if constexpr (MODE == 1) {
                    // the MFMA's products: one v_pk_mul_f32 every second MFMA (two MFMAs' 64 each),
                    // made one MFMA slot ahead of use
                    if (rep % G == 0) {
                        if ((rep / G) % 2 == 0) {
                            asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(d[(rep / G) & 3]) : "v"(am.x), "v"(bsel));
                            asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(am) : "v"(c), "v"(x[0]));
                        } else {
                            asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(d[(rep / G) & 3]) : "v"(am.y), "v"(bsel));
                        }
                    }
                }
            } else if constexpr (MODE == 2) {
#pragma unroll
                for (int i = 0; i < 4; i++)
                    asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(d[i]) : "v"(a), "v"(bsel));
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++)
                    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(d[i]) : "v"(a), "v"(bsel));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7");  // MFMA results read by VALU below
    float s = 0;
#pragma unroll
    for (int i = 0; i < C; i++) s += acc[i].x + acc[i].y;
#pragma unroll
    for (int i = 0; i < 4; i++) s += d[i].x + d[i].y + d[i].z + d[i].w;
    s += am.x + am.y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// exactness: acc_k = acc_{k-1} + a_k over 64 steps, once by v_add_f32 and once by the one-hot MFMA
__global__ void exact_probe(const float* a, const float* c0, float* out_valu, float* out_mfma) {
    const int t = threadIdx.x;
    float v = c0[t];
    for (int k = 0; k < 64; k++) {
        const float ak = a[k * 64 + t];
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(v) : "v"(ak));
    }
    out_valu[t] = v;
    // the MFMA form: lane 4b + i's A is added to D_b[i][0], which lives in VGPR i of lane 4b; so
    // the accumulator of lane 4b + i is D register i of lane 4b
    f4 d = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const int b = t >> 2, i = t & 3;
    // load C: D_b[r][0] (lane 4b, register r) = c0[4b + r]
    if (i == 0) d = f4{c0[4 * b], c0[4 * b + 1], c0[4 * b + 2], c0[4 * b + 3]};
    const float bsel = i == 0 ? 1.0f : 0.0f;
    for (int k = 0; k < 64; k++) {
        const float ak = a[k * 64 + t];
        asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0\n s_nop 7\n s_nop 7" : "+v"(d) : "v"(ak), "v"(bsel));
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7");
    if (i == 0) {
        out_mfma[4 * b] = d.x;
        out_mfma[4 * b + 1] = d.y;
        out_mfma[4 * b + 2] = d.z;
        out_mfma[4 * b + 3] = d.w;
    }
}

static int exactness() {
    std::vector<float> a(64 * 64), c0(64);
    uint32_t r = 12345;
    auto rnd = [&] { r = r * 1664525u + 1013904223u; return r; };
    for (auto& v : a) v = ((int)(rnd() >> 8) - (1 << 23)) * 1.37e-9f * (1 << (rnd() % 12));
    for (auto& v : c0) v = ((int)(rnd() >> 8) - (1 << 23)) * 3.1e-8f;
    float *da, *dc, *dv, *dm;
    CHECK(hipMalloc(&da, a.size() * 4)); CHECK(hipMalloc(&dc, 256)); CHECK(hipMalloc(&dv, 256)); CHECK(hipMalloc(&dm, 256));
    CHECK(hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dc, c0.data(), 256, hipMemcpyHostToDevice));
    exact_probe<<<1, 64>>>(da, dc, dv, dm);
    CHECK(hipDeviceSynchronize());
    std::vector<float> v(64), m(64);
    CHECK(hipMemcpy(v.data(), dv, 256, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(m.data(), dm, 256, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int t = 0; t < 64; t++) bad += std::memcmp(&v[t], &m[t], 4) != 0;
    printf("exactness: MFMA one-hot sums vs v_add_f32 sums, 64 lanes x 64 steps: %d mismatches\n", bad);
    hipFree(da); hipFree(dc); hipFree(dv); hipFree(dm);
    return 0;
}

template <int MODE, int C, int G>
static int run(int wps, const char* name) {
    const int n_cu = 256, blocks = n_cu * wps;  // 256-thread blocks: one wave a SIMD each
    float* out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&out, sizeof(float) * blocks * 256));
    CHECK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks));
    const int iters = 4000;
    probe<MODE, C, G><<<blocks, 256>>>(out, cyc, 20);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    probe<MODE, C, G><<<blocks, 256>>>(out, cyc, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(blocks);
    CHECK(hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost));
    double mean = 0;
    for (auto v : h) mean += (double)v;
    mean /= blocks;
    // useful additions a wave: VALU 128 a v_pk_add_f32 (64 lanes x 2), MFMA 64
    const double steps = (double)iters * 16;
    double adds = 0, valu = 0, mfma = 0;
    if (MODE <= 1) { adds += steps * C * 128; valu = steps * C * 2; }
    if (MODE == 1) { adds += steps / G * 64; mfma = steps / G; valu += steps / G / 2; }
    if (MODE == 2) { adds += steps * 4 * 64; mfma = steps * 4; }
    if (MODE == 3) { adds += steps * 4 * 256; mfma = steps * 4; }  // one-hot B: 256 of 1,024 fmas add
    // s_memtime ticks = shader cycles (MI355X_MICROARCH); per SIMD: wps waves share it
    const double per_simd_cyc = mean;  // the waves of a SIMD run concurrently over this span
    printf("%-34s waves/SIMD=%d  %.3f ms  %7.1f cyc/wave-step  taps (or MFMA adds)/SIMD-cycle %.2f  (VALU %.0f, MFMA %.0f a wave)\n",
           name, wps, ms, per_simd_cyc / steps, adds * wps / per_simd_cyc, valu, mfma);
    hipFree(out);
    hipFree(cyc);
    return 0;
}

int main() {
    if (exactness()) return 1;
    for (int w : {1, 2}) {
        run<0, 4, 1>(w, "FIR stream C=4 (VALU only)");
        run<1, 4, 1>(w, "FIR C=4 + one 4x4x1 MFMA a step");
        run<1, 4, 2>(w, "FIR C=4 + one 4x4x1 MFMA / 2 steps");
        run<1, 4, 4>(w, "FIR C=4 + one 4x4x1 MFMA / 4 steps");
        run<0, 8, 1>(w, "FIR stream C=8 (VALU only)");
        run<1, 8, 1>(w, "FIR C=8 + one 4x4x1 MFMA a step");
        run<1, 8, 2>(w, "FIR C=8 + one 4x4x1 MFMA / 2 steps");
        run<2, 1, 1>(w, "4x4x1 MFMA back to back");
        run<3, 1, 1>(w, "16x16x4 f32 MFMA back to back");
    }
    return 0;
}
