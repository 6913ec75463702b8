// tools/ubench_wgsimd.hip — where do the waves of a multi-wave workgroup land?  Each wave writes
// its HW_ID register (wave id, SIMD id, CU id, SE id) for workgroups of 2 and 4 waves, few and
// many workgroups: pll_pred.hip runs its serial chain and its evaluator as two waves of one
// workgroup and wants them on different SIMDs.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/ubench_wgsimd tools/ubench_wgsimd.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void where(unsigned* out, unsigned* xcc) {
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));     // HW_ID
    const unsigned xc = __builtin_amdgcn_s_getreg(20 | (31 << 11));    // XCC_ID
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        out[blockIdx.x * (blockDim.x >> 6) + w] = hw;
        xcc[blockIdx.x * (blockDim.x >> 6) + w] = xc;
    }
    // keep the waves resident together for a while
    long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < 20000) {
    }
}

int main() {
    for (int waves : {2, 4}) {
        for (int groups : {1, 8, 256, 1024}) {
            const int n = waves * groups;
            unsigned *d, *dx;
            hipMalloc(&d, n * 4);
            hipMalloc(&dx, n * 4);
            hipLaunchKernelGGL(where, dim3(groups), dim3(64 * waves), 0, 0, d, dx);
            std::vector<unsigned> h(n), hx(n);
            hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
            hipMemcpy(hx.data(), dx, n * 4, hipMemcpyDeviceToHost);
            // HW_ID (gfx9): wave_id [3:0], simd_id [5:4], pipe [7:6], cu_id [11:8], sh_id [12], se_id [15:13]
            int same_simd = 0;
            for (int g = 0; g < groups; g++) {
                const unsigned a = h[g * waves], b = h[g * waves + 1];
                if (((a >> 4) & 3) == ((b >> 4) & 3) && ((a >> 8) & 15) == ((b >> 8) & 15)) same_simd++;
            }
            std::printf("waves/group %d groups %4d: wave 0 and 1 on the same SIMD in %d of %d groups;", waves, groups,
                        same_simd, groups);
            std::printf(" group 0:");
            for (int w = 0; w < waves; w++)
                std::printf(" [xcc %u se %u cu %u simd %u]", hx[w], (h[w] >> 13) & 7, (h[w] >> 8) & 15,
                            (h[w] >> 4) & 3);
            std::printf("\n");
            hipFree(d);
            hipFree(dx);
        }
    }
    return 0;
}
