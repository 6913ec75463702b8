// dsp_device.h — scalar arithmetic of the reference, restated for device (and host) code
// with the exact float/double promotions of src/filter.cpp and src/project.cpp.
// Every caller is compiled with -ffp-contract=off: no FMA may replace a mul+add pair.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fmrx {

typedef float float2v __attribute__((ext_vector_type(2)));

// src/iofunc.cpp:67: ((float)u - 128.0) / 128.0 in double, which is exactly u/128 - 1.
// fma(u, 2^-7, -1) is exact (u*2^-7 is exact and u/128 - 1 is representable).
__host__ __device__ inline float u8_to_sample(uint32_t u) {
    return __builtin_fmaf(static_cast<float>(u), 0.0078125f, -1.0f);
}

// src/filter.cpp:110-127, one sample of FMDemod.  The denominator is std::pow(float, 2)
// summed in double then rounded to float; the quotient is an IEEE float division.
// A float squared is exact in double (48 significant bits), so the reference's rounded sum
// of the two squares is one fma of the second square onto the first: the same single
// rounding, one instruction fewer.
__host__ __device__ inline float fm_demod_one(float ci, float cq, float pi, float pq) {
    const float di = ci - pi;
    const float dq = cq - pq;
    const double cid = static_cast<double>(ci), cqd = static_cast<double>(cq);
    const float den = static_cast<float>(__builtin_fma(cqd, cqd, cid * cid));
    // The quotient is formed unconditionally and selected (no divergent branch on device);
    // den == 0 gives 0 exactly as filter.cpp:125-129.
    const float num = (ci * dq) - (cq * di);
    const float q = num / den;
    return den != 0.0f ? q : 0.0f;
}

// src/project.cpp:185-191: NaN -> 0, else static_cast<short>(x * 16384) as the x86-64 build
// of the reference executes it (cvttss2si: out-of-range/inf -> INT32_MIN; then the low 16
// bits are stored).  AMDGPU's v_cvt_i32_f32 saturates instead, so the range test is explicit.
__host__ __device__ inline int16_t quantize_s16(float x) {
    if (x != x) return 0;
    const float v = x * 16384.0f;
    int32_t t;
    if (!(v < 2147483648.0f) || v < -2147483648.0f)
        t = static_cast<int32_t>(0x80000000u);
    else
        t = static_cast<int32_t>(v);
    return static_cast<int16_t>(static_cast<uint16_t>(static_cast<uint32_t>(t) & 0xFFFFu));
}

// src/filter.cpp:196-197: (mono +/- stereo) * 0.5 where 0.5 is a double literal.
__host__ __device__ inline float half_of(float s) {
    return static_cast<float>(static_cast<double>(s) * 0.5);
}

}  // namespace fmrx
