// pll_math.h — float-result sin/cos/atan2 for the PLL recurrence (src/filter.cpp:161-169).
//
// The reference evaluates double libm calls on float arguments and rounds the results to
// float.  The PLL feeds those floats back into itself, so every single result must equal
// float(glibc(x)).  These routines evaluate in double with short fdlibm-style kernels (one
// Cody-Waite reduction with FMA, degree-13/14 sin/cos polynomials, fdlibm's atan reduction)
// and then PROVE the float rounding: if the result interval [r - E, r + E] (E = a bound on
// the evaluation error plus glibc's own <= 1 ulp) rounds to one float, that float is
// float(f(x)) for every double within the interval -- in particular glibc's.  Otherwise the
// caller falls back to the full-precision library call (probability ~1e-7 per call).
//
// Plain C++ so the same code also builds on the host, where tests/test_pll_math.py checks
// the fast path against glibc over hundreds of millions of arguments.
#pragma once

#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#define FMRX_HD __host__ __device__ inline
#else
#define FMRX_HD inline
#endif

namespace fmrx {

// fdlibm __kernel_sin / __kernel_cos minimax coefficients (|r| <= pi/4)
constexpr double kS1 = -1.66666666666666324348e-01, kS2 = 8.33333333332248946124e-03,
                 kS3 = -1.98412698298579493134e-04, kS4 = 2.75573137070700676789e-06,
                 kS5 = -2.50507602534068634195e-08, kS6 = 1.58969099521155010221e-10;
constexpr double kC1 = 4.16666666666666019037e-02, kC2 = -1.38888888888741095749e-03,
                 kC3 = 2.48015872894767294178e-05, kC4 = -2.75573143513906633035e-07,
                 kC5 = 2.08757232129817482790e-09, kC6 = -1.13596475577881948265e-11;
// pi/2 = kPio2Hi + kPio2Lo (+ ~1e-33)
constexpr double kPio2Hi = 1.57079632679489655800e+00, kPio2Lo = 6.12323399573676603587e-17;
constexpr double kInvPio2 = 6.36619772367581382433e-01;

// |float(x) - x| rounding-ambiguity test: true iff every double in [r - e, r + e] rounds to
// the same float, which is then returned in *out.
FMRX_HD bool decide_float(double r, double e, float* out) {
    const float lo = (float)(r - e), hi = (float)(r + e);
    *out = (float)r;
    return lo == hi;
}

// sin and cos of a float argument, results rounded to float.  Returns false when the fast
// path cannot certify the rounding (caller falls back).
FMRX_HD bool fast_sincos_f(float xf, float* s_out, float* c_out) {
    const double x = (double)xf;
    // zeros (signed-zero results), tiny, huge, inf, nan: library path
    if (!(fabs(x) < 1.0e9) || !(fabs(x) > 1.0e-30)) return false;
    const double nd = rint(x * kInvPio2);
    // Cody-Waite with FMA: x - n*pio2 exactly to ~2^-100 relative of n*pio2 (n < 2^30)
    const double r1 = fma(-nd, kPio2Hi, x);
    const double r = fma(-nd, kPio2Lo, r1);
    const double z = r * r;
    const double ps = kS2 + z * (kS3 + z * (kS4 + z * (kS5 + z * kS6)));
    const double sn = r + (z * r) * (kS1 + z * ps);
    const double pc = z * (kC1 + z * (kC2 + z * (kC3 + z * (kC4 + z * (kC5 + z * kC6)))));
    const double cs = 1.0 - (0.5 * z - z * pc);
    const int q = (int)((long long)nd & 3);
    double sv, cv;
    switch (q) {
        case 0: sv = sn; cv = cs; break;
        case 1: sv = cs; cv = -sn; break;
        case 2: sv = -sn; cv = -cs; break;
        default: sv = -cs; cv = sn; break;
    }
    // Error bound, relative to the result: the two FMA reductions round relative to |r|
    // (|r| <= 1.6 |sin r|, |cos r| >= 0.7), the kernels are within a few ulp, glibc within
    // 1 ulp, plus n * 2^-106-ish absolute from the truncated pi/2: ~7 ulp total, E = 1.5e-15.
    const double ea = fabs(nd) * 1.0e-32;
    const bool s_ok = decide_float(sv, 1.5e-15 * fabs(sv) + ea, s_out);
    const bool c_ok = decide_float(cv, 1.5e-15 * fabs(cv) + ea, c_out);
    return s_ok && c_ok;
}

// fdlibm s_atan.c coefficients and breakpoints
constexpr double kAtanHi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                               9.82793723247329054082e-01, 1.57079632679489655800e+00};
constexpr double kAtanLo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                               1.39033110312309984516e-17, 6.12323399573676603587e-17};
constexpr double kAT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                            1.42857142725034663711e-01, -1.11111104054623557880e-01,
                            9.09088713343650656196e-02, -7.69187620504482999495e-02,
                            6.66107313738753120669e-02, -5.83357013379057348645e-02,
                            4.97687799461593236017e-02, -3.65315727442169155270e-02,
                            1.62858201153657823623e-02};
constexpr double kPi = 3.14159265358979311600e+00, kPiLo = 1.2246467991473531772e-16;

// atan(t) for t in [0, 1] (fdlibm reduction, ids 0..1 only).
FMRX_HD double atan01(double t) {
    int id;
    double x;
    if (t < 0.4375) {
        id = -1;
        x = t;
    } else if (t < 0.6875) {
        id = 0;
        x = (2.0 * t - 1.0) / (2.0 + t);
    } else {
        id = 1;
        x = (t - 1.0) / (t + 1.0);
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (kAT[0] + w * (kAT[2] + w * (kAT[4] + w * (kAT[6] + w * (kAT[8] + w * kAT[10])))));
    const double s2 = w * (kAT[1] + w * (kAT[3] + w * (kAT[5] + w * (kAT[7] + w * kAT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    return kAtanHi[id] - ((x * (s1 + s2) - kAtanLo[id]) - x);
}

// atan2(y, x) of float arguments, result rounded to float.  Zeros, infinities and NaNs (the
// signed-zero rules of C99 atan2) always take the library path.
FMRX_HD bool fast_atan2_f(float yf, float xf, float* out) {
    const double y = (double)yf, x = (double)xf;
    const double ay = fabs(y), ax = fabs(x);
    if (!(ay > 0.0 && ax > 0.0) || !(ay < 1.0e300 && ax < 1.0e300)) return false;
    const bool swap = ay > ax;
    const double t = swap ? ax / ay : ay / ax;  // in (0, 1]
    double a = atan01(t);
    if (swap) a = (kPio2Hi - a) + kPio2Lo;
    if (x < 0.0) a = (kPi - a) + kPiLo;
    if (y < 0.0) a = -a;
    // Relative bound: division 0.5 ulp of t (atan(t)/t <= 1 keeps it relative), reduction +
    // kernel ~2 ulp, the pi/2 and pi reflections (results >= pi/4) ~2 ulp, glibc <= 1 ulp.
    return decide_float(a, 3.0e-15 * fabs(a), out);
}

}  // namespace fmrx
