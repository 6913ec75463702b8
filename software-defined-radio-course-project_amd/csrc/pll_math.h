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

// Integer form of the same test for a value known to |v| (1 + 13.5 ulp): the float rounding
// drops the low 29 bits of the double; it is unambiguous unless those bits lie within 16 ulps
// of the halfway point 2^28.  (A bound crossing a float exactly or a binade edge still rounds
// to the same float, so only the halfway point matters.)  3 integer ops instead of ~8.
FMRX_HD bool decide_float_16ulp(double v, float* out) {
    *out = (float)v;
    const uint32_t t = (uint32_t)__builtin_bit_cast(uint64_t, v) & 0x1FFFFFFFu;
    return t - (0x10000000u - 16u) > 32u;
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

// ---- the PLL step (src/filter.cpp:157-171) with a short dependency chain ----------------
//
// The phase error e = atan2(eQ, eI) with (eI, eQ) = v * (fbI, -fbQ), fbI/fbQ = float(cos/sin
// of the previous trigArg phi).  The previous step's sincos left cos(phi), sin(phi) in DOUBLE
// (C, S) and phi's reduction phi = r + q*pi/2 (mod 2 pi).  Rotating (eI, eQ) by +phi gives
// (X, Y) with angle theta + phi = a tiny residual d (float roundings only, |d| < 1e-6) or
// pi + d when v < 0, hence  theta = atan(Y/X) + [X<0] pi - r - q pi/2  (mod 2 pi),  with
// atan(Y/X) = Y/X to 1e-18 at that size.  Absolute error budget: (C, S) angle 1.5e-15,
// rotation 3e-16, r 1e-16, constants 2e-16, glibc 1 ulp(pi) 4.4e-16 -> E = 4e-15, certified
// by decide_float like the kernels above; anything else takes the generic path.

struct PllCtx {
    double C, S, r;  // cos/sin(phi) and phi's reduced argument from the last sincos
    int q;           // phi's quadrant, phi = r + q*pi/2 (mod 2 pi)
    bool valid;
};

constexpr double kPiHi = 3.14159265358979311600e+00;

FMRX_HD bool rot_atan2_f(float eQ, float eI, const PllCtx& c, float* out) {
    // Branch-free: every test folds into one predicate (the PLL runs one lane per stream,
    // where each taken-or-not branch costs as much as several arithmetic ops).
    const double ei = (double)eI, eq = (double)eQ;
    const double X = fma(ei, c.C, -(eq * c.S));
    const double Y = fma(ei, c.S, eq * c.C);
    // 1/X: hardware reciprocal estimate + one Newton step (relative error ~2^-52; |d| < 1e-4
    // makes its contribution < 1e-20 absolute)
#ifdef __HIP_DEVICE_COMPILE__
    const double y0 = __builtin_amdgcn_rcp(X);
#else
    const double y0 = 1.0 / X;
#endif
    const double y1 = fma(y0, fma(-X, y0, 1.0), y0);
    const double d = Y * y1;
    const int k = ((X < 0.0 ? 2 : 0) - c.q) & 3;
    const double kd = (double)k;
    const double t0 = fma(kd, kPio2Lo, fma(kd, kPio2Hi, d - c.r));
    const double th = t0 > kPiHi ? (t0 - 2.0 * kPiHi) - 2.0 * kPiLo : t0;
    const float lo = (float)(th - 4.0e-15), hi = (float)(th + 4.0e-15);
    *out = (float)th;
    // zeros (C99 signed-zero rules), residual too large, too close to the +-pi cut, or an
    // uncertified rounding: generic path
    return (int)c.valid & (int)(eI != 0.0f) & (int)(eQ != 0.0f) & (int)(fabs(d) < 1.0e-4) &
           (int)(fabs(fabs(th) - kPiHi) > 1.0e-9) & (int)(lo == hi);
}

// sin/cos of a float argument with the context for the next rot_atan2_f.
FMRX_HD bool sincos_ctx_f(float xf, float* s_out, float* c_out, PllCtx* ctx) {
    const double x = (double)xf;
    const bool in_range = (int)(fabs(x) < 1.0e9) & (int)(fabs(x) > 1.0e-30);  // rejects inf/nan/0
    const double nd = rint(in_range ? x * kInvPio2 : 0.0);
    const double r1 = fma(-nd, kPio2Hi, x);
    const double r = fma(-nd, kPio2Lo, r1);
    const double z = r * r, z2 = z * z, z4 = z2 * z2;
    // same fdlibm kernels in Estrin form (shorter dependency chain)
    const double ps = fma(z4, fma(z, kS6, kS5), fma(z2, fma(z, kS4, kS3), fma(z, kS2, kS1)));
    const double sn = fma(z * r, ps, r);
    const double pc = fma(z4, fma(z, kC6, kC5), fma(z2, fma(z, kC4, kC3), fma(z, kC2, kC1)));
    const double cs = 1.0 - (0.5 * z - (z * z) * pc);
    const int q = (int)nd & 3;  // |nd| < 6.4e8 fits an int; & 3 is mod 4 for negatives too
    const double sv = (q & 1) ? cs : sn, cv0 = (q & 1) ? sn : cs;
    // quadrant signs as sign-bit flips (q & 2 for sin, (q + 1) & 2 for cos)
    const double s2 = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, sv) ^ ((uint64_t)(q & 2) << 62));
    const double c2 =
        __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, cv0) ^ ((uint64_t)((q + 1) & 2) << 62));
    // Certified rounding: relative error <= 1.5e-15 (13.5 ulp), and the absolute reduction
    // term |nd| 1e-32 stays below 0.03 ulp for |v| >= 2^-20 -> a 16-ulp window; smaller
    // results (probability ~1e-6 per call) take the library path.
    const bool s_ok = (int)decide_float_16ulp(s2, s_out) & (int)(fabs(s2) >= 0x1p-20);
    const bool c_ok = (int)decide_float_16ulp(c2, c_out) & (int)(fabs(c2) >= 0x1p-20);
    // (C, S, r, q) are within the bounds rot_atan2_f assumes whether or not the float
    // rounding could be certified here, so the context is valid either way.
    ctx->C = c2;
    ctx->S = s2;
    ctx->r = r;
    ctx->q = q;
    ctx->valid = in_range;
    return (int)in_range & (int)s_ok & (int)c_ok;
}

struct PllState {
    float integ, phase, fbI, fbQ, trig;
};

// One PLL iteration; returns trigArg (the NCO is cos(trigArg * ncoScale + phaseAdjust)).
// Lib supplies the out-of-line paths: atan2f_(y, x) (fast_atan2_f, then the library) and
// sincosf_(a, &s, &c) (the library).
template <class Lib>
FMRX_HD float pll_step(PllState& p, PllCtx& ctx, float v, float Ki, float Kp, double step,
                       const Lib& lib) {
    const float eI = v * p.fbI;
    const float eQ = v * (-p.fbQ);
    float e;
    if (!rot_atan2_f(eQ, eI, ctx, &e)) e = lib.atan2f_(eQ, eI);  // generic certified path
    p.integ = p.integ + Ki * e;
    p.phase = p.phase + ((Kp * e) + p.integ);
    p.trig = p.trig + 1.0f;
    const double prod = step * (double)p.trig;
    const float arg = (float)(prod + (double)p.phase);
    float sv, cv;
    if (!sincos_ctx_f(arg, &sv, &cv, &ctx)) lib.sincosf_(arg, &sv, &cv);
    p.fbI = cv;
    p.fbQ = sv;
    return arg;
}

// The same step on the certified fast paths only: no library fallback, no branch.  Every
// certification flag is ANDed into `ok`; when it ends false the step's results (and those of
// any later step computed from them) are not to be used -- the caller restores the state and
// redoes the steps with pll_step.  When `ok` stays true the results equal pll_step's exactly
// (the same arithmetic), so a straight-line run of many steps can be validated at once.
FMRX_HD float pll_step_fast(PllState& p, PllCtx& ctx, float v, float Ki, float Kp, double step, int& ok) {
    const float eI = v * p.fbI;
    const float eQ = v * (-p.fbQ);
    float e;
    ok &= (int)rot_atan2_f(eQ, eI, ctx, &e);
    p.integ = p.integ + Ki * e;
    p.phase = p.phase + ((Kp * e) + p.integ);
    p.trig = p.trig + 1.0f;
    const double prod = step * (double)p.trig;
    const float arg = (float)(prod + (double)p.phase);
    float sv, cv;
    ok &= (int)sincos_ctx_f(arg, &sv, &cv, &ctx);
    p.fbI = cv;
    p.fbQ = sv;
    return arg;
}

}  // namespace fmrx
