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

// The cosine alone (the NCO, filter.cpp:170): fast_sincos_f's reduction, kernels and bound, only
// the cosine's rounding certified.  Where it returns true *c_out is float(cos(x)), the same float
// fast_sincos_f or the library fallback gives.
FMRX_HD bool fast_cos_f(float xf, float* c_out) {
    const double x = (double)xf;
    if (!(fabs(x) < 1.0e9) || !(fabs(x) > 1.0e-30)) return false;
    const double nd = rint(x * kInvPio2);
    const double r1 = fma(-nd, kPio2Hi, x);
    const double r = fma(-nd, kPio2Lo, r1);
    const double z = r * r;
    const int q = (int)((long long)nd & 3);
    double cv;
    if (q & 1) {
        const double ps = kS2 + z * (kS3 + z * (kS4 + z * (kS5 + z * kS6)));
        const double sn = r + (z * r) * (kS1 + z * ps);
        cv = q == 1 ? -sn : sn;
    } else {
        const double pc = z * (kC1 + z * (kC2 + z * (kC3 + z * (kC4 + z * (kC5 + z * kC6)))));
        const double cs = 1.0 - (0.5 * z - z * pc);
        cv = q == 0 ? cs : -cs;
    }
    return decide_float(cv, 1.5e-15 * fabs(cv) + fabs(nd) * 1.0e-32, c_out);
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

// ---- the PLL step (src/filter.cpp:157-171) ---------------------------------------------
//
// Per sample the reference computes, in float with double libm calls:
//   eI = v fbI;  eQ = v (-fbQ);  e = float(atan2(eQ, eI));
//   integ += Ki e;  phase += Kp e + integ;  trig += 1;
//   x = float(step trig + phase);  fbI = float(cos x);  fbQ = float(sin x).
//
// Representation.  The sincos of x reduces x = r + nd pi/2 (|r| <= pi/4, q = nd mod 4) and
// evaluates cs = cos r, sn = sin r in double; (fbI, fbQ) is the quadrant permutation (with
// signs) of (float(cs), float(sn)), since float rounding commutes with both.  Undoing that
// permutation on the next step's products gives, exactly,
//     (a, b) := i^q (eI + i eQ) = (fl(v fc), fl(v nfs)),   fc = float(cs), nfs = -float(sn),
// and rotating (a, b) by r in double gives (X, Y) = v (1 + O(2^-23), O(2^-23)), so
//     theta = atan2(eQ, eI) = d + pi [v < 0] - x  (mod 2 pi),   d = atan(Y / X) ~ Y / X.
// B = wrap(pi [v < 0] - x) follows from x alone by a Cody-Waite reduction, so theta = d + B
// is one add on the recurrence's dependency chain and the loop carries no quadrant work.
//
// Error of th = d + B (absolute): (cs, sn) angle <= 1.5e-15 (their relative bound), X/Y
// roundings 1e-16, r 1e-16, B's two roundings 4.4e-16, the add 2.2e-16, atan(d) - d <= 1.5e-16
// (|d| < 2^-17), glibc's own <= 1 ulp(pi) 4.4e-16: <= 3.2e-15 < E = 4e-15.  e = float(th) is
// certified when th - E and th + E round to the same float; |B| <= pi - 2^-12 keeps th off
// atan2's branch cut.  sin/cos keep the fdlibm relative bound (the 16-ulp test above).

constexpr double kInv2Pi = 1.59154943091895345608e-01;  // 1 / (2 pi)
constexpr double kPllE = 4.0e-15;                       // absolute error bound of th
constexpr double kPllEBatch = 2.0e-14;                  // ... with d = Y / v (pll_batch_fast)
constexpr double kPllMaxD = 0x1p-17;                    // |d|: atan(d) = d to 1.5e-16
constexpr double kPiHi = 3.14159265358979311600e+00;
constexpr double kPllMaxB = kPiHi - 0x1p-12;            // |B|: off the branch cut
constexpr double kPllMinR = 0x1p-20;                    // |r|: sin r not tiny
constexpr double kPllMaxX = 1.0e9;                      // |x|: reduction exact enough
constexpr float kPllMinV = 0x1p-100f;                   // |v|: products stay normal

struct PllCtx {
    double cs, sn;  // cos r, sin r of the last trigArg x = r + nd pi/2
    double x;       // that trigArg (a float, exact in double)
    int q;          // nd mod 4
    bool valid;     // fields set and |x| < kPllMaxX
};

// wrap(pi [v < 0] - x) into [-pi, pi]: m = rint(x / (2 pi) + [v < 0] / 2), J = 2m - [v < 0]
// (exact), B = J pi - x with the exact product inside each fma.  hneg = 0.5 [v < 0].
FMRX_HD double pll_offset(double x, double hneg) {
    const double m = rint(fma(x, kInv2Pi, hneg));
    const double J = 2.0 * (m - hneg);
    return fma(J, kPiLo, fma(J, kPiHi, -x));
}

// Y / X for |Y / X| < 2^-17 to ~2^-46 relative: one reciprocal and one Newton step on the
// device (a division costs a dozen dependent ops); the host divides.
FMRX_HD double pll_quot(double Y, double X) {
#ifdef __HIP_DEVICE_COMPILE__
    const double y0 = __builtin_amdgcn_rcp(X);
    return Y * fma(y0, fma(-X, y0, 1.0), y0);
#else
    return Y / X;
#endif
}

// fdlibm's sin/cos kernels for |r| <= pi/4 in Estrin form (shorter dependency chain).
FMRX_HD void pll_sincos_kernel(double r, double* sn, double* cs) {
    const double z = r * r, z2 = z * z, z4 = z2 * z2;
    const double ps = fma(z4, fma(z, kS6, kS5), fma(z2, fma(z, kS4, kS3), fma(z, kS2, kS1)));
    *sn = fma(z * r, ps, r);
    const double pc = fma(z4, fma(z, kC6, kC5), fma(z2, fma(z, kC4, kC3), fma(z, kC2, kC1)));
    *cs = 1.0 - (0.5 * z - z2 * pc);
}

// decide_float_16ulp's margin as a number: > 32 iff the float rounding of v is certified
// (the low 29 bits lie more than 16 ulps from the halfway point 2^28).
FMRX_HD uint32_t pll_margin16(double v) {
    return ((uint32_t)__builtin_bit_cast(uint64_t, v) & 0x1FFFFFFFu) - (0x10000000u - 16u);
}

// atan2(eQ, eI) rounded to float, from the context of the previous sincos.  Returns false
// when the rounding cannot be certified (zeros and tiny products, a first step without a
// context, near the branch cut): the caller falls back to the library.
FMRX_HD bool rot_atan2_f(float eQ, float eI, const PllCtx& c, float* out) {
    const float a0 = (c.q & 1) ? -eQ : eI, b0 = (c.q & 1) ? eI : eQ;  // (a, b) = i^q (eI + i eQ)
    const float a = (c.q & 2) ? -a0 : a0, b = (c.q & 2) ? -b0 : b0;
    const double ad = (double)a, bd = (double)b;
    const double X = fma(ad, c.cs, -(bd * c.sn));
    const double Y = fma(ad, c.sn, bd * c.cs);
    const double d = pll_quot(Y, X);
    const double B = pll_offset(c.x, X < 0.0 ? 0.5 : 0.0);
    const double th = d + B;
    const float lo = (float)(th - kPllE), hi = (float)(th + kPllE);
    *out = lo;
    return (int)c.valid & (int)(fabsf(eI) >= kPllMinV) & (int)(fabsf(eQ) >= kPllMinV) &
           (int)(fabs(d) < kPllMaxD) & (int)(fabs(B) <= kPllMaxB) & (int)(lo == hi);
}

// sin/cos of a float argument rounded to float, leaving the context for the next
// rot_atan2_f.  Returns false when the rounding cannot be certified (caller falls back);
// the context is valid whenever |x| < kPllMaxX either way.
FMRX_HD bool sincos_ctx_f(float xf, float* s_out, float* c_out, PllCtx* ctx) {
    const double x = (double)xf;
    const bool in_range = fabs(x) < kPllMaxX;  // rejects inf / nan too
    const double nd = rint(in_range ? x * kInvPio2 : 0.0);
    const double r = fma(-nd, kPio2Lo, fma(-nd, kPio2Hi, x));
    double sn, cs;
    pll_sincos_kernel(r, &sn, &cs);
    const int q = (int)nd & 3;  // |nd| < 6.4e8 fits an int; & 3 is mod 4 for negatives too
    const float fs = (float)sn, fc = (float)cs;
    // cos x = [cs, -sn, -cs, sn][q], sin x = [sn, cs, -sn, -cs][q]
    const float c = (q & 1) ? fs : fc, s = (q & 1) ? fc : fs;
    *c_out = ((q + 1) & 2) ? -c : c;
    *s_out = (q & 2) ? -s : s;
    ctx->cs = cs;
    ctx->sn = sn;
    ctx->x = x;
    ctx->q = q;
    ctx->valid = in_range;
    return (int)in_range & (int)(pll_margin16(sn) > 32u) & (int)(pll_margin16(cs) > 32u) &
           (int)(fabs(r) >= kPllMinR);
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

// ---- per-sample side data of a segment (pll_prep_kernel, parallel over samples) -----------
//
// Everything of a step that depends only on the input and the step index is computed ahead,
// in parallel, so the serial loop keeps only the recurrence:
//   iv_j = 1 / v_j in double -- the quotient Y / X of the rotation atan2 without a reciprocal
//          (below); NaN when |v_j| < kPllMinV or v_j is not finite, so the batch fails its
//          NaN check and is redone exactly;
//   pr_j = step * (double)trig_j, trig_j = the float trigOffset after step j's increment
//          (filter.cpp:165-166).  From an integer-valued t0 in [0, 2^24] the float increments
//          are exact up to 2^24 and then stick there, so trig_j = min(t0 + j + 1, 2^24); any
//          other t0 (reachable only through fmrx_set_state) or |pr_j| >= kPllMaxPr gives NaN.
constexpr double kPllMaxPr = 4.0e8;
constexpr float kPllMaxPhase = 5.0e8f;  // with |pr| < 4e8: |trigArg| < kPllMaxX over a batch
constexpr float kPllMaxInteg = 1.0e6f;
constexpr float kPllTrigStick = 16777216.0f;  // 2^24: trigOffset + 1.0f == trigOffset from here

FMRX_HD bool pll_trig_domain(float t0) {
    return t0 >= 0.0f && t0 <= kPllTrigStick && t0 == floorf(t0);
}

// The state after step k - 1 of a segment (k >= 1 steps in) from what the speculative runner
// records: (integ, phase) as recorded, trigOffset from the segment's integer-valued start t0
// in the trig domain (min(t0 + k, 2^24), as pll_side), and fbI, fbQ -- not recorded -- rounded
// from the exact sin/cos of that step's trigArg a (filter.cpp:166-169), which also leaves the
// context for the next step.
template <class Lib>
FMRX_HD void pll_state_at(PllState& p, PllCtx& ctx, float integ, float phase, float t0, long long k, float a,
                          const Lib& lib) {
    p.integ = integ;
    p.phase = phase;
    p.trig = (float)fmin((double)t0 + (double)k, (double)kPllTrigStick);
    float sv, cv;
    if (!sincos_ctx_f(a, &sv, &cv, &ctx)) lib.sincosf_(a, &sv, &cv);
    p.fbI = cv;
    p.fbQ = sv;
}

FMRX_HD void pll_side(float v, float t0, long long j, double step, double* iv, double* pr) {
    const double vd = (double)v;
    *iv = (fabs(vd) >= (double)kPllMinV && fabs(vd) < 1.0e300) ? 1.0 / vd : (double)NAN;
    const float trig = (float)fmin((double)t0 + (double)(j + 1), (double)kPllTrigStick);
    const double p = step * (double)trig;
    *pr = (pll_trig_domain(t0) && fabs(p) < kPllMaxPr) ? p : (double)NAN;
}

// pll_offset with the half-integer m - hneg times 2 pi: (m - hneg) 2pi_hi is the same exact
// product as J pi_hi inside the fma, so B is bit-identical, one operation shorter.
constexpr double k2PiHi = 2.0 * kPiHi, k2PiLo = 2.0 * kPiLo;
FMRX_HD double pll_offset_h(double x, double hneg) {
    const double mh = rint(fma(x, kInv2Pi, hneg)) - hneg;
    return fma(mh, k2PiLo, fma(mh, k2PiHi, -x));
}

// decide_float_16ulp's margin scaled by 8: (low dword << 3) - (2^31 - 128), one shift-add;
// > 256 iff the float rounding of v is certified.
FMRX_HD uint32_t pll_margin16x8(double v) {
    return ((uint32_t)__builtin_bit_cast(uint64_t, v) << 3) + 0x80000080u;
}

// ---- sin and cos as ONE polynomial per lane (the batch's SPLIT form) -------------------------
//
// sin r = r (1 + z Ps(z)) and cos r = 1 + z (-1/2 + z Pc(z)), z = r^2, with fdlibm's
// coefficients (Ps = S1 + S2 z + ... + S6 z^5, Pc = C1 + ... + C6 z^5), are the same seven-
// coefficient Estrin evaluation Q(z) followed by w = 1 + z Q: sin lanes use q = (S1..S6, 0) and
// take r w, cos lanes q = (-1/2, C1..C6) and take w.  On the device the even lanes of each
// 16-lane row evaluate sin and the odd lanes cos with the SAME instructions, and two row
// broadcasts (DPP row_newbcast: lane 0 = sin, lane 1 = cos) hand both to every lane of the row
// -- five instructions fewer than evaluating both.  Error: Estrin ~1 ulp of Q, the fma and the
// product 1/2 ulp each: <= 2.5 ulp relative (the 16-ulp margin test assumes <= 13.5).
struct SplitCoef {
    double q[7];
};
FMRX_HD SplitCoef split_coef(bool cos_lane) {
    SplitCoef c;
    const double s[7] = {kS1, kS2, kS3, kS4, kS5, kS6, 0.0};
    const double k[7] = {-0.5, kC1, kC2, kC3, kC4, kC5, kC6};
    for (int i = 0; i < 7; i++) c.q[i] = cos_lane ? k[i] : s[i];
    return c;
}
FMRX_HD double split_w(double z, double z2, double z4, const SplitCoef& c) {
    const double p01 = fma(z, c.q[1], c.q[0]), p23 = fma(z, c.q[3], c.q[2]), p45 = fma(z, c.q[5], c.q[4]);
    const double Q = fma(z4, fma(z2, c.q[6], p45), fma(z2, p23, p01));
    return fma(z, Q, 1.0);
}
// Horner instead of Estrin: two multiplies fewer (z2, z4), a longer dependency chain -- for the
// speculative runner, which is issue-bound, not latency-bound.  Same class of error.
FMRX_HD double split_w_horner(double z, const SplitCoef& c) {
    double Q = fma(z, c.q[6], c.q[5]);
    Q = fma(z, Q, c.q[4]);
    Q = fma(z, Q, c.q[3]);
    Q = fma(z, Q, c.q[2]);
    Q = fma(z, Q, c.q[1]);
    Q = fma(z, Q, c.q[0]);
    return fma(z, Q, 1.0);
}
// sin r, cos r in the split form: on the device lane_coef belongs to this lane (sin or cos by
// lane parity) and the row broadcasts gather both; on the host both are evaluated.
template <bool HORNER = false>
FMRX_HD void pll_sincos_split(double r, const SplitCoef& lane_coef, double* sn, double* cs) {
    const double z = r * r;
    if constexpr (HORNER) {
#ifdef __HIP_DEVICE_COMPILE__
        const double w = split_w_horner(z, lane_coef);
        const double rw = r * w;
        const long long rw_bits = __builtin_bit_cast(long long, rw), w_bits = __builtin_bit_cast(long long, w);
        *sn = __builtin_bit_cast(double, (long long)__builtin_amdgcn_mov_dpp(rw_bits, 0x150, 0xF, 0xF, false));
        *cs = __builtin_bit_cast(double, (long long)__builtin_amdgcn_mov_dpp(w_bits, 0x151, 0xF, 0xF, false));
#else
        (void)lane_coef;
        *sn = r * split_w_horner(z, split_coef(false));
        *cs = split_w_horner(z, split_coef(true));
#endif
        return;
    }
    const double z2 = z * z, z4 = z2 * z2;
#ifdef __HIP_DEVICE_COMPILE__
    const double w = split_w(z, z2, z4, lane_coef);
    const double rw = r * w;
    const long long rw_bits = __builtin_bit_cast(long long, rw), w_bits = __builtin_bit_cast(long long, w);
    // every lane of a row reads lane 0 / lane 1 of its row, so no lane keeps an old value
    const long long sn_bits = __builtin_amdgcn_mov_dpp(rw_bits, 0x150, 0xF, 0xF, false);  // row_newbcast:0
    const long long cs_bits = __builtin_amdgcn_mov_dpp(w_bits, 0x151, 0xF, 0xF, false);   // row_newbcast:1
    *sn = __builtin_bit_cast(double, sn_bits);
    *cs = __builtin_bit_cast(double, cs_bits);
#else
    (void)lane_coef;
    *sn = r * split_w(z, z2, z4, split_coef(false));
    *cs = split_w(z, z2, z4, split_coef(true));
#endif
}

// N steps straight-line on the certified fast paths, with no branch and no quadrant work
// (the representation above): the loop carries (fc, nfs, cs, sn, B) and folds every
// certification into a few accumulators checked once at the end.  Returns true when every
// step was certified -- the outputs and (p, ctx) then equal N pll_step calls bit for bit.
// Otherwise p and ctx are garbage: the caller restores them and redoes the N steps with
// pll_step.  NaN anywhere reaches the phase accumulator or the last trigArg and fails the
// final check.
//
// The quotient without X: d = Y iv, iv = (1/v)(1 + eta) from the pre-pass.  With
// a = fl(v fc), b = fl(v nfs) and fc, fs the floats of (cs, sn) (or glibc's, within an ulp),
// X / v = cs^2 (1 + e_c + e_a) + sn^2 (1 + e_s + e_b) = 1 + delta, |delta| <= 2^-23, and
// |Y / v| = |cs sn (e_c + e_a - e_s - e_b)| <= 2^-23, so |d| <= 2^-23 and
// |Y iv - Y / X| <= |Y / v| (|delta| + |eta|) <= 2^-46 < 1.5e-14.  The batch's bound is E
// (kPllE, the rotation's own budget) plus that term: kPllEBatch = 2e-14.  The wider interval
// leaves about one step in 10^5 uncertified (redone exactly), and saves X, its product and the
// correction of a full quotient -- three operations on the serial chain.
// The half turn of pll_offset for step j is 0.5 [v_j < 0] = 0.5 [iv_j < 0] (a NaN iv fails the
// batch anyway).  refill(j) runs after step j, once the step has consumed v[j], iv[j] (and
// iv[j + 1]'s sign) and pr[j]: the kernel reloads the next batch into the same registers from
// there (one register set, the loads in flight for a whole batch).
//
// SPLIT: sin/cos in the split form (pll_sincos_split; the device caller must run every lane of
// a 16-lane row on the same stream, lane parity choosing `sc`).
//
// SPEC (the speculative runner, pll_spec_kernel): no certification at all -- e is the float
// rounding of th and nothing is accumulated; the result is right unless a rounding went the
// wrong way, which pll_check_kernel detects afterwards by recomputing every batch exactly.
template <int N, bool SPLIT = false, bool SPEC = false, class Refill>
FMRX_HD bool pll_batch_fast(PllState& p, PllCtx& ctx, const float (&v)[N], const double (&iv)[N],
                            const double (&pr)[N], float (&out)[N], float Ki, float Kp, Refill&& refill,
                            const SplitCoef& sc = SplitCoef{}, const double* hh = nullptr) {
    // hh (SPEC): the half turns 0.5 [v_j < 0] from the pre-pass, instead of a compare and a
    // select per step
    auto half = [&](int j) -> double {
        if constexpr (SPEC) return hh[j];
        return iv[j] < 0.0 ? 0.5 : 0.0;
    };
    // undo the quadrant permutation: fc = [fbI, fbQ, -fbI, -fbQ][q], nfs = [-fbQ, fbI, fbQ, -fbI][q]
    const int q0 = ctx.q;
    const float u0 = (q0 & 1) ? p.fbQ : p.fbI, w0 = (q0 & 1) ? p.fbI : -p.fbQ;
    float fc = (q0 & 2) ? -u0 : u0, nfs = (q0 & 2) ? -w0 : w0;
    double cs = ctx.cs, sn = ctx.sn, x = ctx.x, nd = 0.0;
    double B = pll_offset_h(x, half(0));
    uint32_t acc_u = 0xFFFFFFFFu, acc_e = 0u;
    double acc_d = 0.0, acc_B = fabs(B), acc_r = 1.0;
    const bool range_ok = fabsf(p.phase) < kPllMaxPhase && fabsf(p.integ) < kPllMaxInteg;
#ifdef __HIPCC__
#pragma unroll
#endif
    for (int j = 0; j < N; j++) {
#ifdef __HIP_DEVICE_COMPILE__
        const float2v ab = float2v{fc, nfs} * v[j];  // one v_pk_mul_f32
        const float a = ab.x, b = ab.y;
#else
        const float a = v[j] * fc, b = v[j] * nfs;
#endif
        const double ad = (double)a, bd = (double)b;
        const double Y = fma(ad, sn, bd * cs);
        float e;
        if constexpr (SPEC) {
            e = (float)fma(Y, iv[j], B);  // one rounding fewer than d + B: no less accurate
        } else {
            const double d = Y * iv[j];
            const double th = d + B;
            const float lo = (float)(th - kPllEBatch), hi = (float)(th + kPllEBatch);
            acc_e |= __builtin_bit_cast(uint32_t, lo) ^ __builtin_bit_cast(uint32_t, hi);
            acc_d = fmax(acc_d, fabs(d));
            e = lo;
        }
#ifdef __HIP_DEVICE_COMPILE__
        const float2v ke = float2v{Ki, Kp} * e;  // one v_pk_mul_f32
        const float ki_e = ke.x, kp_e = ke.y;
#else
        const float ki_e = Ki * e, kp_e = Kp * e;
#endif
        p.integ = p.integ + ki_e;
        p.phase = p.phase + (kp_e + p.integ);
        const float arg = (float)(pr[j] + (double)p.phase);
        out[j] = arg;
        x = (double)arg;
        nd = rint(x * kInvPio2);
        const double r = fma(-nd, kPio2Lo, fma(-nd, kPio2Hi, x));
        if constexpr (!SPEC) acc_r = fmin(acc_r, fabs(r));
        if constexpr (SPLIT)
            pll_sincos_split<SPEC>(r, sc, &sn, &cs);
        else
            pll_sincos_kernel(r, &sn, &cs);
        fc = (float)cs;
        nfs = -(float)sn;
        if constexpr (!SPEC) {
            const uint32_t mc = pll_margin16x8(cs), ms = pll_margin16x8(sn);
            acc_u = acc_u < mc ? acc_u : mc;
            acc_u = acc_u < ms ? acc_u : ms;
        }
        if (j + 1 < N) {
            B = pll_offset_h(x, half(j + 1));
            if constexpr (!SPEC) acc_B = fmax(acc_B, fabs(B));
        }
        refill(j);
    }
    // trigOffset after N float increments from an integer-valued trig in [0, 2^24] (the only
    // case whose pr is not NaN)
    p.trig = fminf(p.trig + (float)N, kPllTrigStick);
    // the quadrant permutation back: fbI = [fc, nfs, -fc, -nfs][q], fbQ = [-nfs, fc, nfs, -fc][q]
    const int q = (int)nd & 3;
    const float c1 = (q & 1) ? nfs : fc, s1 = (q & 1) ? fc : -nfs;
    p.fbI = (q & 2) ? -c1 : c1;
    p.fbQ = (q & 2) ? -s1 : s1;
    const bool valid0 = ctx.valid;
    ctx.cs = cs;
    ctx.sn = sn;
    ctx.x = x;
    ctx.q = q;
    ctx.valid = true;
    if constexpr (SPEC) return true;
    return (int)valid0 & (int)range_ok & (int)(acc_u > 256u) & (int)(acc_e == 0u) &
           (int)(acc_d < kPllMaxD) & (int)(acc_B <= kPllMaxB) & (int)(acc_r >= kPllMinR) &
           (int)(p.phase == p.phase) & (int)(x == x);
}

}  // namespace fmrx
