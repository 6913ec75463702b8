// pll_cr.h — the PLL's fallback libm: float(sin), float(cos), float(atan2) of float arguments
// as the reference computes them (src/filter.cpp:161,168-170: glibc's DOUBLE sin/cos/atan2 of
// the float argument, rounded to float).
//
// pll_math.h's fast paths certify their float rounding and refuse ~1e-7 of arguments, exactly
// the ones whose value lies close to a float rounding boundary.  On those the float result
// depends on glibc's last double bit, so "some accurate double libm" is not enough: the
// fallback must land on the same side of the boundary as glibc.  glibc 2.35 computes these
// functions internally to far more than double precision and returns that value rounded to
// double (its slow paths were removed, leaving errors below ~0.55 ulp that only matter when the
// exact value is within a hair of a DOUBLE rounding boundary).  So the fallback here evaluates
// the exact value in double-double (~2^-100 relative), rounds it to the nearest double h (the
// correctly rounded double libm result), then to float -- float(glibc) wherever glibc returns
// the correctly rounded double.  tools/check_pll_cr.cpp compares this code with glibc on EVERY
// float argument |x| in [2^-19, 2^30) that any fast path can refuse (2.3 M of them): 0
// mismatches, so no exception table is needed.  atan2 is checked on 4e9 random and PLL-shaped
// pairs (a sample of its 2-D domain, not an enumeration): 0 mismatches.
//
// Only IEEE basic operations and fma (no libm, no approximate reciprocals): the host build and
// the gfx950 build round identically (-ffp-contract=off), so the host sweep pins the device.
// Domain: sin/cos |x| < 2^31 (four-part Cody-Waite; beyond, the caller's library call -- no
// PLL state reaches it: |trigArg| < 1e9 wherever pr is finite); atan2 all floats.
#pragma once

#include <math.h>
#include <stdint.h>

#include "pll_cr_consts.h"

#ifdef __HIPCC__
#define FMRX_CR __host__ __device__ inline
#else
#define FMRX_CR inline
#endif

namespace fmrx {
namespace cr {

struct dd {
    double h, l;
};

FMRX_CR dd two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return dd{s, (a - (s - bb)) + (b - bb)};
}
FMRX_CR dd fast_two_sum(double a, double b) {  // |a| >= |b| (or a == 0)
    const double s = a + b;
    return dd{s, b - (s - a)};
}
FMRX_CR dd two_prod(double a, double b) {
    const double p = a * b;
    return dd{p, fma(a, b, -p)};
}
// accurate double-double sum (both components added exactly)
FMRX_CR dd add(dd x, dd y) {
    dd s = two_sum(x.h, y.h);
    const dd t = two_sum(x.l, y.l);
    s.l += t.h;
    s = fast_two_sum(s.h, s.l);
    s.l += t.l;
    return fast_two_sum(s.h, s.l);
}
FMRX_CR dd neg(dd x) { return dd{-x.h, -x.l}; }
FMRX_CR dd mul(dd x, dd y) {
    dd p = two_prod(x.h, y.h);
    p.l += x.h * y.l + x.l * y.h;
    return fast_two_sum(p.h, p.l);
}
FMRX_CR dd mul_d(dd x, double y) {
    dd p = two_prod(x.h, y);
    p.l += x.l * y;
    return fast_two_sum(p.h, p.l);
}
// x / y: first quotient, exact remainder by fma, correction quotient, one refinement
FMRX_CR dd div(dd x, dd y) {
    const double q1 = x.h / y.h;
    dd r = add(x, neg(mul_d(y, q1)));
    const double q2 = r.h / y.h;
    r = add(r, neg(mul_d(y, q2)));
    const double q3 = r.h / y.h;
    const dd q = fast_two_sum(q1, q2);
    return add(q, dd{q3, 0.0});
}
FMRX_CR dd k(const double (&c)[2]) { return dd{c[0], c[1]}; }

// r = x - n pi/2 as a double-double, x a float (exact in double), n integer, |n| < 2^31:
// every product n * kPi exact by two_prod, the sum accumulated in double-double.
FMRX_CR dd reduce(double x, double n) {
    const dd p0 = two_prod(n, kP0);
    dd r = two_sum(x, -p0.h);  // exact: x and n*kP0 within a factor 2 (or n == 0)
    r = add(r, dd{-p0.l, 0.0});
    r = add(r, neg(two_prod(n, kP1)));
    r = add(r, neg(two_prod(n, kP2)));
    r = add(r, dd{-(n * kP3), 0.0});
    return r;
}

// sin r and cos r for |r| <= ~pi/4 + 2^-20: Taylor series in double-double (terms to 1/27!,
// 1/28!: truncation < 2^-102 relative), Horner on z = r^2.
FMRX_CR void sincos_dd(dd r, dd* s, dd* c) {
    const dd z = mul(r, r);
    dd ps = k(kInvFact[27]);
    for (int n = 25; n >= 1; n -= 2) {  // sin r / r = sum (-1)^m z^m / (2m+1)!
        ps = mul(ps, z);
        ps = add(k(kInvFact[n]), neg(ps));
    }
    *s = mul(ps, r);
    dd pc = k(kInvFact[28]);
    for (int n = 26; n >= 0; n -= 2) {  // cos r = sum (-1)^m z^m / (2m)!
        pc = mul(pc, z);
        pc = add(k(kInvFact[n]), neg(pc));
    }
    *c = pc;
}

// sincos_f's domain (the four-part reduction): |x| < 2^31.
FMRX_CR bool sincos_domain(float x) { return fabsf(x) < 0x1p31f; }

// float(RN_double(sin x)), float(RN_double(cos x)) for a float x, |x| < 2^31.
FMRX_CR void sincos_f(float xf, float* s_out, float* c_out) {
    const double x = (double)xf;
    if (x == 0.0) {  // sin(+-0) = +-0, cos = 1
        *s_out = xf;
        *c_out = 1.0f;
        return;
    }
    const double n = rint(x * kTwoOverPi);
    const dd r = reduce(x, n);
    dd sn, cs;
    sincos_dd(r, &sn, &cs);
    const int q = (int)((long long)n & 3);
    dd sv, cv;
    switch (q) {
        case 0: sv = sn; cv = cs; break;
        case 1: sv = cs; cv = neg(sn); break;
        case 2: sv = neg(sn); cv = neg(cs); break;
        default: sv = neg(cs); cv = sn; break;
    }
    // the normalised head is the double nearest to the double-double value
    *s_out = (float)sv.h;
    *c_out = (float)cv.h;
}

// atan(t) for t in [0, 1] as a double-double: t = c + (t - c), c = k/16 nearest, and
// atan t = atan c + atan u, u = (t - c) / (1 + t c), |u| <= 1/32: odd series to u^31 (< 2^-150).
FMRX_CR dd atan01_dd(dd t) {
    const int kk = (int)rint(t.h * 16.0);
    const double c = (double)kk * 0.0625;
    const dd num = add(t, dd{-c, 0.0});
    const dd den = add(dd{1.0, 0.0}, mul_d(t, c));
    const dd u = div(num, den);
    const dd u2 = mul(u, u);
    dd p = k(kInvOdd[15]);
    for (int m = 14; m >= 0; m--) {
        p = mul(p, u2);
        p = add(k(kInvOdd[m]), neg(p));
    }
    return add(k(kAtanK16[kk]), mul(p, u));
}

// float(RN_double(atan2(y, x))) for floats, with C99's special values (as glibc).
FMRX_CR float atan2_f(float yf, float xf) {
    const double y = (double)yf, x = (double)xf;
    if (y != y || x != x) return yf + xf;  // NaN
    const bool yneg = signbit(y), xneg = signbit(x);
    const double ay = fabs(y), ax = fabs(x);
    double res;
    if (ay == 0.0) {
        res = xneg ? kPiH : 0.0;  // atan2(+-0, -x) = +-pi, atan2(+-0, +x) = +-0
    } else if (ax == 0.0) {
        res = kPio2H;
    } else if (isinf(ay) || isinf(ax)) {
        if (isinf(ay) && isinf(ax)) res = xneg ? 0x1.2d97c7f3321d2p+1 : 0x1.921fb54442d18p-1;  // 3pi/4, pi/4
        else if (isinf(ay)) res = kPio2H;
        else res = xneg ? kPiH : 0.0;
    } else {
        const bool swap = ay > ax;
        const dd t = swap ? div(dd{ax, 0.0}, dd{ay, 0.0}) : div(dd{ay, 0.0}, dd{ax, 0.0});
        dd a = atan01_dd(t);
        if (swap) a = add(dd{kPio2H, kPio2L}, neg(a));
        if (xneg) a = add(dd{kPiH, kPiL}, neg(a));
        res = a.h;
    }
    return (float)(yneg ? -res : res);
}

}  // namespace cr
}  // namespace fmrx
