// dd.h -- double-double ("dd", ~106-bit significand) and complex double-double scalars for the
// point stage's second precision tier.
//
// The reference decides its point stage in EXACT arithmetic: the foliation determinant at
// (rho, z) = (4/5, 6/7) is rejected when it is a non-zero Number or |evalf(50)| >= 1e-20
// (problems/force_free/validator.py:349-402); the Kerr residual at its three points is compared
// with 1e-10 at 40 digits (kerr_magnetosphere/validator.py:163-192).  fp64 jets decide most
// candidates with an error bound (pdeval_point.h); the rest are re-evaluated here at one point
// with these types.  The operations follow the error-free transformations (two_sum,
// two_prod = FMA) and the accurate double-word algorithms of Joldes, Muller & Popescu,
// "Tight and rigorous error bounds for basic building blocks of double-word arithmetic"
// (ACM TOMS 2017): add <= 3u^2, mul <= 4u^2, mul by a double <= 2u^2 (u = 2^-53); division,
// sqrt, exp and log are a few u^2.  dd_unit() is the unit the first-order error jets of the
// point stage are scaled with (2^-100, a 16x margin over those constants).
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>

#ifndef PD_HD
#define PD_HD __host__ __device__ __forceinline__
#endif

// The error-free transformations below depend on every + - * rounding exactly as written:
// no FMA contraction of a product into a following sum (hipcc contracts by default, which
// silently turns fast_two_sum(a*b, t) into fma(a, b, t) and breaks the double-word invariant).
// The pragma needs -ffp-contract=fast-honor-pragmas (Makefile); the code after this header
// gets the default contraction back (contract(fast) at the end).
#ifdef __clang__
#pragma clang fp contract(off)
#endif

namespace pd {

struct dd {
    double hi, lo;
};

PD_HD constexpr double dd_unit() { return 0x1p-100; }

PD_HD dd two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
PD_HD dd fast_two_sum(double a, double b) {  // |a| >= |b| (or a == 0)
    const double s = a + b;
    return {s, b - (s - a)};
}
PD_HD dd two_prod(double a, double b) {
    const double p = a * b;
    return {p, fma(a, b, -p)};
}

PD_HD dd operator+(dd x, dd y) {   // AccurateDWPlusDW
    dd s = two_sum(x.hi, y.hi);
    const dd t = two_sum(x.lo, y.lo);
    s.lo += t.hi;
    dd v = fast_two_sum(s.hi, s.lo);
    v.lo += t.lo;
    return fast_two_sum(v.hi, v.lo);
}
PD_HD dd operator-(dd x) { return {-x.hi, -x.lo}; }
PD_HD dd operator-(dd x, dd y) { return x + (-y); }
PD_HD dd operator+(dd x, double y) {   // DWPlusFP
    const dd s = two_sum(x.hi, y);
    return fast_two_sum(s.hi, s.lo + x.lo);
}
PD_HD dd operator*(dd x, dd y) {   // DWTimesDW3
    const dd c = two_prod(x.hi, y.hi);
    const double tl0 = x.lo * y.lo;
    const double tl1 = fma(x.hi, y.lo, tl0);
    const double cl2 = fma(x.lo, y.hi, tl1);
    return fast_two_sum(c.hi, c.lo + cl2);
}
PD_HD dd operator*(dd x, double y) {   // DWTimesFP3
    const dd c = two_prod(x.hi, y);
    return fast_two_sum(c.hi, fma(x.lo, y, c.lo));
}
PD_HD dd operator*(double y, dd x) { return x * y; }
PD_HD dd dd_from(double v) { return {v, 0.0}; }

// x / y: three quotient digits (the residual is formed in dd after each one)
PD_HD dd dd_div(dd x, dd y) {
    const double q1 = x.hi / y.hi;
    dd r = x - y * q1;
    const double q2 = r.hi / y.hi;
    r = r - y * q2;
    const double q3 = r.hi / y.hi;
    const dd q = fast_two_sum(q1, q2);
    return q + q3;
}
PD_HD dd dd_div(dd x, double y) {
    const double q1 = x.hi / y;
    const dd p = two_prod(q1, y);
    const double r = ((x.hi - p.hi) - p.lo) + x.lo;
    return fast_two_sum(q1, r / y);
}
// exact rational p / q as a dd (host tables: reference points, constants)
PD_HD dd dd_ratio(double p, double q) { return dd_div(dd_from(p), q); }

PD_HD dd dd_sqrt(dd a) {
    if (!(a.hi > 0.0)) return {a.hi == 0.0 ? 0.0 : sqrt(a.hi), 0.0};
    const double s = sqrt(a.hi);
    const dd s2 = two_prod(s, s);
    const double r = ((a.hi - s2.hi) - s2.lo) + a.lo;   // a - s^2 (a.hi - s2.hi is exact)
    return fast_two_sum(s, r / (2.0 * s));
}

// exp: x = k ln2 + 2^9 r, exp(r) - 1 by its Taylor series, then (1 + e)^(2^9) by e <- 2e + e^2
PD_HD dd dd_exp(dd a) {
    if (a.hi > 709.0) return {INFINITY, 0.0};
    if (a.hi < -745.0) return {0.0, 0.0};
    if (!(a.hi == a.hi)) return a;
    const dd ln2 = {0x1.62e42fefa39efp-1, 0x1.abc9e3b39803fp-56};
    const double k = rint(a.hi / ln2.hi);
    dd r = a - ln2 * k;
    r = {r.hi * 0x1p-9, r.lo * 0x1p-9};
    // e = r + r^2/2! + ... + r^12/12!  (|r| < 7e-4: the next term is < 1e-45)
    dd e = r;
    dd term = r;
#pragma unroll 1
    for (int n = 2; n <= 12; ++n) {
        term = dd_div(term * r, (double)n);
        e = e + term;
    }
#pragma unroll 1
    for (int i = 0; i < 9; ++i) e = e * 2.0 + e * e;
    e = e + 1.0;
    return {ldexp(e.hi, (int)k), ldexp(e.lo, (int)k)};
}

// log: one Newton step on exp from the double log (doubles the correct bits)
PD_HD dd dd_log(dd a) {
    if (!(a.hi > 0.0)) return {a.hi == 0.0 ? -INFINITY : NAN, 0.0};
    const dd x = dd_from(log(a.hi));
    const dd t = a * dd_exp(-x);
    return x + (t + (-1.0));
}

// sin / cos by their Taylor series after reduction modulo pi/2 (|x| up to ~1e3 keeps ~1e-29)
PD_HD void dd_sincos(dd a, dd* s_out, dd* c_out) {
    const dd pio2 = {0x1.921fb54442d18p+0, 0x1.1a62633145c07p-54};
    const double k = rint(a.hi / pio2.hi);
    const dd r = a - pio2 * k;
    const dd r2 = r * r;
    // sin r = r - r^3/3! + ...,  cos r = 1 - r^2/2! + ...  (|r| <= 0.79: 15 terms each)
    dd s = r, c = dd_from(1.0), ts = r, tc = dd_from(1.0);
#pragma unroll 1
    for (int n = 1; n <= 15; ++n) {
        ts = dd_div(-(ts * r2), (double)((2 * n) * (2 * n + 1)));
        tc = dd_div(-(tc * r2), (double)((2 * n - 1) * (2 * n)));
        s = s + ts;
        c = c + tc;
    }
    const int q = ((int)fmod(k, 4.0) + 4) & 3;
    if (q == 0) { *s_out = s; *c_out = c; }
    else if (q == 1) { *s_out = c; *c_out = -s; }
    else if (q == 2) { *s_out = -s; *c_out = -c; }
    else { *s_out = -c; *c_out = s; }
}

// atan2(y, x): one Newton step from the double angle (error ~ u^2)
PD_HD dd dd_atan2(dd y, dd x) {
    const dd t = dd_from(atan2(y.hi, x.hi));
    dd s, c;
    dd_sincos(t, &s, &c);
    // f(t) = y cos t - x sin t, f'(t) = -(y sin t + x cos t)
    const dd num = y * c - x * s;
    const dd den = y * s + x * c;
    return t + dd_div(num, den);
}

PD_HD dd dd_hypot(dd a, dd b) { return dd_sqrt(a * a + b * b); }

// ---- jet.h scalar interface for dd
template <class T> PD_HD T zero();
template <class T> PD_HD T from_real(double v);
template <> PD_HD dd zero<dd>() { return {0.0, 0.0}; }
template <> PD_HD dd from_real<dd>(double v) { return {v, 0.0}; }
PD_HD dd fmac(dd a, dd b, dd c) { return a * b + c; }
PD_HD double mag(dd a) { return fabs(a.hi); }
PD_HD bool finite_(dd a) { return isfinite(a.hi) && isfinite(a.lo); }
PD_HD bool is_zero(dd a) { return a.hi == 0.0 && a.lo == 0.0; }
PD_HD dd recip(dd a) { return dd_div(dd_from(1.0), a); }
PD_HD dd qdiv(dd s, dd b0, dd /*inv*/) { return dd_div(s, b0); }
PD_HD dd sqrt_(dd a) { return dd_sqrt(a); }
PD_HD dd exp_(dd a) { return dd_exp(a); }
PD_HD dd log_(dd a) { return dd_log(a); }
PD_HD dd pow_gen(dd a, double e) {
    if (a.hi == 0.0) return {e > 0 ? 0.0 : INFINITY, 0.0};
    if (a.hi < 0.0) return {NAN, 0.0};
    return dd_exp(dd_log(a) * e);
}
PD_HD double hi_of(dd a) { return a.hi; }
PD_HD double hi_of(double a) { return a; }

// ---- complex double-double (principal branch), for candidates not real at the point
struct cdd {
    dd re, im;
};
PD_HD cdd operator+(cdd a, cdd b) { return {a.re + b.re, a.im + b.im}; }
PD_HD cdd operator-(cdd a, cdd b) { return {a.re - b.re, a.im - b.im}; }
PD_HD cdd operator-(cdd a) { return {-a.re, -a.im}; }
PD_HD cdd operator*(cdd a, cdd b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
PD_HD cdd operator*(cdd a, double s) { return {a.re * s, a.im * s}; }
PD_HD cdd operator*(cdd a, dd s) { return {a.re * s, a.im * s}; }
template <> PD_HD cdd zero<cdd>() { return {{0.0, 0.0}, {0.0, 0.0}}; }
template <> PD_HD cdd from_real<cdd>(double v) { return {{v, 0.0}, {0.0, 0.0}}; }
PD_HD cdd fmac(cdd a, cdd b, cdd c) { return a * b + c; }
PD_HD double mag(cdd a) { return hypot(a.re.hi, a.im.hi); }
PD_HD bool finite_(cdd a) { return finite_(a.re) && finite_(a.im); }
PD_HD bool is_zero(cdd a) { return is_zero(a.re) && is_zero(a.im); }
PD_HD cdd recip(cdd a) {
    const dd d = a.re * a.re + a.im * a.im;
    return {dd_div(a.re, d), -dd_div(a.im, d)};
}
PD_HD cdd cdd_div(cdd x, cdd y) {
    const dd d = y.re * y.re + y.im * y.im;
    const cdd n = {x.re * y.re + x.im * y.im, x.im * y.re - x.re * y.im};
    return {dd_div(n.re, d), dd_div(n.im, d)};
}
PD_HD cdd qdiv(cdd s, cdd b0, cdd /*inv*/) { return cdd_div(s, b0); }
PD_HD cdd sqrt_(cdd a) {
    // principal branch, branch cut on the negative real axis (Im >= 0 there)
    const dd m = dd_hypot(a.re, a.im);
    if (m.hi == 0.0) return zero<cdd>();
    if (a.re.hi >= 0.0) {
        const dd t = dd_sqrt((m + a.re) * 0.5);
        return {t, dd_div(a.im, t * 2.0)};
    }
    const dd t = dd_sqrt((m - a.re) * 0.5);
    const dd ai = a.im.hi < 0.0 ? -a.im : a.im;
    return {dd_div(ai, t * 2.0), a.im.hi < 0.0 ? -t : t};
}
PD_HD cdd exp_(cdd a) {
    const dd e = dd_exp(a.re);
    if (is_zero(a.im)) return {e, {0.0, 0.0}};
    dd s, c;
    dd_sincos(a.im, &s, &c);
    return {e * c, e * s};
}
PD_HD cdd log_(cdd a) {
    const dd l = dd_log(dd_hypot(a.re, a.im));
    if (is_zero(a.im) && a.re.hi > 0.0) return {l, {0.0, 0.0}};
    return {l, dd_atan2(a.im, a.re)};
}
PD_HD cdd pow_gen(cdd a, double e) {
    if (is_zero(a)) return {{e > 0 ? 0.0 : INFINITY, 0.0}, {0.0, 0.0}};
    const cdd l = log_(a);
    return exp_(cdd{l.re * e, l.im * e});
}

}  // namespace pd

#ifdef __clang__
#pragma clang fp contract(fast)
#endif
