// jet.h -- truncated bivariate Taylor arithmetic ("jets") for the gfx950 validator.
//
// A jet of order K holds the Taylor coefficients c[i][j] (i + j <= K) of a function of the two
// coordinates around one sample point:  f(x0 + a, y0 + b) = sum c_ij a^i b^j.  Derivatives
// follow as u_ij = i! j! c_ij.  This replaces the reference's symbolic differentiation
// (sp.diff in problems/force_free/validator.py:305-344 and kerr_magnetosphere/validator.py:77-91):
// instead of building the 4th-order derivative tower symbolically and substituting a point,
// every program is evaluated directly in jet arithmetic at every sample point.
//
// Storage is degree-major: index(i, j) = d(d+1)/2 + j with d = i + j.  Every loop below has
// compile-time bounds, so after full unrolling all coefficient indices are constants and a
// jet lives entirely in VGPRs (15 doubles = 30 VGPRs at K = 4).
//
// The scalar type T is double for the real pass and pd_cplx for the complex pass (principal
// branch, used when a candidate is not real at the reference point, as SymPy's exact
// evaluation at validator.py:349-402 is).
#pragma once
#include <hip/hip_runtime.h>

#define PD_HD __host__ __device__ __forceinline__

#include "dd.h"

namespace pd {

PD_HD constexpr int nc(int K) { return (K + 1) * (K + 2) / 2; }
PD_HD constexpr int ji(int i, int j) { return (i + j) * (i + j + 1) / 2 + j; }

// ------------------------------------------------------------------ scalar helpers
struct cplx {
    double re, im;
};
PD_HD cplx operator+(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
PD_HD cplx operator-(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }
PD_HD cplx operator-(cplx a) { return {-a.re, -a.im}; }
PD_HD cplx operator*(cplx a, cplx b) {
    return {fma(a.re, b.re, -a.im * b.im), fma(a.re, b.im, a.im * b.re)};
}
PD_HD cplx operator*(cplx a, double s) { return {a.re * s, a.im * s}; }

template <> PD_HD double zero<double>() { return 0.0; }
template <> PD_HD cplx zero<cplx>() { return {0.0, 0.0}; }
template <> PD_HD double from_real<double>(double v) { return v; }
template <> PD_HD cplx from_real<cplx>(double v) { return {v, 0.0}; }

// Coordinates and constants enter the jets as V = double (fp64 and complex passes) or V = dd
// (the double-double point tier, dd.h); cvt<T>(v) converts them to the jet scalar T.
template <class T, class V> struct Cvt {
    static PD_HD T f(double v) { return from_real<T>(v); }
};
template <> struct Cvt<dd, dd> { static PD_HD dd f(dd v) { return v; } };
template <> struct Cvt<cdd, dd> { static PD_HD cdd f(dd v) { return {v, {0.0, 0.0}}; } };
template <class T, class V> PD_HD T cvt(V v) { return Cvt<T, V>::f(v); }
PD_HD double rcp(double v) { return 1.0 / v; }
PD_HD dd rcp(dd v) { return recip(v); }
PD_HD double vabs(double v) { return fabs(v); }
PD_HD double vabs(dd v) { return fabs(v.hi); }
// v * num / k for a Taylor-coefficient recurrence: fp64 scales by the rounded num / k (as
// the fp64 passes always have); the double-double tier divides exactly-rounded (1/3 is not
// a double)
PD_HD double divk(double v, double num, int k) { return v * (num / k); }
PD_HD cplx divk(cplx v, double num, int k) { return v * (num / k); }
PD_HD dd divk(dd v, double num, int k) { return dd_div(v * num, (double)k); }
PD_HD cdd divk(cdd v, double num, int k) { return {dd_div(v.re * num, (double)k), dd_div(v.im * num, (double)k)}; }
template <class V> PD_HD V vone() { return V(1.0); }
template <> PD_HD dd vone<dd>() { return {1.0, 0.0}; }
template <class V> PD_HD V vzero() { return V(0.0); }
template <> PD_HD dd vzero<dd>() { return {0.0, 0.0}; }

PD_HD double fmac(double a, double b, double c) { return fma(a, b, c); }
PD_HD cplx fmac(cplx a, cplx b, cplx c) {
    return {fma(a.re, b.re, fma(-a.im, b.im, c.re)), fma(a.re, b.im, fma(a.im, b.re, c.im))};
}
PD_HD double mag(double a) { return fabs(a); }
PD_HD double mag(cplx a) { return hypot(a.re, a.im); }
PD_HD bool finite_(double a) { return isfinite(a); }
PD_HD bool finite_(cplx a) { return isfinite(a.re) && isfinite(a.im); }
PD_HD bool is_zero(double a) { return a == 0.0; }
PD_HD bool is_zero(cplx a) { return a.re == 0.0 && a.im == 0.0; }

PD_HD double recip(double a) { return 1.0 / a; }
PD_HD cplx recip(cplx a) {
    // Smith's algorithm
    if (fabs(a.re) >= fabs(a.im)) {
        double r = a.im / a.re, d = a.re + a.im * r;
        return {1.0 / d, -r / d};
    }
    double r = a.re / a.im, d = a.re * r + a.im;
    return {r / d, -1.0 / d};
}
PD_HD double sqrt_(double a) { return sqrt(a); }
PD_HD cplx sqrt_(cplx a) {
    // principal branch, branch cut on the negative real axis (Im >= 0 there)
    double m = hypot(a.re, a.im);
    if (m == 0.0) return {0.0, 0.0};
    if (a.re >= 0.0) {
        double t = sqrt(0.5 * (m + a.re));
        return {t, a.im / (2.0 * t)};
    }
    double t = sqrt(0.5 * (m - a.re));
    return {fabs(a.im) / (2.0 * t), copysign(t, a.im)};
}
// The transcendental routines are kept out of line: inlined, their polynomial constants are
// hoisted out of the interpreter loop by LICM and then spilled to scratch, which costs every
// candidate; called, they cost only the (rare) EXP / LOG / general-POW opcodes.
#if defined(__HIP_DEVICE_COMPILE__)
#define PD_TRANS __host__ __device__ __attribute__((noinline))
#else
#define PD_TRANS __host__ __device__ inline
#endif
PD_TRANS double exp_(double a) { return exp(a); }
PD_TRANS cplx exp_(cplx a) {
    double e = exp(a.re);
    return {e * cos(a.im), e * sin(a.im)};
}
PD_TRANS double log_(double a) { return log(a); }
PD_TRANS cplx log_(cplx a) { return {log(hypot(a.re, a.im)), atan2(a.im, a.re)}; }
PD_TRANS double pow_gen(double a, double e) { return pow(a, e); }
PD_TRANS cplx pow_gen(cplx a, double e) {
    if (a.re == 0.0 && a.im == 0.0) return {e > 0 ? 0.0 : INFINITY, 0.0};
    cplx l = log_(a);
    return exp_(cplx{l.re * e, l.im * e});
}

template <class T> PD_HD T powi_(T x, int n) {
    // x**n for n >= 0 by binary powering
    T r = from_real<T>(1.0);
    T b = x;
    while (n > 0) {
        if (n & 1) r = r * b;
        b = b * b;
        n >>= 1;
    }
    return r;
}

// x0**alpha on the principal branch.  Exponents in (1/4)Z (every exponent the reference's op
// vocabulary expression_operations.py:29-62 can produce) are built from integer powers and
// square roots, which are correctly rounded; anything else goes through pow().
template <class T> PD_HD T pow_real_exp(T x, double alpha) {
    double a4 = alpha * 4.0;
    if (a4 == rint(a4) && fabs(alpha) <= 64.0) {
        int n4 = (int)a4;
        int n = (n4 >= 0) ? n4 / 4 : -((-n4 + 3) / 4);  // floor(n4 / 4)
        int rem = n4 - 4 * n;                           // 0..3
        T p = (n >= 0) ? powi_(x, n) : recip(powi_(x, -n));
        if (rem != 0) {
            T s = sqrt_(x);
            if (rem == 1) p = p * sqrt_(s);
            else if (rem == 2) p = p * s;
            else p = p * (s * sqrt_(s));
        }
        return p;
    }
    return pow_gen(x, alpha);
}

// ------------------------------------------------------------------ jet kernels
// c = a * b, a of order KA, b of order KB, c truncated at order KC.  SKIP_A0: a[0] == 0.
template <class T, int KA, int KB, int KC, bool SKIP_A0 = false>
PD_HD void jmul(const T* a, const T* b, T* c) {
#pragma unroll
    for (int d = 0; d <= KC; ++d) {
#pragma unroll
        for (int j = 0; j <= d; ++j) {
            T s = zero<T>();
            bool first = true;
#pragma unroll
            for (int d1 = SKIP_A0 ? 1 : 0; d1 <= d; ++d1) {
                const int d2 = d - d1;
                if (d1 > KA || d2 > KB) continue;
#pragma unroll
                for (int j1 = 0; j1 <= d1; ++j1) {
                    const int j2 = j - j1;
                    if (j2 < 0 || j2 > d2) continue;
                    if (first) {
                        s = a[ji(d1 - j1, j1)] * b[ji(d2 - j2, j2)];
                        first = false;
                    } else {
                        s = fmac(a[ji(d1 - j1, j1)], b[ji(d2 - j2, j2)], s);
                    }
                }
            }
            c[ji(d - j, j)] = s;
        }
    }
}

// q = s / b0 from a reciprocal plus one FMA residual correction: the correctly rounded quotient
// in practice (Markstein), and exact whenever s / b0 is representable -- so a/a is exactly 1 and
// exact cancellations of the candidate survive, as SymPy's exact arithmetic keeps them.
PD_HD double qdiv(double s, double b0, double inv) {
    const double q = s * inv;
    return fma(fma(-q, b0, s), inv, q);
}
PD_HD cplx qdiv(cplx s, cplx b0, cplx inv) {
    const cplx q = s * inv;
    return q + (s - q * b0) * inv;
}

// c = a / b (all order K).  c must not alias a or b.
template <class T, int K> PD_HD void jdiv(const T* a, const T* b, T* c) {
    const T inv = recip(b[0]);
    c[0] = qdiv(a[0], b[0], inv);
#pragma unroll
    for (int d = 1; d <= K; ++d) {
#pragma unroll
        for (int j = 0; j <= d; ++j) {
            T s = a[ji(d - j, j)];
#pragma unroll
            for (int d1 = 1; d1 <= d; ++d1) {
                const int d2 = d - d1;
#pragma unroll
                for (int j1 = 0; j1 <= d1; ++j1) {
                    const int j2 = j - j1;
                    if (j2 < 0 || j2 > d2) continue;
                    s = fmac(-b[ji(d1 - j1, j1)], c[ji(d2 - j2, j2)], s);
                }
            }
            c[ji(d - j, j)] = qdiv(s, b[0], inv);
        }
    }
}

// Horner composition with truncation: out (order K-L) = sum_{k>=L} f[k] h^(k-L)
template <class T, int K, int L> struct Horner {
    PD_HD static void run(const T* h, const T* f, T* out) {
        T inner[nc(K - L - 1)];
        Horner<T, K, L + 1>::run(h, f, inner);
        jmul<T, K - L, K - L - 1, K - L, true>(h, inner, out);
        out[0] = f[L];
    }
};
template <class T, int K> struct Horner<T, K, K> {
    PD_HD static void run(const T*, const T* f, T* out) { out[0] = f[K]; }
};

// x <- g(x) where g has Taylor coefficients f[0..K] around x[0]
template <class T, int K> PD_HD void jcompose(T* x, const T* f) {
    T h[nc(K)];
    h[0] = zero<T>();
#pragma unroll
    for (int i = 1; i < nc(K); ++i) h[i] = x[i];
    Horner<T, K, 0>::run(h, f, x);
}

// Taylor coefficients of x**alpha around x0 (f0 given)
template <class T, int K> PD_HD void coef_pow(T x0, double alpha, T f0, T* f) {
    const T r = recip(x0);
    f[0] = f0;
#pragma unroll
    for (int k = 1; k <= K; ++k) f[k] = divk(f[k - 1] * r, alpha - (k - 1), k);
}

}  // namespace pd
