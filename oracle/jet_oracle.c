/* jet_oracle.c -- CPU restatement of the candidate validator (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library,
 * and only as the checker / the timed CPU baseline -- the product path (libpdeval.so) never
 * links or calls it.
 *
 * What it restates (all citations into /root/reference):
 *   force-free  problems/force_free/validator.py:260-402 -- derivatives of u (:305-320),
 *               A, B (:323-324, Omega = 0 on the problem path :82-83), the Lie derivative
 *               L_T f = u_z f_rho - u_rho f_z (:335-339), det (:347), the point stage at
 *               (rho, z) = (4/5, 6/7) (:296-297, :349-402) and the zero-gradient exit (:309-312);
 *               the symbolic stage (:404-427) is restated as "zero at every finite grid point".
 *   Kerr        problems/kerr_magnetosphere/validator.py:69-91 (operator), :163-192 (3-point
 *               check, absolute 1e-10), :231-240 (constant exclusion), :283-315 (exact zero).
 * Numerics: double jets for the real pass, double complex for the complex (principal branch)
 * pass; the determinant is written out in closed form in the partials u_ij rather than by
 * jets (the device does the latter), so device and oracle agree only if both are right.
 */
#include <complex.h>
#include <math.h>
#include <quadmath.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/pdeval.h"

#define KMAX 4
#define NCMAX 15
#define NC(K) (((K) + 1) * ((K) + 2) / 2)
#define IDX(i, j) (((i) + (j)) * ((i) + (j) + 1) / 2 + (j))

/* ---------------------------------------------------------------- noise bounds
 * Tier 2 of the zero test: beside every jet value v the interpreter carries a
 * non-negative jet E, a first-order running bound of its rounding error in units of eps:
 * |computed - exact| <~ eps * E, coefficient-wise.  Rules (|a| = coefficient-wise modulus):
 *   leaf x, y : 0 (exact inputs);  constant c : |c|
 *   a +- b    : E_a + E_b + |r|
 *   a * b     : |a| (*) E_b + E_a (*) |b| + |a| (*) |b|             ((*) = jet product)
 *   a / b     : absdiv(E_a + |r| (*) E_b, |b|) + |r|
 *   g(a)      : G1 (*) E_a + sum_k |f_k| |h|^k,  G1 = sum_m (m+1) |f_(m+1)| |h|^m, h = a - a0
 * where absdiv(N, |b|) is the division recurrence with every sign made positive (it bounds
 * the coefficients of N * (1/b)).  Real doubles for both passes (the complex pass bounds
 * moduli). */
static void w_mul(const double* a, const double* b, double* c, int K) {
    double r[NCMAX];
    for (int d = 0; d <= K; ++d)
        for (int j = 0; j <= d; ++j) {
            double s = 0;
            for (int d1 = 0; d1 <= d; ++d1)
                for (int j1 = 0; j1 <= d1; ++j1) {
                    int d2 = d - d1, j2 = j - j1;
                    if (j2 < 0 || j2 > d2) continue;
                    s += a[IDX(d1 - j1, j1)] * b[IDX(d2 - j2, j2)];
                }
            r[IDX(d - j, j)] = s;
        }
    memcpy(c, r, sizeof(double) * NC(K));
}

static void w_absdiv(const double* nmr, const double* b, double* c, int K) {
    double r[NCMAX];
    for (int d = 0; d <= K; ++d)
        for (int j = 0; j <= d; ++j) {
            const int k = IDX(d - j, j);
            double s = nmr[k];
            for (int d1 = 1; d1 <= d; ++d1)
                for (int j1 = 0; j1 <= d1; ++j1) {
                    int d2 = d - d1, j2 = j - j1;
                    if (j2 < 0 || j2 > d2) continue;
                    s += b[IDX(d1 - j1, j1)] * r[IDX(d2 - j2, j2)];
                }
            r[k] = s / b[0];
        }
    memcpy(c, r, sizeof(double) * NC(K));
}

/* out = sum_k F[k] h^k (h[0] ignored), all non-negative */
static void w_horner(const double* h0, const double* F, double* out, int K) {
    double h[NCMAX], hk[NCMAX], acc[NCMAX];
    memcpy(h, h0, sizeof(double) * NC(K));
    h[0] = 0;
    for (int i = 0; i < NCMAX; ++i) { acc[i] = 0; hk[i] = 0; }
    acc[0] = F[0];
    hk[0] = 1;
    for (int k = 1; k <= K; ++k) {
        w_mul(hk, h, hk, K);
        for (int i = 0; i < NC(K); ++i) acc[i] += F[k] * hk[i];
    }
    memcpy(out, acc, sizeof(double) * NC(K));
}

#define CT double
#define CABS cabs
#define CREAL creal
#define CIMAG cimag
#define CEXP cexp
#define CLOG clog
#define RPOW pow
#define REXP exp
#define RLOG log
#define CI I
/* force-free Omega^2 (pdeval_params.omega2), set by oracle_validate / oracle_set_omega2 */
static double OM2 = 0.0;
/* its low part (pdeval_params.omega2_lo): Omega^2 = OM2 + OM2_LO, a double-double -- the quad
 * point stage takes both, the f64 grid stages OM2 alone (as the device) */
static double OM2_LO = 0.0;
int oracle_set_omega2(double w) { OM2 = w; return 0; }
int oracle_set_omega2_lo(double w) { OM2_LO = w; return 0; }

#define S double
#define FN(name) name##_r
#include "jet_oracle_impl.h"
#undef S
#undef FN
#define S double complex
#define FN(name) name##_c
#include "jet_oracle_impl.h"
#undef S
#undef FN
#undef CT
#undef CABS
#undef CREAL
#undef CIMAG
#undef CEXP
#undef CLOG
#undef RPOW
#undef REXP
#undef RLOG
#undef CI
/* quad precision (113-bit significand) for the point stage: the reference decides it in exact
 * arithmetic (validator.py:349-402), so the oracle evaluates the reference points with
 * coordinates and constants wider than f64 (immediates carry their double-double low part) */
#define CT __float128
#define CABS cabsq
#define CREAL crealq
#define CIMAG cimagq
#define CEXP cexpq
#define CLOG clogq
#define RPOW powq
#define REXP expq
#define RLOG logq
#define CI ((__complex128)I)
#define S __complex128
#define FN(name) name##_q
#include "jet_oracle_impl.h"
#undef S
#undef FN

/* ---------------------------------------------------------------- Kerr constants
 * The reference substitutes M = M_value, a = a_value in its fast point check only
 * (kerr validator.py:163-192); its constant test (:231-240) and symbolic stage (:283-300) keep M
 * and a symbolic.  Restated as in pdeval.h (pdeval_kerr_constants): the point stage at
 * (M_value, a_value), the constant test and the grid at stand-ins of the symbols; a constant the
 * validator was built with as a number (op_*_fixed) is that number in the operator of every
 * stage, and u's own symbol is then free (its stand-in everywhere). */
static struct {
    __float128 opM_pt, opa_pt;      /* operator, point stage (exact rationals, quad) */
    double opM_g, opa_g;            /* operator, grid stage */
    double prm_pt[8], prm_g[8];     /* u's constants {M, a, 1/M, 1/a, M^2, a^2, 1/M^2, 1/a^2} */
    __float128 prm_pt_q[8], prm_g_q[8];
    int set;
} KC;

int oracle_set_kerr_constants(int64_t M_num, int64_t M_den, int64_t a_num, int64_t a_den, double M_sym,
                              double a_sym, int op_M_fixed, int op_a_fixed) {
    const __float128 Mq = (__float128)M_num / M_den, aq = (__float128)a_num / a_den;
    KC.opM_pt = Mq;
    KC.opa_pt = aq;
    KC.opM_g = op_M_fixed ? (double)((long double)M_num / M_den) : M_sym;
    KC.opa_g = op_a_fixed ? (double)((long double)a_num / a_den) : a_sym;
    const __float128 uM = op_M_fixed ? (__float128)M_sym : Mq, ua = op_a_fixed ? (__float128)a_sym : aq;
    const __float128 Mg = M_sym, ag = a_sym;
    const __float128 pq[8] = {uM, ua, 1 / uM, 1 / ua, uM * uM, ua * ua, 1 / (uM * uM), 1 / (ua * ua)};
    const __float128 gq[8] = {Mg, ag, 1 / Mg, 1 / ag, Mg * Mg, ag * ag, 1 / (Mg * Mg), 1 / (ag * ag)};
    for (int k = 0; k < 8; ++k) {
        KC.prm_pt_q[k] = pq[k];
        KC.prm_g_q[k] = gq[k];
        KC.prm_pt[k] = (double)pq[k];
        KC.prm_g[k] = (double)gq[k];
    }
    KC.set = 1;
    return 0;
}

static void kc_default(void) {
    /* pdeval_default_kerr_constants: M_value = 1, a_value = 1/10 (problems/__init__.py:283) */
    if (!KC.set) oracle_set_kerr_constants(1, 1, 1, 10, 1.171875, 0.359375, 0, 0);
}

/* the Kerr constant-test points (pdeval.hip build_points): the reference points, then two more */
static const double kCtX[5] = {5.0 / 2.0, 7.0 / 3.0, 5.0, 3.3, 6.1};
static const double kCtY[5] = {3.0 / 5.0, 1.0 / 3.0, -2.0 / 5.0, 0.27, -0.55};

/* ---------------------------------------------------------------- sample points */
/* Restates DESIGN.md "Grids" (the device builds the same table in pdeval_create). */
static int build_points(int problem, double** px, double** py, int* n_ref) {
    const int nx = 64, ny = 64;
    double x_lo, x_hi, y_lo = -2.0, y_hi = 2.0, ph_x = 0.37, ph_y = 0.41;
    int nr;
    double rx[3], ry[3];
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        x_lo = 0.05; x_hi = 3.0;
        nr = 1; rx[0] = 4.0 / 5.0; ry[0] = 6.0 / 7.0;
    } else {
        kc_default();
        /* r+ = M + sqrt(M^2 - a^2) of the grid stage's operator */
        double rp = KC.opM_g + sqrt(KC.opM_g * KC.opM_g - KC.opa_g * KC.opa_g);
        x_lo = rp + 0.1; x_hi = rp + 6.1; y_lo = -0.98; y_hi = 0.98;
        nr = 3;
        rx[0] = 5.0 / 2.0; ry[0] = 3.0 / 5.0;
        rx[1] = 7.0 / 3.0; ry[1] = 1.0 / 3.0;
        rx[2] = 5.0;       ry[2] = -2.0 / 5.0;
    }
    int n = nr + nx * ny;
    *px = (double*)malloc(sizeof(double) * n);
    *py = (double*)malloc(sizeof(double) * n);
    for (int k = 0; k < nr; ++k) { (*px)[k] = rx[k]; (*py)[k] = ry[k]; }
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < ny; ++j) {
            (*px)[nr + i * ny + j] = x_lo + (i + ph_x) * ((x_hi - x_lo) / nx);
            (*py)[nr + i * ny + j] = y_lo + (j + ph_y) * ((y_hi - y_lo) / ny);
        }
    *n_ref = nr;
    return n;
}

/* Kerr linear surrogate at the operator's (M, a), expanded by hand from kerr validator.py:77-91:
 * d_r[G/(1-x^2) u_r] + d_x[G/Delta u_x]
 *   = G/(1-x^2) u_rr + G_r/(1-x^2) u_r + G/Delta u_xx + G_x/Delta u_x            */
static void kerr_terms(double r, double x, const double complex* c, int cplx, double complex* L,
                       double* scale, double M, double a) {
    double s = r * r + a * a * x * x;
    double G = 1.0 - 2.0 * M * r / s;
    double Gr = -2.0 * M / s + 4.0 * M * r * r / (s * s);
    double Gx = 4.0 * M * r * a * a * x / (s * s);
    double D = r * r - 2.0 * M * r + a * a, w = 1.0 - x * x;
    double complex urr = 2.0 * c[IDX(2, 0)], uxx = 2.0 * c[IDX(0, 2)], ur = c[IDX(1, 0)], ux = c[IDX(0, 1)];
    double complex t[4] = {G / w * urr, Gr / w * ur, G / D * uxx, Gx / D * ux};
    (void)cplx;
    *L = t[0] + t[1] + t[2] + t[3];
    *scale = cabs(t[0]) + cabs(t[1]) + cabs(t[2]) + cabs(t[3]);
}

typedef struct {
    double res_abs, res_re, scale;
    int finite, grad_zero, tiny;
    double u0;
    double noise;   /* tier 2 only: first-order rounding-noise bound of the residual */
    double grad[2], grad_err[2];   /* quad tier: |u_x|, |u_y| and their error bounds (EPSQ units) */
} pt_result;

/* gamma for the finite-difference form of the first-order noise bound: the noise is
 * (S(|c| + gamma W) - S(|c|)) * eps / gamma + eps * S, S the magnitude epilogue */
#define NOISE_GAMMA 0x1p-30
#define EPS64 0x1p-52

/* grid: the constant test's / grid stage's constants (else the point stage's) */
static pt_result eval_point(int problem, const int32_t* w, int64_t nw, double x, double y, int cplx,
                            int tier2, int* rc, int grid) {
    pt_result r = {0};
    const int K = problem == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
    double complex cc[NCMAX];
    double W[NCMAX];
    kc_default();
    const double* prm = grid ? KC.prm_g : KC.prm_pt;
    const double opM = grid ? KC.opM_g : (double)KC.opM_pt, opa = grid ? KC.opa_g : (double)KC.opa_pt;
    if (cplx) {
        *rc = run_c(w, nw, x, y, K, 1, cc, tier2 ? W : NULL, 0.0, prm);
    } else {
        double cr[NCMAX];
        *rc = run_r(w, nw, x, y, K, 0, cr, tier2 ? W : NULL, 0.0, prm);
        for (int i = 0; i < NC(K); ++i) cc[i] = cr[i];
    }
    if (*rc) return r;
    int fin = 1;
    /* (the device's jet_coef_ok: below 2^160, so no order-dependent overflow downstream; Kerr:
     * not u_rx, which its operator does not contain -- kerr_epilogue) */
    const int mix = (problem == PDEVAL_PROBLEM_FORCE_FREE || !grid) ? -1 : IDX(1, 1);
    for (int i = 0; i < NC(K); ++i)
        if (i != mix) fin = fin && fabs(creal(cc[i])) < 0x1p160 && fabs(cimag(cc[i])) < 0x1p160;
    double complex res;
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        res = ff_det_c(cc, x, 0);
        r.scale = creal(ff_det_c(cc, x, 1));
    } else {
        kerr_terms(x, y, cc, cplx, &res, &r.scale, opM, opa);
    }
    if (tier2) {
        double complex cp[NCMAX];
        double complex res2;
        double S2;
        for (int i = 0; i < NC(K); ++i) cp[i] = cabs(cc[i]) + NOISE_GAMMA * W[i];
        if (problem == PDEVAL_PROBLEM_FORCE_FREE) S2 = creal(ff_det_c(cp, x, 1));
        else kerr_terms(x, y, cp, 0, &res2, &S2, opM, opa);
        r.noise = (S2 - r.scale) * (EPS64 / NOISE_GAMMA) + EPS64 * r.scale;
    }
    r.res_abs = cabs(res);
    r.res_re = creal(res);
    r.finite = fin && isfinite(creal(res)) && isfinite(cimag(res)) && isfinite(r.scale);
    if (problem != PDEVAL_PROBLEM_FORCE_FREE) {
        /* Kerr: a jet exactly 0 to second order is an underflow, not a sample (pdeval_kernels.h) */
        int allz = 1;
        for (int i = 0; i < NC(K); ++i) allz = allz && (i == mix || cc[i] == 0);
        if (allz) r.finite = 0;
    }
    r.grad_zero = cc[IDX(1, 0)] == 0 && cc[IDX(0, 1)] == 0;
    r.u0 = creal(cc[0]) + 0x1.6a09e667f3bcdp+0 * cimag(cc[0]);   /* fingerprint: Re + sqrt(2) Im */
    return r;
}

static double scaled(double a, double s) { return s > 0 ? a / s : (a == 0 ? 0 : INFINITY); }
/* the grid's zero test, as the device applies it (pdeval_kernels.h grid_fails): a finite point
 * fails iff |res| > tau S -- no division (equal to scaled(res, S) > tau except within a rounding
 * of tau) */
static int grid_fails(double a, double s, double tau) { return a > tau * s; }

/* ---------------------------------------------------------------- point stage (quad)
 * The reference points as exact ratios, evaluated in __float128 (constants carry their
 * double-double low part).  The noise bound is the same first-order E-jet rule as tier 2, in
 * units of EPSQ (quad unit roundoff 2^-113, with a 32x margin for libquadmath's transcendentals). */
#define EPSQ 0x1p-108
static void ref_point_q(int problem, int k, __float128* x, __float128* y) {
    static const int ff[1][4] = {{4, 5, 6, 7}};
    static const int kr[3][4] = {{5, 2, 3, 5}, {7, 3, 1, 3}, {5, 1, -2, 5}};
    const int* t = problem == PDEVAL_PROBLEM_FORCE_FREE ? ff[k] : kr[k];
    *x = (__float128)t[0] / t[1];
    *y = (__float128)t[2] / t[3];
}

static __complex128 kerr_lhs_q(__float128 r, __float128 x, const __complex128* c, double* scale) {
    const __float128 M = KC.opM_pt, a = KC.opa_pt;   /* the point stage's operator */
    __float128 s = r * r + a * a * x * x;
    __float128 G = 1 - 2 * M * r / s;
    __float128 Gr = -2 * M / s + 4 * M * r * r / (s * s);
    __float128 Gx = 4 * M * r * a * a * x / (s * s);
    __float128 D = r * r - 2 * M * r + a * a, w = 1 - x * x;
    __complex128 t[4] = {G / w * 2 * c[IDX(2, 0)], Gr / w * c[IDX(1, 0)], G / D * 2 * c[IDX(0, 2)],
                         Gx / D * c[IDX(0, 1)]};
    *scale = (double)(cabsq(t[0]) + cabsq(t[1]) + cabsq(t[2]) + cabsq(t[3]));
    return t[0] + t[1] + t[2] + t[3];
}

/* value, scale and noise bound of one program at reference point k, in quad precision */
static pt_result eval_point_q(int problem, const int32_t* w, int64_t nw, int k, int cplx, int* rc) {
    pt_result r = {0};
    const int K = problem == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
    __float128 x, y;
    ref_point_q(problem, k, &x, &y);
    __complex128 cq[NCMAX];
    double W[NCMAX];
    /* the reference points are quad-rounded: 2^-113 relative, 1/32 of EPSQ */
    kc_default();
    *rc = run_q(w, nw, x, y, K, cplx, cq, W, 1.0 / 32, KC.prm_pt_q);
    if (*rc) return r;
    int fin = 1;
    double complex cd[NCMAX], cp[NCMAX];
    for (int i = 0; i < NC(K); ++i) {
        fin = fin && fabsq(crealq(cq[i])) < 0x1p160Q && fabsq(cimagq(cq[i])) < 0x1p160Q;
        cd[i] = (double)cabsq(cq[i]);
        cp[i] = cd[i] + NOISE_GAMMA * W[i];
    }
    __complex128 res;
    double S2;
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        res = ff_det_q(cq, x, 0);
        r.scale = creal(ff_det_c(cd, (double)x, 1));
        S2 = creal(ff_det_c(cp, (double)x, 1));
    } else {
        double complex dummy;
        res = kerr_lhs_q(x, y, cq, &r.scale);
        kerr_terms((double)x, (double)y, cp, 0, &dummy, &S2, (double)KC.opM_pt, (double)KC.opa_pt);
    }
    r.noise = (S2 - r.scale) * (EPSQ / NOISE_GAMMA) + EPSQ * r.scale;
    /* an Omega^2 carried as a double-double (OM2_LO != 0) is off by up to 2^-106 relative: the
     * determinant, bilinear in it through A and B, by up to 2^-104 of its scale */
    if (problem == PDEVAL_PROBLEM_FORCE_FREE && OM2_LO != 0) r.noise += 0x1p-104 * r.scale;
    r.res_abs = (double)cabsq(res);
    r.res_re = (double)crealq(res);
    r.finite = fin && finiteq(crealq(res)) && finiteq(cimagq(res)) && isfinite(r.scale) && isfinite(r.noise);
    if (problem != PDEVAL_PROBLEM_FORCE_FREE) {
        /* Kerr: every coefficient below 2^-900 (kTinyJet, pdeval_kernels.h) -- u underflowed in
         * the device's fp64; the reference's N(lhs, 40) finds |lhs| astronomically small: a
         * passing point that decides nothing else */
        int tiny = 1;
        for (int i = 0; i < NC(K); ++i) tiny = tiny && cabsq(cq[i]) < 0x1p-900Q && !(W[i] >= 0x1p-900);
        if (tiny) { r.finite = 1; r.tiny = 1; }
    }
    r.grad_zero = cq[IDX(1, 0)] == 0 && cq[IDX(0, 1)] == 0;
    r.grad[0] = (double)cabsq(cq[IDX(1, 0)]);
    r.grad[1] = (double)cabsq(cq[IDX(0, 1)]);
    r.grad_err[0] = W[IDX(1, 0)];
    r.grad_err[1] = W[IDX(0, 1)];
    r.u0 = (double)crealq(cq[0]) + 0x1.6a09e667f3bcdp+0 * (double)cimagq(cq[0]);
    return r;
}

/* Kerr constant test at the stand-ins of the symbols (pdeval_point.h kerr_constant_test): at
 * every constant-test point, u finite and its gradient within kappa x its rounding bound (quad) */
static int kerr_constant_test(const int32_t* w, int64_t nw, double kappa) {
    kc_default();
    for (int p = 0; p < 5; ++p) {
        __complex128 cq[NCMAX];
        double W[NCMAX];
        if (run_q(w, nw, (__float128)kCtX[p], (__float128)kCtY[p], 2, 0, cq, W, 0.0, KC.prm_g_q)) return 0;
        int tiny = 1;
        for (int i = 0; i < NC(2); ++i) {
            if (!(fabsq(crealq(cq[i])) < 0x1p160Q)) return 0;
            tiny = tiny && cabsq(cq[i]) < 0x1p-900Q && !(W[i] >= 0x1p-900);
        }
        if (tiny) return 0;   /* an underflowed jet is no evidence of a constant */
        if ((double)cabsq(cq[IDX(1, 0)]) > kappa * (double)EPSQ * W[IDX(1, 0)]) return 0;
        if ((double)cabsq(cq[IDX(0, 1)]) > kappa * (double)EPSQ * W[IDX(0, 1)]) return 0;
    }
    return 1;
}

/* Validate n programs; outputs as in pdeval_outputs (host arrays, any may be NULL).
 * Returns 0.  Candidate classes follow include/pdeval.h. */
int oracle_validate(int problem, const int32_t* ops, const int64_t* offsets, int64_t n,
                    const pdeval_params* prm, uint8_t* status, double* q_ref, double* res_ref,
                    double* q_grid, int32_t* n_bad, int32_t* n_nonfinite, double* fingerprint,
                    int64_t first, int64_t count) {
    double *px, *py;
    int nref;
    if (prm) {
        OM2 = problem == PDEVAL_PROBLEM_FORCE_FREE ? prm->omega2 : 0.0;
        OM2_LO = problem == PDEVAL_PROBLEM_FORCE_FREE ? prm->omega2_lo : 0.0;
    }
    int npts = build_points(problem, &px, &py, &nref);
    int G = npts - nref;
    int fp[PDEVAL_FP_N] = {0};
    for (int f = 1; f < PDEVAL_FP_N; ++f) fp[f] = nref + (int)((int64_t)G * f / PDEVAL_FP_N) + 7;
    int64_t last = (count < 0 || first + count > n) ? n : first + count;
    for (int64_t ci = first; ci < last; ++ci) {
        const int32_t* w = ops + offsets[ci];
        int64_t nw = offsets[ci + 1] - offsets[ci];
        int cls = -1, cplx = 0;
        double qr = 0, qmax = 0;
        int nb = 0, nnf = 0, nfin = 0, any_grad = 0, point_reject = 0, gconst = 1, point_nz = 0;
        if (nw < 2 || (w[0] & 0xff) != 0) cls = PDEVAL_CLS_BAD_PROGRAM;
        const uint32_t hdr = nw > 0 ? (uint32_t)w[0] : 0u;
        if (cls < 0 && (hdr & PDEVAL_FLAG_COMPLEX)) {
            if (problem == PDEVAL_PROBLEM_FORCE_FREE) cplx = 1;   /* complex-valued u */
            else cls = PDEVAL_CLS_REJECT_POINT;                   /* Kerr: non-real at a test point */
        }
    again:
        qr = 0; qmax = 0; nb = nnf = nfin = any_grad = point_reject = point_nz = 0; gconst = 1;
        for (int p = 0; p < npts && cls < 0; ++p) {
            int rc;
            pt_result r = eval_point(problem, w, nw, px[p], py[p], cplx, 0, &rc, p >= nref);
            if (rc == -2 || rc == -3) { cls = PDEVAL_CLS_UNSUPPORTED; break; }
            if (rc) { cls = PDEVAL_CLS_BAD_PROGRAM; break; }
            for (int f = 0; f < PDEVAL_FP_N; ++f)
                if (p == fp[f] && fingerprint) fingerprint[ci * PDEVAL_FP_N + f] = r.u0;
            if (p < nref) {
                if (r.finite && !r.grad_zero) any_grad = 1;
                /* the point stage, in quad precision (validator.py:349-402 / kerr :163-192):
                 * force-free rejects a residual that is certainly non-zero (beyond kappa x
                 * its noise bound) when it is rational (an exact Number != 0) or >= 1e-20;
                 * Kerr rejects max |lhs| >= 1e-10.  A residual certainly non-zero but below the
                 * threshold passes the point stage, but then the symbolic stage cannot reduce it
                 * to 0 (validator.py:404-427, kerr :283-315): point_nz */
                int rcq;
                pt_result q = eval_point_q(problem, w, nw, p, cplx, &rcq);
                if (rcq == -2 || rcq == -3) { cls = PDEVAL_CLS_UNSUPPORTED; break; }
                if (rcq) { cls = PDEVAL_CLS_BAD_PROGRAM; break; }
                /* a complex residual is reported as its modulus with the sign of its real part */
                if (res_ref) res_ref[ci * nref + p] = copysign(q.res_abs, q.res_re);
                /* Kerr constant exclusion (kerr validator.py:231-240: simplify(u) has neither r
                 * nor x): at every reference point the gradient is within its rounding bound */
                gconst = gconst && q.finite && !q.tiny &&
                         q.grad[0] <= prm->noise_kappa * (double)EPSQ * q.grad_err[0] &&
                         q.grad[1] <= prm->noise_kappa * (double)EPSQ * q.grad_err[1];
                if (!q.finite) {
                    if (problem == PDEVAL_PROBLEM_FORCE_FREE && !cplx) { cplx = 1; goto again; }
                    point_reject = 1;    /* non-finite at a reference point: final */
                } else if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
                    qr = scaled(q.res_abs, q.scale);
                    if (q.res_abs > prm->noise_kappa * q.noise) {
                        if ((hdr & PDEVAL_FLAG_RATIONAL) || q.res_abs >= prm->point_abs_tol) point_reject = 1;
                        else point_nz = 1;
                    }
                } else {
                    if (!(qr >= q.res_abs)) qr = q.res_abs;
                    if (q.tiny) { /* underflowed: a passing point */ }
                    else if (q.res_abs >= prm->kerr_abs_tol) point_reject = 1;
                    else if (q.res_abs > prm->noise_kappa * q.noise) point_nz = 1;
                }
                if (p == nref - 1 && point_reject && !prm->full_grid) cls = PDEVAL_CLS_REJECT_POINT;
                continue;
            }
            if (r.finite) {
                double q = scaled(r.res_abs, r.scale);
                ++nfin;
                if (q > qmax) qmax = q;
                if (grid_fails(r.res_abs, r.scale, prm->tau_grid)) ++nb;
                if (!r.grad_zero) any_grad = 1;
            } else {
                ++nnf;
            }
        }
        if (cls < 0 && !point_reject && nb > prm->max_bad) {
            /* tier 2 of the grid stage: count only points whose residual also exceeds its
             * rounding-noise bound */
            nb = 0;
            for (int p = nref; p < npts; ++p) {
                int rc2;
                pt_result r2 = eval_point(problem, w, nw, px[p], py[p], cplx, 1, &rc2, 1);
                if (rc2 || !r2.finite) continue;
                if (grid_fails(r2.res_abs, r2.scale, prm->tau_grid) && r2.res_abs > prm->noise_kappa * r2.noise) ++nb;
            }
        }
        if (cls < 0) {
            int structural = problem != PDEVAL_PROBLEM_FORCE_FREE || (hdr & PDEVAL_FLAG_NOCOORD);
            /* Kerr: no coordinate in the program is a constant structurally (kerr validator.py:
             * 231-240), else the numeric constant test */
            const int pconst = problem != PDEVAL_PROBLEM_FORCE_FREE &&
                               ((hdr & PDEVAL_FLAG_NOCOORD) || (gconst && kerr_constant_test(w, nw, prm->noise_kappa)));
            if (pconst) any_grad = 0;
            if (!any_grad && (nfin > 0 || pconst) && structural) cls = PDEVAL_CLS_ZERO_GRADIENT;
            else if (point_reject) cls = PDEVAL_CLS_REJECT_POINT;
            /* Kerr: no finite grid point proves nothing (the device's rule) */
            else if (problem != PDEVAL_PROBLEM_FORCE_FREE && nfin == 0) cls = PDEVAL_CLS_REJECT_GRID;
            else if (nb > prm->max_bad) cls = PDEVAL_CLS_REJECT_GRID;
            else if (problem == PDEVAL_PROBLEM_FORCE_FREE && prm->strict_symbolic &&
                     (hdr & (PDEVAL_FLAG_NONSMOOTH2D | PDEVAL_FLAG_UNPROVABLE))) cls = PDEVAL_CLS_REJECT_SYMBOLIC;
            else if (point_nz) cls = PDEVAL_CLS_REJECT_GRID;   /* residual != 0 identically */
            else cls = PDEVAL_CLS_ACCEPT;
        }
        if (status) status[ci] = (uint8_t)cls;
        if (q_ref) q_ref[ci] = qr;
        if (q_grid) q_grid[ci] = qmax;
        if (n_bad) n_bad[ci] = nb;
        if (n_nonfinite) n_nonfinite[ci] = nnf;
    }
    free(px);
    free(py);
    return 0;
}

/* u and its Taylor jet at one point (for unit tests). */
int oracle_jet(int problem, const int32_t* w, int64_t nw, double x, double y, int cplx, double* re,
               double* im) {
    const int K = problem == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
    double complex cc[NCMAX];
    int rc;
    if (cplx) {
        kc_default();
        rc = run_c(w, nw, x, y, K, 1, cc, NULL, 0.0, KC.prm_g);
    } else {
        double cr[NCMAX];
        kc_default();
        rc = run_r(w, nw, x, y, K, 0, cr, NULL, 0.0, KC.prm_g);
        for (int i = 0; i < NC(K); ++i) cc[i] = cr[i];
    }
    for (int i = 0; i < NC(K) && !rc; ++i) { re[i] = creal(cc[i]); im[i] = cimag(cc[i]); }
    return rc;
}

/* One point with the tier-2 noise bound: out = {|res|, S, noise, finite} (for unit tests and
 * threshold calibration). */
int oracle_point(int problem, const int32_t* w, int64_t nw, double x, double y, int cplx, double* out) {
    int rc;
    pt_result r = eval_point(problem, w, nw, x, y, cplx, 1, &rc, 1);
    out[0] = r.res_abs;
    out[1] = r.scale;
    out[2] = r.noise;
    out[3] = r.finite;
    return rc;
}
