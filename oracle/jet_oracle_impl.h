/* jet_oracle_impl.h -- scalar-type-generic part of the CPU oracle (included three times by
 * jet_oracle.c: S = double for the real pass, S = double complex for the complex pass, and
 * S = __complex128 with quad-precision coordinates and constants (CT = __float128) for the
 * point stage, which the reference decides in exact arithmetic).  TEST INFRASTRUCTURE ONLY:
 * never linked into libpdeval.
 * Per instantiation the includer defines S, CT (coordinate / constant type), FN(name) and the
 * math macros CABS CREAL CIMAG CEXP CLOG RPOW REXP RLOG RFLOOR CI (the imaginary unit).
 *
 * Derivatives are taken by truncated bivariate Taylor arithmetic (the same mathematics as
 * sp.diff in problems/force_free/validator.py:305-344, evaluated at a point instead of
 * symbolically); the residual operators are then written out as CLOSED FORMS in the partial
 * derivatives u_ij (not as jets, as the device epilogue does), so the oracle checks the
 * device's epilogue as well as its interpreter.
 */

/* ---------- jets: c[IDX(i,j)], i + j <= KMAX, degree-major ---------- */
static void FN(jconst)(S* t, S v) { for (int i = 0; i < NCMAX; ++i) t[i] = 0; t[0] = v; }

static void FN(jmul)(const S* a, const S* b, S* c, int K) {
    S r[NCMAX];
    for (int d = 0; d <= K; ++d)
        for (int j = 0; j <= d; ++j) {
            S s = 0;
            for (int d1 = 0; d1 <= d; ++d1)
                for (int j1 = 0; j1 <= d1; ++j1) {
                    int d2 = d - d1, j2 = j - j1;
                    if (j2 < 0 || j2 > d2) continue;
                    s += a[IDX(d1 - j1, j1)] * b[IDX(d2 - j2, j2)];
                }
            r[IDX(d - j, j)] = s;
        }
    memcpy(c, r, sizeof(S) * NC(K));
}

static void FN(jdiv)(const S* a, const S* b, S* c, int K) {  /* c = a / b */
    S r[NCMAX];
    for (int d = 0; d <= K; ++d)
        for (int j = 0; j <= d; ++j) {
            S s = a[IDX(d - j, j)];
            for (int d1 = 1; d1 <= d; ++d1)
                for (int j1 = 0; j1 <= d1; ++j1) {
                    int d2 = d - d1, j2 = j - j1;
                    if (j2 < 0 || j2 > d2) continue;
                    s -= b[IDX(d1 - j1, j1)] * r[IDX(d2 - j2, j2)];
                }
            r[IDX(d - j, j)] = s / b[0];
        }
    memcpy(c, r, sizeof(S) * NC(K));
}

/* x <- f(x) for f with Taylor coefficients f[0..K] at x[0]: sum_k f_k h^k, h = x - x0,
 * by explicit powers of h (the device uses Horner: a different evaluation order) */
static void FN(jcompose)(S* x, const S* f, int K) {
    S h[NCMAX], hk[NCMAX], acc[NCMAX];
    memcpy(h, x, sizeof(S) * NC(K));
    h[0] = 0;
    FN(jconst)(acc, f[0]);
    FN(jconst)(hk, 1);
    for (int k = 1; k <= K; ++k) {
        FN(jmul)(hk, h, hk, K);
        for (int i = 0; i < NC(K); ++i) acc[i] += f[k] * hk[i];
    }
    memcpy(x, acc, sizeof(S) * NC(K));
}

/* principal-branch x0**alpha, with the real pass undefined off the real domain */
static S FN(spow)(S x, double a, int cplx_pass) {
    if (!cplx_pass) {
        CT xr = CREAL(x);
        if (a == floor(a)) return RPOW(xr, (CT)a);
        if (xr < 0) return NAN;
        return RPOW(xr, (CT)a);
    }
    if (x == 0) return a > 0 ? 0 : INFINITY;
    return CEXP((CT)a * CLOG(x));
}

static void FN(wabs)(const S* v, double* w, int K) { for (int i = 0; i < NC(K); ++i) w[i] = (double)CABS(v[i]); }

/* Evaluate a program at (px, py).  eout != NULL: also carry the first-order rounding-error
 * jet E (rules at w_mul in jet_oracle.c) and return it. */
/* cerr: relative rounding of the coordinates in noise units (0 on the exact grid points);
 * prm: the stage's values of the problem's constants {M, a, 1/M, 1/a} (PDEVAL_IMM_PRM) */
static int FN(run)(const int32_t* w, int64_t nw, CT px, CT py, int K, int cplx_pass, S* out,
                   double* eout, double cerr, const CT* prm) {
    S st[16][NCMAX];
    double es[16][NCMAX];
    const int trk = eout != NULL;
    int d = 0;
    for (int64_t pc = 1; pc < nw;) {
        uint32_t word = (uint32_t)w[pc], op = word & 0xffu;
        CT imm = 0;
        if ((word & PDEVAL_IMM_PRM) && (op == PDOP_PUSH_C || op == PDOP_ADDC || op == PDOP_MULC || op == PDOP_RDIVC)) {
            /* one of the problem's constants: descriptor word, then 0 */
            if (pc + 2 >= nw || (word & PDEVAL_IMM_DD)) return -1;
            const uint32_t dsc = (uint32_t)w[pc + 1];
            if (dsc > 15u || w[pc + 2] != 0) return -1;
            imm = prm[dsc & 7u];
            if (dsc & PDEVAL_PRM_NEG) imm = -imm;
            pc += 3;
        } else if (op == PDOP_PUSH_C || op == PDOP_ADDC || op == PDOP_MULC || op == PDOP_RDIVC || op == PDOP_POW) {
            if (word & PDEVAL_IMM_PRM) return -1;      /* (never an exponent) */
            const int nimm = (word & PDEVAL_IMM_DD) ? 2 : 1;
            if (pc + 2 * nimm >= nw + 1) return -1;
            for (int k = 0; k < nimm; ++k) {
                double v;
                uint64_t bits = (uint64_t)(uint32_t)w[pc + 1 + 2 * k] | ((uint64_t)(uint32_t)w[pc + 2 + 2 * k] << 32);
                memcpy(&v, &bits, 8);
                /* the double-double low part matters only where constants are wider than f64 */
                if (k == 0 || sizeof(CT) > sizeof(double)) imm += (CT)v;
            }
            pc += 1 + 2 * nimm;
        } else {
            pc += 1;
        }
        const double immd = (double)imm;
        S* t = d > 0 ? st[d - 1] : NULL;
        S* u = d > 1 ? st[d - 2] : NULL;
        double* et = d > 0 ? es[d - 1] : NULL;
        double* eu = d > 1 ? es[d - 2] : NULL;
        S f[KMAX + 2];
        double A[NCMAX], B[NCMAX], R[NCMAX], T1[NCMAX], T2[NCMAX];
        switch (op) {
            case PDOP_PUSH_X: case PDOP_PUSH_Y: case PDOP_PUSH_C: case PDOP_PUSH_I:
                if (op == PDOP_PUSH_X) { FN(jconst)(st[d], px); st[d][IDX(1, 0)] = 1; }
                else if (op == PDOP_PUSH_Y) { FN(jconst)(st[d], py); st[d][IDX(0, 1)] = 1; }
                else if (op == PDOP_PUSH_C) FN(jconst)(st[d], imm);
                else { if (!cplx_pass) return -2; FN(jconst)(st[d], CI); }
                if (trk) {
                    for (int i = 0; i < NCMAX; ++i) es[d][i] = 0;
                    if (op == PDOP_PUSH_C) es[d][0] = fabs(immd);
                    else if (op == PDOP_PUSH_X) es[d][0] = fabs((double)px) * cerr;
                    else if (op == PDOP_PUSH_Y) es[d][0] = fabs((double)py) * cerr;
                }
                ++d;
                break;
            case PDOP_ADD: case PDOP_SUB: case PDOP_RSUB:
                for (int i = 0; i < NC(K); ++i)
                    u[i] = op == PDOP_ADD ? u[i] + t[i] : (op == PDOP_SUB ? u[i] - t[i] : t[i] - u[i]);
                if (trk) for (int i = 0; i < NC(K); ++i) eu[i] += et[i] + (double)CABS(u[i]);
                --d;
                break;
            case PDOP_MUL:
                if (trk) {
                    FN(wabs)(u, A, K); FN(wabs)(t, B, K);
                    w_mul(A, et, T1, K); w_mul(eu, B, T2, K); w_mul(A, B, R, K);
                    for (int i = 0; i < NC(K); ++i) eu[i] = T1[i] + T2[i] + R[i];
                }
                FN(jmul)(u, t, u, K);
                --d;
                break;
            case PDOP_DIV: case PDOP_RDIV: {
                const double* en = op == PDOP_DIV ? eu : et;
                const double* ed = op == PDOP_DIV ? et : eu;
                if (trk) { memcpy(T1, en, sizeof T1); memcpy(T2, ed, sizeof T2); FN(wabs)(op == PDOP_DIV ? t : u, B, K); }
                FN(jdiv)(op == PDOP_DIV ? u : t, op == PDOP_DIV ? t : u, u, K);
                if (trk) {
                    FN(wabs)(u, R, K);
                    w_mul(R, T2, A, K);
                    for (int i = 0; i < NC(K); ++i) A[i] += T1[i];
                    w_absdiv(A, B, eu, K);
                    for (int i = 0; i < NC(K); ++i) eu[i] += R[i];
                }
                --d;
                break;
            }
            case PDOP_ADDC: t[0] += imm; if (trk) et[0] += fabs(immd) + (double)CABS(t[0]); break;
            case PDOP_MULC:
                for (int i = 0; i < NC(K); ++i) t[i] *= imm;
                if (trk) for (int i = 0; i < NC(K); ++i) et[i] = et[i] * fabs(immd) + (double)CABS(t[i]);
                break;
            case PDOP_RDIVC: {
                S c[NCMAX];
                FN(jconst)(c, imm);
                if (trk) { memcpy(T2, et, sizeof T2); FN(wabs)(t, B, K); }
                FN(jdiv)(c, t, t, K);
                if (trk) {
                    FN(wabs)(t, R, K);
                    w_mul(R, T2, A, K);
                    A[0] += fabs(immd);
                    w_absdiv(A, B, et, K);
                    for (int i = 0; i < NC(K); ++i) et[i] += R[i];
                }
                break;
            }
            case PDOP_PUSH_P: case PDOP_ADD_P: case PDOP_SUB_P: case PDOP_MUL_P: case PDOP_DIV_P:
            case PDOP_RDIV_P: {
                /* p = v**n (v = x or y): its jet by repeated jet products of the coordinate
                 * (the device uses the closed form C(n,k) v^(n-k)); E_p = n |p| */
                const int n = (int)((word >> 8) & 0xffu), ax = (int)((word >> 16) & 1u);
                S v[NCMAX], pj[NCMAX];
                double ep[NCMAX], P_[NCMAX];
                FN(jconst)(v, ax ? py : px);
                v[ax ? IDX(0, 1) : IDX(1, 0)] = 1;
                memcpy(pj, v, sizeof pj);
                for (int k = 1; k < n; ++k) FN(jmul)(pj, v, pj, K);
                if (trk) { FN(wabs)(pj, P_, K); for (int i = 0; i < NC(K); ++i) ep[i] = n * P_[i] * (1 + cerr); }
                if (op == PDOP_PUSH_P) {
                    memcpy(st[d], pj, sizeof(S) * NCMAX);
                    if (trk) memcpy(es[d], ep, sizeof(double) * NCMAX);
                    ++d;
                } else if (op == PDOP_ADD_P || op == PDOP_SUB_P) {
                    for (int i = 0; i < NC(K); ++i) t[i] = op == PDOP_ADD_P ? t[i] + pj[i] : t[i] - pj[i];
                    if (trk) for (int i = 0; i < NC(K); ++i) et[i] += ep[i] + (double)CABS(t[i]);
                } else if (op == PDOP_MUL_P) {
                    if (trk) {
                        FN(wabs)(t, A, K);
                        w_mul(A, ep, T1, K); w_mul(et, P_, T2, K); w_mul(A, P_, R, K);
                        for (int i = 0; i < NC(K); ++i) et[i] = T1[i] + T2[i] + R[i];
                    }
                    FN(jmul)(t, pj, t, K);
                } else {
                    /* DIV_P: t = t / p (num t, den p);  RDIV_P: t = p / t (num p, den t) */
                    const int dv = op == PDOP_DIV_P;
                    double en[NCMAX], ed[NCMAX];
                    if (trk) {
                        memcpy(en, dv ? et : ep, sizeof en);
                        memcpy(ed, dv ? ep : et, sizeof ed);
                        if (dv) memcpy(B, P_, sizeof B); else FN(wabs)(t, B, K);
                    }
                    if (dv) FN(jdiv)(t, pj, t, K); else FN(jdiv)(pj, t, t, K);
                    if (trk) {
                        FN(wabs)(t, R, K);
                        w_mul(R, ed, A, K);
                        for (int i = 0; i < NC(K); ++i) A[i] += en[i];
                        w_absdiv(A, B, et, K);
                        for (int i = 0; i < NC(K); ++i) et[i] += R[i];
                    }
                }
                break;
            }
            case PDOP_NEG: for (int i = 0; i < NC(K); ++i) t[i] = -t[i]; break;
            case PDOP_ADD_X: t[0] += px; t[IDX(1, 0)] += 1; if (trk) et[0] += (double)CABS(t[0]) + fabs((double)px) * cerr; break;
            case PDOP_ADD_Y: t[0] += py; t[IDX(0, 1)] += 1; if (trk) et[0] += (double)CABS(t[0]) + fabs((double)py) * cerr; break;
            case PDOP_SUB_X: t[0] -= px; t[IDX(1, 0)] -= 1; if (trk) et[0] += (double)CABS(t[0]) + fabs((double)px) * cerr; break;
            case PDOP_SUB_Y: t[0] -= py; t[IDX(0, 1)] -= 1; if (trk) et[0] += (double)CABS(t[0]) + fabs((double)py) * cerr; break;
            case PDOP_MUL_X: case PDOP_MUL_Y: case PDOP_DIV_X: case PDOP_DIV_Y: {
                S v[NCMAX];
                int isx = (op == PDOP_MUL_X || op == PDOP_DIV_X);
                FN(jconst)(v, isx ? px : py);
                v[isx ? IDX(1, 0) : IDX(0, 1)] = 1;
                if (trk) { FN(wabs)(v, B, K); memcpy(T1, et, sizeof T1); }
                if (op == PDOP_MUL_X || op == PDOP_MUL_Y) {
                    double cv[NCMAX];
                    if (trk) { FN(wabs)(t, cv, K); for (int i = 0; i < NC(K); ++i) cv[i] *= B[0] * cerr; }
                    FN(jmul)(t, v, t, K);
                    if (trk) { w_mul(T1, B, et, K); FN(wabs)(t, R, K); for (int i = 0; i < NC(K); ++i) et[i] += R[i] + cv[i]; }
                } else {
                    FN(jdiv)(t, v, t, K);
                    if (trk) {
                        FN(wabs)(t, R, K); w_absdiv(T1, B, et, K);
                        for (int i = 0; i < NC(K); ++i) et[i] += R[i] + R[i] * cerr * (K + 1);
                    }
                }
                break;
            }
            case PDOP_POWN: {
                int n = (int)((word >> 8) & 0xffu);
                S b[NCMAX];
                double eb[NCMAX];
                memcpy(b, t, sizeof(S) * NC(K));
                if (trk) { memcpy(eb, et, sizeof eb); FN(wabs)(b, B, K); }
                for (int k = 1; k < n; ++k) {
                    if (trk) {
                        FN(wabs)(t, A, K);
                        w_mul(A, eb, T1, K); w_mul(et, B, T2, K); w_mul(A, B, R, K);
                        for (int i = 0; i < NC(K); ++i) et[i] = T1[i] + T2[i] + R[i];
                    }
                    FN(jmul)(t, b, t, K);
                }
                break;
            }
            case PDOP_POW: case PDOP_SQRT: case PDOP_EXP: case PDOP_LOG: {
                S x0 = t[0];
                if (op == PDOP_POW || op == PDOP_SQRT) {
                    double a = (op == PDOP_SQRT) ? 0.5 : immd;
                    f[0] = FN(spow)(x0, a, cplx_pass);
                    for (int k = 1; k <= K + 1; ++k) f[k] = f[k - 1] * ((CT)(a - (k - 1)) / k) / x0;
                } else if (op == PDOP_EXP) {
                    S e = cplx_pass ? CEXP(x0) : REXP(CREAL(x0));
                    CT fact = 1;
                    for (int k = 0; k <= K + 1; ++k) { if (k) fact *= k; f[k] = e / fact; }
                } else {
                    f[0] = cplx_pass ? CLOG(x0) : (CREAL(x0) > 0 ? RLOG(CREAL(x0)) : (CREAL(x0) == 0 ? -INFINITY : NAN));
                    for (int k = 1; k <= K + 1; ++k) f[k] = (CT)((k & 1) ? 1.0 : -1.0) / (k * FN(spow)(x0, k, cplx_pass));
                }
                if (trk) {
                    double G[KMAX + 1], Fa[KMAX + 1];
                    for (int k = 0; k <= K; ++k) { G[k] = (k + 1) * (double)CABS(f[k + 1]); Fa[k] = (double)CABS(f[k]); }
                    FN(wabs)(t, A, K);
                    w_horner(A, G, T1, K);         /* G1 = sum (m+1)|f_(m+1)| |h|^m */
                    w_horner(A, Fa, R, K);         /* sum |f_k| |h|^k */
                    w_mul(T1, et, T2, K);
                    for (int i = 0; i < NC(K); ++i) et[i] = T2[i] + R[i];
                }
                FN(jcompose)(t, f, K);
                break;
            }
            case PDOP_ABS: {
                double sg;
                if (CIMAG(t[0]) != 0) sg = NAN;
                else sg = CREAL(t[0]) > 0 ? 1 : (CREAL(t[0]) < 0 ? -1 : NAN);
                for (int i = 0; i < NC(K); ++i) t[i] *= sg;
                break;
            }
            case PDOP_UNSUPPORTED: return -3;
            default: return -3;
        }
        if (d > 15 || d < 1) return -4;
    }
    if (d != 1) return -5;
    memcpy(out, st[0], sizeof(S) * NC(K));
    if (trk) memcpy(eout, es[0], sizeof(double) * NC(K));
    return 0;
}

/* partial derivative u_{ij} = i! j! c_ij */
static S FN(partial)(const S* c, int i, int j) {
    static const double fct[5] = {1, 1, 2, 6, 24};
    return c[IDX(i, j)] * (fct[i] * fct[j]);
}

/* Force-free determinant in closed form from partials (validator.py:323-347; OM2 = Omega^2,
 * 0 on the problem path).
 * mag != 0: every term replaced by its magnitude (the scale S). */
static S FN(ff_det)(const S* c, CT rho, int mag) {
#define M_(x) (mag ? (S)CABS(x) : (x))
#define SUB_(a, b) (mag ? ((a) + (b)) : ((a) - (b)))
    S u10 = M_(FN(partial)(c, 1, 0)), u01 = M_(FN(partial)(c, 0, 1));
    S u20 = M_(FN(partial)(c, 2, 0)), u11 = M_(FN(partial)(c, 1, 1)), u02 = M_(FN(partial)(c, 0, 2));
    S u30 = M_(FN(partial)(c, 3, 0)), u21 = M_(FN(partial)(c, 2, 1)), u12 = M_(FN(partial)(c, 1, 2));
    S u03 = M_(FN(partial)(c, 0, 3));
    S u40 = M_(FN(partial)(c, 4, 0)), u31 = M_(FN(partial)(c, 3, 1)), u22 = M_(FN(partial)(c, 2, 2));
    S u13 = M_(FN(partial)(c, 1, 3)), u04 = M_(FN(partial)(c, 0, 4));
    CT r1 = 1 / rho, r2 = r1 * r1, r3 = r2 * r1;
    S p = u10, q = u01;
    /* A = u20 + u02 - u10/rho and its partials */
    S Ar = u30 + u12 + SUB_(0, u20 * r1) + u10 * r2;
    S Az = u21 + SUB_(u03, u11 * r1);
    S Arr = u40 + u22 + SUB_(0, u30 * r1) + 2 * u20 * r2 + SUB_(0, 2 * u10 * r3);
    S Arz = u31 + u13 + SUB_(0, u21 * r1) + u11 * r2;
    S Azz = u22 + SUB_(u04, u12 * r1);
    /* B = p^2 + q^2 */
    S Br = 2 * (p * u20 + q * u11);
    S Bz = 2 * (p * u11 + q * u02);
    S Brr = 2 * (u20 * u20 + p * u30 + u11 * u11 + q * u21);
    S Brz = 2 * (u11 * u20 + p * u21 + u02 * u11 + q * u12);
    S Bzz = 2 * (u11 * u11 + p * u12 + u02 * u02 + q * u03);
    if (OM2 != 0) {
        /* rotating field lines, constant Omega (validator.py:326-329): with w = Omega^2,
         * A = A_0 - w C,  C = rho^2 (u20 + u02) + rho u10;  B = (1 - w rho^2) B_0 -- the
         * partials of both written out (the device does it on jets, ff_rotate_A / _B) */
        const CT w = (CT)OM2 + (CT)OM2_LO, x = rho, x2 = rho * rho;   /* (f64: = OM2) */
        S Cr = 2 * x * (u20 + u02) + x2 * (u30 + u12) + u10 + x * u20;
        S Cz = x2 * (u21 + u03) + x * u11;
        S Crr = 2 * (u20 + u02) + 4 * x * (u30 + u12) + x2 * (u40 + u22) + 2 * u20 + x * u30;
        S Crz = 2 * x * (u21 + u03) + x2 * (u31 + u13) + u11 + x * u21;
        S Czz = x2 * (u22 + u04) + x * u12;
        Ar = SUB_(Ar, w * Cr);
        Az = SUB_(Az, w * Cz);
        Arr = SUB_(Arr, w * Crr);
        Arz = SUB_(Arz, w * Crz);
        Azz = SUB_(Azz, w * Czz);
        const S B0 = p * p + q * q;
        S Brr2 = SUB_(Brr, w * (2 * B0 + 4 * x * Br + x2 * Brr));
        S Brz2 = SUB_(Brz, w * (2 * x * Bz + x2 * Brz));
        S Bzz2 = SUB_(Bzz, w * (x2 * Bzz));
        S Br2 = SUB_(Br, w * (2 * x * B0 + x2 * Br));
        S Bz2 = SUB_(Bz, w * (x2 * Bz));
        Br = Br2; Bz = Bz2; Brr = Brr2; Brz = Brz2; Bzz = Bzz2;
    }
    /* L_T f = q f_r - p f_z;  L_T^2 f = q (L_T f)_r - p (L_T f)_z */
    S LA = SUB_(q * Ar, p * Az), LB = SUB_(q * Br, p * Bz);
    S LAr = SUB_(u11 * Ar + q * Arr, u20 * Az + p * Arz);
    S LAz = SUB_(u02 * Ar + q * Arz, u11 * Az + p * Azz);
    S LBr = SUB_(u11 * Br + q * Brr, u20 * Bz + p * Brz);
    S LBz = SUB_(u02 * Br + q * Brz, u11 * Bz + p * Bzz);
    S L2A = SUB_(q * LAr, p * LAz), L2B = SUB_(q * LBr, p * LBz);
    return SUB_(LA * L2B, LB * L2A);
#undef M_
#undef SUB_
}
