// pdeval_tier2.h -- tier 2 of the zero test: re-decide tier-1 failures with error bounds.
//
// Tier 1 (validate_kernel) rejects a sample point when the scaled residual q = |res| / S
// exceeds a threshold.  S bounds the magnitude of the residual's monomials, but not the
// rounding noise of the jet coefficients they are built from: a true solution whose jets
// carry noise in coefficients that are exactly zero (u = z*(-(rho/z + 1)) = -rho - z, whose
// second derivatives are rounding noise) or that sits near a pole can show q ~ 1 at some
// points.  The reference decides these exactly (problems/force_free/validator.py:349-427),
// so every tier-1 failure is re-evaluated here with a first-order running error bound E
// carried beside every jet (|computed - exact| <~ eps * E, coefficient-wise):
//   leaf x, y : 0          constant c : |c|
//   a +- b    : E_a + E_b + |r|
//   a * b     : |a| (*) (E_b + |b|) + E_a (*) |b|          ((*) = jet product)
//   a / b     : absdiv(E_a + |r| (*) E_b, |b|) + |r|
//   g(a)      : G1 (*) E_a + sum_k |f_k| |h|^k,   G1 = sum_m (m+1) |f_(m+1)| |h|^m
// (absdiv = the division recurrence with every sign positive).  The residual's noise is the
// first-order sensitivity of the magnitude epilogue: noise = (S(|u| + g E) - S(|u|)) eps/g
// + eps S.  A point fails in tier 2 only if it fails tier 1 AND |res| > noise_kappa * noise.
// The CPU oracle (oracle/jet_oracle_impl.h) carries the same bound.
#pragma once
#include "pdeval_kernels.h"

namespace pd {

constexpr double kNoiseGamma = 0x1p-30;
constexpr double kEps = 0x1p-52;

template <int K> struct EJ {
    static constexpr int NC = nc(K);
    // c = a (*) b, non-negative jets (c may alias a or b)
    static PD_HD void mul(const double* a, const double* b, double* c) {
        double r[NC];
        jmul<double, K, K, K>(a, b, r);
#pragma unroll
        for (int i = 0; i < NC; ++i) c[i] = r[i];
    }
    // c = absdiv(n, b): c_k = (n_k + sum_{j>=1} b_j c_(k-j)) / b_0  (c may alias n)
    static PD_HD void absdiv(const double* n, const double* b, double* c) {
        const double inv = 1.0 / b[0];
#pragma unroll
        for (int d = 0; d <= K; ++d)
#pragma unroll
            for (int j = 0; j <= d; ++j) {
                double s = n[ji(d - j, j)];
#pragma unroll
                for (int d1 = 1; d1 <= d; ++d1)
#pragma unroll
                    for (int j1 = 0; j1 <= d1; ++j1) {
                        const int d2 = d - d1, j2 = j - j1;
                        if (j2 < 0 || j2 > d2) continue;
                        s = fma(b[ji(d1 - j1, j1)], c[ji(d2 - j2, j2)], s);
                    }
                c[ji(d - j, j)] = s * inv;
            }
    }
    template <class T> static PD_HD void absv(const T* v, double* w) {
#pragma unroll
        for (int i = 0; i < NC; ++i) w[i] = mag(v[i]);
    }
    template <class T> static PD_HD void add_abs(const T* v, double* e) {
#pragma unroll
        for (int i = 0; i < NC; ++i) e[i] += mag(v[i]);
    }
};

// Taylor coefficients f[0..K+1] of the outer function of a composition opcode at x0, as the
// tier-1 JetOps compute f[0..K] (the value path itself is JetOps, unchanged).
template <class T, int K> __device__ __forceinline__ void outer_coefs(uint32_t op, T x0, double alpha, T* f) {
    if (op == PDOP_EXP) {
        f[0] = exp_(x0);
#pragma unroll
        for (int k = 1; k <= K + 1; ++k) f[k] = divk(f[k - 1], 1.0, k);
    } else if (op == PDOP_LOG) {
        const T r = recip(x0);
        f[0] = log_(x0);
        T rk = r;
#pragma unroll
        for (int k = 1; k <= K + 1; ++k) {
            f[k] = divk(rk, (k & 1) ? 1.0 : -1.0, k);
            rk = rk * r;
        }
    } else {
        const double a = op == PDOP_SQRT ? 0.5 : alpha;
        const T f0 = op == PDOP_SQRT ? sqrt_(x0) : pow_real_exp(x0, a);
        const T r = recip(x0);
        f[0] = f0;
#pragma unroll
        for (int k = 1; k <= K + 1; ++k) f[k] = divk(f[k - 1] * r, a - (k - 1), k);
    }
}

// Operand-stack storage of the error-bounded interpreter (slots below the top of stack):
//   LdsStack   per wave in LDS, [slot][coef][lane] (one wave = one candidate, or one candidate
//              per lane with MAXD = 2)
//   PrivStack  per lane in private memory (the compiler places it in scratch: dynamic slot
//              index), for the rare list-driven point kernels of deep / complex / dd programs
template <class T, int NC> struct LdsStack {
    T* vs;
    double* es;
    int lane;
    __device__ __forceinline__ void store(int slot, const T* t, const double* e) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            vs[(slot * NC + c) * 64 + lane] = t[c];
            es[(slot * NC + c) * 64 + lane] = e[c];
        }
    }
    __device__ __forceinline__ void load(int slot, T* t, double* e) const {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            t[c] = vs[(slot * NC + c) * 64 + lane];
            e[c] = es[(slot * NC + c) * 64 + lane];
        }
    }
};
template <class T, int NC, int SLOTS> struct PrivStack {
    T v[SLOTS][NC];
    double e[SLOTS][NC];
    __device__ __forceinline__ void store(int slot, const T* t, const double* ee) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            v[slot][c] = t[c];
            e[slot][c] = ee[c];
        }
    }
    __device__ __forceinline__ void load(int slot, T* t, double* ee) const {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            t[c] = v[slot][c];
            ee[c] = e[slot][c];
        }
    }
};

// Immediate of an opcode as the coordinate type V: the f64 word pair, plus the double-double
// low part when the opcode carries PDEVAL_IMM_DD and V = dd.
template <class V, bool VEC> __device__ __forceinline__ V read_imm(const int32_t* p, uint32_t w,
                                                                  const PrmTab<V>& P) {
    if (w & PDEVAL_IMM_PRM) {   // one of the problem's constants: the stage's value
        if constexpr (VEC) return prm_value(P, (uint32_t)p[0]);
        else return prm_value(P, rd_word(p));
    }
    double hi, lo = 0.0;
    if constexpr (VEC) {
        hi = __hiloint2double(p[1], p[0]);
        if constexpr (!std::is_same<V, double>::value)
            if (w & PDEVAL_IMM_DD) lo = __hiloint2double(p[3], p[2]);
    } else {
        hi = rd_imm(p);
        if constexpr (!std::is_same<V, double>::value)
            if (w & PDEVAL_IMM_DD) lo = rd_imm(p + 2);
    }
    if constexpr (std::is_same<V, double>::value) {
        (void)w;
        return hi;
    } else {
        return V{hi, lo};
    }
}

template <class T, int K, int MAXD, class V = double> struct ErrInterp {
    using O = JetOps<T, K>;
    using J = typename O::J;
    using E = EJ<K>;
    static constexpr int NC = nc(K);

    // binary op t = a (op) t with error bounds (a = lhs with bound el), op in ADD..RDIV
    static __device__ __forceinline__ void binop_e(uint32_t op, const J& lhs, const double* el, J& acc, double* ea) {
        double A[NC], B[NC], R[NC];
        if (op == PDOP_ADD || op == PDOP_SUB || op == PDOP_RSUB) {
            Interp<T, K, MAXD>::binop(op, lhs, acc);
#pragma unroll
            for (int i = 0; i < NC; ++i) ea[i] += el[i];
            E::add_abs(acc.c, ea);
        } else if (op == PDOP_MUL) {
            // |a| (*) (E_t + |t|) + E_a (*) |t|
            E::absv(lhs.c, A);
            E::absv(acc.c, B);
#pragma unroll
            for (int i = 0; i < NC; ++i) R[i] = ea[i] + B[i];
            E::mul(A, R, R);
            E::mul(el, B, A);
#pragma unroll
            for (int i = 0; i < NC; ++i) ea[i] = R[i] + A[i];
            O::mul(lhs, acc);
        } else {
            // DIV: t = a / t (num a, den t);  RDIV: t = t / a (num t, den a)
            const bool dv = op == PDOP_DIV;
            E::absv(dv ? acc.c : lhs.c, B);            // |den|
            double en[NC];
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                en[i] = dv ? el[i] : ea[i];            // E_num
                A[i] = dv ? ea[i] : el[i];             // E_den
            }
            Interp<T, K, MAXD>::binop(op, lhs, acc);
            E::absv(acc.c, R);
            E::mul(R, A, A);
#pragma unroll
            for (int i = 0; i < NC; ++i) A[i] += en[i];
            E::absdiv(A, B, ea);
#pragma unroll
            for (int i = 0; i < NC; ++i) ea[i] += R[i];
        }
    }

    // value + error bound of program words [pc, end) at (x, y)
    // VEC: the program is per lane (one candidate per lane): vector loads; otherwise it is
    // wave-uniform and read through the scalar cache.  STK: LdsStack / PrivStack.
    // cerr: relative rounding error of the coordinates in noise units (0: exact grid points;
    // the reference points 4/5, 6/7, 1/3 ... are not doubles, and near a pole of the candidate
    // their rounding is amplified like any other error)
    template <bool VEC, class STK>
    static __device__ PD_T2_INLINE_ATTR int run_s(const int32_t* ops, int pc, int end, V x, V y, J& acc, double* ea, STK& stk,
                                const PrmTab<V>& P, double cerr = 0.0) {
        int d = 0;
        if (pc >= end) return RUN_BAD;
        for (;;) {
            uint32_t w;
            if constexpr (VEC) w = (uint32_t)ops[pc];
            else w = rd_word(ops + pc);
            const uint32_t op = w & 0xffu;
            V immv = vzero<V>();
            double imm = 0.0;
            int npc = pc + 1;
            if (op_has_imm(op)) {
                npc = pc + ((w & PDEVAL_IMM_DD) ? 5 : 3);
                if (npc > end) return RUN_BAD;
                immv = read_imm<V, VEC>(ops + pc + 1, w, P);
                imm = hi_of(immv);
            }
            double A[NC], B[NC], R[NC];
            switch (op) {
                case PDOP_PUSH_X: case PDOP_PUSH_Y: case PDOP_PUSH_C: case PDOP_PUSH_I: {
                    if (d > 0 && d < MAXD) stk.store(d - 1, acc.c, ea);
                    if (op == PDOP_PUSH_X) O::set_var(acc, x, 0);
                    else if (op == PDOP_PUSH_Y) O::set_var(acc, y, 1);
                    else if (op == PDOP_PUSH_C) O::set_const(acc, cvt<T>(immv));
                    else {
                        if constexpr (Real<T>::cplx_pass) O::set_const(acc, imag_unit<T>());
                        else return RUN_UNSUPPORTED;
                    }
#pragma unroll
                    for (int i = 0; i < NC; ++i) ea[i] = 0.0;
                    if (op == PDOP_PUSH_C) ea[0] = fabs(imm);
                    else if (op == PDOP_PUSH_X) ea[0] = vabs(x) * cerr;
                    else if (op == PDOP_PUSH_Y) ea[0] = vabs(y) * cerr;
                    ++d;
                    break;
                }
                case PDOP_ADD: case PDOP_SUB: case PDOP_RSUB:
                case PDOP_MUL: case PDOP_DIV: case PDOP_RDIV: {
                    if (d >= 2 && d <= MAXD) {
                        J lhs;
                        double el[NC];
                        stk.load(d - 2, lhs.c, el);
                        binop_e(op, lhs, el, acc, ea);
                    }
                    --d;
                    break;
                }
                case PDOP_ADDC:
                    acc.c[0] = acc.c[0] + cvt<T>(immv);
                    ea[0] += fabs(imm) + mag(acc.c[0]);
                    break;
                case PDOP_MULC:
                    O::scale(acc, cvt<T>(immv));
#pragma unroll
                    for (int i = 0; i < NC; ++i) ea[i] = ea[i] * fabs(imm) + mag(acc.c[i]);
                    break;
                case PDOP_RDIVC: {
                    E::absv(acc.c, B);
#pragma unroll
                    for (int i = 0; i < NC; ++i) A[i] = ea[i];
                    O::rdivc(acc, cvt<T>(immv));
                    E::absv(acc.c, R);
                    E::mul(R, A, A);
                    A[0] += fabs(imm);
                    E::absdiv(A, B, ea);
#pragma unroll
                    for (int i = 0; i < NC; ++i) ea[i] += R[i];
                    break;
                }
                case PDOP_PUSH_P: case PDOP_ADD_P: case PDOP_SUB_P: case PDOP_MUL_P: case PDOP_DIV_P:
                case PDOP_RDIV_P: {
                    // p = v**n as a (value, bound) operand of the generic binary ops; E_p = n |p|
                    const int n = (int)((w >> 8) & 0xffu);
                    V pk[K + 1];
                    double ep[NC];
                    J p;
                    if ((w >> 16) & 1) {
                        O::pcoefs(y, n, pk);
                        O::template set_p<1>(p, pk);
                    } else {
                        O::pcoefs(x, n, pk);
                        O::template set_p<0>(p, pk);
                    }
#pragma unroll
                    for (int i = 0; i < NC; ++i) ep[i] = n * mag(p.c[i]) * (1.0 + cerr);
                    if (op == PDOP_PUSH_P) {
                        if (d > 0 && d < MAXD) stk.store(d - 1, acc.c, ea);
                        acc = p;
#pragma unroll
                        for (int i = 0; i < NC; ++i) ea[i] = ep[i];
                        ++d;
                    } else {
                        // ADD_P: p + t;  SUB_P: t - p;  MUL_P: p * t;  DIV_P: t / p;  RDIV_P: p / t
                        const uint32_t bop = op == PDOP_ADD_P ? PDOP_ADD : op == PDOP_SUB_P ? PDOP_RSUB
                                           : op == PDOP_MUL_P ? PDOP_MUL : op == PDOP_DIV_P ? PDOP_RDIV : PDOP_DIV;
                        binop_e(bop, p, ep, acc, ea);
                    }
                    break;
                }
                case PDOP_NEG:
                    O::scale(acc, from_real<T>(-1.0));
                    break;
                case PDOP_ADD_X: case PDOP_ADD_Y: case PDOP_SUB_X: case PDOP_SUB_Y: {
                    const bool isx = (op == PDOP_ADD_X || op == PDOP_SUB_X);
                    const double sg = (op == PDOP_ADD_X || op == PDOP_ADD_Y) ? 1.0 : -1.0;
                    acc.c[0] = acc.c[0] + cvt<T>((isx ? x : y) * sg);
                    const int idx = isx ? ji(1, 0) : ji(0, 1);
                    acc.c[idx] = acc.c[idx] + from_real<T>(sg);
                    ea[0] += mag(acc.c[0]) + vabs(isx ? x : y) * cerr;
                    break;
                }
                case PDOP_MUL_X: case PDOP_MUL_Y: case PDOP_DIV_X: case PDOP_DIV_Y: {
                    const int axis = (op == PDOP_MUL_X || op == PDOP_DIV_X) ? 0 : 1;
                    const V v = axis == 0 ? x : y;
                    if (op == PDOP_MUL_X || op == PDOP_MUL_Y) {
                        // the coordinate's own rounding: t * dv, |t| |v| cerr per coefficient
                        double cv[NC];
#pragma unroll
                        for (int i = 0; i < NC; ++i) cv[i] = mag(acc.c[i]) * vabs(v) * cerr;
                        O::mul_var(acc, v, axis);
                        // E (*) (|v| + d_axis), in place in decreasing degree
#pragma unroll
                        for (int dd_ = K; dd_ >= 0; --dd_)
#pragma unroll
                            for (int j = 0; j <= dd_; ++j) {
                                const int i = dd_ - j;
                                double s = ea[ji(i, j)] * vabs(v);
                                if (axis == 0 && i > 0) s += ea[ji(i - 1, j)];
                                if (axis == 1 && j > 0) s += ea[ji(i, j - 1)];
                                ea[ji(i, j)] = s + cv[ji(i, j)];
                            }
                    } else {
                        O::div_var(acc, v, axis);
                        // absdiv(E, |v| + d_axis), in place in increasing degree
                        const double inv = 1.0 / vabs(v);
#pragma unroll
                        for (int dd_ = 0; dd_ <= K; ++dd_)
#pragma unroll
                            for (int j = 0; j <= dd_; ++j) {
                                const int i = dd_ - j;
                                double s = ea[ji(i, j)];
                                if (axis == 0 && i > 0) s += ea[ji(i - 1, j)];
                                if (axis == 1 && j > 0) s += ea[ji(i, j - 1)];
                                ea[ji(i, j)] = s * inv;
                            }
                        // the coordinate's rounding: coefficient k of 1/(v + d) moves by (k+1) dv/v
#pragma unroll
                        for (int i = 0; i < NC; ++i) ea[i] += mag(acc.c[i]) * (cerr * (K + 1));
                    }
                    E::add_abs(acc.c, ea);
                    break;
                }
                case PDOP_POWN: {
                    // b^n as n-1 products by b: E' = P (*) (E_b + |b|) + E (*) |b|, P >= |b^k|
                    const int n = (int)((w >> 8) & 0xffu);
                    double P[NC];
                    E::absv(acc.c, B);
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        P[i] = B[i];
                        R[i] = ea[i] + B[i];
                    }
                    for (int k = 1; k < n; ++k) {
                        E::mul(P, R, A);
                        E::mul(ea, B, ea);
#pragma unroll
                        for (int i = 0; i < NC; ++i) ea[i] += A[i];
                        E::mul(P, B, P);
                    }
                    O::pown(acc, n);
                    break;
                }
                case PDOP_POW: case PDOP_SQRT: case PDOP_EXP: case PDOP_LOG: {
                    T f[K + 2];
                    outer_coefs<T, K>(op, acc.c[0], imm, f);
                    double G[K + 1], Fa[K + 1];
#pragma unroll
                    for (int k = 0; k <= K; ++k) {
                        G[k] = (k + 1) * mag(f[k + 1]);
                        Fa[k] = mag(f[k]);
                    }
                    E::absv(acc.c, A);
                    Horner<double, K, 0>::run(A, G, B);     // G1 = sum (m+1)|f_(m+1)| |h|^m
                    Horner<double, K, 0>::run(A, Fa, R);    // sum |f_k| |h|^k
                    E::mul(B, ea, ea);
#pragma unroll
                    for (int i = 0; i < NC; ++i) ea[i] += R[i];
                    if (op == PDOP_POW) O::powa(acc, imm);
                    else if (op == PDOP_SQRT) O::sqrtj(acc);
                    else if (op == PDOP_EXP) O::expj(acc);
                    else O::logj(acc);
                    break;
                }
                case PDOP_ABS: absj<K>(acc); break;
                default: return RUN_UNSUPPORTED;
            }
            if (npc >= end) break;
            pc = npc;
        }
        return d == 1 ? RUN_OK : RUN_BAD;
    }

    // the LDS-stack form used by the tier-2 and diagnostic kernels
    template <bool VEC = false>
    static __device__ int run(const int32_t* ops, int pc, int end, V x, V y, J& acc, double* ea, T* vs,
                              double* es, int lane, const PrmTab<V>& P) {
        LdsStack<T, NC> stk{vs, es, lane};
        return run_s<VEC>(ops, pc, end, x, y, acc, ea, stk, P);
    }
};

// First-order rounding-noise bound of the residual at one point.
template <int PROB, class T> __device__ __forceinline__ double residual_noise(const T* u, const double* e,
                                                                              double x, const double* kc,
                                                                              double S, double om2) {
    constexpr int K = PROB == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
    double up[nc(K)];
#pragma unroll
    for (int i = 0; i < nc(K); ++i) up[i] = mag(u[i]) + kNoiseGamma * e[i];
    double S2;
    if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) S2 = FFEpi<double, true>::eval(up, x, om2);
    else S2 = kerr_epilogue<double>(up, kc).scale;
    return (S2 - S) * (kEps / kNoiseGamma) + kEps * S;
}

// Persistent over a tier-2 list (entries cand | ESC_* << 48 written by validate_kernel).
#ifndef PD_T2_WAVES_PER_SIMD
#define PD_T2_WAVES_PER_SIMD 1   // 512 registers: no spills
#endif
// PRIV: the operand stack in private memory instead of LDS (complex programs of stack 5..8,
// whose value + error slots would need 161 KiB of LDS per wave)
//
// PARTS: every list entry's grid is split over PARTS waves (contiguous chunk ranges).  One wave
// per entry left most of the chip idle on short lists (152 complex entries per 2^20 batch kept
// 152 of 1024 SIMDs busy for 3 ms).  Each part adds its counts into the entry's accumulator
// (a.t2acc, zero between launches) and the part that completes the entry writes the outputs
// and zeroes the accumulator again.  Sums of counts and the max of maxima are the values the
// single-wave loop computes, so the outputs do not depend on PARTS.
template <int PROB, class T, int MAXD, bool PRIV = false, int PARTS = 1>
__global__ __launch_bounds__(64, PD_T2_WAVES_PER_SIMD) void tier2_kernel(KernelArgs a) {
    constexpr int K = (PROB == PDEVAL_PROBLEM_FORCE_FREE) ? 4 : 2;
    constexpr int NC = nc(K);
    using I = ErrInterp<T, K, MAXD>;
    using J = typename I::J;
    const int lane = threadIdx.x & 63;
#ifndef PD_HOST_SIM
    extern __shared__ __align__(16) unsigned char pd_lds[];
#else
    static unsigned char pd_lds[1];
#endif
    T* vs = reinterpret_cast<T*>(pd_lds);
    double* es = reinterpret_cast<double*>(pd_lds + (size_t)(MAXD - 1) * NC * 64 * sizeof(T));
    using STK = typename std::conditional<PRIV, PrivStack<T, NC, MAXD - 1>, LdsStack<T, NC>>::type;
    STK stk;
    if constexpr (!PRIV) stk = STK{vs, es, lane};
    int64_t nwork = (int64_t)(*a.list_count);
    if (nwork > a.list_capacity) nwork = a.list_capacity;
    WorkQueue q;
    for (int64_t wp = q.first(a); wp < nwork * PARTS; wp = q.next(a, wp)) {
        const int64_t wi = wp / PARTS;
        const int part = (int)(wp - wi * PARTS);
        const int64_t entry = a.list[wi];
        const int64_t cand = checked_cand(a, entry < 0 ? -1 : (entry & PD_ESC_CAND_MASK), ERRW_TIER2);
        if (cand < 0) continue;
        const uint32_t flags = (uint32_t)(entry >> PD_ESC_SHIFT);
        const int64_t beg = a.offsets[cand], end = a.offsets[cand + 1];
        const int32_t* prog = a.ops + beg;     // bounds were checked by pass 1
        const int plen = (int)(end - beg);
        const uint32_t hdr = rd_word(prog);
        const int depth = (int)((hdr >> 8) & 0xffu);
        if (depth > MAXD) {
            if (part == 0 && lane == 0 && a.defer_list) list_append(a.defer_list, a.defer_count, a.list_capacity, entry);
            continue;
        }
        // ---- point stage (only if it failed tier 1)
        bool point_reject = false;
        bool grad_nz = false;
        if (flags & ESC_POINT) {
            const bool active = lane < a.n_ref;
            const int l = active ? lane : 0;
            const double x = l == 0 ? a.ref_x[0] : (l == 1 ? a.ref_x[1] : (l == 2 ? a.ref_x[2] : a.ref_x[3]));
            const double y = l == 0 ? a.ref_y[0] : (l == 1 ? a.ref_y[1] : (l == 2 ? a.ref_y[2] : a.ref_y[3]));
            J u;
            double e[NC];
            const int rc = I::template run_s<false>(prog, 1, plen, x, y, u, e, stk, a.prm_pt);
            bool real_fail = rc != RUN_OK;
            if (rc == RUN_OK) {
                const double* kc = a.kc ? a.kc + 4 * l : nullptr;
                PointResult r;
                if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) r = ff_epilogue<T>(u.c, x, a.prm.omega2);
                else r = kerr_epilogue<T>(u.c, kc);
                bool fails;
                if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) fails = !(scaled(r.res_abs, r.scale) <= a.prm.tau_point);
                else fails = !(r.res_abs < a.prm.kerr_abs_tol);
                if (!r.finite) real_fail = true;
                else if (fails) real_fail = r.res_abs > a.prm.noise_kappa * residual_noise<PROB, T>(u.c, e, x, kc, r.scale, a.prm.omega2);
            }
            point_reject = __any(active && real_fail);
            if (point_reject) continue;     // confirmed: pass 1's REJECT_POINT stands
        }
        // ---- grid stage
        int nbad_out = -1, nb1 = 0, nb2 = 0, nfin = 0, nnonfin = 0;
        double qmax = 0.0;
        const bool eval_grid = !(flags & ESC_GRID_EVAL) || (flags & ESC_GRID_FAIL);
        if (!eval_grid && part != 0) continue;     // nothing to split: part 0 decides
        // a grid that tier 1 evaluated and recorded (ESC_MASK): only its failing points are
        // re-checked -- chunks with none are skipped, the other lanes of a chunk count nothing.
        // Its q_grid, non-finite count and finite flag are tier 1's (outputs written by pass 1).
        const bool masked = (flags & ESC_GRID_EVAL) && (flags & ESC_MASK) && a.fmask;
        if (eval_grid) {
            const int per_row = a.ny >> 6;
            const int nchunks = a.nx * per_row;
            const int ch0 = (int)((int64_t)nchunks * part / PARTS);
            const int ch1 = (int)((int64_t)nchunks * (part + 1) / PARTS);
            // (packing the failing points 64 to a batch, x per lane, measured slower: force-free
            // tier 2 7.9 vs 6.5 ms, Kerr 2.1 vs 1.3 ms, profiles/r05_n_ab_*.log)
            // the chunks pass 1 stored a word for (a.fsum: the others had no failing lane)
            uint64_t stored = ~0ull;
            if (masked && a.fsum) {
                const uint64_t v = a.fsum[cand];
                stored = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
            }
            for (int ch = ch0; ch < ch1; ++ch) {
                uint64_t m = ~0ull;
                if (masked) {
                    if (nchunks <= 64 && !((stored >> ch) & 1ull)) continue;
                    const uint64_t v = a.fmask[cand * (int64_t)nchunks + ch];
                    m = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
                    if (m == 0ull) continue;
                }
                const bool sel = (m >> lane) & 1ull;
                const int row = ch / per_row, sl = ch - row * per_row;
                const int p = a.n_ref + row * a.ny + sl * 64 + lane;
                const double x = rd_sf64(a.gx + row);
                const double y = a.gy[sl * 64 + lane];
                J u;
                double e[NC];
                const int rc = I::template run_s<false>(prog, 1, plen, x, y, u, e, stk, a.prm_grid);
                if (rc != RUN_OK) { ++nnonfin; continue; }
                const double* kc = a.kc ? a.kc + 4 * p : nullptr;
                PointResult r;
                if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) r = ff_epilogue<T>(u.c, x, a.prm.omega2);
                else r = kerr_epilogue<T>(u.c, kc);
                if (!r.finite) { ++nnonfin; continue; }
                ++nfin;
                const double qv = scaled(r.res_abs, r.scale);
                qmax = fmax(qmax, qv);
                if (!r.grad_zero) grad_nz = true;
                if (sel && grid_fails(r.res_abs, r.scale, a.prm.tau_grid)) {
                    ++nb1;
                    if (r.res_abs > a.prm.noise_kappa * residual_noise<PROB, T>(u.c, e, x, kc, r.scale, a.prm.omega2)) ++nb2;
                }
            }
            nb1 = wave_sum(nb1);
            nb2 = wave_sum(nb2);
            nfin = wave_sum(nfin);
            nnonfin = wave_sum(nnonfin);
            qmax = wave_max(qmax);
        }
        bool grad_any = __any(grad_nz);
        if constexpr (PARTS > 1) {
            if (eval_grid) {
                // merge this part into the entry's accumulator; the last part carries on
                int last = 0;
                if (lane == 0) {
                    T2Acc* A = a.t2acc + wi;
                    atomicAdd(&A->nb1, nb1);
                    atomicAdd(&A->nb2, nb2);
                    atomicAdd(&A->nfin, nfin);
                    atomicAdd(&A->nnonfin, nnonfin);
                    atomicMax(&A->qmax_bits, (unsigned long long)__double_as_longlong(qmax));  // qmax >= 0
                    if (grad_any) atomicOr(&A->grad, 1u);
                    __threadfence();
                    if (atomicAdd(&A->done, 1) == PARTS - 1) {
                        __threadfence();
                        nb1 = atomicAdd(&A->nb1, 0);
                        nb2 = atomicAdd(&A->nb2, 0);
                        nfin = atomicAdd(&A->nfin, 0);
                        nnonfin = atomicAdd(&A->nnonfin, 0);
                        qmax = __longlong_as_double((long long)atomicMax(&A->qmax_bits, 0ull));
                        grad_any = atomicOr(&A->grad, 0u) != 0u;
                        A->nb1 = A->nb2 = A->nfin = A->nnonfin = A->done = 0;   // ready for the next launch
                        A->grad = 0u;
                        A->qmax_bits = 0ull;
                        last = 1;
                    }
                }
                if (!__builtin_amdgcn_readfirstlane(last)) continue;   // lane 0 is the first active lane
            }
        }
        if (eval_grid) nbad_out = nb1 <= a.prm.max_bad ? nb1 : nb2;
        // (P0_CONST: a Kerr constant whose gradient is rounding noise -- pdeval_kernels.h)
        const bool pconst = a.pstate && (a.pstate[cand] & P0_CONST);
        const bool any_grad = (grad_any || (flags & ESC_ANY_GRAD)) && !pconst;
        if (lane == 0) {
            const bool has_fin = eval_grid && !masked ? nfin > 0 : (flags & ESC_NFIN) != 0;
            const bool structural = (PROB != PDEVAL_PROBLEM_FORCE_FREE) || (hdr & PDEVAL_FLAG_NOCOORD);
            int cls;
            if (!any_grad && (has_fin || pconst) && structural) cls = PDEVAL_CLS_ZERO_GRADIENT;
            else if (PROB != PDEVAL_PROBLEM_FORCE_FREE && !has_fin) cls = PDEVAL_CLS_REJECT_GRID;
            else if (nbad_out > a.prm.max_bad) cls = PDEVAL_CLS_REJECT_GRID;
            else if (PROB == PDEVAL_PROBLEM_FORCE_FREE && a.prm.strict_symbolic && (hdr & (PDEVAL_FLAG_NONSMOOTH2D | PDEVAL_FLAG_UNPROVABLE)))
                cls = PDEVAL_CLS_REJECT_SYMBOLIC;
            else cls = PDEVAL_CLS_ACCEPT;
            if (a.out.status) a.out.status[cand] = (uint8_t)cls;
            if (eval_grid) {
                if (a.out.n_bad) a.out.n_bad[cand] = nbad_out;
                if (!(flags & ESC_GRID_EVAL)) {
                    if (a.out.q_grid) a.out.q_grid[cand] = qmax;
                    if (a.out.n_nonfinite) a.out.n_nonfinite[cand] = nnonfin;
                }
            }
            if (a.out.verdict_bits && cls == PDEVAL_CLS_ACCEPT)
                atomicOr((uint32_t*)a.out.verdict_bits + (cand >> 5), 1u << (cand & 31));
        }
    }
}

}  // namespace pd

namespace pd {
// Diagnostic / test kernel: one program at a list of points (lane = point), tier-1 or tier-2
// arithmetic; out[4 p ..] = {|residual|, S, noise (tier 2), finite}.  Used by the GPU parity
// tests to compare the device's point arithmetic with the oracle's directly.
template <int PROB, int MAXD>
__global__ __launch_bounds__(64, 1) void eval_points_kernel(const int32_t* prog, int plen, const double* xs,
                                                            const double* ys, const double* kc, int npts, int tier2,
                                                            double* out, double* jets) {
    constexpr int K = (PROB == PDEVAL_PROBLEM_FORCE_FREE) ? 4 : 2;
    constexpr int NC = nc(K);
    using EI = ErrInterp<double, K, MAXD>;
    using I = Interp<double, K, MAXD>;
    const int lane = threadIdx.x & 63;
#ifndef PD_HOST_SIM
    extern __shared__ __align__(16) unsigned char pd_lds[];
#else
    static unsigned char pd_lds[1];
#endif
    double* vs = reinterpret_cast<double*>(pd_lds);
    double* es = vs + (size_t)(MAXD - 1) * NC * 64;
    const int p = blockIdx.x * 64 + lane;
    const int pc = p < npts ? p : npts - 1;
    const double x = xs[pc], y = ys[pc];
    typename I::J u;
    double e[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) e[i] = 0.0;
    const PrmTab<double> P{};   // (force-free: no constants of the problem)
    const int rc = tier2 ? EI::template run<false>(prog, 1, plen, x, y, u, e, vs, es, lane, P)
                         : I::run(prog, 1, plen, x, y, u, vs, lane, P);
    PointResult r;
    const double* k4 = kc ? kc + 4 * pc : nullptr;
    if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) r = ff_epilogue<double>(u.c, x);   // (Omega = 0)
    else r = kerr_epilogue<double>(u.c, k4);
    if (p < npts) {
        out[4 * p + 0] = rc ? NAN : r.res_abs;
        out[4 * p + 1] = rc ? NAN : r.scale;
        out[4 * p + 2] = (rc || !tier2) ? 0.0 : residual_noise<PROB, double>(u.c, e, x, k4, r.scale, 0.0);
        out[4 * p + 3] = rc ? -1.0 : (r.finite ? 1.0 : 0.0);
        if (jets) {
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                jets[(size_t)p * 2 * NC + i] = u.c[i];
                jets[(size_t)p * 2 * NC + NC + i] = e[i];
            }
        }
    }
}
}  // namespace pd

