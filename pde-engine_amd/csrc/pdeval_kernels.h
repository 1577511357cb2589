// pdeval_kernels.h -- the gfx950 candidate-validation kernel.
//
// One wavefront validates one candidate.  Its 64 lanes are 64 sample points; the wave walks
// the candidate's postfix program (wave-uniform, read with scalar loads, so the interpreter
// never diverges), evaluating it in jet arithmetic (jet.h) with a register-resident operand
// stack, then applies the problem's residual operator in an epilogue:
//   force-free  det[[L_T A, L_T B], [L_T^2 A, L_T^2 B]]   (problems/force_free/validator.py:323-347)
//   Kerr        d_r[G/(1-x^2) d_r u] + d_x[G/Delta d_x u]  (problems/kerr_magnetosphere/validator.py:77-91)
// and a scaled zero test q = |residual| / S, S = the same epilogue evaluated on magnitudes
// (DESIGN.md "Zero test").  Chunk 0 carries the reference point(s) in its first lanes, so the
// reference's point stage (validator.py:349-402 / kerr :163-192) is decided first; the grid
// chunks then play the role of the symbolic stage (validator.py:404-427 / kerr :283-315).
// Per-lane statistics are reduced across the wave with DPP/shuffles; lane 0 writes the
// per-candidate outputs and sets the verdict bit with one atomicOr.
#pragma once
#include <stdint.h>

#include "../../include/pdeval.h"
#include "jet.h"

namespace pd {

struct KernelArgs {
    const int32_t* ops;
    const int64_t* offsets;
    int64_t n_words;            // size of ops[] (programs are bounds-checked against it)
    int64_t n;                  // candidates in the batch
    const int64_t* list;        // optional: wave -> candidate index (NULL = identity)
    const int32_t* list_count;  // optional device count for list (persistent passes)
    int64_t list_cap;
    const double* px;           // point coordinates, reference points first
    const double* py;
    const double* kc;           // Kerr: 4 operator coefficients per point (NULL for FF)
    int n_ref;
    int n_pts;
    int fp_pts[PDEVAL_FP_N];    // point indices whose u value is the fingerprint
    pdeval_params prm;
    pdeval_outputs out;
    int64_t* defer_list;        // candidates this variant cannot take (deeper stack)
    int32_t* defer_count;
    int64_t* cplx_list;         // FF candidates non-finite at the reference point
    int32_t* cplx_count;
    int64_t list_capacity;      // capacity of defer_list and cplx_list (appends beyond are dropped)
};

// Append a candidate to a device work list (lane 0 only).  Returns false when the list is
// full -- impossible when capacity >= n, which the host guarantees; checked anyway so a bad
// call can never write out of bounds.
__device__ __forceinline__ bool list_append(int64_t* list, int32_t* count, int64_t cap, int64_t cand) {
    const int slot = atomicAdd(count, 1);
    if (slot >= cap) return false;
    list[slot] = cand;
    return true;
}

template <class T> struct Real;
template <> struct Real<double> { static constexpr bool cplx_pass = false; };
template <> struct Real<cplx> { static constexpr bool cplx_pass = true; };

__device__ __forceinline__ uint32_t rd_word(const int32_t* p) {
    return (uint32_t)__builtin_amdgcn_readfirstlane(*p);
}
__device__ __forceinline__ double rd_imm(const int32_t* p) {
    // the two words following an opcode hold the f64 immediate, low word first
    uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane(p[0]);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane(p[1]);
    return __hiloint2double((int)hi, (int)lo);
}

template <class T, int K> struct JetOps {
    static constexpr int NC = nc(K);
    struct J { T c[NC]; };

    static PD_HD void set_const(J& t, T v) {
        t.c[0] = v;
#pragma unroll
        for (int i = 1; i < NC; ++i) t.c[i] = zero<T>();
    }
    static PD_HD void set_var(J& t, double v, int axis) {
        set_const(t, from_real<T>(v));
        t.c[axis == 0 ? ji(1, 0) : ji(0, 1)] = from_real<T>(1.0);
    }
    static PD_HD void add(const J& a, J& t) {
#pragma unroll
        for (int i = 0; i < NC; ++i) t.c[i] = a.c[i] + t.c[i];
    }
    static PD_HD void sub(const J& a, J& t) {  // t = a - t
#pragma unroll
        for (int i = 0; i < NC; ++i) t.c[i] = a.c[i] - t.c[i];
    }
    static PD_HD void rsub(const J& a, J& t) {  // t = t - a
#pragma unroll
        for (int i = 0; i < NC; ++i) t.c[i] = t.c[i] - a.c[i];
    }
    static PD_HD void mul(const J& a, J& t) {
        J r;
        jmul<T, K, K, K>(a.c, t.c, r.c);
        t = r;
    }
    static PD_HD void div(const J& a, J& t) {  // t = a / t
        J r;
        jdiv<T, K>(a.c, t.c, r.c);
        t = r;
    }
    static PD_HD void rdiv(const J& a, J& t) {  // t = t / a
        J r;
        jdiv<T, K>(t.c, a.c, r.c);
        t = r;
    }
    static PD_HD void scale(J& t, T s) {
#pragma unroll
        for (int i = 0; i < NC; ++i) t.c[i] = t.c[i] * s;
    }
    // t *= (v + d_axis)
    static PD_HD void mul_var(J& t, double v, int axis) {
        const T vv = from_real<T>(v);
#pragma unroll
        for (int d = K; d >= 0; --d) {
#pragma unroll
            for (int j = 0; j <= d; ++j) {
                const int i = d - j;
                T s = t.c[ji(i, j)] * vv;
                if (axis == 0 && i > 0) s = s + t.c[ji(i - 1, j)];
                if (axis == 1 && j > 0) s = s + t.c[ji(i, j - 1)];
                t.c[ji(i, j)] = s;
            }
        }
    }
    // t /= (v + d_axis)
    static PD_HD void div_var(J& t, double v, int axis) {
        const T vv = from_real<T>(v);
        const T inv = from_real<T>(1.0 / v);
#pragma unroll
        for (int d = 0; d <= K; ++d) {
#pragma unroll
            for (int j = 0; j <= d; ++j) {
                const int i = d - j;
                T s = t.c[ji(i, j)];
                if (axis == 0 && i > 0) s = s - t.c[ji(i - 1, j)];
                if (axis == 1 && j > 0) s = s - t.c[ji(i, j - 1)];
                t.c[ji(i, j)] = qdiv(s, vv, inv);
            }
        }
    }
    static PD_HD void rdivc(J& t, T c) {  // t = c / t
        J a;
        set_const(a, c);
        div(a, t);
    }
    static PD_HD void pown(J& t, int n) {  // n >= 2
        J base = t, r;
        bool have = false;
        while (n > 0) {
            if (n & 1) {
                if (have) {
                    J tmp;
                    jmul<T, K, K, K>(r.c, base.c, tmp.c);
                    r = tmp;
                } else {
                    r = base;
                    have = true;
                }
            }
            n >>= 1;
            if (n) {
                J sq;
                jmul<T, K, K, K>(base.c, base.c, sq.c);
                base = sq;
            }
        }
        t = r;
    }
    static PD_HD void powa(J& t, double alpha) {
        T f[K + 1];
        coef_pow<T, K>(t.c[0], alpha, pow_real_exp(t.c[0], alpha), f);
        jcompose<T, K>(t.c, f);
    }
    static PD_HD void sqrtj(J& t) {
        T f[K + 1];
        coef_pow<T, K>(t.c[0], 0.5, sqrt_(t.c[0]), f);
        jcompose<T, K>(t.c, f);
    }
    static PD_HD void expj(J& t) {
        T f[K + 1];
        f[0] = exp_(t.c[0]);
#pragma unroll
        for (int k = 1; k <= K; ++k) f[k] = f[k - 1] * (1.0 / k);
        jcompose<T, K>(t.c, f);
    }
    static PD_HD void logj(J& t) {
        T f[K + 1];
        const T r = recip(t.c[0]);
        f[0] = log_(t.c[0]);
        T rk = r;
#pragma unroll
        for (int k = 1; k <= K; ++k) {
            f[k] = rk * (((k & 1) ? 1.0 : -1.0) / k);
            rk = rk * r;
        }
        jcompose<T, K>(t.c, f);
    }
};

// |x| of a jet: sign(x0) * x away from the kink; at x0 == 0 (or non-real x0) undefined.
template <int K> __device__ __forceinline__ void absj(typename JetOps<double, K>::J& t) {
    const double s = t.c[0] > 0.0 ? 1.0 : (t.c[0] < 0.0 ? -1.0 : NAN);
    JetOps<double, K>::scale(t, s);
}
template <int K> __device__ __forceinline__ void absj(typename JetOps<cplx, K>::J& t) {
    // Abs of a complex value is not holomorphic: only real arguments are meaningful
    const double s = (t.c[0].im == 0.0) ? (t.c[0].re > 0.0 ? 1.0 : (t.c[0].re < 0.0 ? -1.0 : NAN)) : NAN;
    JetOps<cplx, K>::scale(t, from_real<cplx>(s));
}

// ------------------------------------------------------------------ residual epilogues
struct PointResult {
    double res_re, res_im;  // residual (complex pass: both parts)
    double res_abs;         // |residual|
    double scale;           // S
    bool grad_zero;         // u_x == u_y == 0 exactly
    bool finite;
};

// Force-free foliation determinant from the order-4 jet of u.
// p = u_rho, q = u_z (order 3);  A = p_rho + q_z - p/rho,  B = p^2 + q^2 (order 2);
// LA = q A_rho - p A_z, LB = q B_rho - p B_z (order 1);  L2A = q LA_rho - p LA_z (order 0);
// det = LA * L2B - LB * L2A.   (validator.py:323-347; Omega = 0 on the problem path)
// MAG = true evaluates the same expression on magnitudes with every difference turned into
// a sum: S >= sum of |monomials| of the fully expanded determinant.
template <class T, bool MAG> struct FFEpi {
    static PD_HD T sgn(T a) { return MAG ? a : -a; }
    static PD_HD T eval(const T* u, double rho) {
        T p[10], q[10];
#pragma unroll
        for (int d = 0; d <= 3; ++d)
#pragma unroll
            for (int j = 0; j <= d; ++j) {
                const int i = d - j;
                p[ji(i, j)] = u[ji(i + 1, j)] * (double)(i + 1);
                q[ji(i, j)] = u[ji(i, j + 1)] * (double)(j + 1);
            }
        // 1/rho jet (rho direction only): (-1)^i / rho^(i+1)
        const double r0 = 1.0 / rho;
        const double ri[3] = {r0, (MAG ? 1.0 : -1.0) * r0 * r0, r0 * r0 * r0};
        T A[6], B[6];
#pragma unroll
        for (int d = 0; d <= 2; ++d)
#pragma unroll
            for (int j = 0; j <= d; ++j) {
                const int i = d - j;
                T s = p[ji(i + 1, j)] * (double)(i + 1) + q[ji(i, j + 1)] * (double)(j + 1);
                T pr = p[ji(i, j)] * ri[0];
#pragma unroll
                for (int i1 = 1; i1 <= i; ++i1) pr = fmac(p[ji(i - i1, j)], from_real<T>(ri[i1]), pr);
                A[ji(i, j)] = s + sgn(pr);
            }
        {
            T pp[6], qq[6];
            jmul<T, 3, 3, 2>(p, p, pp);
            jmul<T, 3, 3, 2>(q, q, qq);
#pragma unroll
            for (int i = 0; i < 6; ++i) B[i] = pp[i] + qq[i];
        }
        // L_T f = q f_rho - p f_z, order 1 from order-2 f
        T LA[3], LB[3];
        lie1(p, q, A, LA);
        lie1(p, q, B, LB);
        // order 0 from order 1
        const T L2A = q[0] * LA[ji(1, 0)] + sgn(p[0] * LA[ji(0, 1)]);
        const T L2B = q[0] * LB[ji(1, 0)] + sgn(p[0] * LB[ji(0, 1)]);
        return LA[0] * L2B + sgn(LB[0] * L2A);
    }
    static PD_HD void lie1(const T* p, const T* q, const T* f, T* out) {
        T fr[3], fz[3];
#pragma unroll
        for (int d = 0; d <= 1; ++d)
#pragma unroll
            for (int j = 0; j <= d; ++j) {
                const int i = d - j;
                fr[ji(i, j)] = f[ji(i + 1, j)] * (double)(i + 1);
                fz[ji(i, j)] = f[ji(i, j + 1)] * (double)(j + 1);
            }
        T a[3], b[3];
        jmul<T, 1, 1, 1>(q, fr, a);
        jmul<T, 1, 1, 1>(p, fz, b);
#pragma unroll
        for (int i = 0; i < 3; ++i) out[i] = a[i] + sgn(b[i]);
    }
};

template <class T> __device__ __forceinline__ PointResult ff_epilogue(const T* u, double rho) {
    PointResult r;
    const T det = FFEpi<T, false>::eval(u, rho);
    double m[15];
#pragma unroll
    for (int i = 0; i < 15; ++i) m[i] = mag(u[i]);
    const double S = FFEpi<double, true>::eval(m, rho);
    r.res_abs = mag(det);
    if constexpr (Real<T>::cplx_pass) {
        r.res_re = ((const cplx*)&det)->re;
        r.res_im = ((const cplx*)&det)->im;
    } else {
        r.res_re = *(const double*)&det;
        r.res_im = 0.0;
    }
    r.scale = S;
    r.grad_zero = is_zero(u[ji(1, 0)]) && is_zero(u[ji(0, 1)]);
    bool fin = finite_(det) && isfinite(S);
#pragma unroll
    for (int i = 0; i < 15; ++i) fin = fin && finite_(u[i]);
    r.finite = fin;
    return r;
}

// Kerr surrogate: L[u] = k1 u_rr + k2 u_xx + k3 u_r + k4 u_x, coefficients per point.
template <class T> __device__ __forceinline__ PointResult kerr_epilogue(const T* u, const double* k) {
    PointResult r;
    const T t1 = u[ji(2, 0)] * (2.0 * k[0]);
    const T t2 = u[ji(0, 2)] * (2.0 * k[1]);
    const T t3 = u[ji(1, 0)] * k[2];
    const T t4 = u[ji(0, 1)] * k[3];
    const T L = (t1 + t2) + (t3 + t4);
    r.scale = (mag(t1) + mag(t2)) + (mag(t3) + mag(t4));
    r.res_abs = mag(L);
    if constexpr (Real<T>::cplx_pass) {
        r.res_re = ((const cplx*)&L)->re;
        r.res_im = ((const cplx*)&L)->im;
    } else {
        r.res_re = *(const double*)&L;
        r.res_im = 0.0;
    }
    r.grad_zero = is_zero(u[ji(1, 0)]) && is_zero(u[ji(0, 1)]);
    bool fin = finite_(L) && isfinite(r.scale);
#pragma unroll
    for (int i = 0; i < 6; ++i) fin = fin && finite_(u[i]);
    r.finite = fin;
    return r;
}

__device__ __forceinline__ double scaled(double res_abs, double S) {
    if (S > 0.0) return res_abs / S;
    return res_abs == 0.0 ? 0.0 : INFINITY;
}

// ------------------------------------------------------------------ wave reductions
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ------------------------------------------------------------------ the interpreter
// Result codes of run_program (wave-uniform).
enum { RUN_OK = 0, RUN_UNSUPPORTED = 1, RUN_BAD = 2 };

template <class T, int K, int MAXD> struct Interp {
    using O = JetOps<T, K>;
    using J = typename O::J;

    static __device__ __forceinline__ void binop(uint32_t op, const J& a, J& t) {
        switch (op) {
            case PDOP_ADD: O::add(a, t); break;
            case PDOP_SUB: O::sub(a, t); break;
            case PDOP_RSUB: O::rsub(a, t); break;
            case PDOP_MUL: O::mul(a, t); break;
            case PDOP_DIV: O::div(a, t); break;
            default: O::rdiv(a, t); break;
        }
    }
    // t = S[d-2] (op) t for the slot just below the top; d uniform.
    template <int I> static __device__ __forceinline__ void below(J* S, int d, uint32_t op, J& t) {
        if constexpr (I < MAXD - 1) {
            if (d == I + 2) {
                binop(op, S[I], t);
                return;
            }
            below<I + 1>(S, d, op, t);
        }
    }
    template <int I> static __device__ __forceinline__ void push_down(J* S, int d, const J& t) {
        if constexpr (I < MAXD - 1) {
            if (d == I + 1) {
                S[I] = t;
                return;
            }
            push_down<I + 1>(S, d, t);
        }
    }

    // Evaluate program words [pc, end) at point (x, y); result jet in T.
    static __device__ __forceinline__ int run(const int32_t* ops, int64_t pc, int64_t end, double x, double y, J& acc) {
        J S[MAXD - 1];
        int d = 0;
        while (pc < end) {
            const uint32_t w = rd_word(ops + pc);
            const uint32_t op = w & 0xffu;
            ++pc;
            switch (op) {
                case PDOP_PUSH_X:
                case PDOP_PUSH_Y:
                case PDOP_PUSH_C:
                case PDOP_PUSH_I: {
                    if (d >= MAXD) return RUN_BAD;
                    if (d > 0) push_down<0>(S, d, acc);
                    if (op == PDOP_PUSH_X) O::set_var(acc, x, 0);
                    else if (op == PDOP_PUSH_Y) O::set_var(acc, y, 1);
                    else if (op == PDOP_PUSH_C) {
                        if (pc + 2 > end) return RUN_BAD;
                        O::set_const(acc, from_real<T>(rd_imm(ops + pc)));
                        pc += 2;
                    } else {
                        if constexpr (Real<T>::cplx_pass) O::set_const(acc, cplx{0.0, 1.0});
                        else return RUN_UNSUPPORTED;
                    }
                    ++d;
                    break;
                }
                case PDOP_ADD: case PDOP_SUB: case PDOP_RSUB:
                case PDOP_MUL: case PDOP_DIV: case PDOP_RDIV: {
                    if (d < 2) return RUN_BAD;
                    below<0>(S, d, op, acc);
                    --d;
                    break;
                }
                case PDOP_ADDC: case PDOP_MULC: case PDOP_RDIVC: {
                    if (d < 1 || pc + 2 > end) return RUN_BAD;
                    const double c = rd_imm(ops + pc);
                    pc += 2;
                    if (op == PDOP_ADDC) acc.c[0] = acc.c[0] + from_real<T>(c);
                    else if (op == PDOP_MULC) O::scale(acc, from_real<T>(c));
                    else O::rdivc(acc, from_real<T>(c));
                    break;
                }
                case PDOP_NEG:
                    if (d < 1) return RUN_BAD;
                    O::scale(acc, from_real<T>(-1.0));
                    break;
                case PDOP_ADD_X: case PDOP_ADD_Y: case PDOP_SUB_X: case PDOP_SUB_Y: {
                    if (d < 1) return RUN_BAD;
                    const bool isx = (op == PDOP_ADD_X || op == PDOP_SUB_X);
                    const double sg = (op == PDOP_ADD_X || op == PDOP_ADD_Y) ? 1.0 : -1.0;
                    acc.c[0] = acc.c[0] + from_real<T>(sg * (isx ? x : y));
                    const int idx = isx ? ji(1, 0) : ji(0, 1);
                    acc.c[idx] = acc.c[idx] + from_real<T>(sg);
                    break;
                }
                case PDOP_MUL_X: if (d < 1) return RUN_BAD; O::mul_var(acc, x, 0); break;
                case PDOP_MUL_Y: if (d < 1) return RUN_BAD; O::mul_var(acc, y, 1); break;
                case PDOP_DIV_X: if (d < 1) return RUN_BAD; O::div_var(acc, x, 0); break;
                case PDOP_DIV_Y: if (d < 1) return RUN_BAD; O::div_var(acc, y, 1); break;
                case PDOP_POWN:
                    if (d < 1) return RUN_BAD;
                    O::pown(acc, (int)((w >> 8) & 0xffu));
                    break;
                case PDOP_POW: {
                    if (d < 1 || pc + 2 > end) return RUN_BAD;
                    const double a = rd_imm(ops + pc);
                    pc += 2;
                    O::powa(acc, a);
                    break;
                }
                case PDOP_SQRT: if (d < 1) return RUN_BAD; O::sqrtj(acc); break;
                case PDOP_EXP: if (d < 1) return RUN_BAD; O::expj(acc); break;
                case PDOP_LOG: if (d < 1) return RUN_BAD; O::logj(acc); break;
                case PDOP_ABS: if (d < 1) return RUN_BAD; absj<K>(acc); break;
                default: return RUN_UNSUPPORTED;
            }
        }
        return d == 1 ? RUN_OK : RUN_BAD;
    }
};

// ------------------------------------------------------------------ the kernel
// PROB: PDEVAL_PROBLEM_FORCE_FREE (K = 4) or PDEVAL_PROBLEM_KERR (K = 2).
template <int PROB, class T, int MAXD, bool PERSISTENT>
__global__ __launch_bounds__(256, 2) void validate_kernel(KernelArgs a) {
    constexpr int K = (PROB == PDEVAL_PROBLEM_FORCE_FREE) ? 4 : 2;
    using I = Interp<T, K, MAXD>;
    using J = typename I::J;
    const int lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wib;
    // persistent variants stride over a device work list; the first pass is one wave per
    // candidate (a single iteration)
    const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6);
    int64_t nwork = a.list_count ? (int64_t)(*a.list_count) : (a.list ? a.list_cap : a.n);
    if (a.list && nwork > a.list_capacity) nwork = a.list_capacity;

    for (int64_t wi = wave0; wi < nwork; wi = PERSISTENT ? wi + wstride : nwork) {
        const int64_t cand = a.list ? (int64_t)__builtin_amdgcn_readfirstlane((int)a.list[wi]) : wi;
        int64_t beg = a.offsets[cand], end = a.offsets[cand + 1];
        const bool in_bounds = beg >= 0 && end > beg && end <= a.n_words;
        if (!in_bounds) beg = end = 0;
        beg = __builtin_amdgcn_readfirstlane((int)beg);
        end = __builtin_amdgcn_readfirstlane((int)end);
        // header word: opcode 0, depth in bits 8-15, flags above
        const uint32_t hdr = in_bounds ? rd_word(a.ops + beg) : 0xffu;
        int status = -1;
        if ((hdr & 0xffu) != 0u) status = PDEVAL_CLS_BAD_PROGRAM;
        if constexpr (!Real<T>::cplx_pass) {
            if (status < 0 && (hdr & PDEVAL_FLAG_COMPLEX)) {
                if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) {
                    // complex-valued program: straight to the complex pass
                    if (lane == 0 && a.cplx_list) list_append(a.cplx_list, a.cplx_count, a.list_capacity, cand);
                    status = PDEVAL_CLS_NONFINITE_REF;
                } else {
                    // Kerr: a non-real value at a test point rejects (kerr validator.py:179-180)
                    status = PDEVAL_CLS_REJECT_POINT;
                }
            }
        }
        const int depth = (int)((hdr >> 8) & 0xffu);
        if (status < 0 && depth > MAXD) {
            if (a.defer_list) {
                if (lane == 0) list_append(a.defer_list, a.defer_count, a.list_capacity, cand);
                continue;
            }
            status = PDEVAL_CLS_UNSUPPORTED;  // deeper than the last variant takes
        }
        double q_ref = 0.0;        // FF: q*, Kerr: max |lhs| over reference points
        bool point_reject = false;
        double qmax = 0.0;
        int nbad = 0, nnonfin = 0, nfin = 0;
        bool grad_nz = false;
        const int nchunks = (a.n_pts + 63) >> 6;
        for (int ch = 0; ch < nchunks && status < 0; ++ch) {
            const int p = ch * 64 + lane;
            const bool active = p < a.n_pts;
            const int pp = active ? p : 0;
            const double x = a.px[pp], y = a.py[pp];
            J u;
            const int rc = I::run(a.ops, beg + 1, end, x, y, u);
            if (rc == RUN_UNSUPPORTED) { status = PDEVAL_CLS_UNSUPPORTED; break; }
            if (rc == RUN_BAD) { status = PDEVAL_CLS_BAD_PROGRAM; break; }
            PointResult r;
            if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) r = ff_epilogue<T>(u.c, x);
            else r = kerr_epilogue<T>(u.c, a.kc + 4 * pp);
            const double qv = scaled(r.res_abs, r.scale);
            if (active) {
#pragma unroll
                for (int f = 0; f < PDEVAL_FP_N; ++f)
                    if (p == a.fp_pts[f] && a.out.fingerprint) {
                        double v;
                        if constexpr (Real<T>::cplx_pass) v = ((const cplx*)&u.c[0])->re;
                        else v = *(const double*)&u.c[0];
                        a.out.fingerprint[cand * PDEVAL_FP_N + f] = v;
                    }
            }
            if (active && p < a.n_ref) {
                if (a.out.res_ref) a.out.res_ref[cand * a.n_ref + p] = r.res_re;
                if (r.finite && !r.grad_zero) grad_nz = true;
            } else if (active) {
                if (r.finite) {
                    ++nfin;
                    qmax = fmax(qmax, qv);
                    if (qv > a.prm.tau_grid) ++nbad;
                    if (!r.grad_zero) grad_nz = true;
                } else {
                    ++nnonfin;
                }
            }
            if (ch == 0) {
                // point stage: lanes 0..n_ref-1 hold the reference points
                double refv;
                if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) refv = (lane == 0) ? qv : 0.0;
                else refv = (lane < a.n_ref) ? r.res_abs : 0.0;
                q_ref = wave_max(refv);
                const bool nf = __any(active && p < a.n_ref && !r.finite);
                if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) {
                    if (nf) {
                        if constexpr (!Real<T>::cplx_pass) {
                            // not real at p*: the complex pass decides (SymPy evaluates the
                            // point exactly, in the complex field: validator.py:363-402)
                            status = PDEVAL_CLS_NONFINITE_REF;
                            if (lane == 0 && a.cplx_list)
                                list_append(a.cplx_list, a.cplx_count, a.list_capacity, cand);
                        } else {
                            point_reject = true;  // not finite even in the complex field
                        }
                    } else {
                        point_reject = !(q_ref <= a.prm.tau_point);
                    }
                } else {
                    // Kerr fast point check (kerr validator.py:163-192): non-real / NaN at a
                    // reference point rejects; otherwise reject iff max|lhs| >= 1e-10 (absolute)
                    point_reject = nf || !(q_ref < a.prm.kerr_abs_tol);
                }
                if (status < 0 && point_reject && !a.prm.full_grid) status = PDEVAL_CLS_REJECT_POINT;
            }
        }
        // wave reductions
        qmax = wave_max(qmax);
        nbad = wave_sum(nbad);
        nnonfin = wave_sum(nnonfin);
        nfin = wave_sum(nfin);
        const bool any_grad = __any(grad_nz);
        if (lane == 0) {
            int cls = status;
            if (cls < 0) {
                // zero gradient: the reference exits only on a structurally zero gradient
                // (validator.py:309-312 compares the symbolic u_rho, u_z with 0), i.e. when u
                // references no coordinate; a numerically constant but structurally
                // non-constant u goes on and its det is identically 0.  Kerr excludes every
                // u that simplify() reduces to a constant (kerr validator.py:231-240).
                const bool structural = (PROB != PDEVAL_PROBLEM_FORCE_FREE) || (hdr & PDEVAL_FLAG_NOCOORD);
                if (!any_grad && nfin > 0 && structural) cls = PDEVAL_CLS_ZERO_GRADIENT;
                else if (point_reject) cls = PDEVAL_CLS_REJECT_POINT;
                else if (nbad > a.prm.max_bad) cls = PDEVAL_CLS_REJECT_GRID;
                else if (PROB == PDEVAL_PROBLEM_FORCE_FREE && a.prm.strict_symbolic &&
                         (hdr & PDEVAL_FLAG_NONSMOOTH2D)) cls = PDEVAL_CLS_REJECT_SYMBOLIC;
                else cls = PDEVAL_CLS_ACCEPT;
            }
            if (a.out.status) a.out.status[cand] = (uint8_t)cls;
            if (a.out.q_ref) a.out.q_ref[cand] = q_ref;
            if (a.out.q_grid) a.out.q_grid[cand] = qmax;
            if (a.out.n_bad) a.out.n_bad[cand] = nbad;
            if (a.out.n_nonfinite) a.out.n_nonfinite[cand] = nnonfin;
            if (a.out.verdict_bits) {
                const uint32_t bit = 1u << (cand & 31);
                uint32_t* wp = (uint32_t*)a.out.verdict_bits + (cand >> 5);
                if (cls == PDEVAL_CLS_ACCEPT) atomicOr(wp, bit);
                else atomicAnd(wp, ~bit);
            }
        }
    }
}

}  // namespace pd
