// pdeval_point.h -- the point stage: the reference's first verdict stage, decided for every
// candidate before the grid passes run.
//
// The reference evaluates its residual EXACTLY at its test point(s):
//   force-free  det at (rho, z) = (4/5, 6/7): reject when cancel(together(det)) is a non-zero
//               Number ("Invalid (point check != 0)") or when |evalf(50)| >= 1e-20 ("Invalid
//               (point check ~ x.xxe+yy)"), pass otherwise      (problems/force_free/validator.py:349-402)
//   Kerr        lhs at (5/2, 3/5), (7/3, 1/3), (5, -2/5), N(., 40): reject when non-real or when
//               max |lhs| >= 1e-10 (absolute)                   (kerr_magnetosphere/validator.py:163-192)
// Here every reference point is evaluated with the error-bounded interpreter (pdeval_tier2.h),
// which carries a first-order bound `noise` of the rounding error beside the value:
//   tier A (fp64): decide where the bound makes the answer certain and the value accurate to
//           res_rel_acc (noise <= 1e-11 |res|, so the reported residual is within 1e-10 of the
//           exact one);
//           where |res| <= kappa*noise the point passes PROVISIONALLY (P0_PROV): the exact value
//           may be 0 (a true solution) or a non-zero hidden in fp64 noise;
//   tier B (double-double, dd.h, at the end of the call): the undecided candidates (P0_DD) and
//           every provisional pass that reached a verdict-bearing class (ACCEPT, REJECT_GRID,
//           REJECT_SYMBOLIC) -- exactly the candidates whose class depends on the hidden value --
//           are re-evaluated with ~106-bit arithmetic, reference points and constants as
//           double-doubles, and decided for good (noise unit 2^-100).
// A provisional pass whose grid stage ACCEPTS is re-evaluated too: the grid accept is a
// tolerance test (q <= tau_grid), so a non-zero determinant that is below 1e-7 of its magnitude
// shadow on the whole grid would pass it, while the reference rejects it at p* (an exact
// non-zero Number, or |det| >= 1e-20).  Accepts are a minority of a batch, so this is cheap.
// Kernels (launch order in pdeval.hip):
//   point_kernel         pass 0: all candidates of stack <= 2, real, one candidate per lane
//   point_list_kernel    deeper real programs (list), then the complex candidates (list)
//   dd_collect_kernel    builds the tier-B lists from pstate and the final classes
//   dd_point_kernel      tier B, real (dd) and complex (cdd) lists
#pragma once
#include "pdeval_tier2.h"

namespace pd {

PD_HD double re_hi(double v) { return v; }
PD_HD double re_hi(cplx v) { return v.re; }
PD_HD double re_hi(dd v) { return v.hi; }
PD_HD double re_hi(cdd v) { return v.re.hi; }
PD_HD double im_hi(double) { return 0.0; }
PD_HD double im_hi(cplx v) { return v.im; }
PD_HD double im_hi(dd) { return 0.0; }
PD_HD double im_hi(cdd v) { return v.im.hi; }

// reference point k (uniform within the loop over points) as the coordinate type V
template <class V> __device__ __forceinline__ V ref_coord(const KernelArgs& a, int k, int axis);
template <> __device__ __forceinline__ double ref_coord<double>(const KernelArgs& a, int k, int axis) {
    const double* t = axis ? a.ref_y : a.ref_x;
    return k == 0 ? t[0] : (k == 1 ? t[1] : (k == 2 ? t[2] : t[3]));
}
template <> __device__ __forceinline__ dd ref_coord<dd>(const KernelArgs& a, int k, int axis) {
    const dd* t = axis ? a.ref_yd : a.ref_xd;
    return k == 0 ? t[0] : (k == 1 ? t[1] : (k == 2 ? t[2] : t[3]));
}

// force-free Omega^2 as the coordinate type V: the double omega2, or omega2 + omega2_lo (a
// rational Omega^2 that is no double, Omega = 1/3) -- and the bound, relative to the residual's
// scale S, of what that representation error moves the determinant (bilinear in Omega^2 through
// A and B: twice its relative error, doubled for margin; dd: 2^-106 relative, well under the
// double-double noise unit)
template <class V> __device__ __forceinline__ V om2_of(const KernelArgs& a);
template <> __device__ __forceinline__ double om2_of<double>(const KernelArgs& a) { return a.prm.omega2; }
template <> __device__ __forceinline__ dd om2_of<dd>(const KernelArgs& a) { return {a.prm.omega2, a.prm.omega2_lo}; }
template <class V> __device__ __forceinline__ double om2_err(const KernelArgs& a) {
    if (a.prm.omega2_lo == 0.0) return 0.0;
    return std::is_same<V, dd>::value ? 0x1p-104 : 4.0 * fabs(a.prm.omega2_lo / a.prm.omega2);
}

// Kerr operator coefficients at reference point k, double-double (selects, as ref_coord)
__device__ __forceinline__ void kc_ref_at(const KernelArgs& a, int k, dd (&kc)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
        kc[i] = k == 0 ? a.kc_ref[i] : (k == 1 ? a.kc_ref[4 + i] : (k == 2 ? a.kc_ref[8 + i] : a.kc_ref[12 + i]));
}

// the problem's constants of the point stage (grid = false) or of the constant test / grid stage
template <class V> __device__ __forceinline__ const PrmTab<V>& stage_prm(const KernelArgs& a, bool grid);
template <> __device__ __forceinline__ const PrmTab<double>& stage_prm<double>(const KernelArgs& a, bool grid) {
    return grid ? a.prm_grid : a.prm_pt;
}
template <> __device__ __forceinline__ const PrmTab<dd>& stage_prm<dd>(const KernelArgs& a, bool grid) {
    return grid ? a.prm_grid_dd : a.prm_pt_dd;
}

struct PtEval {
    double res_re, res_im, res_abs;  // residual (hi parts)
    double S, noise;                 // magnitude scale and first-order noise bound
    double u0;                       // fingerprint value at the point (fp_value)
    bool finite, grad_zero;
    bool grad_noise;                 // |u_x|, |u_y| within kappa x their rounding-error bounds
    bool tiny;                       // Kerr: u's jet underflowed (kTinyJet): a passing point
    int rc;                          // RUN_*
};

// Kerr operator with coefficients of type KC (double table or dd at the reference points)
template <class T, class KC> __device__ __forceinline__ T kerr_lhs(const T* u, const KC* k, double* S) {
    const T t1 = u[ji(2, 0)] * cvt<T>(k[0] * 2.0);
    const T t2 = u[ji(0, 2)] * cvt<T>(k[1] * 2.0);
    const T t3 = u[ji(1, 0)] * cvt<T>(k[2]);
    const T t4 = u[ji(0, 1)] * cvt<T>(k[3]);
    *S = (mag(t1) + mag(t2)) + (mag(t3) + mag(t4));
    return (t1 + t2) + (t3 + t4);
}

// Value and noise bound of one program at reference point k.
template <int PROB, class T, class V, int MAXD, bool VEC, class STK>
__device__ __forceinline__ PtEval point_eval(const KernelArgs& a, const int32_t* prog, int plen, int k,
                                             STK& stk) {
    constexpr int K = PROB == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
    constexpr int NC = nc(K);
    using EI = ErrInterp<T, K, MAXD, V>;
    PtEval r{};
    const V x = ref_coord<V>(a, k, 0), y = ref_coord<V>(a, k, 1);
    typename EI::J u;
    double e[NC];
    // the reference points are rounded to the coordinate type: half a unit of fp64, ~2^-7 of the
    // double-double noise unit (dd_unit = 2^-100 against a rounding of 2^-107)
    const double cerr = std::is_same<V, dd>::value ? 0x1p-6 : 0.5;
    r.rc = EI::template run_s<VEC>(prog, 1, plen, x, y, u, e, stk, stage_prm<V>(a, false), cerr);
    if (r.rc != RUN_OK) return r;
    double m[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) m[i] = mag(u.c[i]);
    const double* kc = a.kc ? a.kc + 4 * k : nullptr;
    T res;
    if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) {
        res = FFEpi<T, false>::eval(u.c, x, om2_of<V>(a));
        r.S = FFEpi<double, true>::eval(m, hi_of(x), a.prm.omega2);
    } else {
        if constexpr (std::is_same<V, dd>::value) {
            dd kcd[4];
            kc_ref_at(a, k, kcd);
            res = kerr_lhs<T, dd>(u.c, kcd, &r.S);
        }
        else res = kerr_lhs<T, double>(u.c, kc, &r.S);
    }
    const double unit = std::is_same<V, dd>::value ? dd_unit() / kEps : 1.0;
    r.noise = residual_noise<PROB, T>(u.c, e, hi_of(x), kc, r.S, a.prm.omega2) * unit;
    if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) r.noise += om2_err<V>(a) * r.S;
    r.res_re = re_hi(res);
    r.res_im = im_hi(res);
    r.res_abs = mag(res);
    r.u0 = re_hi(u.c[0]) + kFpIm * im_hi(u.c[0]);   // (fp_value)
    r.grad_zero = is_zero(u.c[ji(1, 0)]) && is_zero(u.c[ji(0, 1)]);
    // coefficient i is within eps * e[i] of exact (first order; dd: dd_unit * e[i])
    const double gk = a.prm.noise_kappa * kEps * unit;
    r.grad_noise = m[ji(1, 0)] <= gk * e[ji(1, 0)] && m[ji(0, 1)] <= gk * e[ji(0, 1)];
    bool fin = finite_(res) && isfinite(r.S) && isfinite(r.noise);
#pragma unroll
    for (int i = 0; i < NC; ++i) fin = fin && m[i] < kHugeJet;
    r.finite = fin;
    if constexpr (PROB != PDEVAL_PROBLEM_FORCE_FREE) {
        if (underflowed<T, NC>(m, e)) {
            r.tiny = true;
            r.finite = true;
            r.grad_noise = false;
        }
    }
    return r;
}

// Kerr constant test at the stand-ins of the symbols (kerr validator.py:231-240: u is dropped
// when simplify(u), with M and a symbolic, has neither r nor x).  Run only for candidates whose
// gradient is rounding noise at every reference point in the point stage's constants: then at
// every constant-test point (the reference points and two more, so that a u merely stationary
// at the reference points is not taken for a constant) with the grid stage's constants, the
// gradient must lie within kappa x its first-order rounding bound.
template <int PROB, class T, class V, int MAXD, bool VEC, class STK>
__device__ __forceinline__ bool kerr_constant_test(const KernelArgs& a, const int32_t* prog, int plen, STK& stk) {
    constexpr int K = 2;
    constexpr int NC = nc(K);
    using EI = ErrInterp<T, K, MAXD, V>;
    const double unit = std::is_same<V, dd>::value ? dd_unit() / kEps : 1.0;
    const double gk = a.prm.noise_kappa * kEps * unit;
    for (int p = 0; p < a.n_ct && p < 8; ++p) {
        typename EI::J u;
        double e[NC];
        const V x = cvt<V>(a.ct_x[p]), y = cvt<V>(a.ct_y[p]);
        if (EI::template run_s<VEC>(prog, 1, plen, x, y, u, e, stk, stage_prm<V>(a, true), 0.0) != RUN_OK)
            return false;
        double m[NC];
        bool fin = true;
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            m[i] = mag(u.c[i]);
            fin = fin && m[i] < kHugeJet;
        }
        // an underflowed jet is no evidence of a constant
        if (!fin || underflowed<T, NC>(m, e) || m[ji(1, 0)] > gk * e[ji(1, 0)] || m[ji(0, 1)] > gk * e[ji(0, 1)])
            return false;
    }
    return true;
}

// ---- decision rules.  FINAL = the double-double tier (nothing is left undecided).
// Force-free (validator.py:371-397): returns P0_PASS / P0_REJECT, | P0_PROV, | P0_DD, | P0_NZ.
// P0_DD alone with P0_PASS: the class is undecided in fp64 (the grid passes treat it as passed);
// P0_DD with a decided class: only the reported residual needs the double-double value.
// P0_NZ with P0_PASS: certainly non-zero but below 1e-20 (not a solution: det is not == 0).
template <bool FINAL>
__device__ __forceinline__ uint8_t ff_point_rule(double res_abs, double noise, bool rational,
                                                 const pdeval_params& prm) {
    const double kn = prm.noise_kappa * noise;
    if (res_abs > kn) {                                    // certainly non-zero
        // accuracy of the reported value: the first-order bound itself (kappa is the safety
        // factor of the zero DECISION; 1e-11 leaves x10 to the 1e-10 requirement)
        const uint8_t acc = (!FINAL && noise > prm.res_rel_acc * res_abs) ? P0_DD : 0;
        if (rational) return P0_REJECT | acc;             // an exact Number != 0
        if (res_abs - kn >= prm.point_abs_tol) return P0_REJECT | acc;   // |evalf(50)| >= 1e-20
        if (res_abs + kn < prm.point_abs_tol) return P0_PASS | P0_NZ | acc;   // non-zero below 1e-20
        if (!FINAL) return P0_DD | P0_PASS;
        return res_abs >= prm.point_abs_tol ? P0_REJECT : (uint8_t)(P0_PASS | P0_NZ);
    }
    return FINAL ? P0_PASS : (uint8_t)(P0_PASS | P0_PROV);
}

// Kerr, one reference point (kerr validator.py:190, absolute tolerance): 0 pass, 1 reject,
// 2 undecided in fp64; | 4: the value is not accurate enough to report (double-double value);
// | 8: the value is certainly non-zero (beyond kappa x its noise bound).
template <bool FINAL>
__device__ __forceinline__ int kerr_point_rule(double res_abs, double noise, const pdeval_params& prm) {
    const double kn = prm.noise_kappa * noise;
    const int nz = res_abs > kn ? 8 : 0;
    if (FINAL) return (res_abs >= prm.kerr_abs_tol ? 1 : 0) | nz;
    const int acc = (res_abs > kn && noise > prm.res_rel_acc * res_abs) ? 4 : 0;
    if (res_abs - kn >= prm.kerr_abs_tol) return 1 | acc | nz;
    if (res_abs + kn < prm.kerr_abs_tol) return 0 | acc | nz;
    return 2;
}

// The point stage of one candidate (per lane).  Returns the P0_* state; writes q_ref, res_ref and
// the fingerprint of point 0.  *nonfinite: some reference point is not finite (force-free real
// pass: the complex pass takes the candidate).
template <int PROB, class T, class V, int MAXD, bool VEC, bool FINAL, class STK>
__device__ __forceinline__ uint8_t point_stage(const KernelArgs& a, int64_t cand, const int32_t* prog, int plen,
                                               uint32_t hdr, STK& stk, bool* nonfinite, bool* prog_err) {
    double qr = 0.0;
    bool nf = false, grad = false, rej = false, und = false, inacc = false, gconst = true, nzk = false;
    uint8_t ff = P0_PASS;
    *prog_err = false;
    for (int p = 0; p < a.n_ref; ++p) {
        const PtEval r = point_eval<PROB, T, V, MAXD, VEC>(a, prog, plen, p, stk);
        if (r.rc != RUN_OK) {
            *prog_err = true;
            return P0_NONE;
        }
        if (p == 0 && a.out.fingerprint) a.out.fingerprint[cand * PDEVAL_FP_N] = r.u0;
        // the fp64 noise bound, reused (rescaled) by the double-double tier
        if (!FINAL && a.noise_ref) a.noise_ref[cand * a.n_ref + p] = r.noise;
        // (a complex residual: its modulus with the sign of its real part)
        if (a.out.res_ref) a.out.res_ref[cand * a.n_ref + p] = r.res_im == 0.0 ? r.res_re : copysign(r.res_abs, r.res_re);
        gconst = gconst && r.finite && r.grad_noise;
        if (!r.finite) {
            nf = true;
            // finite, but a coefficient beyond the 2^160 guard: a sure reject whose value the
            // double-double tier still reports accurately
            if (!FINAL && isfinite(r.res_abs) && isfinite(r.S)) inacc = true;
            continue;
        }
        if (!r.grad_zero) grad = true;
        if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) {
            qr = scaled(r.res_abs, r.S);
            ff = ff_point_rule<FINAL>(r.res_abs, r.noise, (hdr & PDEVAL_FLAG_RATIONAL) != 0, a.prm);
        } else {
            qr = fmax(qr, r.res_abs);
            if (r.tiny) continue;   // underflowed: |lhs| far below the threshold
            const int k = kerr_point_rule<FINAL>(r.res_abs, r.noise, a.prm);
            rej = rej || (k & 3) == 1;
            und = und || (k & 3) == 2;
            inacc = inacc || (k & 4);
            nzk = nzk || (k & 8);
        }
    }
    *nonfinite = nf;
    if (a.out.q_ref) a.out.q_ref[cand] = qr;
    uint8_t ps;
    if (nf) ps = P0_REJECT;    // Kerr: non-real / NaN at a test point; FF complex: not finite
    else if (PROB == PDEVAL_PROBLEM_FORCE_FREE) ps = ff;
    else ps = und ? (uint8_t)(P0_DD | P0_PASS) : (rej ? P0_REJECT : P0_PASS);
    if (PROB != PDEVAL_PROBLEM_FORCE_FREE && nzk && !nf && !rej) ps |= P0_NZ;
    if (inacc) ps |= P0_DD;
    if (grad) ps |= P0_GRAD;
    if constexpr (PROB != PDEVAL_PROBLEM_FORCE_FREE) {
        // a program with no coordinate is a constant structurally (simplify(u) has neither r
        // nor x); otherwise the numeric constant test
        if ((hdr & PDEVAL_FLAG_NOCOORD) ||
            (gconst && kerr_constant_test<PROB, T, V, MAXD, VEC>(a, prog, plen, stk)))
            ps |= P0_CONST;
    }
    return ps;
}

// A point reject is final: with full_grid = 0 the grid passes skip the candidate (the
// reference's control flow), so its outputs are written here.
__device__ __forceinline__ void write_point_reject(const KernelArgs& a, int64_t cand) {
    if (a.out.status) a.out.status[cand] = PDEVAL_CLS_REJECT_POINT;
    if (!a.prm.full_grid) {
        if (a.out.q_grid) a.out.q_grid[cand] = 0.0;
        if (a.out.n_bad) a.out.n_bad[cand] = 0;
        if (a.out.n_nonfinite) a.out.n_nonfinite[cand] = 0;
    }
}

__device__ __forceinline__ bool prog_bounds(const KernelArgs& a, int64_t cand, int64_t* beg, int64_t* end) {
    *beg = a.offsets[cand];
    *end = a.offsets[cand + 1];
    return *beg >= 0 && *end > *beg && *end <= a.n_words && *end - *beg < (1 << 24);
}

// Pass 0: every candidate, one per LANE (the lanes of a wave interpret different programs: a
// divergent dispatch, still ~64x the lane use of a wave per candidate at one point).  Real
// programs of stack <= 2 are decided here (operand stack in LDS); deeper ones go to the deep
// point pass, complex-valued ones (FF) to the complex list.
template <int PROB>
__global__ __launch_bounds__(256, 1) void point_kernel(KernelArgs a) {
    constexpr int K = (PROB == PDEVAL_PROBLEM_FORCE_FREE) ? 4 : 2;
    constexpr int NC = nc(K);
    constexpr int MAXD = 2;
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
#ifndef PD_HOST_SIM
    extern __shared__ __align__(16) unsigned char pd_lds[];
#else
    static unsigned char pd_lds[1];
#endif
    double* vs = reinterpret_cast<double*>(pd_lds) + (size_t)wib * 2 * (MAXD - 1) * NC * 64;
    double* es = vs + (size_t)(MAXD - 1) * NC * 64;
    LdsStack<double, NC> stk{vs, es, lane};
    const int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= a.n) return;
    const int64_t cand = a.perm ? checked_cand(a, (int64_t)a.perm[li], ERRW_PERM) : li;   // lanes take programs sorted by shape
    if (cand < 0) return;
    int64_t beg, end;
    uint8_t ps = P0_NONE;
    if (prog_bounds(a, cand, &beg, &end)) {
        const int32_t* prog = a.ops + beg;
        const uint32_t hdr = (uint32_t)prog[0];
        const int depth = (int)((hdr >> 8) & 0xffu);
        if ((hdr & 0xffu) == 0u && depth <= PDEVAL_MAX_STACK) {
            if (hdr & PDEVAL_FLAG_COMPLEX) {
                if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) {
                    if (a.cplx_list && list_append(a.cplx_list, a.cplx_count, a.list_capacity, cand)) ps = P0_CPLX;
                } else {
                    ps = P0_REJECT;          // Kerr: non-real at a test point (kerr validator.py:179-180)
                }
            } else if (depth > MAXD) {
                if (a.pdeep_list) list_append(a.pdeep_list, a.pdeep_count, a.list_capacity, cand);
            } else {
                bool nf, perr;
                const uint8_t s = point_stage<PROB, double, double, MAXD, true, false>(
                    a, cand, prog, (int)(end - beg), hdr, stk, &nf, &perr);
                if (!perr) {
                    if (nf && PROB == PDEVAL_PROBLEM_FORCE_FREE) {
                        // not real at p*: the complex passes decide (SymPy evaluates the point
                        // exactly, in the complex field: validator.py:363-402)
                        if (a.cplx_list && list_append(a.cplx_list, a.cplx_count, a.list_capacity, cand))
                            ps = P0_CPLX;
                    } else {
                        ps = s;
                    }
                }
            }
        }
    }
    a.pstate[cand] = ps;
    if ((ps & 3) == P0_REJECT) write_point_reject(a, cand);
}

// The point stage over a device list, one candidate per lane, operand stack in private memory:
// T = double for the real programs deeper than pass 0 takes, T = cplx for the complex list.
template <int PROB, class T>
__global__ __launch_bounds__(64, 1) void point_list_kernel(KernelArgs a) {
    constexpr int K = (PROB == PDEVAL_PROBLEM_FORCE_FREE) ? 4 : 2;
    constexpr int MAXD = PDEVAL_MAX_STACK;
    int64_t nwork = (int64_t)(*a.list_count);
    if (nwork > a.list_capacity) nwork = a.list_capacity;
    PrivStack<T, nc(K), MAXD - 1> stk;
    for (int64_t wi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; wi < nwork;
         wi += (int64_t)gridDim.x * blockDim.x) {
        const int64_t cand = checked_cand(a, a.list[wi], ERRW_POINT_LIST);
        int64_t beg, end;
        if (cand < 0 || !prog_bounds(a, cand, &beg, &end)) continue;   // pass 0 checked these
        const int32_t* prog = a.ops + beg;
        const uint32_t hdr = (uint32_t)prog[0];
        bool nf, perr;
        uint8_t s = point_stage<PROB, T, double, MAXD, true, false>(a, cand, prog, (int)(end - beg), hdr, stk,
                                                                   &nf, &perr);
        uint8_t ps = P0_NONE;
        if (!perr) {
            if constexpr (Real<T>::cplx_pass) {
                ps = (uint8_t)(s | P0_CPLX);   // not finite even in the complex field: reject
            } else {
                if (nf && PROB == PDEVAL_PROBLEM_FORCE_FREE) {
                    if (a.cplx_list && list_append(a.cplx_list, a.cplx_count, a.list_capacity, cand)) ps = P0_CPLX;
                } else {
                    ps = s;
                }
            }
        } else if constexpr (Real<T>::cplx_pass) {
            ps = P0_CPLX;   // malformed: the complex grid pass classifies it (chunk 0)
        }
        a.pstate[cand] = ps;
        if ((ps & 3) == P0_REJECT) write_point_reject(a, cand);
    }
}

// Tier-B lists: the candidates whose point stage fp64 left undecided, and the provisional
// passes whose final class is an accept or a grid reject (either may really be a point reject).
// A point pass certainly non-zero (P0_NZ) that the grid accepted is a REJECT_GRID: the residual
// is not identically zero (the reference's symbolic stage fails on it).
__device__ __forceinline__ void nz_reject(const KernelArgs& a, int64_t cand) {
    a.out.status[cand] = PDEVAL_CLS_REJECT_GRID;
    if (a.out.verdict_bits) atomicAnd((uint32_t*)a.out.verdict_bits + (cand >> 5), ~(1u << (cand & 31)));
}

// The tier-B lists.  EARLY (right after the point stage, before the grid): the candidates the
// point stage left undecided or not accurate enough in fp64 (P0_DD) -- known before any grid
// pass, so their double-double evaluation runs on a second stream beside the grid passes
// (dd_point_kernel<DEFER>) and dd_apply_kernel applies it once the classes are final.  LATE
// (after the grid): the provisional point passes (P0_PROV) whose grid class the double-double
// value may still override; and the P0_NZ accepts.
// MODE: DD_ALL (one tier after the grid: both kinds), DD_EARLY, DD_LATE.
enum { DD_ALL = 0, DD_EARLY = 1, DD_LATE = 2 };
template <int PROB, int MODE>
__global__ __launch_bounds__(256) void dd_collect_kernel(KernelArgs a) {
    const int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= a.n) return;
    const int64_t cand = a.perm ? checked_cand(a, (int64_t)a.perm[li], ERRW_PERM) : li;   // lists in shape order
    if (cand < 0) return;
    const uint8_t ps = a.pstate[cand];
    if ((ps & 3) == P0_NONE) return;
    // (a.dd_spec: the early tier also takes the provisional passes, speculatively)
    const uint8_t early_bits = (uint8_t)(P0_DD | (a.dd_spec ? P0_PROV : 0));
    if (MODE == DD_EARLY) {
        if (!(ps & early_bits)) return;
    } else {
        if (MODE == DD_LATE && (ps & early_bits)) return;      // the early tier took it
        const uint8_t st = a.out.status[cand];
        const bool need = (MODE == DD_ALL && (ps & P0_DD)) ||
                          ((ps & P0_PROV) && (st == PDEVAL_CLS_ACCEPT || st == PDEVAL_CLS_REJECT_GRID ||
                                                st == PDEVAL_CLS_REJECT_SYMBOLIC));
        if (!need) {
            if ((ps & 3) == P0_PASS && (ps & P0_NZ) && st == PDEVAL_CLS_ACCEPT) nz_reject(a, cand);
            return;
        }
    }
    if (ps & P0_CPLX) {
        list_append(a.cplx_list, a.cplx_count, a.list_capacity, cand);
    } else {
        const int depth = (int)((a.ops[a.offsets[cand]] >> 8) & 0xff);
        if (depth <= 2) list_append(a.defer_list, a.defer_count, a.list_capacity, cand);
        else list_append(a.esc_list, a.esc_count, a.list_capacity, cand);
    }
}

// ---- the double-double tier's evaluator: values only.  Its noise bound is the fp64 one
// rescaled from eps = 2^-52 to dd_unit() = 2^-100: the first-order error jets depend on the
// magnitudes of the values (the same to first order in both precisions) and on the unit, so
// the rescaled bound holds for the double-double evaluation (the coordinates' rounding term is
// then 64x too large, which errs on the safe side).
template <class T, int NC> struct LdsVStack {
    T* vs;
    int lane;
    __device__ __forceinline__ void store(int slot, const T* t) {
#pragma unroll
        for (int c = 0; c < NC; ++c) vs[(slot * NC + c) * 64 + lane] = t[c];
    }
    __device__ __forceinline__ void load(int slot, T* t) const {
#pragma unroll
        for (int c = 0; c < NC; ++c) t[c] = vs[(slot * NC + c) * 64 + lane];
    }
};
template <class T, int NC, int SLOTS> struct PrivVStack {
    T v[SLOTS][NC];
    __device__ __forceinline__ void store(int slot, const T* t) {
#pragma unroll
        for (int c = 0; c < NC; ++c) v[slot][c] = t[c];
    }
    __device__ __forceinline__ void load(int slot, T* t) const {
#pragma unroll
        for (int c = 0; c < NC; ++c) t[c] = v[slot][c];
    }
};

// program words [pc, end) at (x, y) in jets over T with coordinates / constants of type V
// (one candidate per lane: vector loads of the program)
template <class T, int K, int MAXD, class V> struct ValInterp {
    using O = JetOps<T, K>;
    using J = typename O::J;
    template <class STK>
    static __device__ PD_DD_INLINE_ATTR int run(const int32_t* ops, int pc, int end, V x, V y, J& acc, STK& stk,
                              const PrmTab<V>& P) {
        int d = 0;
        if (pc >= end) return RUN_BAD;
        for (;;) {
            const uint32_t w = (uint32_t)ops[pc];
            const uint32_t op = w & 0xffu;
            V immv = vzero<V>();
            int npc = pc + 1;
            if (op_has_imm(op)) {
                npc = pc + ((w & PDEVAL_IMM_DD) ? 5 : 3);
                if (npc > end) return RUN_BAD;
                immv = read_imm<V, true>(ops + pc + 1, w, P);
            }
            switch (op) {
                case PDOP_PUSH_X: case PDOP_PUSH_Y: case PDOP_PUSH_C: case PDOP_PUSH_I:
                    if (d > 0 && d < MAXD) stk.store(d - 1, acc.c);
                    if (op == PDOP_PUSH_X) O::set_var(acc, x, 0);
                    else if (op == PDOP_PUSH_Y) O::set_var(acc, y, 1);
                    else if (op == PDOP_PUSH_C) O::set_const(acc, cvt<T>(immv));
                    else {
                        if constexpr (Real<T>::cplx_pass) O::set_const(acc, imag_unit<T>());
                        else return RUN_UNSUPPORTED;
                    }
                    ++d;
                    break;
                case PDOP_ADD: case PDOP_SUB: case PDOP_RSUB:
                case PDOP_MUL: case PDOP_DIV: case PDOP_RDIV:
                    if (d >= 2 && d <= MAXD) {
                        J lhs;
                        stk.load(d - 2, lhs.c);
                        Interp<T, K, MAXD>::binop(op, lhs, acc);
                    }
                    --d;
                    break;
                case PDOP_ADDC: acc.c[0] = acc.c[0] + cvt<T>(immv); break;
                case PDOP_MULC: O::scale(acc, cvt<T>(immv)); break;
                case PDOP_RDIVC: O::rdivc(acc, cvt<T>(immv)); break;
                case PDOP_PUSH_P: case PDOP_ADD_P: case PDOP_SUB_P: case PDOP_MUL_P: case PDOP_DIV_P:
                case PDOP_RDIV_P: {
                    V pk[K + 1];
                    const int n = (int)((w >> 8) & 0xffu);
                    if (op == PDOP_PUSH_P && d > 0 && d < MAXD) stk.store(d - 1, acc.c);
                    if ((w >> 16) & 1) {
                        O::pcoefs(y, n, pk);
                        if (op == PDOP_PUSH_P) O::template set_p<1>(acc, pk);
                        else O::template p_op<1>(op, acc, pk);
                    } else {
                        O::pcoefs(x, n, pk);
                        if (op == PDOP_PUSH_P) O::template set_p<0>(acc, pk);
                        else O::template p_op<0>(op, acc, pk);
                    }
                    if (op == PDOP_PUSH_P) ++d;
                    break;
                }
                case PDOP_NEG: O::scale(acc, from_real<T>(-1.0)); break;
                case PDOP_ADD_X: case PDOP_ADD_Y: case PDOP_SUB_X: case PDOP_SUB_Y: {
                    const bool isx = (op == PDOP_ADD_X || op == PDOP_SUB_X);
                    const double sg = (op == PDOP_ADD_X || op == PDOP_ADD_Y) ? 1.0 : -1.0;
                    acc.c[0] = acc.c[0] + cvt<T>((isx ? x : y) * sg);
                    const int idx = isx ? ji(1, 0) : ji(0, 1);
                    acc.c[idx] = acc.c[idx] + from_real<T>(sg);
                    break;
                }
                case PDOP_MUL_X: O::mul_var(acc, x, 0); break;
                case PDOP_MUL_Y: O::mul_var(acc, y, 1); break;
                case PDOP_DIV_X: O::div_var(acc, x, 0); break;
                case PDOP_DIV_Y: O::div_var(acc, y, 1); break;
                case PDOP_POWN: O::pown(acc, (int)((w >> 8) & 0xffu)); break;
                case PDOP_POW: O::powa(acc, hi_of(immv)); break;
                case PDOP_SQRT: O::sqrtj(acc); break;
                case PDOP_EXP: O::expj(acc); break;
                case PDOP_LOG: O::logj(acc); break;
                case PDOP_ABS: absj<K>(acc); break;
                default: return RUN_UNSUPPORTED;
            }
            if (npc >= end) break;
            pc = npc;
        }
        return d == 1 ? RUN_OK : RUN_BAD;
    }
};

// The double-double tier for one candidate: values at every reference point, the rescaled
// fp64 noise bounds, the final rule; writes res_ref and q_ref.  Returns the P0_* class bits
// (P0_NONE: not evaluated -- program error or not finite, the fp64 decision stands).
template <int PROB, class T, int MAXD, class STK>
__device__ __forceinline__ uint8_t dd_point_stage(const KernelArgs& a, int64_t cand, const int32_t* prog, int plen,
                                                  uint32_t hdr, STK& stk, double* res_out, double* q_out) {
    constexpr int K = PROB == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
    constexpr int NC = nc(K);
    double qr = 0.0;
    bool rej = false, fin_all = true, nzk = false;
    uint8_t ff = P0_PASS;
    for (int p = 0; p < a.n_ref; ++p) {
        // (selects, not a.ref_xd[p]: a dynamic index into the by-value kernel arguments made
        // the compiler copy them to scratch -- ~1.9 KB per lane of this kernel's 2 KB)
        const dd x = ref_coord<dd>(a, p, 0), y = ref_coord<dd>(a, p, 1);
        typename ValInterp<T, K, MAXD, dd>::J u;
        if (ValInterp<T, K, MAXD, dd>::run(prog, 1, plen, x, y, u, stk, a.prm_pt_dd) != RUN_OK) return P0_NONE;
        double m[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) m[i] = mag(u.c[i]);
        T res;
        double S;
        if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) {
            res = FFEpi<T, false>::eval(u.c, x, om2_of<dd>(a));
            S = FFEpi<double, true>::eval(m, x.hi, a.prm.omega2);
        } else {
            dd kc[4];
            kc_ref_at(a, p, kc);
            res = kerr_lhs<T, dd>(u.c, kc, &S);
        }
        const double res_abs = mag(res);
        const double noise = a.noise_ref[cand * a.n_ref + p] * (dd_unit() / kEps);
        if constexpr (PROB != PDEVAL_PROBLEM_FORCE_FREE) {
            bool tiny = true;
#pragma unroll
            for (int i = 0; i < NC; ++i) tiny = tiny && m[i] < kTinyJet;
            if (tiny) {   // underflowed: a passing point (kTinyJet)
                if (res_out) res_out[p] = re_hi(res);
                qr = fmax(qr, res_abs);
                continue;
            }
        }
        bool fin = finite_(res) && isfinite(S) && isfinite(noise);
#pragma unroll
        for (int i = 0; i < NC; ++i) fin = fin && m[i] < kHugeJet;
        const double rr = re_hi(res), ri = im_hi(res);
        if (isfinite(res_abs) && res_out) res_out[p] = ri == 0.0 ? rr : copysign(res_abs, rr);
        if (!fin) {
            fin_all = false;
            continue;
        }
        if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) {
            qr = scaled(res_abs, S);
            ff = ff_point_rule<true>(res_abs, noise, (hdr & PDEVAL_FLAG_RATIONAL) != 0, a.prm);
        } else {
            qr = fmax(qr, res_abs);
            const int k = kerr_point_rule<true>(res_abs, noise, a.prm);
            rej = rej || (k & 3) == 1;
            nzk = nzk || (k & 8);
        }
    }
    // Kerr: a reference point where even the double-double value is not finite is a pole (or
    // a value beyond fp64): the reference's N(., 40) is zoo / nan / a float overflow there, a
    // reject either way (kerr validator.py:178-190).  Force-free keeps the fp64 decision.
    if (!fin_all) return PROB == PDEVAL_PROBLEM_FORCE_FREE ? P0_NONE : P0_REJECT;
    if (q_out) *q_out = qr;
    if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) return ff & (3 | P0_NZ);
    else return rej ? P0_REJECT : (uint8_t)(nzk ? P0_PASS | P0_NZ : P0_PASS);
}

// Tier B: the point stage in double-double (T = dd, or cdd for complex candidates), final,
// one candidate per lane over a device list.  MAXD = 2: operand stack in LDS (the common
// case); deeper or complex programs: private memory.
// waves/SIMD of the stack-2 double-double kernel: at 1 its register spill goes to AGPRs
// (scratch 0, 144 B/lane at 2), and the same-box A/B (profiles/r04_z*) measured no difference in
// the 2^21 step or the worker batch's device call
#ifndef PD_DD2_WAVES
#define PD_DD2_WAVES 1
#endif
// the double-double class s of a candidate, applied to its final grid class
__device__ __forceinline__ void dd_apply_one(const KernelArgs& a, int64_t cand, uint8_t s) {
    const uint8_t st = a.out.status ? a.out.status[cand] : (uint8_t)PDEVAL_CLS_ACCEPT;
    // the reference checks the gradient (and Kerr the constant) before the point stage
    const bool overridable = st == PDEVAL_CLS_ACCEPT || st == PDEVAL_CLS_REJECT_GRID ||
                             st == PDEVAL_CLS_REJECT_SYMBOLIC;
    if ((s & 3) == P0_REJECT && overridable) {
        write_point_reject(a, cand);
        if (a.out.verdict_bits)
            atomicAnd((uint32_t*)a.out.verdict_bits + (cand >> 5), ~(1u << (cand & 31)));
    } else if ((s & 3) == P0_PASS && (s & P0_NZ) && st == PDEVAL_CLS_ACCEPT) {
        nz_reject(a, cand);
    }
    a.pstate[cand] = (uint8_t)((a.pstate[cand] & ~(3 | P0_DD | P0_PROV | P0_NZ)) | s);
}

// "keep the fp64 decision" in a.ddps (never a final class: those have no P0_DD bit)
constexpr uint8_t kDdKeep = 0xfe;
// a side-array value the double-double tier did not write (a quiet NaN it never produces: it
// writes finite residuals only, and q_ref only when every point was finite)
constexpr long long kDdUnset = 0x7ff8dead0000beefll;
// an early-list entry that is a speculative provisional pass (not a P0_DD candidate)
__device__ __forceinline__ bool dd_spec_entry(const KernelArgs& a, int64_t cand) {
    const uint8_t ps = a.pstate[cand];
    return a.dd_spec && (ps & P0_PROV) && !(ps & P0_DD);
}

// DEFER (the early lists, on the second stream while the grid passes run): the class goes to
// a.ddps[cand] and dd_apply_kernel applies it after the grid; nothing else the grid passes
// read or write is touched here (res_ref, q_ref and the p* fingerprint are the point stage's).
template <int PROB, class T, int MAXD, bool DEFER = false>
__global__ __launch_bounds__(64, MAXD == 2 ? PD_DD2_WAVES : 1) void dd_point_kernel(KernelArgs a) {
    constexpr int K = (PROB == PDEVAL_PROBLEM_FORCE_FREE) ? 4 : 2;
    constexpr int NC = nc(K);
    int64_t nwork = (int64_t)(*a.list_count);
    if (nwork > a.list_capacity) nwork = a.list_capacity;
#ifndef PD_HOST_SIM
    extern __shared__ __align__(16) unsigned char pd_lds[];
#else
    static unsigned char pd_lds[1];
#endif
    using STK = typename std::conditional<MAXD == 2, LdsVStack<T, NC>, PrivVStack<T, NC, MAXD - 1>>::type;
    STK stk;
    if constexpr (MAXD == 2) stk = STK{reinterpret_cast<T*>(pd_lds), (int)(threadIdx.x & 63)};
    for (int64_t wi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; wi < nwork;
         wi += (int64_t)gridDim.x * blockDim.x) {
        const int64_t cand = checked_cand(a, a.list[wi], ERRW_DD);
        if (cand < 0) continue;
        int64_t beg, end;
        uint8_t s = P0_NONE;
        double* res_out = a.out.res_ref ? a.out.res_ref + cand * a.n_ref : nullptr;
        double* q_out = a.out.q_ref ? a.out.q_ref + cand : nullptr;
        if (DEFER && dd_spec_entry(a, cand)) {
            // a speculative provisional pass: its outputs to the side arrays, sentinel first
            res_out = a.dd_res + cand * a.n_ref;
            q_out = a.dd_q + cand;
            for (int p = 0; p < a.n_ref; ++p) res_out[p] = __longlong_as_double(kDdUnset);
            *q_out = __longlong_as_double(kDdUnset);
        }
        if (prog_bounds(a, cand, &beg, &end)) {
            const int32_t* prog = a.ops + beg;
            const uint32_t hdr = (uint32_t)prog[0];
            // (the collect pass routes by depth)
            if ((int)((hdr >> 8) & 0xffu) <= MAXD)
                s = dd_point_stage<PROB, T, MAXD>(a, cand, prog, (int)(end - beg), hdr, stk, res_out, q_out);
        }
        if constexpr (DEFER) {
            a.ddps[cand] = s == P0_NONE ? kDdKeep : s;
        } else {
            if (s == P0_NONE) continue;   // not finite: keep the fp64 decision
            dd_apply_one(a, cand, s);
        }
    }
}

// The early tier's classes, applied once the grid classes are final: the entries of the three
// early lists (a.defer_list: real, a.cplx_list: complex, a.esc_list: real stack 3..8).
template <int PROB>
__global__ __launch_bounds__(256) void dd_apply_kernel(KernelArgs a) {
    auto count = [&](const int32_t* c) { const int64_t v = *c; return v < a.list_capacity ? v : a.list_capacity; };
    const int64_t n0 = count(a.defer_count);
    const int64_t n1 = a.cplx_list ? count(a.cplx_count) : 0;
    const int64_t n2 = count(a.esc_count);
    for (int64_t wi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; wi < n0 + n1 + n2;
         wi += (int64_t)gridDim.x * blockDim.x) {
        const int64_t cand = checked_cand(
            a, wi < n0 ? a.defer_list[wi] : (wi < n0 + n1 ? a.cplx_list[wi - n0] : a.esc_list[wi - n0 - n1]), ERRW_DD_APPLY);
        if (cand < 0) continue;
        const uint8_t s = a.ddps[cand];
        if (dd_spec_entry(a, cand)) {
            // the late tier's rule: only where the final class may be overridden does the
            // double-double value count (its outputs, then its class)
            const uint8_t st = a.out.status ? a.out.status[cand] : (uint8_t)PDEVAL_CLS_ACCEPT;
            if (!(st == PDEVAL_CLS_ACCEPT || st == PDEVAL_CLS_REJECT_GRID || st == PDEVAL_CLS_REJECT_SYMBOLIC)) continue;
            if (a.out.res_ref)
                for (int p = 0; p < a.n_ref; ++p) {
                    const double v = a.dd_res[cand * a.n_ref + p];
                    if (__double_as_longlong(v) != kDdUnset) a.out.res_ref[cand * a.n_ref + p] = v;
                }
            if (a.out.q_ref && __double_as_longlong(a.dd_q[cand]) != kDdUnset) a.out.q_ref[cand] = a.dd_q[cand];
        }
        if (s != kDdKeep) dd_apply_one(a, cand, s);
    }
}

// Diagnostic (pdeval_point_eval): one program at every reference point in one precision
// tier, one lane per point; out[6 k ..] = {res_re, res_im, |res|, S, noise, finite (1/0, -1 =
// program error)}; states[0] = the point-stage decision of the tier (P0_* of point_stage).
template <int PROB, class T, class V, bool FINAL>
__global__ __launch_bounds__(64, 1) void point_eval_kernel(KernelArgs a, const int32_t* prog, int plen,
                                                           double* out, uint8_t* states) {
    constexpr int K = (PROB == PDEVAL_PROBLEM_FORCE_FREE) ? 4 : 2;
    PrivStack<T, nc(K), PDEVAL_MAX_STACK - 1> stk;
    const int k = threadIdx.x;
    if (k < a.n_ref) {
        const PtEval r = point_eval<PROB, T, V, PDEVAL_MAX_STACK, true>(a, prog, plen, k, stk);
        double* o = out + 6 * k;
        o[0] = r.res_re; o[1] = r.res_im; o[2] = r.res_abs; o[3] = r.S; o[4] = r.noise;
        o[5] = r.rc ? -1.0 : (r.finite ? 1.0 : 0.0);
    }
    if (k == 0) {
        bool nf, perr;
        states[0] = point_stage<PROB, T, V, PDEVAL_MAX_STACK, true, FINAL>(a, 0, prog, plen, (uint32_t)prog[0], stk,
                                                                         &nf, &perr);
    }
}

}  // namespace pd
