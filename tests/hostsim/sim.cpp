// tests/hostsim/sim.cpp -- the device interpreter (pdeval_kernels.h, pdeval_tier2.h) built
// for the CPU, one lane: value jets and tier-2 error jets of one program at one point.
// Test infrastructure only (tests/test_hostsim.py); the product is built by hipcc for gfx950.
#include <cstdio>
#include <vector>
#include "../../include/pdeval.h"
#include "../../pde-engine_amd/csrc/pdeval_point.h"
using namespace pd;

static double g_om2 = 0.0;   // force-free Omega^2 (pdeval_params.omega2)
extern "C" void sim_set_omega2(double w) { g_om2 = w; }

extern "C" int sim_point(int problem, const int32_t* w, int nw, double x, double y, int tier2,
                         double* jet, double* err, double* res) {
    constexpr int MAXD = PDEVAL_MAX_STACK;
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        using I = Interp<double, 4, MAXD>;
        using E = ErrInterp<double, 4, MAXD>;
        std::vector<double> stk((MAXD - 1) * 15 * 64), es((MAXD - 1) * 15 * 64);
        I::J u;
        double e[15] = {0};
        const PrmTab<double> P{};   // (force-free: no constants of the problem)
        int rc = tier2 ? E::run(w, 1, nw, x, y, u, e, stk.data(), es.data(), 0, P)
                       : I::run(w, 1, nw, x, y, u, stk.data(), 0, P);
        if (rc) return rc;
        for (int i = 0; i < 15; ++i) { jet[i] = u.c[i]; err[i] = e[i]; }
        PointResult r = ff_epilogue<double>(u.c, x, g_om2);
        res[0] = r.res_abs;
        res[1] = r.scale;
        res[2] = tier2 ? residual_noise<PDEVAL_PROBLEM_FORCE_FREE, double>(u.c, e, x, nullptr, r.scale, g_om2) : 0.0;
        res[3] = r.finite;
        return 0;
    }
    return -1;
}

// The point stage's evaluation (pdeval_point.h point_eval) at reference point k, in one of its
// precisions: tier 0 fp64 real, 1 fp64 complex, 2 double-double, 3 complex double-double.
// out = {res_re, res_im, res_abs, S, noise, finite}.
namespace {
void kerr_dd(dd r, dd x, dd* k) {
    const dd M = dd_from(1.0), a = dd_ratio(1.0, 10.0);
    const dd a2x2 = a * a * x * x, s = r * r + a2x2, s2 = s * s;
    const dd G = dd_from(1.0) - dd_div(M * r * 2.0, s);
    const dd Gr = dd_div(M * (r * r - a2x2) * 2.0, s2);
    const dd Gx = dd_div(M * a * a * r * x * 4.0, s2);
    const dd D = r * r - M * r * 2.0 + a * a, w = dd_from(1.0) - x * x;
    k[0] = dd_div(G, w); k[1] = dd_div(G, D); k[2] = dd_div(Gr, w); k[3] = dd_div(Gx, D);
}
template <int PROB, class T, class V>
int run_tier(const KernelArgs& a, const int32_t* w, int nw, int k, double* out) {
    constexpr int K = PROB == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
    PrivStack<T, nc(K), PDEVAL_MAX_STACK - 1> stk;
    const PtEval r = point_eval<PROB, T, V, PDEVAL_MAX_STACK, true>(a, w, nw, k, stk);
    if (r.rc) return r.rc;
    out[0] = r.res_re; out[1] = r.res_im; out[2] = r.res_abs; out[3] = r.S; out[4] = r.noise;
    out[5] = r.finite;
    return 0;
}
}  // namespace

extern "C" int sim_point_tier(int problem, const int32_t* w, int nw, int k, int tier, double* out) {
    KernelArgs a{};
    static double kc[12];
    const double fx[2][3] = {{4, 5, 0}, {6, 7, 0}};
    const double kx[3][2] = {{5, 2}, {7, 3}, {5, 1}}, ky[3][2] = {{3, 5}, {1, 3}, {-2, 5}};
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        a.n_ref = 1;
        a.ref_xd[0] = dd_ratio(fx[0][0], fx[0][1]);
        a.ref_yd[0] = dd_ratio(fx[1][0], fx[1][1]);
    } else {
        a.n_ref = 3;
        for (int i = 0; i < 3; ++i) {
            a.ref_xd[i] = dd_ratio(kx[i][0], kx[i][1]);
            a.ref_yd[i] = dd_ratio(ky[i][0], ky[i][1]);
            kerr_dd(a.ref_xd[i], a.ref_yd[i], &a.kc_ref[4 * i]);
            for (int j = 0; j < 4; ++j) kc[4 * i + j] = a.kc_ref[4 * i + j].hi;
        }
        a.kc = kc;
        // the point stage's constants: M_value = 1, a_value = 1/10 (PDEVAL_IMM_PRM)
        a.prm_pt = PrmTab<double>{{1.0, 0.1, 1.0, 10.0, 1.0, 0.01, 1.0, 100.0}};
        a.prm_pt_dd = PrmTab<dd>{{dd_from(1.0), dd_ratio(1.0, 10.0), dd_from(1.0), dd_from(10.0), dd_from(1.0),
                                  dd_ratio(1.0, 100.0), dd_from(1.0), dd_from(100.0)}};
    }
    for (int i = 0; i < a.n_ref; ++i) {
        a.ref_x[i] = a.ref_xd[i].hi;
        a.ref_y[i] = a.ref_yd[i].hi;
    }
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        if (tier == 0) return run_tier<PDEVAL_PROBLEM_FORCE_FREE, double, double>(a, w, nw, k, out);
        if (tier == 1) return run_tier<PDEVAL_PROBLEM_FORCE_FREE, cplx, double>(a, w, nw, k, out);
        if (tier == 2) return run_tier<PDEVAL_PROBLEM_FORCE_FREE, dd, dd>(a, w, nw, k, out);
        return run_tier<PDEVAL_PROBLEM_FORCE_FREE, cdd, dd>(a, w, nw, k, out);
    }
    if (tier == 0) return run_tier<PDEVAL_PROBLEM_KERR, double, double>(a, w, nw, k, out);
    if (tier == 2) return run_tier<PDEVAL_PROBLEM_KERR, dd, dd>(a, w, nw, k, out);
    return -1;
}

// kerr_epilogue (every tier) and kerr_epilogue_lean (the lean grid passes, doubled table) on
// one jet u[6] and coefficients k[4]: out = {res_abs, scale, res_re, finite, grad_zero} of each
extern "C" void sim_kerr_epi_pair(const double* u, const double* k, double* out) {
    const double k2[4] = {2.0 * k[0], 2.0 * k[1], k[2], k[3]};
    const PointResult a = kerr_epilogue<double>(u, k);
    const PointResult b = kerr_epilogue_lean<double>(u, k2);
    const PointResult* r[2] = {&a, &b};
    for (int i = 0; i < 2; ++i) {
        out[5 * i + 0] = r[i]->res_abs;
        out[5 * i + 1] = r[i]->scale;
        out[5 * i + 2] = r[i]->res_re;
        out[5 * i + 3] = r[i]->finite ? 1.0 : 0.0;
        out[5 * i + 4] = r[i]->grad_zero ? 1.0 : 0.0;
    }
}
