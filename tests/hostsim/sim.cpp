// tests/hostsim/sim.cpp -- the device interpreter (pdeval_kernels.h, pdeval_tier2.h) built
// for the CPU, one lane: value jets and tier-2 error jets of one program at one point.
// Test infrastructure only (tests/test_hostsim.py); the product is built by hipcc for gfx950.
#include <cstdio>
#include <vector>
#include "../../include/pdeval.h"
#include "../../pde-engine_amd/csrc/pdeval_tier2.h"
using namespace pd;

extern "C" int sim_point(int problem, const int32_t* w, int nw, double x, double y, int tier2,
                         double* jet, double* err, double* res) {
    constexpr int MAXD = PDEVAL_MAX_STACK;
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        using I = Interp<double, 4, MAXD>;
        using E = ErrInterp<double, 4, MAXD>;
        std::vector<double> stk((MAXD - 1) * 15 * 64), es((MAXD - 1) * 15 * 64);
        I::J u;
        double e[15] = {0};
        int rc = tier2 ? E::run(w, 1, nw, x, y, u, e, stk.data(), es.data(), 0)
                       : I::run(w, 1, nw, x, y, u, stk.data(), 0);
        if (rc) return rc;
        for (int i = 0; i < 15; ++i) { jet[i] = u.c[i]; err[i] = e[i]; }
        PointResult r = ff_epilogue<double>(u.c, x);
        res[0] = r.res_abs;
        res[1] = r.scale;
        res[2] = tier2 ? residual_noise<PDEVAL_PROBLEM_FORCE_FREE, double>(u.c, e, x, nullptr, r.scale) : 0.0;
        res[3] = r.finite;
        return 0;
    }
    return -1;
}
