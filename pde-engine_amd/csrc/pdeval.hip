// pdeval.hip -- libpdeval.so: the C ABI (include/pdeval.h) around the gfx950 kernels.
//
// Host side of the boundary: contexts (one per GPU), the sample-point tables of each problem
// (reference points first, then the nx*ny grid), device work lists for the two follow-up
// passes (deep-stack programs, complex-valued candidates) and the launch sequence.  All device
// allocation happens at create time or when a batch outgrows the scratch lists, never inside
// an already-sized hot call, so pdeval_validate_device can be captured in a hipGraph.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/pdeval.h"
#include "pdeval_kernels.h"
#include "pdeval_point.h"
#include "pdeval_tier2.h"
#include "pdeval_launch.h"

using namespace pd;

#define PD_VERSION "pdeval 0.2 gfx950"

// Work lists between the passes of one call (pdeval_pass_counts reports their sizes).
enum {
    L_DEFER = 0,      // pass 1 -> pass 2: real, stack 3
    L_CPLX = 1,       // pass 1 -> complex passes: not real at the reference point
    L_DEFER2 = 2,     // pass 2 -> pass 3: real, stack 4..8
    L_ESC = 3,        // tier-1 failures of the real passes -> tier 2
    L_ESC_DEEP = 4,   // tier 2 stack 2 -> tier 2 stack 3
    L_ESC_C = 5,      // tier-1 failures of the complex passes -> complex tier 2
    L_CPLX_DEEP = 6,  // complex stack 2 -> complex stack 8
    L_ESC_DEEP2 = 7,  // tier 2 stack 3 -> tier 2 stack 8
    L_PDEEP = 8,      // pass 0 -> deep point pass: real programs of stack 3..8
    L_DD = 9,         // double-double point tier, real
    L_DDC = 10,       // double-double point tier, complex
    L_DD8 = 11,       // double-double point tier, real, stack 3..8
    L_ESC_C_DEEP = 12,  // complex tier 2, stack 5..8
    L_SLOW = 13,      // lean grid pass -> the generic stack-2 kernel (malformed / undecided)
    L_SLOW2 = 14,     // lean stack-3 pass -> the generic stack-3 kernel
    L_SLOW_C = 15,    // lean complex pass -> the generic complex stack-2 kernel
    L_DDL = 16,       // the late double-double lists (provisional point passes, after the
    L_DDLC = 17,      // grid): real, complex, real stack 3..8; L_DD / L_DDC / L_DD8 are the
    L_DDL8 = 18,      // early ones (P0_DD, beside the grid passes on the side stream)
    PD_N_LISTS = 19
};
// after the list counters in d_counts: the device error word (KernelArgs::errw), then the work
// queue heads of the persistent list kernels (KernelArgs::qhead), one per launch, zeroed with
// the counters at the start of every launch chain
enum { Q_PASS2 = 0, Q_CPLX, Q_T2, Q_T2_3, Q_T2_8, Q_T2_C, Q_T2_C8, Q_N };
// The list passes' schedule (context fields, env at pdeval_create): list_queue 0 static (item
// blockIdx.x, then + gridDim.x), or chunks of list_queue items from a work-queue head
// (KernelArgs::qhead); list_parts waves per candidate at full size.  Measured
// (profiles/r05_g_ab_*, 2^21): one item per atomic made Kerr pass 2 36 ms against 22 ms static
// -- one counter for ~320 k items serializes -- and 4 parts per candidate 65 ms (every part
// pays the accumulator's atomics and device-scope fences)
#ifndef PD_LIST_QUEUE
#define PD_LIST_QUEUE 0
#endif
#ifndef PD_LIST_PARTS
#define PD_LIST_PARTS 1
#endif
constexpr int PD_COUNT_WORDS = PD_N_LISTS + 1 + Q_N;

namespace {
struct Grid {
    double x_lo, x_hi, nx, y_lo, y_hi, ny, x_ph, y_ph;
};
}  // namespace

struct pdeval_ctx {
    int device = 0;
    int problem = 0;
    int n_ref = 0, n_pts = 0;
    int fp_pts[PDEVAL_FP_N] = {0, 0, 0, 0};
    hipStream_t stream = nullptr;
    // the early double-double tier runs on `side`, forked after the point stage and joined
    // before the classes are final (env PDEVAL_DD_EARLY=0: one tier after the grid, A/B)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    bool dd_early = true;
    int list_queue = PD_LIST_QUEUE;   // list passes: 0 static schedule, k > 0 queue chunks of k items
    int list_parts = PD_LIST_PARTS;   // list passes: waves per candidate at full size
    uint8_t* d_ddps = nullptr;      // the early tier's classes, capacity cap
    double* d_dd_res = nullptr;     // speculative provisional passes' outputs (cap * 4, cap)
    double* d_dd_q = nullptr;
    bool dd_spec = true;            // env PDEVAL_DD_SPEC=0: provisional passes after the grid (A/B)
    double ref_x[4] = {0, 0, 0, 0}, ref_y[4] = {0, 0, 0, 0};
    dd ref_xd[4] = {}, ref_yd[4] = {};   // the reference points as double-doubles
    dd kc_ref[16] = {};                  // Kerr operator coefficients there, double-double
    int nx = 0, ny = 0;
    double* d_gx = nullptr;   // nx grid abscissae
    double* d_gy = nullptr;   // ny grid ordinates
    double* d_kc = nullptr;
    double* d_ptab = nullptr;            // coordinate-power tables of the lean passes
    Grid grid{};                         // as given, or the problem's default (grid_default)
    bool grid_default = true;
    // the problem's constants (Kerr M, a; pdeval_kerr_constants) and their per-stage tables
    pdeval_kerr_constants kconst{};
    PrmTab<double> prm_pt{}, prm_grid{};
    PrmTab<dd> prm_pt_dd{}, prm_grid_dd{};
    double ct_x[8] = {}, ct_y[8] = {};   // Kerr constant-test points
    int n_ct = 0;
    // scratch: work lists and their counters
    int64_t cap = 0;
    // device work lists (capacity cap each) and their counters d_counts[L_*]
    int64_t* d_list[PD_N_LISTS] = {};
    int32_t* d_counts = nullptr;
    uint8_t* d_pstate = nullptr;    // point-stage state, capacity cap
    int32_t* d_dec = nullptr;       // decoded programs of the lean grid passes, dec_cap words
    int64_t dec_cap = 0;
    // the hoisted prefixes / segments of the lean passes (pdeval_grid.h PD_HOIST): 8 x
    // kHoistPool slots of hoist_stride doubles and their owner words, whatever the batch size
    // (env PDEVAL_HOIST=0: none, A/B)
    bool hoist = true;
    bool hoist_sub = true;              // env PDEVAL_HOIST_SUB=0: no hoisted segments (A/B)
    double* d_hoist = nullptr;
    uint32_t* d_hoist_own = nullptr;
    bool hoist_slots = true;            // env PDEVAL_HOIST_SLOTS=0: one slot per candidate (A/B)
    int32_t* d_hseg = nullptr;          // the decoder's hoisted segments, cap x 4 words
    // the lean passes' failing lanes per candidate and grid chunk, cap x chunks words, which
    // tier 2 re-checks instead of the whole grid (env PDEVAL_TIER2_MASK=0: none, A/B)
    bool tier2_mask = true;
    uint64_t* d_fsum = nullptr;         // ... and per candidate the chunks whose word was stored
    int deep_parts = PD_DEEP_PARTS;     // the stack-8 lists' waves per candidate (env PDEVAL_DEEP_PARTS)
    uint64_t* d_fmask = nullptr;
    uint8_t* d_status = nullptr;    // classes when the caller asks for no status output
    double* d_noise = nullptr;      // fp64 noise bounds at the reference points, cap * 4
    T2Acc* d_t2acc = nullptr;       // tier-2 accumulators, cap entries, zero between launches
    // shape sort of the batch (pdeval_sort.hip): keys 2 x cap, permutation 2 x cap, scratch
    bool sort = true;               // env PDEVAL_SORT=0 turns it off (measurements)
    bool lean_cplx = true;          // env PDEVAL_LEAN_CPLX=0: the generic complex pass (A/B)
    uint64_t* d_skeys = nullptr;
    int32_t* d_sidx = nullptr;
    void* d_stemp = nullptr;
    size_t stemp_bytes = 0;
    // host-path staging
    int64_t hcap_words = 0, hcap_n = 0;
    int32_t* d_ops = nullptr;
    int64_t* d_off = nullptr;
    uint8_t* d_outbuf = nullptr;
    int64_t outbuf_bytes = 0;
    std::string err;
    // small host batches (validate_small): the launch chain captured once per (n, params) as
    // a HIP graph, inputs and outputs through pinned staging; graphs are dropped whenever a
    // buffer they reference is reallocated (buf_epoch)
    bool use_graph = true;          // env PDEVAL_GRAPH=0 turns it off
    uint64_t buf_epoch = 0;
    void* h_errw = nullptr;        // pinned word: the device error word after a direct-path call
    struct GraphEntry {
        hipGraphExec_t exec = nullptr;
        uint64_t epoch = 0;
    };
    std::map<uint64_t, GraphEntry> graphs;
    uint8_t* h_stage = nullptr;     // pinned: ops + offsets in, the output block out
    size_t h_stage_bytes = 0;
    // optional per-pass timing (pdeval_set_timing): an event before every pass and one after
    // the last, recorded on the launch stream
    bool timing = false;
    hipEvent_t ev[PDEVAL_N_PASSES + 1] = {};
    int ev_recorded = 0;
    // the multi-GPU exchange (pdeval_comm_init)
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0;
};

// RCCL, loaded on first use (dlopen: a process that already holds librccl.so.1, e.g. through
// torch.distributed, shares that instance)
namespace {
struct Rccl {
    bool tried = false;
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};
Rccl& rccl() {
    static Rccl r;
    if (!r.tried) {
        r.tried = true;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (r.h) break;
        }
        if (r.h) {
            r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
            r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.h, "ncclCommInitRank");
            r.all_gather = (decltype(r.all_gather))dlsym(r.h, "ncclAllGather");
            r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
            r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
            if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy || !r.error_string)
                r.h = nullptr;
        }
    }
    return r;
}
}  // namespace

// in launch order (pass k lasts from event k to event k + 1)
static const char* const kPassNames[PDEVAL_N_PASSES] = {
    "pass0_point", "point_deep_complex", "pass1_stack2", "pass2_stack3", "pass3_stack8",
    "complex_stack2", "complex_stack8", "tier2_stack2", "tier2_stack3", "tier2_stack8",
    "tier2_complex", "point_dd"};

static thread_local std::string g_err;

#define HIPCHK(ctx, expr)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
            return PDEVAL_ERR_HIP;                                                          \
        }                                                                                   \
    } while (0)

// ---------------------------------------------------------------------------- point tables
namespace {

// DESIGN.md "Grids": cell-offset grids that avoid the coordinate singular sets exactly.  Kerr:
// r from r+ + 0.1 to r+ + 6.1, r+ = M + sqrt(M^2 - a^2) of the grid stage's operator.
Grid default_grid(int problem, double M = 1.0, double a = 0.1) {
    if (problem == PDEVAL_PROBLEM_FORCE_FREE)
        return {0.05, 3.0, 64, -2.0, 2.0, 64, 0.37, 0.41};
    const double r_plus = M + std::sqrt(M * M - a * a);
    return {r_plus + 0.1, r_plus + 6.1, 64, -0.98, 0.98, 64, 0.37, 0.41};
}

// Kerr operator coefficients (kerr validator.py:69-91):
// L[u] = G/(1-x^2) u_rr + G/Delta u_xx + d_r(G)/(1-x^2) u_r + d_x(G)/Delta u_x
// in double-double at an exact rational point (the point stage's second tier)
void kerr_coeffs_dd(dd r, dd x, dd M, dd a, dd* k) {
    const dd a2x2 = a * a * x * x;
    const dd s = r * r + a2x2;
    const dd s2 = s * s;
    const dd G = dd_from(1.0) - dd_div(M * r * 2.0, s);
    const dd Gr = dd_div(M * (r * r - a2x2) * 2.0, s2);
    const dd Gx = dd_div(M * a * a * r * x * 4.0, s2);
    const dd D = r * r - M * r * 2.0 + a * a;
    const dd w = dd_from(1.0) - x * x;
    k[0] = dd_div(G, w);
    k[1] = dd_div(G, D);
    k[2] = dd_div(Gr, w);
    k[3] = dd_div(Gx, D);
}

void kerr_coeffs(double r_, double x_, long double M, long double a, double* k) {
    const long double r = r_, x = x_;
    const long double s = r * r + a * a * x * x;
    const long double G = 1.0L - 2.0L * M * r / s;
    const long double Gr = 2.0L * M * (r * r - a * a * x * x) / (s * s);
    const long double Gx = 4.0L * M * a * a * r * x / (s * s);
    const long double D = r * r - 2.0L * M * r + a * a;
    const long double w = 1.0L - x * x;
    k[0] = (double)(G / w);
    k[1] = (double)(G / D);
    k[2] = (double)(Gr / w);
    k[3] = (double)(Gx / D);
}

}  // namespace

// The stage tables of the problem's constants and every point table that depends on them: the
// grid (the default Kerr grid follows r+ of the grid stage's operator), its reciprocal
// abscissae, and (Kerr) the operator coefficients -- at the reference points with the point
// stage's operator (fp64 table and double-double), on the grid with the grid stage's.
static int build_points(pdeval_ctx* c) {
    const bool kerr = c->problem == PDEVAL_PROBLEM_KERR;
    long double opM_pt = 1.0L, opa_pt = 0.0L, opM_g = 1.0L, opa_g = 0.0L;
    dd opM_pt_dd = dd_from(1.0), opa_pt_dd = dd_from(0.0);
    if (kerr) {
        const pdeval_kerr_constants& k = c->kconst;
        const dd Mv = dd_ratio((double)k.M_num, (double)k.M_den), av = dd_ratio((double)k.a_num, (double)k.a_den);
        const double Mvd = (double)k.M_num / (double)k.M_den, avd = (double)k.a_num / (double)k.a_den;
        const long double Mvl = (long double)k.M_num / (long double)k.M_den;
        const long double avl = (long double)k.a_num / (long double)k.a_den;
        // the operator: the point stage at (M_value, a_value); the grid stage at the stand-ins,
        // except for a constant the validator was built with as a number
        opM_pt = Mvl;
        opa_pt = avl;
        opM_pt_dd = Mv;
        opa_pt_dd = av;
        opM_g = k.op_M_fixed ? Mvl : (long double)k.M_sym;
        opa_g = k.op_a_fixed ? avl : (long double)k.a_sym;
        // u's own M and a: the stage's values; a free symbol (op_*_fixed) is the stand-in
        const double uM = k.op_M_fixed ? k.M_sym : Mvd, ua = k.op_a_fixed ? k.a_sym : avd;
        const dd uMd = k.op_M_fixed ? dd_from(k.M_sym) : Mv, uad = k.op_a_fixed ? dd_from(k.a_sym) : av;
        (void)uM;
        (void)ua;
        // {M, a, 1/M, 1/a, M^2, a^2, 1/M^2, 1/a^2} in double-double; the fp64 table is the
        // rounded high parts
        auto table = [](dd M, dd a, PrmTab<dd>& t, PrmTab<double>& d) {
            const dd M2 = M * M, a2 = a * a;
            t = PrmTab<dd>{{M, a, recip(M), recip(a), M2, a2, recip(M2), recip(a2)}};
            for (int i = 0; i < 8; ++i) d.v[i] = t.v[i].hi + t.v[i].lo;
        };
        table(uMd, uad, c->prm_pt_dd, c->prm_pt);
        table(dd_from(k.M_sym), dd_from(k.a_sym), c->prm_grid_dd, c->prm_grid);
        // the constant test: the reference points and two more (pdeval_point.h)
        c->n_ct = 0;
        for (int p = 0; p < c->n_ref; ++p) {
            c->ct_x[c->n_ct] = c->ref_x[p];
            c->ct_y[c->n_ct++] = c->ref_y[p];
        }
        c->ct_x[c->n_ct] = 3.3;
        c->ct_y[c->n_ct++] = 0.27;
        c->ct_x[c->n_ct] = 6.1;
        c->ct_y[c->n_ct++] = -0.55;
        if (c->grid_default) c->grid = default_grid(c->problem, (double)opM_g, (double)opa_g);
    }
    const Grid& g = c->grid;
    const int nx = c->nx, ny = c->ny;
    std::vector<double> gx(nx), gy(ny);
    for (int i = 0; i < nx; ++i) gx[i] = g.x_lo + (i + g.x_ph) * ((g.x_hi - g.x_lo) / nx);
    for (int j = 0; j < ny; ++j) gy[j] = g.y_lo + (j + g.y_ph) * ((g.y_hi - g.y_lo) / ny);
    std::vector<double> kc;
    if (kerr) {
        kc.resize(4 * (size_t)c->n_pts);
        for (int p = 0; p < c->n_ref; ++p) {
            kerr_coeffs(c->ref_x[p], c->ref_y[p], opM_pt, opa_pt, &kc[4 * p]);
            kerr_coeffs_dd(c->ref_xd[p], c->ref_yd[p], opM_pt_dd, opa_pt_dd, &c->kc_ref[4 * p]);
        }
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < ny; ++j)
                kerr_coeffs(gx[i], gy[j], opM_g, opa_g, &kc[4 * (c->n_ref + (size_t)i * ny + j)]);
    }
    // d_gx holds the abscissae and then their reciprocals 1.0 / gx (correctly rounded, the
    // value rcp() forms on the device): the grid pass reads 1/x with a scalar load
    for (int i = 0; i < nx; ++i) gx.push_back(1.0 / gx[i]);
    HIPCHK(c, hipMemcpy(c->d_gx, gx.data(), 2 * nx * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_gy, gy.data(), ny * sizeof(double), hipMemcpyHostToDevice));
    if (kerr) {
        // then the same table with k1, k2 doubled (2 k is exact): the lean grid passes' copy,
        // whose epilogue then forms 2 k u_rr, 2 k u_xx without the two multiplies per point
        const size_t n4 = kc.size();
        kc.resize(2 * n4);
        for (size_t p = 0; p < n4; p += 4) {
            kc[n4 + p] = 2.0 * kc[p];
            kc[n4 + p + 1] = 2.0 * kc[p + 1];
            kc[n4 + p + 2] = kc[p + 2];
            kc[n4 + p + 3] = kc[p + 3];
        }
        HIPCHK(c, hipMemcpy(c->d_kc, kc.data(), kc.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    // the lean passes' coordinate-power tables, from the grid just uploaded (same JetOps::pcoefs)
    if (!c->d_ptab) HIPCHK(c, hipMalloc(&c->d_ptab, ptab_bytes(c->problem, nx, ny)));
    launch_ptab(c->problem, c->d_gx, c->d_gy, nx, ny, c->d_ptab, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // captured small-batch graphs hold the old constants by value (kc_ref, prm_pt / prm_grid,
    // ct_x / ct_y in their kernel arguments): drop them, as after a buffer reallocation
    ++c->buf_epoch;
    return PDEVAL_OK;
}

extern "C" int pdeval_default_kerr_constants(pdeval_kerr_constants* k) {
    if (!k) return PDEVAL_ERR_ARG;
    // problems/__init__.py:283: M_value = 1, a_value = 1/10.  Stand-ins of the symbols: dyadic
    // (exact doubles), away from the small-integer ratios the op vocabulary builds
    // (expression_operations.py), a < M
    *k = pdeval_kerr_constants{1, 1, 1, 10, 1.171875, 0.359375, 0, 0};
    return PDEVAL_OK;
}

extern "C" int pdeval_set_kerr_constants(pdeval_ctx* c, const pdeval_kerr_constants* k) {
    if (!c || !k || c->problem != PDEVAL_PROBLEM_KERR || k->M_den <= 0 || k->a_den <= 0 || k->M_num <= 0 ||
        !(k->M_sym > 0.0) || !(std::fabs(k->a_sym) < k->M_sym) || std::fabs((double)k->M_num) >= 0x1p53 ||
        std::fabs((double)k->a_num) >= 0x1p53 || (double)k->M_den >= 0x1p53 || (double)k->a_den >= 0x1p53 ||
        std::fabs((double)k->a_num / (double)k->a_den) >= (double)k->M_num / (double)k->M_den) {
        if (c) c->err = "pdeval_set_kerr_constants: bad argument (Kerr context; M > 0, |a| < M, dens > 0)";
        return PDEVAL_ERR_ARG;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->kconst = *k;
    return build_points(c);
}

extern "C" int pdeval_create(int device_id, int problem_id, const double* grid, int n_grid,
                             pdeval_ctx** out) {
    if (!out || (problem_id != PDEVAL_PROBLEM_FORCE_FREE && problem_id != PDEVAL_PROBLEM_KERR)) {
        g_err = "pdeval_create: bad argument";
        return PDEVAL_ERR_ARG;
    }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        g_err = "pdeval_create: no HIP device";
        return PDEVAL_ERR_NODEVICE;
    }
    if (device_id < 0 || device_id >= ndev) {
        g_err = "pdeval_create: device id out of range";
        return PDEVAL_ERR_ARG;
    }
    pdeval_ctx* c = new pdeval_ctx();
    c->device = device_id;
    c->problem = problem_id;
    c->grid = default_grid(problem_id);
    c->grid_default = !(grid && n_grid >= 8);
    if (!c->grid_default) std::memcpy(&c->grid, grid, sizeof(Grid));
    const int nx = (int)c->grid.nx, ny = (int)c->grid.ny;
    if (nx <= 0 || ny <= 0 || ny % 64 != 0 || nx * ny > (1 << 22)) {
        delete c;
        g_err = "pdeval_create: bad grid";
        return PDEVAL_ERR_ARG;
    }
    // the reference points as exact ratios (numerator, denominator)
    std::vector<std::pair<double, double>> rx, ry;
    if (problem_id == PDEVAL_PROBLEM_FORCE_FREE) {
        // the paper's test point (rho, z) = (4/5, 6/7), validator.py:296-297
        rx = {{4, 5}};
        ry = {{6, 7}};
    } else {
        // kerr validator.py:167-171
        rx = {{5, 2}, {7, 3}, {5, 1}};
        ry = {{3, 5}, {1, 3}, {-2, 5}};
    }
    c->n_ref = (int)rx.size();
    for (int k = 0; k < c->n_ref; ++k) {
        c->ref_xd[k] = dd_ratio(rx[k].first, rx[k].second);
        c->ref_yd[k] = dd_ratio(ry[k].first, ry[k].second);
        c->ref_x[k] = rx[k].first / rx[k].second;
        c->ref_y[k] = ry[k].first / ry[k].second;
    }
    c->nx = nx;
    c->ny = ny;
    c->n_pts = c->n_ref + nx * ny;
    const int G = nx * ny;
    c->fp_pts[0] = 0;
    for (int f = 1; f < PDEVAL_FP_N; ++f) c->fp_pts[f] = c->n_ref + (int)((int64_t)G * f / PDEVAL_FP_N) + 7 % G;
    auto fail = [&](const char* what, hipError_t e) {
        g_err = std::string(what) + ": " + hipGetErrorString(e);
        pdeval_destroy(c);
        return PDEVAL_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(device_id)) != hipSuccess) return fail("hipSetDevice", e);
    if (const char* v = getenv("PDEVAL_SORT")) c->sort = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_LEAN_CPLX")) c->lean_cplx = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_GRAPH")) c->use_graph = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_DD_EARLY")) c->dd_early = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_DD_SPEC")) c->dd_spec = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_LIST_QUEUE")) c->list_queue = std::max(0, atoi(v));
    if (const char* v = getenv("PDEVAL_LIST_PARTS")) c->list_parts = std::min(16, std::max(1, atoi(v)));
    if (const char* v = getenv("PDEVAL_HOIST")) c->hoist = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_HOIST_SUB")) c->hoist_sub = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_HOIST_SLOTS")) c->hoist_slots = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_TIER2_MASK")) c->tier2_mask = atoi(v) != 0;
    if (const char* v = getenv("PDEVAL_DEEP_PARTS")) c->deep_parts = atoi(v) > 1 ? PD_DEEP_PARTS : 1;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
        return fail("hipStreamCreate", e);
    if ((e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking)) != hipSuccess)
        return fail("hipStreamCreate", e);
    if ((e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming)) != hipSuccess)
        return fail("hipEventCreate", e);
    if ((e = hipMalloc(&c->d_gx, 2 * nx * sizeof(double))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc(&c->d_gy, ny * sizeof(double))) != hipSuccess) return fail("hipMalloc", e);
    if (problem_id == PDEVAL_PROBLEM_KERR &&
        (e = hipMalloc(&c->d_kc, 8 * (size_t)c->n_pts * sizeof(double))) != hipSuccess)
        return fail("hipMalloc", e);
    if (problem_id == PDEVAL_PROBLEM_KERR) pdeval_default_kerr_constants(&c->kconst);
    if (int rc = build_points(c)) {
        g_err = c->err;
        pdeval_destroy(c);
        return rc;
    }
    // the list counters and, after them, the device error word (KernelArgs::errw)
    if ((e = hipMalloc(&c->d_counts, PD_COUNT_WORDS * sizeof(int32_t))) != hipSuccess) return fail("hipMalloc", e);
    *out = c;
    return PDEVAL_OK;
}

extern "C" int pdeval_destroy(pdeval_ctx* c) {
    if (!c) return PDEVAL_ERR_ARG;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->side) (void)hipStreamSynchronize(c->side);
    if (c->comm) pdeval_comm_destroy(c);
    for (int64_t* l : c->d_list)
        if (l) (void)hipFree(l);
    if (c->d_pstate) (void)hipFree(c->d_pstate);
    if (c->d_ddps) (void)hipFree(c->d_ddps);
    if (c->d_dd_res) (void)hipFree(c->d_dd_res);
    if (c->d_dd_q) (void)hipFree(c->d_dd_q);
    if (c->d_dec) (void)hipFree(c->d_dec);
    if (c->d_hoist) (void)hipFree(c->d_hoist);
    if (c->d_hoist_own) (void)hipFree(c->d_hoist_own);
    if (c->d_hseg) (void)hipFree(c->d_hseg);
    if (c->d_fmask) (void)hipFree(c->d_fmask);
    if (c->d_fsum) (void)hipFree(c->d_fsum);
    if (c->d_status) (void)hipFree(c->d_status);
    if (c->d_noise) (void)hipFree(c->d_noise);
    if (c->d_t2acc) (void)hipFree(c->d_t2acc);
    if (c->d_skeys) (void)hipFree(c->d_skeys);
    if (c->d_sidx) (void)hipFree(c->d_sidx);
    if (c->d_stemp) (void)hipFree(c->d_stemp);
    for (void* p : {(void*)c->d_gx, (void*)c->d_gy, (void*)c->d_kc, (void*)c->d_ptab,
                    (void*)c->d_counts, (void*)c->d_ops, (void*)c->d_off, (void*)c->d_outbuf})
        if (p) (void)hipFree(p);
    for (auto& g : c->graphs)
        if (g.second.exec) (void)hipGraphExecDestroy(g.second.exec);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->h_errw) (void)hipHostFree(c->h_errw);
    for (hipEvent_t& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return PDEVAL_OK;
}

extern "C" const char* pdeval_last_error(pdeval_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }
extern "C" int pdeval_n_ref_points(pdeval_ctx* c) { return c ? c->n_ref : -1; }
extern "C" int pdeval_n_points(pdeval_ctx* c) { return c ? c->n_pts : -1; }
extern "C" const char* pdeval_version(void) { return PD_VERSION; }

extern "C" int pdeval_default_params(int problem_id, pdeval_params* p) {
    if (!p) return PDEVAL_ERR_ARG;
    // DESIGN.md "Zero test": thresholds calibrated on the reference fixtures
    p->tau_point = 1e-10;
    p->tau_grid = 1e-7;
    p->kerr_abs_tol = 1e-10;  // kerr validator.py:190
    p->full_grid = 1;
    p->max_bad = 0;
    p->strict_symbolic = 1;
    p->reserved = 0;
    p->noise_kappa = 16.0;  // true zeros <= 0.4, real residuals >= 1e8 x noise
    p->point_abs_tol = 1e-20;  // validator.py:389
    p->res_rel_acc = 1e-11;    // residuals reported to 1e-10 relative (BASELINE.json north star)
    p->omega2 = 0.0;           // force-free Omega = 0 (problems/__init__.py:83)
    p->omega2_lo = 0.0;
    (void)problem_id;
    return PDEVAL_OK;
}

// ---------------------------------------------------------------------------- program checks
static int op_has_imm(uint32_t op) {
    return op == PDOP_PUSH_C || op == PDOP_ADDC || op == PDOP_MULC || op == PDOP_RDIVC || op == PDOP_POW;
}
// words taken by an opcode and its immediate(s) (PDEVAL_IMM_DD: a double-double low part too)
static int op_words(int32_t w) {
    if (!op_has_imm((uint32_t)w & 0xffu)) return 1;
    return ((uint32_t)w & PDEVAL_IMM_DD) ? 5 : 3;
}
static int op_stack_delta(uint32_t op, int* need) {
    switch (op) {
        case PDOP_PUSH_X: case PDOP_PUSH_Y: case PDOP_PUSH_C: case PDOP_PUSH_I: case PDOP_PUSH_P:
        case PDOP_UNSUPPORTED:
            *need = 0; return 1;
        case PDOP_ADD: case PDOP_SUB: case PDOP_RSUB: case PDOP_MUL: case PDOP_DIV: case PDOP_RDIV:
            *need = 2; return -1;
        default:
            if (op > 0 && op < PDOP_COUNT_) { *need = 1; return 0; }
            *need = -1; return 0;
    }
}

// Returns the max stack depth of a program (header word included), or < 0 if malformed.
extern "C" int pdeval_program_depth(const int32_t* ops, int64_t n_words) {
    if (!ops || n_words < 2) return -1;
    if ((ops[0] & 0xff) != 0) return -2;
    int d = 0, dmax = 0;
    for (int64_t pc = 1; pc < n_words;) {
        const uint32_t op = (uint32_t)ops[pc] & 0xffu;
        int need;
        const int delta = op_stack_delta(op, &need);
        if (need < 0) return -3;
        if (d < need) return -4;
        if (op == PDOP_POWN || (op >= PDOP_PUSH_P && op <= PDOP_RDIV_P)) {
            const int n = (ops[pc] >> 8) & 0xff;
            if (n < 2 || n > 16) return -5;
        }
        if (op_has_imm(op) && ((uint32_t)ops[pc] & PDEVAL_IMM_PRM)) {   // a constant of the problem
            if (op == PDOP_POW || ((uint32_t)ops[pc] & PDEVAL_IMM_DD)) return -9;
            if (pc + 2 < n_words && ((uint32_t)ops[pc + 1] > 15u || ops[pc + 2] != 0)) return -9;
        }
        d += delta;
        if (d > dmax) dmax = d;
        pc += op_words(ops[pc]);
        if (pc > n_words) return -6;
    }
    if (d != 1) return -7;
    if (dmax != ((ops[0] >> 8) & 0xff)) return -8;  // header must state the true depth
    return dmax;
}

// FP64 flop model per sample point (DESIGN.md section 7 "Roofline"): the FP64 operations the lean
// grid pass executes for each opcode at one point, plus the residual epilogue -- measured once per
// problem on the calibration programs (scripts/microbench.py --set calib under PMC, fitted by
// scripts/flop_calib.py: FLOPs = 2 FMA + MUL + ADD per lane, TRANS estimates not counted;
// profiles/r06_c_calib_force_free.json, profiles/r06_g_calib_kerr_magnetosphere.json), so that the
// model and the SQ counters of a whole batch agree (the round-5 algorithmic
// table was 8 % above the counters for force-free and 7 % below for Kerr).  Where the kernel does
// more than the textbook jet operation, the table says so: a quotient coefficient is a
// Markstein-corrected division (a/a == 1 exactly), a division by a coordinate divides every
// coefficient; a coordinate push reads the power tables (no arithmetic); NEG is folded into the
// tracked sign by the decoder (PD_FOLD_NEG).  Force-free order 4 (15 coefficients); Kerr's 5 live
// coefficients of order 2 (no mixed term, kerr validator.py:77-91).
struct OpCost {
    double add, mul, sq, div, addc, mulc, var, divvar, exp, log, sqrt, pow, padd, pmul, pdiv, prdiv, fused_var,
        fused_p, epi;
};
// force-free: r06_c calibration, POWN from r06_h (n = 2: 66, 3: 193, 4: 132, 5: 501, 7: 751 -- the
// square and product costs below); Kerr: r06_g (the fused PUSH_C + MUL_X / MUL_Y / MUL_P of the
// decoder, pdeval_grid.h decode_kernel: c times the coordinate, or c times K + 1 power coefficients)
static constexpr OpCost kCostFF = {15.0, 125.0, 66.0, 198.0, 1.0, 15.0, 25.0, 85.0, 181.0, 248.0, 188.0, 220.0,
                                   5.5, 66.0, 75.0, 198.0, 25.0, 66.0, 244.0};
static constexpr OpCost kCostKerr = {5.0, 18.0, 11.5, 50.0, 2.5, 6.5, 5.0, 26.0, 41.0, 104.5, 43.5, 57.0,
                                     7.0, 13.5, 26.0, 50.0, 2.0, 3.0, 15.3};
// prev: the opcode before w (Kerr's decoder fuses PUSH_C with a following MUL_X / MUL_Y / MUL_P)
static double op_flops(bool ff, uint32_t w, uint32_t prev = 0xffu) {
    const OpCost& k = ff ? kCostFF : kCostKerr;
    const uint32_t op = w & 0xffu;
    if (!ff && (prev & 0xffu) == PDOP_PUSH_C) {
        if (op == PDOP_MUL_X || op == PDOP_MUL_Y) return k.fused_var;
        if (op == PDOP_MUL_P) return k.fused_p;
    }
    switch (op) {
        case PDOP_ADD: case PDOP_SUB: case PDOP_RSUB: return k.add;
        case PDOP_MUL: return k.mul;
        case PDOP_DIV: case PDOP_RDIV: case PDOP_RDIVC: return k.div;
        case PDOP_ADDC: case PDOP_ADD_X: case PDOP_ADD_Y: case PDOP_SUB_X: case PDOP_SUB_Y: return k.addc;
        case PDOP_MULC: case PDOP_ABS: return k.mulc;
        case PDOP_NEG: return 0.0;
        case PDOP_MUL_X: case PDOP_MUL_Y: return k.var;
        case PDOP_DIV_X: case PDOP_DIV_Y: return k.divvar;
        case PDOP_POWN: {
            // pdeval_grid.h Lean::pown_lean: n = 2 a square, 3 a square and a product, 4 two
            // squares, 5..8 n - 1 products
            const int n = (w >> 8) & 0xff;
            return n == 2 ? k.sq : n == 3 ? k.sq + k.mul : n == 4 ? 2.0 * k.sq : (n - 1) * k.mul;
        }
        case PDOP_EXP: return k.exp;
        case PDOP_LOG: return k.log;
        case PDOP_SQRT: return k.sqrt;
        case PDOP_POW: return k.pow;
        case PDOP_ADD_P: case PDOP_SUB_P: return k.padd;
        case PDOP_MUL_P: return k.pmul;
        case PDOP_DIV_P: return k.pdiv;
        case PDOP_RDIV_P: return k.prdiv;
        default: return 0.0;   // pushes: the jet of a coordinate, a constant or a power table entry
    }
}

extern "C" double pdeval_program_flops(int problem_id, const int32_t* ops, int64_t n_words) {
    const bool ff = problem_id == PDEVAL_PROBLEM_FORCE_FREE;
    double f = 0.0;
    uint32_t prev = 0xffu;
    for (int64_t pc = 1; pc < n_words;) {
        f += op_flops(ff, (uint32_t)ops[pc], prev);
        prev = (uint32_t)ops[pc];
        pc += op_words(ops[pc]);
    }
    // epilogue: force-free determinant + its magnitude shadow + the zero test; Kerr's 4-term
    // operator + scale + the zero test
    f += (ff ? kCostFF : kCostKerr).epi;
    return f;
}

// The part of pdeval_program_flops that the lean passes evaluate once per grid row (x alone)
// or once per lane (y alone) instead of once per point: the program's hoisted prefix as
// pdeval_grid.h decode_kernel finds it (the longest prefix ending at stack depth 1 whose value
// depends on one coordinate only, holding a heavy opcode, not the whole program; Kerr: PUSH_C +
// MUL_X / MUL_Y / MUL_P decode into one push).
extern "C" double pdeval_program_hoist_flops(int problem_id, const int32_t* ops, int64_t n_words) {
    const bool ff = problem_id == PDEVAL_PROBLEM_FORCE_FREE;
    if (pdeval_program_depth(ops, n_words) < 1) return 0.0;
    uint32_t msk[PDEVAL_MAX_STACK + 2] = {};
    int d = 0;
    double f = 0.0, f_at = 0.0;
    bool heavy = false, heavy_at = false, alive = true, cplx = false;
    uint32_t msk_at = 0u;
    int64_t at = -1;
    // Kerr's hoisted segment (pdeval_grid.h PD_HOIST_SUB): depth-2 segments of one coordinate
    // holding a heavy opcode, at most 31 words, after the prefix; the one with most heavy opcodes
    struct Seg { int64_t hs, he; int nh; double f; bool y; };
    Seg segs[4];
    int nseg = 0, seg_nh = 0;
    int64_t seg_start = -1;
    double seg_f0 = 0.0;
    auto heavy_op = [](uint32_t op) {
        return op == PDOP_MUL || op == PDOP_DIV || op == PDOP_RDIV || op == PDOP_RDIVC || op == PDOP_POWN ||
               op == PDOP_POW || op == PDOP_SQRT || op == PDOP_EXP || op == PDOP_LOG || op == PDOP_MUL_P ||
               op == PDOP_DIV_P || op == PDOP_RDIV_P || op == PDOP_DIV_X;
    };
    auto track_prefix = [&](int64_t pc_next) {
        if (!alive || d != 1) return;
        if ((msk[1] & 4u) || msk[1] == 3u) {
            alive = false;
            return;
        }
        at = pc_next; f_at = f; heavy_at = heavy; msk_at = msk[1];
    };
    for (int64_t pc = 1; pc < n_words;) {
        const uint32_t w = (uint32_t)ops[pc];
        const uint32_t op = w & 0xffu;
        int64_t len = op_words(ops[pc]);
        const bool on_y = (w >> 16) & 1u;
        if (!ff && op == PDOP_PUSH_C && pc + len < n_words) {   // (PD_FUSE_PUSHC = 1)
            const uint32_t w2 = (uint32_t)ops[pc + len], op2 = w2 & 0xffu;
            if (op2 == PDOP_MUL_X || op2 == PDOP_MUL_Y || op2 == PDOP_MUL_P) {
                ++d;
                msk[d] = (op2 == PDOP_MUL_Y || (op2 == PDOP_MUL_P && ((w2 >> 16) & 1u))) ? 2u : 1u;
                if (d == 2) { seg_start = pc; seg_nh = 0; seg_f0 = f; }
                f += op_flops(ff, w) + op_flops(ff, w2, w);
                pc += len + 1;
                track_prefix(pc);
                continue;
            }
        }
        switch (op) {
            case PDOP_PUSH_X: msk[++d] = 1u; break;
            case PDOP_PUSH_Y: msk[++d] = 2u; break;
            case PDOP_PUSH_C: msk[++d] = 0u; break;
            case PDOP_PUSH_I: msk[++d] = 4u; cplx = true; break;
            case PDOP_PUSH_P: msk[++d] = on_y ? 2u : 1u; break;
            case PDOP_ADD: case PDOP_SUB: case PDOP_RSUB: case PDOP_MUL: case PDOP_DIV: case PDOP_RDIV:
                --d;
                if (d == 1 && seg_start >= 0) {
                    const uint32_t m2 = msk[2];
                    if (seg_nh > 0 && m2 <= 2u && pc - seg_start <= 31 && nseg < 4)
                        segs[nseg++] = {seg_start, pc, seg_nh, f - seg_f0, m2 == 2u};
                    seg_start = -1;
                }
                msk[d] |= msk[d + 1];
                break;
            case PDOP_ADD_X: case PDOP_SUB_X: case PDOP_MUL_X: case PDOP_DIV_X: msk[d] |= 1u; break;
            case PDOP_ADD_Y: case PDOP_SUB_Y: case PDOP_MUL_Y: case PDOP_DIV_Y: msk[d] |= 2u; break;
            case PDOP_ADD_P: case PDOP_SUB_P: case PDOP_MUL_P: case PDOP_DIV_P: case PDOP_RDIV_P:
                msk[d] |= on_y ? 2u : 1u;
                break;
            default: break;
        }
        if ((op == PDOP_PUSH_X || op == PDOP_PUSH_Y || op == PDOP_PUSH_C || op == PDOP_PUSH_I ||
             op == PDOP_PUSH_P) && d == 2) {
            seg_start = pc; seg_nh = 0; seg_f0 = f;
        }
        f += op_flops(ff, w);
        heavy = heavy || heavy_op(op);
        if (d >= 2 && heavy_op(op)) ++seg_nh;
        pc += len;
        track_prefix(pc);
    }
    // (a NEG costs nothing in the model -- the decoder folds it into the tracked sign; force-free
    // hoists prefixes of x only, pdeval_grid.h)
    double h = 0.0;
    int64_t hp = 0;
    if (!(ff && (msk_at & 2u)) && at > 0 && at < n_words && at < (1 << 14) && heavy_at) {
        h = f_at;
        hp = at;
    }
    if (!ff && !cplx) {
        int best = -1;
        for (int k = 0; k < nseg; ++k)
            if (segs[k].hs >= hp && (best < 0 || segs[k].nh > segs[best].nh)) best = k;
        if (best >= 0) h += segs[best].f;
    }
    return h;
}

// ---------------------------------------------------------------------------- launches
static void copy_constants(const pdeval_ctx* c, KernelArgs& a) {
    a.prm_pt = c->prm_pt;
    a.prm_grid = c->prm_grid;
    a.prm_pt_dd = c->prm_pt_dd;
    a.prm_grid_dd = c->prm_grid_dd;
    a.n_ct = c->n_ct;
    for (int k = 0; k < 8; ++k) {
        a.ct_x[k] = c->ct_x[k];
        a.ct_y[k] = c->ct_y[k];
    }
}

// the decoded-program array of the lean grid passes: as many words as the batch's programs
// (grown when a batch outgrows it, like the work lists; never inside a sized call)
static int ensure_dec(pdeval_ctx* c, int64_t n_words) {
    if (n_words <= c->dec_cap) return PDEVAL_OK;
    ++c->buf_epoch;
    if (c->d_dec) (void)hipFree(c->d_dec);
    c->d_dec = nullptr;
    c->dec_cap = 0;
    const int64_t cap = n_words < 4096 ? 4096 : n_words;
    // + 4 words: the lean interpreter reads an opcode word with the two after it (pdeval_grid.h)
    HIPCHK(c, hipMalloc(&c->d_dec, (cap + 4) * sizeof(int32_t)));
    c->dec_cap = cap;
    return PDEVAL_OK;
}

static int ensure_scratch(pdeval_ctx* c, int64_t n) {
    if (n <= c->cap) return PDEVAL_OK;
    ++c->buf_epoch;
    for (int64_t*& l : c->d_list) {
        if (l) (void)hipFree(l);
        l = nullptr;
    }
    c->cap = 0;
    const int64_t cap = n < 1024 ? 1024 : n;
    for (int64_t*& l : c->d_list) HIPCHK(c, hipMalloc(&l, cap * sizeof(int64_t)));
    if (c->d_pstate) (void)hipFree(c->d_pstate);
    c->d_pstate = nullptr;
    HIPCHK(c, hipMalloc(&c->d_pstate, cap));
    if (c->d_ddps) (void)hipFree(c->d_ddps);
    c->d_ddps = nullptr;
    HIPCHK(c, hipMalloc(&c->d_ddps, cap));
    if (c->d_dd_res) (void)hipFree(c->d_dd_res);
    if (c->d_dd_q) (void)hipFree(c->d_dd_q);
    c->d_dd_res = c->d_dd_q = nullptr;
    HIPCHK(c, hipMalloc(&c->d_dd_res, cap * 4 * sizeof(double)));   // (n_ref <= 4)
    HIPCHK(c, hipMalloc(&c->d_dd_q, cap * sizeof(double)));
    if (c->d_hseg) (void)hipFree(c->d_hseg);
    c->d_hseg = nullptr;
    if (c->hoist) {
        // per slot (8 pools of kHoistPool, one per XCD; pdeval_grid.h hoist_acquire): the
        // prefix's pure coefficients (K + 1 rows of 64) and the segment's whole jet (nc(K) rows
        // of 64, Kerr only) -- pd::hoist_stride; allocated once, it does not grow with the batch
        const int K = c->problem == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
        if (c->hoist_slots && !c->d_hoist) {
            HIPCHK(c, hipMalloc(&c->d_hoist, (size_t)8 * pd::kHoistPool * pd::hoist_stride(K) * sizeof(double)));
            HIPCHK(c, hipMalloc(&c->d_hoist_own, (size_t)8 * pd::kHoistPool * sizeof(uint32_t)));
            HIPCHK(c, hipMemset(c->d_hoist_own, 0, (size_t)8 * pd::kHoistPool * sizeof(uint32_t)));   // all free
        } else if (!c->hoist_slots) {   // (A/B: the round-5 layout, one slot per candidate)
            if (c->d_hoist) (void)hipFree(c->d_hoist);
            c->d_hoist = nullptr;
            HIPCHK(c, hipMalloc(&c->d_hoist, (size_t)std::max<int64_t>(cap, 8 * pd::kHoistPool) * pd::hoist_stride(K) * sizeof(double)));
        }
        // the decoder's per-candidate segment records
        HIPCHK(c, hipMalloc(&c->d_hseg, (size_t)cap * 4 * sizeof(int32_t)));
    }
    if (c->d_fmask) (void)hipFree(c->d_fmask);
    c->d_fmask = nullptr;
    if (c->d_fsum) (void)hipFree(c->d_fsum);
    c->d_fsum = nullptr;
    if (c->tier2_mask) {
        HIPCHK(c, hipMalloc(&c->d_fmask, (size_t)cap * c->nx * (c->ny / 64) * sizeof(uint64_t)));
        HIPCHK(c, hipMalloc(&c->d_fsum, (size_t)cap * sizeof(uint64_t)));
    }
    if (c->d_status) (void)hipFree(c->d_status);
    c->d_status = nullptr;
    HIPCHK(c, hipMalloc(&c->d_status, cap));
    if (c->d_noise) (void)hipFree(c->d_noise);
    c->d_noise = nullptr;
    HIPCHK(c, hipMalloc(&c->d_noise, cap * 4 * sizeof(double)));
    if (c->d_t2acc) (void)hipFree(c->d_t2acc);
    c->d_t2acc = nullptr;
    HIPCHK(c, hipMalloc(&c->d_t2acc, cap * sizeof(T2Acc)));
    HIPCHK(c, hipMemset(c->d_t2acc, 0, cap * sizeof(T2Acc)));   // tier 2 leaves it zero
    if (c->d_skeys) (void)hipFree(c->d_skeys);
    if (c->d_sidx) (void)hipFree(c->d_sidx);
    if (c->d_stemp) (void)hipFree(c->d_stemp);
    c->d_skeys = nullptr;
    c->d_sidx = nullptr;
    c->d_stemp = nullptr;
    HIPCHK(c, hipMalloc(&c->d_skeys, 2 * cap * sizeof(uint64_t)));
    HIPCHK(c, hipMalloc(&c->d_sidx, 2 * cap * sizeof(int32_t)));
    c->stemp_bytes = sort_temp_bytes(cap);
    HIPCHK(c, hipMalloc(&c->d_stemp, c->stemp_bytes ? c->stemp_bytes : 16));
    c->cap = cap;
    return PDEVAL_OK;
}

// dynamic LDS of one block: waves x (MAXD-1) stack slots x jet x 64 lanes (<= 160 KiB/CU)
template <class T, int K, int MAXD> constexpr size_t stack_lds(int waves) {
    return (size_t)waves * (MAXD - 1) * ((K + 1) * (K + 2) / 2) * 64 * sizeof(T);
}

// dynamic LDS of one tier-2 wave: (MAXD-1) slots of a value jet (T) and an error jet (f64)
// waves per tier-2 list entry (pdeval_tier2.h): real lists are long (thousands of entries per
// 2^20 batch), the complex list short (~150)
#ifndef PD_T2_PARTS
#define PD_T2_PARTS 4
#endif
#ifndef PD_T2_PARTS_C
#define PD_T2_PARTS_C 16
#endif
template <class T, int K, int MAXD> constexpr size_t tier2_lds() {
    return (size_t)(MAXD - 1) * ((K + 1) * (K + 2) / 2) * 64 * (sizeof(T) + sizeof(double));
}

#ifndef PD_DD_EARLY_MIN_N
#define PD_DD_EARLY_MIN_N 1024
#endif

// The entries of a work list checked in a pass of their own, before the hot list kernels
// (pass 2, the complex pass) read them unchecked: an entry outside [0, n) sets `code` in the
// error word and empties the list (the call then reports the error; no kernel follows the entry).
__global__ __launch_bounds__(256) void sanitize_list_kernel(const int64_t* list, int32_t* count, int64_t cap,
                                                            int64_t n, uint32_t* errw, uint32_t code) {
    int64_t m = (int64_t)*count;
    if (m > cap) m = cap;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = list[i];
        bad = bad || c < 0 || c >= n;
    }
    if (bad) {
        atomicOr(errw, code);
        *count = 0;
    }
}

// zeroes `words` 32-bit words (the list counters, a small batch's verdict bits) -- a kernel node
// in the captured graphs rather than a memset node
__global__ void zero_words_kernel(uint32_t* p, int64_t words) {
    for (int64_t i = threadIdx.x; i < words; i += blockDim.x) p[i] = 0u;
}

template <int PROB>
static int launch_all(pdeval_ctx* c, const int32_t* d_ops, int64_t n_words, const int64_t* d_off, int64_t n,
                      const pdeval_params& prm, const pdeval_outputs& o, hipStream_t s,
                      int dmax = PDEVAL_MAX_STACK) {
    // dmax: the batch's largest program depth when the host knows it (pdeval_validate_batch
    // checks every header); the kernels of the lists only deeper programs reach are skipped --
    // they would read a zero count and exit (what a small batch mostly pays for is launches)
    auto mark = [&](int k) {
        if (c->timing) (void)hipEventRecord(c->ev[k], s);
    };
    KernelArgs a{};
    a.ops = d_ops;
    a.offsets = d_off;
    a.n_words = n_words;
    a.n = n;
    for (int k = 0; k < 4; ++k) {
        a.ref_x[k] = c->ref_x[k];
        a.ref_y[k] = c->ref_y[k];
        a.ref_xd[k] = c->ref_xd[k];
        a.ref_yd[k] = c->ref_yd[k];
    }
    for (int k = 0; k < 16; ++k) a.kc_ref[k] = c->kc_ref[k];
    copy_constants(c, a);
    a.gx = c->d_gx;
    a.gy = c->d_gy;
    a.nx = c->nx;
    a.ny = c->ny;
    a.kc = c->d_kc;
    a.kc2 = c->d_kc ? c->d_kc + 4 * (size_t)c->n_pts : nullptr;
    a.ptab = c->d_ptab;
    a.n_ref = c->n_ref;
    a.n_pts = c->n_pts;
    for (int f = 0; f < PDEVAL_FP_N; ++f) a.fp_pts[f] = c->fp_pts[f];
    a.prm = prm;
    a.out = o;
    // the double-double tier reads the final classes: keep them even if the caller does not
    if (!a.out.status) a.out.status = c->d_status;
    a.list_capacity = c->cap;
    int32_t* const cnt = c->d_counts;
    // (a kernel, not hipMemsetAsync: captured into the small-batch graphs, a memset node was
    // seen to leave these counters unzeroed on replay -- the stale counts of an earlier, larger
    // batch then sent the list passes to entries outside the batch, profiles/r05_e_pytest_gpu.log)
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, s, (uint32_t*)cnt, (int64_t)PD_COUNT_WORDS);
    HIPCHK(c, hipGetLastError());
    a.errw = (uint32_t*)(cnt + PD_N_LISTS);
    auto queue = [&](KernelArgs b, int q) {   // a persistent list launch with its own work queue
        if (c->list_queue > 0) {
            b.qhead = (uint32_t*)(cnt + PD_N_LISTS + 1 + q);
            b.qchunk = c->list_queue;
        }
        return b;
    };
    const int lparts = std::max(grid_parts(n), c->list_parts);
    constexpr int K = PROB == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2;
    constexpr bool FF = PROB == PDEVAL_PROBLEM_FORCE_FREE;
    constexpr int WPB = 4;  // waves (candidates) per 256-thread block of pass 1
    const int64_t blocks = (n + WPB - 1) / WPB;
    // one list-driven pass: persistent blocks over list `in`, programs deeper than the variant's
    // stack appended to `out`, tier-1 failures to `esc`
    auto follow = [&](int in, int out, int esc) {
        KernelArgs b = a;
        b.list = c->d_list[in];
        b.list_count = cnt + in;
        b.defer_list = out >= 0 ? c->d_list[out] : nullptr;
        b.defer_count = out >= 0 ? cnt + out : nullptr;
        b.cplx_list = FF ? c->d_list[L_CPLX] : nullptr;   // real passes: not real at p* -> complex
        b.cplx_count = cnt + L_CPLX;
        b.esc_list = c->d_list[esc];
        b.esc_count = cnt + esc;
        return b;
    };
    // (small batches: enough blocks for every (candidate, part) of the split grid passes)
    const unsigned pgrid = (unsigned)std::min<int64_t>(std::max<int64_t>(4 * blocks, n * lparts), 8192);
    // list-driven point kernels (one candidate per lane): enough blocks for the rare lists
    const unsigned lgrid = (unsigned)std::min<int64_t>((n + 63) / 64, 2048);
    a.defer_list = c->d_list[L_DEFER];
    a.defer_count = cnt + L_DEFER;
    a.cplx_list = FF ? c->d_list[L_CPLX] : nullptr;
    a.cplx_count = cnt + L_CPLX;
    a.esc_list = c->d_list[L_ESC];
    a.esc_count = cnt + L_ESC;
    a.pstate = c->d_pstate;
    a.ddps = c->d_ddps;
    a.dd_res = c->d_dd_res;
    a.dd_q = c->d_dd_q;
    a.dd_spec = 0;   // (set in launch_all when the early tier runs)
    a.pdeep_list = c->d_list[L_PDEEP];
    a.pdeep_count = cnt + L_PDEEP;
    a.noise_ref = c->d_noise;
    a.t2acc = c->d_t2acc;
    a.dec = c->d_dec;
    a.hoist = c->nx <= 64 ? c->d_hoist : nullptr;   // (one grid row per lane)
    a.hoist_own = c->hoist_slots ? c->d_hoist_own : nullptr;
    a.hoist_pool = pd::kHoistPool;
    a.hseg = a.hoist && c->hoist_sub ? c->d_hseg : nullptr;
    a.fmask = c->d_fmask;
    a.fsum = c->d_fsum;
    // ---- the point stage (pdeval_point.h), decided for every candidate before the grid
    // pass 0: real programs of stack <= 2, one candidate per lane; deeper ones -> L_PDEEP,
    // complex-valued ones -> L_CPLX.  Lanes take the candidates sorted by opcode sequence
    // (pdeval_sort.hip; the sort is part of pass 0's time)
    mark(0);
    if (c->sort && n > 1) {
        const int rc = sort_batch(d_ops, d_off, n_words, n, c->d_skeys, c->d_sidx, c->d_stemp, c->stemp_bytes, s);
        if (rc != 0) {
            c->err = std::string("shape sort: ") + hipGetErrorString((hipError_t)rc);
            return PDEVAL_ERR_HIP;
        }
        a.perm = c->d_sidx + n;
    }
    hipLaunchKernelGGL((point_kernel<PROB>), dim3((unsigned)((n + 255) / 256)), dim3(256),
                       (size_t)4 * 2 * nc(K) * 64 * sizeof(double), s, a);
    HIPCHK(c, hipGetLastError());
    // the deep real programs, then (force-free) the complex list, operand stacks in private memory
    mark(1);
    if (dmax > 2) {
        KernelArgs b = follow(L_PDEEP, -1, L_ESC);
        launch_point_list(PROB, 0, lgrid, s, b);
        HIPCHK(c, hipGetLastError());
    }
    if constexpr (FF) {
        KernelArgs b = follow(L_CPLX, -1, L_ESC_C);
        launch_point_list(PROB, 1, lgrid, s, b);
        HIPCHK(c, hipGetLastError());
    }
    // the double-double lists: early = L_DD / L_DDC / L_DD8, late = L_DDL / L_DDLC / L_DDL8
    auto dd_lists = [&](int l0, int lc, int l8) {
        KernelArgs b = a;
        b.defer_list = c->d_list[l0];
        b.defer_count = cnt + l0;
        b.cplx_list = c->d_list[lc];   // (Kerr: never appended to, count 0)
        b.cplx_count = cnt + lc;
        b.esc_list = c->d_list[l8];
        b.esc_count = cnt + l8;
        return b;
    };
    const unsigned cgrid = (unsigned)((n + 255) / 256);
    // (below ~1,000 candidates the double-double tier is short and the fork only adds launches:
    // 512 candidates 2.40 vs 2.36 ms, 1,024: 2.89 vs 3.24 ms, profiles/r04_k_device_batch.log)
    const bool early = c->dd_early && n >= PD_DD_EARLY_MIN_N;
    // the provisional point passes join the early tier speculatively (PD_DD_SPEC): the late tier
    // after the grid -- on the critical path of every batch, 1.5 ms of a 4,096-candidate call,
    // profiles/r06_g_device_batch.log -- is left with nothing but its collect pass
    a.dd_spec = early && c->dd_spec ? 1 : 0;
    if (early) {
        // ---- the early double-double tier (pdeval_point.h): the candidates the point stage
        // left undecided or not accurate enough in fp64 are known now, so their evaluation runs
        // on the side stream beside the grid passes (classes to ddps, applied after the grid)
        hipLaunchKernelGGL((dd_collect_kernel<PROB, DD_EARLY>), dim3(cgrid), dim3(256), 0, s, dd_lists(L_DD, L_DDC, L_DD8));
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(c->ev_fork, s));
        HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
        launch_dd_point(PROB, 0, lgrid, c->side, follow(L_DD, -1, L_ESC), true);
        if (dmax > 2) launch_dd_point(PROB, 1, lgrid, c->side, follow(L_DD8, -1, L_ESC), true);
        if constexpr (FF) launch_dd_point(PROB, 2, lgrid, c->side, follow(L_DDC, -1, L_ESC), true);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(c->ev_join, c->side));
    }
    // ---- the grid stage
    // pass 1: programs whose stack fits 2 jets (99 % of force-free depth 4), one wave per
    // candidate; deeper programs go to L_DEFER, tier-1 grid failures to L_ESC
    mark(2);
    launch_decode(PROB, n, s, a);   // (part of pass 1's time)
    HIPCHK(c, hipGetLastError());
    launch_grid(PROB, n, s, a, c->d_list[L_SLOW], cnt + L_SLOW);
    HIPCHK(c, hipGetLastError());
    // what the lean pass did not take (normally nothing): the generic kernel, same pass slot
    hipLaunchKernelGGL((validate_kernel<PROB, double, 2, true>), dim3((unsigned)std::min<int64_t>(blocks, 256)),
                       dim3(64), (stack_lds<double, K, 2>(1)), s, follow(L_SLOW, L_DEFER, L_ESC));
    HIPCHK(c, hipGetLastError());
    // pass 2: stack 3, the lean interpreter over the L_DEFER list (64-thread blocks, 2 LDS
    // slots); what it does not take, the generic stack-3 kernel
    mark(3);
    if (dmax > 2) {
        hipLaunchKernelGGL(sanitize_list_kernel, dim3(64), dim3(256), 0, s, c->d_list[L_DEFER], cnt + L_DEFER, c->cap, n,
                           a.errw, (uint32_t)ERRW_GRID_LIST);
        launch_grid_list(PROB, pgrid, s, queue(follow(L_DEFER, L_DEFER2, L_ESC), Q_PASS2), c->d_list[L_SLOW2],
                         cnt + L_SLOW2, lparts);
        HIPCHK(c, hipGetLastError());
        hipLaunchKernelGGL((validate_kernel<PROB, double, 3, true>), dim3((unsigned)std::min<int64_t>(blocks, 256)),
                           dim3(64), (stack_lds<double, K, 3>(1)), s, follow(L_SLOW2, L_DEFER2, L_ESC));
        HIPCHK(c, hipGetLastError());
    }
    // pass 3: stack 4..8 (rare; the flattener guarantees <= PDEVAL_MAX_STACK)
    mark(4);
    if (dmax > 3) {
        // (the stack-8 list: a few dozen to a few hundred candidates, each grid split over
        // PD_DEEP_PARTS waves -- pdeval_kernels.h validate_kernel; env PDEVAL_DEEP_PARTS=1: one wave)
        if (c->deep_parts > 1)
            hipLaunchKernelGGL((validate_kernel<PROB, double, PDEVAL_MAX_STACK, true, PD_DEEP_PARTS>),
                               dim3((unsigned)std::min<int64_t>(4 * blocks, 1024)), dim3(64),
                               (stack_lds<double, K, PDEVAL_MAX_STACK>(1)), s, follow(L_DEFER2, -1, L_ESC));
        else
            hipLaunchKernelGGL((validate_kernel<PROB, double, PDEVAL_MAX_STACK, true>),
                               dim3((unsigned)std::min<int64_t>(4 * blocks, 1024)), dim3(64),
                               (stack_lds<double, K, PDEVAL_MAX_STACK>(1)), s, follow(L_DEFER2, -1, L_ESC));
        HIPCHK(c, hipGetLastError());
    }
    if constexpr (FF) {
        // complex passes: candidates not real at the reference point, in complex arithmetic
        // (SymPy evaluates the point exactly, in the complex field: validator.py:363-402)
        mark(5);
        // the lean interpreter in complex arithmetic over the decoded programs; what it does not
        // take (point stage undecided, malformed) the generic complex kernel drains
        if (c->lean_cplx) {
            hipLaunchKernelGGL(sanitize_list_kernel, dim3(64), dim3(256), 0, s, c->d_list[L_CPLX], cnt + L_CPLX, c->cap,
                               n, a.errw, (uint32_t)ERRW_CPLX);
            launch_grid_cplx(pgrid, s, queue(follow(L_CPLX, L_CPLX_DEEP, L_ESC_C), Q_CPLX), c->d_list[L_SLOW_C],
                             cnt + L_SLOW_C, lparts);
            HIPCHK(c, hipGetLastError());
            hipLaunchKernelGGL((validate_kernel<PROB, cplx, 2, true>), dim3((unsigned)std::min<int64_t>(blocks, 256)),
                               dim3(64), (stack_lds<cplx, K, 2>(1)), s, follow(L_SLOW_C, L_CPLX_DEEP, L_ESC_C));
        } else {
            hipLaunchKernelGGL((validate_kernel<PROB, cplx, 2, true>), dim3(pgrid), dim3(64),
                               (stack_lds<cplx, K, 2>(1)), s, follow(L_CPLX, L_CPLX_DEEP, L_ESC_C));
        }
        HIPCHK(c, hipGetLastError());
        mark(6);
        if (dmax > 2) {
            if (c->deep_parts > 1)
                hipLaunchKernelGGL((validate_kernel<PROB, cplx, PDEVAL_MAX_STACK, true, PD_DEEP_PARTS>),
                                   dim3((unsigned)std::min<int64_t>(4 * blocks, 512)), dim3(64),
                                   (stack_lds<cplx, K, PDEVAL_MAX_STACK>(1)), s, follow(L_CPLX_DEEP, -1, L_ESC_C));
            else
                hipLaunchKernelGGL((validate_kernel<PROB, cplx, PDEVAL_MAX_STACK, true>),
                                   dim3((unsigned)std::min<int64_t>(4 * blocks, 512)), dim3(64),
                                   (stack_lds<cplx, K, PDEVAL_MAX_STACK>(1)), s, follow(L_CPLX_DEEP, -1, L_ESC_C));
            HIPCHK(c, hipGetLastError());
        }
    } else {
        mark(5);
        mark(6);
    }
    // tier 2 (pdeval_tier2.h): re-decide every tier-1 grid failure with error bounds, by stack
    KernelArgs t = queue(follow(L_ESC, L_ESC_DEEP, L_ESC), Q_T2);
    mark(7);
    // (PARTS waves per entry: pdeval_tier2.h)
    hipLaunchKernelGGL((tier2_kernel<PROB, double, 2, false, PD_T2_PARTS>), dim3((unsigned)std::min<int64_t>(n * PD_T2_PARTS, 8192)),
                       dim3(64), (tier2_lds<double, K, 2>()), s, t);
    HIPCHK(c, hipGetLastError());
    mark(8);
    if (dmax > 2) {
        hipLaunchKernelGGL((tier2_kernel<PROB, double, 3, false, PD_T2_PARTS>), dim3((unsigned)std::min<int64_t>(n * PD_T2_PARTS, 4096)),
                           dim3(64), (tier2_lds<double, K, 3>()), s, queue(follow(L_ESC_DEEP, L_ESC_DEEP2, L_ESC), Q_T2_3));
        HIPCHK(c, hipGetLastError());
    }
    mark(9);
    if (dmax > 3) {
        hipLaunchKernelGGL((tier2_kernel<PROB, double, PDEVAL_MAX_STACK>), dim3((unsigned)std::min<int64_t>(n, 512)),
                           dim3(64), (tier2_lds<double, K, PDEVAL_MAX_STACK>()), s, queue(follow(L_ESC_DEEP2, -1, L_ESC), Q_T2_8));
        HIPCHK(c, hipGetLastError());
    }
    if constexpr (FF) {
        mark(10);
        hipLaunchKernelGGL((tier2_kernel<PROB, cplx, 4, false, PD_T2_PARTS_C>),
                           dim3((unsigned)std::min<int64_t>(n * PD_T2_PARTS_C, 4096)), dim3(64),
                           (tier2_lds<cplx, K, 4>()), s, queue(follow(L_ESC_C, L_ESC_C_DEEP, L_ESC_C), Q_T2_C));
        HIPCHK(c, hipGetLastError());
        // complex programs of stack 5..8: operand stack in private memory (161 KiB of LDS would
        // not fit)
        if (dmax > 4) {
            hipLaunchKernelGGL((tier2_kernel<PROB, cplx, PDEVAL_MAX_STACK, true>), dim3((unsigned)std::min<int64_t>(n, 256)),
                               dim3(64), 0, s, queue(follow(L_ESC_C_DEEP, -1, L_ESC_C), Q_T2_C8));
            HIPCHK(c, hipGetLastError());
        }
    } else {
        mark(10);
    }
    // ---- the point stage's double-double tier (pdeval_point.h): candidates fp64 left
    // undecided, and provisional point passes whose grid stage rejected
    mark(11);
    if (early) {
        // join the side stream; the late lists (provisional point passes the grid classes
        // now make relevant), then the early tier's classes applied to the final grid classes
        HIPCHK(c, hipStreamWaitEvent(s, c->ev_join, 0));
        hipLaunchKernelGGL((dd_collect_kernel<PROB, DD_LATE>), dim3(cgrid), dim3(256), 0, s, dd_lists(L_DDL, L_DDLC, L_DDL8));
        HIPCHK(c, hipGetLastError());
        launch_dd_point(PROB, 0, lgrid, s, follow(L_DDL, -1, L_ESC));
        if (dmax > 2) launch_dd_point(PROB, 1, lgrid, s, follow(L_DDL8, -1, L_ESC));
        if constexpr (FF) launch_dd_point(PROB, 2, lgrid, s, follow(L_DDLC, -1, L_ESC));
        HIPCHK(c, hipGetLastError());
        launch_dd_apply(PROB, (unsigned)std::min<int64_t>(cgrid, 1024), s, dd_lists(L_DD, L_DDC, L_DD8));
        HIPCHK(c, hipGetLastError());
    } else {
        hipLaunchKernelGGL((dd_collect_kernel<PROB, DD_ALL>), dim3(cgrid), dim3(256), 0, s, dd_lists(L_DD, L_DDC, L_DD8));
        HIPCHK(c, hipGetLastError());
        launch_dd_point(PROB, 0, lgrid, s, follow(L_DD, -1, L_ESC));
        if (dmax > 2) launch_dd_point(PROB, 1, lgrid, s, follow(L_DD8, -1, L_ESC));
        if constexpr (FF) launch_dd_point(PROB, 2, lgrid, s, follow(L_DDC, -1, L_ESC));
        HIPCHK(c, hipGetLastError());
    }
    mark(PDEVAL_N_PASSES);
    c->ev_recorded = c->timing ? 1 : 0;
    return PDEVAL_OK;
}

static int check_errw(pdeval_ctx* c, uint32_t w, const char* path, int64_t n, int captured);

static int validate_device(pdeval_ctx* c, const int32_t* d_ops, int64_t n_words, const int64_t* d_offsets,
                           int64_t n, const pdeval_params* params, const pdeval_outputs* d_out, void* stream,
                           int zero_bits, int dmax) {
    if (!c || !d_out || n < 0 || (n > 0 && (!d_ops || !d_offsets)) || n_words < 0) {
        if (c) c->err = "pdeval_validate_device: bad argument";
        return PDEVAL_ERR_ARG;
    }
    if (n > PDEVAL_MAX_BATCH) {
        // work-list counters are int32 and candidate indices travel as 32-bit wave-uniform
        // values: larger batches are split by the caller
        c->err = "pdeval_validate_device: n exceeds PDEVAL_MAX_BATCH";
        return PDEVAL_ERR_ARG;
    }
    if (n == 0) return PDEVAL_OK;
    HIPCHK(c, hipSetDevice(c->device));
    pdeval_params prm;
    if (params) prm = *params;
    else pdeval_default_params(c->problem, &prm);
    int rc = ensure_scratch(c, n);
    if (rc) return rc;
    rc = ensure_dec(c, n_words);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (zero_bits && d_out->verdict_bits)
        HIPCHK(c, hipMemsetAsync(d_out->verdict_bits, 0, ((n + 31) / 32) * 4, s));
    if (c->problem == PDEVAL_PROBLEM_FORCE_FREE)
        return launch_all<PDEVAL_PROBLEM_FORCE_FREE>(c, d_ops, n_words, d_offsets, n, prm, *d_out, s, dmax);
    return launch_all<PDEVAL_PROBLEM_KERR>(c, d_ops, n_words, d_offsets, n, prm, *d_out, s, dmax);
}

extern "C" int pdeval_validate_device(pdeval_ctx* c, const int32_t* d_ops, int64_t n_words,
                                      const int64_t* d_offsets, int64_t n, const pdeval_params* params,
                                      const pdeval_outputs* d_out, void* stream, int zero_bits) {
    // device-resident programs: their depths are not known here, every pass is launched
    return validate_device(c, d_ops, n_words, d_offsets, n, params, d_out, stream, zero_bits, PDEVAL_MAX_STACK);
}

extern "C" int pdeval_device_error(pdeval_ctx* c, uint32_t* word) {
    if (!c || !word) return PDEVAL_ERR_ARG;
    *word = 0u;
    if (!c->d_counts) return PDEVAL_OK;   // no call yet
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(word, c->d_counts + PD_N_LISTS, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return check_errw(c, *word, "device", -1, -1);
}

// ---- small host batches (the plugin's one-candidate validate(), the inline driver loop
// general_method_paper_reproduction.py:1288-1339).  The launch chain is ~22 kernels whose work
// is tiny for a handful of candidates; launched one by one, submission dominates the call.  So
// the chain is captured once per (n, params) as a HIP graph over fixed-capacity context
// buffers (programs bounds-checked against the capacity: the host already validated every
// program and offset), and one graph launch replays it; inputs go up and the whole output
// block comes back through one pinned staging buffer.  Same kernels, same arguments, same
// results as the direct path.
#ifndef PD_GRAPH_MAX_N
#define PD_GRAPH_MAX_N 64
#endif
static constexpr int64_t kSmallWords = 4096;   // input capacity of the graph path (words)
static constexpr int kGraphFallback = -1000;

// the device error word of the last launch chain (KernelArgs::errw): a work-list entry outside
// [0, n) was met and skipped -- the outputs of the call are not to be trusted
static int check_errw(pdeval_ctx* c, uint32_t w, const char* path = "direct", int64_t n = -1, int captured = -1) {
    if (!w) return PDEVAL_OK;
    // the state of the call, for the report: list counters, capacity, the buffer epoch
    int32_t h[PD_N_LISTS] = {0};
    (void)hipMemcpy(h, c->d_counts, sizeof(h), hipMemcpyDeviceToHost);
    std::string cnt;
    for (int k = 0; k < PD_N_LISTS; ++k) cnt += (k ? "," : "") + std::to_string(h[k]);
    char buf[256];
    std::snprintf(buf, sizeof(buf),
                  "device work-list check failed (kernel families 0x%x; 0x100: no free hoist slot): a list entry "
                  "outside the batch [%s n=%lld "
                  "captured=%d cap=%lld epoch=%llu graphs=%zu counts=",
                  (unsigned)w, path, (long long)n, captured, (long long)c->cap, (unsigned long long)c->buf_epoch,
                  c->graphs.size());
    c->err = std::string(buf) + cnt + "]";
    return PDEVAL_ERR_HIP;
}

static int64_t outbuf_layout(const pdeval_ctx* c, int64_t n, pdeval_outputs* d) {
    const int64_t nb = ((n + 31) / 32) * 4;
    const int64_t sz_bits = (nb + 15) / 16 * 16, sz_st = (n + 15) / 16 * 16;
    const int64_t need = sz_bits + sz_st + 8 * n * (3 + c->n_ref + PDEVAL_FP_N) + 8 * n * 2;
    if (d) {
        uint8_t* p = c->d_outbuf;
        d->verdict_bits = p; p += sz_bits;
        d->status = p; p += sz_st;
        d->q_ref = (double*)p; p += 8 * n;
        d->q_grid = (double*)p; p += 8 * n;
        d->res_ref = (double*)p; p += 8 * n * c->n_ref;
        d->fingerprint = (double*)p; p += 8 * n * PDEVAL_FP_N;
        d->n_bad = (int32_t*)p; p += 4 * n;
        d->n_nonfinite = (int32_t*)p;
    }
    return need;
}

static int validate_small(pdeval_ctx* c, const int32_t* ops, int64_t n_words, const int64_t* offsets, int64_t n,
                          const pdeval_params* params, pdeval_outputs* out, int dmax) {
    if (n_words > kSmallWords) return kGraphFallback;
    // fixed-capacity buffers (growing them drops every captured graph)
    if (c->hcap_words < kSmallWords || c->hcap_n < PD_GRAPH_MAX_N + 1) {
        ++c->buf_epoch;
        const int64_t w = std::max<int64_t>(kSmallWords, c->hcap_words);
        const int64_t m = std::max<int64_t>(PD_GRAPH_MAX_N + 1, c->hcap_n);
        if (c->d_ops) (void)hipFree(c->d_ops);
        if (c->d_off) (void)hipFree(c->d_off);
        c->d_ops = nullptr;
        c->d_off = nullptr;
        c->hcap_words = c->hcap_n = 0;
        HIPCHK(c, hipMalloc(&c->d_ops, w * sizeof(int32_t)));
        HIPCHK(c, hipMalloc(&c->d_off, m * sizeof(int64_t)));
        c->hcap_words = w;
        c->hcap_n = m;
    }
    const int64_t need_max = outbuf_layout(c, PD_GRAPH_MAX_N, nullptr);
    if (c->outbuf_bytes < need_max) {
        ++c->buf_epoch;
        if (c->d_outbuf) (void)hipFree(c->d_outbuf);
        c->d_outbuf = nullptr;
        c->outbuf_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_outbuf, need_max));
        c->outbuf_bytes = need_max;
    }
    int rc = ensure_scratch(c, n);
    if (rc) return rc;
    rc = ensure_dec(c, c->hcap_words);
    if (rc) return rc;
    const size_t in_bytes = kSmallWords * 4 + (PD_GRAPH_MAX_N + 1) * 8;
    if (!c->h_stage) {
        HIPCHK(c, hipHostMalloc((void**)&c->h_stage, in_bytes + need_max + 16, hipHostMallocDefault));
        c->h_stage_bytes = in_bytes + need_max + 16;
    }
    pdeval_params prm;
    if (params) prm = *params;
    else pdeval_default_params(c->problem, &prm);
    // graph key: n, the depth class and the parameter bytes (FNV-1a)
    dmax = dmax <= 2 ? 2 : dmax <= 4 ? dmax : PDEVAL_MAX_STACK;
    uint64_t key = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t len) {
        const uint8_t* b = (const uint8_t*)p;
        for (size_t i = 0; i < len; ++i) key = (key ^ b[i]) * 1099511628211ull;
    };
    mix(&n, sizeof(n));
    mix(&dmax, sizeof(dmax));
    mix(&prm, sizeof(prm));
    pdeval_outputs d{};
    const int64_t need = outbuf_layout(c, n, &d);
    hipStream_t s = c->stream;
    auto it = c->graphs.find(key);
    if (it != c->graphs.end() && it->second.epoch != c->buf_epoch) {
        (void)hipGraphExecDestroy(it->second.exec);
        c->graphs.erase(it);
        it = c->graphs.end();
    }
    int fresh = 0;
    if (it == c->graphs.end()) {
        fresh = 1;
        if (c->graphs.size() >= 256) {   // bounded cache
            for (auto& g : c->graphs) (void)hipGraphExecDestroy(g.second.exec);
            c->graphs.clear();
        }
        hipGraph_t g = nullptr;
        if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) return kGraphFallback;
        int lrc = PDEVAL_OK;
        hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, s, (uint32_t*)d.verdict_bits, (int64_t)((n + 31) / 32));
        if (hipGetLastError() != hipSuccess) lrc = PDEVAL_ERR_HIP;
        if (lrc == PDEVAL_OK)
            lrc = c->problem == PDEVAL_PROBLEM_FORCE_FREE
                      ? launch_all<PDEVAL_PROBLEM_FORCE_FREE>(c, c->d_ops, c->hcap_words, c->d_off, n, prm, d, s, dmax)
                      : launch_all<PDEVAL_PROBLEM_KERR>(c, c->d_ops, c->hcap_words, c->d_off, n, prm, d, s, dmax);
        const hipError_t ee = hipStreamEndCapture(s, &g);
        hipGraphExec_t exec = nullptr;
        if (lrc != PDEVAL_OK || ee != hipSuccess || !g || hipGraphInstantiate(&exec, g, nullptr, nullptr, 0) != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            (void)hipGetLastError();
            c->use_graph = false;         // the direct path from now on
            return kGraphFallback;
        }
        (void)hipGraphDestroy(g);
        it = c->graphs.emplace(key, pdeval_ctx::GraphEntry{exec, c->buf_epoch}).first;
    }
    uint8_t* hin = c->h_stage;
    uint8_t* hout = c->h_stage + in_bytes;
    std::memcpy(hin, offsets, (n + 1) * sizeof(int64_t));
    std::memcpy(hin + (PD_GRAPH_MAX_N + 1) * 8, ops, n_words * sizeof(int32_t));
    HIPCHK(c, hipMemcpyAsync(c->d_off, hin, (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_ops, hin + (PD_GRAPH_MAX_N + 1) * 8, n_words * sizeof(int32_t),
                             hipMemcpyHostToDevice, s));
    HIPCHK(c, hipGraphLaunch(it->second.exec, s));
    HIPCHK(c, hipMemcpyAsync(hout, c->d_outbuf, need, hipMemcpyDeviceToHost, s));
    uint32_t* herr = reinterpret_cast<uint32_t*>(c->h_stage + in_bytes + need_max);
    HIPCHK(c, hipMemcpyAsync(herr, c->d_counts + PD_N_LISTS, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (int erc = check_errw(c, *herr, "graph", n, fresh)) return erc;
    auto take = [&](void* h, const void* dv, size_t bytes) {
        if (h) std::memcpy(h, hout + ((const uint8_t*)dv - c->d_outbuf), bytes);
    };
    take(out->verdict_bits, d.verdict_bits, (n + 7) / 8);
    take(out->status, d.status, n);
    take(out->q_ref, d.q_ref, 8 * n);
    take(out->q_grid, d.q_grid, 8 * n);
    take(out->res_ref, d.res_ref, 8 * n * c->n_ref);
    take(out->fingerprint, d.fingerprint, 8 * n * PDEVAL_FP_N);
    take(out->n_bad, d.n_bad, 4 * n);
    take(out->n_nonfinite, d.n_nonfinite, 4 * n);
    return PDEVAL_OK;
}

extern "C" int pdeval_validate_batch(pdeval_ctx* c, const int32_t* ops, int64_t n_words,
                                     const int64_t* offsets, int64_t n, const pdeval_params* params,
                                     pdeval_outputs* out) {
    if (!c || !out || n < 0 || (n > 0 && (!ops || !offsets))) {
        if (c) c->err = "pdeval_validate_batch: bad argument";
        return PDEVAL_ERR_ARG;
    }
    if (n > PDEVAL_MAX_BATCH) {
        c->err = "pdeval_validate_batch: n exceeds PDEVAL_MAX_BATCH";
        return PDEVAL_ERR_ARG;
    }
    if (n == 0) return PDEVAL_OK;
    if (offsets[0] != 0 || offsets[n] != n_words) {
        c->err = "pdeval_validate_batch: offsets must start at 0 and end at n_words";
        return PDEVAL_ERR_ARG;
    }
    int dmax = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (offsets[i + 1] < offsets[i]) {
            c->err = "pdeval_validate_batch: offsets not monotone at " + std::to_string(i);
            return PDEVAL_ERR_ARG;
        }
        const int d = pdeval_program_depth(ops + offsets[i], offsets[i + 1] - offsets[i]);
        if (d < 0 || d > PDEVAL_MAX_STACK) {
            c->err = "pdeval_validate_batch: malformed program " + std::to_string(i) + " (code " +
                     std::to_string(d) + ")";
            return PDEVAL_ERR_PROGRAM;
        }
        dmax = std::max(dmax, d);
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (n <= PD_GRAPH_MAX_N && c->use_graph && !c->timing) {
        const int rc = validate_small(c, ops, n_words, offsets, n, params, out, dmax);
        if (rc != kGraphFallback) return rc;
    }
    if (n_words > c->hcap_words) {
        ++c->buf_epoch;
        if (c->d_ops) (void)hipFree(c->d_ops);
        c->d_ops = nullptr;
        c->hcap_words = 0;
        HIPCHK(c, hipMalloc(&c->d_ops, n_words * sizeof(int32_t)));
        c->hcap_words = n_words;
    }
    if (n + 1 > c->hcap_n) {
        ++c->buf_epoch;
        if (c->d_off) (void)hipFree(c->d_off);
        c->d_off = nullptr;
        c->hcap_n = 0;
        HIPCHK(c, hipMalloc(&c->d_off, (n + 1) * sizeof(int64_t)));
        c->hcap_n = n + 1;
    }
    // device output block
    const int64_t nb = ((n + 31) / 32) * 4;
    const int64_t sz_bits = (nb + 15) / 16 * 16, sz_st = (n + 15) / 16 * 16;
    const int64_t need = sz_bits + sz_st + 8 * n * (3 + c->n_ref + PDEVAL_FP_N) + 8 * n * 2;
    if (need > c->outbuf_bytes) {
        ++c->buf_epoch;
        if (c->d_outbuf) (void)hipFree(c->d_outbuf);
        c->d_outbuf = nullptr;
        c->outbuf_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_outbuf, need));
        c->outbuf_bytes = need;
    }
    uint8_t* p = c->d_outbuf;
    pdeval_outputs d{};
    d.verdict_bits = p; p += sz_bits;
    d.status = p; p += sz_st;
    d.q_ref = (double*)p; p += 8 * n;
    d.q_grid = (double*)p; p += 8 * n;
    d.res_ref = (double*)p; p += 8 * n * c->n_ref;
    d.fingerprint = (double*)p; p += 8 * n * PDEVAL_FP_N;
    d.n_bad = (int32_t*)p; p += 4 * n;
    d.n_nonfinite = (int32_t*)p; p += 4 * n;
    hipStream_t s = c->stream;
    HIPCHK(c, hipMemcpyAsync(c->d_ops, ops, n_words * sizeof(int32_t), hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_off, offsets, (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    int rc = validate_device(c, c->d_ops, n_words, c->d_off, n, params, &d, s, 1, dmax);
    if (rc) return rc;
    auto dl = [&](void* h, const void* dv, size_t bytes) -> int {
        if (h) HIPCHK(c, hipMemcpyAsync(h, dv, bytes, hipMemcpyDeviceToHost, s));
        return PDEVAL_OK;
    };
    if ((rc = dl(out->verdict_bits, d.verdict_bits, (n + 7) / 8))) return rc;
    if ((rc = dl(out->status, d.status, n))) return rc;
    if ((rc = dl(out->q_ref, d.q_ref, 8 * n))) return rc;
    if ((rc = dl(out->q_grid, d.q_grid, 8 * n))) return rc;
    if ((rc = dl(out->res_ref, d.res_ref, 8 * n * c->n_ref))) return rc;
    if ((rc = dl(out->fingerprint, d.fingerprint, 8 * n * PDEVAL_FP_N))) return rc;
    if ((rc = dl(out->n_bad, d.n_bad, 4 * n))) return rc;
    if ((rc = dl(out->n_nonfinite, d.n_nonfinite, 4 * n))) return rc;
    uint32_t* herr = reinterpret_cast<uint32_t*>(c->h_errw);
    if (!herr) {
        HIPCHK(c, hipHostMalloc((void**)&c->h_errw, 16, hipHostMallocDefault));
        herr = reinterpret_cast<uint32_t*>(c->h_errw);
    }
    HIPCHK(c, hipMemcpyAsync(herr, c->d_counts + PD_N_LISTS, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return check_errw(c, *herr, "direct", n);
}

extern "C" int pdeval_set_timing(pdeval_ctx* c, int enable) {
    if (!c) return PDEVAL_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (enable && !c->ev[0])
        for (hipEvent_t& e : c->ev) HIPCHK(c, hipEventCreate(&e));
    c->timing = enable != 0;
    c->ev_recorded = 0;
    return PDEVAL_OK;
}

extern "C" int pdeval_pass_times(pdeval_ctx* c, float* ms, int max_passes, const char** names) {
    if (!c || !ms || max_passes < 0) return PDEVAL_ERR_ARG;
    if (!c->ev_recorded) {
        c->err = "pdeval_pass_times: no timed call (pdeval_set_timing(ctx, 1) first)";
        return PDEVAL_ERR_ARG;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipEventSynchronize(c->ev[PDEVAL_N_PASSES]));
    const int n = max_passes < PDEVAL_N_PASSES ? max_passes : PDEVAL_N_PASSES;
    for (int k = 0; k < n; ++k) {
        HIPCHK(c, hipEventElapsedTime(&ms[k], c->ev[k], c->ev[k + 1]));
        if (names) names[k] = kPassNames[k];
    }
    return PDEVAL_OK;
}

extern "C" int pdeval_pass_counts(pdeval_ctx* c, int64_t* counts, int max_counts) {
    if (!c || !counts || max_counts < 0) return PDEVAL_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int32_t h[PD_N_LISTS] = {0};
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(h, c->d_counts, sizeof(h), hipMemcpyDeviceToHost));
    for (int k = 0; k < max_counts && k < PD_N_LISTS; ++k) counts[k] = h[k];
    return PDEVAL_OK;
}

extern "C" int pdeval_eval_points(pdeval_ctx* c, const int32_t* prog, int64_t n_words, const double* xs,
                                  const double* ys, int n_pts, int tier2, double* out, double* jets) {
    if (!c || !prog || !xs || !ys || !out || n_pts <= 0 || n_pts > (1 << 20)) return PDEVAL_ERR_ARG;
    const int d = pdeval_program_depth(prog, n_words);
    if (d < 0 || d > PDEVAL_MAX_STACK) {
        c->err = "pdeval_eval_points: malformed program";
        return PDEVAL_ERR_PROGRAM;
    }
    if (c->problem == PDEVAL_PROBLEM_KERR) {
        c->err = "pdeval_eval_points: force-free only";
        return PDEVAL_ERR_ARG;
    }
    HIPCHK(c, hipSetDevice(c->device));
    int32_t* d_prog = nullptr;
    double *d_x = nullptr, *d_y = nullptr, *d_out = nullptr, *d_jets = nullptr;
    const size_t jet_bytes = (size_t)n_pts * 2 * 15 * sizeof(double);
    auto cleanup = [&]() {
        for (void* q : {(void*)d_prog, (void*)d_x, (void*)d_y, (void*)d_out, (void*)d_jets})
            if (q) (void)hipFree(q);
    };
    hipError_t e = hipSuccess;
    if ((e = hipMalloc(&d_prog, n_words * 4)) == hipSuccess && (e = hipMalloc(&d_x, n_pts * 8)) == hipSuccess &&
        (e = hipMalloc(&d_y, n_pts * 8)) == hipSuccess && (e = hipMalloc(&d_out, n_pts * 32)) == hipSuccess &&
        (e = hipMemcpy(d_prog, prog, n_words * 4, hipMemcpyHostToDevice)) == hipSuccess &&
        (e = hipMemcpy(d_x, xs, n_pts * 8, hipMemcpyHostToDevice)) == hipSuccess &&
        (e = hipMemcpy(d_y, ys, n_pts * 8, hipMemcpyHostToDevice)) == hipSuccess &&
        (!jets || (e = hipMalloc(&d_jets, jet_bytes)) == hipSuccess)) {
        constexpr int K = 4, MAXD = PDEVAL_MAX_STACK;
        hipLaunchKernelGGL((eval_points_kernel<PDEVAL_PROBLEM_FORCE_FREE, MAXD>), dim3((n_pts + 63) / 64), dim3(64),
                           (tier2_lds<double, K, MAXD>()), c->stream, d_prog, (int)n_words, d_x, d_y,
                           (const double*)nullptr, n_pts, tier2, d_out, d_jets);
        if ((e = hipGetLastError()) == hipSuccess && (e = hipStreamSynchronize(c->stream)) == hipSuccess)
            e = hipMemcpy(out, d_out, n_pts * 32, hipMemcpyDeviceToHost);
        if (e == hipSuccess && jets) e = hipMemcpy(jets, d_jets, jet_bytes, hipMemcpyDeviceToHost);
    }
    cleanup();
    if (e != hipSuccess) {
        c->err = std::string("pdeval_eval_points: ") + hipGetErrorString(e);
        return PDEVAL_ERR_HIP;
    }
    return PDEVAL_OK;
}

extern "C" int pdeval_point_states(pdeval_ctx* c, uint8_t* out, int64_t n) {
    if (!c || !out || n < 0 || n > c->cap) {
        if (c) c->err = "pdeval_point_states: bad argument";
        return PDEVAL_ERR_ARG;
    }
    if (n == 0) return PDEVAL_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(out, c->d_pstate, n, hipMemcpyDeviceToHost));
    return PDEVAL_OK;
}

extern "C" int pdeval_point_eval(pdeval_ctx* c, const int32_t* prog, int64_t n_words, int tier, double* out,
                                 uint8_t* state) {
    if (!c || !prog || !out || !state || tier < 0 || tier > 3 ||
        (c->problem == PDEVAL_PROBLEM_KERR && (tier & 1))) {
        if (c) c->err = "pdeval_point_eval: bad argument";
        return PDEVAL_ERR_ARG;
    }
    const int d = pdeval_program_depth(prog, n_words);
    if (d < 0 || d > PDEVAL_MAX_STACK) {
        c->err = "pdeval_point_eval: malformed program";
        return PDEVAL_ERR_PROGRAM;
    }
    HIPCHK(c, hipSetDevice(c->device));
    pdeval_params prm;
    pdeval_default_params(c->problem, &prm);
    KernelArgs a{};
    for (int k = 0; k < 4; ++k) {
        a.ref_x[k] = c->ref_x[k];
        a.ref_y[k] = c->ref_y[k];
        a.ref_xd[k] = c->ref_xd[k];
        a.ref_yd[k] = c->ref_yd[k];
    }
    for (int k = 0; k < 16; ++k) a.kc_ref[k] = c->kc_ref[k];
    copy_constants(c, a);
    a.kc = c->d_kc;
    a.kc2 = c->d_kc ? c->d_kc + 4 * (size_t)c->n_pts : nullptr;
    a.ptab = c->d_ptab;
    a.n_ref = c->n_ref;
    a.prm = prm;
    int32_t* d_prog = nullptr;
    double* d_out = nullptr;
    uint8_t* d_st = nullptr;
    hipError_t e = hipSuccess;
    if ((e = hipMalloc(&d_prog, n_words * 4)) == hipSuccess && (e = hipMalloc(&d_out, 6 * 4 * 8)) == hipSuccess &&
        (e = hipMalloc(&d_st, 1)) == hipSuccess &&
        (e = hipMemcpy(d_prog, prog, n_words * 4, hipMemcpyHostToDevice)) == hipSuccess) {
        launch_point_eval(c->problem, tier, c->stream, a, d_prog, (int)n_words, d_out, d_st);
        if ((e = hipGetLastError()) == hipSuccess && (e = hipStreamSynchronize(c->stream)) == hipSuccess &&
            (e = hipMemcpy(out, d_out, 6 * c->n_ref * 8, hipMemcpyDeviceToHost)) == hipSuccess)
            e = hipMemcpy(state, d_st, 1, hipMemcpyDeviceToHost);
    }
    for (void* q : {(void*)d_prog, (void*)d_out, (void*)d_st})
        if (q) (void)hipFree(q);
    if (e != hipSuccess) {
        c->err = std::string("pdeval_point_eval: ") + hipGetErrorString(e);
        return PDEVAL_ERR_HIP;
    }
    return PDEVAL_OK;
}

// ---------------------------------------------------------------------------- multi-GPU
extern "C" int pdeval_comm_unique_id(uint8_t* id) {
    if (!id) return PDEVAL_ERR_ARG;
    Rccl& r = rccl();
    if (!r.h) {
        g_err = "pdeval_comm_unique_id: librccl.so.1 not found";
        return PDEVAL_ERR_NODEVICE;
    }
    ncclUniqueId u;
    const ncclResult_t e = r.get_unique_id(&u);
    if (e != ncclSuccess) {
        g_err = std::string("ncclGetUniqueId: ") + r.error_string(e);
        return PDEVAL_ERR_HIP;
    }
    std::memcpy(id, u.internal, PDEVAL_UNIQUE_ID_BYTES);
    return PDEVAL_OK;
}

extern "C" int pdeval_comm_init(pdeval_ctx* c, int world, int rank, const uint8_t* id) {
    if (!c || !id || world < 1 || rank < 0 || rank >= world || c->comm) {
        if (c) c->err = "pdeval_comm_init: bad argument (or already initialized)";
        return PDEVAL_ERR_ARG;
    }
    Rccl& r = rccl();
    if (!r.h) {
        c->err = "pdeval_comm_init: librccl.so.1 not found";
        return PDEVAL_ERR_NODEVICE;
    }
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId u;
    std::memcpy(u.internal, id, PDEVAL_UNIQUE_ID_BYTES);
    const ncclResult_t e = r.comm_init_rank(&c->comm, world, u, rank);
    if (e != ncclSuccess) {
        c->comm = nullptr;
        c->err = std::string("ncclCommInitRank: ") + r.error_string(e);
        return PDEVAL_ERR_HIP;
    }
    c->world = world;
    c->rank = rank;
    return PDEVAL_OK;
}

extern "C" int pdeval_gather_bits(pdeval_ctx* c, const uint8_t* d_local, int64_t nbytes, uint8_t* d_global,
                                  void* stream) {
    if (!c || !c->comm || !d_local || !d_global || nbytes <= 0) {
        if (c) c->err = "pdeval_gather_bits: bad argument (pdeval_comm_init first)";
        return PDEVAL_ERR_ARG;
    }
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const ncclResult_t e = rccl().all_gather(d_local, d_global, (size_t)nbytes, ncclUint8, c->comm, s);
    if (e != ncclSuccess) {
        c->err = std::string("ncclAllGather: ") + rccl().error_string(e);
        return PDEVAL_ERR_HIP;
    }
    return PDEVAL_OK;
}

extern "C" int pdeval_comm_destroy(pdeval_ctx* c) {
    if (!c) return PDEVAL_ERR_ARG;
    if (c->comm && rccl().h) rccl().comm_destroy(c->comm);
    c->comm = nullptr;
    c->world = 1;
    c->rank = 0;
    return PDEVAL_OK;
}
