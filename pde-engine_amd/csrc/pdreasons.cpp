// pdreasons.cpp -- the reference's reason strings for a whole validated batch (host only).
//
// The reference returns (bool, reason) per candidate from validate()
// (problems/force_free/validator.py:309-427, problems/kerr_magnetosphere/validator.py:231-323);
// the driver's writer stores the reason text (general_method_paper_reproduction.py:1140-1196).
// pdeval/batch.py::reason_for maps one device class to that text; this is the same mapping for
// n candidates at once, written newline-separated into one buffer, so the host side of the
// worker builds its result tuples with one decode + split instead of one Python call per row.
// Numbers are formatted with printf's %.2e / %.3e, which round the exact binary value to
// nearest-even exactly as Python's format() does (tests/test_abi.py checks identity).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <cmath>

#include "../../include/pdeval.h"

namespace {

struct Out {
    char* p;
    int64_t cap, len = 0;
    bool ok = true;
    void put(const char* s, size_t k) {
        if (len + (int64_t)k > cap) { ok = false; return; }
        memcpy(p + len, s, k);
        len += (int64_t)k;
    }
    void put(const char* s) { put(s, strlen(s)); }
    // Python's format(v, '.Ne') for a finite or non-finite double
    void num(double v, int digits) {
        char t[64];
        int k;
        if (std::isnan(v)) k = snprintf(t, sizeof t, "nan");
        else if (std::isinf(v)) k = snprintf(t, sizeof t, v > 0 ? "inf" : "-inf");
        else k = snprintf(t, sizeof t, "%.*e", digits, v);
        put(t, (size_t)k);
    }
};

const char kAcceptFF[] = "Valid foliation (Lean: det = 0 symbolically)";
const char kPointNe[] = "Invalid (point check != 0)";
const char kPointApprox[] = "Invalid (point check \xe2\x89\x88 ";
const char kGridFF[] = "Invalid (Lean could not simplify det to 0 symbolically)";
const char kZeroFF[] = "Zero gradient (constant expression)";
const char kNonfinFF[] = "Could not evaluate point check";
const char kAcceptK[] = "Valid (exact zero; heavy checks deferred)";
const char kPointK[] = "PDE residual != 0 (fast point check) | residual: max|lhs| at test points \xe2\x89\x88 ";
const char kGridK[] = "PDE residual != 0 | residual: max scaled |lhs| on grid \xe2\x89\x88 ";
const char kZeroK[] = "Trivial constant solution excluded";
const char kNonfinK[] = "Invalid (non-real at test point)";
const char kUnsupported[] = "Error: unsupported construct (opcode)";
const char kMalformed[] = "Error: malformed program";

}  // namespace

extern "C" int pdeval_format_reasons(int problem_id, int64_t n, const uint8_t* status, const double* res_ref,
                                     int n_ref, const double* q_ref, const double* q_grid,
                                     const uint8_t* rational, char* buf, int64_t cap, int64_t* len_out) {
    if (n < 0 || (n > 0 && (!status || !res_ref || n_ref < 1 || !q_ref || !q_grid || !rational)) || !buf ||
        cap < 0 || !len_out)
        return PDEVAL_ERR_ARG;
    if (problem_id != PDEVAL_PROBLEM_FORCE_FREE && problem_id != PDEVAL_PROBLEM_KERR) return PDEVAL_ERR_ARG;
    const bool ff = problem_id == PDEVAL_PROBLEM_FORCE_FREE;
    Out o{buf, cap};
    for (int64_t i = 0; i < n && o.ok; ++i) {
        if (i) o.put("\n", 1);
        const int cls = status[i];
        if (ff) {
            switch (cls) {
                case PDEVAL_CLS_ACCEPT: o.put(kAcceptFF); continue;
                case PDEVAL_CLS_REJECT_POINT: {
                    const double v = res_ref[i * n_ref];
                    if (!std::isfinite(v) || rational[i]) { o.put(kPointNe); continue; }
                    o.put(kPointApprox);
                    o.num(std::fabs(v), 2);
                    o.put(")", 1);
                    continue;
                }
                case PDEVAL_CLS_REJECT_GRID: case PDEVAL_CLS_REJECT_SYMBOLIC: o.put(kGridFF); continue;
                case PDEVAL_CLS_ZERO_GRADIENT: o.put(kZeroFF); continue;
                case PDEVAL_CLS_NONFINITE_REF: o.put(kNonfinFF); continue;
                default: break;
            }
        } else {
            switch (cls) {
                case PDEVAL_CLS_ACCEPT: o.put(kAcceptK); continue;
                case PDEVAL_CLS_REJECT_POINT: o.put(kPointK); o.num(q_ref[i], 3); continue;
                case PDEVAL_CLS_REJECT_GRID: o.put(kGridK); o.num(q_grid[i], 3); continue;
                case PDEVAL_CLS_ZERO_GRADIENT: o.put(kZeroK); continue;
                case PDEVAL_CLS_NONFINITE_REF: o.put(kNonfinK); continue;
                default: break;
            }
        }
        o.put(cls == PDEVAL_CLS_UNSUPPORTED ? kUnsupported : kMalformed);
    }
    if (!o.ok) {
        *len_out = -1;   // buffer too small
        return PDEVAL_ERR_ARG;
    }
    *len_out = o.len;
    return PDEVAL_OK;
}
