// The lean grid pass (pass 1): the 64 x 64 grid of every candidate the point stage decided, for
// real programs whose operand stack fits 2 jets (99 % of the force-free depth-4 stream).
//
// Same arithmetic as validate_kernel<PROB, double, 2, ...> -- the same JetOps calls in the same
// order, so every residual is bit-identical -- but laid out for the CDNA issue model rather than
// as one generic kernel:
//  * the program is checked ONCE per candidate (lean_prescan: opcodes, immediates in bounds,
//    stack depth 1..2, ends at depth 1) instead of at every opcode of every grid row; the
//    interpreter then runs with no bounds checks and no stack-depth bookkeeping (the stack is
//    one LDS slot: every push after the first spills the accumulator there, every binary op
//    reads it back);
//  * the reference points (chunk 0) are not part of the loop: pass 0 decided them, so the loop
//    is rows x row-slices with no per-chunk divisions or point-stage branches;
//  * 1/y of the lane's ordinate (DIV_Y) is formed once per wave, 1/x once per row (scalar x);
//  * non-finite counts come from the finite count (one ballot fewer per row).
// Candidates the lean path does not take (malformed programs, P0_NONE, a complex flag without
// the point stage's P0_CPLX) go to the slow list, which the generic validate_kernel<PROB,
// double, 2, true> drains right after this launch -- normally an empty list.
//
// Measured per-wave instruction mix (scripts/gpu_pmc_micro.sh): the generic kernel issued
// ~0.8 SALU per VALU instruction, most of it opcode dispatch, bounds checks and structurizer
// flow masks; that scalar stream competes with the FP64 stream for issue slots.
#pragma once

#include "pdeval_kernels.h"

namespace pd {

constexpr uint64_t op_bit(int op) { return 1ull << op; }
constexpr uint64_t kImmMask = op_bit(PDOP_PUSH_C) | op_bit(PDOP_ADDC) | op_bit(PDOP_MULC) |
                              op_bit(PDOP_RDIVC) | op_bit(PDOP_POW);
constexpr uint64_t kPushMask = op_bit(PDOP_PUSH_X) | op_bit(PDOP_PUSH_Y) | op_bit(PDOP_PUSH_C) |
                               op_bit(PDOP_PUSH_P);
constexpr uint64_t kBinMask = op_bit(PDOP_ADD) | op_bit(PDOP_SUB) | op_bit(PDOP_RSUB) |
                              op_bit(PDOP_MUL) | op_bit(PDOP_DIV) | op_bit(PDOP_RDIV);
constexpr uint64_t kUnaryMask =
    op_bit(PDOP_ADDC) | op_bit(PDOP_MULC) | op_bit(PDOP_RDIVC) | op_bit(PDOP_NEG) |
    op_bit(PDOP_ADD_X) | op_bit(PDOP_ADD_Y) | op_bit(PDOP_SUB_X) | op_bit(PDOP_SUB_Y) |
    op_bit(PDOP_MUL_X) | op_bit(PDOP_MUL_Y) | op_bit(PDOP_DIV_X) | op_bit(PDOP_DIV_Y) |
    op_bit(PDOP_POWN) | op_bit(PDOP_POW) | op_bit(PDOP_EXP) | op_bit(PDOP_LOG) | op_bit(PDOP_ABS) |
    op_bit(PDOP_SQRT) | op_bit(PDOP_ADD_P) | op_bit(PDOP_SUB_P) | op_bit(PDOP_MUL_P) |
    op_bit(PDOP_DIV_P) | op_bit(PDOP_RDIV_P);
// (PUSH_I -- a complex program -- and unknown opcodes are not lean)
constexpr uint64_t kCheapMask = op_bit(PDOP_ADDC) | op_bit(PDOP_NEG) | op_bit(PDOP_MULC) |
                                op_bit(PDOP_ADD_X) | op_bit(PDOP_SUB_X) | op_bit(PDOP_ADD_Y) |
                                op_bit(PDOP_SUB_Y);
constexpr uint64_t kPOpMask = op_bit(PDOP_ADD_P) | op_bit(PDOP_SUB_P) | op_bit(PDOP_MUL_P) |
                              op_bit(PDOP_DIV_P) | op_bit(PDOP_RDIV_P);
constexpr uint64_t kVarMask = op_bit(PDOP_MUL_X) | op_bit(PDOP_MUL_Y) | op_bit(PDOP_DIV_X) |
                              op_bit(PDOP_DIV_Y);

// Program words [1, plen) run by Lean::run with a 2-jet stack?  Wave-uniform, scalar only.
__device__ __forceinline__ bool lean_prescan(const int32_t* prog, int plen) {
    if (plen < 2) return false;
    int pc = 1, d = 0;
    while (pc < plen) {
        const uint32_t w = rd_word(prog + pc);
        const uint32_t op = w & 0xffu;
        if (op >= 64u) return false;
        const uint64_t b = 1ull << op;
        const int len = (kImmMask & b) ? ((w & PDEVAL_IMM_DD) ? 5 : 3) : 1;
        if (pc + len > plen) return false;
        if (kPushMask & b) {
            if (++d > 2) return false;
        } else if (kBinMask & b) {
            if (d < 2) return false;
            --d;
        } else if (kUnaryMask & b) {
            if (d < 1) return false;
        } else {
            return false;
        }
        pc += len;
    }
    return d == 1;
}

template <int K> struct Lean {
    using O = JetOps<double, K>;
    using J = typename O::J;
    static constexpr int NCJ = nc(K);

    static __device__ __forceinline__ void store(double* stk, int lane, const J& t) {
#pragma unroll
        for (int c = 0; c < NCJ; ++c) stk[c * 64 + lane] = t.c[c];
    }
    static __device__ __forceinline__ void load(const double* stk, int lane, J& t) {
#pragma unroll
        for (int c = 0; c < NCJ; ++c) t.c[c] = stk[c * 64 + lane];
    }

    // Evaluate a prescanned program at (x, y); inv_x = 1/x, inv_y = 1/y (as rcp() forms them).
    static __device__ __forceinline__ void run(const int32_t* prog, int plen, double x, double y,
                                               double inv_x, double inv_y, J& acc, double* stk,
                                               int lane) {
        int pc = 1;
        uint32_t w = rd_word(prog + 1);
        bool first = true;
        for (;;) {
            const uint32_t op = w & 0xffu;
            const bool has_imm = (kImmMask >> op) & 1u;
            const int npc = pc + (has_imm ? ((w & PDEVAL_IMM_DD) ? 5 : 3) : 1);
            const bool more = npc < plen;
            // the next opcode word is fetched before this op's arithmetic (its scalar-load
            // latency hides under it); the last op re-reads its own word
            const uint32_t wn = rd_word(prog + (more ? npc : pc));
            const int pn = (int)((w >> 8) & 0xffu);   // POWN exponent / coordinate power n
            const bool on_y = (w >> 16) & 1u;         // coordinate-power axis
            // dispatch: a tree of wave-uniform bit tests over opcode groups (most frequent
            // first), each a structured if/else -- a flat switch lowers to a compare tree whose
            // unstructured joins the structurizer turns into extra flow masks and copies
            const uint64_t b = 1ull << op;
            if (b & kPushMask) {
                if (!first) store(stk, lane, acc);
                if (op == PDOP_PUSH_X) {
                    O::set_var(acc, x, 0);
                } else if (op == PDOP_PUSH_P) {
                    double pk[K + 1];
                    if (on_y) {
                        O::pcoefs(y, pn, pk);
                        O::template set_p<1>(acc, pk);
                    } else {
                        O::pcoefs(x, pn, pk);
                        O::template set_p<0>(acc, pk);
                    }
                } else if (op == PDOP_PUSH_Y) {
                    O::set_var(acc, y, 1);
                } else {
                    O::set_const(acc, rd_imm(prog + pc + 1));
                }
            } else if (b & kCheapMask) {
                if (op == PDOP_ADDC) {
                    acc.c[0] = acc.c[0] + rd_imm(prog + pc + 1);
                } else if (op == PDOP_NEG) {
                    O::scale(acc, -1.0);
                } else if (op == PDOP_MULC) {
                    O::scale(acc, rd_imm(prog + pc + 1));
                } else if (op == PDOP_ADD_X) {
                    acc.c[0] = acc.c[0] + x;
                    acc.c[ji(1, 0)] = acc.c[ji(1, 0)] + 1.0;
                } else if (op == PDOP_SUB_X) {
                    acc.c[0] = acc.c[0] + (-x);
                    acc.c[ji(1, 0)] = acc.c[ji(1, 0)] + (-1.0);
                } else if (op == PDOP_ADD_Y) {
                    acc.c[0] = acc.c[0] + y;
                    acc.c[ji(0, 1)] = acc.c[ji(0, 1)] + 1.0;
                } else {
                    acc.c[0] = acc.c[0] + (-y);
                    acc.c[ji(0, 1)] = acc.c[ji(0, 1)] + (-1.0);
                }
            } else if (b & kPOpMask) {
                double pk[K + 1];
                if (on_y) {
                    O::pcoefs(y, pn, pk);
                    O::template p_op<1>(op, acc, pk);
                } else {
                    O::pcoefs(x, pn, pk);
                    O::template p_op<0>(op, acc, pk);
                }
            } else if (b & kBinMask) {
                J l;
                load(stk, lane, l);
                if (op == PDOP_DIV) O::div(l, acc);
                else if (op == PDOP_SUB) O::sub(l, acc);
                else if (op == PDOP_ADD) O::add(l, acc);
                else if (op == PDOP_MUL) O::mul(l, acc);
                else if (op == PDOP_RDIV) O::rdiv(l, acc);
                else O::rsub(l, acc);
            } else if (b & kVarMask) {
                if (op == PDOP_DIV_Y) div_var(acc, y, inv_y, 1);
                else if (op == PDOP_MUL_X) O::mul_var(acc, x, 0);
                else if (op == PDOP_DIV_X) div_var(acc, x, inv_x, 0);
                else O::mul_var(acc, y, 1);
            } else {
                if (op == PDOP_EXP) O::expj(acc);
                else if (op == PDOP_POW) O::powa(acc, rd_imm(prog + pc + 1));
                else if (op == PDOP_RDIVC) O::rdivc(acc, rd_imm(prog + pc + 1));
                else if (op == PDOP_SQRT) O::sqrtj(acc);
                else if (op == PDOP_LOG) O::logj(acc);
                else if (op == PDOP_POWN) O::pown(acc, pn);
                else absj<K>(acc);
            }
            if (!more) break;
            first = false;
            pc = npc;
            w = wn;
        }
    }

    // JetOps::div_var with the reciprocal supplied (identical arithmetic: qdiv(s, v, 1/v))
    static __device__ __forceinline__ void div_var(J& t, double v, double inv, int axis) {
#pragma unroll
        for (int d = 0; d <= K; ++d) {
#pragma unroll
            for (int j = 0; j <= d; ++j) {
                const int i = d - j;
                double s = t.c[ji(i, j)];
                if (axis == 0 && i > 0) s = s - t.c[ji(i - 1, j)];
                if (axis == 1 && j > 0) s = s - t.c[ji(i, j - 1)];
                t.c[ji(i, j)] = qdiv(s, v, inv);
            }
        }
    }
};

// Class and escalation of one candidate from its grid counts (lane 0; shared with
// validate_kernel's epilogue, whose logic it restates for the point-decided case).
__device__ __forceinline__ void grid_finish(const KernelArgs& a, int64_t cand, uint32_t hdr, int prob,
                                            bool point_reject, double qmax, int nbad, int nfin,
                                            int nnonfin, bool any_grad) {
    int cls;
    uint32_t esc = 0;
    const bool structural = (prob != PDEVAL_PROBLEM_FORCE_FREE) || (hdr & PDEVAL_FLAG_NOCOORD);
    if (!any_grad && nfin > 0 && structural) cls = PDEVAL_CLS_ZERO_GRADIENT;
    else if (point_reject) cls = PDEVAL_CLS_REJECT_POINT;   // decided by the point stage: final
    else if (nbad > a.prm.max_bad) {
        cls = PDEVAL_CLS_REJECT_GRID;
        esc = ESC_GRID_EVAL | ESC_GRID_FAIL;
    } else if (prob == PDEVAL_PROBLEM_FORCE_FREE && a.prm.strict_symbolic && (hdr & PDEVAL_FLAG_NONSMOOTH2D)) {
        cls = PDEVAL_CLS_REJECT_SYMBOLIC;
    } else {
        cls = PDEVAL_CLS_ACCEPT;
    }
    if (esc && a.esc_list) {
        esc |= (any_grad ? ESC_ANY_GRAD : 0u) | (nfin > 0 ? ESC_NFIN : 0u);
        list_append(a.esc_list, a.esc_count, a.list_capacity, cand | ((int64_t)esc << PD_ESC_SHIFT));
    }
    if (a.out.status) a.out.status[cand] = (uint8_t)cls;
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

#ifndef PD_GRID_WAVES_PER_SIMD
#define PD_GRID_WAVES_PER_SIMD 4
#endif
// One wave per candidate, 4 per 256-thread block; a.defer_list takes stack-3+ programs (pass 2),
// a.slow_list what the lean path does not take (drained by the generic kernel).
template <int PROB>
__global__ __launch_bounds__(256, PD_GRID_WAVES_PER_SIMD) void grid_kernel(KernelArgs a, int64_t* slow_list,
                                                                          int32_t* slow_count) {
    constexpr int K = (PROB == PDEVAL_PROBLEM_FORCE_FREE) ? 4 : 2;
    using L = Lean<K>;
    using J = typename L::J;
    const int lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifndef PD_HOST_SIM
    extern __shared__ __align__(16) unsigned char pd_lds[];
#else
    static unsigned char pd_lds[1];
#endif
    double* stk = reinterpret_cast<double*>(pd_lds) + (size_t)wib * nc(K) * 64;
    const int64_t cand = (int64_t)blockIdx.x * (blockDim.x >> 6) + wib;
    if (cand >= a.n) return;
    const int64_t beg = a.offsets[cand], end = a.offsets[cand + 1];
    const bool in_bounds = beg >= 0 && end > beg && end <= a.n_words && end - beg < (1 << 24);
    const int32_t* prog = a.ops + (in_bounds ? beg : 0);
    const int plen = __builtin_amdgcn_readfirstlane(in_bounds ? (int)(end - beg) : 0);
    const uint32_t hdr = in_bounds ? rd_word(prog) : 0xffu;
    const uint8_t ps = (uint8_t)__builtin_amdgcn_readfirstlane((int)a.pstate[cand]);
    if (ps & P0_CPLX) return;                                    // the complex passes take it
    if ((ps & 3) == P0_REJECT && !a.prm.full_grid) return;      // final after the point stage
    bool slow = !in_bounds || (hdr & 0xffu) != 0u || (ps & 3) == P0_NONE || (hdr & PDEVAL_FLAG_COMPLEX);
    if (!slow && (int)((hdr >> 8) & 0xffu) > 2) {
        if (lane == 0) list_append(a.defer_list, a.defer_count, a.list_capacity, cand);
        return;
    }
    if (!slow) slow = !lean_prescan(prog, plen);
    if (slow) {
        if (lane == 0) list_append(slow_list, slow_count, a.list_capacity, cand);
        return;
    }
    const int per_row = a.ny >> 6;
    const double y0 = a.gy[lane];
    const double inv_y0 = rcp(y0);
    double qmax = 0.0;
    int nbad = 0, nfin = 0;
    bool grad_nz = (ps & P0_GRAD) != 0;
    for (int row = 0; row < a.nx; ++row) {
        const double x = rd_sf64(a.gx + row);
        const double inv_x = rcp(x);
        for (int sl = 0; sl < per_row; ++sl) {
            const double y = per_row == 1 ? y0 : a.gy[sl * 64 + lane];
            const double inv_y = per_row == 1 ? inv_y0 : rcp(y);
            const int base = a.n_ref + row * a.ny + sl * 64;   // point index of lane 0
            J u;
            L::run(prog, plen, x, y, inv_x, inv_y, u, stk, lane);
            PointResult r;
            if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE) r = ff_epilogue<double>(u.c, x);
            else r = kerr_epilogue<double>(u.c, a.kc + 4 * (base + lane));
            const double qv = scaled(r.res_abs, r.scale);
            if (a.out.fingerprint) {
#pragma unroll
                for (int f = 0; f < PDEVAL_FP_N; ++f) {
                    const int rel = a.fp_pts[f] - base;   // uniform
                    if (rel >= 0 && rel < 64 && lane == rel) a.out.fingerprint[cand * PDEVAL_FP_N + f] = u.c[0];
                }
            }
            if (r.finite) {
                qmax = fmax(qmax, qv);
                if (!r.grad_zero) grad_nz = true;
            }
            nfin += (int)__popcll(__ballot(r.finite));
            nbad += (int)__popcll(__ballot(r.finite && qv > a.prm.tau_grid));
        }
    }
    qmax = wave_max(qmax);
    const bool any_grad = __any(grad_nz);
    if (lane == 0)
        grid_finish(a, cand, hdr, PROB, (ps & 3) == P0_REJECT, qmax, nbad, nfin, a.nx * a.ny - nfin, any_grad);
}

}  // namespace pd
