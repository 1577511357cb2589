// The lean grid pass (pass 1): the 64 x 64 grid of every candidate the point stage decided, for
// real programs whose operand stack fits 2 jets (99 % of the force-free depth-4 stream).
//
// Same arithmetic as validate_kernel<PROB, double, 2, ...> -- the same JetOps calls in the same
// order, so every residual is bit-identical -- but laid out for the CDNA issue model rather than
// as one generic kernel:
//  * the program is checked and decoded ONCE per candidate (decode_kernel: opcodes, immediates
//    in bounds, stack depth, ends at depth 1; instruction lengths, dispatch groups and problem
//    constants resolved) instead of at every opcode of every grid row; the interpreter then
//    runs with no bounds checks and no stack-depth bookkeeping (the stack is one LDS slot:
//    every push after the first spills the accumulator there, every binary op reads it back);
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

// Pass 2's register operand slot (Lean::RSLOT): Kerr pass 2 21.4 -> 18.3 ms, force-free
// 2.26 -> 2.10 ms (profiles/r03_ab1_*.log; 0 builds the variant without it).  Peephole
// superinstructions tested on every opcode (PUSH_C+MUL_P, any op + MULC / ADDC in one
// dispatch) were measured slower on the same box (pass 1 83.5 vs 77.6 ms force-free, 40.6 vs
// 38.8 ms Kerr) and removed; the PUSH_C + MUL fusion that survives is done by the decode pass
// into the push group (PD_FUSE_PUSHC), at no cost to other opcodes.
#ifndef PD_LEAN_RSLOT
#define PD_LEAN_RSLOT 1
#endif

constexpr uint64_t op_bit(int op) { return 1ull << op; }
constexpr int PTAB_N = 17;   // coordinate-power tables: 0 <= n <= 16 (the compilers emit 2 <= n <= 16)
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

// ---- pre-decoded programs.  The lean interpreter's per-opcode scalar work -- instruction
// length (immediate? double-double?), the next word's address, "was that the last opcode",
// the dispatch-group tests, the problem-constant lookup of an immediate -- is the same for
// every grid row of a candidate.  decode_kernel does it once per candidate, before pass 1, into
// a word array laid out like the programs (same offsets, n_words long):
//   at the header position     0 and the program's true stack depth in bits 8-15, or 0xff if
//                              the lean passes cannot take it (lean_prescan<3> fails)
//   at each opcode position    op (bits 0-7), the word's own bits 8-16 (POWN / coordinate power
//                              n, axis), the dispatch group (17-19), last-opcode bit (20), the
//                              distance to the next opcode (21-25: 1, 3 or 5, more after folded
//                              NEGs, up to 31 over a hoisted segment), and the dispatch group
//                              again as one bit of 26-31 (PD_ONEHOT: one bit test each)
//   after an immediate opcode  the immediate as a double (low word first), a problem constant
//                              (PDEVAL_IMM_PRM) already resolved to the grid stage's value
// The lean passes then read only the decoded array.
enum : uint32_t { DG_PUSH = 0, DG_CHEAP = 1, DG_POP = 2, DG_BIN = 3, DG_VAR = 4, DG_OTHER = 5 };
constexpr int DEC_DIST = 21;          // distance field: bits 21-25
constexpr uint32_t DEC_DIST_MAX = 31u;
constexpr int DEC_ONEHOT = 26;        // one-hot group: bits 26-31
// decoded-only opcode: push the hoisted jet of a single-coordinate segment (PD_HOIST_SUB); its
// distance steps over the segment to the binary opcode that consumes it
constexpr uint32_t DOP_PUSH_H = 40u;
#ifndef PD_KERR_NOMIX
#define PD_KERR_NOMIX 1
#endif
#ifndef PD_FOLD_NEG
#define PD_FOLD_NEG 1
#endif
#ifndef PD_FUSE_PUSHC
#define PD_FUSE_PUSHC 1
#endif
__device__ __forceinline__ uint32_t dec_group(uint64_t b) {
    if (b & (kPushMask | op_bit(PDOP_PUSH_I) | op_bit((int)DOP_PUSH_H))) return DG_PUSH;
    if (b & kCheapMask) return DG_CHEAP;
    if (b & kPOpMask) return DG_POP;
    if (b & kBinMask) return DG_BIN;
    if (b & kVarMask) return DG_VAR;
    return DG_OTHER;
}

// decode_kernel's sign folding, simulated: true when no folded sign reaches EXP / LOG / SQRT /
// POW (the programs that can drop every NEG).  Malformed programs return true; the decoder
// rejects them itself.
__device__ __forceinline__ bool neg_fold_ok(const int32_t* prog, int plen) {
    int sg[5] = {1, 1, 1, 1, 1};
    int d = 0;
    for (int pc = 1; pc < plen;) {
        const uint32_t w = (uint32_t)prog[pc];
        const uint32_t op = w & 0xffu;
        if (op >= 64u) return true;
        const uint64_t b = 1ull << op;
        if ((kPushMask | op_bit(PDOP_PUSH_I)) & b) {
            if (++d > 3) return true;
            sg[d] = 1;
        } else if (kBinMask & b) {
            if (d < 2) return true;
            --d;
            const int sl = sg[d], sa = sg[d + 1];
            if (op == PDOP_MUL || op == PDOP_DIV || op == PDOP_RDIV) sg[d] = sl * sa;
            else if (sl == sa) sg[d] = sa;
            else sg[d] = op == PDOP_ADD ? 1 : (op == PDOP_SUB ? sl : sa);
        } else if (d >= 1) {
            if (op == PDOP_NEG) sg[d] = -sg[d];
            else if (op == PDOP_ABS || (op == PDOP_POWN && !(((w >> 8) & 0xffu) & 1u))) sg[d] = 1;
            else if ((op == PDOP_EXP || op == PDOP_LOG || op == PDOP_SQRT || op == PDOP_POW) && sg[d] < 0)
                return false;
        }
        pc += (kImmMask & b) ? ((w & PDEVAL_IMM_DD) ? 5 : 3) : 1;
    }
    return true;
}

// ---- single-coordinate prefixes (PD_HOIST).  A program whose first opcodes compute a value of x alone
// (u = exp(rho) * z: PUSH_X EXP | PUSH_Y MUL) computes the same jet at every lane of a grid row:
// the lean passes evaluate that prefix once per candidate for all rows at once (one row per
// lane), keep the jets in a per-candidate buffer and start every row's run after it.  A prefix
// of y alone (u = sqrt(z + 1) * rho) is the same at every row: evaluated once at the lanes'
// ordinates.  The decoder records the longest prefix of one coordinate ending at stack depth 1
// in bits 17-30 of the header word (the position of the first opcode after it; 0 = none) and
// bit 31 (1: a prefix of y), when it holds a heavy opcode.
#ifndef PD_HOIST
#define PD_HOIST 1
#endif
// single-coordinate segments (a right operand: the PUSH_Y SQRT of PUSH_X EXP PUSH_Y SQRT MUL)
// hoisted the same way, as a push of the stored jet inside the row loop -- Kerr only: same box,
// 2^21, Kerr 25.38 -> 26.04 M cand/s, but force-free 13.43 -> 13.29 (the push's code in its
// interpreter cost more than the segments saved; profiles/r05_p_ab_*.log)
#ifndef PD_HOIST_SUB
#define PD_HOIST_SUB 1
#endif
template <int PROB> constexpr bool hoist_sub() { return PD_HOIST_SUB && PROB != PDEVAL_PROBLEM_FORCE_FREE; }
constexpr uint64_t kHeavyMask = op_bit(PDOP_MUL) | op_bit(PDOP_DIV) | op_bit(PDOP_RDIV) | op_bit(PDOP_RDIVC) |
                                op_bit(PDOP_POWN) | op_bit(PDOP_POW) | op_bit(PDOP_SQRT) | op_bit(PDOP_EXP) |
                                op_bit(PDOP_LOG) | op_bit(PDOP_MUL_P) | op_bit(PDOP_DIV_P) | op_bit(PDOP_RDIV_P) |
                                op_bit(PDOP_DIV_X);
__device__ __forceinline__ void hoist_track(int d, const uint32_t (&msk)[5], int pc, bool heavy, bool& alive,
                                            int& hoist_last, bool& hoist_heavy, bool& hoist_y) {
    if (!alive || d != 1) return;
    if ((msk[1] & 4u) || msk[1] == 3u) {   // both coordinates, or the imaginary unit
        alive = false;
        return;
    }
    hoist_last = pc;
    hoist_heavy = heavy;
    hoist_y = msk[1] == 2u;
}

template <int PROB>
__global__ __launch_bounds__(256) void decode_kernel(KernelArgs a) {
    const int64_t cand = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cand >= a.n) return;
    const int64_t beg = a.offsets[cand], end = a.offsets[cand + 1];
    if (!(beg >= 0 && end > beg && end <= a.n_words && end - beg < (1 << 24))) return;   // slow path
    const int32_t* prog = a.ops + beg;
    int32_t* dec = a.dec + beg;
    const int plen = (int)(end - beg);
    const uint32_t hdr = (uint32_t)prog[0];
    bool ok = plen >= 2 && (hdr & 0xffu) == 0u;   // (COMPLEX programs: the lean complex pass)
    int pc = 1, d = 0, dmax = 0, last = -1;
    int sg[5] = {1, 1, 1, 1, 1};   // PD_FOLD_NEG: sign of the value at each stack depth (1-based)
    // PD_HOIST: which coordinates the value at each stack depth depends on (bit 0 x, bit 1 y,
    // bit 2 the imaginary unit), and the longest prefix of one coordinate that ends at depth 1
    // (its last visited opcode, whether it holds a heavy opcode, whether it is of y)
    uint32_t msk[5] = {0u, 0u, 0u, 0u, 0u};
    int hoist_last = -1;
    bool hoist_alive = true, heavy = false, hoist_heavy = false, hoist_y = false;
    // PD_HOIST_SUB: the depth-2 segments (a push from depth 1 to the binary opcode back to 1)
    // whose value depends on one coordinate alone and that hold a heavy opcode
    int seg_start = -1, seg_nh = 0, nseg = 0;
    int sg_hs[4] = {0, 0, 0, 0}, sg_he[4] = {0, 0, 0, 0}, sg_nh[4] = {0, 0, 0, 0};
    bool sg_y[4] = {false, false, false, false};
    const bool fold = PD_FOLD_NEG && ok && neg_fold_ok(prog, plen);
    while (ok && pc < plen) {
        const uint32_t w = (uint32_t)prog[pc];
        const uint32_t op = w & 0xffu;
        if (op >= 64u) { ok = false; break; }
        const uint64_t b = 1ull << op;
        const int len = (kImmMask & b) ? ((w & PDEVAL_IMM_DD) ? 5 : 3) : 1;
        if (pc + len > plen) { ok = false; break; }
        if (op == PDOP_POWN && ((w >> 8) & 0xffu) > 8u) { ok = false; break; }   // (pown_lean)
        // coordinate powers come from the power tables (ptab_kernel): 2 <= n < PTAB_N
        if ((kPOpMask | op_bit(PDOP_PUSH_P)) & b) {
            const uint32_t pn = (w >> 8) & 0xffu;
            if (pn < 2u || pn >= (uint32_t)PTAB_N) { ok = false; break; }
        }
        if ((kPushMask | op_bit(PDOP_PUSH_I)) & b) {
            if (++d > 3) { ok = false; break; }
            dmax = max(dmax, d);
        } else if (kBinMask & b) {
            if (d < 2) { ok = false; break; }
            --d;
        } else if (kUnaryMask & b) {
            if (d < 1) { ok = false; break; }
        } else {
            ok = false;
            break;
        }
        if (kImmMask & b) {
            double v;
            if (w & PDEVAL_IMM_PRM) {
                const uint32_t desc = (uint32_t)prog[pc + 1];
                if (op == PDOP_POW || (w & PDEVAL_IMM_DD) || desc > 15u) { ok = false; break; }
                v = prm_value(a.prm_grid, desc);
            } else {
                v = __hiloint2double(prog[pc + 2], prog[pc + 1]);
            }
            dec[pc + 1] = __double2loint(v);
            dec[pc + 2] = __double2hiint(v);
        }
        // Kerr: PUSH_C c followed by MUL_X / MUL_Y / MUL_P (c x, c y, c x^n: 1.9 of its 13.4
        // opcodes per depth-4 candidate; force-free has 0.14) decode into one push: the second opcode with the
        // PUSH group, c as its immediate, the distance over both.  The interpreter runs the
        // same two JetOps calls (set_const, then the multiply), so the values are the same.
        if (PD_FUSE_PUSHC && PROB != PDEVAL_PROBLEM_FORCE_FREE && op == PDOP_PUSH_C && pc + len < plen) {
            const uint32_t w2 = (uint32_t)prog[pc + len];
            const uint32_t op2 = w2 & 0xffu;
            if (op2 == PDOP_MUL_X || op2 == PDOP_MUL_Y || (PD_FUSE_PUSHC == 1 && op2 == PDOP_MUL_P)) {
                dec[pc] = (int32_t)(op2 | (w2 & 0x1ff00u) | (DG_PUSH << 17) | ((uint32_t)(len + 1) << DEC_DIST) |
                                    (1u << (DEC_ONEHOT + DG_PUSH)));
                sg[d] = 1;
                msk[d] = (op2 == PDOP_MUL_Y || (op2 == PDOP_MUL_P && ((w2 >> 16) & 1u))) ? 2u : 1u;
                if (d == 2) {
                    seg_start = pc;
                    seg_nh = 0;
                }
                hoist_track(d, msk, pc, heavy, hoist_alive, hoist_last, hoist_heavy, hoist_y);
                last = pc;
                pc += len + 1;
                continue;
            }
        }
        // Negations folded into the program (PD_FOLD_NEG): NEG flips the sign of the value
        // at the top of the stack instead of negating 15 (Kerr: 6) coefficients, and the
        // opcodes that follow absorb it -- s*a + c = s*(a + s*c) (ADDC with s*c; ADD_X <->
        // SUB_X, ADD_P <-> SUB_P), products and quotients carry it (MULC, MUL_X, DIV_Y, MUL_P,
        // RDIVC, MUL, DIV, ...: s1*s2), a sum of two signed operands picks ADD / SUB / RSUB and
        // a sign, an even POWN or ABS clears it.  Negation is exact and every rounding is
        // symmetric, so each coefficient is the one the program computes, up to the tracked
        // sign.  Programs in which a folded sign would reach an opcode that needs the value
        // itself (EXP, LOG, SQRT, POW) keep their NEGs (neg_fold_ok).  What is left at the end
        // is bit 16 of the header word: the force-free determinant is even in u and Kerr's
        // |L[u]| and scale are unchanged under u -> -u, so only the fingerprint (linear in u)
        // reads it.
        uint32_t dop = op;
        if (fold) {
            if (op == PDOP_NEG) {
                const uint32_t pw = last >= 0 ? (uint32_t)dec[last] : 0u;
                if (last >= 0 && ((pw >> DEC_DIST) & DEC_DIST_MAX) + 1u <= DEC_DIST_MAX) {
                    sg[d] = -sg[d];
                    dec[last] = (int32_t)(pw + (1u << DEC_DIST));   // the previous opcode steps over it
                    pc += 1;
                    continue;
                }
            } else if ((kPushMask | op_bit(PDOP_PUSH_I)) & b) {
                sg[d] = 1;
            } else if (kBinMask & b) {
                const int sl = sg[d], sa = sg[d + 1];   // operands at depths d (lhs) and d + 1
                if (op == PDOP_MUL || op == PDOP_DIV || op == PDOP_RDIV) {
                    sg[d] = sl * sa;
                } else if (sl == sa) {
                    sg[d] = sa;                          // s*(l op a)
                } else if (op == PDOP_ADD) {             // l - a or a - l
                    dop = sl > 0 ? PDOP_SUB : PDOP_RSUB;
                    sg[d] = 1;
                } else if (op == PDOP_SUB) {             // sl*l - sa*a
                    dop = PDOP_ADD;
                    sg[d] = sl;
                } else {                                 // RSUB: sa*a - sl*l
                    dop = PDOP_ADD;
                    sg[d] = sa;
                }
            } else if (sg[d] < 0) {
                if (op == PDOP_ADDC) {
                    const double v = -__hiloint2double(dec[pc + 2], dec[pc + 1]);
                    dec[pc + 1] = __double2loint(v);
                    dec[pc + 2] = __double2hiint(v);
                } else if (op == PDOP_ADD_X) {
                    dop = PDOP_SUB_X;
                } else if (op == PDOP_SUB_X) {
                    dop = PDOP_ADD_X;
                } else if (op == PDOP_ADD_Y) {
                    dop = PDOP_SUB_Y;
                } else if (op == PDOP_SUB_Y) {
                    dop = PDOP_ADD_Y;
                } else if (op == PDOP_ADD_P) {
                    dop = PDOP_SUB_P;
                } else if (op == PDOP_SUB_P) {
                    dop = PDOP_ADD_P;
                } else if (op == PDOP_ABS || (op == PDOP_POWN && !(((w >> 8) & 0xffu) & 1u))) {
                    sg[d] = 1;
                } else if (op == PDOP_EXP || op == PDOP_LOG || op == PDOP_SQRT || op == PDOP_POW) {
                    ok = false;   // (neg_fold_ok rules this out; the generic pass takes it)
                    break;
                }
            }
        }
        dec[pc] = (int32_t)(dop | (w & 0x1ff00u & ((kImmMask & b) ? 0u : ~0u)) | (dec_group(op_bit((int)dop)) << 17) |
                            ((uint32_t)len << DEC_DIST) | (1u << (DEC_ONEHOT + dec_group(op_bit((int)dop)))));
        // (masks follow the original opcode: a folded sign does not change what it depends on)
        if ((kPushMask | op_bit(PDOP_PUSH_I)) & b) {
            msk[d] = op == PDOP_PUSH_X ? 1u : op == PDOP_PUSH_Y ? 2u : op == PDOP_PUSH_I ? 4u
                   : op == PDOP_PUSH_P ? (((w >> 16) & 1u) ? 2u : 1u) : 0u;
            if (d == 2) {
                seg_start = pc;
                seg_nh = 0;
            }
        } else if (kBinMask & b) {
            if (d == 1 && seg_start >= 0) {   // a depth-2 segment closes here
                const uint32_t m2 = msk[2];
                if (seg_nh > 0 && (m2 == 0u || m2 == 1u || m2 == 2u) && pc - seg_start <= (int)DEC_DIST_MAX &&
                    nseg < 4) {
                    sg_hs[nseg] = seg_start;
                    sg_he[nseg] = pc;
                    sg_nh[nseg] = seg_nh;
                    sg_y[nseg] = m2 == 2u;
                    ++nseg;
                }
                seg_start = -1;
            }
            msk[d] |= msk[d + 1];
        } else if ((kPOpMask & b) || op == PDOP_ADD_X || op == PDOP_SUB_X || op == PDOP_MUL_X ||
                   op == PDOP_DIV_X || op == PDOP_ADD_Y || op == PDOP_SUB_Y || op == PDOP_MUL_Y ||
                   op == PDOP_DIV_Y) {
            const bool on_y = (kPOpMask & b) ? ((w >> 16) & 1u) != 0u
                                             : (op == PDOP_ADD_Y || op == PDOP_SUB_Y || op == PDOP_MUL_Y || op == PDOP_DIV_Y);
            msk[d] |= on_y ? 2u : 1u;
        }
        heavy = heavy || (kHeavyMask & b);
        if (d >= 2 && (kHeavyMask & b)) ++seg_nh;
        hoist_track(d, msk, pc, heavy, hoist_alive, hoist_last, hoist_heavy, hoist_y);
        last = pc;
        pc += len;
    }
    ok = ok && d == 1 && last >= 0;
    if (ok) dec[last] |= (int32_t)(1u << 20);
    // the hoisted prefix: the position of the first opcode after it (its last opcode's distance
    // is final now -- a folded NEG after it extends that distance), or 0 for none
    uint32_t hp = 0u;
    if (PD_HOIST && ok && hoist_last >= 0 && hoist_heavy) {
        const uint32_t at = (uint32_t)hoist_last + (((uint32_t)dec[hoist_last] >> DEC_DIST) & DEC_DIST_MAX);
        if (at < (uint32_t)plen && at < (1u << 14)) hp = at;   // (not a whole program of x alone)
    }
    dec[0] = ok ? (int32_t)(((uint32_t)dmax << 8) | (sg[1] < 0 ? 1u << 16 : 0u) | (hp << 17) |
                            (hp && hoist_y ? 1u << 31 : 0u)) : (int32_t)0xff;
    // the hoisted segment: the heaviest one after the prefix (force-free: x alone), its first
    // opcode word replaced by DOP_PUSH_H, the original kept in a.hseg with its span and kind
    if (a.hseg) {
        int best = -1;
        // (not for the complex pass's candidates: the complex interpreter hoists nothing)
        const bool cplx = (hdr & PDEVAL_FLAG_COMPLEX) || (a.pstate && (a.pstate[cand] & P0_CPLX));
        if (hoist_sub<PROB>() && ok && !cplx)
            for (int k = 0; k < nseg; ++k)
                if (sg_hs[k] >= (int)hp && (!sg_y[k] || (PROB != PDEVAL_PROBLEM_FORCE_FREE && a.ny == 64)) &&
                    (best < 0 || sg_nh[k] > sg_nh[best]))
                    best = k;
        int32_t* hs = a.hseg + 4 * cand;
        if (best >= 0) {
            const int at = sg_hs[best], to = sg_he[best];
            hs[0] = dec[at];
            hs[1] = at;
            hs[2] = to;
            hs[3] = sg_y[best] ? 1 : 0;
            dec[at] = (int32_t)(DOP_PUSH_H | (DG_PUSH << 17) | ((uint32_t)(to - at) << DEC_DIST) |
                                (1u << (DEC_ONEHOT + DG_PUSH)));
        } else {
            hs[1] = 0;
        }
    }
}

// ---- coordinate-power tables.  A coordinate power v**n (PDOP_*_P) enters the interpreter as
// the univariate jet p_k = C(n,k) v^(n-k), k <= K (JetOps::pcoefs): per opcode and grid row,
// a loop of n - K multiplications, K + 1 more, and the binomials by division.  The values
// depend only on (n, v), and v takes nx + ny values per context, so ptab_kernel evaluates
// JetOps::pcoefs once for every (n, grid abscissa) and (n, grid ordinate) -- the same function,
// so the interpreter reads bit-identical values -- and the lean passes load them:
//   x part  [n][row][k]   wave-uniform (one grid row per W slot): scalar loads
//   y part  [n][k][j]     lane j: one coalesced vector load per coefficient
template <int K> constexpr size_t ptab_doubles(int nx, int ny) { return (size_t)PTAB_N * (K + 1) * (size_t)(nx + ny); }
template <int K>
__global__ __launch_bounds__(256) void ptab_kernel(const double* gx, const double* gy, int nx, int ny, double* tab) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nxt = (int64_t)PTAB_N * nx;
    double pk[K + 1];
    if (t < nxt) {
        const int n = (int)(t / nx), i = (int)(t % nx);
        JetOps<double, K>::pcoefs(gx[i], n, pk);
#pragma unroll
        for (int k = 0; k <= K; ++k) tab[((size_t)n * nx + i) * (K + 1) + k] = pk[k];
    } else if (t < nxt + (int64_t)PTAB_N * ny) {
        const int64_t u = t - nxt;
        const int n = (int)(u / ny), j = (int)(u % ny);
        JetOps<double, K>::pcoefs(gy[j], n, pk);
        double* ty = tab + nxt * (K + 1);
#pragma unroll
        for (int k = 0; k <= K; ++k) ty[((size_t)n * (K + 1) + k) * ny + j] = pk[k];
    }
}
// PD_PTAB (force-free) / PD_PTAB_KERR: 1 = both tables, 2 = the x table only (the lane's y
// powers computed in place: a vector load of the y table is a dependent global-memory access
// per opcode), 0 = none.  Force-free pass 1, same box (profiles/r04_c_*): none 150.3 ms, both
// 151.7, x only 149.3; at 5 waves/SIMD (fewer VGPRs with the tables) x only 146.9, both 147.9,
// none 155.5 (96 B of spill).
#ifndef PD_PTAB
#define PD_PTAB 2
#endif
// Kerr at W = 3 rows per dispatch: no tables (the x powers formed in place, no scalar loads of
// the table per opcode) 47.4 -> 46.6 ms for pass 1, three alternations on one box, classes
// identical (profiles/r06_ae_*; x table only was the round-4 choice at W = 2)
#ifndef PD_PTAB_KERR
#define PD_PTAB_KERR 0
#endif
// Where a lane finds its coordinate-power coefficients: x rows px[q] (wave-uniform), the
// lane's ordinate py; strides per n: sx (x part), sy (y part), and ny between coefficients.
template <int W> struct PowTab {
    const double* px[W];
    const double* py;
    int sx, sy, ny;
};

// W sample points per lane (W grid rows per dispatch of one opcode): the opcode decode, the
// dispatch branches and the immediate loads are paid once for W jets.  Force-free runs W = 1
// (two 15-coefficient jets per operand would not fit 128 VGPRs); Kerr's 6-coefficient jets run
// W = 2.  For every point the arithmetic is the same JetOps sequence as at W = 1.
#ifndef PD_LEAN_IMM_PREFETCH
#define PD_LEAN_IMM_PREFETCH 1
#endif
#ifndef PD_PREFETCH_SELECT
#define PD_PREFETCH_SELECT 0
#endif
#ifndef PD_ONEHOT
#define PD_ONEHOT 1
#endif
// the force-free epilogue's 1/rho from the grid's reciprocal table (the value rcp() forms)
// instead of a division per row
#ifndef PD_EPI_TABLE_RCP
#define PD_EPI_TABLE_RCP 1
#endif
// the row's 1/x^2 and 1/x^3 moved into SGPRs (uniform_f64) rather than left in VGPRs: the pass-1
// spill drops from 64 to 32 B, but the same-box A/B (r04_w) measured no gain, so it stays off
// Kerr: the lean epilogue (kerr_epilogue_lean: the doubled coefficient table, one maximum for
// the coefficient tests)
#ifndef PD_KERR_LEAN
#define PD_KERR_LEAN 1
#endif
// the per-point scaled residual as a select, no branch (scaled_sel)
#ifndef PD_SCALED_SEL
#define PD_SCALED_SEL 1
#endif
// the division-free zero test (grid_fails: |res| > tau S) and the lane's maximum of q as a
// (|res|, S) pair divided once (GridMax), instead of q = |res| / S at every point
#ifndef PD_DIVFREE
#define PD_DIVFREE 1
#endif
// keep the lane's 1/y out of the row loop (pin_f64 above)
#ifndef PD_INVY_PIN
#define PD_INVY_PIN 1
#endif
#ifndef PD_EPI_UNIFORM
#define PD_EPI_UNIFORM 0
#endif
// the per-point scaled residual by reciprocal + Newton steps instead of an IEEE division
// (scaled_fast)
#ifndef PD_FAST_SCALED
#define PD_FAST_SCALED 0
#endif
#ifndef PD_LEAN_PTR
#define PD_LEAN_PTR 1
#endif
#ifndef PD_DISPATCH_FREQ
#define PD_DISPATCH_FREQ 1
#endif
#ifndef PD_PIN_Y
#define PD_PIN_Y 1
#endif
template <class T, int K, int W, int MAXD> struct Lean {
    using O = JetOps<T, K>;
    using J = typename O::J;
    static constexpr int NCJ = nc(K);

    // Kerr (K = 2): the mixed coefficient u_rx feeds only itself through every jet operation
    // and the operator has no mixed term (kerr_epilogue), so it is not stored, not loaded and
    // forced to 0 after each opcode; the compiler then drops its arithmetic (PD_KERR_NOMIX=0:
    // the full jets, an A/B variant -- same values of every other coefficient)
    static constexpr bool NOMIX = PD_KERR_NOMIX && K == 2;
    static constexpr int MIX = ji(1, 1);
    static __device__ __forceinline__ bool live(int c) { return !(NOMIX && c == MIX); }
    // LDS layout: the live coefficients only (Kerr: 5 of 6 -- an operand slot of W = 8 jets is
    // 20 KiB per wave instead of 24, which is what 8 waves per CU fit in 160 KiB)
#ifndef PD_LDS_COMPACT
#define PD_LDS_COMPACT 1
#endif
    static constexpr bool COMPACT = PD_LDS_COMPACT && NOMIX;
    static constexpr int NCL = NCJ - (COMPACT ? 1 : 0);
    static __device__ __forceinline__ constexpr int lidx(int c) { return COMPACT && c > MIX ? c - 1 : c; }
    static constexpr int SLOT = W * NCL * 64;   // T values per operand slot
    static constexpr bool RSLOT = PD_LEAN_RSLOT && MAXD == 3;   // operand slot 1 in registers (run below)
    static constexpr int LDS_SLOTS = RSLOT ? 1 : MAXD - 1;

    // LDS operand slot of one wave: [w][coef][lane]
    static __device__ __forceinline__ void store(T* stk, int lane, const J (&t)[W]) {
#pragma unroll
        for (int w = 0; w < W; ++w)
#pragma unroll
            for (int c = 0; c < NCJ; ++c)
                if (live(c)) stk[(w * NCL + lidx(c)) * 64 + lane] = t[w].c[c];
    }
    static __device__ __forceinline__ void load(const T* stk, int lane, J (&t)[W]) {
#pragma unroll
        for (int w = 0; w < W; ++w)
#pragma unroll
            for (int c = 0; c < NCJ; ++c) t[w].c[c] = live(c) ? stk[(w * NCL + lidx(c)) * 64 + lane] : zero<T>();
    }

    // Evaluate a decoded program (decode_kernel; `dec` at the program's header word) at
    // (x[w], y), w < W; inv_x = 1/x, inv_y = 1/y (as rcp() forms them).  x[] is wave-uniform
    // (one grid row each), y is the lane's ordinate.
    // coordinate-power coefficients of v**n at row slot q (x) or at the lane's ordinate (y)
    static constexpr int PTAB = K == 4 ? PD_PTAB : PD_PTAB_KERR;
    // XL: x differs per lane (the hoisted prefix, one grid row per lane): vector loads
    template <bool XL = false>
    static __device__ __forceinline__ void pco_x(const PowTab<W>& pt, const double (&x)[W], int q, int n, double* pk) {
        if constexpr (PTAB != 0) {
            const double* p = pt.px[q] + (size_t)n * pt.sx;
#pragma unroll
            for (int k = 0; k <= K; ++k) pk[k] = XL ? p[k] : rd_sf64(p + k);
        } else {
            O::pcoefs(x[q], n, pk);
        }
    }
    static __device__ __forceinline__ void pco_y(const PowTab<W>& pt, double y, int n, double* pk) {
        if constexpr (PTAB == 1) {
            const double* p = pt.py + (size_t)n * pt.sy;
#pragma unroll
            for (int k = 0; k <= K; ++k) pk[k] = p[(size_t)k * pt.ny];
        } else {
            O::pcoefs(y, n, pk);
        }
    }

    // pc0: the first opcode to run -- 1, or the position after a hoisted prefix (PD_HOIST), with
    // acc holding the prefix's value at stack depth 1.  PRE (XL: x per lane): stop before the
    // opcode at `stop` (the hoisted prefix alone).
    // h2 (PD_HOIST_SUB): the candidate's hoisted segment jet, [coefficient][row or lane]; its
    // DOP_PUSH_H pushes row h2row + q (clamped to h2last) or, h2y, the lane's own.  w0 / fresh:
    // the pre-phase of a segment starts at its first opcode with the original word w0 and an
    // empty stack.
    template <bool XL = false, bool PRE = false>
    static __device__ __forceinline__ void run(const int32_t* dec, const double (&x)[W], double y_in,
                                               const double (&inv_x)[W], double inv_y, J (&acc)[W],
                                               T* stk, int lane, const PowTab<W>& pt, int pc0 = 1,
                                               int stop = 0, const double* h2 = nullptr, int h2row = 0,
                                               int h2last = 0, bool h2y = false, uint32_t w0 = 0u,
                                               bool fresh = false) {
        // MAXD = 3 (pass 2): the upper of the two operand slots lives in VGPRs, the lower in
        // LDS -- two LDS slots of W = 2 Kerr jets (12 KiB per wave) held pass 2 at ~3 waves
        // per SIMD; with one, VGPRs set the occupancy
        J reg[RSLOT ? W : 1];
        // (PD_LEAN_PTR) the position as a pointer: the next word's address is one 64-bit add of
        // the scaled distance, not a sign extension, a shift and an add of an index per opcode
        const int32_t* cur = dec + pc0;
        int pc = pc0;
        // an opcode word and the two after it (its f64 immediate, when it has one) are read
        // together, one op ahead, so an op's immediate is in SGPRs when its turn comes instead
        // of costing a dependent scalar load (dec[] is padded by 4 words past its end)
        uint32_t w = w0 ? w0 : rd_word(dec + pc0);
        double imm = PD_LEAN_IMM_PREFETCH ? rd_imm(dec + pc0 + 1) : 0.0;
        bool first = fresh || pc0 == 1;
        int d = first ? 0 : 1;   // operand stack depth (wave-uniform); MAXD = 2 needs only `first`
        for (;;) {
            // (PD_PIN_Y) the lane's ordinate made opaque once per opcode: values derived from it
            // (the powers y^k of a coordinate power) are formed where an opcode uses them instead
            // of being hoisted out of the loop and kept live -- spilled to scratch -- through it
            // (force-free only: same box, pass 1 129.4 -> 125.4 ms and its scratch frame 96 -> 64
            // B/lane; Kerr's pass 1 went 48.5 -> 50.0 ms with it, profiles/r06_m_ab_*)
            double y = y_in;
            if constexpr (PD_PIN_Y && K == 4) pin_f64(y);
            const uint32_t op = w & 0xffu;
            const uint32_t grp = (w >> 17) & 7u;
            // group tests: a bit test on the one-hot copy (s_bitcmp + branch) or a compare of
            // the 3-bit field (extract + compare + branch)
            auto in_grp = [&](uint32_t g) -> bool {
                if constexpr (PD_ONEHOT) return (w >> (DEC_ONEHOT + g)) & 1u;
                else return grp == g;
            };
            const bool more = !((w >> 20) & 1u);
            const int npc = pc + (int)((w >> DEC_DIST) & DEC_DIST_MAX);
            // the next opcode word is fetched before this op's arithmetic (its scalar-load
            // latency hides under it); after the last op the three words past the program are
            // read and ignored -- they exist: the decoded array is padded by 4 words
            // (ensure_dec), so no select of the address is needed
#if PD_PREFETCH_SELECT   // (A/B: the round-3 form, re-reading its own word after the last op)
            const int pn_at = more ? npc : pc;
#else
            const int pn_at = npc;
#endif
            const int32_t* nxt = PD_LEAN_PTR && !PD_PREFETCH_SELECT ? cur + ((w >> DEC_DIST) & DEC_DIST_MAX) : dec + pn_at;
            const uint32_t wn = rd_word(nxt);
            const double immn = PD_LEAN_IMM_PREFETCH ? rd_imm(nxt + 1) : 0.0;
            const double cimm = PD_LEAN_IMM_PREFETCH ? imm : rd_imm(dec + pc + 1);
            const int pn = (int)((w >> 8) & 0xffu);   // POWN exponent / coordinate power n
            const bool on_y = (w >> 16) & 1u;         // coordinate-power axis
            // dispatch: the decoded group, then the opcode, each a structured if/else (a flat
            // switch lowers to a compare tree whose unstructured joins the structurizer turns
            // into extra flow masks and copies)
            if (in_grp(DG_PUSH)) {
                if (!first) {
                    if (RSLOT && d == 2) {
#pragma unroll
                        for (int q = 0; q < W; ++q) reg[q] = acc[q];
                    } else {
                        store(stk + (MAXD == 2 || RSLOT ? 0 : d - 1) * SLOT, lane, acc);
                    }
                }
                ++d;
                // a fused PUSH_C + MUL_X / MUL_Y / MUL_P of the decoder (Kerr), in closed form:
                // c (v + d_axis) is (c v, c along the axis, 0 elsewhere) and c P = (c p_k along
                // the axis) -- the values set_const + mul_var / mul_p compute (their other terms
                // are products with exact zeros), without the products by zero that the compiler
                // may not fold (0 * v is -0 or NaN for some v) and kept live across the loop,
                // which spilled 48 B per lane in round 3
                const bool fused = PD_FUSE_PUSHC && K == 2 &&
                                   (op == PDOP_MUL_X || op == PDOP_MUL_Y || (PD_FUSE_PUSHC == 1 && op == PDOP_MUL_P));
                auto fused_push = [&]() {
                    double pk[K + 1];
                    if (op == PDOP_MUL_P && on_y) pco_y(pt, y, pn, pk);
                    const T c = cvt<T>(cimm);
#pragma unroll
                    for (int q = 0; q < W; ++q) {
                        if (op == PDOP_MUL_X) {
                            O::set_const(acc[q], c * cvt<T>(x[q]));
                            acc[q].c[ji(1, 0)] = c;
                        } else if (op == PDOP_MUL_Y) {
                            O::set_const(acc[q], c * cvt<T>(y));
                            acc[q].c[ji(0, 1)] = c;
                        } else if (on_y) {
                            O::set_const(acc[q], c * cvt<T>(pk[0]));
#pragma unroll
                            for (int k = 1; k <= K; ++k) acc[q].c[ji(0, k)] = c * cvt<T>(pk[k]);
                        } else {
                            pco_x<XL>(pt, x, q, pn, pk);
                            O::set_const(acc[q], c * cvt<T>(pk[0]));
#pragma unroll
                            for (int k = 1; k <= K; ++k) acc[q].c[ji(k, 0)] = c * cvt<T>(pk[k]);
                        }
                    }
                };
                // (PD_DISPATCH_FREQ, Kerr: the fused push -- 1.5 of its 2.7 pushes per program --
                // is tested first; the interpreter is scalar-issue bound there)
                if (PD_DISPATCH_FREQ && K == 2 && fused) {
                    fused_push();
                } else if (op == PDOP_PUSH_X) {
#pragma unroll
                    for (int q = 0; q < W; ++q) O::set_var(acc[q], x[q], 0);
                } else if (op == PDOP_PUSH_P) {
                    double pk[K + 1];
                    if (on_y) {
                        pco_y(pt, y, pn, pk);
#pragma unroll
                        for (int q = 0; q < W; ++q) O::template set_p<1>(acc[q], pk);
                    } else {
#pragma unroll
                        for (int q = 0; q < W; ++q) {
                            pco_x<XL>(pt, x, q, pn, pk);
                            O::template set_p<0>(acc[q], pk);
                        }
                    }
                } else if (op == PDOP_PUSH_Y) {
#pragma unroll
                    for (int q = 0; q < W; ++q) O::set_var(acc[q], y, 1);
                } else if (!PD_DISPATCH_FREQ && fused) {
                    fused_push();
                } else if (Real<T>::cplx_pass && op == PDOP_PUSH_I) {
                    if constexpr (Real<T>::cplx_pass) {
#pragma unroll
                        for (int q = 0; q < W; ++q) O::set_const(acc[q], imag_unit<T>());
                    }
                } else if (!Real<T>::cplx_pass && PD_HOIST_SUB && K != 4 && op == DOP_PUSH_H) {
                    if constexpr (!Real<T>::cplx_pass && PD_HOIST_SUB && K != 4) {   // (Kerr only)
#pragma unroll
                        for (int q = 0; q < W; ++q) {
                            const int at = h2y ? lane : min(h2row + q, h2last);
#pragma unroll
                            for (int c = 0; c < NCJ; ++c) acc[q].c[c] = live(c) ? h2[c * 64 + at] : zero<T>();
                        }
                    }
                } else {
                    const double c = cimm;
#pragma unroll
                    for (int q = 0; q < W; ++q) O::set_const(acc[q], cvt<T>(c));
                }
            } else if (in_grp(DG_CHEAP)) {
                if (op == PDOP_ADDC) {
                    const double c = cimm;
#pragma unroll
                    for (int q = 0; q < W; ++q) acc[q].c[0] = acc[q].c[0] + cvt<T>(c);
                } else if (PD_DISPATCH_FREQ && K == 2 && op == PDOP_MULC) {   // (1.2 per Kerr program; NEG is folded)
                    const double c = cimm;
#pragma unroll
                    for (int q = 0; q < W; ++q) O::scale(acc[q], cvt<T>(c));
                } else if (op == PDOP_NEG) {
#pragma unroll
                    for (int q = 0; q < W; ++q) O::scale(acc[q], from_real<T>(-1.0));
                } else if (op == PDOP_MULC) {
                    const double c = cimm;
#pragma unroll
                    for (int q = 0; q < W; ++q) O::scale(acc[q], cvt<T>(c));
                } else if (op == PDOP_ADD_X) {
#pragma unroll
                    for (int q = 0; q < W; ++q) {
                        acc[q].c[0] = acc[q].c[0] + cvt<T>(x[q]);
                        acc[q].c[ji(1, 0)] = acc[q].c[ji(1, 0)] + from_real<T>(1.0);
                    }
                } else if (op == PDOP_SUB_X) {
#pragma unroll
                    for (int q = 0; q < W; ++q) {
                        acc[q].c[0] = acc[q].c[0] + cvt<T>(-x[q]);
                        acc[q].c[ji(1, 0)] = acc[q].c[ji(1, 0)] + from_real<T>(-1.0);
                    }
                } else if (op == PDOP_ADD_Y) {
#pragma unroll
                    for (int q = 0; q < W; ++q) {
                        acc[q].c[0] = acc[q].c[0] + cvt<T>(y);
                        acc[q].c[ji(0, 1)] = acc[q].c[ji(0, 1)] + from_real<T>(1.0);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < W; ++q) {
                        acc[q].c[0] = acc[q].c[0] + cvt<T>(-y);
                        acc[q].c[ji(0, 1)] = acc[q].c[ji(0, 1)] + from_real<T>(-1.0);
                    }
                }
            } else if (in_grp(DG_POP)) {
                double pk[K + 1];
                if (on_y) {
                    pco_y(pt, y, pn, pk);
#pragma unroll
                    for (int q = 0; q < W; ++q) O::template p_op<1>(op, acc[q], pk);
                } else {
#pragma unroll
                    for (int q = 0; q < W; ++q) {
                        pco_x<XL>(pt, x, q, pn, pk);
                        O::template p_op<0>(op, acc[q], pk);
                    }
                }
            } else if (in_grp(DG_BIN)) {
                const T* src = stk + (MAXD == 2 || RSLOT ? 0 : d - 2) * SLOT;
                const bool from_reg = RSLOT && d == 3;
                --d;
                // one operand jet at a time: W > 2 would not hold W operand jets beside the
                // W accumulators in registers
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    J l;
                    if (from_reg) {
                        l = reg[RSLOT ? q : 0];
                    } else {
#pragma unroll
                        for (int c = 0; c < NCJ; ++c) l.c[c] = live(c) ? src[(q * NCL + lidx(c)) * 64 + lane] : zero<T>();
                    }
                    if (op == PDOP_DIV) O::div(l, acc[q]);
                    else if (op == PDOP_SUB) O::sub(l, acc[q]);
                    else if (op == PDOP_ADD) O::add(l, acc[q]);
                    else if (op == PDOP_MUL) O::mul(l, acc[q]);
                    else if (op == PDOP_RDIV) O::rdiv(l, acc[q]);
                    else O::rsub(l, acc[q]);
                }
            } else if (in_grp(DG_VAR)) {
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    if (op == PDOP_DIV_Y) div_var(acc[q], y, inv_y, 1);
                    else if (op == PDOP_MUL_X) O::mul_var(acc[q], x[q], 0);
                    else if (op == PDOP_DIV_X) div_var(acc[q], x[q], inv_x[q], 0);
                    else O::mul_var(acc[q], y, 1);
                }
            } else {
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    if (op == PDOP_EXP) O::expj(acc[q]);
                    else if (op == PDOP_POW) O::powa(acc[q], cimm);
                    else if (op == PDOP_RDIVC) O::rdivc(acc[q], cvt<T>(cimm));
                    else if (op == PDOP_SQRT) O::sqrtj(acc[q]);
                    else if (op == PDOP_LOG) O::logj(acc[q]);
                    else if (op == PDOP_POWN) pown_lean(acc[q], pn);
                    else absj<K>(acc[q]);
                }
            }
            if constexpr (NOMIX) {
#pragma unroll
                for (int q = 0; q < W; ++q) acc[q].c[MIX] = zero<T>();
            }
            if (!more || (PRE && npc == stop)) break;
            first = false;
            pc = npc;
            cur = nxt;
            w = wn;
            imm = immn;
        }
    }

    // JetOps::pown for 2 <= n <= 8 (lean_prescan admits no other), the same arithmetic, with
    // no loop: JetOps::pown's repeated-multiplication loop for n > 4, nested in the interpreter
    // loop, made the register allocator copy the whole accumulator jet on every back edge
    // (14 v_mov_b64 per opcode, ~10 % of pass 1); the guarded products below are unrolled
    static __device__ __forceinline__ void pown_lean(J& t, int n) {
        if (n <= 4) {
            if (n == 3) {
                const J base = t;
                O::square(t);
                O::mul(base, t);
            } else {
                O::square(t);
                if (n == 4) O::square(t);
            }
        } else {
            const J base = t;
#pragma unroll
            for (int k = 1; k < 8; ++k)
                if (k < n) O::mul(base, t);
        }
    }

    // JetOps::div_var with the reciprocal supplied (identical arithmetic: qdiv(s, v, 1/v))
    static __device__ __forceinline__ void div_var(J& t, double v, double inv, int axis) {
        const T vv = cvt<T>(v), iv = cvt<T>(inv);
#pragma unroll
        for (int d = 0; d <= K; ++d) {
#pragma unroll
            for (int j = 0; j <= d; ++j) {
                const int i = d - j;
                T s = t.c[ji(i, j)];
                if (axis == 0 && i > 0) s = s - t.c[ji(i - 1, j)];
                if (axis == 1 && j > 0) s = s - t.c[ji(i, j - 1)];
                t.c[ji(i, j)] = qdiv(s, vv, iv);
            }
        }
    }
};

// Class and escalation of one candidate from its grid counts (lane 0; shared with
// validate_kernel's epilogue, whose logic it restates for the point-decided case).
__device__ __forceinline__ void grid_finish(const KernelArgs& a, int64_t cand, uint32_t hdr, int prob,
                                            bool point_reject, double qmax, int nbad, int nfin,
                                            int nnonfin, bool any_grad, bool pconst) {
    int cls;
    uint32_t esc = 0;
    const bool structural = (prob != PDEVAL_PROBLEM_FORCE_FREE) || (hdr & PDEVAL_FLAG_NOCOORD);
    // (P0_CONST: the Kerr constant test passed -- also for u == 0, whose grid jets are all 0)
    if (!any_grad && (nfin > 0 || pconst) && structural) cls = PDEVAL_CLS_ZERO_GRADIENT;
    else if (point_reject) cls = PDEVAL_CLS_REJECT_POINT;   // decided by the point stage: final
    // Kerr: no finite grid point (u not real, or underflowed, everywhere on the grid at the
    // stand-ins of the symbols): nothing proves lhs == 0 -- the reference's symbolic stage does
    // not prove these either (kerr validator.py:283-315).  Final, no tier 2.
    else if (prob != PDEVAL_PROBLEM_FORCE_FREE && nfin == 0) cls = PDEVAL_CLS_REJECT_GRID;
    else if (nbad > a.prm.max_bad) {
        cls = PDEVAL_CLS_REJECT_GRID;
        esc = ESC_GRID_EVAL | ESC_GRID_FAIL;
    } else if (prob == PDEVAL_PROBLEM_FORCE_FREE && a.prm.strict_symbolic && (hdr & (PDEVAL_FLAG_NONSMOOTH2D | PDEVAL_FLAG_UNPROVABLE))) {
        cls = PDEVAL_CLS_REJECT_SYMBOLIC;
    } else {
        cls = PDEVAL_CLS_ACCEPT;
    }
    if (esc && a.esc_list) {
        esc |= (any_grad ? ESC_ANY_GRAD : 0u) | (nfin > 0 ? ESC_NFIN : 0u) | (PD_DIVFREE && a.fmask ? ESC_MASK : 0u);
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

// waves per SIMD of pass 1: force-free 5 (96 VGPRs with the x power table, 48 B of spill;
// 4 waves 149.3 vs 146.9 ms, profiles/r04_c_*), Kerr 6 at W = 2 (80 VGPRs with the late coefficient
// loads; 5: 49.0 ms, 6: 46.5)
#ifndef PD_GRID_WAVES_PER_SIMD
#define PD_GRID_WAVES_PER_SIMD 5
#endif
// Kerr pass 1 at W = 3 rows per dispatch (below): 94 VGPRs, 5 waves/SIMD, no spill (W = 2 at 6
// waves: 48.6 ms per 2^21 step; W = 3 at 5: 47.1-47.5; W = 4 at 4: 47.6-47.8, profiles/r06_s_*)
#ifndef PD_KERR_WAVES_PER_SIMD
#define PD_KERR_WAVES_PER_SIMD 5
#endif
// Kerr pass 1 loads the operator coefficients after the interpreter: 16 fewer VGPRs live
// through it, so 6 waves/SIMD fit without spilling (80 VGPRs): pass 1 48.6 -> 46.5 ms
// (early loads at 6 waves spill 64 B; late loads at 5 waves 49.0, at 7 waves 47.5)
#ifndef PD_KV_LATE
#define PD_KV_LATE 1
#endif
#ifndef PD_KV_LATE_DEEP
#define PD_KV_LATE_DEEP 0
#endif
#ifndef PD_LIST_WAVES_PER_SIMD
#define PD_LIST_WAVES_PER_SIMD 4
#endif
#ifndef PD_KERR_W
#define PD_KERR_W 3
#endif
// Kerr pass 2 (the stack-3 list) at W = 4 rows per dispatch, 4 waves/SIMD (128 VGPRs + 192 B/lane
// of spill): W = 2 (96 B spill) 19.8 ms per 2^21 step, W = 3 18.0, W = 4 17.4 (without the power
// tables, three alternations); W = 1 27.4 ms, W = 3 at 3 waves 20.9, W = 4 at 3 waves 19.0, W = 5
// 21.7 and W = 6 29.9 (their LDS operand slots cap the waves per CU) (profiles/r06_t_*, r06_w_*,
// r06_w2_*, r06_ah_*, r06_aj_*)
#ifndef PD_DEEP_W
#define PD_DEEP_W 4
#endif
// Two lean passes share one body (grid_body):
//   pass 1  grid_kernel       every candidate, one wave each (256-thread blocks), stack <= 2
//                             (one LDS operand slot); deeper programs -> a.defer_list
//   pass 2  grid_list_kernel  persistent over the stack-3 list (64-thread blocks, two slots);
//                             deeper -> a.defer_list (the generic stack-8 pass)
// Folding stack 3 into pass 1 (a runtime slot index, and two slots of LDS per wave for every
// candidate) measured slower for Kerr: 66.1 ms against 49.9 + 13.5 ms (d<=3 batch).
// W = grid rows per dispatch (Lean above): 1 for force-free, PD_KERR_W for Kerr in pass 1,
// PD_DEEP_W for Kerr in pass 2; the rows of a last, partial group past nx are evaluated (their
// x clamped to the last row) and skipped by the epilogue (64 rows at W = 3: 22 groups, 2 spare).
template <int PROB, int MAXD> constexpr int grid_w() {
    return PROB == PDEVAL_PROBLEM_FORCE_FREE ? 1 : (MAXD == 2 ? PD_KERR_W : PD_DEEP_W);
}
template <int PROB> constexpr int grid_k() { return PROB == PDEVAL_PROBLEM_FORCE_FREE ? 4 : 2; }
// dynamic LDS of one block of `waves` waves: the LDS operand slots (Lean::LDS_SLOTS) of W jets
template <int PROB, int MAXD, class T = double> constexpr size_t grid_lds(int waves) {
    using L = Lean<T, grid_k<PROB>(), grid_w<PROB, MAXD>(), MAXD>;
    return (size_t)waves * L::LDS_SLOTS * L::SLOT * sizeof(T);
}

// The hoisted parts (PD_HOIST) of one candidate, in one loop so that the interpreter is inlined
// once.  Job 0, the prefix: x alone, lane r = grid row r, its pure-x coefficients into
// hb[k][row]; y alone, lane j at its own ordinate (the prefix reads no x), the pure-y ones into
// hb[k][j]; returns 0 for `hoist` when some lane carries a non-zero coefficient outside those (a
// non-finite value: the row loop then runs the prefix itself).  Job 1, the segment
// (PD_HOIST_SUB): from its first opcode (original word w0) with an empty stack to the opcode
// before the binary one that consumes it, every coefficient into hb2[c][row or lane] -- the
// whole jet, so no lane's value can differ from the one the row loop would compute.
template <int K, int MAXD, bool SUB>
__device__ __forceinline__ void hoist_parts(const int32_t* dec, int& hoist, bool hy, int h_at, int h_to, uint32_t h_w0,
                                            bool h_y, const double* gx, int nx, int ny, const double* ptab,
                                            double* hb, double* hb2, int lane, double* stk, double y0,
                                            double inv_y0) {
    using L1 = Lean<double, K, 1, MAXD>;
    const int r = min(lane, nx - 1);
    const double xl[1] = {gx[r]}, ixl[1] = {gx[nx + r]};
    PowTab<1> p1;
    p1.sx = nx * (K + 1);
    p1.sy = (K + 1) * ny;
    p1.ny = ny;
    p1.px[0] = ptab + (size_t)r * (K + 1);
    p1.py = ptab + (size_t)PTAB_N * nx * (K + 1) + lane;
#pragma unroll 1
    for (int job = 0; job < (SUB ? 2 : 1); ++job) {
        if (job == 0 ? hoist == 0 : h_at == 0) continue;   // (uniform)
        typename L1::J h[1];
        L1::template run<true, true>(dec, xl, y0, ixl, inv_y0, h, stk, lane, p1, job ? h_at : 1, job ? h_to : hoist,
                                     nullptr, 0, 0, false, job ? h_w0 : 0u, job != 0);
        if (job == 0) {
            bool dirty = false;
#pragma unroll
            for (int c = 0; c < nc(K); ++c) {
                bool pure = false;
#pragma unroll
                for (int k = 0; k <= K; ++k) pure = pure || c == (hy ? ji(0, k) : ji(k, 0));
                if (!pure) dirty = dirty || !(h[0].c[c] == 0.0);
            }
            if (__any(dirty)) {
                hoist = 0;
                continue;
            }
#pragma unroll
            for (int k = 0; k <= K; ++k) hb[k * 64 + lane] = h[0].c[hy ? ji(0, k) : ji(k, 0)];
        } else {
#pragma unroll
            for (int c = 0; c < nc(K); ++c) hb2[c * 64 + lane] = h[0].c[c];
        }
    }
    __threadfence_block();   // the rows read other lanes' values
}

// ---- hoist-buffer slots.  The hoisted parts of a candidate are needed only while its wave runs,
// so the buffer holds slots, not candidates: 8 pools (one per XCD, so that a slot's successive
// owners share one L2 -- the XCD L2s are not coherent with each other) of a.hoist_pool slots, more
// than the waves an XCD holds at once.  A wave takes the slot of its candidate within its pool
// (linear probing past slots other waves still hold) with a compare-and-swap on the slot's owner
// word and frees it when its rows are done; its new owner writes every value it reads before
// reading it.  The buffer stays 30 MiB (force-free) / 54 MiB (Kerr) at any batch size and mostly
// in L2 / MALL: force-free pass 1 wrote the 2.5 KiB of every hoisted candidate to HBM before
// (round 5: n x 2.5 KiB, 5.4 GB at 2^21).  A split launch (a small batch's parts: several waves
// per candidate) indexes by candidate instead (n < 1024 <= the slot count).
#ifndef PD_HOIST_SLOTS
#define PD_HOIST_SLOTS 1
#endif
// the failing-lane words of tier 1 stored sparsely (a.fsum; see grid_body)
#ifndef PD_FMASK_SPARSE
#define PD_FMASK_SPARSE 1
#endif
__device__ __forceinline__ uint32_t xcc_id() {
#ifndef PD_HOST_SIM
    // HW_REG_XCC_ID (hwreg 20), bits 3:0
    return (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;
#else
    return 0u;
#endif
}
// the slot of wave-uniform `cand` (lane 0 takes it; every lane gets it), or -1 when there is no
// hoist buffer.  A wave that cannot take a slot after every probe of many sweeps (it cannot
// happen while a pool has more slots than an XCD holds waves) sets ERRW_HOIST and uses its
// home slot: the call then reports an error rather than hanging
__device__ __forceinline__ int64_t hoist_acquire(const KernelArgs& a, int64_t cand, int lane, bool split) {
    if (!PD_HOIST_SLOTS || !a.hoist_own) return cand;   // one slot per candidate (A/B layout)
    if (split || a.hoist_pool <= 0) {
        if (cand < (int64_t)8 * a.hoist_pool) return cand;
        if (lane == 0 && a.errw) atomicOr(a.errw, (uint32_t)ERRW_HOIST);
        return 0;
    }
    const int64_t P = a.hoist_pool, base = (int64_t)xcc_id() * P, home = cand % P;
    int got = -1;
    if (lane == 0) {
        for (int k = 0; k < 64 * kHoistPool && got < 0; ++k) {
            const int64_t t = base + (home + k) % P;
            if (atomicCAS(a.hoist_own + t, 0u, 1u) == 0u) got = (int)t;
            else if (k >= 16) __builtin_amdgcn_s_sleep(1);
        }
        if (got < 0) {
            if (a.errw) atomicOr(a.errw, (uint32_t)ERRW_HOIST);
            got = (int)(base + home);
        }
    }
    return (int64_t)__builtin_amdgcn_readfirstlane(got);
}
// every lane's accesses to the slot are complete (vmcnt(0) waits for the wave's loads and
// stores), then the owner word is cleared
__device__ __forceinline__ void hoist_release(const KernelArgs& a, int64_t slot, int lane, bool split) {
    if (!PD_HOIST_SLOTS || split || !a.hoist_own || a.hoist_pool <= 0 || slot < 0) return;
#ifndef PD_HOST_SIM
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    if (lane == 0) __hip_atomic_store(a.hoist_own + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The grid stage of one candidate (wave-uniform cand), lean interpreter with MAXD slots, jets
// over T: double, or cplx for the force-free candidates not real at p* (the complex pass, whose
// point stage point_list_kernel<.., cplx> decided).
// Small batches (a handful of candidates: the inline driver's one validate() per candidate)
// would leave all but a few SIMDs idle while one wave walks a candidate's 64 grid rows, so the
// rows of each candidate are split over `parts` waves (contiguous ranges, whole W groups):
// every part adds its counts into the candidate's accumulator (a.t2acc, zero between
// launches, as tier 2's parts do) and the part that completes the candidate writes the
// outputs and zeroes the accumulator.  Sums of counts and the max of maxima do not depend on
// the split, so the outputs are those of one wave.
// ROT: the rotating force-free constraint (params.omega2 != 0, FFEpi::rotate_A / _B) -- its own
// kernel instances, so the Omega = 0 epilogue compiles to the code it was (a runtime branch there
// cost pass 1 20 %: 161.4 vs 133.7 ms, profiles/r04_o_ff.log)
template <int PROB, int MAXD, class T = double, bool ROT = false>
__device__ __forceinline__ void grid_body(const KernelArgs& a, int64_t cand, int lane, T* stk,
                                          int64_t* slow_list, int32_t* slow_count, int part = 0,
                                          int parts = 1) {
    constexpr int K = grid_k<PROB>();
    constexpr int W = grid_w<PROB, MAXD>();
    constexpr bool CX = Real<T>::cplx_pass;
    using L = Lean<T, K, W, MAXD>;
    using J = typename L::J;
    const int64_t beg = a.offsets[cand], end = a.offsets[cand + 1];
    const bool in_bounds = beg >= 0 && end > beg && end <= a.n_words && end - beg < (1 << 24);
    const int32_t* prog = a.ops + (in_bounds ? beg : 0);
    const uint32_t hdr = in_bounds ? rd_word(prog) : 0xffu;
    const uint8_t ps = (uint8_t)__builtin_amdgcn_readfirstlane((int)a.pstate[cand]);
    if (!CX && (ps & P0_CPLX)) return;                           // the complex passes take it
    if ((ps & 3) == P0_REJECT && !a.prm.full_grid) return;      // final after the point stage
    bool slow = !in_bounds || (hdr & 0xffu) != 0u || (ps & 3) == P0_NONE || (!CX && (hdr & PDEVAL_FLAG_COMPLEX));
    if (!slow && (int)((hdr >> 8) & 0xffu) > MAXD) {
        if (lane == 0 && part == 0) list_append(a.defer_list, a.defer_count, a.list_capacity, cand);
        return;
    }
    // the decoded program (decode_kernel, run before pass 1): 0xff = not for the lean passes;
    // its true stack depth must fit this pass's slots
    uint32_t u_sgn = 0u;   // a sign the decoder folded out of the program (PD_FOLD_NEG), bit 31
    int hoist = 0;         // PD_HOIST: the first opcode after the program's hoisted prefix, or 0
    bool hy = false;       // ... a prefix of y alone
    int h_at = 0, h_to = 0;   // PD_HOIST_SUB: the hoisted segment's span, its kind, first word
    bool h_y = false;
    uint32_t h_w0 = 0u;
    if (!slow) {
        const uint32_t dh = rd_word(a.dec + beg);
        slow = (dh & 0xffu) != 0u || (int)((dh >> 8) & 0xffu) > MAXD;
        u_sgn = (dh & 0x10000u) << 15;
        if (!CX && hoist_sub<PROB>() && a.hseg && !slow) {
            // (the decoder rewrote the segment's first opcode: every part of a split launch
            // evaluates it -- the same values into the same slot)
            const int32_t* hs = a.hseg + 4 * cand;
            h_at = __builtin_amdgcn_readfirstlane(hs[1]);
            if (h_at) {
                h_w0 = (uint32_t)__builtin_amdgcn_readfirstlane(hs[0]);
                h_to = __builtin_amdgcn_readfirstlane(hs[2]);
                h_y = __builtin_amdgcn_readfirstlane(hs[3]) != 0;
            }
        }
        if (!CX && PD_HOIST && a.hoist && parts == 1) {
            hoist = (int)((dh >> 17) & 0x3fffu);
            hy = (dh >> 31) != 0u;
            // (y alone: one ordinate per lane; Kerr only -- the force-free row loop with the y
            // form measured 4 % slower in both modes, 132.7 vs 126.5 ms unhoisted, r05_j/r05_i)
            if (hy && (PROB == PDEVAL_PROBLEM_FORCE_FREE || a.ny != 64)) hoist = 0;
            if (PROB == PDEVAL_PROBLEM_FORCE_FREE) hy = false;
        }
    }
    if (slow) {
        if (lane == 0 && part == 0) list_append(slow_list, slow_count, a.list_capacity, cand);
        return;
    }
    const int per_row = a.ny >> 6;
    const double y0 = a.gy[lane];
    double inv_y0 = rcp(y0);
    // opaque to the optimizer: otherwise "per_row == 1 ? inv_y0 : rcp(y)" below is rewritten as
    // rcp(per_row == 1 ? y0 : y) and the IEEE reciprocal (11 VALU) runs once per row instead of
    // once per candidate
    if constexpr (PD_INVY_PIN) pin_f64(inv_y0);
    // the prefix of one coordinate (PD_HOIST), once for every row: x alone, lane r evaluates it
    // at x = gx[r]; y alone, each lane at its own ordinate -- the same opcodes on the same values
    // as the row loop would, so the same jets -- and its pure-x (pure-y) coefficients go to the
    // candidate's slot of a.hoist; every row then starts its run after the prefix with those
    // coefficients and the others 0.  The others are exact zeros of either sign (products with
    // the 0 coefficients of the coordinate's jet), and no jet operation divides by a coefficient
    // other than the value, so a zero's sign changes no result; where a lane carries a
    // non-finite coefficient (0 * inf = NaN in the others) the candidate is not hoisted.
    // (a.nx <= 64, checked by the host, which passes a.hoist = NULL otherwise)
    int64_t hslot = -1;   // the candidate's hoist-buffer slot while this wave holds it
    if constexpr (!CX && PD_HOIST) {
        if (hoist || h_at) {
            hslot = hoist_acquire(a, cand, lane, parts > 1);
            hoist_parts<K, MAXD, hoist_sub<PROB>()>(a.dec + beg, hoist, PROB != PDEVAL_PROBLEM_FORCE_FREE && hy, h_at, h_to, h_w0, h_y,
                                 a.gx, a.nx, a.ny, a.ptab, a.hoist + (size_t)hslot * hoist_stride(K),
                                 a.hoist + (size_t)hslot * hoist_stride(K) + (K + 1) * 64, lane, stk, y0, inv_y0);
        }
    }
    const double* hbuf = a.hoist + (size_t)(hslot < 0 ? 0 : hslot) * hoist_stride(K);
    GridMax<PROB != PDEVAL_PROBLEM_FORCE_FREE> gm;   // (PD_DIVFREE) the lane's running maximum of q
    double qmax = 0.0;
    int nbad = 0, nfin = 0;
    bool grad_nz = (ps & P0_GRAD) != 0;
    // grid rows holding a fingerprint point (one bit per row; nx > 64: every row)
    uint64_t fp_rows = 0;
#pragma unroll
    for (int f = 0; f < PDEVAL_FP_N; ++f) {
        const int r = (a.fp_pts[f] - a.n_ref) / a.ny;
        if (a.fp_pts[f] >= a.n_ref && r < 64) fp_rows |= 1ull << r;
    }
    if (a.nx > 64) fp_rows = ~0ull;
    // this part's rows: whole groups of W
    // PD_FMASK_SPARSE: lane 0 stores only the non-zero failing-lane words and, at the end, the
    // bitmap of the chunks it stored (a.fsum); a split launch (parts > 1), or a grid of more
    // than 64 chunks, stores every word and an all-ones bitmap
    const bool fsparse = PD_FMASK_SPARSE && a.fsum && parts == 1 && a.nx * per_row <= 64;
    uint64_t fsum = 0ull;
    const int groups = (a.nx + W - 1) / W;
    const int row0 = W * (int)((int64_t)groups * part / parts), row1 = min(a.nx, W * (int)((int64_t)groups * (part + 1) / parts));
    for (int row = row0; row < row1; row += W) {
        double x[W], inv_x[W], inv_x2[W], inv_x3[W];
#pragma unroll
        for (int q = 0; q < W; ++q) {
            x[q] = rd_sf64(a.gx + min(row + q, a.nx - 1));   // a tail row past nx: unused
            inv_x[q] = rd_sf64(a.gx + a.nx + min(row + q, a.nx - 1));   // = rcp(x[q]), host table
            // the epilogue's 1/x^2, 1/x^3 (as ff_epilogue_r forms them), kept in SGPRs
            inv_x2[q] = inv_x[q] * inv_x[q];
            inv_x3[q] = inv_x2[q] * inv_x[q];
            if constexpr (PD_EPI_UNIFORM) {
                inv_x2[q] = uniform_f64(inv_x2[q]);
                inv_x3[q] = uniform_f64(inv_x3[q]);
            }
        }
        PowTab<W> pt;
        pt.sx = a.nx * (K + 1);
        pt.sy = (K + 1) * a.ny;
        pt.ny = a.ny;
#pragma unroll
        for (int q = 0; q < W; ++q) pt.px[q] = a.ptab + (size_t)min(row + q, a.nx - 1) * (K + 1);
        for (int sl = 0; sl < per_row; ++sl) {
            const double y = per_row == 1 ? y0 : a.gy[sl * 64 + lane];
            pt.py = a.ptab + (size_t)PTAB_N * a.nx * (K + 1) + sl * 64 + lane;
            double inv_y = inv_y0;
            if (per_row != 1) inv_y = rcp(y);
            // Kerr: this point's operator coefficients (a 128 KiB table, L2-resident) are loaded
            // before the program runs, so their latency hides under the interpreter
            // (W > 2: after it, so that 4W doubles are not live through the interpreter)
            double kv[W][4];
            auto load_kv = [&]() {
                if constexpr (PROB != PDEVAL_PROBLEM_FORCE_FREE) {
#pragma unroll
                    for (int q = 0; q < W; ++q) {
                        const double* kp = (PD_KERR_LEAN ? a.kc2 : a.kc) + 4 * (a.n_ref + min(row + q, a.nx - 1) * a.ny + sl * 64 + lane);
#pragma unroll
                        for (int i = 0; i < 4; ++i) kv[q][i] = kp[i];
                    }
                }
            };
            constexpr bool kv_late = W > 2 || (MAXD == 2 && PD_KV_LATE) || (MAXD > 2 && PD_KV_LATE_DEEP);
            if constexpr (!kv_late) load_kv();
            J u[W];
            if (!CX && PD_HOIST && hoist) {
                const double* hb = hbuf;
#pragma unroll
                for (int q = 0; q < W; ++q) {
#pragma unroll
                    for (int c = 0; c < nc(K); ++c) u[q].c[c] = zero<T>();
                    if (PROB != PDEVAL_PROBLEM_FORCE_FREE && hy) {
#pragma unroll
                        for (int k = 0; k <= K; ++k) u[q].c[ji(0, k)] = cvt<T>(hb[k * 64 + lane]);
                    } else {
#pragma unroll
                        for (int k = 0; k <= K; ++k) u[q].c[ji(k, 0)] = cvt<T>(hb[k * 64 + min(row + q, a.nx - 1)]);
                    }
                }
            }
            L::run(a.dec + beg, x, y, inv_x, inv_y, u, stk, lane, pt, hoist ? hoist : 1, 0,
                   h_at ? hbuf + (K + 1) * 64 : nullptr, row, a.nx - 1, h_y);
            if constexpr (kv_late) load_kv();
#pragma unroll
            for (int q = 0; q < W; ++q) {
                if (W > 1 && row + q >= a.nx) break;                     // uniform
                const int base = a.n_ref + (row + q) * a.ny + sl * 64;   // point index of lane 0
                PointResult r;
                if constexpr (PROB == PDEVAL_PROBLEM_FORCE_FREE)
                    r = PD_EPI_TABLE_RCP ? ff_epilogue_p<T>(u[q].c, inv_x[q], inv_x2[q], inv_x3[q], x[q], ROT ? a.prm.omega2 : 0.0)
                                         : ff_epilogue<T>(u[q].c, x[q], ROT ? a.prm.omega2 : 0.0);
                else if constexpr (PD_KERR_LEAN && !Real<T>::cplx_pass) r = kerr_epilogue_lean<T>(u[q].c, kv[q]);
                else r = kerr_epilogue<T>(u[q].c, kv[q]);
                // the zero test: |res| > tau S (PD_DIVFREE, no division per point; the lane's
                // maximum of q is kept as a (|res|, S) pair and divided once, GridMax) or the
                // round-4 form q = |res| / S per point, q > tau
                double qv = 0.0;
                if constexpr (!PD_DIVFREE)
                    qv = PD_FAST_SCALED ? scaled_fast(r.res_abs, r.scale)
                                        : PD_SCALED_SEL ? scaled_sel(r.res_abs, r.scale) : scaled(r.res_abs, r.scale);
                if constexpr (PD_DIVFREE) {
                    gm.add(r.finite, r.res_abs, r.scale);
                    grad_nz = grad_nz | (r.finite & !r.grad_zero);
                    nfin += (int)__popcll(r.fin_lanes);
                    const uint64_t fm = r.fin_lanes & lane_mask(grid_fails(r.res_abs, r.scale, a.prm.tau_grid));
                    nbad += (int)__popcll(fm);
                    // the chunk's failing lanes, for tier 2 (a candidate the point stage rejected
                    // is final and never escalates)
                    if (a.fmask && (ps & 3) != P0_REJECT) {
                        const int ch = (row + q) * per_row + sl;
                        if (lane == 0 && (!fsparse || fm)) a.fmask[cand * (int64_t)(a.nx * per_row) + ch] = fm;
                        // (outside lane 0's branch: the bitmap stays wave-uniform, in SGPRs -- in
                        // the branch it was a VGPR pair spilled to scratch and reloaded per point)
                        if (fm) fsum |= 1ull << (ch & 63);
                    }
                } else {
                    if (r.finite) {
                        qmax = fmax(qmax, qv);
                        if (!r.grad_zero) grad_nz = true;
                    }
                    nfin += (int)__popcll(__ballot(r.finite));
                    nbad += (int)__popcll(__ballot(r.finite && qv > a.prm.tau_grid));
                }
                // the fingerprint points of this row, after the counts: its lane-divergent stores
                // between the point's flags and their ballots made the compiler keep each flag in
                // a VGPR across them (a select and a compare more per ballot, every point)
                if (a.out.fingerprint && (row + q >= 64 || ((fp_rows >> (row + q)) & 1ull))) {
#pragma unroll
                    for (int f = 0; f < PDEVAL_FP_N; ++f) {
                        const int rel = a.fp_pts[f] - base;   // uniform
                        if (rel >= 0 && rel < 64 && lane == rel) {
                            const double v = fp_value(u[q].c[0]);
                            a.out.fingerprint[cand * PDEVAL_FP_N + f] =
                                __hiloint2double((int)((uint32_t)__double2hiint(v) ^ u_sgn), __double2loint(v));
                        }
                    }
                }
            }
        }
    }
    if constexpr (!CX && PD_HOIST) {
        if (hslot >= 0) hoist_release(a, hslot, lane, parts > 1);
    }
    if (PD_DIVFREE && a.fmask && a.fsum && (ps & 3) != P0_REJECT && lane == 0) a.fsum[cand] = fsparse ? fsum : ~0ull;
    if constexpr (PD_DIVFREE) qmax = gm.q();
    qmax = wave_max(qmax);
    bool grad_any = __any(grad_nz);
    if (parts > 1) {
        int last = 0;
        if (lane == 0) {
            T2Acc* A = a.t2acc + cand;
            atomicAdd(&A->nb1, nbad);
            atomicAdd(&A->nfin, nfin);
            atomicMax(&A->qmax_bits, (unsigned long long)__double_as_longlong(qmax));   // qmax >= 0
            if (grad_any) atomicOr(&A->grad, 1u);
            __threadfence();
            if (atomicAdd(&A->done, 1) == parts - 1) {
                __threadfence();
                nbad = atomicAdd(&A->nb1, 0);
                nfin = atomicAdd(&A->nfin, 0);
                qmax = __longlong_as_double((long long)atomicMax(&A->qmax_bits, 0ull));
                grad_any = atomicOr(&A->grad, 0u) != 0u;
                A->nb1 = A->nfin = A->done = 0;   // ready for the next launch
                A->grad = 0u;
                A->qmax_bits = 0ull;
                last = 1;
            }
        }
        if (!__builtin_amdgcn_readfirstlane(last)) return;   // lane 0 is the first active lane
    }
    const bool any_grad = grad_any && !(ps & P0_CONST);
    if (lane == 0)
        grid_finish(a, cand, hdr, PROB, (ps & 3) == P0_REJECT, qmax, nbad, nfin, a.nx * a.ny - nfin, any_grad,
                    (ps & P0_CONST) != 0);
}

// pass 1: one wave per candidate, 4 per 256-thread block; a.defer_list takes stack-3+ programs,
// slow_list what the lean path does not take (drained by the generic kernel)
// Waves (candidates) per pass-1 block: one.  A block's LDS is released only when its last wave
// ends, and the waves of a 4-wave block ran programs of unrelated lengths, so finished waves
// left their share idle until the slowest one ended.  With one wave per block:
// force-free pass 1 83.6 -> 76.6 ms, Kerr 46.8 -> 38.0 ms (profiles/r02_bench_*_wpb*.log).
// PD_GRID_PERM = 1 instead keeps 4-wave blocks but takes the candidates in the shape order of
// pdeval_sort.hip, so a block's waves run programs of one opcode sequence (78.3 / 43.9 ms).
#ifndef PD_GRID_WPB
#define PD_GRID_WPB 1
#endif
#ifndef PD_GRID_XCD
#define PD_GRID_XCD 1
#endif
#ifndef PD_GRID_PERM
#define PD_GRID_PERM 0
#endif
// SPLIT: the small-batch instance (grid_body's parts); the full-batch instance has parts == 1
// folded in, so its code is the one-wave-per-candidate kernel
template <int PROB, bool SPLIT, bool ROT = false>
__global__ __launch_bounds__(64 * PD_GRID_WPB, PROB == PDEVAL_PROBLEM_FORCE_FREE ? PD_GRID_WAVES_PER_SIMD : PD_KERR_WAVES_PER_SIMD)
void grid_kernel(KernelArgs a, int64_t* slow_list, int32_t* slow_count, int parts_arg) {
    const int parts = SPLIT ? parts_arg : 1;
#ifndef PD_HOST_SIM
    extern __shared__ __align__(16) unsigned char pd_lds[];
#else
    static unsigned char pd_lds[1];
#endif
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double* stk = reinterpret_cast<double*>(pd_lds) + (size_t)wib * grid_lds<PROB, 2>(1) / sizeof(double);
    // Workgroups are dispatched round-robin over the 8 XCDs, each with its own L2.  One-wave
    // blocks in launch order would send neighbouring candidates -- whose programs share cache
    // lines -- to 8 different L2s; instead each XCD takes a contiguous range of blocks.
    // Force-free: HBM traffic 518 -> 187 B per candidate at the same time (76.0 ms); Kerr
    // measured 38.0 -> 38.7 ms with it, so Kerr keeps the launch order
    // (profiles/r02_bench_*_xcd*.log, r02_xcd_ff_pmc.json).
    int64_t blk = blockIdx.x;
    if (PD_GRID_XCD && PROB == PDEVAL_PROBLEM_FORCE_FREE && parts == 1) {
        const int64_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + (x < r ? x : r) + blk / 8;
    }
    int64_t wi = blk * (blockDim.x >> 6) + wib;
    int part = 0;
    if (parts > 1) {   // small batches: wave wi = (candidate, part)
        part = (int)(wi % parts);
        wi /= parts;
    }
    if (wi >= a.n) return;
    const int64_t cand = (PD_GRID_PERM && a.perm) ? checked_cand(a, (int64_t)__builtin_amdgcn_readfirstlane(a.perm[wi]), ERRW_PERM) : wi;
    if (cand < 0) return;
    grid_body<PROB, 2, double, ROT>(a, cand, threadIdx.x & 63, stk, slow_list, slow_count, part, parts);
}

// pass 2: the stack-3 list a.list (count *a.list_count), persistent 64-thread blocks
template <int PROB, bool SPLIT, bool ROT = false>
__global__ __launch_bounds__(64, PROB == PDEVAL_PROBLEM_FORCE_FREE ? 1 : PD_LIST_WAVES_PER_SIMD) void grid_list_kernel(KernelArgs a, int64_t* slow_list, int32_t* slow_count, int parts_arg) {
    const int parts = SPLIT ? parts_arg : 1;
#ifndef PD_HOST_SIM
    extern __shared__ __align__(16) unsigned char pd_lds[];
#else
    static unsigned char pd_lds[1];
#endif
    double* stk = reinterpret_cast<double*>(pd_lds);
    int64_t nwork = (int64_t)(*a.list_count);
    if (nwork > a.list_capacity) nwork = a.list_capacity;
    WorkQueue q;
    for (int64_t wp = q.first(a); wp < nwork * parts; wp = q.next(a, wp)) {
        const int64_t wi = wp / parts;
        // (entries checked before the launch: sanitize_list_kernel -- a check here, in the loop,
        // cost this kernel 112 B of spill)
        const int64_t cand = (int64_t)__builtin_amdgcn_readfirstlane((int)a.list[wi]);
        grid_body<PROB, 3, double, ROT>(a, cand, threadIdx.x & 63, stk, slow_list, slow_count, (int)(wp % parts), parts);
    }
}

// the complex pass: the force-free candidates not real at p* (list a.list = L_CPLX, count
// *a.list_count), complex jets, persistent one-wave blocks; deeper programs -> a.defer_list,
// what the lean path does not take -> slow_list (the generic complex kernel drains it)
#ifndef PD_CPLX_WAVES_PER_SIMD
#define PD_CPLX_WAVES_PER_SIMD 2
#endif
template <bool SPLIT, bool ROT = false>
__global__ __launch_bounds__(64, PD_CPLX_WAVES_PER_SIMD) void grid_cplx_kernel(KernelArgs a, int64_t* slow_list,
                                                                                int32_t* slow_count, int parts_arg) {
    const int parts = SPLIT ? parts_arg : 1;
#ifndef PD_HOST_SIM
    extern __shared__ __align__(16) unsigned char pd_lds[];
#else
    static unsigned char pd_lds[1];
#endif
    cplx* stk = reinterpret_cast<cplx*>(pd_lds);
    int64_t nwork = (int64_t)(*a.list_count);
    if (nwork > a.list_capacity) nwork = a.list_capacity;
    WorkQueue q;
    for (int64_t wp = q.first(a); wp < nwork * parts; wp = q.next(a, wp)) {
        const int64_t wi = wp / parts;
        // (entries checked before the launch: sanitize_list_kernel -- 432 B of spill otherwise)
        const int64_t cand = (int64_t)__builtin_amdgcn_readfirstlane((int)a.list[wi]);
        grid_body<PDEVAL_PROBLEM_FORCE_FREE, 2, cplx, ROT>(a, cand, threadIdx.x & 63, stk, slow_list, slow_count,
                                                      (int)(wp % parts), parts);
    }
}

}  // namespace pd
