/*
 * pdeval.h -- C ABI of libpdeval.so, the MI355X (gfx950) candidate validator.
 *
 * Drop-in boundary for the per-candidate PDE-residual check of PimDeWitte/pde-engine.
 * One call validates a whole batch of candidate expressions; it replaces, per candidate,
 *   - problems/force_free/validator.py:260-437           PreciseFoliationValidator.validate
 *   - problems/kerr_magnetosphere/validator.py:210-345   KerrMagnetosphereValidator.validate
 * as called by the validator worker pool (general_method_paper_reproduction.py:1671-1824,
 * the per-candidate loop :1753-1812) and by the inline path (:1288-1339).  The reference has
 * no native code and no FFI; the Python side of this boundary (ctypes) lives in
 * pde-engine_amd/pdeval/_lib.py and is the "binding a maintainer would add" (INTEGRATION.md).
 *
 * Conventions: plain C, no exceptions cross the boundary, every entry point returns an int
 * status (PDEVAL_OK = 0), caller-owned host buffers, library-owned device buffers and HIP
 * stream, one context per GPU, calls on one context serialized by the caller.
 *
 * Candidate programs (the flattened SymPy tree, see DESIGN.md "Program format"):
 *   ops      int32 words of ALL programs, concatenated; program i is ops[offsets[i] ..
 *            offsets[i+1]).  Word = opcode (bits 0-7) | small operand (bits 8-31); opcodes
 *            that carry an f64 immediate are followed by two words holding its IEEE bits
 *            (low word first); if the immediate is not exactly representable (1/3, 1/10, E)
 *            the opcode word has PDEVAL_IMM_DD set and two more words follow: the f64 low
 *            part of the double-double value (value - hi), used by the point stage's
 *            double-double tier (the fp64 passes skip it).
 *   offsets  int64[n+1], offsets[0] = 0, non-decreasing.
 */
#ifndef PDEVAL_H
#define PDEVAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes returned by every entry point ---- */
#define PDEVAL_OK              0
#define PDEVAL_ERR_ARG         1   /* bad argument (null ctx, n < 0, bad offsets ...) */
#define PDEVAL_ERR_HIP         2   /* a HIP runtime call failed; see pdeval_last_error */
#define PDEVAL_ERR_PROGRAM     3   /* a program failed host-side validation */
#define PDEVAL_ERR_NODEVICE    4

/* ---- problems (the problems/ plugin registry, problems/__init__.py:355-361) ---- */
#define PDEVAL_PROBLEM_FORCE_FREE   0   /* foliation determinant, jets of order 4 */
#define PDEVAL_PROBLEM_KERR         1   /* Kerr linear surrogate, jets of order 2 */

/* ---- per-candidate class (status[] output) ---- */
#define PDEVAL_CLS_ACCEPT          0   /* residual ~ 0 at the reference point(s) and on the grid */
#define PDEVAL_CLS_REJECT_POINT    1   /* rejected by the reference-point stage            */
#define PDEVAL_CLS_REJECT_GRID     2   /* passed the point stage, residual != 0 on the grid */
#define PDEVAL_CLS_ZERO_GRADIENT   3   /* u is constant (force-free :309-312, Kerr :231-240) */
#define PDEVAL_CLS_NONFINITE_REF   4   /* non-finite at a reference point in real arithmetic */
#define PDEVAL_CLS_UNSUPPORTED     5   /* program uses an opcode this build does not handle */
#define PDEVAL_CLS_BAD_PROGRAM     6   /* malformed program (stack under/overflow)          */
#define PDEVAL_CLS_REJECT_SYMBOLIC 7   /* zero on the grid, but non-smooth (Abs) in both
                                          coordinates: the reference's symbolic stage cannot
                                          prove it (assumptions are lost in its string round
                                          trip, validator.py:242-252 / lean_bridge.py:73), so
                                          with strict_symbolic it is rejected as there     */

/* ---- opcodes (bits 0-7 of a program word) ---- */
enum pdeval_opcode {
    PDOP_PUSH_X   = 1,   /* push coordinate 1 (rho | r)                          */
    PDOP_PUSH_Y   = 2,   /* push coordinate 2 (z | x)                            */
    PDOP_PUSH_C   = 3,   /* push constant            [f64 imm]                   */
    PDOP_ADD      = 4,   /* b=pop, a=pop, push a+b                               */
    PDOP_SUB      = 5,   /* a-b                                                  */
    PDOP_RSUB     = 6,   /* b-a                                                  */
    PDOP_MUL      = 7,   /* a*b                                                  */
    PDOP_DIV      = 8,   /* a/b                                                  */
    PDOP_RDIV     = 9,   /* b/a                                                  */
    PDOP_ADDC     = 10,  /* top += c                 [f64 imm]                   */
    PDOP_MULC     = 11,  /* top *= c                 [f64 imm]                   */
    PDOP_RDIVC    = 12,  /* top = c / top            [f64 imm]                   */
    PDOP_NEG      = 13,  /* top = -top                                           */
    PDOP_ADD_X    = 14,  /* top += x                                             */
    PDOP_ADD_Y    = 15,  /* top += y                                             */
    PDOP_MUL_X    = 16,  /* top *= x                                             */
    PDOP_MUL_Y    = 17,  /* top *= y                                             */
    PDOP_SUB_X    = 18,  /* top -= x                                             */
    PDOP_SUB_Y    = 19,  /* top -= y                                             */
    PDOP_POWN     = 20,  /* top = top**n, n = operand bits 8-15, 2 <= n <= 16    */
    PDOP_POW      = 21,  /* top = top**alpha (principal branch) [f64 imm alpha]  */
    PDOP_EXP      = 22,
    PDOP_LOG      = 23,
    PDOP_ABS      = 24,
    PDOP_SQRT     = 25,  /* = POW 1/2, kept separate (common, cheaper x0**alpha) */
    PDOP_DIV_X    = 26,  /* top /= x                                             */
    PDOP_DIV_Y    = 27,  /* top /= y                                             */
    PDOP_PUSH_I   = 28,  /* push the imaginary unit (complex pass only)          */
    /* fused coordinate powers p = v**n: n = operand bits 8-15 (2..16), v = x if bit 16 is
       0 else y; the jet of p is univariate with C(n,k) v^(n-k) coefficients          */
    PDOP_PUSH_P   = 29,  /* push p                                               */
    PDOP_ADD_P    = 30,  /* top += p                                             */
    PDOP_SUB_P    = 31,  /* top -= p                                             */
    PDOP_MUL_P    = 32,  /* top *= p                                             */
    PDOP_DIV_P    = 33,  /* top /= p                                             */
    PDOP_RDIV_P   = 34,  /* top = p / top                                        */
    PDOP_COUNT_   = 35,
    PDOP_UNSUPPORTED = 254  /* placeholder for a construct the flattener cannot lower;
                               the candidate is classified PDEVAL_CLS_UNSUPPORTED       */
};

#define PDEVAL_MAX_STACK  8   /* deepest program stack any kernel variant accepts */
#define PDEVAL_MAX_BATCH  ((int64_t)1 << 30)  /* largest n of one validate call (2^30 candidates;
                                                 int32 work-list counters): PDEVAL_ERR_ARG beyond */

/* Immediate-carrying opcode word (PUSH_C, ADDC, MULC, RDIVC): bit 8 set = a double-double
   low part follows the f64 immediate (2 more words, low word first).                    */
#define PDEVAL_IMM_DD     (1u << 8)
/* bit 9 set (PUSH_C, ADDC, MULC, RDIVC; never with PDEVAL_IMM_DD) = the immediate is one of the
   problem's constants (Kerr M, a), not a literal: the first word is a descriptor, bits 0-2 =
   PDEVAL_PRM_* (M, a, 1/M, 1/a, M^2, a^2, 1/M^2, 1/a^2), bit 3 = negated; the second word is
   0.  Its value is the
   stage's: the point stage substitutes the validator's M_value / a_value, the constant test and
   the grid stage the stand-ins of the symbols (pdeval_kerr_constants).                   */
#define PDEVAL_IMM_PRM    (1u << 9)
#define PDEVAL_PRM_M      0
#define PDEVAL_PRM_A      1
#define PDEVAL_PRM_INV_M  2
#define PDEVAL_PRM_INV_A  3
#define PDEVAL_PRM_M2     4   /* (index + 4: the square; index ^ 2: the reciprocal) */
#define PDEVAL_PRM_A2     5
#define PDEVAL_PRM_INV_M2 6
#define PDEVAL_PRM_INV_A2 7
#define PDEVAL_PRM_NEG    8

/* Program header word: opcode 0 | stack depth << 8 | flags */
#define PDEVAL_FLAG_COMPLEX  (1u << 16)  /* pushes the imaginary unit: complex pass only   */
#define PDEVAL_FLAG_NOCOORD  (1u << 17)  /* references no coordinate (u is a constant)   */
#define PDEVAL_FLAG_RATIONAL (1u << 18)  /* rational operations and constants only: the
                                            residual at a rational point is rational (host
                                            reason strings, validator.py:371-380)      */
#define PDEVAL_FLAG_NONSMOOTH2D (1u << 19) /* contains Abs and references both coordinates */
#define PDEVAL_FLAG_UNPROVABLE (1u << 20)  /* u = c*exp(g)**(p/4), p > 0, c a number: the reference's symbolic
                                              stage cannot reduce det to 0 (force-free
                                              validator.py:404-416)       */

/* Thresholds of the scaled zero test (DESIGN.md "Zero test"). */
typedef struct pdeval_params {
    double tau_point;    /* point stage: reject iff q* > tau_point                 */
    double tau_grid;     /* grid stage: a finite grid point is "bad" iff q > tau_grid */
    double kerr_abs_tol; /* Kerr fast point check: reject iff max|lhs| >= this (1e-10) */
    int32_t full_grid;   /* 1: evaluate the whole grid for every candidate;
                            0: stop after the point stage for point-rejects (as the
                               reference does, validator.py:371-402)                 */
    /* (tau_point is kept for ABI compatibility; the point stage is decided by the
        error-bounded rule of point_abs_tol / res_rel_acc)              */
    int32_t max_bad;     /* grid stage rejects iff n_bad > max_bad                   */
    int32_t strict_symbolic; /* 1: reproduce the reference's symbolic-stage verdict on
                                non-smooth candidates (PDEVAL_CLS_REJECT_SYMBOLIC)       */
    int32_t reserved;
    double noise_kappa;  /* tier 2: a failing point counts only if |residual| > noise_kappa x
                            its first-order rounding-noise bound     */
    double point_abs_tol;/* force-free point stage: a residual that is certainly non-zero
                            rejects if it is rational (an exact Number != 0) or if
                            |det| >= point_abs_tol = 1e-20 (validator.py:371-397)     */
    double res_rel_acc;  /* point stage: a residual decided in fp64 must carry a
                            first-order error bound noise <= res_rel_acc x |res| (1e-11),
                            else it is re-evaluated in double-double  */
    double omega2;       /* force-free: Omega^2 of rotating field lines, a constant
                            (validator.py:326-329); 0 = the problem path's Omega = 0  */
    double omega2_lo;    /* its low part: Omega^2 = omega2 + omega2_lo as a double-double, so a
                            rational Omega^2 that is no double (Omega = 1/3: 1/9) is carried to
                            2^-106 in the point stage's second tier; 0 when Omega^2 is a double */
} pdeval_params;

/* Per-candidate outputs; any pointer may be NULL (not produced).  Host or device memory
 * depending on the entry point.  n_ref = pdeval_n_ref_points(ctx).                    */
typedef struct pdeval_outputs {
    uint8_t* verdict_bits;   /* ceil(n/8) bytes, bit i = candidate i accepted (LSB first) */
    uint8_t* status;         /* n, PDEVAL_CLS_*                                            */
    double*  q_ref;          /* n, scaled residual at the point stage (Kerr: max |lhs|)    */
    double*  res_ref;        /* n * n_ref, raw residual at each reference point (complex:
                                its modulus with the sign of its real part)              */
    double*  q_grid;         /* n, max scaled residual q = |res| / S over the finite grid
                                points.  Kerr: the IEEE quotient of the point with the largest
                                estimate (its grid-reject text prints it).  Force-free: the
                                maximum of the estimates |res| * rcp(S) themselves (hardware
                                reciprocal, ~1 ulp; no reason text reads it), so a diagnostic  */
    int32_t* n_bad;          /* n, grid points that fail the zero test |res| > tau_grid * S
                                (no division; equal to q > tau_grid except within a rounding
                                of tau_grid); after tier 2, only points whose residual also
                                exceeds its rounding-noise bound.  Tier 2 re-checks the 64-point
                                chunks where tier 1 failed a point (ESC_MASK): a point tier 1
                                passed is the same comparison on the same values and is not
                                re-counted                                                  */
    int32_t* n_nonfinite;    /* n, grid points where the evaluation was not finite         */
    double*  fingerprint;    /* n * PDEVAL_FP_N, u at fixed points (known-solution tags)   */
} pdeval_outputs;

#define PDEVAL_FP_N 4

typedef struct pdeval_ctx pdeval_ctx;

/* grid: {x_lo, x_hi, nx, y_lo, y_hi, ny, x_phase, y_phase}; NULL = the problem's default
 * grid (DESIGN.md "Grids").  Point i of axis x is x_lo + (i + x_phase) * (x_hi-x_lo)/nx. */
int pdeval_create(int device_id, int problem_id, const double* grid, int n_grid, pdeval_ctx** out);
int pdeval_destroy(pdeval_ctx* ctx);
const char* pdeval_last_error(pdeval_ctx* ctx);

/* Kerr constants (kerr_magnetosphere/validator.py:36-44, :69-91, :163-192).  The reference
 * substitutes M = M_value, a = a_value only in its fast point check; its constant test
 * (simplify(u) free of r and x, :231-240) and its symbolic stage (:283-300) keep M and a as the
 * problem's symbols.  The device therefore evaluates the point stage at (M_value, a_value) and
 * the constant test and the grid stage -- the symbolic stage's surrogate -- at (M_sym, a_sym),
 * stand-ins for the symbols (generic values; a_sym < M_sym so that the horizon r+ exists).
 * op_M_fixed / op_a_fixed: the validator was built with the NUMBER M_value (a_value) in place of
 * the symbol (KerrMagnetosphereValidator(r, x, M, 0, ...)): the operator then uses that number
 * in every stage, and u's own M (a) is a free symbol, evaluated at M_sym (a_sym) in every stage.
 * pdeval_create uses the defaults (M_value = 1, a_value = 1/10, problems/__init__.py:283); the
 * default grid follows r+ of the grid stage's operator (DESIGN.md "Grids").              */
typedef struct pdeval_kerr_constants {
    int64_t M_num, M_den;   /* M_value = M_num / M_den (|M_num|, M_den < 2^53)             */
    int64_t a_num, a_den;   /* a_value                                                     */
    double  M_sym, a_sym;   /* stand-ins for the symbols M and a                           */
    int32_t op_M_fixed, op_a_fixed;
} pdeval_kerr_constants;
int pdeval_default_kerr_constants(pdeval_kerr_constants* out);
/* Kerr contexts only; rebuilds the operator tables (and the default grid).  Not while a call
 * on the context is in flight.                                                            */
int pdeval_set_kerr_constants(pdeval_ctx* ctx, const pdeval_kerr_constants* k);

int pdeval_n_ref_points(pdeval_ctx* ctx);
int pdeval_n_points(pdeval_ctx* ctx);          /* n_ref + grid points */
int pdeval_default_params(int problem_id, pdeval_params* out);

/* Host pointers in and out: upload, validate, download (synchronous). */
int pdeval_validate_batch(pdeval_ctx* ctx, const int32_t* ops, int64_t n_words,
                          const int64_t* offsets, int64_t n, const pdeval_params* params,
                          pdeval_outputs* out);

/* Device pointers in and out, asynchronous on `stream` (a hipStream_t; NULL = the
 * context's own non-blocking stream, which does NOT wait for work on the legacy null
 * stream: the caller must have made the inputs ready on it).  Inputs already resident in
 * HBM: this is the timed hot path.  verdict_bits must hold ceil(n/32)*4 bytes, 4-byte
 * aligned, zeroed by the caller or by passing zero_bits = 1.  Programs whose offsets fall
 * outside [0, n_words] are classified PDEVAL_CLS_BAD_PROGRAM, never dereferenced.       */
int pdeval_validate_device(pdeval_ctx* ctx, const int32_t* d_ops, int64_t n_words,
                           const int64_t* d_offsets, int64_t n, const pdeval_params* params,
                           const pdeval_outputs* d_out, void* stream, int zero_bits);

/* The device error word of the most recent pdeval_validate_device call on this context: call
 * it after the caller has synchronized that call's stream.  *word = 0 and PDEVAL_OK when the
 * call was clean; otherwise *word holds the kernel families whose check failed -- a work-list
 * entry outside [0, n) (skipped), or 0x100: a wave found no free hoist-buffer slot -- the
 * call's outputs are not to be trusted, and the return is PDEVAL_ERR_HIP with
 * pdeval_last_error describing the call's state.  (pdeval_validate_batch checks the same
 * word itself before it returns.)                                                         */
int pdeval_device_error(pdeval_ctx* ctx, uint32_t* word);

/* Per-pass device timing (bench / profiling).  With timing enabled, pdeval_validate_device
 * records a HIP event before each of its PDEVAL_N_PASSES launches and one after the last, on
 * the launch stream (passes a problem does not run take 0 ms).  pdeval_pass_times waits for
 * the last event of the most recent call and writes min(max_passes, PDEVAL_N_PASSES)
 * durations in ms (and, if names != NULL, a static name per pass).                       */
#define PDEVAL_N_PASSES 12
int pdeval_set_timing(pdeval_ctx* ctx, int enable);
int pdeval_pass_times(pdeval_ctx* ctx, float* ms, int max_passes, const char** names);
/* Work-list sizes of the most recent call (synchronizes the device): [0] deferred to the
 * stack-3 pass, [1] complex passes, [2] deferred to the stack-8 pass, [3] tier-2 entries,
 * [4] tier-2 stack 3, [5] tier-2 complex, [6] complex stack 8, [7] tier-2 stack 8,
 * [8] deep point pass (real, stack 3..8), [9] double-double point tier (real, stack <= 2),
 * [10] double-double point tier (complex), [11] double-double point tier (real, stack 3..8),
 * [12] complex tier 2, stack 5..8, [13] candidates the lean grid pass handed to the generic
 * stack-2 kernel (malformed or point-stage-undecided programs; normally 0).              */
int pdeval_pass_counts(pdeval_ctx* ctx, int64_t* counts, int max_counts);

/* Diagnostics (force-free): one program at n_pts points (host arrays), tier-1 (tier2 = 0) or
 * tier-2 arithmetic; out[4p..4p+3] = {|residual|, S, noise bound (tier 2), finite (1/0,
 * -1 = program error)}; jets (may be NULL): 30 doubles per point, the 15 Taylor
 * coefficients of u then their error bounds.  Synchronous; allocates.  Not a hot path.  */
int pdeval_eval_points(pdeval_ctx* ctx, const int32_t* prog, int64_t n_words, const double* xs,
                       const double* ys, int n_pts, int tier2, double* out, double* jets);

/* Diagnostics of the point stage (pdeval_point.h).  pdeval_point_eval: one program at the
 * context's reference points in precision tier 0 (fp64), 1 (complex fp64), 2 (double-double)
 * or 3 (complex double-double); out[6k..6k+5] = {Re res, Im res, |res|, S, noise bound, finite
 * (1/0, -1 = program error)} for each reference point k, *state = the tier's point-stage
 * decision (PDEVAL_PS_* bits).  pdeval_point_states: the point-stage state of every candidate
 * of the most recent validate call (n bytes; synchronizes).  Not hot paths.                 */
#define PDEVAL_PS_PASS    1    /* passed the point stage                                   */
#define PDEVAL_PS_REJECT  2    /* rejected by it (final)                                    */
#define PDEVAL_PS_COMPLEX 4    /* not real at a reference point: complex passes             */
#define PDEVAL_PS_PROV    8    /* fp64 pass within the noise: re-decided in double-double if
                                  the grid rejects                                           */
#define PDEVAL_PS_GRAD    16   /* non-zero gradient at a reference point                    */
#define PDEVAL_PS_DD      32   /* undecided in fp64: decided in double-double               */
int pdeval_point_eval(pdeval_ctx* ctx, const int32_t* prog, int64_t n_words, int tier, double* out,
                      uint8_t* state);
int pdeval_point_states(pdeval_ctx* ctx, uint8_t* out, int64_t n);

/* ---- multi-GPU: the one exchange step ----
 * Candidate batches shard across GPUs with no data-path communication; the per-rank verdict
 * bitmaps are then assembled with one RCCL all-gather over xGMI.  RCCL (librccl.so.1) is
 * loaded on first use, so the library has no link-time dependency on it.
 *   pdeval_comm_unique_id  on one rank: the 128-byte RCCL id, to be shared with every rank
 *   pdeval_comm_init       on every rank (collective): world ranks, this one = rank, on the
 *                          context's GPU
 *   pdeval_gather_bits     d_local: this rank's nbytes (device), d_global: world * nbytes
 *                          (device), rank r's bytes at offset r * nbytes; asynchronous on
 *                          `stream` (NULL = the context's stream)
 *   pdeval_comm_destroy    releases the communicator (also done by pdeval_destroy)        */
#define PDEVAL_UNIQUE_ID_BYTES 128
int pdeval_comm_unique_id(uint8_t* id);
int pdeval_comm_init(pdeval_ctx* ctx, int world, int rank, const uint8_t* id);
int pdeval_gather_bits(pdeval_ctx* ctx, const uint8_t* d_local, int64_t nbytes, uint8_t* d_global, void* stream);
int pdeval_comm_destroy(pdeval_ctx* ctx);

/* Host-side program analysis (no GPU): required stack depth, or < 0 if malformed.      */
int pdeval_program_depth(const int32_t* ops, int64_t n_words);

/* Algorithmic cost model: FP64 flops per grid point for one program.      */
double pdeval_program_flops(int problem_id, const int32_t* ops, int64_t n_words);
/* The part of it the lean grid passes evaluate 64 times per candidate (once per grid row or
 * lane), not per point: the program's hoisted prefix of one coordinate (DESIGN.md §3
 * "Hoisted prefixes"); 0 if none.                                                      */
double pdeval_program_hoist_flops(int problem_id, const int32_t* ops, int64_t n_words);

const char* pdeval_version(void);

/* ---- native candidate compiler (host only, no GPU; pdcompile.cpp) ----
 * Replaces, per candidate, the reference's parse  sp.sympify(expr_str, locals=symbols ∪
 * constants ∪ UNARY_OPS)  (general_method_paper_reproduction.py:84-93, :1257, :1767) plus
 * this build's lowering of the tree (pdeval/flatten.py).  Strings are concatenated in
 * text[str_offsets[i] .. str_offsets[i+1]).  Per string, status[i] is
 *   PDEVAL_COMPILE_OK        program written to ops[offsets[i] .. offsets[i+1])
 *   PDEVAL_COMPILE_DECLINED  outside the SymPy evaluation rules restated natively (floats,
 *                            I/E/pi, log, irrational numeric powers, sign-dependent Abs ...):
 *                            compile this one through SymPy (empty slot)
 *   PDEVAL_COMPILE_PARSE     not an expression (empty slot; SymPy fails on it too)
 * Returns PDEVAL_ERR_ARG (and *n_words_out = -1) if ops_cap words are not enough.       */
#define PDEVAL_COMPILE_OK        0
#define PDEVAL_COMPILE_DECLINED  1
#define PDEVAL_COMPILE_PARSE     2
int pdeval_compile_batch(int problem_id, const char* text, const int64_t* str_offsets, int64_t n,
                         int32_t* ops, int64_t ops_cap, int64_t* offsets, int32_t* status,
                         int64_t* n_words_out);
/* The same, compiled by n_threads host threads (0 = every hardware thread); identical
 * output.  Replaces the per-candidate sympify of the worker (:1767) at the rate one GPU
 * validates.                                                                              */
int pdeval_compile_batch_mt(int problem_id, const char* text, const int64_t* str_offsets, int64_t n,
                            int32_t* ops, int64_t ops_cap, int64_t* offsets, int32_t* status,
                            int64_t* n_words_out, int n_threads);
/* The reference's reason strings of n validated candidates (host only, pdreasons.cpp), as
 * validate() returns them (problems/force_free/validator.py:309-427 "Valid foliation ...",
 * "Invalid (point check ≈ x.xxe±yy)" ...; problems/kerr_magnetosphere/validator.py:231-323),
 * the same texts as pdeval/batch.py::reason_for, newline-separated into buf[0 .. *len_out).
 * rational[i] != 0: det at p* is a rational Number (header PDEVAL_FLAG_RATIONAL).  An
 * UNSUPPORTED row reads "Error: unsupported construct (opcode)".  Returns PDEVAL_ERR_ARG
 * (and *len_out = -1) when cap bytes are not enough.                                       */
int pdeval_format_reasons(int problem_id, int64_t n, const uint8_t* status, const double* res_ref,
                          int n_ref, const double* q_ref, const double* q_grid, const uint8_t* rational,
                          char* buf, int64_t cap, int64_t* len_out);
/* Canonical form of the evaluated expression tree of one string (parity tests against
 * SymPy's tree): returns a PDEVAL_COMPILE_* status, or -1 on a bad argument / small buffer. */
int pdeval_canonical(int problem_id, const char* s, int64_t len, char* out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* PDEVAL_H */
