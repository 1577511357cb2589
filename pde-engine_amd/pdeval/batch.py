"""Batch validation with the reference's verdict semantics.

``BatchValidator.validate_exprs`` is the batched replacement for calling
``validator.validate(u, check_regularity=False, fast_point_only=False, lean_first=True,
defer_heavy_checks=True, enforce_anchor=False)`` once per candidate
(``general_method_paper_reproduction.py:1299-1316`` inline, ``:1768-1782`` worker).  One call
flattens every tree on the host, sends the whole batch through libpdeval.so, and maps each
candidate's class to the reference's ``(bool, reason)`` strings:

force-free (``problems/force_free/validator.py``)
  zero gradient  -> (False, "Zero gradient (constant expression)")                  :309-312
  point reject   -> (False, "Invalid (point check != 0)") for a rational det at p*,  :371-380
                    (False, "Invalid (point check ≈ {|det|:.2e})") otherwise        :388-397
  grid reject    -> (False, "Invalid (Lean could not simplify det to 0 symbolically)") :414-416
  accept         -> (True,  "Valid foliation (Lean: det = 0 symbolically)")           :410-413
Kerr (``problems/kerr_magnetosphere/validator.py``)
  zero gradient  -> (False, "Trivial constant solution excluded")                     :231-240
  point reject   -> (False, "PDE residual != 0 (fast point check) | residual: ...")  :264-269
  grid reject    -> (False, "PDE residual != 0 | residual: ...")                     :308-315
  accept         -> (True,  "Valid (exact zero; heavy checks deferred)")              :318-323
The residual text after "residual:" is numeric here (the reference prints a symbolic
numerator/denominator, which is not reproduced).
"""
from __future__ import annotations

import math
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import sympy as sp

from . import hostpool
from . import problem_defs as P
from . import symbolic as S
from .flatten import Unsupported
from .opcodes import (CLS_ACCEPT, CLS_BAD_PROGRAM, CLS_NONFINITE_REF, CLS_REJECT_GRID,
                      CLS_REJECT_POINT, CLS_REJECT_SYMBOLIC, CLS_UNSUPPORTED, CLS_ZERO_GRADIENT, FLAG_NOCOORD,
                      FLAG_RATIONAL, HAS_IMM, IMM_PRM, OP_NAME, PDOP, PROBLEM_FORCE_FREE, PROBLEM_KERR, op_len)


@dataclass
class Verdict:
    ok: bool
    reason: str
    cls: int
    q_ref: float
    res_ref: Tuple[float, ...]
    q_grid: float
    n_bad: int
    n_nonfinite: int
    fingerprint: Tuple[float, ...]
    evidence: Optional[dict] = None   # Kerr, symbolic 'text' / 'replay': the reference's last_evidence()


def _fmt_point(v: float) -> str:
    return f'Invalid (point check ≈ {abs(v):.2e})'


def reason_for(problem_id: int, cls: int, res_ref: Sequence[float], q_ref: float,
               q_grid: float, rational: bool, note: Optional[str] = None) -> Tuple[bool, str]:
    if problem_id == PROBLEM_FORCE_FREE:
        if cls == CLS_ACCEPT:
            return True, 'Valid foliation (Lean: det = 0 symbolically)'
        if cls == CLS_REJECT_POINT:
            if not np.isfinite(res_ref[0]):
                return False, 'Invalid (point check != 0)'
            return False, 'Invalid (point check != 0)' if rational else _fmt_point(res_ref[0])
        if cls in (CLS_REJECT_GRID, CLS_REJECT_SYMBOLIC):
            return False, 'Invalid (Lean could not simplify det to 0 symbolically)'
        if cls == CLS_ZERO_GRADIENT:
            return False, 'Zero gradient (constant expression)'
        if cls == CLS_NONFINITE_REF:
            return False, 'Could not evaluate point check'
    else:
        if cls == CLS_ACCEPT:
            return True, 'Valid (exact zero; heavy checks deferred)'
        if cls == CLS_REJECT_POINT:
            return False, (f'PDE residual != 0 (fast point check) | residual: '
                           f'max|lhs| at test points ≈ {q_ref:.3e}')
        if cls == CLS_REJECT_GRID:
            return False, f'PDE residual != 0 | residual: max scaled |lhs| on grid ≈ {q_grid:.3e}'
        if cls == CLS_ZERO_GRADIENT:
            return False, 'Trivial constant solution excluded'
        if cls == CLS_NONFINITE_REF:
            return False, 'Invalid (non-real at test point)'
    if cls == CLS_UNSUPPORTED:
        return False, f'Error: unsupported construct ({note or "opcode"})'
    return False, 'Error: malformed program'


def rational_flags(ops, off) -> np.ndarray:
    """Per candidate: header flag PDEVAL_FLAG_RATIONAL (det at p* is a rational Number)."""
    off = np.asarray(off, dtype=np.int64)
    if len(off) < 2:
        return np.zeros(0, dtype=np.uint8)
    hdr = np.asarray(ops, dtype=np.int32)[np.minimum(off[:-1], max(len(ops) - 1, 0))] if len(ops) else \
        np.zeros(len(off) - 1, dtype=np.int32)
    return ((hdr & FLAG_RATIONAL) != 0).astype(np.uint8)


def format_reasons(problem_id: int, status, res_ref, q_ref, q_grid, rational,
                   notes: Optional[Sequence[Optional[str]]] = None) -> List[str]:
    """reason_for over a whole batch, in one native call (pdeval_format_reasons,
    csrc/pdreasons.cpp): the same strings, newline-joined by the library and split once here.
    ``notes[i]`` (UNSUPPORTED stubs) replaces the generic construct name as in reason_for."""
    import ctypes as C
    from ._lib import load, PdevalError
    st = np.ascontiguousarray(status, dtype=np.uint8)
    n = len(st)
    if n == 0:
        return []
    rr = np.ascontiguousarray(res_ref, dtype=np.float64).reshape(n, -1)
    qr = np.ascontiguousarray(q_ref, dtype=np.float64)
    qg = np.ascontiguousarray(q_grid, dtype=np.float64)
    ra = np.ascontiguousarray(rational, dtype=np.uint8)
    cap = 112 * n + 64
    buf = C.create_string_buffer(cap)
    ln = C.c_int64(0)
    rc = load().pdeval_format_reasons(problem_id, n, st.ctypes.data, rr.ctypes.data, rr.shape[1],
                                      qr.ctypes.data, qg.ctypes.data, ra.ctypes.data, buf, cap,
                                      C.byref(ln))
    if rc != 0:
        raise PdevalError(f'pdeval_format_reasons failed ({rc})')
    out = buf.raw[:ln.value].decode('utf-8').split('\n')
    if notes is not None:
        for i in np.flatnonzero(st == CLS_UNSUPPORTED):
            if notes[i]:
                out[i] = f'Error: unsupported construct ({notes[i]})'
    return out


def symbolic_zero_gradient(pd, items, out) -> List[int]:
    """Force-free: the reference's zero-gradient test is symbolic -- ``u.diff(rho) == 0 and
    u.diff(z) == 0`` on SymPy's tree (``problems/force_free/validator.py:305-312``).  SymPy can
    keep a constant u unevaluated while its derivative cancels term by term: in
    ``exp_neg(rho**2 + z**2)*exp(rho**2)*exp(z**2)`` the product stays a product, but the
    product rule gives ``2*rho*P - 2*rho*P`` = 0, so the reference reports "Zero gradient".
    The device sees only values, and its structural test (header NOCOORD) misses such u; a
    constant u whose derivative SymPy does NOT cancel goes on to the determinant, which is 0.
    So the candidates whose value agrees at the 4 fingerprint points (a constant has no other
    way to be) and whose class says the grid was evaluated are re-checked here with the
    reference's own test, and reclassified ZERO_GRADIENT (verdict False) where it holds.
    ``items`` are SymPy trees or candidate strings; ``out`` the result dict of one validate call
    (``status``, ``verdict``, ``fingerprint``), updated in place.  Returns the changed rows."""
    if pd.problem_id != PROBLEM_FORCE_FREE:
        return []
    st = np.asarray(out['status'])
    fp = np.asarray(out['fingerprint'], dtype=np.float64).reshape(len(st), -1)
    with np.errstate(invalid='ignore'):
        flat = (np.all(np.isfinite(fp), axis=1) &
                (fp.max(axis=1) - fp.min(axis=1) <= 1e-9 * np.maximum(np.abs(fp).max(axis=1), 1e-300)) &
                np.isin(st, (CLS_ACCEPT, CLS_REJECT_GRID, CLS_REJECT_SYMBOLIC)))
    idx = np.flatnonzero(flat)
    # each check has a time bound (SymPy's diff of a pathological tree has none of its own); one
    # that hits it keeps the device's class
    if len(idx) and all(isinstance(items[i], str) for i in idx):
        # strings: over the SymPy pool when it runs, even one at a time (the caller's thread then
        # keeps the GIL free for the worker's other pipeline stages)
        zero = hostpool.run(_zero_gradient_str, [(pd.slug, items[i]) for i in idx], min_items=1,
                            item_timeout=HOST_CHECK_TIMEOUT_S, default=False)
    else:
        zero = [hostpool._call_bounded(lambda u: _zero_gradient(pd, u), items[i], HOST_CHECK_TIMEOUT_S, False)
                for i in idx]
    rows = []
    for i, z in zip(idx.tolist(), zero):
        if z:
            st[i] = CLS_ZERO_GRADIENT
            if 'verdict' in out:
                out['verdict'][i] = False
            rows.append(i)
    return rows


def _zero_gradient(pd, u) -> bool:
    """The reference's test on one candidate (tree or string); a tree SymPy cannot
    differentiate keeps its class."""
    try:
        u = u if isinstance(u, sp.Basic) else pd.parse(u)
        return bool(u.diff(pd.x) == 0 and u.diff(pd.y) == 0)
    except Exception:   # noqa: BLE001
        return False


_PDS: Dict[str, object] = {}
# the time bound of one host SymPy check (zero gradient, the Kerr exact point check): the
# reference's own check has none; past it the device's class stands
HOST_CHECK_TIMEOUT_S = 30.0


def _zero_gradient_str(args) -> bool:
    slug, s = args
    if slug not in _PDS:
        _PDS[slug] = P.get(slug)
    return _zero_gradient(_PDS[slug], s)


_NONRATIONAL_OPS = {PDOP['ABS'], PDOP['SQRT'], PDOP['POW'], PDOP['LOG']}
_EXP_OPS = {PDOP['EXP']}


def _has_op(words, codes) -> bool:
    i = 1
    while i < len(words):
        w = int(words[i])
        if (w & 0xff) in codes:
            return True
        i += op_len(w)
    return False


def kerr_symbolic_constant(pd, items, out, ops, off) -> List[int]:
    """Kerr: the reference's constant exclusion is structural -- ``simplify(u)`` has neither r
    nor x (``problems/kerr_magnetosphere/validator.py:231-240``).  The device decides it
    numerically (P0_CONST: u's gradient is rounding noise at every constant-test point), which
    is the same thing for rational and exp combinations, but not for a u that is constant only
    on the domain through an Abs or a fractional power: ``Delta - sqrt(square(Delta))`` is 0
    for every r > r+, yet SymPy keeps ``Abs(Delta)`` and the reference goes on to its symbolic
    stage, which cannot prove lhs == 0 ("PDE residual != 0 | ...").  So the numeric constants
    whose program has an Abs, sqrt, fractional power or log (and that reference a coordinate;
    no coordinate is a constant structurally) are re-checked here with the reference's own test
    and reclassified REJECT_GRID where simplify(u) keeps a coordinate.  Updates ``out`` in
    place; returns the changed rows."""
    if pd.problem_id != PROBLEM_KERR:
        return []
    st = np.asarray(out['status'])
    sel = []
    for i in np.flatnonzero(st == CLS_ZERO_GRADIENT):
        w = ops[off[i]:off[i + 1]]
        if len(w) == 0 or int(w[0]) & FLAG_NOCOORD or not _has_op(w, _NONRATIONAL_OPS):
            continue
        sel.append(int(i))
    if not sel:
        return []
    # SymPy's simplify has no time bound of its own: each check runs with one (over the SymPy
    # pool when it runs, so the worker's pipeline does not stall); a check that hits it keeps
    # the device's class
    if all(isinstance(items[i], str) for i in sel):
        keeps = hostpool.run(_kerr_keeps_coordinate_str, [(pd.slug, items[i]) for i in sel], min_items=1,
                    item_timeout=KERR_SIMPLIFY_TIMEOUT_S, default=None)
    else:
        keeps = [hostpool._call_bounded(lambda u: _kerr_keeps_coordinate(pd, u), items[i],
                                        KERR_SIMPLIFY_TIMEOUT_S, None) for i in sel]
    rows = []
    for i, k in zip(sel, keeps):
        if k:
            st[i] = CLS_REJECT_GRID
            if 'verdict' in out:
                out['verdict'][i] = False
            rows.append(i)
    return rows


KERR_SIMPLIFY_TIMEOUT_S = 30.0


def _kerr_keeps_coordinate(pd, u) -> Optional[bool]:
    """``simplify(u).has(r) or .has(x)`` (kerr validator.py:231-240); None when SymPy fails."""
    try:
        u = u if isinstance(u, sp.Basic) else pd.parse(u)
        us = sp.simplify(u)
        return bool(us.has(pd.x) or us.has(pd.y))
    except Exception:   # noqa: BLE001  (SymPy failed: the device's class stands)
        return None


def _kerr_keeps_coordinate_str(args) -> Optional[bool]:
    slug, s = args
    if slug not in _PDS:
        _PDS[slug] = P.get(slug)
    return _kerr_keeps_coordinate(_PDS[slug], s)


def _has_prm(words) -> bool:
    i = 1
    while i < len(words):
        w = int(words[i])
        if (w & 0xff) in HAS_IMM and w & IMM_PRM:
            return True
        i += op_len(w)
    return False


_KERR_REF_POINTS = ((2.5, 0.6), (7 / 3, 1 / 3), (5.0, -0.4))   # kerr validator.py:168-172


def _fdiv(a: float, b: float) -> float:
    """IEEE division as the device does it: x/0 is +-inf (nan for 0/0), never an exception."""
    if b == 0.0:
        if a != a or a == 0.0:
            return float('nan')
        return math.copysign(math.inf, a) * math.copysign(1.0, b)
    return a / b


_FF_REF_POINT = ((0.8, 6 / 7),)   # force-free p* (validator.py:296-297)


def _exp_overflows(words, prm_values, points=_KERR_REF_POINTS, magnitude: bool = False) -> bool:
    """Does evaluating the program (values only, fp64, host) at a reference point take exp of
    an argument beyond the fp64 range (|arg| > 708: inf, or 0 / a subnormal that a fractional
    power or a product with an overflowed factor turns into inf or 0 * inf)?  The device's point
    stage then sees a non-finite value where the reference's arbitrary-range evaluation sees a
    finite one.  A non-real
    intermediate (sqrt of a negative value) ends that point's evaluation without an answer;
    a division by zero gives +-inf or nan, as on the device, and the evaluation goes on.

    ``magnitude`` (force-free, a point the device found non-finite): True unless a value turns
    non-finite -- a division by an exact zero, a log of 0: a pole at the point, which the
    reference's exact evaluation sees too -- or non-real; every value finite and real means the
    jets' range failed (a coefficient past the device's 2^160 guard: derivatives of e^84 /
    0.0095, or a fractional power of a tiny value: the higher coefficients of sqrt(e^-403))."""
    for x, y in points:
        st: List[float] = []
        acc = 0.0
        try:
            i = 1
            while i < len(words):
                w = int(words[i])
                op = w & 0xff
                n = (w >> 8) & 0xff
                if op in HAS_IMM:
                    if w & IMM_PRM:
                        d = int(words[i + 1])
                        imm = prm_values[d & 7] * (-1.0 if d & 8 else 1.0)
                    else:
                        imm = float(np.array([words[i + 1], words[i + 2]], dtype=np.int32).view(np.float64)[0])
                name = OP_NAME.get(op, '')
                v = y if (w >> 16) & 1 else x
                if name.startswith('PUSH'):
                    st.append(acc)
                    if name == 'PUSH_X':
                        acc = x
                    elif name == 'PUSH_Y':
                        acc = y
                    elif name == 'PUSH_C':
                        acc = imm
                    else:
                        acc = v ** n
                elif name in ('ADD', 'SUB', 'RSUB', 'MUL', 'DIV', 'RDIV'):
                    a = st.pop()
                    if name == 'ADD':
                        acc = a + acc
                    elif name == 'SUB':
                        acc = a - acc
                    elif name == 'RSUB':
                        acc = acc - a
                    elif name == 'MUL':
                        acc = a * acc
                    elif name == 'DIV':
                        acc = _fdiv(a, acc)
                    else:
                        acc = _fdiv(acc, a)
                elif name == 'ADDC':
                    acc = acc + imm
                elif name == 'MULC':
                    acc = acc * imm
                elif name == 'RDIVC':
                    acc = _fdiv(imm, acc)
                elif name == 'NEG':
                    acc = -acc
                elif name in ('ADD_X', 'ADD_Y', 'SUB_X', 'SUB_Y', 'MUL_X', 'MUL_Y', 'DIV_X', 'DIV_Y'):
                    c = x if name.endswith('X') else y
                    if name.startswith('ADD'):
                        acc = acc + c
                    elif name.startswith('SUB'):
                        acc = acc - c
                    elif name.startswith('MUL'):
                        acc = acc * c
                    else:
                        acc = _fdiv(acc, c)
                elif name in ('ADD_P', 'SUB_P', 'MUL_P', 'DIV_P', 'RDIV_P'):
                    p_ = v ** n
                    if name == 'ADD_P':
                        acc = acc + p_
                    elif name == 'SUB_P':
                        acc = acc - p_
                    elif name == 'MUL_P':
                        acc = acc * p_
                    elif name == 'DIV_P':
                        acc = _fdiv(acc, p_)
                    else:
                        acc = _fdiv(p_, acc)
                elif name == 'POWN':
                    acc = acc ** n
                elif name == 'POW':
                    acc = math.pow(acc, imm)
                elif name == 'SQRT':
                    acc = math.sqrt(acc)
                elif name == 'EXP':
                    if abs(acc) > 708.0:    # beyond the fp64 range, or into its subnormals
                        return True
                    acc = math.exp(acc)
                elif name == 'LOG':
                    acc = math.log(acc)
                elif name == 'ABS':
                    acc = abs(acc)
                else:
                    break
                if magnitude and not math.isfinite(acc):
                    return False              # (a pole: the exact value is not finite either)
                i += op_len(w)
        except OverflowError:
            if magnitude:
                return True
            continue
        except (ValueError, ZeroDivisionError, IndexError):
            if magnitude:
                return False                  # (not real there: the complex passes' case)
            continue
        if magnitude:
            # every value finite and real at p*: the device's non-finite point came from the
            # jets' range -- a coefficient past the 2^160 guard (derivatives of e^84 / 0.0095),
            # or a fractional power of a tiny value
            return True
    return False


def ff_range_point_check(pd, items, out, ops, off, n_grid: int, full_grid: bool, max_bad: int) -> List[int]:
    """Force-free point rejects that only the fp64 range caused: the device could not evaluate
    the determinant at p* (a non-finite value, q_ref not > 0) because an intermediate value of
    the program there lies beyond the range its jets tolerate (``exp(exp(rho/(1 - z)))``: e^270;
    ``sqrt(exp_neg(exp(z/(1 - z))))``: sqrt of e^-403, whose higher Taylor coefficients overflow)
    -- while the reference's exact evaluation (validator.py:349-402) finds the value, 0 for a
    true solution.  Found by the host's fp64 value interpreter at p* (_exp_overflows with
    ``magnitude``; a pole at p* is not range trouble and keeps the reject).  The grid stage
    then decides, as after a passing point stage: no more failing points than ``max_bad`` and
    at least one finite point -> ACCEPT, else REJECT_GRID (needs full_grid, which evaluates the
    grid of point rejects).  Measured against the reference's own verdicts on every such row of
    the depth-4 stream and the depth-5 sample (tests/golden/ref/ff_range_rows.jsonl).  Updates
    ``out`` in place; returns the changed rows."""
    if pd.problem_id != PROBLEM_FORCE_FREE or not full_grid:
        return []
    st = np.asarray(out['status'])
    with np.errstate(invalid='ignore'):
        sel = np.flatnonzero((st == CLS_REJECT_POINT) & ~(np.asarray(out['q_ref']) > 0))
    rows = []
    nb = np.asarray(out['n_bad'])
    nn = np.asarray(out['n_nonfinite'])
    off = np.asarray(off)
    for i in sel.tolist():
        if not _exp_overflows(ops[off[i]:off[i + 1]], (0.0,) * 8, _FF_REF_POINT, magnitude=True):
            continue
        ok = int(nb[i]) <= max_bad and n_grid - int(nn[i]) > 0
        st[i] = CLS_ACCEPT if ok else CLS_REJECT_GRID
        if 'verdict' in out:
            out['verdict'][i] = ok
        rows.append(i)
    return rows


def kerr_exact_point_check(pd, kerr, items, out, ops, off, abs_tol: float = 1e-10,
                           n_grid: int = 4096, full_grid: bool = True, max_bad: int = 0) -> List[int]:
    """Kerr point rejects that only the fp64 representation caused, re-checked with the
    reference's own rule (its fast point check substitutes the values into the SYMBOLIC lhs
    and evaluates with N(., 40), kerr validator.py:163-192 -- no fp64 range, and after
    differentiation):
    * a constant whose point-stage value is 0 (a_value = 0): a u that is singular or undefined
      at a = 0 can still pass -- its lhs may not contain a at all (``x + a**(-2)``), or be
      0 * (a finite value) (``a**2/x**(-3/2)`` at x < 0); the device evaluates u itself at the
      point and sees a non-finite value.  Candidates rejected for non-finiteness (rejected with
      max|lhs| below the threshold) whose program uses the constants;
    * an exponential beyond the fp64 range at a reference point: ``exp(r**2/a**2)`` at r = 5,
      a = 1/10 is e^2500, so ``pow_neg_3_2(exp(r**2/a**2)*exp(a**2*x**2))`` is inf * 0 there on
      the device while the reference finds |lhs| ~ 1e-1600 and passes.  Candidates rejected with
      a non-finite value at some reference point and every finite one below the threshold,
      whose program takes exp of an argument beyond +-708 at a reference point
      (_exp_overflows, a host fp64 value interpreter).
    Where the reference's rule passes, the grid stage (evaluated at the stand-ins of the
    symbols; needs full_grid) decides: more failing points than the device's ``max_bad``, or no
    finite point at all (the device's rule), rejects.  Updates ``out`` in place; returns the changed rows."""
    if pd.problem_id != PROBLEM_KERR or kerr is None or not full_grid:
        return []
    st = np.asarray(out['status'])
    rr = np.asarray(out['res_ref'], dtype=np.float64).reshape(len(st), -1)
    with np.errstate(invalid='ignore'):
        fin = np.isfinite(rr)
        q_fin = np.where(fin, np.abs(np.where(fin, rr, 0.0)), 0.0).max(axis=1)
        a0_sel = (st == CLS_REJECT_POINT) & ~(np.asarray(out['q_ref']) >= abs_tol) if kerr.a_num == 0 else \
            np.zeros(len(st), dtype=bool)
        ovf_sel = (st == CLS_REJECT_POINT) & ~fin.all(axis=1) & (q_fin < abs_tol)
    Mv, av = kerr.M_num / kerr.M_den, kerr.a_num / kerr.a_den
    with np.errstate(divide='ignore'):
        prm_pt = [Mv, av] + [float(np.float64(1.0) / np.float64(t)) for t in (Mv, av)] + [Mv * Mv, av * av] + \
                 [float(np.float64(1.0) / np.float64(t * t)) for t in (Mv, av)]
    sel = []
    for i in np.flatnonzero(a0_sel | ovf_sel):
        w = ops[off[i]:off[i + 1]]
        a0 = bool(a0_sel[i]) and _has_prm(w)
        ovf = bool(ovf_sel[i]) and _has_op(w, _EXP_OPS) and _exp_overflows(w, prm_pt)
        if a0 or ovf:
            sel.append(int(i))
    if not sel:
        return []
    # the reference's 3-point check (SymPy diff + N(., 40)) per candidate, with a time bound
    # (over the SymPy pool for strings); one that hits it, or fails, keeps the device's reject
    kspec = (kerr.M_num, kerr.M_den, kerr.a_num, kerr.a_den, bool(kerr.op_M_fixed), bool(kerr.op_a_fixed))
    if all(isinstance(items[i], str) for i in sel):
        passes = hostpool.run(_kerr_point_check_str, [(pd.slug, kspec, items[i], abs_tol) for i in sel],
                              min_items=1, item_timeout=HOST_CHECK_TIMEOUT_S, default=False)
    else:
        passes = [hostpool._call_bounded(lambda u: _kerr_point_check_safe(pd, kspec, u, abs_tol), items[i],
                                         HOST_CHECK_TIMEOUT_S, False) for i in sel]
    rows = []
    for i, ok in zip(sel, passes):
        if not ok:
            continue
        no_grid = int(out['n_nonfinite'][i]) >= n_grid
        st[i] = CLS_REJECT_GRID if (out['n_bad'][i] > max_bad or no_grid) else CLS_ACCEPT
        if 'verdict' in out:
            out['verdict'][i] = st[i] == CLS_ACCEPT
        rows.append(i)
    return rows


def _kerr_point_check_safe(pd, kspec, u, abs_tol) -> bool:
    try:
        u = u if isinstance(u, sp.Basic) else pd.parse(u)
        return _kerr_fast_point_check(pd, kspec, u, abs_tol)
    except Exception:   # noqa: BLE001  (the device's reject stands)
        return False


def _kerr_point_check_str(args) -> bool:
    slug, kspec, s, abs_tol = args
    if slug not in _PDS:
        _PDS[slug] = P.get(slug)
    return _kerr_point_check_safe(_PDS[slug], kspec, s, abs_tol)


def _kerr_fast_point_check(pd, kspec, u, abs_tol) -> bool:
    """kerr validator.py:77-91 (lhs) and :163-192 (the 3-point check) in SymPy.  ``kspec`` =
    (M_num, M_den, a_num, a_den, op_M_fixed, op_a_fixed) of the context's Kerr constants."""
    M_num, M_den, a_num, a_den, op_M_fixed, op_a_fixed = kspec
    r, x = pd.x, pd.y
    M = sp.Rational(M_num, M_den) if op_M_fixed else pd.constants['M']
    a = sp.Rational(a_num, a_den) if op_a_fixed else pd.constants['a']
    G = 1 - (2 * M * r) / (r**2 + a**2 * x**2)
    lhs = sp.diff(G / (1 - x**2) * sp.diff(u, r), r) + sp.diff(G / (r**2 - 2 * M * r + a**2) * sp.diff(u, x), x)
    base = {pd.constants['M']: sp.Rational(M_num, M_den),
            pd.constants['a']: sp.Rational(a_num, a_den)}
    worst, n_ok = 0.0, 0
    for px, py in ((sp.Rational(5, 2), sp.Rational(3, 5)), (sp.Rational(7, 3), sp.Rational(1, 3)),
                   (sp.Integer(5), sp.Rational(-2, 5))):
        try:
            v = sp.N(lhs.subs({**base, r: px, x: py}), 40)
            if v.is_real is False:
                return False
            fv = float(v)
            if fv != fv:
                return False
            worst = max(worst, abs(fv))
            n_ok += 1
        except Exception:   # noqa: BLE001  (the reference skips the point)
            continue
    return n_ok > 0 and worst < abs_tol


SYMBOLIC_MODES = ('off', 'strict', 'text', 'replay')
SYMBOLIC_TIMEOUT_S = 60.0    # per candidate: the limit the reference fixtures were made with


def symbolic_stage(pd, items, out, mode: str = 'text', timeout: float = SYMBOLIC_TIMEOUT_S,
                   kerr=None, omega: str = '0') -> List[int]:
    """Force-free: the reference's symbolic stage replayed on the host (pdeval.symbolic) where
    it decides the verdict or the text (``problems/force_free/validator.py:404-427``):

    * ``text``   -- grid rejects and structural-rule rejects (REJECT_SYMBOLIC): SymPy's det_M and
      its printed length choose between "Invalid (Lean could not simplify det to 0
      symbolically)" and "Invalid (expanded det != 0)";
    * ``replay`` -- also every candidate the grid found zero (ACCEPT, REJECT_SYMBOLIC): the
      reference's symbolic verdict and text replace the device's (its false negatives, e.g. an
      expanded det that keeps sqrt(rho/z) and rho/z apart, become rejects).

    Kerr (``_kerr_symbolic_stage``): the reference's reject texts with their 240-character
    symbolic residual, and its ``last_evidence()`` dict for the candidates that pass the point
    stage; ``replay`` also takes the reference's exact-zero verdict.

    Each candidate runs with a time bound (over the SymPy pool when items are strings); one that
    hits it keeps the device's verdict and text.  Updates ``out`` in place (``status``,
    ``verdict``, ``reason_override``: row -> text, and for Kerr ``evidence``: row -> dict);
    returns the changed rows."""
    if mode not in SYMBOLIC_MODES:
        raise ValueError(f'symbolic mode {mode!r}: one of {SYMBOLIC_MODES}')
    if mode == 'off':
        return []
    if pd.problem_id == PROBLEM_KERR:
        if mode == 'strict':        # (the force-free symbolic stage's shapes; Kerr keeps 'off')
            return []
        return _kerr_symbolic_stage(pd, items, out, mode, timeout, kerr)
    if pd.problem_id != PROBLEM_FORCE_FREE:
        return []
    st = np.asarray(out['status'])
    if mode == 'strict':
        return _strict_stage(pd, items, out, timeout, omega)
    cls = (CLS_REJECT_GRID, CLS_REJECT_SYMBOLIC) if mode == 'text' else (CLS_REJECT_GRID, CLS_ACCEPT, CLS_REJECT_SYMBOLIC)
    sel = np.flatnonzero(np.isin(st, cls)).tolist()
    if not sel:
        return []
    # the reference's symbolic verdict is needed for grid zeros in 'replay' mode only; a grid
    # reject (det not zero) and, in 'text' mode, a structural-rule reject take the branch text
    def need_verdict(c):
        return mode == 'replay' and c != CLS_REJECT_GRID
    args = [(pd.slug, items[i] if isinstance(items[i], str) else None, need_verdict(int(st[i])), omega) for i in sel]
    if all(a[1] is not None for a in args):
        res = hostpool.run(S.replay_str, args, min_items=1, item_timeout=timeout, default=None)
    else:
        om = sp.sympify(omega)
        res = [hostpool._call_bounded(lambda it: S.ff_replay(it[0], pd.x, pd.y, it[1], om),
                             (items[i] if isinstance(items[i], sp.Basic) else pd.parse(items[i]),
                              need_verdict(int(st[i]))), timeout, None) for i in sel]
    ov = out.setdefault('reason_override', {})
    rows = []
    for i, r in zip(sel, res):
        if r is None:
            continue
        ok, text = r
        new = CLS_ACCEPT if ok else (CLS_REJECT_GRID if st[i] == CLS_REJECT_GRID else CLS_REJECT_SYMBOLIC)
        ov[i] = text
        if new != st[i]:
            st[i] = new
            if 'verdict' in out:
                out['verdict'][i] = bool(ok)
        rows.append(i)
    return rows


def _strict_stage(pd, items, out, timeout, omega) -> List[int]:
    """'strict': the grid zeros (ACCEPT, REJECT_SYMBOLIC) of a suspect shape
    (pdeval.symbolic.suspect) get the reference's symbolic verdict and text; every other
    candidate keeps the device's.  One pool task per grid zero: parse, shape test, and the
    replay when suspect, under the per-candidate time bound (past it: the device's verdict).
    ``out['strict']`` receives {'grid_zero', 'suspect', 'replayed', 'timeouts'}."""
    st = np.asarray(out['status'])
    sel = np.flatnonzero(np.isin(st, (CLS_ACCEPT, CLS_REJECT_SYMBOLIC))).tolist()
    stats = out.setdefault('strict', {'grid_zero': 0, 'suspect': 0, 'replayed': 0, 'timeouts': 0})
    stats['grid_zero'] += len(sel)
    if not sel:
        return []
    args = [(pd.slug, items[i] if isinstance(items[i], str) else str(items[i]), omega) for i in sel]
    res = hostpool.run(S.strict_str, args, min_items=1, item_timeout=timeout, default='timeout')
    ov = out.setdefault('reason_override', {})
    rows = []
    for i, r in zip(sel, res):
        if r == 'keep' or r is None:
            continue
        stats['suspect'] += 1
        if r == 'timeout':
            stats['timeouts'] += 1
            continue
        stats['replayed'] += 1
        ok, text = r
        ov[i] = text
        new = CLS_ACCEPT if ok else CLS_REJECT_SYMBOLIC
        if new != st[i]:
            st[i] = new
            if 'verdict' in out:
                out['verdict'][i] = bool(ok)
        rows.append(i)
    return rows


def kerr_operator_spec(pd, kerr) -> Tuple[str, str, str, str]:
    """(M, a) of the Kerr operator -- the problem's symbols, or the numbers a validator was
    built with -- and the values its fast point check substitutes, as strings."""
    Mv = str(sp.Rational(kerr.M_num, kerr.M_den))
    av = str(sp.Rational(kerr.a_num, kerr.a_den))
    return (Mv if kerr.op_M_fixed else 'M', av if kerr.op_a_fixed else 'a', Mv, av)


def _kerr_symbolic_stage(pd, items, out, mode, timeout, kerr) -> List[int]:
    if kerr is None:
        from ._lib import default_kerr_constants
        kerr = default_kerr_constants()
    spec = kerr_operator_spec(pd, kerr)
    st = np.asarray(out['status'])
    code = {CLS_REJECT_POINT: 1, CLS_REJECT_GRID: 2, CLS_ACCEPT: 0}
    sel = [i for i in range(len(st)) if int(st[i]) in code]
    if not sel:
        return []
    strs = [items[i] if isinstance(items[i], str) else str(items[i]) for i in sel]
    args = [(s_, code[int(st[i])], spec) for s_, i in zip(strs, sel)]
    res = hostpool.run(S.kerr_text, args, min_items=1, item_timeout=timeout, default=None)
    ov = out.setdefault('reason_override', {})
    evid = out.setdefault('evidence', {})
    rows = []
    for i, r in zip(sel, res):
        if r is None:
            continue
        text, ev, zero = r
        if ev is not None:
            evid[i] = ev
        if mode == 'replay' and int(st[i]) == CLS_ACCEPT and zero is False:
            st[i] = CLS_REJECT_GRID
            if 'verdict' in out:
                out['verdict'][i] = False
        if text is not None and int(st[i]) != CLS_ACCEPT:
            ov[i] = text
        rows.append(i)
    return rows


def apply_host_steps(pd, kerr, params, n_grid: int, items, r, ops, off, symbolic: str = 'off',
                     symbolic_timeout: float = SYMBOLIC_TIMEOUT_S, omega: str = '0'):
    """The host steps every device result goes through (in place): the symbolic zero-gradient
    re-check (force-free), the structural constant re-check of numeric constants with an Abs
    or fractional power (Kerr), the reference's exact point check for Kerr values beyond the
    fp64 range, and (``symbolic`` != 'off') the replay of the reference's symbolic stage.
    ``r`` is one validate call's outputs (``status``, ``verdict``, ``res_ref``, ``q_ref``,
    ``n_bad``, ``n_nonfinite``, ``fingerprint``); ``n_grid`` the grid's point count.  Needs no
    GPU: the multi-rank path runs it per shard before the gather (pdeval.shard.final_verdicts)."""
    ff_range_point_check(pd, items, r, ops, off, n_grid, bool(params.full_grid), int(params.max_bad))
    symbolic_zero_gradient(pd, items, r)
    kerr_symbolic_constant(pd, items, r, ops, off)
    kerr_exact_point_check(pd, kerr, items, r, ops, off, params.kerr_abs_tol, n_grid, bool(params.full_grid),
                           int(params.max_bad))
    if symbolic != 'off' and (params.full_grid or pd.problem_id == PROBLEM_KERR):
        symbolic_stage(pd, items, r, symbolic, symbolic_timeout, kerr, omega=omega)
    return r


class BatchValidator:
    """One problem on one GPU.  Thread-safe (calls are serialized per context).

    ``symbolic``: the host replay of the reference's symbolic stage (``symbolic_stage``):
    'off' (the device's verdicts and texts), 'text' (grid rejects get the reference's branch
    text) or 'replay' (the reference's symbolic verdicts too)."""

    def __init__(self, problem: str = 'force_free', device: int = 0, params=None, kerr=None,
                 symbolic: str = 'off', symbolic_timeout: float = SYMBOLIC_TIMEOUT_S, omega: str = '0'):
        from ._lib import Context, default_params, default_kerr_constants
        self.pd = P.get(problem)
        self.device = device
        self.kerr = kerr if kerr is not None or self.pd.problem_id != PROBLEM_KERR else default_kerr_constants()
        self.ctx = Context(self.pd.problem_id, device=device, kerr=kerr)
        self.params = params if params is not None else default_params(self.pd.problem_id)
        # force-free, rotating field lines: Omega (a constant whose square is rational, as a
        # string: omega2_value) -> params.omega2 + omega2_lo (validator.py:326-329)
        self.omega = omega
        if self.pd.problem_id == PROBLEM_FORCE_FREE:
            self.params.omega2, self.params.omega2_lo = omega2_value(omega)
        if symbolic not in SYMBOLIC_MODES:
            raise ValueError(f'symbolic mode {symbolic!r}: one of {SYMBOLIC_MODES}')
        self.symbolic = symbolic
        self.symbolic_timeout = symbolic_timeout
        self._lock = threading.Lock()

    @property
    def problem_id(self) -> int:
        return self.pd.problem_id

    def compile(self, exprs: Sequence[sp.Basic]):
        return P.compile_exprs(self.pd, exprs)

    def run(self, ops, offsets):
        with self._lock:
            return self.ctx.validate(ops, offsets, self.params)

    def validate_exprs(self, exprs: Sequence[sp.Basic], symbolic: Optional[str] = None,
                       symbolic_timeout: Optional[float] = None) -> List[Verdict]:
        if not exprs:
            return []
        ops, off, notes = self.compile(exprs)
        return self._verdicts(ops, off, notes, exprs, symbolic, symbolic_timeout)

    def host_steps(self, r, ops, off, items, symbolic: Optional[str] = None,
                   symbolic_timeout: Optional[float] = None):
        """The host steps every device result goes through (in place): :func:`apply_host_steps`
        with this validator's problem, constants and mode."""
        return apply_host_steps(self.pd, self.kerr, self.params, self.ctx.n_points - self.ctx.n_ref, items, r,
                                ops, off, self.symbolic if symbolic is None else symbolic,
                                self.symbolic_timeout if symbolic_timeout is None else symbolic_timeout,
                                self.omega)

    def table(self, r, ops, off, notes) -> dict:
        """Device result (after host_steps) -> {'ok': bool array, 'reasons': list of str} plus
        the raw outputs: the reference's (bool, reason) of every candidate, vectorized."""
        st = np.asarray(r['status'])
        reasons = format_reasons(self.problem_id, st, r['res_ref'], r['q_ref'], r['q_grid'],
                                 rational_flags(ops, off), notes)
        for i, text in r.get('reason_override', {}).items():
            reasons[i] = text
        return {**r, 'ok': st == CLS_ACCEPT, 'reasons': reasons}

    def _verdicts(self, ops, off, notes, items, symbolic: Optional[str] = None,
                  symbolic_timeout: Optional[float] = None) -> List[Verdict]:
        r = self.host_steps(self.run(ops, off), ops, off, items, symbolic, symbolic_timeout)
        t = self.table(r, ops, off, notes)
        ok, reasons = t['ok'].tolist(), t['reasons']
        st, qr, qg = r['status'].tolist(), r['q_ref'].tolist(), r['q_grid'].tolist()
        rr, fp = r['res_ref'].tolist(), r['fingerprint'].tolist()
        nb, nn = r['n_bad'].tolist(), r['n_nonfinite'].tolist()
        ev = r.get('evidence', {})
        return [Verdict(ok[i], reasons[i], st[i], qr[i], tuple(rr[i]), qg[i], nb[i], nn[i], tuple(fp[i]),
                        ev.get(i)) for i in range(len(st))]

    # ---- the worker's fast path in three phases (pdeval/worker.py pipelines them):
    # prepare (host threads, GIL released in the native compiler), run (one device call,
    # GIL released), finish (host steps + vectorized reasons)
    def prepare_strings(self, strings: Sequence[str]) -> dict:
        from .native import compile_strings
        stats: dict = {}
        ops, off, notes = compile_strings(self.pd, list(strings), stats=stats)
        return {'strings': list(strings), 'ops': ops, 'off': off, 'notes': notes,
                'compile_status': stats.get('status')}

    def run_prepared(self, p: dict):
        return self.run(p['ops'], p['off'])

    def finish(self, p: dict, r, symbolic: Optional[str] = None, symbolic_timeout: Optional[float] = None) -> dict:
        r = self.host_steps(r, p['ops'], p['off'], p['strings'], symbolic, symbolic_timeout)
        return self.table(r, p['ops'], p['off'], p['notes'])

    def validate_strings(self, strings: Sequence[str], stats: Optional[dict] = None,
                         symbolic: Optional[str] = None, symbolic_timeout: Optional[float] = None) -> List[Verdict]:
        """Candidate strings in: compiled by the native compiler (csrc/pdcompile.cpp), SymPy
        only for the strings it declines (pdeval/native.py); unparsable strings get the
        UNSUPPORTED stub and an "Error: ..." reason, as on the SymPy path.  ``stats`` receives
        the compile statistics and the native per-string status (native.compile_strings)."""
        if not strings:
            return []
        from .native import compile_strings
        ops, off, notes = compile_strings(self.pd, list(strings), stats=stats)
        return self._verdicts(ops, off, notes, list(strings), symbolic, symbolic_timeout)

    def close(self):
        self.ctx.close()


_VALIDATORS: Dict[tuple, BatchValidator] = {}
_VLOCK = threading.Lock()


def omega2_value(omega) -> Tuple[float, float]:
    """Omega**2 of the force-free rotating constraint as a double-double (hi, lo), hi the
    nearest double and lo = the rest rounded: Omega a constant whose square is rational (1, 2,
    1/2, sqrt(2), 1/3, sqrt(2)/3, ...).  The grid stages take hi; the point stage's
    double-double tier takes hi + lo, which carries a square that is no double (1/9) to 2^-106
    relative, and its error bounds carry that representation error (pdeval_point.h om2_err).
    A Float Omega is its exact binary value.  A symbolic Omega (the reference allows a function
    of u, validator.py:45) or an irrational square raises NotImplementedError."""
    w = sp.sympify(omega)
    if w.free_symbols:
        raise NotImplementedError(f'Omega = {omega!r}: only a constant Omega is implemented')
    if w.is_Float:
        w = sp.Rational(w)
    w2 = sp.simplify(sp.expand(w ** 2))
    if not w2.is_Rational:
        raise NotImplementedError(f'Omega = {omega!r}: Omega**2 must be rational')
    hi = float(w2)
    lo = float(w2 - sp.Rational(hi))
    return hi, lo


def get_validator(problem: str, device: int = 0, kerr=None, omega: str = '0') -> BatchValidator:
    """Process-wide BatchValidator per (problem, device, Kerr constants, force-free Omega): one
    libpdeval context per GPU and parameter set.  (The symbolic host mode is chosen per call by
    the plugins.)"""
    key = (P.get(problem).slug, device, kerr.key() if kerr is not None else None, str(omega))
    with _VLOCK:
        if key not in _VALIDATORS:
            _VALIDATORS[key] = BatchValidator(problem, device, kerr=kerr, omega=str(omega))
        return _VALIDATORS[key]
