"""The reference's symbolic stage, replayed on the host in SymPy for the candidates whose
verdict or reason text it decides (force-free).

The device decides the point stage exactly and replaces the reference's symbolic proof of
``det == 0`` by the 64 x 64 grid.  The two agree except where the
reference's symbolic stage is not a proof procedure:

* **the branch** (``problems/force_free/validator.py:404-427``): ``len(str(det_M)) < 3000`` ->
  the "Lean" normalizer, whose text is "Valid foliation (Lean: det = 0 symbolically)" /
  "Invalid (Lean could not simplify det to 0 symbolically)"; otherwise ``expand(det_M) == 0``
  with "Valid foliation (expanded det = 0)" / "Invalid (expanded det != 0)" (and "Could not
  simplify det symbolically" if expand raises).  Which one runs depends on the printed length
  of SymPy's determinant -- ``det(Matrix(...))`` applies ``dotprodsimp`` to ``a*d - b*c``
  (``sympy/matrices/determinant.py``), so only SymPy's own det gives that length;
* **its false negatives**: the normalizer round-trips the det through a string (losing the
  ``positive`` / ``real`` assumptions of rho and z, ``_simplify_with_lean`` :224-258 ->
  ``LeanNormalizer.normalize`` ``lean_normalizer/lean_bridge.py:67-112``), and ``expand`` does
  not combine ``sqrt(rho/z)`` with ``rho/z``; a true solution can then be rejected, e.g.
  ``exp_neg(rho/z - sqrt(rho/z))`` ("Invalid (expanded det != 0)").

Two host steps restate it (SymPy, per candidate, each with a time bound; a candidate whose
replay hits the bound keeps the device's verdict and text):

* ``text``   -- for grid rejects: SymPy's det_M and its printed length choose the text
  (the verdict is already False: a det that is non-zero on the grid is non-zero);
* ``strict`` -- the reference's symbolic verdict and text only for the grid zeros of the
  shapes where it is known to differ from det == 0 (:func:`suspect`); the throughput mode with
  the reference's verdicts on every decided depth-4 and depth-5 fixture row;
* ``replay`` -- additionally, for every candidate the device accepts or rejects by a
  structural rule (REJECT_SYMBOLIC): the reference's whole symbolic stage on SymPy's det_M,
  including the normalizer's 5 s wall-clock fallback to ``expand(det_M)``
  (``validator.py:241-245``, which makes the reference's verdict depend on machine speed).

Kerr (``problems/kerr_magnetosphere/validator.py``): the reference's reject texts carry a
240-character SymPy repr of the symbolic residual, ``numer/denom`` of ``lhs``
(``_short_residual_repr`` :249-261), and its ``last_evidence()`` -- written into the run
table's ``validator_evidence`` column by the inline driver (``general_method_paper_reproduction.py
:1324-1365``) -- is the dict ``{lhs_string, lean_normalized, sympy_simplified_is_zero, params}``
of the last candidate that passed its fast point check (:296-306).  ``kerr_lhs``,
``short_residual_repr`` and ``kerr_evidence`` restate them (the ``text`` mode of the Kerr host
step).

Nothing here is used to decide the point stage or the grid; it only reproduces which of the
reference's texts (and, in ``replay``, which symbolic verdict) a candidate gets.
"""
from __future__ import annotations

import time
from typing import Dict, Optional, Tuple

import sympy as sp

DET_STR_LIMIT = 3000        # validator.py:408
LEAN_STR_LIMIT = 10000      # validator.py:237
LEAN_TIMEOUT_S = 5.0        # validator.py:224 (timeout), :243-245

TEXT_LEAN_OK = 'Valid foliation (Lean: det = 0 symbolically)'
TEXT_LEAN_FAIL = 'Invalid (Lean could not simplify det to 0 symbolically)'
TEXT_EXPAND_OK = 'Valid foliation (expanded det = 0)'
TEXT_EXPAND_FAIL = 'Invalid (expanded det != 0)'
TEXT_EXPAND_ERR = 'Could not simplify det symbolically'


def ff_det(u: sp.Basic, rho: sp.Symbol, z: sp.Symbol, Omega: sp.Basic = sp.Integer(0)) -> Optional[sp.Basic]:
    """SymPy's det_M for u, built in the reference's order (validator.py:305-347, the rotating
    form :326-329 when Omega != 0); None for a zero gradient (the reference stops there)."""
    u_r = u.diff(rho)
    u_z = u.diff(z)
    if u_r == 0 and u_z == 0:
        return None
    if Omega != 0:
        A = (1 - rho**2 * Omega**2) * (u_r.diff(rho) + u_z.diff(z)) - (1 + rho**2 * Omega**2) / rho * u_r
        B = (1 - rho**2 * Omega**2) * (u_r**2 + u_z**2)
    else:
        A = u_r.diff(rho) + u_z.diff(z) - u_r / rho
        B = u_r**2 + u_z**2

    def lie(f):
        return u_z * f.diff(rho) - u_r * f.diff(z)
    la, lb = lie(A), lie(B)
    return sp.det(sp.Matrix([[la, lb], [lie(la), lie(lb)]]))


def _normalize(s: str) -> str:
    """LeanNormalizer.normalize (lean_bridge.py:67-112): sympify WITHOUT locals (plain
    symbols: the assumptions are lost), expand, collect in rho and z when both occur, the five
    substitution rules, str; the input string itself if anything raises."""
    try:
        e = sp.expand(sp.sympify(s))
        R, Z = sp.Symbol('rho'), sp.Symbol('z')
        if e.has(R) and e.has(Z):
            e = sp.collect(e, [R, Z])
        rp, zz = sp.Symbol('rho', positive=True), sp.Symbol('z')
        for pat, rep in ((sp.exp(sp.log(rp)), rp), (sp.log(sp.exp(zz)), zz), (sp.sqrt(rp**2), rp),
                         (rp / rp, 1), (zz - zz, 0)):
            e = e.subs(pat, rep)
        return str(e)
    except Exception:   # noqa: BLE001  (normalize's bare except)
        return s


def _lean_is_zero(det_M: sp.Basic, det_str: str) -> bool:
    """_simplify_with_lean(det_M) == 0 (validator.py:224-258), use_lean on."""
    try:
        if len(det_str) > LEAN_STR_LIMIT:
            return sp.expand(det_M) == 0
        t0 = time.time()
        n = _normalize(det_str)
        if time.time() - t0 > LEAN_TIMEOUT_S:
            return sp.expand(det_M) == 0
        if n.strip() == '0':
            return True
        return sp.sympify(n) == 0
    except Exception:   # noqa: BLE001  (the reference falls back to expand)
        try:
            return sp.expand(det_M) == 0
        except Exception:   # noqa: BLE001
            return False


def ff_symbolic_stage(det_M: sp.Basic, verdict: bool = True) -> Tuple[bool, str]:
    """The reference's symbolic stage on det_M (validator.py:404-427).  ``verdict=False``:
    only the branch's reject text (the caller knows det is not identically zero)."""
    s = str(det_M)
    if len(s) < DET_STR_LIMIT:
        if verdict and _lean_is_zero(det_M, s):
            return True, TEXT_LEAN_OK
        return False, TEXT_LEAN_FAIL
    if not verdict:
        return False, TEXT_EXPAND_FAIL
    try:
        if sp.expand(det_M) == 0:
            return True, TEXT_EXPAND_OK
        return False, TEXT_EXPAND_FAIL
    except Exception:   # noqa: BLE001
        return False, TEXT_EXPAND_ERR


def ff_replay(u: sp.Basic, rho: sp.Symbol, z: sp.Symbol, verdict: bool = True,
              Omega: sp.Basic = sp.Integer(0)) -> Optional[Tuple[bool, str]]:
    """(ok, reason) of the reference's symbolic stage for a candidate that passed its point
    stage; None if SymPy fails (the device's verdict stands)."""
    try:
        det_M = ff_det(u, rho, z, Omega)
        if det_M is None:
            return None
        return ff_symbolic_stage(det_M, verdict)
    except Exception:   # noqa: BLE001
        return None


def ff_point_stage(u: sp.Basic, rho: sp.Symbol, z: sp.Symbol,
                   point=(sp.Rational(4, 5), sp.Rational(6, 7))) -> Optional[Tuple[bool, str]]:
    """The reference's point stage in SymPy (validator.py:349-402, fast_point_only off):
    ``det_M.subs(p*)``, ``cancel(together(.))`` -- a Number decides it ("point check != 0") --
    then ``simplify`` and ``abs(complex(evalf(50)))``: below 1e-20 it passes to the symbolic
    stage (None here), else "Invalid (point check ≈ {:.2e})".

    The device decides the point stage from the exact value of det_M at p* (double-double
    tier), which is what ``det_M.subs(p*).evalf(50)`` gives.  SymPy's ``cancel``/``simplify``
    of the substituted (radical-laden) number can return a different number -- a
    point-check text the reference prints that is not the value of its own det at p*
    (golden_data.FF_D5_POINT_TEXT_DIVERGENCE).  Not used by any mode: at seconds per candidate
    it is for pinning such rows in tests."""
    det_M = ff_det(u, rho, z)
    if det_M is None:
        return None
    v = det_M.subs({rho: point[0], z: point[1]})
    s = sp.cancel(sp.together(v))
    if s.is_Number:
        return None if s == 0 else (False, 'Invalid (point check != 0)')
    s = sp.simplify(s)
    d = abs(complex(s.evalf(50)))
    return None if d < 1e-20 else (False, f'Invalid (point check ≈ {d:.2e})')


FF_POINT = (sp.Rational(4, 5), sp.Rational(6, 7))   # validator.py:296-297


def ff_point_exact(u: sp.Basic, rho: sp.Symbol, z: sp.Symbol, Omega: sp.Basic = sp.Integer(0),
                   point=FF_POINT) -> Optional[Tuple[bool, str]]:
    """The reference's zero-gradient test and point stage, statement for statement
    (validator.py:305-312, :349-402 with fast_point_only off): None when the point stage
    passes (the symbolic stage comes next), else the reference's (False, reason) -- "Zero
    gradient (constant expression)", "Invalid (point check != 0)" for a non-zero Number after
    ``cancel(together(.))`` (nan included), "Invalid (point check ≈ {:.2e})" from
    ``complex(evalf(50))`` (inf and nan included), "Could not evaluate point check" when that
    evaluation raises.  Exceptions of the cheap reductions are swallowed, as there.  For the
    force-free point rejects the device could not evaluate at p* (pdeval.batch.ff_exact_point_check)."""
    det_M = ff_det(u, rho, z, Omega)
    if det_M is None:
        return False, 'Zero gradient (constant expression)'
    s = det_M.subs({rho: point[0], z: point[1]})
    try:
        s = sp.cancel(sp.together(s))
        if s.is_Number and s != 0:
            return False, 'Invalid (point check != 0)'
        s = sp.simplify(s)
    except Exception:   # noqa: BLE001
        pass
    try:
        d = abs(complex(s.evalf(50)))
    except Exception:   # noqa: BLE001
        return False, 'Could not evaluate point check'
    return None if d < 1e-20 else (False, f'Invalid (point check ≈ {d:.2e})')


def ff_point_exact_str(args):
    """ff_point_exact of a candidate string in a SymPy pool process: ``(slug, expr_str[,
    Omega])`` -> 'pass', or the reference's (False, reason); None if SymPy fails."""
    slug, s = args[:2]
    omega = sp.sympify(args[2]) if len(args) > 2 else sp.Integer(0)
    from . import problem_defs as P
    if slug not in _PDS:
        _PDS[slug] = P.get(slug)
    pd = _PDS[slug]
    try:
        r = ff_point_exact(pd.parse(s), pd.x, pd.y, omega)
    except Exception:   # noqa: BLE001
        return None
    return 'pass' if r is None else r


# ------------------------------------------------------------------ 'strict': targeted replay
def suspect(u: sp.Basic, rho: sp.Symbol, z: sp.Symbol) -> bool:
    """The shapes in which the reference's symbolic stage disagrees with det == 0 on the grid,
    or in which the structural rules (NONSMOOTH2D, UNPROVABLE) stand in for it -- the only
    candidates the 'strict' mode replays (fitted to every decided depth-4
    and depth-5 reference row):
      * an Abs anywhere (SymPy's Abs of real expressions: sqrt(square(.)), ((.)**2)**(p/2));
      * a fractional power of a power (sqrt(1/(1 - z)), ((.)**2)**(3/2)) or of an exp
        (exp(g)**(9/4));
      * inside an exp, a fractional power whose base also occurs on its own
        (exp(sqrt(rho/z) - rho/z): expand keeps sqrt(rho/z) and rho/z apart).
    Every other grid zero keeps the device's verdict."""
    for e in sp.preorder_traversal(u):
        if isinstance(e, sp.Abs):
            return True
        if isinstance(e, sp.Pow) and not e.exp.is_Integer and e.base.has(rho, z):
            if isinstance(e.base, (sp.Pow, sp.exp, sp.Abs)):
                return True
        if isinstance(e, sp.exp):
            arg = e.args[0]
            for f in sp.preorder_traversal(arg):
                if isinstance(f, sp.Pow) and not f.exp.is_Integer and f.base.has(rho, z):
                    b = f.base
                    if sum(1 for g in sp.preorder_traversal(u) if g == b) >= 2:
                        return True
    return False


# the string forms through which a candidate's SymPy tree can get a non-integer power or an Abs
# (the only nodes suspect() looks for): the unary ops whose exponent is fractional, sqrt,
# an explicit Abs, a parenthesised exponent (p/q), a float
_SUSPECT_TOKENS = ('sqrt', 'pow_3_2', 'pow_neg_3_2', 'Abs', '**(', '.')


def may_be_suspect(s: str) -> bool:
    """A necessary condition for :func:`suspect` on the candidate string, without SymPy: a
    string with none of these tokens parses to a tree of integer powers, exp and the four
    arithmetic operations only, which suspect() never flags (the streaming strict mode,
    pdeval.worker, keeps the device's verdict for it without a pool round trip)."""
    return any(t in s for t in _SUSPECT_TOKENS)


_PDS: Dict[str, object] = {}


def strict_str(args) -> Optional[Tuple[bool, str]]:
    """'strict' mode for one grid-zero candidate string, in a SymPy pool process:
    ``(slug, expr_str[, Omega])`` -> the reference's symbolic verdict and text if the candidate
    is :func:`suspect`, else ``'keep'`` (the device's verdict stands); None if SymPy fails."""
    slug, s = args[:2]
    omega = sp.sympify(args[2]) if len(args) > 2 else sp.Integer(0)
    from . import problem_defs as P
    if slug not in _PDS:
        _PDS[slug] = P.get(slug)
    pd = _PDS[slug]
    try:
        u = pd.parse(s)
        if not suspect(u, pd.x, pd.y):
            return 'keep'
    except Exception:   # noqa: BLE001
        return None
    return ff_replay(u, pd.x, pd.y, True, omega)


def replay_str(args) -> Optional[Tuple[bool, str]]:
    """ff_replay of a candidate string, in a SymPy pool process (pdeval.hostpool.run):
    ``(slug, expr_str, verdict[, Omega])``; parsed with the driver's sympify locals
    (general_method_paper_reproduction.py:84-93)."""
    slug, s, verdict = args[:3]
    omega = sp.sympify(args[3]) if len(args) > 3 else sp.Integer(0)
    from . import problem_defs as P
    if slug not in _PDS:
        _PDS[slug] = P.get(slug)
    pd = _PDS[slug]
    try:
        u = pd.parse(s)
    except Exception:   # noqa: BLE001
        return None
    return ff_replay(u, pd.x, pd.y, verdict, omega)


# ------------------------------------------------------------------ Kerr (text mode)
KERR_LEAN_STR_MAX = 12000     # kerr validator.py:39 (lean_det_str_max_len)
KERR_EVIDENCE_STR_MAX = 4000  # :302


def kerr_lhs(u: sp.Basic, r, x, M, a) -> sp.Basic:
    """The reference's residual (kerr validator.py:69-91), in its order: no simplification."""
    Delta = r**2 - 2 * M * r + a**2
    G = 1 - (2 * M * r) / (r**2 + a**2 * x**2)
    ur = sp.diff(u, r)
    ux = sp.diff(u, x)
    return sp.diff(G / (1 - x**2) * ur, r) + sp.diff(G / Delta * ux, x)


def short_residual_repr(expr: sp.Basic) -> str:
    """_short_residual_repr (kerr validator.py:249-261): derivatives replaced by a symbol d,
    then ``sstr(numer)/sstr(denom)``, cut to 240 characters."""
    try:
        s_expr = expr.replace(lambda e: isinstance(e, sp.Derivative), lambda e: sp.Symbol('d'))
        num, den = sp.as_numer_denom(s_expr)
        return f"{sp.sstr(num)}/{sp.sstr(den)}"[:240]
    except Exception:   # noqa: BLE001
        try:
            return sp.sstr(expr)[:240]
        except Exception:   # noqa: BLE001
            return '<residual-unavailable>'


def kerr_evidence(lhs: sp.Basic, M_value, a_value, use_lean: bool = True) -> Tuple[dict, bool]:
    """The reference's symbolic stage after a passed fast point check (kerr validator.py
    :283-306): the "Lean" normal form of str(lhs) when it is at most 12,000 characters, then,
    unless that is '0', ``together(cancel(lhs)) == 0 or simplify(.) == 0``.  Returns
    (last_evidence dict, exact zero)."""
    normalized = None
    lean_zero = sympy_zero = False
    if use_lean:
        s = str(lhs)
        if len(s) <= KERR_LEAN_STR_MAX:
            normalized = _normalize(s)
            lean_zero = normalized.strip() == '0'
    if not lean_zero:
        try:
            q = sp.together(sp.cancel(lhs))
            sympy_zero = bool((q == 0) or (sp.simplify(q) == 0))
        except Exception:   # noqa: BLE001
            sympy_zero = False
    try:
        lhs_str = str(lhs)
    except Exception:   # noqa: BLE001
        lhs_str = '<lhs-string-error>'
    ev = {'lhs_string': lhs_str if len(lhs_str) <= KERR_EVIDENCE_STR_MAX
          else lhs_str[:KERR_EVIDENCE_STR_MAX] + '...truncated...',
          'lean_normalized': normalized,
          'sympy_simplified_is_zero': bool(sympy_zero),
          'params': {'M': str(M_value), 'a': str(a_value)}}
    return ev, bool(lean_zero or sympy_zero)


def kerr_text(args):
    """Kerr host step for one candidate, in a SymPy pool process: ``(expr_str, cls, spec)``
    with spec = (M_op, a_op, M_value, a_value) as strings (the validator's operator symbols or
    numbers, and the values its fast point check substitutes) -> (reason, evidence or None,
    exact zero or None).  cls: 1 point reject, 2 grid reject, 0 accept."""
    s, cls, spec = args
    from . import problem_defs as P
    pd = _PDS.get('kerr_magnetosphere') or _PDS.setdefault('kerr_magnetosphere', P.get('kerr_magnetosphere'))
    try:
        u = pd.parse(s)
        loc = {**pd.constants}
        M_op, a_op = sp.sympify(spec[0], locals=loc), sp.sympify(spec[1], locals=loc)
        lhs = kerr_lhs(u, pd.x, pd.y, M_op, a_op)
        if cls == 1:
            return f"PDE residual != 0 (fast point check) | residual: {short_residual_repr(lhs)[:240]}", None, None
        ev, zero = kerr_evidence(lhs, spec[2], spec[3])
        if cls == 2 or not zero:
            return f"PDE residual != 0 | residual: {short_residual_repr(lhs)[:240]}", ev, zero
        return None, ev, zero
    except Exception:   # noqa: BLE001
        return None
