"""The driver's pre-validate filters, parallel on the host.

Between the enumerator and ``validate`` the reference's inline path does, per streamed
candidate string, in stream order (``general_method_paper_reproduction.py:1252-1294``):

1. parse with the driver's locals and drop the candidate if ``_has_degenerate_denominator``
   (``:134-199``) holds; the same on the plain ``sympify(s)`` (no locals);
2. key it by ``normalized = str(simplify(expand(sympify(s))))`` with
   ``signature = int(sha256(normalized)[:8], 16)`` and insert the row; the run table's
   ``normalized`` column is UNIQUE, so a later candidate with a key already seen is not
   inserted (``:1277-1286``);
3. skip constant-only candidates (no coordinate symbol) before ``validate`` (``:1292-1294``).

Steps 1 and 2 are pure SymPy per candidate and dominate the depth-4 wall time on the host (the
``simplify`` of every denominator and of every expanded candidate); here they run over the
forked SymPy pool (``pdeval.hostpool``) in chunks, and the order-dependent part -- the UNIQUE
dedupe -- runs afterwards in stream order, so the surviving rows, their keys and signatures are
the reference's.  No GPU is involved.  ``tests/test_prefilter.py`` pins it against the
reference-generated fixtures (``tests/golden/streams/*_validated.txt.gz``, made by
``tests/golden/gen_reference_verdicts.py --mode filters`` from the reference itself).
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, NamedTuple, Optional, Sequence, Tuple

import sympy as sp

_INF = (sp.zoo, sp.oo, -sp.oo, sp.nan)


def _simplifies_to_zero(e: sp.Basic) -> bool:
    try:
        return sp.simplify(e) == 0
    except Exception:   # noqa: BLE001  (the reference skips a node whose simplify raises)
        return False


def _node_degenerate(sub: sp.Basic) -> bool:
    """One node of the traversal (``:152-195``)."""
    try:
        if sub.has(*_INF):
            return True
    except Exception:   # noqa: BLE001
        pass
    # a negative integer power is a denominator of its base: (1 - 1)**-1
    if isinstance(sub, sp.Pow) and getattr(sub.exp, 'is_integer', False) and bool(sub.exp.is_negative):
        if _simplifies_to_zero(sub.base):
            return True
    try:
        joined = sp.together(sub)
    except Exception:   # noqa: BLE001
        joined = sub
    try:
        _, den = sp.fraction(joined)
    except Exception:   # noqa: BLE001
        try:
            _, den = sp.fraction(sub)
        except Exception:   # noqa: BLE001
            return False
    if den is None or den == 1:
        return False
    return _simplifies_to_zero(den)


def has_degenerate_denominator(expr: sp.Basic) -> bool:
    """True if the expression or any subexpression (preorder) is infinite / NaN, or has a
    denominator -- an explicit negative integer power's base, or the denominator ``fraction``
    finds after ``together`` -- that ``simplify`` reduces to 0 (``:134-199``)."""
    try:
        try:
            if expr.has(*_INF):
                return True
        except Exception:   # noqa: BLE001
            pass
        for sub in sp.preorder_traversal(expr):
            try:
                if _node_degenerate(sub):
                    return True
            except Exception:   # noqa: BLE001  (a node that fails is skipped)
                continue
    except Exception:   # noqa: BLE001
        return False
    return False


class Filtered(NamedTuple):
    degenerate: bool        # dropped by step 1
    normalized: str         # the UNIQUE key (the string itself when simplify raises)
    signature: int          # int(sha256(normalized)[:8], 16)
    const_only: bool        # no coordinate symbol (skipped before validate)


_LOCALS: Dict[str, Dict] = {}


def _locals(slug: str) -> Tuple[dict, tuple]:
    if slug not in _LOCALS:
        from problems import load_problem
        from expression_operations import UNARY_OPS
        prob = load_problem(slug)
        loc = {**prob.symbols, **getattr(prob, 'constants', {})}
        loc.update(UNARY_OPS)                         # (the driver's order, :84-93)
        syms = prob.symbols
        coords = tuple(syms.get(n, sp.Symbol(n)) for n in ('rho', 'z', 'r', 'x'))
        _LOCALS[slug] = {'locals': loc, 'coords': coords}
    d = _LOCALS[slug]
    return d['locals'], d['coords']


def filter_one(args) -> Filtered:
    """Steps 1-3 for one candidate string, ``(slug, s)``; pure (a SymPy pool job)."""
    slug, s = args
    loc, coords = _locals(slug)
    try:
        u = sp.sympify(s, locals=loc)
    except Exception:   # noqa: BLE001
        u = None
    try:
        if u is not None and has_degenerate_denominator(u):
            return Filtered(True, s, 0, False)
    except Exception:   # noqa: BLE001
        pass
    try:
        plain = sp.sympify(s)
    except Exception:   # noqa: BLE001
        plain = None
    if plain is not None and has_degenerate_denominator(plain):
        return Filtered(True, s, 0, False)
    try:
        normalized = str(sp.simplify(sp.expand(plain if plain is not None else sp.sympify(s))))
    except Exception:   # noqa: BLE001
        normalized = s
    sig = int(hashlib.sha256(normalized.encode()).hexdigest()[:8], 16)
    try:
        uc = u if u is not None else sp.sympify(s, locals=loc)
        const_only = not any(uc.has(c) for c in coords)
    except Exception:   # noqa: BLE001
        const_only = False
    return Filtered(False, normalized, sig, const_only)


class StreamResult(NamedTuple):
    inserted: List[int]     # rows the driver inserts (not degenerate, key not seen before)
    kept: List[int]         # of those, the ones that reach validate (not constant-only)
    recs: List[Filtered]    # every candidate's record
    stats: dict


def filter_stream(slug: str, strings: Sequence[str], seen: Optional[set] = None,
                  item_timeout: Optional[float] = None) -> StreamResult:
    """The driver's filters over a stream (in stream order): the indices of the rows it
    inserts into the run table and of those that reach ``validate`` (a constant-only row is
    inserted and recorded as 'constant-only (skipped)', :1292-1294), every candidate's
    ``Filtered`` record, and counts.
    ``seen``: the run table's keys so far (updated in place; a resumed run passes its table's
    ``normalized`` column).  The per-candidate work runs over the SymPy pool when it runs
    (``pdeval.hostpool``); ``item_timeout`` (the reference has none) keeps a candidate whose
    simplify runs past it under its own string as key."""
    from . import hostpool
    items = [(slug, s) for s in strings]
    recs = hostpool.run(filter_one, items, min_items=1, item_timeout=item_timeout, default=None)
    recs = [r if r is not None else Filtered(False, s, int(hashlib.sha256(s.encode()).hexdigest()[:8], 16), False)
            for r, (_, s) in zip(recs, items)]
    seen = set() if seen is None else seen
    kept: List[int] = []
    inserted: List[int] = []
    stats = {'streamed': len(strings), 'degenerate': 0, 'duplicate': 0, 'const_only': 0}
    for i, r in enumerate(recs):            # UNIQUE(normalized), in stream order
        if r.degenerate:
            stats['degenerate'] += 1
            continue
        if r.normalized in seen:
            stats['duplicate'] += 1
            continue
        seen.add(r.normalized)
        inserted.append(i)
        if r.const_only:
            stats['const_only'] += 1
            continue
        kept.append(i)
    stats['validated'] = len(kept)
    return StreamResult(inserted, kept, recs, stats)
