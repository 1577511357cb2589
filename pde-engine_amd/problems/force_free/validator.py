"""Force-free foliation validator backed by the MI355X kernel.

Drop-in for ``problems/force_free/validator.py`` of the reference: same class name, same
``validate(u, check_regularity=True, fast_point_only=False) -> (bool, str)`` contract
(``:260-437``), same verdicts and reason strings (see ``pdeval.batch`` for the mapping).  The
work -- derivatives of u to 4th order, the determinant of Compere et al. eq. 2.14 (``:323-347``),
the exact-point stage at (4/5, 6/7) (``:349-402``) and the whole-plane stage (``:404-427``) --
runs on the GPU for whole batches (``validate_batch``).

Differences, all deliberate:
* no persistent SQLite verdict cache (``:182-222``): it made committed verdicts stale (SURVEY.md
  §4); an in-memory memo keyed by ``str(u)`` is kept instead;
* ``fast_point_only=True`` returns the point-stage verdict ("Valid foliation (point check = 0)")
  -- the reference's fast branch fails on its own symbolic stand-ins (``:298-303, :323``);
* ``Omega``: 0 on the problem path (``problems/__init__.py:83``); a constant Omega != 0 (the
  rotating constraint, ``:326-329``) is evaluated on the device too (``params.omega2``, the
  rotation terms of ``FFEpi``), for any constant Omega whose square is an exact double (1, 2,
  1/2, sqrt(2), ...); an Omega that is a function of u raises NotImplementedError;
* ``symbolic`` chooses how much of the reference's symbolic stage (``:404-427``) is replayed
  on the host in SymPy (``pdeval.symbolic``): ``'off'`` (default: the device's verdicts, and
  the Lean text for every grid reject), ``'text'`` (grid rejects get the reference's branch
  text, "Invalid (expanded det != 0)" when SymPy's det_M prints to 3,000 characters or more)
  or ``'replay'`` (also the reference's symbolic verdict for every candidate the grid finds
  zero: its false negatives become rejects).  Each replayed candidate is bounded by
  ``symbolic_timeout`` seconds and keeps the device's verdict past it.  The env var
  ``PDEVAL_SYMBOLIC`` sets the default.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Sequence, Tuple

import sympy as sp


class PreciseFoliationValidator:
    def __init__(self, cache_db: Optional[str] = None, use_lean: bool = True, Omega: Any = 0,
                 device: int = 0, symbolic: Optional[str] = None, symbolic_timeout: float = 60.0):
        from pdeval.batch import SYMBOLIC_MODES, omega2_value
        if Omega != 0:
            omega2_value(Omega)     # a constant whose square is rational, else NotImplementedError
        self._omega_key = '0' if Omega == 0 else str(sp.nsimplify(sp.sympify(Omega)))
        self.symbolic = symbolic or os.environ.get('PDEVAL_SYMBOLIC', 'off')
        if self.symbolic not in SYMBOLIC_MODES:
            raise ValueError(f'symbolic mode {self.symbolic!r}: one of {SYMBOLIC_MODES}')
        self.symbolic_timeout = symbolic_timeout
        self.rho = sp.Symbol('rho', real=True, positive=True)
        self.z = sp.Symbol('z', real=True)
        self.Omega = Omega
        self.use_lean = use_lean
        self.cache_db = cache_db
        self.device = device
        self._memo: Dict[Tuple[sp.Basic, bool, bool, str], Tuple[bool, str]] = {}
        self._bv = None

    # the GPU context is created on first use (one per process and device)
    def _validator(self):
        if self._bv is None:
            from pdeval.batch import get_validator
            self._bv = get_validator('force_free', self.device, omega=self._omega_key)
        return self._bv

    def _canon(self, u: sp.Basic) -> sp.Basic:
        # rename free symbols called rho / z to the validator's symbols (validator.py:283-284);
        # the driver's trees already hold them (problems/__init__.py:70-71): no substitution
        sub = {s: (self.rho if s.name == 'rho' else self.z)
               for s in u.free_symbols if getattr(s, 'name', '') in ('rho', 'z')}
        sub = {k: v for k, v in sub.items() if k is not v}
        return u.subs(sub) if sub else u

    def validate(self, u: sp.Basic, check_regularity: bool = True,
                 fast_point_only: bool = False) -> Tuple[bool, str]:
        return self.validate_batch([u], check_regularity, fast_point_only)[0]

    def validate_batch(self, us: Sequence[sp.Basic], check_regularity: bool = True,
                       fast_point_only: bool = False) -> List[Tuple[bool, str]]:
        out: List[Optional[Tuple[bool, str]]] = [None] * len(us)
        todo, idx = [], []
        for i, u0 in enumerate(us):
            try:
                u = self._canon(sp.sympify(u0))
                # (the tree itself is the memo key: structural equality, and its hash is cached;
                # str(u) cost a fifth of a one-candidate call)
                key = (u, bool(check_regularity), bool(fast_point_only), self.symbolic)
                if key in self._memo:
                    out[i] = self._memo[key]
                    continue
                if check_regularity:
                    # axis regularity (validator.py:288-293)
                    if u.subs(self.rho, 0).has(sp.oo, sp.zoo, sp.nan):
                        out[i] = self._memo[key] = (False, 'Singular on axis')
                        continue
                todo.append((key, u))
                idx.append(i)
            except Exception as e:  # noqa: BLE001  (validate never raises, :434-437)
                out[i] = (False, f'Error: {e}')
        if todo:
            bv = self._validator()
            if fast_point_only:
                prm = _copy_params(bv.params)
                prm.full_grid = 0
                saved, bv.params = bv.params, prm
                try:
                    res = bv.validate_exprs([u for _, u in todo], symbolic='off')
                finally:
                    bv.params = saved
            else:
                res = self._symbolic_call(bv.validate_exprs, [u for _, u in todo])
            for (key, _), i, v in zip(todo, idx, res):
                r = (v.ok, v.reason)
                if fast_point_only and v.cls in (0, 2, 7):   # passed the point stage
                    r = (True, 'Valid foliation (point check = 0)')
                out[i] = self._memo[key] = r
        return out  # type: ignore[return-value]

    def validate_strings(self, strings: Sequence[str]) -> List[Tuple[bool, str]]:
        """The driver's queue items are strings (general_method_paper_reproduction.py:1767):
        validate them without building SymPy trees (native compiler, SymPy only for the
        strings it declines), with the driver's kwargs check_regularity=False,
        fast_point_only=False.  Same (bool, reason) as validate_batch(sympify(s))."""
        res = self._symbolic_call(self._validator().validate_strings, list(strings))
        return [(v.ok, v.reason) for v in res]

    def _symbolic_call(self, fn, items):
        return fn(items, symbolic=self.symbolic, symbolic_timeout=self.symbolic_timeout)

    def symbolic_args(self) -> Dict[str, Any]:
        """The host-replay mode of this validator, as BatchValidator.finish takes it (worker)."""
        return {'symbolic': self.symbolic, 'symbolic_timeout': self.symbolic_timeout}

    def validate_known_solutions(self) -> Dict[str, bool]:
        rho, z = self.rho, self.z
        known = {
            'Vertical': rho**2,
            'X-point': rho**2 * z,
            'Radial': 1 - z / sp.sqrt(rho**2 + z**2),
            'Dipolar': rho**2 / (rho**2 + z**2)**sp.Rational(3, 2),
            'Parabolic': sp.sqrt(rho**2 + z**2) - z,
            'Hyperbolic': sp.sqrt(z**2 + (rho - 1)**2) - sp.sqrt(z**2 + (rho + 1)**2),
            'Bent': rho**2 * sp.exp(-2 * z),
        }
        res = self.validate_batch(list(known.values()))
        return {name: ok for name, (ok, _) in zip(known, res)}

    def get_cache_stats(self) -> Dict[str, int]:
        valid = sum(1 for ok, _ in self._memo.values() if ok)
        return {'total': len(self._memo), 'valid': valid, 'invalid': len(self._memo) - valid}

    def clear_cache(self):
        self._memo.clear()


def _copy_params(p):
    from pdeval._lib import Params
    q = Params()
    for f, _ in Params._fields_:
        setattr(q, f, getattr(p, f))
    return q
