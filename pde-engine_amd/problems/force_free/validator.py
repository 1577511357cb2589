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
* ``Omega`` must be 0 (the problem path, ``problems/__init__.py:83``).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple

import sympy as sp


class PreciseFoliationValidator:
    def __init__(self, cache_db: Optional[str] = None, use_lean: bool = True, Omega: Any = 0,
                 device: int = 0):
        if Omega != 0:
            raise NotImplementedError('only the non-rotating constraint (Omega = 0) is implemented')
        self.rho = sp.Symbol('rho', real=True, positive=True)
        self.z = sp.Symbol('z', real=True)
        self.Omega = Omega
        self.use_lean = use_lean
        self.cache_db = cache_db
        self.device = device
        self._memo: Dict[Tuple[str, bool, bool], Tuple[bool, str]] = {}
        self._bv = None

    # the GPU context is created on first use (one per process and device)
    def _validator(self):
        if self._bv is None:
            from pdeval.batch import get_validator
            self._bv = get_validator('force_free', self.device)
        return self._bv

    def _canon(self, u: sp.Basic) -> sp.Basic:
        # rename free symbols called rho / z to the validator's symbols (validator.py:283-284)
        sub = {s: (self.rho if s.name == 'rho' else self.z)
               for s in u.free_symbols if getattr(s, 'name', '') in ('rho', 'z')}
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
                key = (str(u), bool(check_regularity), bool(fast_point_only))
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
                    res = bv.validate_exprs([u for _, u in todo])
                finally:
                    bv.params = saved
            else:
                res = bv.validate_exprs([u for _, u in todo])
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
        res = self._validator().validate_strings(list(strings))
        return [(v.ok, v.reason) for v in res]

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
