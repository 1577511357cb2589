"""Kerr magnetosphere surrogate validator backed by the MI355X kernel.

Drop-in for ``problems/kerr_magnetosphere/validator.py``: same class and constructor, same
``validate(u, check_regularity=True, fast_point_only=False, *, lean_first=True,
defer_heavy_checks=True, enforce_anchor=None) -> (bool, str)`` (``:210-345``), ``describe()``
(``:369-378``) and ``last_evidence()`` (``:380-381``).  The operator
``d_r[G/(1-x^2) d_r u] + d_x[G/Delta d_x u]`` (``:77-91``), the 3-point check (absolute 1e-10,
``:163-192``) and the exact-zero stage (``:283-315``) run on the GPU for whole batches.

Any ``M_value`` / ``a_value`` (``:36-37``): the device's point stage substitutes them, as the
reference's fast point check does, while its constant test and grid stage -- the surrogates of
the reference's ``simplify(u)`` test and symbolic stage, which keep ``M`` and ``a`` symbolic --
use stand-ins of the symbols (``pdeval_kerr_constants``, include/pdeval.h).  A validator built
with a number for ``M`` or ``a`` (e.g. ``a = 0``, the Schwarzschild operator) uses that number
in its operator everywhere; ``u``'s own symbol is then free.

With ``defer_heavy_checks=False`` the reference's heavy checks on exact zeros (constancy,
finiteness, axis/horizon regularity, a -> 0 monopole anchor, ``:325-342``) run on the host in
SymPy -- only for the (rare) candidates the GPU accepts.

``symbolic`` (constructor; env ``PDEVAL_SYMBOLIC``): ``'off'`` (default) gives class-level
reject texts (a numeric residual after "residual:") and a device evidence dict; ``'text'``
reproduces the reference's texts -- the 240-character ``numer/denom`` repr of the symbolic
residual (``_short_residual_repr`` :249-261) -- and its ``last_evidence()`` dict
``{lhs_string, lean_normalized, sympy_simplified_is_zero, params}`` (:296-306), which like the
reference's is the one of the last candidate that passed the fast point check (point rejects
leave it as it was); ``'replay'`` also takes the reference's exact-zero verdict.  Those modes
run SymPy per candidate on the host (``pdeval.symbolic``), each bounded by ``symbolic_timeout``.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple

import sympy as sp


class KerrMagnetosphereValidator:
    def __init__(self, r: sp.Symbol, x: sp.Symbol, M: sp.Symbol, a: sp.Symbol,
                 M_value: Any = sp.Integer(1), a_value: Any = sp.Rational(1, 10),
                 use_lean: bool = True, lean_det_str_max_len: int = 12000,
                 require_monopole_extension: bool = True, monopole_target: str = '1-x',
                 allow_normalization: bool = False, strict_sympy_check: bool = True,
                 exclude_constants: bool = True, device: int = 0, symbolic: Optional[str] = None,
                 symbolic_timeout: float = 60.0) -> None:
        import os
        from pdeval.batch import SYMBOLIC_MODES
        self.symbolic = symbolic or os.environ.get('PDEVAL_SYMBOLIC', 'off')
        if self.symbolic not in SYMBOLIC_MODES:
            raise ValueError(f'symbolic mode {self.symbolic!r}: one of {SYMBOLIC_MODES}')
        self.symbolic_timeout = symbolic_timeout
        self._kerr = self.device_constants(M, a, M_value, a_value)
        self.r, self.x, self.M, self.a = r, x, M, a
        self.M_value, self.a_value = M_value, a_value
        self.use_lean = use_lean
        self.lean_det_str_max_len = lean_det_str_max_len
        self.require_monopole_extension = require_monopole_extension
        self.monopole_target = monopole_target
        self.allow_normalization = allow_normalization
        self.strict_sympy_check = strict_sympy_check
        self.exclude_constants = exclude_constants
        self.device = device
        self._residual_zero_cache: Dict[str, bool] = {}
        self._last_evidence: Dict[str, Any] = {}
        self._bv = None

    @staticmethod
    def device_constants(M, a, M_value, a_value):
        """pdeval_kerr_constants for this validator: exact rationals M_value, a_value; the
        operator's M (a) fixed when the constructor got a number for it (which must then be
        the value the fast point check substitutes for it, ``:165-166``)."""
        from pdeval._lib import default_kerr_constants
        k = default_kerr_constants()
        Mv, av = sp.Rational(sp.nsimplify(M_value)), sp.Rational(sp.nsimplify(a_value))
        if not (Mv > 0 and abs(av) < Mv):
            raise ValueError('Kerr constants: need M_value > 0 and |a_value| < M_value (a horizon)')
        k.M_num, k.M_den, k.a_num, k.a_den = int(Mv.p), int(Mv.q), int(av.p), int(av.q)
        for name, sym, val in (('M', M, Mv), ('a', a, av)):
            if not isinstance(sym, sp.Symbol):
                if sp.nsimplify(sym) != val:
                    raise NotImplementedError(f'operator {name} = {sym} differs from {name}_value = {val}')
                setattr(k, f'op_{name}_fixed', 1)
        return k

    def _validator(self):
        if self._bv is None:
            from pdeval.batch import get_validator
            self._bv = get_validator('kerr', self.device, kerr=self._kerr)
        return self._bv

    # --------------------------------------------------------------- operator (host, symbolic)
    def _delta(self):
        return self.r**2 - 2 * self.M * self.r + self.a**2

    def _G(self):
        return 1 - (2 * self.M * self.r) / (self.r**2 + self.a**2 * self.x**2)

    def describe(self) -> Dict[str, str]:
        u = sp.Function('u')(self.r, self.x)
        lhs = (sp.Derivative(self._G() / (1 - self.x**2) * sp.Derivative(u, self.r), self.r)
               + sp.Derivative(self._G() / self._delta() * sp.Derivative(u, self.x), self.x))
        return {'method_name': f'{self.__class__.__module__}.{self.__class__.__name__}.validate',
                'math_definition': str(lhs)}

    def last_evidence(self) -> Dict[str, Any]:
        return self._last_evidence

    def symbolic_args(self) -> Dict[str, Any]:
        """The host-text mode of this validator, as BatchValidator.finish takes it (worker)."""
        return {'symbolic': self.symbolic, 'symbolic_timeout': self.symbolic_timeout}

    # --------------------------------------------------------------- validation
    def validate(self, u: sp.Basic, check_regularity: bool = True, fast_point_only: bool = False,
                 *, lean_first: bool = True, defer_heavy_checks: bool = True,
                 enforce_anchor: Optional[bool] = None) -> Tuple[bool, str]:
        return self.validate_batch([u], check_regularity, fast_point_only,
                                   lean_first=lean_first, defer_heavy_checks=defer_heavy_checks,
                                   enforce_anchor=enforce_anchor)[0]

    def validate_batch(self, us: Sequence[sp.Basic], check_regularity: bool = True,
                       fast_point_only: bool = False, *, lean_first: bool = True,
                       defer_heavy_checks: bool = True,
                       enforce_anchor: Optional[bool] = None) -> List[Tuple[bool, str]]:
        out: List[Optional[Tuple[bool, str]]] = [None] * len(us)
        exprs, idx = [], []
        for i, u in enumerate(us):
            try:
                u = sp.sympify(u)
                key = str(u)
                if self._residual_zero_cache.get(key) is False:
                    out[i] = (False, 'PDE residual != 0 (cached)')     # :274-281
                    continue
                exprs.append(u)
                idx.append(i)
            except Exception as e:  # noqa: BLE001
                out[i] = (False, f'Validation error: {e}')
        if exprs:
            res = self._validator().validate_exprs(exprs, symbolic=self.symbolic,
                                                   symbolic_timeout=self.symbolic_timeout)
            for u, i, v in zip(exprs, idx, res):
                ok, reason = v.ok, v.reason
                if self.symbolic == 'off':
                    self._last_evidence = {
                        'kernel_class': v.cls, 'max_abs_lhs_at_test_points': v.q_ref,
                        'max_scaled_lhs_on_grid': v.q_grid,
                        'params': {'M': str(self.M_value), 'a': str(self.a_value)},
                    }
                elif v.evidence is not None:
                    # the reference records evidence only past its fast point check (:296-306)
                    self._last_evidence = v.evidence
                # the reference consults its cache only after the fast point check passed and
                # writes False only when the exact-zero stage failed (:274-281, :308-315): a
                # repeated point reject is re-checked (same reason), a grid reject is "(cached)"
                if v.cls == 2:
                    self._residual_zero_cache[str(u)] = False
                if ok and not defer_heavy_checks:
                    ok, reason = self._heavy_checks(u, check_regularity, enforce_anchor)
                elif ok:
                    self._residual_zero_cache[str(u)] = True
                out[i] = (ok, reason)
        return out  # type: ignore[return-value]

    # --------------------------------------------------------------- heavy checks (host)
    def _heavy_checks(self, u, check_regularity, enforce_anchor) -> Tuple[bool, str]:
        r, x, M, a = self.r, self.x, self.M, self.a
        try:
            if self.exclude_constants:
                if sp.simplify(sp.diff(u, r)) == 0 and sp.simplify(sp.diff(u, x)) == 0:
                    return False, 'Trivial constant solution excluded'
            lhs = (sp.diff(self._G() / (1 - x**2) * sp.diff(u, r), r)
                   + sp.diff(self._G() / self._delta() * sp.diff(u, x), x))
            if not self._finite(u):
                return False, 'non-finite'
            if not self._finite(lhs):
                return False, 'residual non-finite'
            if check_regularity and not self._regular(u):
                return False, 'Symbolic zero but fails regularity checks'
            anchor = self.require_monopole_extension if enforce_anchor is None else bool(enforce_anchor)
            if anchor and not self._monopole(u):
                return False, 'fails a->0 monopole anchor'
            return True, 'valid'
        except Exception as e:  # noqa: BLE001
            return False, f'Validation error: {e}'

    def _finite(self, e) -> bool:
        """No infinities, and finite at two sample points away from Delta = 0, x = +-1."""
        bad = (sp.zoo, sp.oo, -sp.oo, sp.nan)
        try:
            e = sp.simplify(e)
        except Exception:   # noqa: BLE001
            pass
        if e.has(*bad):
            return False
        for pt in ((1, sp.Rational(3, 5), sp.Rational(7, 3), sp.Rational(1, 3)),
                   (1, sp.Rational(4, 5), 3, -sp.Rational(2, 5))):
            val = sp.simplify(e.subs({self.M: pt[0], self.a: pt[1], self.r: pt[2], self.x: pt[3]}))
            if val.has(*bad):
                return False
        return True

    def _regular(self, u) -> bool:
        r, x, M, a = self.r, self.x, self.M, self.a
        flux = self._G() / (1 - x**2) * sp.diff(u, r)
        if any(sp.limit(flux, x, s) in (sp.oo, -sp.oo, sp.zoo) for s in (1, -1)):
            return False
        Mv, av = self.M_value, self.a_value
        r_h = Mv + sp.sqrt(Mv**2 - av**2)
        hz = sp.limit((self._G() / self._delta()).subs({M: Mv, a: av}) * sp.diff(u, x), r, r_h)
        return hz not in (sp.oo, -sp.oo, sp.zoo)

    def _monopole(self, u) -> bool:
        targets = []
        if self.monopole_target in ('1-x', 'either'):
            targets.append(1 - self.x)
        if self.monopole_target in ('x', 'either'):
            targets.append(self.x)
        for t in targets:
            try:
                lim = sp.simplify(sp.limit(sp.simplify(u - t), self.a, 0))
            except Exception:   # noqa: BLE001
                lim = sp.simplify((u - t).subs(self.a, 0))
            if lim == 0:
                return True
            if self.allow_normalization and not lim.has(sp.oo, sp.zoo, sp.nan) and \
                    (lim.free_symbols <= {self.M} or lim.is_number):
                return True
        return False
