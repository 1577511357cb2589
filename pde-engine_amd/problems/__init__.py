"""Problem plugin interface -- drop-in for the reference's ``problems/__init__.py``.

Same names and contract as the reference: ``ProblemSpec`` (``problems/__init__.py:34-63``)
and ``load_problem(name)`` (``:355-361``) with the two built-in problems.  The difference is
the validator object: here it is backed by the MI355X kernel (``pdeval``), and besides the
per-candidate ``validate(u, ...)`` of the reference contract (``:52``) it exposes
``validate_batch(list_of_u)``, which the worker pool uses to send whole batches to the GPU.
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass
from typing import Any, Callable, Dict, List

import sympy as sp

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from expression_operations import ALL_BINARY_OPS, BINARY_OPS, SPECIAL_OPS, UNARY_OPS  # noqa: E402


@dataclass
class ProblemSpec:
    """Specification container for a PDE discovery problem."""

    name: str
    slug: str
    symbols: Dict[str, sp.Symbol]
    constants: Dict[str, sp.Symbol]
    primitives: List[sp.Basic]
    unary_ops: Dict[str, Callable]
    binary_ops: Dict[str, Callable]
    special_ops: Dict[str, Callable]
    all_binary_ops: Dict[str, Callable]
    # validate(u, check_regularity=True, fast_point_only=False) -> (bool, str); here also
    # validate_batch(us, **kw) -> [(bool, str)]
    validator: Any
    known_solutions: Dict[str, str]
    output_root: str

    def get_output_dir(self) -> str:
        os.makedirs(self.output_root, exist_ok=True)
        return self.output_root


def _force_free() -> ProblemSpec:
    from pdeval.problem_defs import force_free
    from problems.force_free.validator import PreciseFoliationValidator
    d = force_free()
    rho, z = d.x, d.y
    return ProblemSpec(
        name='Force-Free Foliations', slug='force_free',
        symbols={'rho': rho, 'z': z}, constants={},
        primitives=[rho, z, rho**2 + z**2, rho / z, sp.Integer(1)],     # :73-79
        unary_ops=UNARY_OPS, binary_ops=BINARY_OPS, special_ops=SPECIAL_OPS,
        all_binary_ops=ALL_BINARY_OPS,
        validator=PreciseFoliationValidator(),
        known_solutions=dict(d.known_solutions),
        output_root=os.path.join('problems', 'force_free', 'outputs'))


def _kerr() -> ProblemSpec:
    from pdeval.problem_defs import kerr
    from problems.kerr_magnetosphere.validator import KerrMagnetosphereValidator
    d = kerr()
    r, x = d.x, d.y
    M, a = d.constants['M'], d.constants['a']
    Delta = r**2 - 2 * M * r + a**2
    G = 1 - (2 * M * r) / (r**2 + a**2 * x**2)
    return ProblemSpec(
        name='Kerr Magnetosphere (linear surrogate)', slug='kerr_magnetosphere',
        symbols={'r': r, 'x': x}, constants={'M': M, 'a': a},
        primitives=[r, x, sp.Integer(1), sp.Rational(1, 3), 1 - x, a**2,       # :271-281
                    r**2 + a**2 * x**2, Delta, G],
        unary_ops=UNARY_OPS, binary_ops=BINARY_OPS, special_ops=SPECIAL_OPS,
        all_binary_ops=ALL_BINARY_OPS,
        validator=KerrMagnetosphereValidator(r, x, M, a, M_value=sp.Integer(1),
                                             a_value=sp.Rational(1, 10)),
        known_solutions=dict(d.known_solutions),
        output_root=os.path.join('problems', 'kerr_magnetosphere', 'outputs'))


def load_problem(name: str) -> ProblemSpec:
    key = (name or '').strip().lower()
    if key in ('force_free', 'forcefree', 'foliation', 'foliations'):
        return _force_free()
    if key in ('kerr', 'kerr_magnetosphere', 'kerr-magnetosphere'):
        return _kerr()
    raise ValueError(f"Unknown problem '{name}'. Available: 'force_free', 'kerr_magnetosphere'")


__all__ = ['ProblemSpec', 'load_problem']
