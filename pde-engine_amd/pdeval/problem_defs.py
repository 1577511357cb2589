"""Per-problem symbols, sympify locals and program compilation.

Mirrors the plugin registry of the reference (``problems/__init__.py:66-108`` force-free,
``:259-302`` Kerr) for what the validator needs: the two coordinates, the constants (Kerr
``M`` and ``a``, which programs keep symbolic: the device gives them the validator's
``M_value`` / ``a_value`` in the point stage, ``kerr validator.py:36-37, :163-171``, and
stand-ins of the symbols in the constant test and the grid stage, ``:231-300``) and the locals
mapping the driver hands to ``sympify`` (symbols + constants + UNARY_OPS, ``general_method_paper_reproduction.py:
84-93``).
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import sympy as sp

from .flatten import Unsupported, flatten, pack
from .opcodes import PROBLEM_FORCE_FREE, PROBLEM_KERR, PDOP, PRM_A, PRM_M

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)
from expression_operations import UNARY_OPS  # noqa: E402


@dataclass
class ProblemDef:
    slug: str
    problem_id: int
    x: sp.Symbol
    y: sp.Symbol
    constants: Dict[str, sp.Symbol]
    params: Dict[sp.Symbol, int]          # the constants as program parameters (PRM_*)
    known_solutions: Dict[str, str] = field(default_factory=dict)

    @property
    def symbols(self) -> Dict[str, sp.Symbol]:
        return {self.x.name: self.x, self.y.name: self.y}

    @property
    def sympify_locals(self) -> Dict[str, object]:
        loc: Dict[str, object] = {}
        loc.update(self.symbols)
        loc.update(self.constants)
        loc.update(UNARY_OPS)
        return loc

    def parse(self, s: str) -> sp.Basic:
        return sp.sympify(s, locals=self.sympify_locals)

    def compile(self, expr: sp.Basic) -> List[int]:
        return flatten(expr, self.x, self.y, self.params)


def force_free() -> ProblemDef:
    rho = sp.Symbol('rho', real=True, positive=True)
    z = sp.Symbol('z', real=True)
    known = {   # problems/__init__.py:85-93
        'rho**2': 'Vertical field',
        'rho**2*z': 'X-point',
        '1 - z/sqrt(rho**2 + z**2)': 'Radial',
        'rho**2/(rho**2 + z**2)**(3/2)': 'Dipolar',
        'sqrt(rho**2 + z**2) - z': 'Parabolic',
        'sqrt(z**2 + (rho - 1)**2) - sqrt(z**2 + (rho + 1)**2)': 'Hyperbolic',
        'rho**2*exp(-2*z)': 'Bent',
    }
    return ProblemDef('force_free', PROBLEM_FORCE_FREE, rho, z, {}, {}, known)


def kerr() -> ProblemDef:
    r = sp.Symbol('r', real=True, positive=True)
    x = sp.Symbol('x', real=True)
    M = sp.Symbol('M', real=True, positive=True)
    a = sp.Symbol('a', real=True)
    return ProblemDef('kerr_magnetosphere', PROBLEM_KERR, r, x, {'M': M, 'a': a},
                      {M: PRM_M, a: PRM_A},
                      {'1 - x': 'Monopole (a -> 0 limit)'})   # problems/__init__.py:285-287


def get(name: str) -> ProblemDef:
    key = (name or '').strip().lower()
    if key in ('force_free', 'forcefree', 'foliation', 'foliations'):
        return force_free()
    if key in ('kerr', 'kerr_magnetosphere', 'kerr-magnetosphere'):
        return kerr()
    raise ValueError(f"Unknown problem '{name}'")


# a program the kernels classify as UNSUPPORTED without evaluating anything
UNSUPPORTED_PROGRAM = [PDOP['HEADER'] | (1 << 8), PDOP['UNSUPPORTED']]


def compile_exprs(pd_: ProblemDef, exprs: Sequence[sp.Basic]) -> Tuple[np.ndarray, np.ndarray, List[Optional[str]]]:
    """Compile SymPy trees; constructs the kernels cannot evaluate become a stub program
    that the device classifies as UNSUPPORTED (so batch indices stay aligned)."""
    progs, notes = [], []
    for e in exprs:
        try:
            progs.append(pd_.compile(e))
            notes.append(None)
        except Unsupported as ex:
            progs.append(UNSUPPORTED_PROGRAM)
            notes.append(str(ex))
    ops, off = pack(progs)
    return ops, off, notes


def compile_strings(pd_: ProblemDef, strings: Sequence[str]):
    exprs = []
    for s in strings:
        try:
            exprs.append(pd_.parse(s))
        except Exception:   # noqa: BLE001 -- unparsable strings become UNSUPPORTED stubs
            exprs.append(sp.Function('unparsable')(pd_.x))
    return compile_exprs(pd_, exprs)
