"""CPU tests of the C-ABI boundary: the library loads, exports every entry point the header
declares, and the host-side helpers (program checks, flop model) behave."""
import os
import re

import numpy as np
import pytest
import sympy as sp

from pdeval import _lib
from pdeval import opcodes as OPC
from pdeval import problem_defs as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = open(os.path.join(ROOT, 'include', 'pdeval.h')).read()


def test_header_functions_exported():
    declared = set(re.findall(r'^\s*(?:int|double|const char\*)\s+(pdeval_\w+)\s*\(', HEADER, re.M))
    assert declared == set(_lib.EXPORTS)
    lib = _lib.load()
    for name in declared:
        assert hasattr(lib, name)


def test_opcodes_match_header():
    for name, val in OPC.PDOP.items():
        if name == 'HEADER':
            continue
        m = re.search(rf'PDOP_{name}\s*=\s*(\d+)', HEADER)
        assert m and int(m.group(1)) == val, name
    for name in ('ACCEPT', 'REJECT_POINT', 'REJECT_GRID', 'ZERO_GRADIENT', 'NONFINITE_REF',
                 'UNSUPPORTED', 'BAD_PROGRAM', 'REJECT_SYMBOLIC'):
        m = re.search(rf'PDEVAL_CLS_{name}\s+(\d+)', HEADER)
        assert int(m.group(1)) == getattr(OPC, f'CLS_{name}')
    for name in ('COMPLEX', 'NOCOORD', 'RATIONAL', 'NONSMOOTH2D', 'UNPROVABLE'):
        m = re.search(rf'PDEVAL_FLAG_{name}\s+\(1u << (\d+)\)', HEADER)
        assert (1 << int(m.group(1))) == getattr(OPC, f'FLAG_{name}')
    assert int(re.search(r'PDEVAL_MAX_STACK\s+(\d+)', HEADER).group(1)) == OPC.MAX_STACK
    assert int(re.search(r'PDEVAL_FP_N\s+(\d+)', HEADER).group(1)) == OPC.FP_N


def test_params_struct_layout():
    import ctypes as C
    assert C.sizeof(_lib.Params) == 80
    assert C.sizeof(_lib.Outputs) == 64
    p = _lib.default_params(0)
    assert p.tau_point == 1e-10 and p.kerr_abs_tol == 1e-10 and p.full_grid == 1
    assert p.point_abs_tol == 1e-20 and p.res_rel_acc == 1e-11 and p.noise_kappa == 16.0
    assert p.omega2 == 0.0 and p.omega2_lo == 0.0
    assert int(re.search(r'PDEVAL_N_PASSES\s+(\d+)', HEADER).group(1)) == _lib.N_PASSES
    assert int(re.search(r'PDEVAL_IMM_DD\s+\(1u << (\d+)\)', HEADER).group(1)) == OPC.IMM_DD.bit_length() - 1


def test_program_depth_checks():
    pd_ = P.force_free()
    w = np.array(pd_.compile(pd_.parse('sqrt(z**2 + (rho - 1)**2) - sqrt(z**2 + (rho + 1)**2)')),
                 dtype=np.int32)
    assert _lib.program_depth(w) == 2           # (rho +- 1)**2 + z**2: z**2 is a fused operand
    bad = w.copy()
    bad[0] = (bad[0] & ~0xff00) | (3 << 8)      # header lies about the depth
    assert _lib.program_depth(bad) < 0
    assert _lib.program_depth(w[:-1]) < 0        # truncated: stack not reduced to one value
    assert _lib.program_depth(np.array([0x100, 99], dtype=np.int32)) < 0   # unknown opcode


def test_flop_model_monotone():
    pd_ = P.force_free()
    f1 = _lib.program_flops(0, np.array(pd_.compile(pd_.parse('rho*z')), np.int32))
    f2 = _lib.program_flops(0, np.array(pd_.compile(pd_.parse('exp(rho*z)*sqrt(z)')), np.int32))
    assert 0 < f1 < f2


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(_lib.PdevalError):
        _lib.Context(0)


def test_plugin_omega_contract():
    """Omega != 0 (validator.py:326-329): a constant whose square is rational is taken, as a
    double-double (params.omega2, omega2_lo: 1/9 to 2^-106); a symbolic Omega -- the reference
    allows a function of u -- or an irrational square raises NotImplementedError before any GPU
    use."""
    from fractions import Fraction
    from pdeval.batch import omega2_value
    from problems.force_free.validator import PreciseFoliationValidator
    assert omega2_value(1) == (1.0, 0.0) and omega2_value('1/2') == (0.25, 0.0)
    assert omega2_value('sqrt(2)') == (2.0, 0.0)
    for w, exact in (('1/3', Fraction(1, 9)), ('sqrt(2)/3', Fraction(2, 9)), ('7/10', Fraction(49, 100))):
        hi, lo = omega2_value(w)
        assert lo != 0.0 and hi == float(exact) and abs(Fraction(hi) + Fraction(lo) - exact) <= exact * 2.0 ** -106
    assert omega2_value(0.5) == (0.25, 0.0)     # a Float: its exact binary value
    assert PreciseFoliationValidator(Omega=1)._omega_key == '1'
    assert PreciseFoliationValidator(Omega=sp.Rational(1, 3))._omega_key == '1/3'
    for bad in ('2**(1/4)', 'pi', 'rho'):
        with pytest.raises(NotImplementedError):
            PreciseFoliationValidator(Omega=bad)
