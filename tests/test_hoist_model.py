"""CPU tests of the hoisted-prefix cost model (pdeval_program_hoist_flops, include/pdeval.h):
the part of a program the lean grid passes evaluate 64 times per candidate instead of at every
point -- its prefix of x alone (once per grid row) or of z alone (once per lane), as
pdeval_grid.h decode_kernel (PD_HOIST) finds it -- on hand-made programs and on the force-free
d4 workload the bench tiles.  The device side (same verdicts and residuals with the prefix
hoisted or not) is tests/test_gpu_parity.py::test_hoisted_prefix_equals_unhoisted."""
import os

import numpy as np
import pytest

from pdeval import _lib
from pdeval import problem_defs as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _flops(pd_, s):
    ops, off, _ = P.compile_strings(pd_, [s])
    w = np.ascontiguousarray(ops[off[0]:off[1]], dtype=np.int32)
    lib = _lib.load()
    ptr = w.ctypes.data
    return lib.pdeval_program_flops(pd_.problem_id, ptr, w.size), lib.pdeval_program_hoist_flops(pd_.problem_id, ptr, w.size)


@pytest.mark.parametrize('prob, s, hoisted', [
    ('force_free', 'exp(rho)*z', True),          # PUSH_X EXP | ... z: the exponential once per row
    ('force_free', 'sqrt(rho + 1)*exp(z)', True),
    ('force_free', 'rho*z', False),              # no heavy opcode before z enters
    ('force_free', 'exp(rho)', False),           # the whole program is x alone: not hoisted
    ('force_free', 'exp(z)*rho', False),         # a prefix of z alone: hoisted for Kerr only
    ('kerr_magnetosphere', 'exp(x)*r', True),    # Kerr's lane coordinate x: once per lane
    ('kerr_magnetosphere', 'sqrt(r + 1)*x', True),
    # a segment of one coordinate as a right operand (PD_HOIST_SUB: Kerr only)
    ('kerr_magnetosphere', 'exp(r*x) + sqrt(x + 1)', True),
    ('force_free', 'exp(rho*z) + sqrt(z + 3)', False),
])
def test_prefix_rule(prob, s, hoisted):
    pd_ = P.get(prob)
    total, pre = _flops(pd_, s)
    assert (pre > 0) is hoisted, (s, total, pre)
    # the per-point epilogue: the model of a one-push program (a push itself costs nothing)
    epi, _ = _flops(pd_, 'rho' if pd_.problem_id == 0 else 'r')
    assert 0 <= pre < total - epi


def test_kerr_segment_and_prefix_add():
    """Kerr hoists a prefix and a later segment of one coordinate together (the segment after
    the prefix's end): exp(r) * x + log(x + 2) -- the prefix PUSH_X EXP and the segment
    log(x + 2) -- counts both."""
    pd_ = P.get('kerr_magnetosphere')
    _, both = _flops(pd_, 'exp(r) * x + log(x + 2)')
    _, pre = _flops(pd_, 'exp(r) * x')
    _, seg = _flops(pd_, 'r * x + log(x + 2)')
    assert pre > 0 and seg > 0 and both == pytest.approx(pre + seg)


def test_d4_workload_share():
    """Over the force-free d4 programs (data/force_free_d4_validated.npz): the hoisted part is
    never more than the program's own opcodes, and it is a sizeable share of the model."""
    d = np.load(os.path.join(ROOT, 'data', 'force_free_d4_validated.npz'))
    ops, off = np.ascontiguousarray(d['ops'], dtype=np.int32), d['offsets']
    lib = _lib.load()
    base = ops.ctypes.data
    n = min(len(off) - 1, 20000)
    epi, _ = _flops(P.force_free(), 'rho')
    tot = pre = 0.0
    for i in range(n):
        p, m = base + 4 * int(off[i]), int(off[i + 1] - off[i])
        f, h = lib.pdeval_program_flops(0, p, m), lib.pdeval_program_hoist_flops(0, p, m)
        assert 0.0 <= h <= f - epi
        tot += f
        pre += h
    assert 0.03 < pre / tot < 0.5, pre / tot
