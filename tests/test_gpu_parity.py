"""GPU parity: libpdeval.so on the MI355X vs the CPU oracle and vs the reference's verdicts.

Bar (north star): accept/reject verdicts identical to the reference's on every fixture the
reference decided; residuals at the reference point(s) within 1e-10 relative of the oracle's
(absolute floor 1e-13 * S for residuals that are rounding noise of an exact zero).
"""
import numpy as np
import pytest

import golden_data as G
import oracle_lib as O
from pdeval import problem_defs as P
from pdeval._lib import Context

pytestmark = pytest.mark.gpu

REL_TOL = 1e-10
EPS = 2.0 ** -52


def check_residuals(dev, ora, strings, tau=1e-10):
    """Residual at the reference point(s) of every point-stage reject (class REJECT_POINT):
    the device value agrees with the oracle's to 1e-10 relative -- or, where the residual
    itself is the result of cancellation, to the fp64 conditioning limit 64 eps / q (neither
    side is exact there).  Every other candidate's residual is rounding noise of an exact
    zero (q <= tau, or |res| within its noise bound: tier 2), which the equal classes already
    assert."""
    q = np.asarray(ora['q_ref'])
    d, o = dev['res_ref'], ora['res_ref']
    for i in range(len(q)):
        if ora['status'][i] != 1 or not (q[i] > tau) or not np.all(np.isfinite(o[i])):
            continue
        tol = max(REL_TOL, 64 * EPS / q[i]) if dev['res_ref'].shape[1] == 1 else REL_TOL
        err = np.max(np.abs(d[i] - o[i]) / np.maximum(np.abs(o[i]), 1e-300))
        assert err <= tol, (strings[i], d[i], o[i], err, tol)


@pytest.fixture(scope='module')
def ff_ctx():
    return Context(0)


def _cmp_device_oracle(ctx, pd_, strings):
    ops, off, _ = P.compile_strings(pd_, strings)
    dev = ctx.validate(ops, off)
    ora = O.validate(pd_.problem_id, ops, off)
    assert np.array_equal(dev['status'], ora['status']), \
        [(s, int(a), int(b)) for s, a, b in zip(strings, dev['status'], ora['status']) if a != b][:10]
    bad = np.flatnonzero(dev['n_bad'] != ora['n_bad'])
    assert not bad.size, [(strings[i], int(dev['status'][i]), int(dev['n_bad'][i]), int(ora['n_bad'][i]))
                          for i in bad[:10]]
    # n_nonfinite: points where an intermediate jet of the program overflows (exp(exp(..)))
    # depend on the evaluation order (device Horner vs oracle explicit powers); allow 1 % of
    # the grid there -- the classes above are exact
    d = np.abs(dev['n_nonfinite'].astype(np.int64) - ora['n_nonfinite'])
    assert d.max(initial=0) <= 41, [(strings[i], int(dev['n_nonfinite'][i]), int(ora['n_nonfinite'][i]))
                                    for i in np.flatnonzero(d > 41)[:10]]
    check_residuals(dev, ora, strings)
    return dev, ora


def test_known_solutions_ff(ff_ctx):
    pd_ = P.force_free()
    dev, _ = _cmp_device_oracle(ff_ctx, pd_, list(pd_.known_solutions))
    assert dev['verdict'].all(), dev['status']


def test_ff_reference_verdicts(ff_ctx):
    pd_ = P.force_free()
    rows = G.decided(G.ref_rows(*G.FF_REF))
    dev, _ = _cmp_device_oracle(ff_ctx, pd_, [r['expr'] for r in rows])
    ref = np.array([bool(r['ok']) for r in rows])
    mism = [(r['expr'], r['reason'], int(s)) for r, v, s in zip(rows, dev['verdict'], dev['status'])
            if bool(v) != bool(r['ok'])]
    assert not mism, mism[:10]
    assert (dev['verdict'] == ref).all()


@pytest.fixture(scope='module')
def kerr_ctx():
    return Context(1)


def test_ff_edge_cases(ff_ctx):
    pd_ = P.force_free()
    rows = G.decided(G.ref_rows('ff_edge.jsonl'))
    dev, _ = _cmp_device_oracle(ff_ctx, pd_, [r['expr'] for r in rows])
    mism = [(r['expr'], r['reason'], int(s)) for r, v, s in zip(rows, dev['verdict'], dev['status'])
            if bool(v) != bool(r['ok'])]
    assert not mism, mism


def test_kerr_reference_verdicts(kerr_ctx):
    pd_ = P.kerr()
    rows = G.decided(G.ref_rows(*G.KERR_REF, 'kerr_edge.jsonl'))
    dev, _ = _cmp_device_oracle(kerr_ctx, pd_, [r['expr'] for r in rows])
    mism = [(r['expr'], r['reason'][:60], int(s)) for r, v, s in zip(rows, dev['verdict'], dev['status'])
            if bool(v) != bool(r['ok'])]
    assert not mism, mism[:10]


def test_plugin_api_reasons():
    """The drop-in problems/ package answers with the reference's (bool, reason) pairs."""
    from problems import load_problem
    rows = G.decided(G.ref_rows(*G.FF_REF, 'ff_edge.jsonl'))
    prob = load_problem('force_free')
    locs = {**prob.symbols, **prob.constants, **prob.unary_ops}
    import sympy as sp
    us = [sp.sympify(r['expr'], locals=locs) for r in rows]
    got = prob.validator.validate_batch(us, check_regularity=False, fast_point_only=False)
    verdicts = sum(g[0] == r['ok'] for g, r in zip(got, rows))
    cls = sum(g[1].split('≈')[0] == r['reason'].split('≈')[0] for g, r in zip(got, rows))
    assert verdicts == len(rows)
    assert cls >= 0.95 * len(rows), (cls, len(rows))
    # the per-candidate contract of problems/__init__.py:52
    assert prob.validator.validate(us[0], check_regularity=False) == got[0]
    assert all(prob.validator.validate_known_solutions().values())


def test_ff_tier2_exact_ground_truth(ff_ctx):
    """Tier 2 on the device: true solutions (exact det = 0) accepted, the rest rejected, and
    the classes equal the oracle's."""
    pd_ = P.force_free()
    rows = G.exact_rows()
    dev, _ = _cmp_device_oracle(ff_ctx, pd_, [r['expr'] for r in rows])
    wrong = [(r['expr'], int(s)) for r, s in zip(rows, dev['status']) if (s in (0, 7)) != r['det_zero']]
    assert not wrong, wrong[:10]


def test_ff_early_exit_same_verdicts(ff_ctx):
    """The reference's control flow (stop after the point stage) gives the same verdicts."""
    from pdeval._lib import default_params
    pd_ = P.force_free()
    rows = G.exact_rows() + G.decided(G.ref_rows(*G.FF_REF))
    ops, off, _ = P.compile_strings(pd_, [r['expr'] for r in rows])
    full = ff_ctx.validate(ops, off)
    prm = default_params(0)
    prm.full_grid = 0
    early = ff_ctx.validate(ops, off, prm)
    assert np.array_equal(full['verdict'], early['verdict'])
    ora = O.validate(0, ops, off, O.params(full_grid=0))
    assert np.array_equal(early['status'], ora['status'])


POINT_EXPRS = ['rho**2 + z**2', 'z*neg(rho/z + 1)', 'exp(z/(-rho**2 + z**2))',
               'exp_neg(square(rho/(-rho/z + 1)))', 'rho**2/(rho**2 + z**2)**(3/2)',
               'sqrt(z**2 + (rho - 1)**2) - sqrt(z**2 + (rho + 1)**2)',
               'rho**2 + z**2/(1 - square(rho)/(rho**2 + z**2))',
               'square(rho/(rho**2/z**2 - 2*rho/z + 1))', 'z**4/(rho**3 + 2)']


@pytest.mark.parametrize('s', POINT_EXPRS)
def test_ff_point_arithmetic(ff_ctx, s):
    """Device tier-2 point arithmetic (pdeval_eval_points) vs the oracle on the whole grid:
    residual and S within 4 noise bounds (S's first-order sensitivity to the coefficient
    errors is the noise bound itself) or 1e-9 relative, noise bounds within a factor 4."""
    pd_ = P.force_free()
    w = np.array(pd_.compile(pd_.parse(s)), dtype=np.int32)
    gx = 0.05 + (np.arange(64) + 0.37) * (2.95 / 64)
    gy = -2 + (np.arange(64) + 0.41) * (4 / 64)
    xs = np.concatenate([[0.8], np.repeat(gx, 64)])
    ys = np.concatenate([[6 / 7], np.tile(gy, 64)])
    dev = ff_ctx.eval_points(w, xs, ys, tier2=True)
    bad = []
    for i in range(len(xs)):
        o = O.point(0, w, xs[i], ys[i])
        d = dev[i]
        if not (o[3] and d[3] == 1):
            if bool(o[3]) != (d[3] == 1):
                bad.append(('finite', xs[i], ys[i], d, o))
            continue
        tol = 4 * max(o[2], d[2])
        ok = (abs(d[1] - o[1]) <= 1e-9 * o[1] + tol + 1e-300 and
              abs(d[0] - o[0]) <= tol + 1e-12 * o[1] and
              d[2] <= 4 * o[2] + 1e-300 and o[2] <= 4 * d[2] + 1e-300)
        if not ok:
            bad.append((xs[i], ys[i], d.tolist(), o.tolist()))
    assert len(bad) <= 2, (len(bad), bad[:5])   # 2 of 4097: exact-boundary overflow cases


def test_native_compile_full_d4(ff_ctx):
    """All 142,004 validated force-free depth-4 strings: programs from the native compiler
    (csrc/pdcompile.cpp; SymPy only for the strings it declines) get the same class on the
    device as the SymPy-compiled programs of data/force_free_d4_validated.npz."""
    import os
    from pdeval import native
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             'data', 'force_free_d4_validated.npz'))
    strings = [str(s) for s in d['exprs']]
    _, _, st = native.compile_native(0, strings)
    ok = np.flatnonzero(st == native.COMPILE_OK)
    assert len(ok) >= 0.97 * len(strings)
    ops, off, _ = native.compile_strings(P.force_free(), strings)   # declined: through SymPy
    nat = ff_ctx.validate(ops, off)
    ref = ff_ctx.validate(d['ops'], d['offsets'])
    diff = ok[nat['status'][ok] != ref['status'][ok]]
    assert not diff.size, [(strings[i], int(nat['status'][i]), int(ref['status'][i])) for i in diff[:10]]
    assert np.array_equal(nat['verdict'][ok], ref['verdict'][ok])


def test_native_compile_full_kerr_d3(kerr_ctx):
    """All 16,323 validated Kerr depth<=3 strings: native compile (SymPy for declined ones)
    vs the SymPy-compiled programs of data/kerr_magnetosphere_d3_validated.npz, same class."""
    import os
    from pdeval import native
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             'data', 'kerr_magnetosphere_d3_validated.npz'))
    strings = [str(s) for s in d['exprs']]
    ops, off, _ = native.compile_strings(P.kerr(), strings)
    nat = kerr_ctx.validate(ops, off)
    ref = kerr_ctx.validate(d['ops'], d['offsets'])
    diff = np.flatnonzero(nat['status'] != ref['status'])
    assert not diff.size, [(strings[i], int(nat['status'][i]), int(ref['status'][i])) for i in diff[:10]]
