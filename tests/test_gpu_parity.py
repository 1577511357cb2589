"""GPU parity: libpdeval.so on the MI355X vs the CPU oracle and vs the reference's verdicts.

Bar (north star): accept/reject verdicts identical to the reference's on every fixture the
reference decided, reason classes identical (100 %), and residuals at the reference point(s)
within 1e-10 relative of the exact values (tests/golden/exact/, SymPy exact arithmetic) and of
the oracle's quad-precision point stage wherever the residual is non-zero.
"""
import json
import os

import numpy as np
import pytest

import golden_data as G
import oracle_lib as O
from pdeval import problem_defs as P
from pdeval._lib import Context
from pdeval.opcodes import FLAG_COMPLEX

pytestmark = pytest.mark.gpu

REL_TOL = 1e-10
EPS = 2.0 ** -52


def check_residuals(dev, ora, strings):
    """Residual at the reference point(s) of every point-stage reject (class REJECT_POINT, so
    the residual is non-zero): the device value (fp64 where its error bound makes it accurate
    to 1e-11, else the double-double tier) agrees with the oracle's quad-precision value to
    1e-10 relative, with no loosening.  (Force-free rejects at one point; a Kerr point reject
    needs one of its three points >= 1e-10, so only those points are compared.)  Every other
    residual is rounding noise of an exact zero, which the equal classes already assert."""
    d, o = dev['res_ref'], ora['res_ref']
    for i in range(len(o)):
        if ora['status'][i] != 1 or not np.all(np.isfinite(o[i])) or not np.all(np.isfinite(d[i])):
            continue    # (a non-finite value is an exact pole: both reject, kerr validator.py:179-183)
        pts = [0] if o.shape[1] == 1 else [k for k in range(o.shape[1]) if abs(o[i, k]) >= 1e-10]
        for k in pts:
            # magnitudes (what the reference prints, "point check ≈ |det|"): a complex residual
            # is reported as its modulus with the sign of its real part, and for a purely
            # imaginary one (det = -8 I q of (1 + I) H) that sign is rounding noise
            err = abs(abs(d[i, k]) - abs(o[i, k])) / max(abs(o[i, k]), 1e-300)
            assert err <= REL_TOL, (strings[i], k, d[i, k], o[i, k], err)


@pytest.fixture(scope='module')
def ff_ctx():
    return Context(0)


def _cmp_device_oracle(ctx, pd_, strings):
    ops, off, _ = P.compile_strings(pd_, strings)
    dev = ctx.validate(ops, off)
    ora = O.validate(pd_.problem_id, ops, off)
    if pd_.problem_id == 1:
        # the host step for values beyond the fp64 range at a reference point (pdeval.batch), on
        # both sides (the quad-precision oracle rarely needs it)
        from pdeval import _lib
        from pdeval.batch import kerr_exact_point_check
        for r in (dev, ora):
            kerr_exact_point_check(pd_, _lib.default_kerr_constants(), strings, r, ops, off)
    assert np.array_equal(dev['status'], ora['status']), \
        [(s, int(a), int(b)) for s, a, b in zip(strings, dev['status'], ora['status']) if a != b][:10]
    # grid counts: equal for every candidate, exactly, except
    #  * a constant u (ZERO_GRADIENT, decided before the grid): its residual is rounding noise
    #    (or exactly 0, by evaluation order), its counts are reported only;
    #  * the candidates listed in golden_data.FF_COUNT_SLACK / KERR_COUNT_SLACK (measured): tier-1
    #    counts of point rejects near tau_grid, and jets overflowing near the 2^160 guard --
    #    within the listed per-candidate amounts
    st = dev['status']
    bad = []
    for i in np.flatnonzero(((dev['n_bad'] != ora['n_bad']) | (dev['n_nonfinite'] != ora['n_nonfinite'])) & (st != 3)):
        nb, nf = (G.FF_COUNT_SLACK if pd_.problem_id == 0 else G.KERR_COUNT_SLACK).get(strings[i], (0, 0))
        if abs(int(dev['n_bad'][i]) - int(ora['n_bad'][i])) > nb or \
                abs(int(dev['n_nonfinite'][i]) - int(ora['n_nonfinite'][i])) > nf:
            bad.append((strings[i], int(st[i]), int(dev['n_bad'][i]), int(ora['n_bad'][i]),
                        int(dev['n_nonfinite'][i]), int(ora['n_nonfinite'][i])))
    assert not bad, bad[:10]
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
    # the host's symbolic zero-gradient step (pdeval.batch), as the product path applies it
    from pdeval.batch import symbolic_zero_gradient
    fixed = symbolic_zero_gradient(pd_, [r['expr'] for r in rows], dev)
    assert all(rows[i]['reason'] == 'Zero gradient (constant expression)' for i in fixed)
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
    text = [(r['expr'], r['reason'], g[1]) for g, r in zip(got, rows)
            if g[1] != r['reason'] and r['expr'] not in G.FF_DET_TEXT]
    assert verdicts == len(rows)
    assert not text, text[:10]     # the reference's reason strings, digits included
    # the per-candidate contract of problems/__init__.py:52
    assert prob.validator.validate(us[0], check_regularity=False) == got[0]
    assert all(prob.validator.validate_known_solutions().values())


def test_plugin_api_reasons_kerr():
    """The Kerr plugin object through validate() / validate_batch() on the GPU: verdicts and
    reason classes of every decided Kerr fixture (kerr validator.py:231-323)."""
    from problems import load_problem
    import sympy as sp
    rows = G.decided(G.ref_rows(*G.KERR_REF, 'kerr_edge.jsonl'))
    prob = load_problem('kerr_magnetosphere')
    locs = {**prob.symbols, **prob.constants, **prob.unary_ops}
    us = [sp.sympify(r['expr'], locals=locs) for r in rows]
    got = prob.validator.validate_batch(us, check_regularity=False, fast_point_only=False,
                                        lean_first=True, defer_heavy_checks=True, enforce_anchor=False)
    bad = [(r['expr'], r['reason'][:60], g[1][:60]) for g, r in zip(got, rows)
           if g[0] != r['ok'] or g[1].split('|')[0] != r['reason'].split('|')[0]]
    assert not bad, bad[:10]
    assert prob.validator.validate(us[0], check_regularity=False) == got[0]


def test_ff_point_stage_exact_ground_truth(ff_ctx):
    """The point stage decides like the reference (validator.py:371-397): on the 905
    exact-determinant ground-truth candidates the device class is REJECT_POINT exactly when
    |det(p*)| >= 1e-20, and res_ref is within 1e-10 relative of the exact |det(p*)|."""
    pd_ = P.force_free()
    rows = G.exact_rows()
    ops, off, _ = P.compile_strings(pd_, [r['expr'] for r in rows])
    dev = ff_ctx.validate(ops, off)
    wrong = [(r['expr'], r['det_abs'][0], int(s)) for r, s in zip(rows, dev['status'])
             if (s == 1) != (r['det_abs'][0] >= 1e-20)]
    assert not wrong, wrong[:10]
    err = [(rows[i]['expr'], abs(abs(dev['res_ref'][i, 0]) - rows[i]['det_abs'][0]) / rows[i]['det_abs'][0])
           for i in range(len(rows)) if rows[i]['det_abs'][0] >= 1e-20]
    assert max(e for _, e in err) <= REL_TOL, sorted(err, key=lambda t: -t[1])[:5]
    counts = ff_ctx.pass_counts()
    assert counts['point_dd'] > 0      # the double-double tier took part


def test_ff_point_reject_hidden_in_fp64_noise(ff_ctx):
    """exp(z/(-rho**2 + z**2)): exact det(p*) = -6.546893155e35, but S = 2.6e48 so fp64 cannot
    tell it from 0.  The reference says 'Invalid (point check ≈ 6.55e+35)'
    (tests/golden/ref/ff_d4_s500.jsonl); so must the device (double-double tier)."""
    from pdeval.batch import reason_for
    pd_ = P.force_free()
    s = 'exp(z/(-rho**2 + z**2))'
    ops, off, _ = P.compile_strings(pd_, [s])
    dev = ff_ctx.validate(ops, off)
    assert int(dev['status'][0]) == 1
    ok, reason = reason_for(0, 1, dev['res_ref'][0], dev['q_ref'][0], dev['q_grid'][0], False)
    assert reason == 'Invalid (point check ≈ 6.55e+35)', reason
    assert abs(dev['res_ref'][0, 0] - (-6.546893154784001770635766939e35)) <= 1e-10 * 6.55e35


def _exact_fixture(name):
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'exact', name)
    if not os.path.exists(p):
        pytest.skip(f'{name} not generated')
    with open(p) as f:
        return [json.loads(line) for line in f]


@pytest.mark.parametrize('prob,name', [('force_free', 'ff_ref_exact.jsonl'),
                                       ('force_free', 'ff_gt_exact.jsonl'),
                                       ('kerr', 'kerr_ref_exact.jsonl')])
def test_residuals_match_exact_values(ff_ctx, kerr_ctx, prob, name):
    """Device res_ref against the exact residuals of every fixture (gen_exact_ref.py: sp.diff,
    exact rational points, evalf(50)): within 1e-10 relative wherever |res| >= 1e-20
    (force-free; complex residuals as their signed modulus) or >= 1e-10 (Kerr, the
    reference's absolute threshold; below it the value is only compared with that threshold)."""
    pd_ = P.get(prob)
    ctx = ff_ctx if pd_.problem_id == 0 else kerr_ctx
    rows = [r for r in _exact_fixture(name) if not r.get('timeout') and 'res' in r]
    ops, off, _ = P.compile_strings(pd_, [r['expr'] for r in rows])
    dev = ctx.validate(ops, off)
    floor = 1e-20 if pd_.problem_id == 0 else 1e-10
    bad, n = [], 0
    for i, r in enumerate(rows):
        if dev['status'][i] in (3, 5, 6):       # constant / unsupported: no point stage
            continue
        if pd_.problem_id == 1 and int(ops[off[i]]) & FLAG_COMPLEX:
            continue                            # Kerr rejects non-real programs unevaluated
        for k, (re_s, im_s) in enumerate(r['res']):
            ex = complex(float(re_s), float(im_s))
            if abs(ex) < floor or not np.isfinite(dev['res_ref'][i, k]):
                continue
            n += 1
            err = abs(abs(dev['res_ref'][i, k]) - abs(ex)) / abs(ex)
            if err > REL_TOL:
                bad.append((r['expr'], k, dev['res_ref'][i, k], abs(ex), err))
    assert n > 0
    assert not bad, (len(bad), n, bad[:8])


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


def test_validate_device_limits_and_bad_programs(ff_ctx):
    """pdeval_validate_device on device buffers: a batch beyond PDEVAL_MAX_BATCH is refused
    (PDEVAL_ERR_ARG, nothing launched); a program whose offsets leave the ops array is
    classified BAD_PROGRAM without being dereferenced; an UNSUPPORTED opcode gives
    UNSUPPORTED; the good programs around them keep their classes."""
    import torch
    from pdeval import _lib
    pd_ = P.force_free()
    progs = [pd_.compile(pd_.parse(s)) for s in ('rho*z', 'rho**2')] + [P.UNSUPPORTED_PROGRAM]
    ops, off = P.pack(progs)
    off = np.concatenate([off, [off[-1] + 1000]])          # a 4th program past the end of ops
    dev = torch.device('cuda:0')
    d_ops = torch.from_numpy(ops).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    n = len(off) - 1
    outs = dict(verdict_bits=torch.zeros(4, dtype=torch.uint8, device=dev),
                status=torch.full((n,), 255, dtype=torch.uint8, device=dev),
                q_ref=torch.zeros(n, dtype=torch.float64, device=dev),
                res_ref=torch.zeros(n, dtype=torch.float64, device=dev),
                q_grid=torch.zeros(n, dtype=torch.float64, device=dev),
                n_bad=torch.zeros(n, dtype=torch.int32, device=dev),
                n_nonfinite=torch.zeros(n, dtype=torch.int32, device=dev),
                fingerprint=torch.zeros(4 * n, dtype=torch.float64, device=dev))
    d_out = _lib.Outputs(*[outs[f].data_ptr() for f, _ in _lib.Outputs._fields_])
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    with pytest.raises(_lib.PdevalError, match='PDEVAL_MAX_BATCH'):
        ff_ctx.validate_device(d_ops.data_ptr(), d_ops.numel(), d_off.data_ptr(), _lib.MAX_BATCH + 1, d_out,
                               stream=stream.cuda_stream)
    ff_ctx.validate_device(d_ops.data_ptr(), d_ops.numel(), d_off.data_ptr(), n, d_out,
                           stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    assert ff_ctx.device_error() == 0
    st = outs['status'].cpu().numpy()
    assert st.tolist() == [1, 0, 5, 6], st           # reject, accept, UNSUPPORTED, BAD_PROGRAM
    bits = np.unpackbits(outs['verdict_bits'].cpu().numpy(), bitorder='little')[:n]
    assert bits.tolist() == [0, 1, 0, 0]


def test_sharded_chain_world1_native_and_torch_gather():
    """The multi-GPU chain at world size 1 on the GPU: shard_ranges -> validate_device on
    the shard -> the one all-gather, both through the C ABI's RCCL communicator
    (pdeval_gather_bits) and through torch.distributed (gloo), equal to the unsharded bitmap."""
    import socket
    import torch
    import torch.distributed as dist
    from pdeval import _lib
    from pdeval.shard import gather_verdicts, gather_verdicts_native, init_native_comm, shard_ranges
    pd_ = P.force_free()
    rows = G.decided(G.ref_rows(*G.FF_REF))
    ops, off, _ = P.compile_strings(pd_, [r['expr'] for r in rows])
    ctx = Context(0)
    ref = ctx.validate(ops, off)
    with socket.socket() as s_:
        s_.bind(('127.0.0.1', 0))
        port = s_.getsockname()[1]
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    try:
        ranges = shard_ranges(len(rows), 1, weights=np.diff(off).astype(float))
        assert ranges == [(0, len(rows))]
        dev = torch.device('cuda:0')
        d_ops = torch.from_numpy(ops).to(dev)
        d_off = torch.from_numpy(off).to(dev)
        n = len(rows)
        bits = torch.zeros(((n + 31) // 32) * 4, dtype=torch.uint8, device=dev)
        d_out = _lib.Outputs(bits.data_ptr(), None, None, None, None, None, None, None)
        stream = torch.cuda.Stream(dev)
        torch.cuda.synchronize(dev)
        ctx.validate_device(d_ops.data_ptr(), d_ops.numel(), d_off.data_ptr(), n, d_out, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        assert ctx.device_error() == 0
        via_torch = gather_verdicts(bits.cpu(), ranges)
        init_native_comm(ctx, 0, 1)
        via_rccl = gather_verdicts_native(ctx, bits, ranges)
        assert np.array_equal(via_torch, ref['verdict'])
        assert np.array_equal(via_rccl, ref['verdict'])
    finally:
        dist.destroy_process_group()
        ctx.close()


@pytest.mark.parametrize('cfg', list(G.KERR_CONFIGS))
def test_kerr_constants_configs(cfg):
    """Kerr at other constants (pdeval_set_kerr_constants): the reference's validator at
    a = 1/10, at a_value = 0 (point check at a = 0, constant test and symbolic stage symbolic in
    a, kerr validator.py:163-192, :231-300) and with the Schwarzschild operator (a = 0 in the
    operator; 66 reference accepts).  Device class == oracle class for every fixture; the
    plugin object, built as the reference's was, answers with the reference's verdict and
    reason class for every decided fixture."""
    import sympy as sp
    from pdeval import _lib
    from pdeval.batch import kerr_exact_point_check
    from problems import load_problem
    kc, files = G.KERR_CONFIGS[cfg]
    pd_ = P.kerr()
    rows = G.decided(G.ref_rows(*files))
    strings = [r['expr'] for r in rows]
    ops, off, _ = P.compile_strings(pd_, strings)
    ctx = Context(1, kerr=_lib.KerrConstants(*kc))
    dev = ctx.validate(ops, off)
    O.set_kerr_constants(kc)
    try:
        ora = O.validate_mt(1, ops, off)
    finally:
        O.set_kerr_constants()
    # the device's classes after the host's exact point check (a = 0, values beyond the fp64
    # range at a reference point); the quad-precision oracle's need no such step
    fixed = kerr_exact_point_check(pd_, _lib.KerrConstants(*kc), strings, dev, ops, off)
    kerr_exact_point_check(pd_, _lib.KerrConstants(*kc), strings, ora, ops, off)
    diff = np.flatnonzero(dev['status'] != ora['status'])
    assert not diff.size, [(strings[i], int(dev['status'][i]), int(ora['status'][i])) for i in diff[:10]]
    ref = np.array([bool(r['ok']) for r in rows])
    assert np.array_equal(dev['verdict'], ref), [(strings[i], rows[i]['reason'][:50]) for i in
                                                 np.flatnonzero(dev['verdict'] != ref)[:10]]
    ctx.close()
    # the drop-in plugin, constructed like the reference's (problems/__init__.py:283)
    from problems.kerr_magnetosphere.validator import KerrMagnetosphereValidator
    prob = load_problem('kerr_magnetosphere')
    s, c = prob.symbols, prob.constants
    a_op = sp.Integer(0) if kc[-1] else c['a']
    v = KerrMagnetosphereValidator(s['r'], s['x'], c['M'], a_op, M_value=sp.Integer(1),
                                   a_value=sp.Rational(kc[2], kc[3]))
    locs = {**s, **c, **prob.unary_ops}
    got = v.validate_batch([sp.sympify(t, locals=locs) for t in strings], check_regularity=False,
                           fast_point_only=False, lean_first=True, defer_heavy_checks=True,
                           enforce_anchor=False)
    bad = [(r['expr'], r['reason'][:60], g[1][:60]) for g, r in zip(got, rows)
           if g[0] != r['ok'] or (g[1].split('|')[0] != r['reason'].split('|')[0] and
                                  (cfg, r['expr']) not in G.KERR_CLASS_DIVERGENCE)]
    assert not bad, bad[:10]
    if kc[-1]:
        assert sum(g[0] for g in got) == 66
    assert cfg != 'a_value=0' or len(fixed) >= 3     # the host step took part


def test_plugin_api_depth5_sample():
    """configs[3]'s depth: the reference's verdicts on the seeded depth-5 sample
    (golden_data.FF_D5) through the plugin on the GPU.  Default mode ('off'): every decided row
    agrees except exactly the rows golden_data.FF_OFF_MODE_DIVERGENCE lists (decided in the
    reference's symbolic stage: its false negatives, squares under fractional powers the
    NONSMOOTH2D rule rejects) -- no allowance; texts equal except the recorded replay's branch
    texts and the point-check numbers of golden_data.FF_D5_POINT_TEXT_DIVERGENCE.  'strict'
    mode: those rows and a seeded sample of the other decided grid zeros get the reference's
    verdict (the whole decided sample, through the recorded replay:
    tests/test_symbolic_replay.py::test_strict_mode_every_decided_row)."""
    import json
    import os
    import random
    from problems import load_problem
    from problems.force_free.validator import PreciseFoliationValidator
    import sympy as sp
    rows = G.decided(G.ref_rows(*G.FF_D5))
    prob = load_problem('force_free')
    locs = {**prob.symbols, **prob.constants, **prob.unary_ops}
    us = [sp.sympify(r['expr'], locals=locs) for r in rows]
    got = prob.validator.validate_batch(us, check_regularity=False, fast_point_only=False)
    with open(os.path.join(G.GOLDEN, 'replay', 'ff_replay.jsonl')) as f:
        rep = {r['expr']: r for r in map(json.loads, f)}
    wrong = {r['expr'] for g, r in zip(got, rows) if g[0] != r['ok']}
    assert wrong <= G.FF_OFF_MODE_DIVERGENCE, sorted(wrong - G.FF_OFF_MODE_DIVERGENCE)
    assert G.FF_D5_SYMBOLIC_DIVERGENCE <= wrong
    for g, r in zip(got, rows):
        if g[0] == r['ok'] and g[1] != r['reason']:
            if r['expr'] in G.FF_D5_POINT_TEXT_DIVERGENCE:
                assert (r['reason'], g[1]) == G.FF_D5_POINT_TEXT_DIVERGENCE[r['expr']]
            else:   # the symbolic stage's other branch text ('text' / 'replay' modes)
                x = rep.get(r['expr'])
                assert x is not None and (x['ok'], x['reason']) == (r['ok'], r['reason']), (r['expr'], r['reason'])
    # 'strict': the divergent rows and a seeded sample of grid zeros (accepted or rule-rejected)
    zero = [i for i, g in enumerate(got) if g[0] or 'Lean could not' in g[1]]
    pick = sorted({i for i, r in enumerate(rows) if r['expr'] in G.FF_OFF_MODE_DIVERGENCE} |
                  set(random.Random(0).sample(zero, min(24, len(zero)))))
    v = PreciseFoliationValidator(symbolic='strict')
    got_s = v.validate_batch([us[i] for i in pick], check_regularity=False, fast_point_only=False)
    bad = [(rows[i]['expr'], rows[i]['reason'], g) for g, i in zip(got_s, pick) if g[0] != rows[i]['ok']]
    assert not bad, bad


def test_plugin_omega1_reference_verdicts():
    """Rotating field lines on the GPU: PreciseFoliationValidator(Omega=1) -- params.omega2 = 1,
    the rotation terms of the device's epilogue in every tier -- gives the reference's verdict
    and text on every decided row it ran with Omega = 1 (the 7 known solutions and a seeded
    d <= 3 sample, tests/golden/ref/ff_omega1_*.jsonl), through trees and through strings."""
    from problems import load_problem
    from problems.force_free.validator import PreciseFoliationValidator
    import sympy as sp
    rows = G.decided(G.ref_rows('ff_omega1_known.jsonl', 'ff_omega1_d3_s600.jsonl'))
    prob = load_problem('force_free')
    locs = {**prob.symbols, **prob.constants, **prob.unary_ops}
    v = PreciseFoliationValidator(Omega=1)
    got = v.validate_batch([sp.sympify(r['expr'], locals=locs) for r in rows], check_regularity=False,
                           fast_point_only=False)
    bad = [(r['expr'], r['reason'], g) for g, r in zip(got, rows) if g != (r['ok'], r['reason'])]
    # (only the symbolic stage's branch text of a grid reject: reproduced in 'text' mode below)
    assert all(g[0] is False and 'expanded det' in rr for _, rr, g in bad) and len(bad) <= 2, bad[:5]
    if bad:
        vt = PreciseFoliationValidator(Omega=1, symbolic='text')
        assert vt.validate_batch([sp.sympify(e, locals=locs) for e, _, _ in bad], check_regularity=False) == \
            [(False, rr) for _, rr, _ in bad]
    got_s = v.validate_strings([r['expr'] for r in rows])
    assert got_s == got
    # and Omega = 0 is untouched: the default validator's verdicts on the same rows differ
    # exactly where the reference's do (Dipolar, Bent ... pass at Omega = 0)
    v0 = PreciseFoliationValidator()
    assert v0.validate(sp.sympify('rho**2*exp(-2*z)'), check_regularity=False)[0] is True


def test_plugin_omega_third_reference_verdicts():
    """Omega = 1/3 on the GPU: Omega^2 = 1/9 is no double, so params carry it as a double-double
    (omega2 + omega2_lo) into the point stage's second tier.  The reference's verdict and text
    on every decided row it ran with Omega = 1/3 (tests/golden/ref/ff_omega13_*.jsonl), among
    them u = z + log(1 - rho**2/9), a solution only at Omega^2 = 1/9 exactly (accepted; with
    Omega^2 rounded to a double the point stage rejects it, test_oracle_omega_third_*)."""
    import os
    from problems import load_problem
    from problems.force_free.validator import PreciseFoliationValidator
    import sympy as sp
    files = [f for f in ('ff_omega13_known.jsonl', 'ff_omega13_d3_s300.jsonl')
             if os.path.exists(os.path.join(G.GOLDEN, 'ref', f))]
    rows = G.decided(G.ref_rows(*files))
    prob = load_problem('force_free')
    locs = {**prob.symbols, **prob.constants, **prob.unary_ops}
    v = PreciseFoliationValidator(Omega=sp.Rational(1, 3))
    assert v.validate(sp.sympify('z + log(1 - rho**2/9)', locals=locs), check_regularity=False) == \
        (True, 'Valid foliation (Lean: det = 0 symbolically)')
    got = v.validate_batch([sp.sympify(r['expr'], locals=locs) for r in rows], check_regularity=False,
                           fast_point_only=False)
    bad = [(r['expr'], r['reason'], g) for g, r in zip(got, rows) if g != (r['ok'], r['reason'])]
    assert all(g[0] is False and 'expanded det' in rr for _, rr, g in bad) and len(bad) <= 2, bad[:5]
    if bad:
        vt = PreciseFoliationValidator(Omega=sp.Rational(1, 3), symbolic='text')
        assert vt.validate_batch([sp.sympify(e, locals=locs) for e, _, _ in bad], check_regularity=False) == \
            [(False, rr) for _, rr, _ in bad]
    assert v.validate_strings([r['expr'] for r in rows]) == got


def _validate_env(pid, ops, off, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ctx = Context(pid)       # (PDEVAL_* are read when the context is created)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        return ctx.validate(ops, off)
    finally:
        ctx.close()


@pytest.mark.parametrize('pid, data, n', [(0, 'force_free_d4_validated.npz', None),
                                          (1, 'kerr_magnetosphere_d4_stream.npz', 200000)])
def test_hoisted_prefix_equals_unhoisted(pid, data, n):
    """The lean passes' hoisted prefixes (pdeval_grid.h PD_HOIST: a program's prefix of x alone
    evaluated once per grid row, of y alone once per lane) change no class, count, point-stage
    residual or fingerprint of the force-free d4 workload (142,004 programs) and of 200,000
    Kerr d4 programs against the run with PDEVAL_HOIST=0, and the grid maxima only in their
    last bits: the prefix runs as a second inlined copy of the interpreter, where the compiler
    may contract a different multiply-add pair into an FMA (measured: 11 force-free point
    rejects, q_grid within 3 ulp).  The rule applies to a good share of the programs
    (pdeval_program_hoist_flops > 0)."""
    from pdeval import workload as WL
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'data', data))
    ops, off = d['ops'], d['offsets']
    if n is not None and len(off) - 1 > n:
        ops, off = WL.gather_programs(ops, off, np.arange(n))
    assert (WL.flops_per_program(pid, ops, off, hoisted=True) > 0).mean() > 0.1   # (FF 44 %, Kerr 12 %)
    on = _validate_env(pid, ops, off, {'PDEVAL_HOIST': '1'})
    off_ = _validate_env(pid, ops, off, {'PDEVAL_HOIST': '0'})
    for k in ('status', 'verdict', 'n_bad', 'n_nonfinite', 'q_ref', 'res_ref', 'fingerprint'):
        if k in on:
            assert np.array_equal(on[k], off_[k], equal_nan=on[k].dtype.kind == 'f'), \
                (k, np.flatnonzero(np.any((on[k] != off_[k]).reshape(len(on[k]), -1), axis=1))[:10])
    a, b = on['q_grid'], off_['q_grid']
    both = np.isfinite(a) & np.isfinite(b)
    assert np.array_equal(np.isfinite(a), np.isfinite(b))
    rel = np.abs(a[both] - b[both]) / np.maximum(np.abs(b[both]), 1e-300)
    assert rel.max(initial=0.0) <= 1e-13 and (rel > 0).mean() < 1e-3, (rel.max(initial=0.0), (rel > 0).sum())


@pytest.mark.parametrize('pid, data, n', [(0, 'force_free_d4_validated.npz', None),
                                          (1, 'kerr_magnetosphere_d4_stream.npz', 200000)])
def test_tier2_masked_equals_full(pid, data, n):
    """Tier 2 re-checks only the grid points tier 1 failed (the lean passes' per-chunk lane masks,
    a.fmask / ESC_MASK) instead of the whole grid: against PDEVAL_TIER2_MASK=0 every class,
    verdict, grid count, maximum and residual of the force-free d4 workload and of 200,000
    Kerr d4 programs is the same.  (A point tier 1 passed cannot be a tier-2 failure: tier 2's
    own tier-1 test is the same arithmetic on the same values.)"""
    from pdeval import workload as WL
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'data', data))
    ops, off = d['ops'], d['offsets']
    if n is not None and len(off) - 1 > n:
        ops, off = WL.gather_programs(ops, off, np.arange(n))
    on = _validate_env(pid, ops, off, {'PDEVAL_TIER2_MASK': '1'})
    off_ = _validate_env(pid, ops, off, {'PDEVAL_TIER2_MASK': '0'})
    for k in ('status', 'verdict', 'n_bad', 'n_nonfinite', 'q_grid', 'q_ref', 'res_ref', 'fingerprint'):
        if k in on:
            assert np.array_equal(on[k], off_[k], equal_nan=on[k].dtype.kind == 'f'), \
                (k, np.flatnonzero(np.any((on[k] != off_[k]).reshape(len(on[k]), -1), axis=1))[:10])


@pytest.mark.parametrize('pid, data', [(0, 'force_free_d4_validated.npz'), (1, 'kerr_magnetosphere_d4_stream.npz')])
def test_deep_lists_split_equals_single_wave(pid, data):
    """The stack-8 lists' generic kernel with each grid split over PD_DEEP_PARTS waves (counts
    merged in the list entry's accumulator) gives every output of the single-wave kernel, on the
    force-free d4 workload (its complex stack-8 list) and the whole Kerr d4 stream (its pass 3)."""
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'data', data))
    ops, off = d['ops'], d['offsets']
    split = _validate_env(pid, ops, off, {'PDEVAL_DEEP_PARTS': '16'})
    single = _validate_env(pid, ops, off, {'PDEVAL_DEEP_PARTS': '1'})
    for k in ('status', 'verdict', 'n_bad', 'n_nonfinite', 'q_grid', 'q_ref', 'res_ref', 'fingerprint'):
        if k in split:
            assert np.array_equal(split[k], single[k], equal_nan=split[k].dtype.kind == 'f'), \
                (k, np.flatnonzero(np.any((split[k] != single[k]).reshape(len(split[k]), -1), axis=1))[:10])


def test_plugin_range_rows_reference_verdicts():
    """The force-free point rejects only the fp64 range caused (tests/test_range_rows.py): on the
    GPU, through the plugin (the device and the host steps), every row the reference decided
    at 120 s gets its verdict -- 10 of the 12 are true solutions the device alone rejects."""
    from problems import load_problem
    import sympy as sp
    rows = G.decided(G.ref_rows('ff_range_rows.jsonl'))
    assert len(rows) >= 12
    prob = load_problem('force_free')
    locs = {**prob.symbols, **prob.constants, **prob.unary_ops}
    got = prob.validator.validate_batch([sp.sympify(r['expr'], locals=locs) for r in rows],
                                        check_regularity=False, fast_point_only=False)
    bad = [(r['expr'], r['ok'], g) for g, r in zip(got, rows) if g[0] != r['ok']]
    assert not bad, bad
    assert sum(g[0] for g in got) >= 10


def test_plugin_api_depth5_faithful():
    """configs[3]'s depth on the reference's OWN depth-5 distribution: the
    faithful sample's decided rows (G.ff_d5f_files(); the suspect rule frozen before the sample
    was drawn) through the plugin on the GPU, default mode: every verdict equals the
    reference's except the rows G.FF_D5F_OFF_DIVERGENCE lists (4 of 2,066 decided rows, all
    functions of rho/z whose det == 0 the reference's symbolic stage does not reduce); reason
    texts are reported."""
    from problems import load_problem
    import sympy as sp
    files = G.ff_d5f_files()
    if not files:
        pytest.skip('no faithful d5 verdicts recorded')
    rows = G.decided(G.ref_rows(*files))
    prob = load_problem('force_free')
    locs = {**prob.symbols, **prob.constants, **prob.unary_ops}
    us = [sp.sympify(r['expr'], locals=locs) for r in rows]
    got = prob.validator.validate_batch(us, check_regularity=False, fast_point_only=False)
    wrong = {r['expr'] for g, r in zip(got, rows) if g[0] != r['ok']}
    assert wrong <= G.FF_D5F_OFF_DIVERGENCE, sorted(wrong - G.FF_D5F_OFF_DIVERGENCE)[:20]
    texts = sum(1 for g, r in zip(got, rows) if g[1] == r['reason'])
    print(f'faithful d5: {len(rows)} decided rows, verdicts equal {len(rows) - len(wrong)}, texts equal {texts}')
