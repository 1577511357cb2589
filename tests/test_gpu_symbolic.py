"""GPU tests of the named host modes that reproduce the reference's symbolic stage
(pdeval.symbolic; plugin argument / env PDEVAL_SYMBOLIC) and of the small-batch graph path.

* 'text'   -- force-free grid rejects get the reference's branch text ("Invalid (expanded det
  != 0)" for a det string of 3,000+ characters, validator.py:404-427): golden_data.FF_DET_TEXT
  is reproduced; Kerr rejects get the reference's exact text with its 240-character residual
  repr and last_evidence() its evidence dict (kerr validator.py:249-306).  The reference
  driver's Kerr run table replays through the inline loop (reason, method, math, evidence)
  and the worker + writer (reason) with identical columns.
* 'replay' -- the reference's symbolic verdict for grid zeros: the depth-5 false negative
  golden_data.FF_D5_SYMBOLIC_DIVERGENCE is reproduced.
* pdeval_validate_batch's HIP-graph path for batches of <= 64 candidates gives exactly the
  direct path's outputs.
"""
import json
import os
import queue
import random

import numpy as np
import pytest
import sympy as sp

import golden_data as G

pytestmark = pytest.mark.gpu

FF_SYMBOLIC_FILES = ('ff_d1.jsonl', 'ff_d2.jsonl', 'ff_d3_s500.jsonl', 'ff_d4_s500.jsonl', 'ff_d4_s2000.jsonl',
                     'ff_d4_exp_quarter.jsonl', 'ff_edge.jsonl', 'ff_exp_power_forms.jsonl')


def _locs(prob):
    return {**prob.unary_ops, **prob.symbols, **prob.constants}


def test_ff_text_mode_reject_texts():
    """Every decided force-free fixture row the reference rejected in its symbolic stage, through
    the plugin in 'text' mode: verdict and exact text (the FF_DET_TEXT row included)."""
    from problems.force_free.validator import PreciseFoliationValidator
    from problems import load_problem
    prob = load_problem('force_free')
    rows = [r for r in G.decided(G.ref_rows(*FF_SYMBOLIC_FILES))
            if not r['ok'] and ('Lean could not' in r['reason'] or 'expanded det' in r['reason'])]
    assert {r['expr'] for r in rows} >= G.FF_DET_TEXT
    v = PreciseFoliationValidator(symbolic='text')
    us = [sp.sympify(r['expr'], locals=_locs(prob)) for r in rows]
    got = v.validate_batch(us, check_regularity=False, fast_point_only=False)
    bad = [(r['expr'], r['reason'], g) for g, r in zip(got, rows) if (g[0], g[1]) != (r['ok'], r['reason'])]
    assert not bad, bad[:5]
    by = {r['expr']: g for g, r in zip(got, rows)}
    for e in G.FF_DET_TEXT:
        assert by[e] == (False, 'Invalid (expanded det != 0)')


def test_ff_replay_mode_depth5():
    """configs[3]'s depth in 'replay' mode: the reference's verdict and text on the depth-5
    false negative and on a seeded sample of decided depth-5 rows that reached its symbolic
    stage (the whole decided sample is checked on the CPU: test_oracle_golden.py)."""
    from problems.force_free.validator import PreciseFoliationValidator
    from problems import load_problem
    prob = load_problem('force_free')
    rows = G.decided(G.ref_rows(*G.FF_D5))
    sym = [r for r in rows if r['ok'] or 'Lean could not' in r['reason'] or 'expanded det' in r['reason']]
    pick = [r for r in sym if r['expr'] in G.FF_D5_SYMBOLIC_DIVERGENCE]
    pick += random.Random(0).sample([r for r in sym if r['expr'] not in G.FF_D5_SYMBOLIC_DIVERGENCE], 16)
    pick += random.Random(1).sample([r for r in rows if 'point check' in r['reason']
                                     and r['expr'] not in G.FF_D5_POINT_TEXT_DIVERGENCE], 8)
    v = PreciseFoliationValidator(symbolic='replay')
    us = [sp.sympify(r['expr'], locals=_locs(prob)) for r in pick]
    got = v.validate_batch(us, check_regularity=False, fast_point_only=False)
    bad = [(r['expr'], r['reason'], g) for g, r in zip(got, pick) if (g[0], g[1]) != (r['ok'], r['reason'])]
    assert not bad, bad
    # and 'off' keeps the device's (true) verdict on the false negative
    off = PreciseFoliationValidator(symbolic='off')
    e = sorted(G.FF_D5_SYMBOLIC_DIVERGENCE)[0]
    assert off.validate(sp.sympify(e, locals=_locs(prob)), check_regularity=False)[0] is True


def _kerr_driver_rows():
    with open(os.path.join(G.GOLDEN, 'ref', 'driver_kerr_d2_rows.jsonl')) as f:
        return [json.loads(l) for l in f]


def test_kerr_driver_inline_rows_text_mode():
    """The reference driver's Kerr run table (--problem kerr_magnetosphere --max-depth 2
    --validators 0, tests/golden/gen_driver_rows.py) through its inline loop
    (general_method_paper_reproduction.py:1288-1365) with this plugin in 'text' mode:
    validation_status, is_valid, validation_reason, validator_method, validator_math and
    validator_evidence (json of last_evidence()) identical on every row."""
    from problems import load_problem
    prob = load_problem('kerr_magnetosphere')
    v = prob.validator
    v.symbolic = 'text'
    locs = _locs(prob)
    coords = [prob.symbols.get(n, sp.Symbol(n)) for n in ('rho', 'z', 'r', 'x')]
    rows = _kerr_driver_rows()
    assert len(rows) == 306
    bad = []
    for r in rows:
        u = sp.sympify(r['expression'], locals=locs)
        if not any(u.has(c) for c in coords):                               # :1292-1294
            ok, reason = False, 'constant-only (skipped)'
        else:
            ok, reason = v.validate(u, check_regularity=False, fast_point_only=False, lean_first=True,
                                    defer_heavy_checks=True, enforce_anchor=False)
        desc, ev = v.describe() or {}, v.last_evidence() or {}              # :1324-1335 (every row)
        got = ('completed', int(bool(ok)), reason, desc.get('method_name'), desc.get('math_definition'),
               json.dumps(ev))
        want = (r['validation_status'], r['is_valid'], r['validation_reason'], r['validator_method'],
                r['validator_math'], r['validator_evidence'])
        if got != want:
            bad.append((r['expression'], got[2][:80], want[2][:80]))
    assert not bad, bad[:5]


def test_kerr_driver_rows_worker_text_mode(tmp_path, monkeypatch):
    """The same run table drained by the GPU worker pool and the centralized writer with
    PDEVAL_SYMBOLIC=text: identical status, is_valid and reason (the worker's result tuples
    carry no evidence: general_method_paper_reproduction.py:1799-1816)."""
    import sqlite3
    import threading
    from pdeval import persist
    from pdeval.worker import validator_worker
    monkeypatch.setenv('PDEVAL_SYMBOLIC', 'text')
    rows = [r for r in _kerr_driver_rows() if r['validation_reason'] != 'constant-only (skipped)']
    db = os.path.join(tmp_path, 'run.db')
    run_id = 'kerr-driver-replay'
    table = persist.init_run_db(db, run_id, max_depth=2)
    ids = persist.insert_candidates(db, table, [(r['expression'], r['normalized'], r['signature'], r['depth'])
                                                for r in rows])
    rq = queue.Queue()
    wt = threading.Thread(target=persist.result_writer, args=(run_id, table, db, rq), kwargs={'poll_s': 0.05})
    wt.start()
    n = validator_worker(run_id, table, db, 'kerr_magnetosphere', None, rq, batch_size=64, idle_exit_s=1.0)
    rq.put(None)
    wt.join(timeout=120)
    assert n == len(rows)
    got = {r[0]: r[1:] for r in sqlite3.connect(db).execute(
        f'SELECT id, validation_status, is_valid, validation_reason FROM {table}')}
    bad = [(r['expression'], got[i][2][:60]) for i, r in zip(ids, rows)
           if got[i] != (r['validation_status'], r['is_valid'], r['validation_reason'])]
    assert not bad, bad[:5]


def test_kerr_plugin_evidence_text_mode():
    """last_evidence() after validate(u) in 'text' mode: the reference's dict for rows past
    its fast point check (gen_reference_verdicts.py --evidence; a fresh validator per row)."""
    from problems.kerr_magnetosphere.validator import KerrMagnetosphereValidator
    from problems import load_problem
    prob = load_problem('kerr_magnetosphere')
    locs = _locs(prob)
    s, c = prob.symbols, prob.constants
    rows = [r for r in G.decided(G.ref_rows('kerr_evidence.jsonl'))
            if 'fast point' not in r['reason'] and '(cached)' not in r['reason']][:12]
    assert rows
    for r in rows:
        v = KerrMagnetosphereValidator(s['r'], s['x'], c['M'], c['a'], symbolic='text')
        ok, reason = v.validate(sp.sympify(r['expr'], locals=locs), check_regularity=False,
                                fast_point_only=False, lean_first=True, defer_heavy_checks=True,
                                enforce_anchor=False)
        assert (ok, reason) == (r['ok'], r['reason']), r['expr']
        assert v.last_evidence() == r['evidence'], r['expr']


def _device_outputs(ctx, o, f, n_ref):
    """pdeval_validate_device on device-resident programs: their depths are unknown to the host,
    so every pass of the chain is launched."""
    import torch
    from pdeval import _lib
    n = len(f) - 1
    dev = torch.device('cuda:0')
    d_ops = torch.from_numpy(np.ascontiguousarray(o, dtype=np.int32)).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(f, dtype=np.int64)).to(dev)
    outs = dict(verdict_bits=torch.zeros(((n + 31) // 32) * 4, dtype=torch.uint8, device=dev),
                status=torch.zeros(n, dtype=torch.uint8, device=dev),
                q_ref=torch.zeros(n, dtype=torch.float64, device=dev),
                res_ref=torch.zeros(n * n_ref, dtype=torch.float64, device=dev),
                q_grid=torch.zeros(n, dtype=torch.float64, device=dev),
                n_bad=torch.zeros(n, dtype=torch.int32, device=dev),
                n_nonfinite=torch.zeros(n, dtype=torch.int32, device=dev),
                fingerprint=torch.zeros(4 * n, dtype=torch.float64, device=dev))
    d_out = _lib.Outputs(*[outs[k].data_ptr() for k, _ in _lib.Outputs._fields_])
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    ctx.validate_device(d_ops.data_ptr(), d_ops.numel(), d_off.data_ptr(), n, d_out, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    assert ctx.device_error() == 0
    r = {k: v.cpu().numpy() for k, v in outs.items()}
    r['verdict'] = np.unpackbits(r.pop('verdict_bits'), bitorder='little')[:n].astype(bool)
    return r


def test_small_batch_graph_path_equals_direct():
    """pdeval_validate_batch replays the launch chain of <= 64 candidates as a captured HIP
    graph; a context created with PDEVAL_GRAPH=0 takes the direct path.  Every output is equal,
    for batch sizes on both sides of the limit and after the buffers grow.  Both skip the
    passes only deeper programs reach (the host knows the batch's largest depth); the device
    entry, which launches them all, gives the same outputs too."""
    from pdeval import problem_defs as P
    from pdeval._lib import Context
    pd_ = P.force_free()
    strs = list(pd_.known_solutions) + [r['expr'] for r in G.decided(G.ref_rows('ff_edge.jsonl', 'ff_d2.jsonl'))]
    strs += [r['expr'] for r in G.decided(G.ref_rows('ff_d4_s500.jsonl'))][:200]
    ops, off, _ = P.compile_strings(pd_, strs)
    g = Context(pd_.problem_id, device=0)
    old = os.environ.get('PDEVAL_GRAPH')
    os.environ['PDEVAL_GRAPH'] = '0'
    try:
        d = Context(pd_.problem_id, device=0)
    finally:
        if old is None:
            del os.environ['PDEVAL_GRAPH']
        else:
            os.environ['PDEVAL_GRAPH'] = old
    from pdeval.workload import gather_programs
    try:
        for start, n in ((0, 7), (0, 1), (0, 1), (3, 3), (7, 64), (71, 64), (0, 65), (0, 200), (9, 2), (5, 1), (0, 7)):
            idx = (start + np.arange(n)) % len(strs)
            o, f = gather_programs(ops, off, idx)
            a, b = g.validate(o, f), d.validate(o, f)
            full = _device_outputs(d, o, f, d.n_ref)
            for k in ('status', 'verdict', 'q_ref', 'res_ref', 'q_grid', 'n_bad', 'n_nonfinite', 'fingerprint'):
                x = np.asarray(a[k])
                assert np.array_equal(x, np.asarray(b[k]), equal_nan=x.dtype.kind == 'f'), (n, k)
                assert np.array_equal(x.ravel(), full[k].ravel(), equal_nan=x.dtype.kind == 'f'), (n, k, 'device')
    finally:
        g.close()
        d.close()


def test_graph_replay_after_large_batches():
    """The round-5 fault's sequence (DESIGN.md §3 "Robustness of the launch chain"): a small
    batch captures its graph, a large direct batch (and a large device-entry batch) leaves the
    list counters high, then the SAME small graph is replayed.  Every replay must start from
    zeroed counters: the device error word stays 0 and the outputs equal a PDEVAL_GRAPH=0
    context's, call after call."""
    from pdeval import problem_defs as P
    from pdeval.workload import gather_programs
    pd_ = P.force_free()
    strs = [r['expr'] for r in G.decided(G.ref_rows('ff_d4_s2000.jsonl'))]
    ops, off, _ = P.compile_strings(pd_, strs)
    g = _ctx_with_env(pd_.problem_id, {})
    d = _ctx_with_env(pd_.problem_id, {'PDEVAL_GRAPH': '0'})
    small = gather_programs(ops, off, np.arange(7))
    big_idx = np.arange(20000) % len(strs)
    big = gather_programs(ops, off, big_idx)
    keys = ('status', 'verdict', 'q_ref', 'res_ref', 'q_grid', 'n_bad', 'n_nonfinite', 'fingerprint')
    try:
        want = d.validate(*small)
        for step in ('capture', 'direct', 'replay', 'device', 'replay'):
            if step == 'direct':
                big_out = g.validate(*big)
                assert np.array_equal(np.asarray(big_out['status']), np.asarray(d.validate(*big)['status']))
                continue
            if step == 'device':
                _device_outputs(g, big[0], big[1], g.n_ref)   # asserts the error word itself
                continue
            got = g.validate(*small)
            assert g.device_error() == 0, step
            for k in keys:
                x = np.asarray(got[k])
                assert np.array_equal(x, np.asarray(want[k]), equal_nan=x.dtype.kind == 'f'), (step, k)
    finally:
        g.close()
        d.close()


def _ctx_with_env(problem_id, env, **kw):
    """A Context created with the given PDEVAL_* environment (read once, at pdeval_create)."""
    from pdeval._lib import Context
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Context(problem_id, device=0, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def test_small_batch_graph_after_set_kerr_constants():
    """A captured small-batch graph holds the Kerr constants by value; pdeval_set_kerr_constants
    must drop it.  Validate <= 64 candidates, change the constants, validate again: the outputs
    equal those of a fresh context built with the new constants and of one with PDEVAL_GRAPH=0."""
    from pdeval import problem_defs as P
    from pdeval import _lib
    from pdeval.workload import gather_programs
    pd_ = P.kerr()
    kc_a, _ = G.KERR_CONFIGS['a=1/10']
    kc_b, files_b = G.KERR_CONFIGS['a_value=0']
    strs = [r['expr'] for r in G.ref_rows(*files_b)][:400]
    ops, off, _ = P.compile_strings(pd_, strs)
    g = _ctx_with_env(pd_.problem_id, {}, kerr=_lib.KerrConstants(*kc_a))
    fresh = _ctx_with_env(pd_.problem_id, {}, kerr=_lib.KerrConstants(*kc_b))
    direct = _ctx_with_env(pd_.problem_id, {'PDEVAL_GRAPH': '0'}, kerr=_lib.KerrConstants(*kc_b))
    try:
        changed = 0
        for start, n in ((0, 64), (64, 1), (100, 37)):
            idx = (start + np.arange(n)) % len(strs)
            o, f = gather_programs(ops, off, idx)
            g.set_kerr_constants(_lib.KerrConstants(*kc_a))
            before = g.validate(o, f)                      # captures / replays the a = 1/10 graph
            g.set_kerr_constants(_lib.KerrConstants(*kc_b))
            a, b, c = g.validate(o, f), fresh.validate(o, f), direct.validate(o, f)
            changed += int(np.any(before['res_ref'] != a['res_ref']))
            for k in ('status', 'verdict', 'q_ref', 'res_ref', 'q_grid', 'n_bad', 'n_nonfinite', 'fingerprint'):
                x = np.asarray(a[k])
                assert np.array_equal(x, np.asarray(b[k]), equal_nan=x.dtype.kind == 'f'), (n, k, 'fresh')
                assert np.array_equal(x, np.asarray(c[k]), equal_nan=x.dtype.kind == 'f'), (n, k, 'direct')
        assert changed, 'the constants change the reference-point residuals'
    finally:
        g.close()
        fresh.close()
        direct.close()


@pytest.mark.parametrize('n', [1023, 1024, 4096])
def test_dd_early_split_equals_single_tier(n):
    """The double-double tier beside the grid (PDEVAL_DD_EARLY=1: the P0_DD lists on a side
    stream, dd_apply_kernel after the join) gives exactly the outputs of the single tier after
    the grid (PDEVAL_DD_EARLY=0), at sizes on both sides of where the early path starts (1,024)
    and where the small-batch row split ends."""
    from pdeval import problem_defs as P
    from pdeval.workload import gather_programs
    pd_ = P.force_free()
    strs = [r['expr'] for r in G.ref_rows('ff_d4_s2000.jsonl', 'ff_d4_s500.jsonl', 'ff_edge.jsonl', 'ff_d3_s500.jsonl')]
    ops, off, _ = P.compile_strings(pd_, strs)
    idx = np.random.default_rng(n).permutation(np.resize(np.arange(len(strs)), n))
    o, f = gather_programs(ops, off, idx)
    e1 = _ctx_with_env(pd_.problem_id, {'PDEVAL_DD_EARLY': '1'})
    e0 = _ctx_with_env(pd_.problem_id, {'PDEVAL_DD_EARLY': '0'})
    try:
        a, b = e1.validate(o, f), e0.validate(o, f)
        da, db = _device_outputs(e1, o, f, e1.n_ref), _device_outputs(e0, o, f, e0.n_ref)
        for k in ('status', 'verdict', 'q_ref', 'res_ref', 'q_grid', 'n_bad', 'n_nonfinite', 'fingerprint'):
            x = np.asarray(a[k])
            assert np.array_equal(x, np.asarray(b[k]), equal_nan=x.dtype.kind == 'f'), (n, k)
            assert np.array_equal(da[k], db[k], equal_nan=da[k].dtype.kind == 'f'), (n, k, 'device')
        assert np.array_equal(da['status'], np.asarray(a['status']))
    finally:
        e1.close()
        e0.close()


@pytest.mark.gpu
@pytest.mark.parametrize('problem, name, n', [('force_free', 'force_free_d4_validated', 0),
                                              ('kerr_magnetosphere', 'kerr_magnetosphere_d4_stream', 200000)])
def test_dd_speculative_provisional_equals_late(problem, name, n):
    """PD_DD_SPEC: the provisional point passes (P0_PROV) run in the early double-double tier
    beside the grid, their outputs held in side arrays and applied after the grid only where the
    final class calls for them -- exactly the outputs of the late tier after the grid
    (PDEVAL_DD_SPEC=0), on the whole force-free d4 workload and 200,000 Kerr d4 programs, at the
    workload size and at a worker queue batch."""
    from pdeval import problem_defs as P
    from pdeval.workload import load_programs, gather_programs
    pd_ = P.get(problem)
    ops, off, _ = load_programs(name)
    idx = np.arange(len(off) - 1)
    if n:
        idx = np.random.default_rng(0).choice(idx, n, replace=False)
    on = _ctx_with_env(pd_.problem_id, {'PDEVAL_DD_SPEC': '1'})
    no = _ctx_with_env(pd_.problem_id, {'PDEVAL_DD_SPEC': '0'})
    try:
        for sel in (idx, idx[:4096]):
            o, f = gather_programs(ops, off, sel)
            a, b = on.validate(o, f), no.validate(o, f)
            for k in ('status', 'verdict', 'q_ref', 'res_ref', 'q_grid', 'n_bad', 'n_nonfinite', 'fingerprint'):
                x = np.asarray(a[k])
                assert np.array_equal(x, np.asarray(b[k]), equal_nan=x.dtype.kind == 'f'), (problem, len(sel), k)
            assert on.device_error() == 0 and no.device_error() == 0
    finally:
        on.close()
        no.close()
