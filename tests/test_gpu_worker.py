"""GPU: the batched validator worker speaks the reference's queue protocol
(general_method_paper_reproduction.py:1723-1816) and tags the paper's known solutions."""
import queue

import pytest

import golden_data as G

pytestmark = pytest.mark.gpu


def test_worker_queue_protocol_and_tags():
    from pdeval.worker import validator_worker
    rows = G.decided(G.ref_rows('ff_edge.jsonl', 'ff_d2.jsonl'))
    tq, rq = queue.Queue(), queue.Queue()
    for i, r in enumerate(rows):
        tq.put((i + 1, r['expr']))
    tq.put(None)
    n = validator_worker('run_test', None, None, 'force_free', tq, rq, batch_size=64)
    assert n == len(rows)
    msgs = []
    while not rq.empty():
        msgs.append(rq.get())
    ends = [m for m in msgs if m[2] == 'end']
    assert all(m[0] == 'run_test' and m[2] in ('start', 'end') for m in msgs)
    res = {t[5]: t for m in ends for t in m[3]}
    assert len(res) == len(rows)
    for i, r in enumerate(rows):
        status, ok, reason, is_paper, name, eid = res[i + 1]
        assert status == 'completed' and ok == r['ok'], (r['expr'], reason)
    tagged = {rows[eid - 1]['expr']: name for eid, t in res.items() for name in [t[4]] if t[3]}
    # the 6 paper solutions the reference decides, in original and stream forms
    for s in ('rho**2', 'rho**2*z', '1 - z/sqrt(rho**2 + z**2)', 'rho**2/(rho**2 + z**2)**(3/2)',
              'sqrt(rho**2 + z**2) - z', 'rho**2*exp(-2*z)', '-z/sqrt(rho**2 + z**2) + 1',
              'square(rho*exp_neg(z))'):
        assert s in tagged, (s, tagged)


def test_worker_string_fast_path_matches_sympy_path():
    """process_batch on strings (native compiler) == the SymPy-tree path, row for row."""
    from problems import load_problem
    from pdeval.worker import KnownSolutionTagger, _process_batch_strings, process_batch
    rows = G.decided(G.ref_rows(*G.FF_REF, 'ff_edge.jsonl'))
    claimed = [(i + 1, r['expr']) for i, r in enumerate(rows)] + [(0, 'rho +')]
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger(prob, locs)
    kw = {'check_regularity': False, 'fast_point_only': False}
    fast = sorted(_process_batch_strings(claimed, prob.validator, locs, tagger), key=lambda t: t[5])
    slow = sorted(_slow(claimed, prob.validator, kw, locs, tagger), key=lambda t: t[5])
    assert [t[:2] + t[3:] for t in fast] == [t[:2] + t[3:] for t in slow]
    assert [t[2] for t in fast[1:]] == [t[2] for t in slow[1:]]     # same reason strings
    assert fast[0][0] == 'error' and fast[0][2].startswith('Validator Error')
    # process_batch takes the fast path with the driver's kwargs
    assert sorted(process_batch(claimed, prob.validator, kw, locs, tagger), key=lambda t: t[5]) == fast


def _slow(claimed, validator, kw, locs, tagger):
    import sympy as sp
    out, us, ids = [], [], []
    for eid, s in claimed:
        try:
            us.append(sp.sympify(s, locals=locs))
            ids.append(eid)
        except Exception as e:   # noqa: BLE001
            out.append(('error', None, str(e), None, None, eid))
    v = validator.validate_batch(us, **kw)
    valid = [i for i, (ok, _) in enumerate(v) if ok]
    tags = dict(zip(valid, tagger.tag([us[i] for i in valid])))
    for i, (ok, reason) in enumerate(v):
        t = tags.get(i, (False, None))
        out.append(('completed', bool(ok), reason, t[0], t[1], ids[i]))
    return out


def test_worker_with_run_database_and_writer(tmp_path):
    """End to end on the GPU: candidates INSERTed 'pending' into a run table with the
    reference's schema, the GPU worker claims them from the database (compare-and-set claims,
    :1736-1751), the centralized writer applies its result tuples (:1178-1204), and the report
    --print-run-id prints (_generate_report_from_db) has the reference's valid count and the
    paper solutions of the fixtures."""
    import hashlib
    import os
    import threading
    from pdeval import persist
    from pdeval.worker import validator_worker
    rows = G.decided(G.ref_rows('ff_d1.jsonl', 'ff_d2.jsonl', 'ff_edge.jsonl'))
    db = os.path.join(tmp_path, 'run.db')
    run_id = 'gpu-run'
    table = persist.init_run_db(db, run_id)
    seen, items = set(), []
    for r in rows:
        if r['expr'] not in seen:
            seen.add(r['expr'])
            items.append((r['expr'], r['expr'], int(hashlib.sha256(r['expr'].encode()).hexdigest()[:12], 16),
                          r.get('depth', 0)))
    persist.insert_candidates(db, table, items)
    rq = queue.Queue()
    wt = threading.Thread(target=persist.result_writer, args=(run_id, table, db, rq), kwargs={'poll_s': 0.05})
    wt.start()
    n = validator_worker(run_id, table, db, 'force_free', None, rq, batch_size=64, idle_exit_s=1.0)
    rq.put(None)
    wt.join(timeout=60)
    assert n == len(items)
    rep = persist.report(db, table)
    ok = {r['expr']: r['ok'] for r in rows}
    assert rep['not_completed'] == 0
    assert rep['valid'] == sum(ok[e] for e, *_ in items)
    names = {name for _, name in rep['paper_solutions']}
    assert {'Vertical field', 'X-point', 'Radial', 'Dipolar', 'Parabolic', 'Bent'} <= names, names


def _driver_rows():
    import json
    import os
    p = os.path.join(os.path.dirname(__file__), 'golden', 'ref', 'driver_ff_d2_rows.jsonl')
    with open(p) as f:
        return [json.loads(l) for l in f]


def test_reference_driver_inline_rows():
    """The reference driver's own run table (``--max-depth 2 --validators 0``, the rows it
    completed; tests/golden/gen_driver_rows.py) replayed through its inline loop
    (general_method_paper_reproduction.py:1288-1365) with this plugin as ``discovery.validator``:
    every row gets the same validation_status, is_valid and validation_reason text."""
    import sympy as sp
    from problems import load_problem
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    coords = [prob.symbols.get(n, sp.Symbol(n)) for n in ('rho', 'z', 'r', 'x')]
    rows = _driver_rows()
    assert len(rows) == 50
    for r in rows:
        u = sp.sympify(r['expression'], locals=locs)
        if not any(u.has(c) for c in coords):                              # :1292-1294
            ok, reason = False, 'constant-only (skipped)'
        else:
            try:                                                            # :1299-1316
                ok, reason = prob.validator.validate(u, check_regularity=False, fast_point_only=False,
                                                     lean_first=True, defer_heavy_checks=True,
                                                     enforce_anchor=False)
            except TypeError:
                ok, reason = prob.validator.validate(u, check_regularity=False, fast_point_only=False)
        status = 'completed' if ok is not None else 'error'                 # :1358
        assert (status, int(bool(ok)), reason) == \
            (r['validation_status'], r['is_valid'], r['validation_reason']), r['expression']
    desc = prob.validator.describe() if hasattr(prob.validator, 'describe') else {}
    assert (desc or {}).get('method_name') is None and (desc or {}).get('math_definition') is None


def test_reference_driver_rows_through_worker_and_writer(tmp_path):
    """The same run table rebuilt with the reference's schema (same ids, expressions,
    normalized keys, signatures, depths, all 'pending'), drained by the GPU worker pool's claim
    loop and the centralized writer: the rows the reference validated get the same status,
    is_valid and reason (the constant-only row is skipped before validation by the inline
    loop only, so it is not compared)."""
    import os
    import sqlite3
    import threading
    from pdeval import persist
    from pdeval.worker import validator_worker
    rows = _driver_rows()
    db = os.path.join(tmp_path, 'run.db')
    run_id = 'driver-replay'
    table = persist.init_run_db(db, run_id, max_depth=2)
    ids = persist.insert_candidates(db, table, [(r['expression'], r['normalized'], r['signature'], r['depth'])
                                                for r in rows])
    assert ids == [r['id'] for r in rows]
    rq = queue.Queue()
    wt = threading.Thread(target=persist.result_writer, args=(run_id, table, db, rq), kwargs={'poll_s': 0.05})
    wt.start()
    n = validator_worker(run_id, table, db, 'force_free', None, rq, batch_size=16, idle_exit_s=1.0)
    rq.put(None)
    wt.join(timeout=60)
    assert n == len(rows)
    got = {r[0]: r[1:] for r in sqlite3.connect(db).execute(
        f'SELECT id, validation_status, is_valid, validation_reason FROM {table}')}
    for r in rows:
        if r['validation_reason'] == 'constant-only (skipped)':
            continue
        assert got[r['id']] == (r['validation_status'], r['is_valid'], r['validation_reason']), r['expression']


def test_strict_stream_equals_batch_strict():
    """the streaming 'strict' mode (worker.StrictStream inside
    process_batches) emits the same result tuples as the batch-synchronous strict mode
    (process_batch, whose host steps replay every suspect before the batch returns) -- as a
    multiset, since held rows come later -- on the depth-5 rows the default mode gets wrong
    (their replays change verdicts) and a depth-4 sample; the stream's counts add up."""
    from problems import load_problem
    from problems.force_free.validator import PreciseFoliationValidator
    from pdeval.worker import KnownSolutionTagger, process_batch, process_batches
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger(prob, locs)
    strs = sorted(G.FF_OFF_MODE_DIVERGENCE) + [r['expr'] for r in G.ref_rows('ff_d4_s500.jsonl')[:150]]
    strs += list(prob.known_solutions)[:6]
    claimed = [(i + 1, s) for i, s in enumerate(strs)]
    v = PreciseFoliationValidator(symbolic='strict')
    kw = {'check_regularity': False, 'fast_point_only': False}
    sync = []
    for k in range(0, len(claimed), 64):
        sync.extend(process_batch(claimed[k:k + 64], v, kw, locs, tagger))
    stats = {}
    got = [t for r in process_batches((claimed[k:k + 64] for k in range(0, len(claimed), 64)), v, kw, locs,
                                      tagger, stats=stats) for t in r]
    assert sorted(got, key=lambda t: t[5]) == sorted(sync, key=lambda t: t[5])
    assert len(got) == len(claimed)
    assert stats['sent'] >= stats['suspect'] >= stats['replayed'] >= 1
    assert stats['grid_zero'] >= stats['sent']
    off = process_batch(claimed, prob.validator, kw, locs, tagger)
    assert sorted(off, key=lambda t: t[5]) != sorted(got, key=lambda t: t[5])   # the replays changed rows
