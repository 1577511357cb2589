"""CPU tests: the native candidate compiler (csrc/pdcompile.cpp, C ABI pdeval_compile_batch)
against SymPy, which is what the reference parses with (``sp.sympify(s, locals=...)``,
general_method_paper_reproduction.py:84-93, :1767).

* structure: for every string it compiles, the canonical form of its evaluated tree equals that
  of sympify's tree (same Add/Mul/Pow/exp/Abs nodes, same exact rationals), on the committed
  candidate streams (all of force-free d<=3, a seeded sample of d4 and of Kerr d<=3);
* programs: header flags (NOCOORD, RATIONAL, NONSMOOTH2D, COMPLEX) equal flatten.py's;
* verdicts: the hybrid compile (native, SymPy for declined strings) gives the oracle the same
  class as the SymPy path on every reference fixture, and the reference's verdict;
* the declined share stays small (those strings cost what they cost today).
The full streams (142,004 d4 strings) are checked by scripts/native_parity.py and on the GPU by
tests/test_gpu_parity.py::test_native_compile_full_d4.
"""
import gzip
import os
import random

import numpy as np
import pytest

import golden_data as G
import oracle_lib as O
from pdeval import native
from pdeval import problem_defs as P
from pdeval.batch import reason_for
from pdeval.opcodes import FLAG_RATIONAL

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STREAMS = os.path.join(ROOT, 'tests', 'golden', 'streams')
DEPTH_MASK = ~0xff00   # the stack depth may differ (argument order of equal-need terms)


def _stream(name):
    with gzip.open(os.path.join(STREAMS, name), 'rt') as f:
        return [line.rstrip('\n').split('\t')[-1] for line in f]


def _sample(xs, k, seed=0):
    if len(xs) <= k:
        return xs
    return random.Random(seed).sample(xs, k)


def _check_structure(prob, strings, max_declined):
    pd_ = P.get(prob)
    ops, off, st = native.compile_native(pd_.problem_id, strings)
    bad = []
    for i, s in enumerate(strings):
        if st[i] != native.COMPILE_OK:
            continue
        _, cn = native.canonical(pd_.problem_id, s)
        e = pd_.parse(s)
        cs = native.sympy_canonical(e)
        if cn != cs:
            bad.append((s, cn, cs))
            continue
        w = pd_.compile(e)
        if (int(ops[off[i]]) & DEPTH_MASK) != (w[0] & DEPTH_MASK):
            bad.append((s, hex(int(ops[off[i]])), hex(w[0])))
    assert not bad, bad[:10]
    declined = int((st != native.COMPILE_OK).sum())
    assert declined <= max_declined * len(strings), declined
    return declined


def test_structure_force_free_d3_all():
    _check_structure('force_free', _stream('force_free_d3_validated.txt.gz'), 0.02)


def test_structure_force_free_d4_sample():
    _check_structure('force_free', _sample(_stream('force_free_d4_validated.txt.gz'), 3000), 0.03)


def test_structure_kerr_d3_sample():
    _check_structure('kerr', _sample(_stream('kerr_magnetosphere_d3_validated.txt.gz'), 2000), 0.03)


# constructs whose SymPy evaluation depends on assumptions or on nested-power rules
EDGE = ['sqrt(rho**2/z**2)', 'sqrt(z**2)', 'pow_3_2(square(z))', '(z**(3/2))**(3/2)',
        '(rho**(3/2))**(3/2)', 'sqrt(exp(z))', 'sqrt(exp(rho/z))', 'exp(z)/exp(z)**2',
        '(rho*z)**(3/2)', '(-z)**(1/2)', '-(rho+z)', '2*(rho+z)/3', '(rho+z)*2*rho',
        'rho**2 - rho + z**2 - square(rho)', 'neg(z)/z', 'inv(rho/z)', '(1/z)**(1/2)',
        'sqrt(1/rho)', 'pow_neg_3_2(1/z)', 'square(pow_3_2(square(z)))',
        'inv(pow_3_2(square(rho/z)))', 'neg(pow_3_2(square(rho/z)))', 'square(sqrt(neg(rho/z)))',
        'E*exp(rho)', 'exp(-1)*exp(rho)', 'Abs(-rho-1)', 'Abs(rho*z)', 'exp(rho+z)**2',
        'z**(1/2)*z**(3/2)*rho', 'rho/(2*(rho+z))', '1/(1/z)', 'sqrt((rho-z)**2)',
        '(z**2*(rho+z))**(1/2)', 'rho**2*exp(-2*z)', 'sqrt(z**2 + (rho - 1)**2) - sqrt(z**2 + (rho + 1)**2)']


@pytest.mark.parametrize('s', EDGE)
def test_edge_structure(s):
    pd_ = P.force_free()
    st, cn = native.canonical(pd_.problem_id, s)
    if st != native.COMPILE_OK:
        pytest.skip('declined (compiled through SymPy)')
    assert cn == native.sympy_canonical(pd_.parse(s))


def test_parse_errors_and_declines():
    pd_ = P.force_free()
    ops, off, st = native.compile_native(pd_.problem_id, ['rho +', 'log(rho)', '1.5*rho', 'I*z', 'rho'])
    assert list(st) == [native.COMPILE_PARSE, native.COMPILE_DECLINED, native.COMPILE_DECLINED,
                        native.COMPILE_DECLINED, native.COMPILE_OK]
    assert off[4] == off[0] and off[5] > off[4]


def test_hybrid_equals_sympy_programs_where_identical():
    """The splice of native and SymPy-compiled programs keeps every candidate in place."""
    pd_ = P.force_free()
    strings = ['rho', 'log(rho)', 'rho**2*z', '1.5*rho', 'sqrt(2)*sqrt(z)', 'exp(rho*z)']
    ops, off, notes = native.compile_strings(pd_, strings)
    s_ops, s_off, _ = P.compile_strings(pd_, strings)
    for i in range(len(strings)):
        a = ops[off[i]:off[i + 1]]
        b = s_ops[s_off[i]:s_off[i + 1]]
        assert (a[0] & DEPTH_MASK) == (b[0] & DEPTH_MASK), strings[i]
    for i in (1, 3, 4):   # declined: compiled by SymPy, so identical
        assert np.array_equal(ops[off[i]:off[i + 1]], s_ops[s_off[i]:s_off[i + 1]])


@pytest.mark.parametrize('prob,files', [('force_free', G.FF_REF + ('ff_edge.jsonl',)),
                                        ('kerr', G.KERR_REF + ('kerr_edge.jsonl',))])
def test_native_verdicts_match_reference_and_sympy_path(prob, files):
    pd_ = P.get(prob)
    rows = G.decided(G.ref_rows(*files))
    strings = [r['expr'] for r in rows]
    ops, off, notes = native.compile_strings(pd_, strings)
    s_ops, s_off, _ = P.compile_strings(pd_, strings)
    res = O.validate(pd_.problem_id, ops, off)
    ref = O.validate(pd_.problem_id, s_ops, s_off)
    assert np.array_equal(res['status'], ref['status']), \
        [(strings[i], int(res['status'][i]), int(ref['status'][i]))
         for i in np.flatnonzero(res['status'] != ref['status'])[:10]]
    from pdeval.batch import symbolic_zero_gradient
    symbolic_zero_gradient(pd_, strings, res)      # the host step of pdeval.batch
    bad = []
    for i, r in enumerate(rows):
        ok, _ = reason_for(pd_.problem_id, int(res['status'][i]), res['res_ref'][i], res['q_ref'][i],
                           res['q_grid'][i], bool(int(ops[off[i]]) & FLAG_RATIONAL), notes[i])
        if ok != r['ok']:
            bad.append((r['expr'], r['reason']))
    assert not bad, bad[:10]


def test_compile_batch_mt_identical_to_single_thread():
    """pdeval_compile_batch_mt (host threads, chunks claimed dynamically) writes exactly the
    single-threaded compile: same words, offsets and statuses, at several thread counts."""
    strings = _stream('force_free_d4_validated.txt.gz')[:20000] + ['rho +', 'sqrt(2)*rho', '']
    pd_ = P.force_free()
    ops1, off1, st1 = native.compile_native(pd_.problem_id, strings, threads=1)
    for t in (2, 3, 8):
        ops, off, st = native.compile_native(pd_.problem_id, strings, threads=t)
        assert np.array_equal(st, st1) and np.array_equal(off, off1) and np.array_equal(ops, ops1), t


@pytest.mark.parametrize('prob', ['force_free', 'kerr_magnetosphere'])
def test_format_reasons_equals_reason_for(prob):
    """pdeval_format_reasons (csrc/pdreasons.cpp) == batch.reason_for for every class, with
    residuals across the whole double range (printf %.2e/%.3e vs Python's format rounding),
    non-finite values and the rational flag."""
    from pdeval.batch import format_reasons
    pd_ = P.get(prob)
    rng = np.random.default_rng(7)
    n = 200000
    st = rng.integers(0, 9, n).astype(np.uint8)
    vals = rng.standard_normal(n) * 10.0 ** rng.integers(-320, 308, n)
    # values that sit on a rounding boundary of 3 / 4 significant digits, and specials
    vals[:2000] = np.array([1.005, 2.675, 9.995, 1.0049999999999999, 0.125, 6.0650e-5] * 334)[:2000]
    vals[2000:2010] = [np.inf, -np.inf, np.nan, -np.nan, 0.0, -0.0, 5e-324, 1.7976931348623157e308, 1e-20, 1e-10]
    n_ref = 1 if prob == 'force_free' else 3
    res = np.repeat(vals[:, None], n_ref, axis=1) * (1 + np.arange(n_ref))
    q_ref, q_grid = np.abs(np.roll(vals, 1)), np.abs(np.roll(vals, 2))
    q_ref[5:10] = [np.nan, np.inf, 0.0, 1e-300, 9.9995e-11]
    rat = (rng.random(n) < 0.3).astype(np.uint8)
    notes = [None] * n
    notes[np.flatnonzero(st == 5)[0]] = 'Float'
    got = format_reasons(pd_.problem_id, st, res, q_ref, q_grid, rat, notes)
    want = [reason_for(pd_.problem_id, int(st[i]), res[i], float(q_ref[i]), float(q_grid[i]),
                       bool(rat[i]), notes[i])[1] for i in range(n)]
    bad = [(i, got[i], want[i]) for i in range(n) if got[i] != want[i]]
    assert not bad, bad[:5]


def _hostpool_compile_body():
    """pdeval.hostpool (the SymPy process pool for declined strings, forked before any GPU
    use) returns exactly what problem_defs.compile_strings returns in-process."""
    from pdeval import hostpool
    strs = [s for s in _stream('force_free_d4_validated.txt.gz')[:40000]]
    ops, off, st = native.compile_native(0, strs)
    declined = [s for s, x in zip(strs, st) if x != native.COMPILE_OK][:40]
    assert declined
    want = P.compile_strings(P.force_free(), declined)
    assert hostpool.start(2) is not None          # a fresh process: the GPU is not live
    try:
        got = hostpool.compile_strings(P.force_free(), declined)
    finally:
        hostpool.stop()
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]) and got[2] == want[2]


def _hostpool_host_steps_body():
    """The host steps' per-candidate SymPy checks over the pool (pdeval.hostpool.run): the
    symbolic zero-gradient test and the known-solution confirmation give what they give
    in-process."""
    from pdeval import hostpool
    from pdeval.batch import symbolic_zero_gradient
    from pdeval.worker import KnownSolutionTagger, _confirm
    from problems import load_problem
    pd_ = P.force_free()
    strs = ['exp(rho**2)*exp(z**2)*exp(neg(rho**2 + z**2))', 'neg(rho**2 + z**2)/(rho**2 + z**2)',
            'rho**2', 'sqrt(rho**2)*exp(z)*exp_neg(z)', '1 + neg(rho**2 + z**2)/(rho**2 + z**2)',
            'exp(z)*exp_neg(z)', 'rho*z/(rho*z)', 'square(exp(rho))*exp_neg(2*rho)', 'rho**2*z']
    n = len(strs)

    def fresh():
        return {'status': np.zeros(n, dtype=np.uint8), 'verdict': np.ones(n, dtype=bool),
                'fingerprint': np.ones((n, 4))}

    a = fresh()
    rows_in = symbolic_zero_gradient(pd_, strs, a)
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger.__new__(KnownSolutionTagger)
    tagger.slug, tagger.locals = 'force_free', locs
    tagger.known_str = ['rho**2', 'rho**2*z']
    tagger.known = [(__import__('sympy').sympify(k, locals=locs), k) for k in tagger.known_str]
    want = [[_confirm(s, ke, locs) for ke, _ in tagger.known] for s in strs]
    assert hostpool.start(2) is not None          # a fresh process: the GPU is not live
    try:
        b = fresh()
        rows_pool = symbolic_zero_gradient(pd_, strs, b)
        from pdeval.worker import _confirm_str
        got = hostpool.run(_confirm_str, [('force_free', s, k) for s in strs for k in tagger.known_str],
                           min_items=1)
    finally:
        hostpool.stop()
    assert rows_in == rows_pool and np.array_equal(a['status'], b['status'])
    assert sum(want, []) == got
    assert rows_in                              # the constant products are found


def _in_fresh_process(fn_name):
    """Run one of the pool bodies in a fresh interpreter: the pool forks only from a process
    whose GPU is not live, and earlier tests of this session may have created a context."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = (f"import sys; sys.path[:0] = [{here!r}, {os.path.join(os.path.dirname(here), 'pde-engine_amd')!r}]; "
            f"import test_native_compile as t; t.{fn_name}(); print('BODY-OK')")
    p = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0 and 'BODY-OK' in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])


def test_hostpool_compile_equals_in_process():
    """pdeval.hostpool (the SymPy process pool for declined strings, forked before any GPU
    use) returns exactly what problem_defs.compile_strings returns in-process."""
    _in_fresh_process('_hostpool_compile_body')


def test_hostpool_host_steps_equal_in_process():
    """The host steps' per-candidate SymPy checks over the pool (pdeval.hostpool.run) give
    what they give in-process."""
    _in_fresh_process('_hostpool_host_steps_body')


def _square(x):
    return x * x


def _slow_or_die(x):
    import time
    if x == 'die':
        os._exit(3)             # a child that dies (as an OOM kill would)
    if x == 'slow':
        time.sleep(30)
    return x


def _hostpool_faults_body():
    from pdeval import hostpool
    assert hostpool.start(2) is not None
    try:
        assert hostpool.run(_square, list(range(20))) == [i * i for i in range(20)]
        # a per-item bound: the slow item yields the default, the others their value
        got = hostpool.run(_slow_or_die, ['a', 'slow', 'b'] * 3, min_items=1, item_timeout=1.0, default='T')
        assert got == ['a', 'T', 'b'] * 3, got
        # a child dies: the pool is marked broken (never re-forked), the job completes in-process
        pids = [p.pid for p in hostpool._POOL.procs]
        hostpool._POOL.tasks.put((-1, 0, _slow_or_die, ['die'], None, None))
        import time
        t0 = time.time()
        while hostpool.active() and time.time() - t0 < 20:
            time.sleep(0.1)
        assert not hostpool.active()
        assert hostpool.run(_square, list(range(10)), min_items=1) == [i * i for i in range(10)]
        # (the collector thread terminates the surviving children after marking the pool
        # broken; under load that takes a moment)
        t0 = time.time()
        while any(p.is_alive() for p in hostpool._POOL.procs) and time.time() - t0 < 20:
            time.sleep(0.1)
        assert all(not p.is_alive() for p in hostpool._POOL.procs)
        assert pids
    finally:
        hostpool.stop()


def test_hostpool_fixed_children_timeout_and_death():
    """The pool's children are never replaced: a dead child marks the pool broken and the
    work runs in-process; a per-item time bound yields the default."""
    _in_fresh_process('_hostpool_faults_body')
