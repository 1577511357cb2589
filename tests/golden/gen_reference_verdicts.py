#!/usr/bin/env python3
"""Fixture generator (runs ONLY in the build container, never on the GPU box).

Imports the reference from a scratch copy (see ``gen_streams.py``) and records, as data:

* ``filters``  -- the driver's pre-validate filters of the inline path
  (``general_method_paper_reproduction.py:1253-1294``): degenerate denominators
  (``_has_degenerate_denominator`` ``:134-199``, applied to the locals-parse and the plain
  parse), the ``UNIQUE(str(simplify(expand(sympify(s)))))`` dedupe (``:1277-1286``, sequential
  in stream order) and the constant-only skip (``:1292-1294``).  Output: the candidates that
  reach ``validate``:  streams/<slug>_d<D>_validated.txt.gz  ("<stream idx>\t<depth>\t<expr>").
* ``verdicts`` -- the reference's ``validator.validate`` verdict ``(ok, reason)`` for a list of
  candidates, called exactly as the inline path calls it (``:1299-1316``, incl. the TypeError
  fallback), with FRESH per-process caches (in-memory SQLite for the verdict cache
  ``problems/force_free/validator.py:182-222`` and for the normalizer memo
  ``lean_normalizer/lean_bridge_fixed.py:29-68``) and a per-candidate wall-clock timeout
  (SIGALRM raising a ``BaseException`` so that ``validate``'s blanket ``except Exception``
  cannot swallow it).  Output: JSONL, one object per candidate.
"""
import argparse
import gzip
import queue as _queue
import json
import multiprocessing as mp
import os
import random
import signal
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_streams import make_scratch_copy  # noqa: E402

_D = None      # GeneralFoliationDiscovery (reference) per worker
_TIMEOUT = 60
_FILTER_TIMEOUT = 120


class _Timeout(BaseException):
    pass


def _alarm(_sig, _frm):
    raise _Timeout()


def _init_worker(ref, problem, kerr_a_value='1/10', kerr_op_a_zero=False, ff_omega='0'):
    global _D
    os.chdir(ref)
    sys.path.insert(0, ref)
    import sympy as sp
    from general_method_paper_reproduction import GeneralFoliationDiscovery
    from lean_normalizer.lean_bridge_fixed import LeanNormalizer
    d = GeneralFoliationDiscovery(use_lean_normalizer=True, problem_name=problem, mode='parallel')
    if d.problem.slug == 'force_free':
        from problems.force_free.validator import PreciseFoliationValidator
        # (a fixture run may pass a non-zero Omega, validator.py:38-49: the rotating constraint)
        v = PreciseFoliationValidator(cache_db=':memory:', use_lean=False, Omega=sp.sympify(ff_omega))
        v.use_lean = True
        v.lean_normalizer = LeanNormalizer(cache_db=':memory:')
    else:
        from problems.kerr_magnetosphere.validator import KerrMagnetosphereValidator
        s, c = d.problem.symbols, d.problem.constants
        # the problem's validator (problems/__init__.py:283): M_value = 1, a_value = 1/10; a
        # fixture run may pass another a_value (kerr validator.py:36-37), or build the operator
        # with the number 0 for a (the Schwarzschild operator; u's a is then a free symbol)
        a_op = sp.Integer(0) if kerr_op_a_zero else c['a']
        v = KerrMagnetosphereValidator(s['r'], s['x'], c['M'], a_op,
                                       M_value=sp.Integer(1), a_value=sp.Rational(kerr_a_value),
                                       use_lean=False)
        v.use_lean = True
        v._lean = LeanNormalizer(cache_db=':memory:')
    d.validator = v
    _D = d
    signal.signal(signal.SIGALRM, _alarm)


def _filter_one(item):
    """Per-candidate part of the pre-validate filters (pure); dedupe happens in the parent."""
    import sympy as sp
    idx, depth, s = item
    d = _D
    out = {'idx': idx, 'depth': depth, 'expr': s, 'degenerate': False, 'normalized': s,
           'const_only': False}
    try:
        try:
            u = sp.sympify(s, locals=d._sympify_locals)
        except Exception:
            u = None
        try:
            if u is not None and d._has_degenerate_denominator(u):
                out['degenerate'] = True
                return out
        except Exception:
            pass
        try:
            sym = sp.sympify(s)
        except Exception:
            sym = None
        if sym is not None and d._has_degenerate_denominator(sym):
            out['degenerate'] = True
            return out
        # the reference has no limit here; a fixture run bounds the dedupe key's simplify so
        # one pathological candidate cannot stall the pool (such a row keeps its own string
        # as key and is counted as 'simplify_timeout')
        signal.alarm(_FILTER_TIMEOUT)
        try:
            out['normalized'] = str(sp.simplify(sp.expand(sym if sym is not None else sp.sympify(s))))
        except _Timeout:
            out['normalized'] = s
            out['simplify_timeout'] = True
        except Exception:
            out['normalized'] = s
        finally:
            signal.alarm(0)
        syms = d.problem.symbols
        uc = u if u is not None else sp.sympify(s, locals=d._sympify_locals)
        if not (uc.has(syms.get('rho', sp.Symbol('rho'))) or uc.has(syms.get('z', sp.Symbol('z')))
                or uc.has(syms.get('r', sp.Symbol('r'))) or uc.has(syms.get('x', sp.Symbol('x')))):
            out['const_only'] = True
    except Exception as e:  # noqa: BLE001
        out['error'] = repr(e)
    return out


_EVIDENCE = False


def _verdict_one(item):
    import sympy as sp
    idx, depth, s = item
    d = _D
    rec = {'idx': idx, 'depth': depth, 'expr': s}
    t0 = time.time()
    signal.alarm(_TIMEOUT)
    try:
        if _EVIDENCE:
            d.validator._last_evidence = {}     # a fresh validator's state (kerr validator.py:380-381)
        u = sp.sympify(s, locals=d._sympify_locals)
        try:
            ok, reason = d.validator.validate(u, check_regularity=False, fast_point_only=False,
                                              lean_first=True, defer_heavy_checks=True,
                                              enforce_anchor=False)
        except TypeError:
            ok, reason = d.validator.validate(u, check_regularity=False, fast_point_only=False)
        rec.update(ok=bool(ok), reason=reason, timeout=False)
        if _EVIDENCE:
            rec['evidence'] = d.validator.last_evidence() if hasattr(d.validator, 'last_evidence') else None
    except _Timeout:
        rec.update(ok=None, reason=None, timeout=True)
    except Exception as e:  # noqa: BLE001  (the caller records status='error')
        rec.update(ok=None, reason=f'Validator Error: {e}', timeout=False)
    finally:
        signal.alarm(0)
    rec['t'] = round(time.time() - t0, 4)
    return rec


def _hard_worker(init, tasks, results):
    """A verdict worker of run_hard: announces each item before it starts it."""
    _init_worker(*init)
    while True:
        item = tasks.get()
        if item is None:
            return
        results.put(('start', os.getpid(), item, time.time()))
        results.put(('done', os.getpid(), _verdict_one(item), 0.0))


def run_hard(items, procs, init, hard_s, emit):
    """The verdicts of ``items`` on ``procs`` forked workers, each item under a HARD deadline:
    SIGALRM cannot interrupt SymPy inside a C-level call (one depth-5 row ran for an hour past its
    20 s alarm), so the parent kills a worker whose item passed ``hard_s`` seconds, records the
    item as undecided (timeout, ``hard_kill``) and starts a new worker for the rest.  ``emit``
    receives every record as it completes."""
    ctx = mp.get_context('fork')
    tasks, results = ctx.Queue(), ctx.Queue()
    for it in items:
        tasks.put(it)
    workers = {}

    def spawn():
        w = ctx.Process(target=_hard_worker, args=(init, tasks, results), daemon=True)
        w.start()
        workers[w.pid] = [w, None, 0.0]

    for _ in range(procs):
        spawn()
    left = len(items)
    while left:
        try:
            kind, pid, obj, t0 = results.get(timeout=2.0)
            if kind == 'start':
                workers[pid][1], workers[pid][2] = obj, t0
            else:
                workers[pid][1] = None
                emit(obj)
                left -= 1
        except _queue.Empty:
            pass
        now = time.time()
        for pid, (w, it, t0) in list(workers.items()):
            if it is not None and now - t0 > hard_s:
                w.kill()
                w.join(5)
                del workers[pid]
                emit({'idx': it[0], 'depth': it[1], 'expr': it[2], 'ok': None, 'reason': None, 'timeout': True,
                      't': round(now - t0, 1), 'hard_kill': True})
                left -= 1
                spawn()
            elif not w.is_alive() and it is not None:   # died on its own (OOM, crash)
                del workers[pid]
                emit({'idx': it[0], 'depth': it[1], 'expr': it[2], 'ok': None, 'reason': 'worker died',
                      'timeout': False, 't': round(now - t0, 1)})
                left -= 1
                spawn()
    for _ in workers:
        tasks.put(None)
    for w, _, _ in workers.values():
        w.join(10)
        if w.is_alive():
            w.kill()


def read_stream(path):
    with gzip.open(path, 'rt') as f:
        return [(i, int(l.split('\t', 1)[0]), l.rstrip('\n').split('\t', 1)[1]) for i, l in enumerate(f)]


def main():
    global _TIMEOUT, _EVIDENCE
    ap = argparse.ArgumentParser()
    ap.add_argument('mode', choices=['filters', 'verdicts'])
    ap.add_argument('--ref', default='/tmp/refcopy')
    ap.add_argument('--problem', default='force_free')
    ap.add_argument('--input', required=True, help='stream .txt.gz or validated .txt.gz or .txt list')
    ap.add_argument('--out', required=True)
    ap.add_argument('--depth', type=int, default=None, help='only candidates of this depth')
    ap.add_argument('--sample', type=int, default=0, help='seeded sample size (0 = all)')
    ap.add_argument('--start', type=int, default=0, help='skip the first START input rows')
    ap.add_argument('--stop', type=int, default=0, help='input rows before STOP only (0 = all)')
    ap.add_argument('--evidence', action='store_true', help="also record the validator's last_evidence()")
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--timeout', type=int, default=60)
    ap.add_argument('--procs', type=int, default=os.cpu_count())
    ap.add_argument('--hard', type=int, default=0,
                    help='per-item hard deadline in seconds (the parent kills a stuck worker); 0 = off')
    ap.add_argument('--kerr-a-value', default='1/10', help="Kerr validator's a_value")
    ap.add_argument('--ff-omega', default='0', help="force-free validator's Omega (a constant)")
    ap.add_argument('--kerr-op-a-zero', action='store_true',
                    help='Kerr operator built with a = 0 (validator a argument = the number 0)')
    a = ap.parse_args()
    _TIMEOUT = a.timeout
    _EVIDENCE = a.evidence
    make_scratch_copy('/root/reference', a.ref)
    t0 = time.time()
    if a.mode == 'filters':
        items = read_stream(a.input)
        with mp.get_context('fork').Pool(a.procs, _init_worker, (a.ref, a.problem)) as pool:
            res = []
            for r in pool.imap(_filter_one, items, chunksize=16):
                res.append(r)
                if len(res) % 10000 == 0:
                    print(f'[filters] {len(res)}/{len(items)} {time.time()-t0:.0f}s', flush=True)
        seen, kept, stats = set(), [], {'degenerate': 0, 'duplicate': 0, 'const_only': 0,
                                        'simplify_timeout': 0}
        for r in res:                       # sequential, stream order (UNIQUE(normalized))
            stats['simplify_timeout'] += int(bool(r.get('simplify_timeout')))
            if r['degenerate']:
                stats['degenerate'] += 1
                continue
            if r['normalized'] in seen:
                stats['duplicate'] += 1
                continue
            seen.add(r['normalized'])
            if r['const_only']:
                stats['const_only'] += 1
                continue
            kept.append(r)
        with gzip.open(a.out, 'wt') as f:
            for r in kept:
                f.write(f"{r['idx']}\t{r['depth']}\t{r['expr']}\n")
        print(json.dumps({'streamed': len(items), 'validated': len(kept), **stats,
                          'wall_s': round(time.time() - t0, 1)}))
        return
    if a.input.endswith('.gz'):
        with gzip.open(a.input, 'rt') as f:
            rows = [l.rstrip('\n').split('\t') for l in f]
        items = [(int(r[0]), int(r[1]), r[2]) for r in rows] if len(rows[0]) == 3 else \
                [(i, int(r[0]), r[1]) for i, r in enumerate(rows)]
    else:
        with open(a.input) as f:
            items = [(i, 0, l.strip()) for i, l in enumerate(f) if l.strip()]
    items = items[a.start:a.stop] if a.stop else items[a.start:]
    if a.depth is not None:
        items = [it for it in items if it[1] == a.depth]
    if a.sample and a.sample < len(items):
        items = sorted(random.Random(a.seed).sample(items, a.sample))
    init = (a.ref, a.problem, a.kerr_a_value, a.kerr_op_a_zero, a.ff_omega)
    if a.hard:
        with open(a.out, 'w') as f:
            cnt = [0]

            def emit(rec):
                rec['problem'] = a.problem
                if a.timeout != 60:
                    rec['limit_s'] = a.timeout
                f.write(json.dumps(rec) + '\n')
                f.flush()
                cnt[0] += 1
                if cnt[0] % 50 == 0:
                    print(f'[verdicts] {cnt[0]}/{len(items)} {time.time()-t0:.0f}s', flush=True)
            run_hard(items, a.procs, init, a.hard, emit)
        print(f'wrote {len(items)} verdicts to {a.out} in {time.time()-t0:.0f}s')
        return
    with mp.get_context('fork').Pool(a.procs, _init_worker, init,
                                     maxtasksperchild=200) as pool, open(a.out, 'w') as f:
        n = 0
        for rec in pool.imap_unordered(_verdict_one, items, chunksize=1):
            rec['problem'] = a.problem
            if a.timeout != 60:
                rec['limit_s'] = a.timeout
            if a.problem != 'force_free' and (a.kerr_a_value != '1/10' or a.kerr_op_a_zero):
                rec['kerr'] = {'M_value': '1', 'a_value': a.kerr_a_value, 'op_a_zero': a.kerr_op_a_zero}
            if a.problem == 'force_free' and a.ff_omega != '0':
                rec['omega'] = a.ff_omega
            f.write(json.dumps(rec) + '\n')
            f.flush()
            n += 1
            if n % 50 == 0:
                print(f'[verdicts] {n}/{len(items)} {time.time()-t0:.0f}s', flush=True)
    print(f'wrote {len(items)} verdicts to {a.out} in {time.time()-t0:.0f}s')


if __name__ == '__main__':
    main()
