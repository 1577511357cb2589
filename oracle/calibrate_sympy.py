#!/usr/bin/env python3
"""Calibrate the SymPy CPU baseline (BENCH INFRASTRUCTURE, build container only; never on the
GPU box, where /root/reference does not exist).

bench.py's cpu_baseline times oracle/sympy_validator.py -- this build's SymPy restatement of
the reference's PreciseFoliationValidator.validate -- because the reference cannot travel to
the GPU box.  SURVEY.md §8d asks for that restatement's per-candidate time to be calibrated
against the reference's own validate on the same candidates in this container.  This script
runs both, one candidate per task on a process pool with the same per-candidate timeout, on a
seed-0 sample of the depth-4 candidates that reach validate, and writes the per-candidate
times and their ratio to profiles/r03_sympy_calibration.json (bench.py reports the ratio).

The reference is imported from a scratch copy (tests/golden/gen_streams.make_scratch_copy),
with fresh in-memory caches, and called as the inline path calls it
(general_method_paper_reproduction.py:1299-1316).
"""
import gzip
import json
import multiprocessing as mp
import os
import random
import signal
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
_V = None
_MODE = None
_LOCS = None


class _Timeout(BaseException):
    pass


def _alarm(*_):
    raise _Timeout()


def _init(mode, ref):
    global _V, _MODE, _LOCS
    _MODE = mode
    signal.signal(signal.SIGALRM, _alarm)
    if mode == 'reference':
        os.chdir(ref)
        sys.path.insert(0, ref)
        from problems.force_free.validator import PreciseFoliationValidator
        from lean_normalizer.lean_bridge_fixed import LeanNormalizer
        v = PreciseFoliationValidator(cache_db=':memory:', use_lean=False)
        v.use_lean = True
        v.lean_normalizer = LeanNormalizer(cache_db=':memory:')
        _V = v
        import sympy as sp
        from expression_operations import UNARY_OPS
        # the driver's sympify locals for force_free (problems/__init__.py:70-71, :84-93)
        _LOCS = {'rho': sp.Symbol('rho', real=True, positive=True), 'z': sp.Symbol('z', real=True),
                 **UNARY_OPS}
    else:
        sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
        sys.path.insert(0, HERE)


def _one(args):
    expr, timeout = args
    import sympy as sp
    t0 = time.perf_counter()
    signal.alarm(timeout)
    try:
        if _MODE == 'reference':
            u = sp.sympify(expr, locals=_LOCS)
            ok, reason = _V.validate(u, check_regularity=False, fast_point_only=False)
        else:
            from pdeval import problem_defs as P
            import sympy_validator as SV
            pd_ = P.force_free()
            ok, reason = SV.ff_validate(pd_.parse(expr), pd_.x, pd_.y)
        out = ('done', bool(ok), reason)
    except _Timeout:
        out = ('timeout', None, None)
    except Exception as e:   # noqa: BLE001
        out = ('error', None, str(e)[:80])
    finally:
        signal.alarm(0)
    return (expr,) + out + (time.perf_counter() - t0,)


def run(mode, exprs, ref, procs, timeout):
    with mp.get_context('fork').Pool(procs, _init, (mode, ref), maxtasksperchild=50) as pool:
        return {r[0]: r[1:] for r in pool.imap_unordered(_one, [(e, timeout) for e in exprs])}


def main():
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    from gen_streams import make_scratch_copy
    ref = make_scratch_copy('/root/reference', '/tmp/refcopy')
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    procs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    timeout = 60
    with gzip.open(os.path.join(ROOT, 'tests', 'golden', 'streams', 'force_free_d4_validated.txt.gz'), 'rt') as f:
        d4 = [l.rstrip('\n').split('\t')[-1] for l in f]
    sample = random.Random(0).sample(d4, n)
    res = {}
    for mode in ('reference', 'restatement'):
        t0 = time.perf_counter()
        res[mode] = run(mode, sample, ref, procs, timeout)
        res[mode + '_wall_s'] = time.perf_counter() - t0
    both = [e for e in sample if res['reference'][e][0] == 'done' and res['restatement'][e][0] == 'done']
    agree = sum(res['reference'][e][1] == res['restatement'][e][1] for e in both)
    tr = sorted(res['reference'][e][3] for e in both)
    ts = sorted(res['restatement'][e][3] for e in both)
    summary = {
        'sample': f'seed-0 sample of {n} depth-4 candidates that reach validate '
                  f'(tests/golden/streams/force_free_d4_validated.txt.gz), {timeout} s per-candidate timeout, '
                  f'Pool({procs}) per side, this container',
        'completed_both': len(both), 'verdicts_agree': agree,
        'timeouts': {m: sum(1 for e in sample if res[m][e][0] == 'timeout') for m in ('reference', 'restatement')},
        'wall_s': {m: round(res[m + '_wall_s'], 1) for m in ('reference', 'restatement')},
        'reference_total_s': round(sum(tr), 2), 'restatement_total_s': round(sum(ts), 2),
        'median_s': {'reference': tr[len(tr) // 2], 'restatement': ts[len(ts) // 2]} if both else None,
        'restatement_vs_reference_time_ratio': round(sum(ts) / sum(tr), 3) if both else None,
        'per_candidate': {e: {'reference': list(res['reference'][e]), 'restatement': list(res['restatement'][e])}
                          for e in sample},
    }
    out = os.path.join(ROOT, 'profiles', 'r03_sympy_calibration.json')
    with open(out, 'w') as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != 'per_candidate'}))


if __name__ == '__main__':
    main()
