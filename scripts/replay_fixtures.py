#!/usr/bin/env python3
"""Run the product's symbolic-stage replay (pde-engine_amd/pdeval/symbolic.py) on every decided
force-free reference fixture row that passed the reference's point stage (its verdict or text
came from the symbolic stage, problems/force_free/validator.py:404-427), and record what the
replay says -- ``tests/golden/replay/ff_replay.jsonl``: {expr, ok, reason, t, timeout}.

This is the product's own code run ahead of time on the fixtures (no reference import): the
CPU tests compare these outputs with the reference's verdicts on every row and re-run a seeded
subset live (tests/test_symbolic_replay.py), so the file stays pinned to the code.
"""
import argparse
import glob
import json
import multiprocessing as mp
import os
import signal
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
REF = os.path.join(ROOT, 'tests', 'golden', 'ref')
OUT = os.path.join(ROOT, 'tests', 'golden', 'replay', 'ff_replay.jsonl')


class _TO(BaseException):
    pass


def _alarm(*_):
    raise _TO()


def symbolic_rows():
    """Decided force-free rows whose reason comes from the symbolic stage, one per expr."""
    seen, rows = set(), []
    for f in sorted(glob.glob(os.path.join(REF, 'ff_*.jsonl'))):
        for line in open(f):
            r = json.loads(line)
            if r.get('timeout') or r.get('ok') is None or not r.get('reason'):
                continue
            if r.get('omega', '0') != '0':      # rotating-field fixtures: tested with their Omega
                continue
            rs = r['reason']
            if not (r['ok'] or 'Lean could not' in rs or 'expanded det' in rs or 'simplify det' in rs):
                continue
            if r['expr'] in seen:
                continue
            seen.add(r['expr'])
            rows.append(r['expr'])
    return rows


def one(args):
    expr, limit = args
    from pdeval import symbolic as S
    signal.signal(signal.SIGALRM, _alarm)
    t0 = time.time()
    signal.alarm(limit)
    try:
        r = S.replay_str(('force_free', expr, True))
        out = {'expr': expr, 'ok': None if r is None else r[0], 'reason': None if r is None else r[1],
               'timeout': False}
    except _TO:
        out = {'expr': expr, 'ok': None, 'reason': None, 'timeout': True}
    finally:
        signal.alarm(0)
    out['t'] = round(time.time() - t0, 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=4)
    ap.add_argument('--limit', type=int, default=60)
    a = ap.parse_args()
    exprs = symbolic_rows()
    done = {}
    if os.path.exists(OUT):
        for line in open(OUT):
            r = json.loads(line)
            done[r['expr']] = r
    todo = [e for e in exprs if e not in done]
    print(f'{len(exprs)} symbolic-stage rows, {len(todo)} to replay', flush=True)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with mp.get_context('fork').Pool(a.procs, maxtasksperchild=50) as pool, open(OUT, 'a') as f:
        for k, r in enumerate(pool.imap_unordered(one, [(e, a.limit) for e in todo], chunksize=1)):
            f.write(json.dumps(r) + '\n')
            f.flush()
            if k % 50 == 0:
                print(f'[replay] {k}/{len(todo)}', flush=True)
    print('done')


if __name__ == '__main__':
    main()
