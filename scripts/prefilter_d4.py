#!/usr/bin/env python3
"""The driver's pre-validate filters (pdeval/prefilter.py) over the WHOLE
force-free depth-4 stream of the reference's enumerator (tests/golden/streams/force_free_d4.txt.gz,
147,247 rows), on the forked SymPy pool, pinned against the set the reference's own filters kept
(tests/golden/streams/force_free_d4_validated.txt.gz, 142,004 rows; gen_reference_verdicts.py
filters, 120 s simplify bound).  Writes profiles/<tag>_prefilter_d4.json: wall time, pool size,
counts, and whether the kept rows equal the reference's (plus the differing rows, if any).

    python scripts/prefilter_d4.py --procs 7 --tag r05
"""
import argparse
import gzip
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=7)
    ap.add_argument('--tag', default='r05')
    ap.add_argument('--limit', type=int, default=0, help='first N stream rows only (0: all)')
    ap.add_argument('--item-timeout', type=float, default=120.0)
    a = ap.parse_args()
    from pdeval import hostpool, prefilter as F
    streams = os.path.join(ROOT, 'tests', 'golden', 'streams')
    with gzip.open(os.path.join(streams, 'force_free_d4.txt.gz'), 'rt') as f:
        rows = [l.rstrip('\n').split('\t') for l in f]
    if a.limit:
        rows = rows[:a.limit]
    with gzip.open(os.path.join(streams, 'force_free_d4_validated.txt.gz'), 'rt') as f:
        ref = [int(l.split('\t')[0]) for l in f]
    ref = [i for i in ref if i < len(rows)]
    hostpool.start(a.procs)
    t0 = time.time()
    res = F.filter_stream('force_free', [r[-1] for r in rows], item_timeout=a.item_timeout)
    wall = time.time() - t0
    hostpool.stop()
    kept = res.kept
    sk, sr = set(kept), set(ref)
    rec = {'stream': 'force_free_d4.txt.gz', 'rows': len(rows), 'procs': a.procs,
           'item_timeout_s': a.item_timeout, 'wall_s': round(wall, 1),
           'rows_per_s': round(len(rows) / wall, 1), 'stats': res.stats,
           'kept_equals_reference': kept == ref, 'kept': len(kept), 'reference_kept': len(ref),
           'only_here': sorted(sk - sr)[:50], 'only_reference': sorted(sr - sk)[:50],
           'kept_sha256': hashlib.sha256(','.join(map(str, kept)).encode()).hexdigest()}
    out = os.path.join(ROOT, 'profiles', f'{a.tag}_prefilter_d4.json')
    with open(out, 'w') as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k not in ('only_here', 'only_reference')}))


if __name__ == '__main__':
    main()
