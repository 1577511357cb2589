#!/usr/bin/env python3
"""Summarize the separate rocprofv3 --pmc passes of scripts/gpu_pmc.sh into profiles/<tag>_pmc.json.

HBM traffic per launch = FETCH_SIZE x 2 (gfx950: FETCH_SIZE reports half the bytes of wide
reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB as rocprofv3 derives them.  Also
records the SQ instruction mix used in DESIGN.md.  Usage:
    python scripts/pmc_summary.py gpurun_out/pmc profiles/r01_pmc.json
"""
import collections
import csv
import glob
import json
import os
import sys


def load(pass_dir):
    files = glob.glob(os.path.join(pass_dir, '**', '*counter_collection.csv'), recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            if 'pd::' not in k:
                continue
            k = k.split('(pd::')[0].replace('void pd::', '')
            agg[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add(r.get('Dispatch_Id', '0'))
    return agg, disp


def pass1_candidates(src):
    """The candidates pass 1 actually evaluated in the profiled bench run (its JSON line's
    roofline.kernel_candidates), per dominant kernel: the divisor of the per-candidate counter
    values -- SQ_WAVES counts every launched wave, and the candidates pass 1 does not take
    (deeper stacks, complex at p*) leave after a few instructions."""
    got = {}
    for f in glob.glob(os.path.join(src, '*.log')):
        for line in open(f, errors='replace'):
            if not line.startswith('{'):
                continue
            try:
                r = json.loads(line)
            except ValueError:
                continue
            roof = r.get('roofline') or {}
            if roof.get('kernel') and roof.get('kernel_candidates'):
                got[roof['kernel']] = roof['kernel_candidates']
    return got


def main():
    src, out = sys.argv[1], sys.argv[2]
    p1 = pass1_candidates(src)
    kern = collections.defaultdict(dict)
    for p in sorted(os.listdir(src)):
        d = os.path.join(src, p)
        if not os.path.isdir(d):
            continue
        agg, disp = load(d)
        for k, v in agg.items():
            nd = max(1, len(disp[k]))
            for c, x in v.items():
                kern[k][c] = x / nd          # per launch
            kern[k]['dispatches_' + p] = nd
    res = {}
    for k, v in kern.items():
        r = dict(v)
        r['candidates'] = v.get('SQ_WAVES')           # every launched wave (one per candidate)
        if k in p1:
            r['pass1_candidates'] = p1[k]              # the ones pass 1 evaluated
        if 'FETCH_SIZE' in v and 'WRITE_SIZE' in v:
            r['hbm_bytes_per_launch'] = 2 * v['FETCH_SIZE'] * 1024 + v['WRITE_SIZE'] * 1024
        res[k] = r
    with open(out, 'w') as f:
        json.dump({'source': src, 'note': 'per-launch values; FETCH_SIZE/WRITE_SIZE in KiB; '
                   'hbm_bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)',
                   'kernels': res}, f, indent=1)
    for k, v in res.items():
        print(k, {c: f'{x:.4g}' for c, x in v.items() if isinstance(x, float)})


if __name__ == '__main__':
    main()
