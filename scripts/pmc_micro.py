#!/usr/bin/env python3
"""Per-program PMC table for scripts/gpu_pmc_micro.sh: counters of the pass-1 kernel launch of
each microbenchmark program, per wave (= per candidate).
Usage: pmc_micro.py gpurun_out/pmcm [force_free|kerr_magnetosphere] [default|calib] [out.json]"""
import json
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
from microbench import programs  # noqa: E402

KERNEL = 'grid_kernel<0, false'


def load(d):
    rows = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r['Kernel_Name']:
                continue
            rows[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
    return [rows[k] for k in sorted(rows)]


def main():
    global KERNEL
    src = sys.argv[1]
    problem = sys.argv[2] if len(sys.argv) > 2 else 'force_free'
    which = sys.argv[3] if len(sys.argv) > 3 else 'default'
    pid = 0 if problem == 'force_free' else 1
    KERNEL = f'grid_kernel<{pid}, false'
    PROGS = programs(pid, which)
    passes = [load(os.path.join(src, p)) for p in sorted(os.listdir(src)) if os.path.isdir(os.path.join(src, p))]
    per = [dict() for _ in PROGS]
    for p in passes:
        for i, c in enumerate(p[:len(PROGS)]):
            per[i].update(c)
    if len(sys.argv) > 4:
        with open(sys.argv[4], 'w') as f:
            json.dump({'problem': problem, 'set': which, 'kernel': KERNEL,
                       'per_wave': {s: {k: v / (c.get('SQ_WAVES', 1.0) or 1.0) for k, v in c.items()}
                                    for s, c in zip(PROGS, per)}}, f, indent=1)
    keys = sorted({k for c in per for k in c} - {'SQ_WAVES'})
    print('program'.ljust(34), ' '.join(k.replace('SQ_', '')[:14].rjust(14) for k in keys))
    for s, c in zip(PROGS, per):
        w = c.get('SQ_WAVES', 1.0) or 1.0
        print(s.ljust(34), ' '.join(f'{c.get(k, 0) / w:14.1f}' for k in keys))


if __name__ == '__main__':
    main()
