#!/usr/bin/env python3
"""The device call of one worker batch (pdeval_validate_batch from host buffers: upload, launch
chain, download, sync) by batch size, on the validated force-free d4 programs (GPU box).

Prints one JSON line per (batch size, context setting): the median wall time of ctx.validate
over repeated calls, the pass times of one call with the library's events, and the per-candidate
cost.  Usage: python scripts/profile_device_batch.py [--sizes 1024,4096,16384] [--reps 15]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes', default='512,1024,2048,4096,8192,16384')
    ap.add_argument('--reps', type=int, default=15)
    a = ap.parse_args()
    from pdeval import _lib
    from pdeval.workload import load_programs, gather_programs
    ops, off, _ = load_programs("force_free_d4_validated")
    rng = np.random.default_rng(0)
    perm = rng.permutation(len(off) - 1)
    for env in ({}, {'PDEVAL_DD_EARLY': '0'}):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            ctx = _lib.Context(0)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        for n in [int(s) for s in a.sizes.split(',')]:
            o, f = gather_programs(ops, off, perm[:n])
            ctx.validate(o, f)                      # warm (buffers sized)
            ts = []
            for r in range(a.reps):
                o, f = gather_programs(ops, off, perm[(r + 1) * n % (len(perm) - n):][:n])
                t0 = time.perf_counter()
                ctx.validate(o, f)
                ts.append(time.perf_counter() - t0)
            ctx.set_timing(True)
            ctx.validate(o, f)
            pt = ctx.pass_times()
            ctx.set_timing(False)
            med = float(np.median(ts))
            print(json.dumps({'env': env, 'n': n, 'wall_ms_median': round(1e3 * med, 3),
                              'wall_ms_min': round(1e3 * min(ts), 3), 'ns_per_cand': round(1e9 * med / n, 1),
                              'chain_ms': round(sum(pt.values()), 3),
                              'pass_ms': {k: round(v, 3) for k, v in pt.items() if v > 0.005}}), flush=True)
        ctx.close()


if __name__ == '__main__':
    main()
