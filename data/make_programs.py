#!/usr/bin/env python3
"""Compile a candidate-string fixture into a program batch (data/<name>.npz).

Input: a tests/golden/streams/*.txt.gz file ("<depth>\t<expr>" or "<idx>\t<depth>\t<expr>").
Output: npz with ops (int32), offsets (int64), depth (int8) and the expression strings, so
the GPU box can load the benchmark workload without re-running SymPy.  --native compiles with
the product's path (pdeval.native.compile_strings: csrc/pdcompile.cpp, SymPy only for the
strings it declines) instead of SymPy for every string.
"""
import argparse
import gzip
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
from pdeval import problem_defs as P  # noqa: E402
from pdeval.flatten import pack  # noqa: E402

_PD = None


def _one(s):
    ops, off, notes = P.compile_strings(_PD, [s])
    return ops.tolist()


def main():
    global _PD
    ap = argparse.ArgumentParser()
    ap.add_argument('--problem', default='force_free')
    ap.add_argument('--input', required=True)
    ap.add_argument('--out', required=True)
    ap.add_argument('--procs', type=int, default=os.cpu_count())
    ap.add_argument('--native', action='store_true')
    a = ap.parse_args()
    _PD = P.get(a.problem)
    with gzip.open(a.input, 'rt') as f:
        rows = [l.rstrip('\n').split('\t') for l in f]
    exprs = [r[-1] for r in rows]
    depth = np.array([int(r[-2]) for r in rows], dtype=np.int8)
    if a.native:
        from pdeval import native
        st = {}
        ops, offsets, _ = native.compile_strings(_PD, exprs, stats=st)
        print(f"native {st['native']}, SymPy fallback {st['host']}")
        progs = exprs
    else:
        with mp.get_context('fork').Pool(a.procs) as pool:
            progs = pool.map(_one, exprs, chunksize=256)
        ops, offsets = pack(progs)
    np.savez_compressed(a.out, ops=ops, offsets=offsets, depth=depth,
                        exprs=np.array(exprs, dtype=object).astype(str))
    print(f'{len(progs)} programs, {ops.size} words -> {a.out}')


if __name__ == '__main__':
    main()
