#!/usr/bin/env python3
"""Native compiler vs SymPy over a committed candidate stream (development check; the CPU test
suite runs the same comparison on a sample, tests/test_native_compile.py).

For every string: canonical form of pdcompile.cpp's tree vs sympify's tree, and program words
vs flatten.py's.  Prints counts and the first mismatches.
    python scripts/native_parity.py tests/golden/streams/force_free_d4_validated.txt.gz force_free
"""
import gzip
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))

from pdeval import native, problem_defs as P  # noqa: E402
from pdeval.flatten import Unsupported  # noqa: E402


def read_stream(path):
    op = gzip.open if path.endswith('.gz') else open
    out = []
    with op(path, 'rt') as f:
        for line in f:
            parts = line.rstrip('\n').split('\t')
            out.append(parts[-1])
    return out


def check(args):
    prob, strings = args
    pd_ = P.get(prob)
    res = []
    ops, off, st = native.compile_native(pd_.problem_id, strings)
    for i, s in enumerate(strings):
        if st[i] != 0:
            res.append(('declined' if st[i] == 1 else 'parse', s, None))
            continue
        _, cn = native.canonical(pd_.problem_id, s)
        try:
            e = pd_.parse(s)
            cs = native.sympy_canonical(e)
        except Exception as ex:  # noqa: BLE001
            res.append(('sympy_error', s, repr(ex)))
            continue
        if cn != cs:
            res.append(('canon_mismatch', s, (cn, cs)))
            continue
        try:
            w = pd_.compile(e)
        except Unsupported as ex:
            res.append(('sympy_unsupported', s, str(ex)))
            continue
        mine = list(ops[off[i]:off[i + 1]])
        if mine == list(w):
            res.append(('identical', s, None))
        elif mine[0] == w[0]:
            res.append(('same_header', s, None))
        elif (mine[0] & ~0xff00) == (w[0] & ~0xff00):
            res.append(('depth_only', s, (hex(mine[0]), hex(w[0]))))
        else:
            res.append(('header_mismatch', s, (hex(mine[0]), hex(w[0]))))
    return res


def main():
    path, prob = sys.argv[1], sys.argv[2]
    limit = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    strings = read_stream(path)
    if limit:
        strings = strings[:limit]
    chunks = [(prob, strings[i:i + 500]) for i in range(0, len(strings), 500)]
    t0 = time.time()
    with mp.Pool(8) as pool:
        results = [r for part in pool.map(check, chunks) for r in part]
    counts = {}
    for k, _, _ in results:
        counts[k] = counts.get(k, 0) + 1
    print(f'{len(strings)} strings in {time.time() - t0:.1f}s:', counts)
    shown = {}
    for k, s, d in results:
        if k in ('identical', 'same_header'):
            continue
        if shown.get(k, 0) < 12:
            shown[k] = shown.get(k, 0) + 1
            print(k, '|', s, '|', d)


if __name__ == '__main__':
    main()
