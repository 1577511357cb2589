#!/usr/bin/env python3
"""Exact-arithmetic ground truth for the zero test (our own SymPy mathematics -- it does not
import the reference).

For candidates of the depth-4 validated force-free batch (data/force_free_d4_validated.npz)
it evaluates the foliation determinant det[[L_T A, L_T B], [L_T^2 A, L_T^2 B]]
(problems/force_free/validator.py:323-347) EXACTLY at rational points and records |det| (30
digits).  A candidate whose det vanishes exactly at every point is a true solution (the
reference, in exact arithmetic, accepts it when it finishes); a non-zero value anywhere makes
it a true non-solution.  Used to pin tier 2 of the zero test, where fp64 noise
alone cannot decide.

    python tests/golden/gen_exact_det.py --idx-file IDX.npy --out tests/golden/exact/X.jsonl
"""
import argparse
import json
import multiprocessing as mp
import os
import signal
import sys

import numpy as np
import sympy as sp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
from pdeval import problem_defs as P  # noqa: E402

POINTS = ((4, 5, 6, 7), (13, 10, -5, 9), (2, 3, 7, 4))


class _Timeout(BaseException):
    pass


def _alarm(*_):
    raise _Timeout()


def exact_det(u, rho, z, pt):
    ur, uz = sp.diff(u, rho), sp.diff(u, z)
    A = sp.diff(ur, rho) + sp.diff(uz, z) - ur / rho
    B = ur**2 + uz**2
    LT = lambda f: uz * sp.diff(f, rho) - ur * sp.diff(f, z)   # noqa: E731
    LA, LB = LT(A), LT(B)
    return (LA * LT(LB) - LB * LT(LA)).subs(pt)


def _one(args):
    i, expr, timeout = args
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(timeout)
    pd_ = P.force_free()
    try:
        u = pd_.parse(expr)
        vals = []
        for a, b, c, d in POINTS:
            v = exact_det(u, pd_.x, pd_.y, {pd_.x: sp.Rational(a, b), pd_.y: sp.Rational(c, d)})
            vals.append(abs(complex(sp.N(v, 30))))
        signal.alarm(0)
        return {'idx': int(i), 'expr': expr, 'points': [list(p) for p in POINTS], 'det_abs': vals,
                'det_zero': all(v < 1e-25 for v in vals)}
    except _Timeout:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--idx-file', required=True)
    ap.add_argument('--out', required=True)
    ap.add_argument('--timeout', type=int, default=60)
    ap.add_argument('--procs', type=int, default=os.cpu_count())
    a = ap.parse_args()
    z = np.load(os.path.join(ROOT, 'data', 'force_free_d4_validated.npz'))
    idx = np.load(a.idx_file)
    with mp.Pool(a.procs) as pool:
        rows = pool.map(_one, [(int(i), str(z['exprs'][i]), a.timeout) for i in idx], chunksize=4)
    with open(a.out, 'w') as f:
        for r in rows:
            if r is not None:
                f.write(json.dumps(r) + '\n')


if __name__ == '__main__':
    main()
