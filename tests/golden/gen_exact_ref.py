#!/usr/bin/env python3
"""Exact residuals at the reference points, for every reference fixture (our own SymPy
mathematics -- it does not import the reference; runs in the build container only).

The reference decides its point stage on the EXACT value of the residual at its test points:
  force-free  det[[L_T A, L_T B], [L_T^2 A, L_T^2 B]] at (rho, z) = (4/5, 6/7), rejected when it is
              a non-zero Number or |evalf(50)| >= 1e-20   (problems/force_free/validator.py:305-402)
  Kerr        d_r[G/(1-x^2) u_r] + d_x[G/Delta u_x] at M = 1, a = 1/10 and the three points
              (5/2, 3/5), (7/3, 1/3), (5, -2/5), N(., 40)   (kerr_magnetosphere/validator.py:77-91,
              :163-192)
This script restates those formulas with sp.diff, substitutes the exact rational points and
evaluates with evalf(50) (SymPy raises the working precision until 50 digits are correct, so
cancellation does not hurt).  Output, one JSON object per candidate:
  {"expr", "res": [[re, im], ...] (40-digit strings, one pair per reference point),
   "exact_number": bool (force-free: the value at p* is a Number after cancel(together())),
   "timeout": bool}
The GPU residual test (tests/test_gpu_parity.py) checks the device's res_ref against these to
1e-10 relative wherever |res| >= 1e-20.

    python tests/golden/gen_exact_ref.py --problem force_free --out tests/golden/exact/ff_ref_exact.jsonl \
        ff_d1.jsonl ff_d2.jsonl ...
"""
import argparse
import json
import multiprocessing as mp
import os
import signal
import sys

import sympy as sp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from pdeval import problem_defs as P  # noqa: E402

FF_POINT = (sp.Rational(4, 5), sp.Rational(6, 7))
KERR_POINTS = ((sp.Rational(5, 2), sp.Rational(3, 5)), (sp.Rational(7, 3), sp.Rational(1, 3)),
               (sp.Integer(5), sp.Rational(-2, 5)))


class _Timeout(BaseException):
    pass


def _alarm(*_):
    raise _Timeout()


def ff_det(u, rho, z):
    ur, uz = sp.diff(u, rho), sp.diff(u, z)
    A = sp.diff(ur, rho) + sp.diff(uz, z) - ur / rho
    B = ur**2 + uz**2
    LT = lambda f: uz * sp.diff(f, rho) - ur * sp.diff(f, z)   # noqa: E731
    LA, LB = LT(A), LT(B)
    return LA * LT(LB) - LB * LT(LA)


def kerr_lhs(u, r, x, M, a):
    Delta = r**2 - 2 * M * r + a**2
    G = 1 - (2 * M * r) / (r**2 + a**2 * x**2)
    return sp.diff(G / (1 - x**2) * sp.diff(u, r), r) + sp.diff(G / Delta * sp.diff(u, x), x)


def _num(v):
    c = sp.N(v, 50)
    re, im = c.as_real_imag()
    return [sp.sstr(sp.N(re, 40)), sp.sstr(sp.N(im, 40))]


def _one(args):
    prob, expr, timeout = args
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(timeout)
    pd_ = P.get(prob)
    rec = {'expr': expr, 'timeout': False}
    try:
        u = pd_.parse(expr)
        if pd_.problem_id == 0:
            d = ff_det(u, pd_.x, pd_.y).subs({pd_.x: FF_POINT[0], pd_.y: FF_POINT[1]})
            ds = sp.cancel(sp.together(d))
            rec['exact_number'] = bool(ds.is_Number)
            rec['res'] = [_num(ds)]
        else:
            M, a = pd_.constants['M'], pd_.constants['a']
            lhs = kerr_lhs(u, pd_.x, pd_.y, M, a).subs({M: 1, a: sp.Rational(1, 10)})
            rec['res'] = [_num(lhs.subs({pd_.x: px, pd_.y: py})) for px, py in KERR_POINTS]
    except _Timeout:
        rec['timeout'] = True
    except Exception as e:   # noqa: BLE001 -- zoo / nan at the point etc.
        rec['error'] = repr(e)[:200]
    finally:
        signal.alarm(0)
    return rec


def main():
    import golden_data as G
    ap = argparse.ArgumentParser()
    ap.add_argument('--problem', required=True)
    ap.add_argument('--out', required=True)
    ap.add_argument('--timeout', type=int, default=120)
    ap.add_argument('--procs', type=int, default=4)
    ap.add_argument('--exact', action='store_true', help='inputs are exact/*.jsonl files')
    ap.add_argument('files', nargs='+')
    a = ap.parse_args()
    exprs, seen = [], set()
    for f in a.files:
        rows = G.exact_rows(f) if a.exact else G.ref_rows(f)
        for r in rows:
            if r['expr'] not in seen:
                seen.add(r['expr'])
                exprs.append(r['expr'])
    done = set()
    if os.path.exists(a.out):
        with open(a.out) as f:
            done = {json.loads(line)['expr'] for line in f}
    todo = [e for e in exprs if e not in done]
    print(f'{len(exprs)} candidates, {len(todo)} to do', flush=True)
    with mp.Pool(a.procs, maxtasksperchild=50) as pool, open(a.out, 'a') as f:
        for k, rec in enumerate(pool.imap_unordered(_one, [(a.problem, e, a.timeout) for e in todo])):
            f.write(json.dumps(rec) + '\n')
            f.flush()
            if k % 100 == 0:
                print(f'{k}/{len(todo)}', flush=True)


if __name__ == '__main__':
    main()
