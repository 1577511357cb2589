#!/usr/bin/env python3
"""GPU debugging aid: device vs oracle, per candidate, for a handful of programs (status,
q_ref, res_ref, n_bad) plus the work-list sizes.  Usage: python scripts/debug_point.py [N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'pde-engine_amd'), os.path.join(ROOT, 'tests')]
import golden_data as G  # noqa: E402
import oracle_lib as O  # noqa: E402
from pdeval import problem_defs as P  # noqa: E402
from pdeval._lib import Context, default_params  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    pd_ = P.force_free()
    z = np.load(os.path.join(ROOT, 'data', 'force_free_d4_validated.npz'))
    hdr = z['ops'][z['offsets'][:-1]]
    deep = np.flatnonzero(((hdr >> 8) & 0xff) == 3)[:4]
    exprs = ['exp(rho/(-rho/z + 1))', 'exp(z/(-rho**2 + z**2))', 'rho*z', 'rho**2']
    exprs += [str(z['exprs'][i]) for i in deep]
    exprs += [r['expr'] for r in G.exact_rows()[:n]]
    ops, off, _ = P.compile_strings(pd_, exprs)
    ctx = Context(0)
    for full in (1, 0):
        prm = default_params(0)
        prm.full_grid = full
        dev = ctx.validate(ops, off, prm)
        print('full_grid', full, 'counts', ctx.pass_counts())
        ps = ctx.point_states(len(exprs))
        ora = O.validate(0, ops, off, O.params(full_grid=full))
        for i, s in enumerate(exprs):
            d, o = int(dev['status'][i]), int(ora['status'][i])
            flag = '' if d == o else '   <-- MISMATCH'
            if i < 8 + 8 or flag:
                print(f'{s[:50]:50s} dev {d} q {dev["q_ref"][i]:.3e} r {dev["res_ref"][i, 0]:+.9e} nb {dev["n_bad"][i]:4d} | '
                      f'ora {o} q {ora["q_ref"][i]:.3e} r {ora["res_ref"][i, 0]:+.9e} nb {ora["n_bad"][i]:4d} ps {ps[i]}{flag}')
    for s in exprs[:3] + exprs[8:12]:
        w = np.array(pd_.compile(pd_.parse(s)), np.int32)
        for tier in range(4):
            out, st = ctx.point_eval(w, tier)
            print(f'{s[:40]:40s} tier {tier} st {st:3d} res {out[0, 0]:+.12e} im {out[0, 1]:+.3e} S {out[0, 3]:.3e} '
                  f'noise {out[0, 4]:.3e} fin {out[0, 5]}')
        print('   oracle point', O.point(0, w, 0.8, 6 / 7))
    ctx.close()


if __name__ == '__main__':
    main()
