#!/usr/bin/env python3
"""Device vs oracle on a few expressions, with tier 2 on (default kappa) and effectively off
(kappa = 0: every tier-1 failure stands).  Usage: python scripts/debug_cand.py [ff|kerr] EXPR..."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    prob = sys.argv[1]
    exprs = sys.argv[2:]
    import oracle_lib as O
    from pdeval import _lib, problem_defs as P
    from pdeval.flatten import disasm
    pd_ = P.get(prob)
    ops, off, _ = P.compile_strings(pd_, exprs)
    ctx = _lib.Context(pd_.problem_id)
    for kappa in (16.0, 0.0):
        prm = _lib.default_params(pd_.problem_id)
        prm.noise_kappa = kappa
        dev = ctx.validate(ops, off, prm)
        ora = O.validate(pd_.problem_id, ops, off, O.params(noise_kappa=kappa))
        for i, e in enumerate(exprs):
            print(f'kappa={kappa:4} {e[:50]:50s} dev st={dev["status"][i]} qref={dev["q_ref"][i]:.3e} '
                  f'qgrid={dev["q_grid"][i]:.3e} nbad={dev["n_bad"][i]} nnf={dev["n_nonfinite"][i]} | '
                  f'ora st={ora["status"][i]} qref={ora["q_ref"][i]:.3e} qgrid={ora["q_grid"][i]:.3e} '
                  f'nbad={ora["n_bad"][i]} nnf={ora["n_nonfinite"][i]}')
    for i, e in enumerate(exprs):
        print(e, '::', disasm(ops[off[i]:off[i + 1]].tolist()).replace('\n', ' | '))


if __name__ == '__main__':
    main()
