#!/usr/bin/env python3
"""Validate a whole program set on the GPU and write the candidates the device accepts (and a
class histogram), so that the reference's verdicts can be collected for exactly those rows in the
build container (tests/golden/gen_reference_verdicts.py).  The reference fixtures sampled at
random hold no Kerr accept; this enriches them with the accept path.

    python scripts/kerr_accepts.py data/kerr_magnetosphere_d4_stream.npz gpurun_out/kerr_d4_accepts.txt
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))


def main(npz, out, problem='kerr_magnetosphere'):
    from pdeval import _lib
    from pdeval.opcodes import PROBLEM_FORCE_FREE, PROBLEM_KERR
    pid = PROBLEM_KERR if problem.startswith('kerr') else PROBLEM_FORCE_FREE
    z = np.load(npz, allow_pickle=False)
    ops, off, exprs, depth = z["ops"], z["offsets"], z["exprs"], z["depth"]
    ctx = _lib.Context(pid, device=0)
    res = ctx.validate(ops, off)
    ctx.close()
    acc = np.flatnonzero(res['verdict'])
    with open(out, 'w') as f:
        for i in acc:
            f.write(f"{i}\t{depth[i]}\t{exprs[i]}\n")
    print(json.dumps({'candidates': len(off) - 1, 'accepted': int(len(acc)),
                      'status_hist': np.bincount(res['status'], minlength=8).tolist()}))


if __name__ == '__main__':
    main(*sys.argv[1:])
