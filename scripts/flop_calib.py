#!/usr/bin/env python3
"""Per-opcode FP64 operations the lean grid pass executes per sample point, from the PMC
calibration run (scripts/microbench.py --set calib under scripts/gpu_pmc_micro.sh, summarized by
scripts/pmc_micro.py into profiles/*_calib_<problem>.json): one program per opcode the FLOP model
prices, FLOPs per point = (2 FMA + MUL + ADD) per wave / 64 rows (TRANS -- rcp, rsq estimates --
not counted, as in bench.py's counter fraction).  A least-squares fit over the opcode counts of
the calibration programs gives the cost of each opcode and of the per-point epilogue; the table
is what pdeval.hip op_flops / the epilogue constant use.

Usage: python scripts/flop_calib.py profiles/r06_c_calib_force_free.json [...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))


# pushes of a coordinate, a constant or a coordinate power set a jet from the row / lane values
# and the power tables: no FP64 arithmetic (PUSH_P's table values are loaded, not computed)
FREE = ('PUSH_X', 'PUSH_Y', 'PUSH_C', 'PUSH_P', 'PUSH_I')


def opcode_counts(pd_, s):
    from pdeval import problem_defs as P
    from pdeval.opcodes import OP_NAME, op_len
    ops, off, _ = P.compile_strings(pd_, [s])
    w = ops[off[0]:off[1]]
    out = {}
    pc = 1
    while pc < len(w):
        name = OP_NAME.get(int(w[pc]) & 0xff, str(int(w[pc]) & 0xff))
        if name in ('POWN',):
            name = f'POWN{(int(w[pc]) >> 8) & 0xff}'
        out[name] = out.get(name, 0) + 1
        pc += op_len(int(w[pc]))
    return out


def fit(path):
    from pdeval import problem_defs as P
    d = json.load(open(path))
    pd_ = P.force_free() if d['problem'] == 'force_free' else P.kerr()
    rows, y, names = [], [], []
    cnts = {}
    for prog, v in d['per_wave'].items():
        fl = (2 * v['SQ_INSTS_VALU_FMA_F64'] + v['SQ_INSTS_VALU_MUL_F64'] + v['SQ_INSTS_VALU_ADD_F64']) / 64.0
        c = opcode_counts(pd_, prog)
        cnts[prog] = (c, fl)
        for k in c:
            if k in FREE:
                continue
            if k not in names:
                names.append(k)
    names = ['EPILOGUE'] + sorted(names)
    A = np.array([[1.0] + [cnts[p][0].get(k, 0) for k in names[1:]] for p in cnts])
    y = np.array([cnts[p][1] for p in cnts])
    # costs >= 0; pushes of a coordinate / constant cost nothing but are kept in the fit
    x, *_ = np.linalg.lstsq(A, y, rcond=None)
    res = A @ x - y
    return d['problem'], dict(zip(names, np.round(x, 2))), float(np.abs(res).max())


def main():
    for path in sys.argv[1:]:
        prob, tab, err = fit(path)
        print(json.dumps({'problem': prob, 'source': os.path.basename(path), 'flops_per_point': tab,
                          'max_abs_residual': round(err, 3)}))


if __name__ == '__main__':
    main()
