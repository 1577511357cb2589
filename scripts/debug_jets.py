#!/usr/bin/env python3
"""Device vs oracle jets and error bounds of single programs at given points (debug aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import oracle_lib as O
    from pdeval import _lib, problem_defs as P
    pd_ = P.force_free()
    ctx = _lib.Context(0)
    np.set_printoptions(precision=4, linewidth=200)
    for spec in sys.argv[1:]:
        s, x, y = spec.split('@')
        x, y = float(eval(x)), float(eval(y))
        # prefixes of the program: evaluate after each op by truncating the postfix where the
        # stack depth is 1
        w = np.array(pd_.compile(pd_.parse(s)), dtype=np.int32)
        out, jt = ctx.eval_points(w, [x], [y], tier2=True, jets=True)
        print(s, (x, y), 'dev res/S/noise', out[0][:3], 'ora', O.point(0, w, x, y)[:3])
        print('  dev u  ', jt[0, 0])
        print('  ora u  ', O.jet(0, w, x, y))
        print('  dev E  ', jt[0, 1])


if __name__ == '__main__':
    main()
