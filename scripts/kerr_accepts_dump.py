"""Dump the Kerr depth<=4 stream's device accepts (diagnostic): expr, class, oracle class."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import oracle_lib as O  # noqa: E402
from pdeval import workload as W  # noqa: E402
from pdeval._lib import Context  # noqa: E402

ops, off, exprs = W.load_programs('kerr_magnetosphere_d4_stream')
ctx = Context(1)
res = ctx.validate(ops, off)
acc = np.flatnonzero(res['status'] == 0)
print('accepts', len(acc))
o, f = W.gather_programs(ops, off, acc)
ora = O.validate(1, o, f)
for k, i in enumerate(acc):
    print(str(exprs[i]), int(res['status'][i]), int(ora['status'][k]), res['q_ref'][i], res['q_grid'][i],
          res['n_bad'][i])
