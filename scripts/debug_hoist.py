"""Debug: q_grid of the force-free d4 workload with PDEVAL_HOIST on / off, repeated, and the
candidates where they differ (GPU)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'pde-engine_amd'))
from pdeval._lib import Context  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
d = np.load(os.path.join(ROOT, 'data', 'force_free_d4_validated.npz'))
ops, off = d['ops'], d['offsets']


def run(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    ctx = Context(0)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    r = ctx.validate(ops, off)
    ctx.close()
    return r


res = {}
for tag, env in [('h1a', {'PDEVAL_HOIST': '1'}), ('h1b', {'PDEVAL_HOIST': '1'}), ('h0a', {'PDEVAL_HOIST': '0'}),
                 ('h0b', {'PDEVAL_HOIST': '0'}), ('h1s', {'PDEVAL_HOIST': '1', 'PDEVAL_DD_EARLY': '0'}),
                 ('h0s', {'PDEVAL_HOIST': '0', 'PDEVAL_DD_EARLY': '0'})]:
    res[tag] = run(env)
    print(tag, 'done', flush=True)
base = res['h0a']
for tag, r in res.items():
    diff = {k: np.flatnonzero(np.any((r[k] != base[k]).reshape(len(r[k]), -1), axis=1)) for k in
            ('status', 'n_bad', 'n_nonfinite', 'q_grid', 'q_ref', 'fingerprint')}
    print(tag, {k: (len(v), v[:8].tolist()) for k, v in diff.items()}, flush=True)
idx = [10763, 12392, 14345, 15353, 21611, 29859, 30316, 35664, 50854, 92822]
for i in idx:
    print(i, str(d['exprs'][i]), int(base['status'][i]), int(base['n_bad'][i]), int(base['n_nonfinite'][i]),
          ' '.join(f"{t}:{res[t]['q_grid'][i]!r}" for t in res), flush=True)
