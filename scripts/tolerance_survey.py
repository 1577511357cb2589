"""Diagnostic: every fixture candidate where the device's n_bad / n_nonfinite differ from the
oracle's (tests/test_gpu_parity.py's per-candidate tolerances are set from this survey)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import golden_data as G  # noqa: E402
import oracle_lib as O  # noqa: E402
from pdeval import _lib, problem_defs as P  # noqa: E402
from pdeval._lib import Context  # noqa: E402

sets = [('force_free', None, [r['expr'] for r in G.decided(G.ref_rows(*G.FF_REF, 'ff_edge.jsonl'))]
         + [r['expr'] for r in G.exact_rows()])]
for k, files in G.KERR_CONFIGS.values():
    sets.append(('kerr', k, [r['expr'] for r in G.decided(G.ref_rows(*files))]))
out = []
for prob, k, strings in sets:
    pd_ = P.get(prob)
    ops, off, _ = P.compile_strings(pd_, strings)
    ctx = Context(pd_.problem_id, kerr=_lib.KerrConstants(*k) if k else None)
    dev = ctx.validate(ops, off)
    O.set_kerr_constants(k or O.DEFAULT_KERR)
    ora = O.validate_mt(pd_.problem_id, ops, off)
    for i in range(len(strings)):
        if dev['n_bad'][i] != ora['n_bad'][i] or dev['n_nonfinite'][i] != ora['n_nonfinite'][i] or \
                dev['status'][i] != ora['status'][i]:
            out.append({'problem': prob, 'kerr': k, 'expr': strings[i], 'status': [int(dev['status'][i]), int(ora['status'][i])],
                        'n_bad': [int(dev['n_bad'][i]), int(ora['n_bad'][i])],
                        'n_nonfinite': [int(dev['n_nonfinite'][i]), int(ora['n_nonfinite'][i])]})
    ctx.close()
for o in out:
    print(json.dumps(o))
print('TOTAL', len(out))
