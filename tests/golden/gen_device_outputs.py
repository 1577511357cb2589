#!/usr/bin/env python3
"""Record the DEVICE's raw outputs (pdeval_validate_batch, before the host steps) for the
fixture rows the multi-rank final-verdict test needs -- run on the GPU box:

    python tests/golden/gen_device_outputs.py

* Kerr: the depth-4 stream rows whose class the host steps decide (``ref/kerr_d4_range.jsonl``,
  among them the fp64-range rows the exact point check turns into accepts) plus a seeded
  sample of ``kerr_d4_s2000.jsonl``;
* force-free: ``ref/ff_edge.jsonl`` and ``ref/ff_d2.jsonl``, plus the 'Zero gradient' rows of
  ``ref/ff_d4_s2000.jsonl`` (the symbolic zero-gradient host step) and a seeded sample of it.

Output ``tests/golden/device/<case>.npz``: the strings, the compiled programs
and every raw output array (no pickles).  ``tests/test_shard_gloo.py`` then runs the per-rank
host steps + gather on the CPU with these as each rank's device results.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'pde-engine_amd')]

import golden_data as G  # noqa: E402


def record(case, problem, files, extra=(), n_extra=0, kerr=None):
    import random
    from pdeval import problem_defs as P
    from pdeval._lib import Context, KerrConstants
    rows = G.ref_rows(*files)
    if extra:
        ex = G.ref_rows(*extra)
        # (every 'Zero gradient' row of the extra files -- the symbolic zero-gradient host step's
        # cases -- and a seeded sample of the rest)
        zg = [r for r in ex if (r.get('reason') or '').startswith('Zero gradient')]
        rows += zg + random.Random(0).sample(ex, min(n_extra, len(ex)))
    strs = [r['expr'] for r in rows]
    pd_ = P.get(problem)
    ops, off, _ = P.compile_strings(pd_, strs)
    ctx = Context(pd_.problem_id, device=0, kerr=KerrConstants(*kerr) if kerr else None)
    try:
        r = ctx.validate(ops, off)
    finally:
        ctx.close()
    ref = np.array([-1 if x.get('ok') is None else int(bool(x['ok'])) for x in rows], np.int8)
    out = os.path.join(HERE, 'device', f'{case}.npz')
    np.savez_compressed(out, problem=np.array(problem), kerr=np.array(kerr or [], np.float64),
                        strings=np.array(strs), ops=np.asarray(ops, np.int32), off=np.asarray(off, np.int64),
                        ref_ok=ref, **{k: np.asarray(v) for k, v in r.items()})
    print(out, len(strs), 'device accepts', int(np.asarray(r['verdict']).sum()))


if __name__ == '__main__':
    # the depth-4 stream rows whose class the host steps decide (default constants) ...
    record('kerr_d4_range', 'kerr_magnetosphere', ('kerr_d4_range.jsonl',), ('kerr_d4_s2000.jsonl',), 300)
    # ... and the validator at a_value = 0, where the exact point check turns device point
    # rejects into accepts (golden_data.KERR_CONFIGS['a_value=0'])
    record('kerr_a_value0', 'kerr_magnetosphere', G.KERR_CONFIGS['a_value=0'][1],
           kerr=G.KERR_CONFIGS['a_value=0'][0])
    record('ff_edge_d2', 'force_free', ('ff_edge.jsonl', 'ff_d2.jsonl'), ('ff_d4_s2000.jsonl',), 200)
