"""The depth-4 candidates whose reference verdict is unknown: class histogram and accept shapes.

The reference's `validate` ran past the 60 s limit on 1,078 of the seeded 2,000 force-free d4
sample (ff_d4_s2000) and on 257 of ff_d4_s500; 16 of the 23 re-run at 600 s stayed undecided
(ff_d4_t600).  For those candidates nothing pins the device's verdict.  The device gives the
mathematically right class there (its grid and tier-2 tests do not time out), but the
reference's symbolic stage has false negatives (problems/force_free/validator.py:404-427):
`Abs` of both coordinates (NONSMOOTH2D) and exp(g)**(p/4) (UNPROVABLE) among the decided rows.
This script does NOT import the reference.  It runs the CPU oracle (oracle/jet_oracle.c, equal
class-for-class to the device by the -m gpu parity tests) with the host steps of pdeval.batch:

  * over the undecided fixture rows: the class histogram;
  * over the whole headline workload (data/force_free_d4_validated.npz, the 142,004 d4
    candidates that reach validate): the accepts split by shape --
      abs        contains Abs (NONSMOOTH2D is the two-coordinate subset, a reject already),
      exp_frac   a non-integer power of an expression containing exp,
      radical    another non-integer power,
      plain      none of these --
    and, per shape, how the reference decided the decided fixture rows of that shape (accepts
    vs symbolic-stage rejects).  A shape whose decided rows contain symbolic-stage rejects
    beyond the flagged rules is a shape where device accepts rest on unpinned parity.

Writes tests/golden/ff_d4_undecided.json.  Usage: python tests/golden/summarize_timeouts.py
"""
import collections
import json
import os
import sys
import time

import numpy as np
import sympy as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, 'pde-engine_amd'), os.path.dirname(HERE)]

import golden_data as G            # noqa: E402
import oracle_lib as O             # noqa: E402
from pdeval import problem_defs as P   # noqa: E402
from pdeval.batch import symbolic_zero_gradient   # noqa: E402
from pdeval.opcodes import FLAG_NONSMOOTH2D, FLAG_UNPROVABLE   # noqa: E402

CLASSES = ['ACCEPT', 'REJECT_POINT', 'REJECT_GRID', 'ZERO_GRADIENT', 'NONFINITE_REF', 'UNSUPPORTED',
           'MALFORMED', 'REJECT_SYMBOLIC']
SYMBOLIC_TEXT = 'Invalid (Lean could not simplify det to 0 symbolically)'


def shape(u) -> str:
    if u.has(sp.Abs):
        return 'abs'
    frac = [p for p in u.atoms(sp.Pow) if not p.exp.is_integer]
    if any(p.base.has(sp.exp) for p in frac):
        return 'exp_frac'
    return 'radical' if frac else 'plain'


def classify(pd_, strings):
    ops, off, _ = P.compile_strings(pd_, strings)
    res = O.validate_mt(pd_.problem_id, ops, off)
    symbolic_zero_gradient(pd_, strings, res)
    return res['status'].astype(int), ops, off


def main():
    pd_ = P.force_free()
    t0 = time.time()
    rows = G.ref_rows('ff_d4_s2000.jsonl', 'ff_d4_s500.jsonl')
    t600 = {r['expr']: r for r in G.ref_rows('ff_d4_t600.jsonl')}
    undecided, seen = [], set()
    for r in rows:
        if r.get('timeout') and r['expr'] not in seen:
            seen.add(r['expr'])
            r2 = t600.get(r['expr'])
            if r2 is None or r2.get('timeout'):
                undecided.append(r['expr'])
    st, _, _ = classify(pd_, undecided)
    hist = collections.Counter(CLASSES[c] for c in st)
    und_acc = [s for s, c in zip(undecided, st) if c == 0]
    und_shapes = collections.Counter(shape(pd_.parse(s)) for s in und_acc)

    # decided fixture rows by shape: how the reference decided them
    dec = {}
    for r in G.decided(G.ref_rows(*G.FF_REF)):
        if r['depth'] == 4:
            dec.setdefault(r['expr'], r)
    dec_rows = list(dec.values())
    dec_st, _, _ = classify(pd_, [r['expr'] for r in dec_rows])
    by_shape = collections.defaultdict(collections.Counter)
    for r, c in zip(dec_rows, dec_st):
        if c not in (0, 7):        # only rows the grid finds zero everywhere can split this way
            continue
        key = 'ref_accept' if r['ok'] else ('ref_symbolic_reject' if r['reason'] == SYMBOLIC_TEXT
                                             else 'ref_other_reject')
        by_shape[shape(pd_.parse(r['expr']))][key] += 1

    # the whole headline workload
    d = np.load(os.path.join(ROOT, 'data', 'force_free_d4_validated.npz'))
    exprs = [str(s) for s in d['exprs']]
    res = O.validate_mt(pd_.problem_id, d['ops'], d['offsets'])
    symbolic_zero_gradient(pd_, exprs, res)
    wst = res['status'].astype(int)
    whist = collections.Counter(CLASSES[c] for c in wst)
    acc = np.flatnonzero(wst == 0)
    wshape = collections.Counter(shape(pd_.parse(exprs[i])) for i in acc)
    hdr = d['ops'][d['offsets'][:-1]]
    flagged = {'nonsmooth2d': int(((hdr & FLAG_NONSMOOTH2D) != 0).sum()),
               'unprovable': int(((hdr & FLAG_UNPROVABLE) != 0).sum())}
    pinned = set(exprs[i] for i in acc) & set(r['expr'] for r in dec_rows)
    out = {
        'generated_by': 'tests/golden/summarize_timeouts.py (CPU oracle + pdeval.batch host steps; no reference import)',
        'undecided_fixture_rows': len(undecided),
        'undecided_class_histogram': dict(sorted(hist.items())),
        'undecided_accept_shapes': dict(sorted(und_shapes.items())),
        'decided_d4_rows_zero_on_grid_by_shape': {k: dict(sorted(v.items())) for k, v in sorted(by_shape.items())},
        'workload': {'candidates': len(exprs), 'class_histogram': dict(sorted(whist.items())),
                     'accepts': int(acc.size), 'accept_shapes': dict(sorted(wshape.items())),
                     'accepts_with_a_decided_fixture': len(pinned), 'flagged_rejects': flagged},
        'seconds': round(time.time() - t0, 1),
    }
    with open(os.path.join(HERE, 'ff_d4_undecided.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
