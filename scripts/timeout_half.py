#!/usr/bin/env python3
"""How much of the depth-4 headline workload rests on parity that no reference verdict pins
(DESIGN.md §4).

The reference decided only part of its own depth-4 fixtures within its 60 s per-candidate
timeout (tests/golden/ref/ff_d4_s500.jsonl, ff_d4_s2000.jsonl; 23 of the s500 timeouts re-run at
600 s in ff_d4_t600.jsonl).  For the candidates it never decided, and for the whole 142,004
candidate workload, this reports the classes this build gives (the oracle's golden vector,
tests/golden/oracle/force_free_d4_validated.npz, which the GPU tests hold the device to), and
the accepts whose shapes are those where the reference's symbolic stage is known to give false
negatives (problems/force_free/validator.py:404-427): Abs (its assumptions are lost in the
string round trip, lean_bridge.py:73) and exp(..)**(p/q) with a non-integer exponent.
Output: tests/golden/ff_d4_timeout_half.json.
"""
import json
import os
import re
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
import golden_data as G  # noqa: E402
from pdeval.opcodes import CLS_NAME  # noqa: E402
from pdeval.workload import load_programs  # noqa: E402

_EXP_FRAC = re.compile(r'(exp|exp_neg)\(.*\)\*\*\(-?\d+/\d+\)|pow_3_2\(.*exp|pow_neg_3_2\(.*exp|sqrt\(.*exp')


def risky(s: str) -> bool:
    return 'Abs' in s or bool(_EXP_FRAC.search(s))


def main():
    _, _, exprs = load_programs('force_free_d4_validated')
    exprs = [str(e) for e in exprs]
    z = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle', 'force_free_d4_validated.npz'))
    status = z['status']
    where = {s: i for i, s in enumerate(exprs)}
    rows = G.ref_rows('ff_d4_s500.jsonl', 'ff_d4_s2000.jsonl')
    t600 = {r['expr']: r for r in G.ref_rows('ff_d4_t600.jsonl')}
    decided, undecided = {}, {}
    for r in rows:
        if r['expr'] not in where:
            continue
        rr = t600.get(r['expr'], r) if r.get('timeout') else r
        (undecided if rr.get('timeout') or rr.get('ok') is None else decided)[r['expr']] = rr
    undecided = {k: v for k, v in undecided.items() if k not in decided}
    cls_und = Counter(CLS_NAME[int(status[where[s]])] for s in undecided)
    cls_dec = Counter(CLS_NAME[int(status[where[s]])] for s in decided)
    acc = [s for s, c in zip(exprs, status) if c == 0]
    acc_risky = [s for s in acc if risky(s)]
    und_acc_risky = [s for s in undecided if status[where[s]] == 0 and risky(s)]
    out = {
        'workload': 'force_free depth-4 candidates that reach validate (142,004)',
        'classes_all': {CLS_NAME[k]: int(v) for k, v in enumerate(np.bincount(status, minlength=8)) if v},
        'fixtures_decided_by_reference': len(decided),
        'fixtures_undecided_by_reference': len(undecided),
        'classes_on_decided_fixtures': dict(cls_dec),
        'classes_on_undecided_fixtures': dict(cls_und),
        'accepts_all': len(acc),
        'accepts_pinned_by_a_reference_verdict': sum(1 for s in decided if status[where[s]] == 0),
        'accepts_unpinned': len(acc) - sum(1 for s in decided if status[where[s]] == 0),
        'accepts_with_abs_or_fractional_exp_power': len(acc_risky),
        'undecided_fixture_accepts_with_abs_or_fractional_exp_power': und_acc_risky,
        'examples_accepts_with_abs_or_fractional_exp_power': acc_risky[:40],
    }
    path = os.path.join(ROOT, 'tests', 'golden', 'ff_d4_timeout_half.json')
    with open(path, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if not k.startswith('examples')}, indent=1))


if __name__ == '__main__':
    main()
