"""The force-free point rejects that only the fp64 range caused (pdeval.batch.ff_range_point_check):
every row of the reference's depth-4 stream that reaches validate and that the device rejects
for a non-finite value at p* (26 of the 142,004), plus the one such row of the faithful
depth-5 sample, with the reference's verdicts recorded at a 120 s limit
(tests/golden/ref/ff_range_rows.jsonl, gen_reference_verdicts.py verdicts --timeout 120 on
tests/golden/ff_range_rows.txt).  CPU: the device's classes from the C oracle, then the host
steps as the plugin applies them."""
import json
import os

import numpy as np

import golden_data as G
import oracle_lib as O
from pdeval import _lib
from pdeval import problem_defs as P
from pdeval.batch import apply_host_steps, ff_range_point_check


def _rows():
    with open(os.path.join(G.GOLDEN, 'ref', 'ff_range_rows.jsonl')) as f:
        return [json.loads(l) for l in f]


def test_range_rows_take_the_reference_verdict():
    pd = P.force_free()
    rows = _rows()
    strs = [r['expr'] for r in rows]
    ops, off, _ = P.compile_strings(pd, strs)
    r = O.validate_mt(0, ops, off)
    r['verdict'] = r['status'] == 0
    dev = r['verdict'].copy()
    # every row is a point reject with no finite scaled residual at p*
    assert np.all(r['status'] == 1) and not np.any(r['q_ref'] > 0)
    apply_host_steps(pd, None, _lib.default_params(0), 4096, strs, r, ops, off)
    dec = [i for i, x in enumerate(rows) if x['ok'] is not None]
    assert len(dec) >= 12
    # before the step the device agreed on 2 of them (the reference's rejects), after it on all
    assert sum(bool(dev[i]) == rows[i]['ok'] for i in dec) == 2
    bad = [strs[i] for i in dec if bool(r['verdict'][i]) != rows[i]['ok']]
    assert not bad, bad


def test_range_step_leaves_every_decided_fixture_row():
    """No decided force-free fixture row (depth 1-5, every sample) is a range-caused point
    reject: the step changes none of them."""
    pd = P.force_free()
    rows = {}
    for name in sorted(os.listdir(os.path.join(G.GOLDEN, 'ref'))):
        if name.startswith('ff_') and name.endswith('.jsonl') and name != 'ff_range_rows.jsonl':
            for x in G.decided(G.ref_rows(name)):
                if x.get('omega', '0') == '0':
                    rows.setdefault(x['expr'], x)
    strs = list(rows)
    ops, off, _ = P.compile_strings(pd, strs)
    r = O.validate_mt(0, ops, off)
    r['verdict'] = r['status'] == 0
    assert ff_range_point_check(pd, strs, r, ops, off, 4096, True, 0) == []


def test_range_step_keeps_poles():
    """A pole at p* (a division by an exact zero in the value evaluation) is the reference's
    reject too: the step leaves it."""
    from pdeval.batch import _exp_overflows, _FF_REF_POINT
    pd = P.force_free()
    ops, off, _ = P.compile_strings(pd, ['1/(5*rho - 4)', 'exp(exp(z/(1 - z)))'])
    assert not _exp_overflows(ops[off[0]:off[1]], (0.0,) * 8, _FF_REF_POINT, magnitude=True)
    assert _exp_overflows(ops[off[1]:off[2]], (0.0,) * 8, _FF_REF_POINT, magnitude=True)
