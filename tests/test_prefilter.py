"""The driver's pre-validate filters on the host (pdeval/prefilter.py) against
what the reference itself produced:

* the candidates that reach ``validate`` -- streams/<slug>_d3_validated.txt.gz, made by running
  the reference's ``_has_degenerate_denominator`` / UNIQUE(normalized) / constant-only steps
  over its own enumerator's stream (tests/golden/gen_reference_verdicts.py --mode filters) --
  on a prefix of each problem's depth-3 stream (the dedupe is sequential, so a prefix is
  self-contained; the whole force-free d3 stream, 3,786 rows, agrees too: 3,687 kept, 81
  duplicates, 18 constant-only -- 90 s on 7 pool processes, not run here);
* the ``normalized`` / ``signature`` columns of the run table the reference driver wrote
  (tests/golden/ref/driver_kerr_d2_rows.jsonl, gen_driver_rows.py).
"""
import gzip
import json
import os

import pytest

import golden_data as G
from pdeval import prefilter as F


@pytest.mark.parametrize('s, degenerate', [
    ('1/(rho - rho)', True), ('rho/(z - z)', True), ('(1 - 1)**-1', True), ('inv(rho - rho)', True),
    ('exp(rho)/(rho**2 - rho*rho)', True), ('rho/z', False), ('exp_neg(rho/z)', False),
])
def test_degenerate_denominator(s, degenerate):
    assert F.filter_one(('force_free', s)).degenerate is degenerate


@pytest.mark.parametrize('slug, n', [('force_free', 300), ('kerr_magnetosphere', 200)])
def test_stream_prefix_reaches_validate_as_in_reference(slug, n):
    with gzip.open(os.path.join(G.GOLDEN, 'streams', f'{slug}_d3.txt.gz'), 'rt') as f:
        rows = [l.rstrip('\n').split('\t') for l in f][:n]
    with gzip.open(os.path.join(G.GOLDEN, 'streams', f'{slug}_d3_validated.txt.gz'), 'rt') as f:
        ref = [int(l.split('\t')[0]) for l in f]
    res = F.filter_stream(slug, [r[1] for r in rows])
    assert res.kept == [i for i in ref if i < n]
    st = res.stats
    assert st['validated'] + st['degenerate'] + st['duplicate'] + st['const_only'] == n
    assert len(res.inserted) == st['validated'] + st['const_only'] and set(res.kept) <= set(res.inserted)


def test_keys_equal_the_reference_run_table():
    with open(os.path.join(G.GOLDEN, 'ref', 'driver_kerr_d2_rows.jsonl')) as f:
        rows = [json.loads(l) for l in f][:120]
    bad = []
    for r in rows:
        got = F.filter_one(('kerr_magnetosphere', r['expression']))
        if got.degenerate or (got.normalized, got.signature) != (r['normalized'], r['signature']):
            bad.append((r['expression'], got, r['normalized'], r['signature']))
    assert not bad, bad[:3]
