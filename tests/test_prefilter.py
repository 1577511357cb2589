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


def test_d4_stream_prefix_reaches_validate_as_in_reference():
    """The force-free depth-4 stream (147,247 rows of the reference's enumerator, in stream
    order; its first rows are the shallower candidates): the prefix's kept rows equal the
    reference's own filters' (streams/force_free_d4_validated.txt.gz, 142,004 rows)."""
    n = 250
    with gzip.open(os.path.join(G.GOLDEN, 'streams', 'force_free_d4.txt.gz'), 'rt') as f:
        rows = [l.rstrip('\n').split('\t') for _, l in zip(range(n), f)]
    with gzip.open(os.path.join(G.GOLDEN, 'streams', 'force_free_d4_validated.txt.gz'), 'rt') as f:
        ref = [int(l.split('\t')[0]) for l in f]
    res = F.filter_stream('force_free', [r[-1] for r in rows])
    assert res.kept == [i for i in ref if i < n]


def test_d4_full_run_record():
    """The whole depth-4 stream through pdeval.prefilter over the SymPy pool
    (scripts/prefilter_d4.py, run in the build container; its record is committed): the kept
    rows equal the reference's, and the record carries the wall time and pool size the
    end-to-end figure uses."""
    import glob
    recs = sorted(glob.glob(os.path.join(os.path.dirname(G.GOLDEN), '..', 'profiles', '*_prefilter_d4.json')))
    assert recs, 'no committed prefilter_d4 record (scripts/prefilter_d4.py)'
    with open(recs[-1]) as f:
        rec = json.load(f)
    assert rec['rows'] == 147247 and rec['kept'] == 142004 == rec['reference_kept']
    assert rec['kept_equals_reference'] is True, (rec['only_here'][:5], rec['only_reference'][:5])
    assert rec['wall_s'] > 0 and rec['procs'] >= 1
