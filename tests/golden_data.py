"""Loaders for the committed golden fixtures (tests/golden/)."""
import gzip
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def ref_rows(*names):
    rows = []
    for n in names:
        with open(os.path.join(GOLDEN, 'ref', n)) as f:
            rows.extend(json.loads(l) for l in f)
    return rows


def decided(rows):
    """Rows with a reference verdict (no timeout, no validator error)."""
    return [r for r in rows if not r.get('timeout') and r.get('ok') is not None]


def stream(name, with_index=False):
    with gzip.open(os.path.join(GOLDEN, 'streams', name), 'rt') as f:
        rows = [l.rstrip('\n').split('\t') for l in f]
    return rows


FF_REF = ('ff_d1.jsonl', 'ff_d2.jsonl', 'ff_d3_s500.jsonl', 'ff_d4_s500.jsonl', 'ff_d4_s2000.jsonl',
          'ff_d4_exp_quarter.jsonl', 'ff_d4_t600.jsonl')
KERR_REF = ('kerr_d1.jsonl', 'kerr_d2.jsonl', 'kerr_d3_s1000.jsonl', 'kerr_d4_s2000.jsonl',
            'kerr_d4_accepts.jsonl')
# Kerr candidates whose reason class differs from the reference's, with the same verdict: the
# device and the oracle substitute M = 1, a = 1/10 before validating (the reference's point
# check values), while the reference's constant test and symbolic stage keep M and a symbolic
# (kerr validator.py:231-240, :279-300).  This u is constant only at M = 1: here "Trivial
# constant solution excluded", there "PDE residual != 0".  (1 of the 1,024,799
# candidates of the Kerr depth<=4 stream.)
KERR_PARAM_CLASS = {'exp(a**2)*exp(2*r)*exp(-2*M*r)'}
# Force-free candidates whose reject TEXT differs, with the same verdict and the same stage:
# when the reference's symbolic stage is reached with a determinant whose string is >= 3000
# characters it expands instead of calling Lean and prints "Invalid (expanded det != 0)"
# (validator.py:407-426); choosing between the two texts needs SymPy's symbolic det, which this
# path never builds, so the device prints the Lean text.
FF_DET_TEXT = {'rho/z - pow_3_2(rho**2/z**2)'}


def exact_rows(name='ff_d4_exact_det.jsonl'):
    """Exact-arithmetic ground truth (gen_exact_det.py): det_zero = true solution."""
    with open(os.path.join(GOLDEN, 'exact', name)) as f:
        return [json.loads(l) for l in f]
