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
          'ff_exp_power_forms.jsonl',
          'ff_d4_exp_quarter.jsonl', 'ff_d4_t600.jsonl')
# kerr_d4_range: the 243 depth-4 stream candidates whose oracle class changed with the round-3
# rules (edge_kerr_range.txt): underflow at a reference point or on the whole grid (a pass, no
# evidence of a constant), a value beyond the fp64 range there, and constants that are constant
# only on the domain (Delta - Abs(Delta)) -- the reference decides 236 of them
KERR_REF = ('kerr_d1.jsonl', 'kerr_d2.jsonl', 'kerr_d3_s1000.jsonl', 'kerr_d4_s2000.jsonl',
            'kerr_d4_accepts.jsonl', 'kerr_d4_range.jsonl')
# The reference's Kerr validator at other constants (gen_reference_verdicts.py --kerr-a-value 0
# [--kerr-op-a-zero]): a_value = 0 with M and a symbolic (kerr validator.py:36-44: the fast point
# check substitutes a = 0, the constant test and the symbolic stage keep a symbolic, so u = 1 - x
# passes the point check and fails the symbolic stage), and the operator built with the number
# 0 for a (the Schwarzschild operator; u's own a is then a free symbol): the reference accepts
# 66 of these (61 of the streams, 5 edge cases), the only Kerr accepts it produces (forms
# c1 + c2*x, with c1, c2 free of r and x).  The edge files (edge_kerr2.txt) hold the rules'
# corner cases: stationary at the reference points, constant only at M = 1, underflow on the
# grid, not real on the grid, u == 0, singular at a = 0, a pole at a reference point.
KERR_A0 = ('kerr_a0_d1.jsonl', 'kerr_a0_d2.jsonl', 'kerr_a0_d3_s1000.jsonl', 'kerr_a0_edge.jsonl')
KERR_OP0 = ('kerr_op0_d1.jsonl', 'kerr_op0_d2.jsonl', 'kerr_op0_d3_s1000.jsonl', 'kerr_op0_edge.jsonl')
# One reason-class divergence, same verdict (False): with the Schwarzschild operator u's own a
# is a free symbol, so the reference cannot evaluate an lhs that contains it and rejects at its
# fast point check ("Indeterminate", kerr validator.py:186-189); the device evaluates u's a at
# its stand-in, where this u underflows to 0 at every reference point, and rejects at the grid.
KERR_CLASS_DIVERGENCE = {('operator_a=0', 'exp_neg(E*exp(r**2)*exp(a**2*x**2))')}
# configuration -> (pdeval_kerr_constants fields, fixture files)
KERR_CONFIGS = {
    'a=1/10': ((1, 1, 1, 10, 1.171875, 0.359375, 0, 0), KERR_REF + ('kerr_edge.jsonl', 'kerr_edge2.jsonl')),
    'a_value=0': ((1, 1, 0, 1, 1.171875, 0.359375, 0, 0), KERR_A0),
    'operator_a=0': ((1, 1, 0, 1, 1.171875, 0.359375, 0, 1), KERR_OP0),
}
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


# Force-free fixture candidates whose grid counts differ between the device and the oracle,
# with the class equal: (|n_bad difference|, |n_nonfinite difference|), measured by
# scripts/tolerance_survey.py on the MI355X (profiles/r03_tolerance_survey.log).  n_bad differs
# only on point rejects, where it is a reported tier-1 count whose points with q near tau_grid
# depend on the evaluation order (device Horner vs oracle explicit powers); n_nonfinite only on
# exp(exp(..)) candidates whose jets overflow near the 2^160 guard at a few grid points.  Every
# other candidate's counts are equal exactly (tests/test_gpu_parity.py).
# Kerr (measured on the MI355X, r03_e): the four depth-4 candidates whose grid values underflow
# into the fp64 subnormals on a band of grid rows (exp(-1.5 r**2/a**2) at the stand-in a): a jet
# there is exactly 0 (not a sample) or subnormal (a sample, failing) depending on the evaluation
# order, so whole rows of 64 points move between n_bad and n_nonfinite.  Class equal.
KERR_COUNT_SLACK = {
    'pow_neg_3_2(exp(r**2/a**2)*exp(a**2*x**2))': (64, 64),
    'pow_3_2(exp_neg(a**2*x**2 + r**2/a**2))': (128, 0),
    'pow_neg_3_2(exp(a**2)*exp(-2*M*r)*exp(r**2/a**2))': (64, 64),
    'pow_3_2(exp_neg(-2*M*r + a**2 + r**2/a**2))': (128, 0),
}
FF_COUNT_SLACK = {
    '1/(-rho/(-rho + z**2 + z) + 1)': (8, 0),
    '1/(-rho/(-rho**2*z + z**3 + z) + z)': (7, 0),
    '1/(-rho/(-rho**2*z + z**3 + z**2) + 1)': (11, 0),
    '1/(-rho/(-rho**2*z**2 + z**4 + z**2) + 1)': (9, 0),
    '1/(1 - 1/(-rho**2 + z**3 + 1))': (6, 0),
    '1/(rho/(-rho**2*z + z**3 + z) - z)': (7, 0),
    'exp(rho/(1 - 1/(-rho**2 + z**2 + 1)))': (6, 0),
    'exp(z/(1 - 1/(-rho**2 + z**2 + 1)))': (6, 0),
    'exp_neg(exp(rho**2)*exp(z**2/(-rho/z + 1)))': (0, 8),
    'exp_neg(exp(rho**2)*exp(z**2/(1 - rho)))': (0, 20),
    'exp_neg(exp(rho/(-rho*z + z)))': (0, 16),
    'exp_neg(exp(rho/(-rho/z + 1)))': (0, 4),
    'exp_neg(exp(z/(-rho/z + 1)))': (0, 4),
    'exp_neg(exp(z/(1 - rho)))': (0, 2),
    'inv(-rho/(-rho**2*z + z**3 + z) + z)': (7, 0),
    'inv(rho/(-rho**2*z + z**3 + z) - z)': (7, 0),
    'pow_neg_3_2(exp(rho/(-rho/z + 1)))': (0, 4),
    'pow_neg_3_2(exp(z/(-rho/z + 1)))': (0, 4),
    'pow_neg_3_2(exp_neg(rho/(-rho/z + 1)))': (0, 4),
    'pow_neg_3_2(exp_neg(z/(-rho/z + 1)))': (0, 4),
    'rho**2 + z**2/(-rho/(-rho + z**2 + z) + 1)': (1, 0),
    'rho**2 + z**2/(-rho/(-rho**2*z + z**3 + z) + z)': (2, 0),
    'rho**2 + z**2/(-rho/(-rho**2*z**2 + z**4 + z**2) + 1)': (5, 0),
    'rho**2 + z**2/(1 - 1/(-rho**2 + z**3 + 1))': (2, 0),
    'rho**2 + z**2/(rho/(-rho**2*z + z**3 + z) - z)': (5, 0),
    'rho/(-rho*z/(-rho + z**2 + z) + z)': (12, 0),
    'rho/(-rho*z/(-rho**2*z + z**3 + z) + z**2)': (7, 0),
    'rho/(-rho*z/(-rho**2*z + z**3 + z**2) + z)': (12, 0),
    'rho/(-rho/(-rho + z**2 + z) + 1)': (7, 0),
    'rho/(-rho/(-rho**2*z + z**3 + z) + z)': (9, 0),
    'rho/(-rho/(-rho**2*z + z**3 + z**2) + 1)': (7, 0),
    'rho/(-rho/(-rho**2*z**2 + z**4 + z**2) + 1)': (7, 0),
    'rho/(1 - 1/(-rho**2 + z**3 + 1))': (2, 0),
    'rho/(rho*z/(-rho**2*z + z**3 + z) - z**2)': (7, 0),
    'rho/(rho/(-rho**2*z + z**3 + z) - z)': (9, 0),
    'rho/(z*(1 - 1/(-rho**2 + z**3 + 1)))': (4, 0),
    'z/(-rho/(-rho + z**2 + z) + 1)': (10, 0),
    'z/(-rho/(-rho**2*z + z**3 + z) + z)': (7, 0),
    'z/(-rho/(-rho**2*z + z**3 + z**2) + 1)': (5, 0),
    'z/(-rho/(-rho**2*z**2 + z**4 + z**2) + 1)': (7, 0),
    'z/(1 - 1/(-rho**2 + z**3 + 1))': (4, 0),
    'z/(rho*(1/(-rho**2*z + z**3 + z) - 1/z) + 1 - 1/(-rho**2 + z**2 + 1))': (7, 0),
    'z/(rho/(-rho**2*z + z**3 + z) - z)': (7, 0),
}

# Depth 5 (configs[3]'s depth; the stream is not enumerable here): the reference's
# verdicts on seeded depth-5 strings of the stream's grammar (gen_d5_sample.py ->
# streams/force_free_d5_sample.txt.gz -> ref/ff_d5_s400.jsonl, the first 400 with a 60 s limit;
# ref/ff_d5_s4000_t20.jsonl, the next 3,600 with a 20 s limit).  The rows the reference decided
# in its symbolic stage against the true verdict -- its false negatives, e.g.
# u = exp(-rho/z + sqrt(rho/z)), a function of rho/z alone (det == 0) whose determinant string is
# long enough for the reference to expand it (validator.py:407-426, "expanded det != 0") while
# SymPy leaves the sqrt(rho/z) terms un-merged -- are reproduced by the 'replay' mode
# (pdeval/symbolic.py); the default mode gives the true verdict.
FF_D5 = ('ff_d5_s400.jsonl', 'ff_d5_s4000_t20.jsonl', 'ff_d5_s7000_t20.jsonl', 'ff_d5_s7600_t20.jsonl')
# the faithful depth-5 sample (tests/golden/gen_d5_faithful.py: the reference's own enumerator
# rules, normalize_batch, signature dedupe and pre-validate filters), the reference's verdicts at
# the 20 s limit in 1,000-row chunks (tests/golden/run_d5f_verdicts.sh)
def ff_d5f_files():
    import glob
    return tuple(sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, 'ref', 'd5f_*_t20.jsonl'))))


# decided faithful-d5 rows where the default mode's verdict differs from the reference's (scored
# by tests/golden/score_d5f.py with pdeval.symbolic.suspect frozen at commit 5708cbc, held out:
# the rule was not refitted): functions of rho/z, det == 0 identically, that the reference's
# symbolic stage cannot reduce (its false negatives) ...
FF_D5F_OFF_DIVERGENCE = frozenset({'2*rho/z - pow_3_2(sqrt(rho/z))', 'rho/z - pow_3_2(sqrt(neg(rho/z)))',
                                   # (rows 4,000-6,350 of the sample, scored after they were
                                   # drawn, the rule still frozen: the same family)
                                   '(rho/z)**(1/4) + z/rho', '-inv(rho/z) + pow_neg_3_2(sqrt(rho/z))'})
# ... of which the frozen suspect rule flags all but 'rho/z - pow_3_2(sqrt(neg(rho/z)))' (strict
# replays them and agrees); that one, a radical of neg(rho/z), it does not flag: strict keeps the
# device's accept
FF_D5F_STRICT_DIVERGENCE = frozenset({'rho/z - pow_3_2(sqrt(neg(rho/z)))'})
FF_D5_SYMBOLIC_DIVERGENCE = {'exp_neg(rho/z - sqrt(rho/z))'}
# Every decided force-free fixture row on which the default mode ('off': the grid's det == 0
# and the structural rules) and the reference's verdict differ -- all decided in the reference's
# symbolic stage, all in a shape pdeval.symbolic.suspect flags, so the 'strict' mode replays
# them and agrees (tests/test_symbolic_replay.py::test_strict_mode_every_decided_row):
#   the reference's false negatives (det == 0, SymPy cannot reduce it) ...
FF_OFF_MODE_DIVERGENCE = {'exp_neg(rho/z - sqrt(rho/z))', 'sqrt(square(inv(rho))/(1 - z))',
                          'exp_neg(rho/z - pow_neg_3_2(exp(rho/z)))',   # (d5 s7000: a function of rho/z)
                          # ... and squares under a fractional power that the NONSMOOTH2D rule
                          # rejects but SymPy's Abs form lets the reference prove
                          'pow_neg_3_2(square(rho - z))', 'pow_neg_3_2(square(rho**2 + z**2 - z - 1))',
                          'pow_3_2(square(-z + neg(rho)))',
                          'sqrt(square(rho**2 + z**2 - 1/(rho**2 + z**2)))'}   # (d5 s7600)
# depth-5 point rejects whose reference text carries a number SymPy's cancel/simplify made up:
# det_M.subs(p*).evalf(50) -- the exact value, what the device and the oracle print -- against
# the reference's cancel(together(.)) -> simplify -> evalf pipeline (validator.py:366-394).
# Same verdict; test_oracle_golden.test_point_text_divergence_is_sympys shows both numbers.
FF_D5_POINT_TEXT_DIVERGENCE = {
    '(pow_neg_3_2(sqrt(z) - z)) - (exp_neg(rho))': ('Invalid (point check ≈ 4.10e+03)',
                                                    'Invalid (point check ≈ 6.13e+12)'),
}
