"""Known-solution recovery (pdeval.discovery) on the CPU, with the oracle standing in for the
device context: fingerprint matching + the reference's simplify(u - known) == 0 confirmation
(general_method_paper_reproduction.py:1783-1798), and the direct validation of the 7 known
solutions (:481-499)."""
import numpy as np

import golden_data as G
import oracle_lib as O
from pdeval import problem_defs as P
from pdeval.discovery import find_known_solutions, fingerprint_matches


class _OracleCtx:
    def validate(self, ops, off, params=None):
        return O.validate(0, ops, off, O.params(full_grid=0))


def test_fingerprint_matches():
    ref = np.array([[1.0, 2.0, 3.0, 4.0], [0.5, 0.5, np.nan, 1.0]])
    fp = np.array([[1.0, 2.0, 3.0, 4.0 + 1e-14],     # equal to ref 0 within rtol
                   [1.0, 2.0, 3.0, 4.1],             # differs
                   [0.5, 0.5, 7.0, 1.0],             # equal to ref 1 where both finite
                   [np.nan, np.nan, np.nan, 1.0]])   # too few finite points
    m = fingerprint_matches(fp, ref)
    assert m.tolist() == [[True, False], [False, False], [False, True], [False, False]]


def test_recovers_known_solutions_depth3():
    rows = G.stream('force_free_d3_validated.txt.gz')
    exprs = [r[-1] for r in rows]
    pd_ = P.force_free()
    ops, off, _ = P.compile_strings(pd_, exprs)
    rec = find_known_solutions(_OracleCtx(), pd_, ops, off, exprs)
    assert rec.n_found == 7, rec.found
    assert all(rec.direct_valid.values())
    # depth <= 3 streams Vertical, X-point and Parabolic forms
    for name in ('Vertical field', 'X-point', 'Parabolic'):
        assert rec.found[name] == 'stream', (name, rec)
    assert rec.found['Hyperbolic'] == 'direct'
