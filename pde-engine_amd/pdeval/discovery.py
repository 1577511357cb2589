"""Known-solution recovery over a validated batch.

The reference tags a valid candidate as a paper solution when ``simplify(u - known) == 0`` for
one of ``problem.known_solutions`` (``general_method_paper_reproduction.py:1783-1798``; the
force-free dict is ``problems/__init__.py:85-93``).  Sequential mode additionally validates the
known solutions themselves before anything generated (``:481-499``) -- the only way the
Hyperbolic solution, which the depth-4 stream cannot produce, is ever found.

Here the device does the heavy part: one batch validation yields, per candidate, the verdict
and a fingerprint (u at 4 fixed sample points).  Accepted candidates whose fingerprint matches
a known solution's are confirmed on the host with the reference's own ``simplify`` test, in
stream order, until every known solution has a confirmed hit (or the hits run out).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import sympy as sp

from .opcodes import CLS_ACCEPT


def fingerprint_matches(fp: np.ndarray, ref: np.ndarray, rtol: float = 1e-9,
                        atol: float = 1e-12) -> np.ndarray:
    """bool[n, k]: candidate i's fingerprint equals known solution k's on every point where
    both are finite, and at least two such points exist."""
    a = fp[:, None, :]
    b = ref[None, :, :]
    fin = np.isfinite(a) & np.isfinite(b)
    with np.errstate(invalid='ignore'):
        close = np.abs(a - b) <= atol + rtol * np.abs(b)
    return (fin.sum(axis=2) >= 2) & np.all(close | ~fin, axis=2)


@dataclass
class Recovery:
    found: Dict[str, Optional[str]] = field(default_factory=dict)   # name -> how it was found
    direct_valid: Dict[str, bool] = field(default_factory=dict)     # known solution accepted itself
    stream_hits: Dict[str, int] = field(default_factory=dict)       # fingerprint hits in the batch
    confirmed: Dict[str, str] = field(default_factory=dict)         # name -> first confirmed expr
    n_accepted: int = 0
    seconds: Dict[str, float] = field(default_factory=dict)

    @property
    def n_found(self) -> int:
        return sum(1 for v in self.found.values() if v)


def find_known_solutions(ctx, pd_, ops: np.ndarray, offsets: np.ndarray,
                         exprs: Sequence[str], params=None, confirm: bool = True) -> Recovery:
    """Validate the batch (device), then recover every known solution of ``pd_``.

    ``ctx`` is a ``pdeval._lib.Context`` for ``pd_``'s problem; ``exprs[i]`` is the candidate
    string of program i (used only for the host confirmation of fingerprint hits).
    """
    from . import problem_defs as P
    rec = Recovery()
    t0 = time.perf_counter()
    names = list(pd_.known_solutions.values())
    kexprs = [pd_.parse(s) for s in pd_.known_solutions]
    kops, koff, _ = P.compile_exprs(pd_, kexprs)
    kres = ctx.validate(kops, koff, params)
    t1 = time.perf_counter()
    res = ctx.validate(ops, offsets, params)
    t2 = time.perf_counter()
    acc = np.flatnonzero(res['status'] == CLS_ACCEPT)
    rec.n_accepted = int(acc.size)
    hits = fingerprint_matches(res['fingerprint'][acc], kres['fingerprint'])
    t3 = time.perf_counter()
    for k, name in enumerate(names):
        rec.direct_valid[name] = bool(kres['status'][k] == CLS_ACCEPT)
        rows = acc[hits[:, k]]
        rec.stream_hits[name] = int(rows.size)
        if confirm:
            for i in rows:
                try:
                    if sp.simplify(pd_.parse(str(exprs[i])) - kexprs[k]) == 0:
                        rec.confirmed[name] = str(exprs[i])
                        break
                except Exception:   # noqa: BLE001 -- an unparsable row is simply not a match
                    continue
        if name in rec.confirmed:
            rec.found[name] = 'stream'
        elif rec.direct_valid[name]:
            rec.found[name] = 'direct'
        else:
            rec.found[name] = None
    t4 = time.perf_counter()
    rec.seconds = {'validate_known': t1 - t0, 'validate_batch': t2 - t1,
                   'fingerprint_match': t3 - t2, 'confirm_simplify': t4 - t3, 'total': t4 - t0}
    return rec
