"""The SymPy CPU path timed on the host cores -- BENCH INFRASTRUCTURE ONLY (bench.py's
cpu_baseline leg; nothing under pde-engine_amd/ imports it).

BASELINE.json's north star asks for "the SymPy CPU path timed on the box's own host cores
(core count stated)".  The path is the reference's per-candidate validate
(problems/force_free/validator.py:260-437), restated in oracle/sympy_validator.py, run the way
BASELINE.md §3 plans it: a multiprocessing.Pool over the host cores, a 60 s per-candidate
timeout (SIGALRM raising a BaseException, so the restatement's blanket ``except Exception``
cannot swallow it), candidates parsed with the driver's sympify locals
(general_method_paper_reproduction.py:84-93).  A wall-clock budget bounds the whole leg:
candidates still running when it expires are reported as unfinished.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import signal
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))


class _Timeout(BaseException):
    pass


def _alarm(*_):
    raise _Timeout()


def _init():
    sys.path.insert(0, os.path.join(os.path.dirname(_HERE), 'pde-engine_amd'))
    sys.path.insert(0, _HERE)
    signal.signal(signal.SIGALRM, _alarm)


def _one(args):
    expr, timeout = args
    from pdeval import problem_defs as P
    import sympy_validator as SV
    pd_ = P.force_free()
    t0 = time.perf_counter()
    signal.alarm(timeout)
    try:
        ok, reason = SV.ff_validate(pd_.parse(expr), pd_.x, pd_.y)
        out = ('done', ok, reason)
    except _Timeout:
        out = ('timeout', None, None)
    except Exception as e:   # noqa: BLE001
        out = ('error', None, str(e)[:80])
    finally:
        signal.alarm(0)
    return (expr,) + out + (time.perf_counter() - t0,)


def run(exprs, procs: int, timeout: int = 60, budget_s: float = 100.0):
    """Validate `exprs` on `procs` processes; returns a summary dict (rates over the wall
    time, with and without timed-out candidates)."""
    t0 = time.perf_counter()
    done, timeouts, errors, per = 0, 0, 0, []
    pool = mp.get_context('fork').Pool(procs, _init)
    try:
        it = pool.imap_unordered(_one, [(e, timeout) for e in exprs])
        n_seen = 0
        while n_seen < len(exprs):
            left = budget_s - (time.perf_counter() - t0)
            if left <= 0:
                break
            try:
                _, st, _, _, dt = it.next(timeout=left)
            except mp.TimeoutError:
                break
            n_seen += 1
            if st == 'done':
                done += 1
                per.append(dt)
            elif st == 'timeout':
                timeouts += 1
            else:
                errors += 1
        wall = time.perf_counter() - t0
    finally:
        pool.terminate()
        pool.join()
    unfinished = len(exprs) - done - timeouts - errors
    per.sort()
    return {'candidates': len(exprs), 'completed': done, 'timeouts_60s': timeouts, 'errors': errors,
            'unfinished_at_budget': unfinished, 'wall_s': round(wall, 2), 'procs': procs,
            'rate_completed': done / wall, 'rate_incl_timeouts': (done + timeouts) / wall,
            'median_s': per[len(per) // 2] if per else None}
