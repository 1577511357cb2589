"""Validator worker pool -- the batched, GPU-backed ``_parallel_validator_worker``.

Reproduces the INTENDED semantics of ``general_method_paper_reproduction.py:1671-1824`` (the
snapshot's worker dies on a broken import):

* input  : ``(expr_id, expr_str)`` tuples from ``task_queue`` (``None`` = shut down), or, when the
           queue is idle, up to 50 ``pending`` rows claimed from the run table with the
           compare-and-set ``UPDATE ... WHERE id=? AND validation_status='pending'`` (:1736-1751);
* parse  : ``sympify(expr_str, locals=UNARY_OPS + symbols + constants)`` (:1703-1714, :1767);
* verdict: ``problem.validator.validate_batch(us, **kwargs)`` with the kwargs of :1768-1782
           filtered by the validator's signature -- one GPU call per batch instead of one
           SymPy ``validate`` per candidate; batches are pipelined (``process_batches``: the
           next batch compiles on host threads while the current one is on the device);
* tagging: valid rows are matched against ``problem.known_solutions`` (:1783-1798): a grid
           fingerprint pre-filter on the device, then the reference's ``simplify(u - known)
           == 0`` on the host for fingerprint hits only;
* output : ``(run_id, pid, 'start', expr_id, snippet[:120])`` and ``(run_id, pid, 'end',
           [(status, is_valid, reason, is_paper, paper_name, expr_id), ...])`` on
           ``result_queue`` (:1764, :1816), the protocol ``_db_update_writer`` consumes.
"""
from __future__ import annotations

import inspect
import os
import queue as _queue
import sqlite3
import sys
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import sympy as sp

from . import hostpool

BASE_KWARGS = {'check_regularity': False, 'fast_point_only': False, 'lean_first': True,
               'defer_heavy_checks': True, 'enforce_anchor': False}


def filtered_kwargs(validator) -> Dict[str, object]:
    try:
        fn = getattr(validator, 'validate_batch', None) or validator.validate
        allowed = set(inspect.signature(fn).parameters)
        return {k: v for k, v in BASE_KWARGS.items() if k in allowed}
    except (TypeError, ValueError):
        return {'check_regularity': False, 'fast_point_only': False}


class KnownSolutionTagger:
    """Fingerprint pre-filter + exact SymPy confirmation of known-solution matches."""

    def __init__(self, problem, locals_: Dict[str, object], device: int = 0, rtol: float = 1e-9):
        from .batch import get_validator
        self.known = []
        self.locals = locals_
        self.rtol = rtol
        self.slug = getattr(problem, 'slug', None)
        items = list((getattr(problem, 'known_solutions', None) or {}).items())
        self.known_str = [k for k, _ in items]
        if not items:
            self.fps = np.zeros((0, 4))
            return
        self.bv = get_validator(problem.slug, device)
        exprs = [sp.sympify(k, locals=locals_) for k, _ in items]
        res = self.bv.validate_exprs(exprs)
        self.known = [(e, name) for e, (_, name) in zip(exprs, items)]
        self.fps = np.array([v.fingerprint for v in res])

    def fingerprints(self, us: Sequence[sp.Basic]) -> np.ndarray:
        return np.array([v.fingerprint for v in self.bv.validate_exprs(list(us))])

    def tag(self, us: Sequence[sp.Basic], fps: Optional[np.ndarray] = None) -> List[Tuple[bool, Optional[str]]]:
        """Known-solution tags of valid rows.  ``us``: SymPy trees, or strings (parsed only
        when their fingerprint matches); ``fps``: their fingerprints from the validation call
        that accepted them (validated again on the device when not given)."""
        out: List[Tuple[bool, Optional[str]]] = [(False, None)] * len(us)
        if not self.known or not len(us):
            return out
        fp = np.asarray(fps) if fps is not None else self.fingerprints(
            [sp.sympify(u, locals=self.locals) if isinstance(u, str) else u for u in us])
        hits = self.fingerprint_hits(fp)
        pairs = [(i, k) for i in np.flatnonzero(hits.any(axis=1)).tolist()
                 for k in np.flatnonzero(hits[i]).tolist()]
        if self.slug and pairs and all(isinstance(us[i], str) for i, _ in pairs):
            # strings: the SymPy confirmations over the pool, even one at a time (the worker's
            # result thread then keeps the GIL free for the compile and device threads)
            same = hostpool.run(_confirm_str, [(self.slug, us[i], self.known_str[k]) for i, k in pairs],
                                min_items=1)
        else:
            same = [_confirm(us[i], self.known[k][0], self.locals) for i, k in pairs]
        for (i, k), eq in zip(pairs, same):
            if eq and not out[i][0]:          # the first known solution that confirms
                out[i] = (True, self.known[k][1])
        return out

    def fingerprint_hits(self, fp) -> np.ndarray:
        """(n, n_known) bool: fingerprint i matches known solution k -- at least 2 points
        finite in both and np.allclose(rtol, atol=1e-12) on those, for all pairs at once."""
        a = np.asarray(fp, dtype=np.float64).reshape(-1, 1, self.fps.shape[1])
        b = self.fps.reshape(1, -1, self.fps.shape[1])
        with np.errstate(invalid='ignore', over='ignore'):
            fin = np.isfinite(a) & np.isfinite(b)
            close = np.abs(a - b) <= 1e-12 + self.rtol * np.abs(b)
        return (fin.sum(axis=2) >= 2) & np.all(close | ~fin, axis=2)


def _confirm(u, ke, locs) -> bool:
    """The reference's known-solution test, ``simplify(u - known) == 0`` (:1791)."""
    try:
        ue = sp.sympify(u, locals=locs) if isinstance(u, str) else u
        return bool(sp.simplify(ue - ke) == 0)
    except Exception:   # noqa: BLE001
        return False


_LOCS: Dict[str, Dict[str, object]] = {}


def _confirm_str(args) -> bool:
    """_confirm in a pool process: the worker's sympify locals rebuilt from the problem
    (validator_worker's, :1703-1712)."""
    slug, u, known = args
    if slug not in _LOCS:
        from problems import load_problem
        p = load_problem(slug)
        _LOCS[slug] = {**p.unary_ops, **p.symbols, **p.constants}
    locs = _LOCS[slug]
    kt = _KNOWN.get((slug, known))
    if kt is None:
        kt = _KNOWN[(slug, known)] = sp.sympify(known, locals=locs)
    return _confirm(u, kt, locs)


_KNOWN: Dict[Tuple[str, str], sp.Basic] = {}


def validator_worker(run_id: str, table_name: Optional[str], db_path: Optional[str],
                     problem_name: str = 'force_free', task_queue=None, result_queue=None,
                     batch_size: int = 4096, device: int = 0, idle_exit_s: Optional[float] = None,
                     local_workers: Optional[int] = None):
    """Worker process body (``--validators`` process; two per GPU keep the device busy, one
    process's Python parts share a GIL: INTEGRATION.md §3).  Returns the number of candidates
    validated.  ``local_workers``: worker processes on this host (their SymPy pools share its
    cores)."""
    # the SymPy pool for declined strings and host checks, before the GPU is touched
    hostpool.start(local_workers=local_workers)
    try:
        return _worker_loop(run_id, table_name, db_path, problem_name, task_queue, result_queue,
                            batch_size, device, idle_exit_s)
    finally:
        hostpool.stop()


def _worker_loop(run_id, table_name, db_path, problem_name, task_queue, result_queue, batch_size,
                 device, idle_exit_s):
    from problems import load_problem
    problem = load_problem(problem_name)
    validator = problem.validator
    if hasattr(validator, 'device'):
        validator.device = device
    locs: Dict[str, object] = {}
    locs.update(problem.unary_ops)
    locs.update(problem.symbols)
    locs.update(problem.constants)
    kwargs = filtered_kwargs(validator)
    tagger = KnownSolutionTagger(problem, locs, device)
    conn = None
    if db_path and table_name:
        conn = sqlite3.connect(db_path)
        conn.execute('PRAGMA journal_mode=WAL')
        conn.execute('PRAGMA busy_timeout=5000')
    pid = os.getpid()
    done = 0

    def claims():
        """Claimed batches, as the reference's loop claims them; None when idle (the pipeline
        then flushes the batch it holds, so no result waits for the next claim)."""
        stop = False
        last_work = time.time()
        while not stop:
            claimed: List[Tuple[int, str]] = []
            if task_queue is not None:
                try:
                    item = task_queue.get(timeout=0.2)
                    if item is None:
                        stop = True
                    else:
                        claimed.append(item)
                        while len(claimed) < batch_size:
                            item = task_queue.get_nowait()
                            if item is None:
                                stop = True
                                break
                            claimed.append(item)
                except _queue.Empty:
                    pass
            if not claimed and conn is not None and not stop:
                cur = conn.execute(f"SELECT id, expression FROM {table_name} "
                                   f"WHERE validation_status = 'pending' LIMIT 50")
                for expr_id, expr_str in cur.fetchall():
                    c2 = conn.execute(f"UPDATE {table_name} SET validation_status = 'in_progress' "
                                      f"WHERE id = ? AND validation_status = 'pending'", (expr_id,))
                    if c2.rowcount == 1:
                        claimed.append((expr_id, expr_str))
                conn.commit()
            if not claimed:
                if idle_exit_s is not None and time.time() - last_work > idle_exit_s:
                    break
                yield None
                if not stop:
                    time.sleep(0.2)
                continue
            last_work = time.time()
            if result_queue is not None:
                try:
                    result_queue.put((run_id, pid, 'start', claimed[0][0], claimed[0][1][:120]), timeout=0.5)
                except Exception:   # noqa: BLE001
                    pass
            yield claimed

    for results in process_batches(claims(), validator, kwargs, locs, tagger):
        done += len(results)
        if result_queue is not None:
            result_queue.put((run_id, pid, 'end', results), timeout=5.0)
    if conn is not None:
        conn.close()
    return done


def process_batch(claimed, validator, kwargs, locs, tagger):
    """(expr_id, expr_str) list -> result tuples of the reference's writer protocol."""
    if (hasattr(validator, 'validate_strings') and not kwargs.get('check_regularity', False)
            and not kwargs.get('fast_point_only', False)):
        return _process_batch_strings(claimed, validator, locs, tagger)
    us, ids, results = [], [], []
    for expr_id, expr_str in claimed:
        try:
            us.append(sp.sympify(expr_str, locals=locs))
            ids.append(expr_id)
        except Exception as e:   # noqa: BLE001
            results.append(('error', None, f'Validator Error: {e}', None, None, expr_id))
    if us:
        if hasattr(validator, 'validate_batch'):
            verdicts = validator.validate_batch(us, **kwargs)
        else:
            verdicts = [validator.validate(u, **kwargs) for u in us]
        valid = [i for i, (ok, _) in enumerate(verdicts) if ok]
        tags = dict(zip(valid, tagger.tag([us[i] for i in valid])))
        for i, (ok, reason) in enumerate(verdicts):
            is_paper, name = tags.get(i, (False, None))
            results.append(('completed', bool(ok), reason, is_paper, name, ids[i]))
    return results


def _process_batch_strings(claimed, validator, locs, tagger):
    """Fast path of process_batch: one native compile of the batch (SymPy only for the
    strings the native compiler declines), one device call, and the known-solution tags
    from that call's fingerprints -- SymPy parses only parse errors (whose message the
    reference reports as 'Validator Error: ...', :1703-1714) and fingerprint hits (the
    reference's simplify(u - known) == 0, :1785-1798)."""
    bv = validator._validator()
    p = bv.prepare_strings([s for _, s in claimed])
    return _results(claimed, p, bv.finish(p, bv.run_prepared(p), **_symbolic_args(validator)), locs, tagger)


def _symbolic_args(validator) -> dict:
    """The plugin's host replay of the reference's symbolic stage (pdeval.batch.symbolic_stage)."""
    fn = getattr(validator, 'symbolic_args', None)
    return fn() if fn is not None else {}


def _results(claimed, p, t, locs, tagger, hold=None):
    """Result tuples of one batch from its compile (p) and its verdict table (t): errors
    first, then the completed rows in claim order (the order process_batch has always used).
    ``hold`` (optional, bool[n]): rows left out of the list, returned as {row: tuple} beside it
    (the streaming strict mode emits them when their replay resolves)."""
    from itertools import repeat
    from .native import COMPILE_PARSE
    cst = p.get('compile_status')
    ok, reasons = t['ok'], t['reasons']
    ids = [e for e, _ in claimed]
    results = []
    drop = np.zeros(len(claimed), dtype=bool)
    if cst is not None:
        for i in np.flatnonzero(np.asarray(cst) == COMPILE_PARSE):
            try:
                sp.sympify(claimed[i][1], locals=locs)
            except Exception as e:   # noqa: BLE001
                results.append(('error', None, f'Validator Error: {e}', None, None, ids[i]))
                drop[i] = True
    valid = np.flatnonzero(ok & ~drop)
    strs = p['strings']
    tags = tagger.tag([strs[i] for i in valid], fps=np.asarray(t['fingerprint'])[valid].reshape(-1, 4))
    is_paper = [False] * len(claimed)
    names: List[Optional[str]] = [None] * len(claimed)
    for i, (tagged, name) in zip(valid.tolist(), tags):
        if tagged:
            is_paper[i], names[i] = True, name
    rows = zip(repeat('completed'), ok.tolist(), reasons, is_paper, names, ids)
    if hold is not None:
        held = {}
        for i, (r, d, h) in enumerate(zip(rows, drop.tolist(), hold.tolist())):
            if h and not d:
                held[i] = r
            elif not d:
                results.append(r)
        return results, held
    if drop.any():
        results.extend(r for r, d in zip(rows, drop.tolist()) if not d)
    else:
        results.extend(rows)
    return results


class StrictStream:
    """The 'strict' symbolic mode of the worker pipeline, streamed: a batch's
    rows are emitted at device rate except its grid zeros of a possibly suspect shape
    (pdeval.symbolic.may_be_suspect, a string test), which go to the SymPy pool one by one
    (pdeval.symbolic.strict_str: the shape test, then the reference's symbolic stage replayed
    under the per-candidate bound) and are emitted when their task resolves.  Each row's final
    tuple is the one the batch-synchronous strict mode gives (pdeval.batch._strict_stage): a
    replay's verdict and text, 'keep' / a timeout / a SymPy failure the device's; a row the
    replay turns valid gets its known-solution tag from its fingerprint then.  ``stats``:
    grid zeros, rows sent to the pool, suspects, replays, timeouts."""

    def __init__(self, bv, tagger, timeout: float):
        import threading
        from collections import deque
        self.bv, self.tagger, self.timeout = bv, tagger, timeout
        self.pending = deque()   # (future, held tuple, string, fingerprint, device ok)
        self.lock = threading.Lock()   # split() runs on the pipeline's result thread
        self.stats = {'grid_zero': 0, 'sent': 0, 'suspect': 0, 'replayed': 0, 'timeouts': 0}

    def split(self, claimed, p, t, locs):
        """Ready tuples of one batch (finished with symbolic='off'); its held rows are queued."""
        from .opcodes import CLS_ACCEPT, CLS_REJECT_SYMBOLIC
        from . import symbolic as S
        st = np.asarray(t['status'])
        strs = p['strings']
        gz = np.isin(st, (CLS_ACCEPT, CLS_REJECT_SYMBOLIC))
        self.stats['grid_zero'] += int(gz.sum())
        hold = gz & np.fromiter((S.may_be_suspect(x) for x in strs), dtype=bool, count=len(strs))
        ready, held = _results(claimed, p, t, locs, self.tagger, hold)
        fp = np.asarray(t['fingerprint']).reshape(len(st), -1)
        for i, row in held.items():
            self.stats['sent'] += 1
            fut = hostpool.submit(S.strict_str, (self.bv.pd.slug, strs[i], self.bv.omega),
                                  item_timeout=self.timeout, default='timeout')
            with self.lock:
                self.pending.append((fut, row, strs[i], fp[i], bool(t['ok'][i])))
        return ready

    def _final(self, r, row, s, fp, dev_ok):
        if r == 'keep' or r is None:
            return row
        self.stats['suspect'] += 1
        if r == 'timeout':
            self.stats['timeouts'] += 1
            return row
        self.stats['replayed'] += 1
        ok, text = r
        tagged, name = (row[3], row[4]) if (ok and dev_ok) else (False, None)
        if ok and not dev_ok:
            tagged, name = self.tagger.tag([s], fps=np.asarray([fp]))[0]
        return (row[0], bool(ok), text, tagged, name, row[5])

    def drain(self, wait: bool = False):
        """The held rows resolved so far (all of them with wait=True), as one tuple list."""
        with self.lock:
            items = list(self.pending)
            self.pending.clear()
        out, keep = [], []
        for it in items:
            if wait or it[0].done():
                out.append(self._final(it[0].result(), *it[1:]))
            else:
                keep.append(it)
        if keep:
            with self.lock:
                self.pending.extendleft(reversed(keep))
        return out


def process_batches(batches, validator, kwargs, locs, tagger, depth: Optional[int] = None,
                    compilers: Optional[int] = None, stream_strict: bool = True, stats: Optional[dict] = None):
    """process_batch over an iterable of claimed batches, pipelined in four stages on their own
    threads: the next batches compile on the host (``compilers`` threads, so that one batch's
    native compile -- C++ threads, GIL released -- overlaps another's wait for the SymPy pool),
    the batch before them runs on the device (one library call, GIL released), the one before
    that gets its host steps and verdict table (``finish``), and the oldest its known-solution
    tags and result tuples.  The last two mostly wait for the SymPy pool processes
    (pdeval.hostpool: gradient checks, simplify confirmations), so on separate threads those
    waits overlap instead of adding up (r04_e profile: finish 0.071 s + results 0.097 s per
    142 k rows on one thread was the pipeline's critical path).  ``depth`` batches are in
    flight at most.  Yields each batch's result tuples, in order, identical to
    process_batch's.  An empty or None batch (the queue is idle) flushes.

    In the 'strict' symbolic mode (``stream_strict``, the default) the replays do not hold
    their batch: each batch yields its other rows at once, and the held rows come later in
    lists of their own as their replays resolve (:class:`StrictStream`) -- the same tuples as
    process_batch's, in another order; ``stats`` (a dict) receives the mode's counts."""
    if not (hasattr(validator, 'validate_strings') and not kwargs.get('check_regularity', False)
            and not kwargs.get('fast_point_only', False)):
        for claimed in batches:
            if claimed:
                yield process_batch(claimed, validator, kwargs, locs, tagger)
        return
    from collections import deque
    from concurrent.futures import ThreadPoolExecutor
    # (defaults 8 batches in flight and 4 compile threads; PDEVAL_PIPE_DEPTH / _COMPILERS)
    if depth is None:
        depth = int(os.environ.get('PDEVAL_PIPE_DEPTH', '8'))
    if compilers is None:
        compilers = int(os.environ.get('PDEVAL_PIPE_COMPILERS', '4'))
    bv = validator._validator()
    sym = _symbolic_args(validator)
    # the pipeline's threads hand the GIL to each other often: with the interpreter's default
    # 5 ms switch interval, a thread back from a GIL-free C call (the device call, the native
    # compile) can wait a whole interval for a stage thread holding it (PDEVAL_SWITCH_INTERVAL)
    sw_old = sys.getswitchinterval()
    # (default: the interpreter's own; 0.5 ms measured no better -- the single-process pipeline
    # 866 k/s before, 711 k/s with it and the 128-string compile chunks, profiles/r06_final_bench)
    sw = float(os.environ.get('PDEVAL_SWITCH_INTERVAL', '0'))
    if sw > 0:
        sys.setswitchinterval(sw)
    strict = None
    if stream_strict and sym.get('symbolic') == 'strict' and bv.pd.slug == 'force_free':
        strict = StrictStream(bv, tagger, sym.get('symbolic_timeout') or bv.symbolic_timeout)
        sym = {**sym, 'symbolic': 'off'}

    # each stage is one thread and takes its batches in submission order, so a stage only ever
    # waits for an earlier stage's future of the same batch
    def run(pf):              # device thread: waits for its batch's compile, then runs it
        p = pf.result()
        return p, bv.run_prepared(p)

    def fin(df):
        p, r = df.result()
        return p, bv.finish(p, r, **sym)

    def res(claimed, ff):
        p, t = ff.result()
        if strict is not None:
            return strict.split(claimed, p, t, locs)
        return _results(claimed, p, t, locs, tagger)

    with ThreadPoolExecutor(max_workers=max(1, compilers)) as comp, ThreadPoolExecutor(max_workers=1) as dev, \
            ThreadPoolExecutor(max_workers=1) as fins, ThreadPoolExecutor(max_workers=1) as outs:
        inflight = deque()    # futures of each batch's result tuples

        def resolved(wait=False):
            if strict is not None:
                done = strict.drain(wait)
                if done:
                    yield done

        for claimed in batches:
            if not claimed:
                while inflight:
                    yield inflight.popleft().result()
                yield from resolved(wait=True)
                continue
            pf = comp.submit(bv.prepare_strings, [s for _, s in claimed])
            ff = fins.submit(fin, dev.submit(run, pf))
            inflight.append(outs.submit(res, claimed, ff))
            while len(inflight) > depth:
                yield inflight.popleft().result()
            yield from resolved()
        while inflight:
            yield inflight.popleft().result()
            yield from resolved()
        yield from resolved(wait=True)
    sys.setswitchinterval(sw_old)
    if strict is not None and stats is not None:
        stats.update(strict.stats)
