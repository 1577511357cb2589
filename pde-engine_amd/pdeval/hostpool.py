"""Host process pool for the SymPy work the native compiler and the device leave to the host.

The native compiler (csrc/pdcompile.cpp) compiles 99.9 % of the candidate strings on host
threads; the few it declines go through SymPy (``sp.sympify`` + ``pdeval.flatten``, ~1.5 ms
each), which holds the GIL, and so do the host steps' per-candidate SymPy checks
(``pdeval.batch``: the zero-gradient test, the Kerr structural constant test, the known-solution
``simplify``).  At the rate one GPU validates, those few dominate the worker's host time, so
they are spread over a pool of SymPy processes -- the reference parallelizes its SymPy
validation over processes the same way (``--validators N``,
``general_method_paper_reproduction.py:1671-1824``).

The pool is FORKED, so it must be started before the process touches the GPU (a fork of a
process whose HIP runtime is live is not safe, and an exec from it is forbidden on the GPU
hosts): :func:`start` refuses once torch has initialized CUDA/HIP or a libpdeval context
exists, and the callers then run the work in-process.  For the same reason the pool is a
FIXED set of ``fork`` children that is never replenished (``multiprocessing.Pool`` would fork a
replacement from the parent -- by then GPU-live -- whenever a child exits): if a child dies
(a SymPy crash, an OOM kill), the pool is marked broken and stopped, the job's missing chunks
are computed in-process, and every later call runs in-process.  Children never touch the GPU.
A per-item time bound (``run(..., item_timeout=s, default=d)``) is enforced inside the child
with SIGALRM (raised as a ``BaseException`` SymPy cannot swallow); the item then yields
``default``.  The job as a whole has a deadline too (a child stuck in a C-level call ignores the
signal): chunks still missing then yield ``default``.  In-process, the bound is SIGALRM on the
main thread and an abandoned helper thread elsewhere, so no bounded call can stall a worker
thread past its bound.
"""
from __future__ import annotations

import concurrent.futures as cf
import multiprocessing as mp
import os
import queue as _queue
import signal
import sys
import threading
import time
from typing import List, Optional, Sequence

import numpy as np

_POOL = None
DEADLINE_MARGIN_S = 30.0     # map_chunks: slack of a bounded job's deadline beyond its items' bounds


class _ItemTimeout(BaseException):
    pass


def _alarm(_sig, _frm):
    raise _ItemTimeout()


def _gpu_live() -> bool:
    torch = sys.modules.get('torch')
    try:
        if torch is not None and torch.cuda.is_initialized():
            return True
    except Exception:   # noqa: BLE001
        return True
    lib = sys.modules.get('pdeval._lib')
    return bool(lib is not None and getattr(lib, 'CONTEXTS_CREATED', 0))


def _call_bounded(fn, x, item_timeout, default):
    """fn(x), or ``default`` after ``item_timeout`` seconds.  On the main thread the bound is
    SIGALRM (raised as ``_ItemTimeout``, a BaseException SymPy cannot swallow); the previous
    SIGALRM handler and interval timer are restored afterwards.  On any other thread (the
    worker's pipeline threads, when the pool is not running) fn runs on a helper daemon thread
    that is abandoned at the bound: the caller gets ``default`` in time, and the abandoned
    call finishes (or not) on its own without holding anything the caller needs."""
    if not item_timeout:
        return fn(x)
    if threading.current_thread() is not threading.main_thread():
        return _call_on_thread(fn, x, item_timeout, default)
    old = signal.signal(signal.SIGALRM, _alarm)
    prev = signal.setitimer(signal.ITIMER_REAL, float(item_timeout))
    t0 = time.monotonic()
    try:
        try:
            r = fn(x)
        finally:
            # disarmed inside the try: a timer that fires between fn's return and here still
            # lands in the handler below, never in the caller
            signal.setitimer(signal.ITIMER_REAL, 0)
        return r
    except _ItemTimeout:
        return default
    finally:
        signal.signal(signal.SIGALRM, old)
        if prev[0] > 0:
            # an outer timer keeps its deadline: re-armed with what is left of it
            signal.setitimer(signal.ITIMER_REAL, max(prev[0] - (time.monotonic() - t0), 1e-3), prev[1])


_ABANDONED: List[threading.Thread] = []
MAX_ABANDONED = 4     # bounded calls left running past their bound, at most (they hold the GIL)


def _call_on_thread(fn, x, item_timeout, default):
    # once MAX_ABANDONED timed-out calls are still running, further items take their default
    # without starting another thread that would compete for the GIL with the pipeline threads
    _ABANDONED[:] = [t for t in _ABANDONED if t.is_alive()]
    if len(_ABANDONED) >= MAX_ABANDONED:
        return default
    box = []

    def body():
        try:
            box.append((True, fn(x)))
        except BaseException as e:   # noqa: BLE001  (re-raised in the caller)
            box.append((False, e))

    t = threading.Thread(target=body, daemon=True, name='pdeval-bounded')
    t.start()
    t.join(float(item_timeout))
    if not box:
        _ABANDONED.append(t)
        return default
    ok, v = box[0]
    if not ok:
        raise v
    return v


_CANCEL_SLOTS = 4096    # ring of per-job cancel flags shared with the children (job % slots)


def _child(tasks, results, cancelled=None):
    # children: SymPy only (no GPU, no threads of their own); the SymPy side is imported here,
    # once per child, not inside the first batch that reaches it.  A job the parent gave up on
    # (its deadline passed) is flagged in ``cancelled``: its chunks still queued are answered
    # with the default at once instead of running ahead of the next jobs.
    os.environ['OMP_NUM_THREADS'] = '1'
    signal.signal(signal.SIGINT, signal.SIG_IGN)
    from . import problem_defs   # noqa: F401  (sympy, the flattener, the problems' locals)
    from . import batch          # noqa: F401
    while True:
        msg = tasks.get()
        if msg is None:
            return
        job, k, fn, items, item_timeout, default = msg
        try:
            out = []
            for x in items:
                if cancelled is not None and cancelled[job % _CANCEL_SLOTS]:
                    out.append(default)
                    continue
                try:
                    out.append(_call_bounded(fn, x, item_timeout, default))
                except _ItemTimeout:     # (a late timer: the item counts as timed out)
                    out.append(default)
            results.put((job, k, True, out))
        except Exception as e:   # noqa: BLE001  (the parent recomputes the chunk in-process)
            results.put((job, k, False, repr(e)))


class _FixedPool:
    """``n`` forked SymPy processes that are never replaced.  Jobs from several threads may be
    in flight at once: a collector thread routes each result to its job."""

    def __init__(self, n: int):
        ctx = mp.get_context('fork')
        self.n = n
        self.tasks = ctx.Queue()
        self.results = ctx.Queue()
        self.cancelled = ctx.RawArray('b', _CANCEL_SLOTS)
        self.procs = [ctx.Process(target=_child, args=(self.tasks, self.results, self.cancelled), daemon=True)
                      for _ in range(n)]
        for p in self.procs:
            p.start()
        self.broken = False
        self.overdue = 0                     # jobs that hit their deadline (map_chunks)
        self.job = 0
        self.lock = threading.Lock()
        self.inbox = {}                      # job -> queue.Queue of (k, ok, out)
        self.futures = {}                    # job -> (Future, deadline, default): submit()
        self._stop = False
        self.collector = threading.Thread(target=self._collect, daemon=True)
        self.collector.start()

    def _collect(self):
        while not self._stop:
            try:
                j, k, ok, out = self.results.get(timeout=0.5)
            except _queue.Empty:
                if not self._stop and not all(p.is_alive() for p in self.procs):
                    self._break()
                    return
                self._expire()
                continue
            except (EOFError, OSError):
                return
            with self.lock:
                box = self.inbox.get(j)
                fut = self.futures.pop(j, None)
            if box is not None:
                box.put((k, ok, out))
            elif fut is not None and not fut[0].done():
                fut[0].set_result(out[0] if ok else fut[2])
            self._expire()

    def _expire(self):
        """submit()'s futures past their deadline (a child stuck in a C-level call that SIGALRM
        cannot interrupt) resolve to their default."""
        now = time.monotonic()
        with self.lock:
            late = [j for j, (_f, dl, _d) in self.futures.items() if dl is not None and now > dl]
            got = [self.futures.pop(j) for j in late]
        for j in late:
            self.cancelled[j % _CANCEL_SLOTS] = 1
        for f, _dl, d in got:
            if not f.done():
                self.overdue += 1
                f.set_result(d)

    def submit(self, fn, x, item_timeout=None, default=None) -> cf.Future:
        """fn(x) in a child, as a Future (resolved by the collector thread): the streaming
        callers' form of map_chunks.  With an ``item_timeout`` the item yields ``default`` at its
        bound in the child, and the Future resolves to ``default`` at a deadline that counts
        the items queued before it (spread over the children) plus a margin."""
        fut: cf.Future = cf.Future()
        with self.lock:
            if self.broken:
                fut.set_result(default)
                return fut
            self.job += 1
            job = self.job
            self.cancelled[job % _CANCEL_SLOTS] = 0
            dl = None
            if item_timeout:
                ahead = len(self.futures) + 1
                dl = time.monotonic() + float(item_timeout) * (ahead / max(1, self.n) + 1) + DEADLINE_MARGIN_S
            self.futures[job] = (fut, dl, default)
        self.tasks.put((job, 0, fn, [x], item_timeout, default))
        return fut

    def map_chunks(self, fn, chunks, item_timeout=None, default=None) -> list:
        """Per chunk: its result list, or None where the pool could not deliver it (a child
        died, or fn raised in the child); the caller computes those in-process.  With an
        ``item_timeout`` the whole job has a deadline (every item at its bound, spread over the
        children, plus the longest chunk and a margin): a chunk still missing then -- a child
        stuck in a C-level call that SIGALRM cannot interrupt -- yields ``default`` per item
        (the device's verdict stands) instead of blocking the caller."""
        deadline = None
        if item_timeout:
            n_items = sum(len(c) for c in chunks)
            longest = max((len(c) for c in chunks), default=0)
            deadline = time.monotonic() + float(item_timeout) * (n_items / max(1, self.n) + longest) + DEADLINE_MARGIN_S
        with self.lock:
            if self.broken:
                return [None] * len(chunks)
            self.job += 1
            job = self.job
            self.cancelled[job % _CANCEL_SLOTS] = 0
            box = self.inbox[job] = _queue.Queue()
        try:
            for k, ch in enumerate(chunks):
                self.tasks.put((job, k, fn, ch, item_timeout, default))
            got = {}
            while len(got) < len(chunks):
                try:
                    k, ok, out = box.get(timeout=0.5)
                except _queue.Empty:
                    if self.broken:
                        break
                    if deadline is not None and time.monotonic() > deadline:
                        self.overdue += 1
                        # its chunks still queued yield the default in the children at once
                        self.cancelled[job % _CANCEL_SLOTS] = 1
                        return [got[k] if k in got else [default] * len(chunks[k]) for k in range(len(chunks))]
                    continue
                got[k] = out if ok else None
            return [got.get(k) for k in range(len(chunks))]
        finally:
            with self.lock:
                self.inbox.pop(job, None)

    def _break(self):
        self.broken = True
        self.close(graceful=False)
        with self.lock:
            got = list(self.futures.values())
            self.futures.clear()
        for f, _dl, d in got:      # (a dead child: the streaming callers keep the default)
            if not f.done():
                f.set_result(d)

    def close(self, graceful: bool = True):
        if graceful and not self.broken:
            for _ in self.procs:
                self.tasks.put(None)
            for p in self.procs:
                p.join(timeout=5)
        self._stop = True
        for p in self.procs:
            if p.is_alive():
                p.terminate()
                p.join(timeout=5)


def pool_size(local_workers: int = 1) -> int:
    """The box's host-thread share divided among the GPU workers of this host (one SymPy pool
    per worker), less one for the worker's own thread."""
    from .native import host_threads
    return max(1, host_threads() // max(1, local_workers) - 1)


def start(procs: Optional[int] = None, local_workers: Optional[int] = None):
    """Start the pool (idempotent).  Returns it, or None when the GPU is already live in this
    process (the callers then run their SymPy work in-process).  ``local_workers``: GPU
    workers sharing this host (default: LOCAL_WORLD_SIZE, else 1)."""
    global _POOL
    if _POOL is not None and not _POOL.broken:
        return _POOL
    if _gpu_live():
        return None
    if local_workers is None:
        local_workers = int(os.environ.get('LOCAL_WORLD_SIZE', '1') or 1)
    n = procs if procs is not None else pool_size(local_workers)
    _POOL = _FixedPool(n)
    return _POOL


def stop():
    global _POOL
    if _POOL is not None:
        _POOL.close()
        _POOL = None


def active() -> bool:
    return _POOL is not None and not _POOL.broken


def run(fn, items, min_items: int = 8, item_timeout: Optional[float] = None, default=None) -> list:
    """``[fn(x) for x in items]`` over the pool when it runs (order kept; ``fn`` a module-level
    function of picklable arguments), else in-process.  For the per-candidate SymPy checks
    of the host steps (pdeval.batch).  ``item_timeout``: seconds per item, after which the item
    yields ``default`` (in the pool; in-process only on the main thread)."""
    items = list(items)
    if not active() or len(items) < min_items:
        return [_call_bounded(fn, x, item_timeout, default) for x in items]
    k = max(1, min(_POOL.n * 2, len(items)))
    step = (len(items) + k - 1) // k
    chunks = [items[i:i + step] for i in range(0, len(items), step)]
    parts = _POOL.map_chunks(fn, chunks, item_timeout, default)
    out: list = []
    for ch, part in zip(chunks, parts):
        out.extend(part if part is not None else [_call_bounded(fn, x, item_timeout, default) for x in ch])
    return out


_LOCAL = None      # submit() without the pool: a few helper threads (SymPy holds the GIL anyway)


def submit(fn, x, item_timeout: Optional[float] = None, default=None) -> cf.Future:
    """fn(x) as a Future: in a pool child when the pool runs (``_FixedPool.submit``), else on a
    small in-process thread pool, bounded by ``item_timeout`` as ``run`` bounds it off the main
    thread.  For the streaming strict mode (pdeval.worker): items resolve as they finish."""
    global _LOCAL
    if active():
        return _POOL.submit(fn, x, item_timeout, default)
    if _LOCAL is None:
        _LOCAL = cf.ThreadPoolExecutor(max_workers=2, thread_name_prefix='pdeval-submit')
    return _LOCAL.submit(_call_bounded, fn, x, item_timeout, default)


def _compile_chunk(args):
    slug, strings = args
    from . import problem_defs as P
    ops, off, notes = P.compile_strings(P.get(slug), strings)
    return np.asarray(ops, dtype=np.int32), np.asarray(off, dtype=np.int64), notes


def compile_strings(pd_, strings: Sequence[str]):
    """problem_defs.compile_strings over the pool when it runs (chunks in order), else
    in-process.  Same (ops, offsets, notes)."""
    from . import problem_defs as P
    strings = list(strings)
    # (even one string: SymPy parses a declined string in ~1 ms holding the GIL, which the
    # worker's other pipeline threads need; the pool round trip is cheaper than that stall)
    if not active() or not strings:
        return P.compile_strings(pd_, strings)
    k = max(1, min(_POOL.n * 2, (len(strings) + 1) // 2))
    step = (len(strings) + k - 1) // k
    args = [(pd_.slug, strings[i:i + step]) for i in range(0, len(strings), step)]
    parts = [p[0] if p is not None else _compile_chunk(a)
             for a, p in zip(args, _POOL.map_chunks(_compile_chunk, [[a] for a in args]))]
    ops_l: List[np.ndarray] = []
    offs = [np.zeros(1, dtype=np.int64)]
    notes: List[Optional[str]] = []
    base = 0
    for ops, off, nt in parts:
        ops_l.append(ops)
        offs.append(off[1:] + base)
        base += int(off[-1])
        notes.extend(nt)
    return np.concatenate(ops_l) if ops_l else np.zeros(0, np.int32), np.concatenate(offs), notes
