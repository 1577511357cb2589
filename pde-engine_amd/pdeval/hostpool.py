"""Host process pool for the SymPy work the native compiler leaves (pdeval/native.py).

The native compiler (csrc/pdcompile.cpp) compiles 99.9 % of the candidate strings on host
threads; the few it declines go through SymPy (``sp.sympify`` + ``pdeval.flatten``, ~1.5 ms
each), which holds the GIL.  At the rate one GPU validates, those few dominate the worker's
host time, so they are spread over a pool of SymPy processes -- the reference parallelizes
its SymPy validation over processes the same way (``--validators N``,
``general_method_paper_reproduction.py:1671-1824``).

The pool is FORKED, so it must be started before the process touches the GPU (a fork of a
process whose HIP runtime is live is not safe, and an exec from it is forbidden on the GPU
hosts): :func:`start` refuses once torch has initialized CUDA/HIP or a libpdeval context exists,
and :func:`compile_strings` then compiles in-process, as before.  Children never touch the GPU.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import sys
from typing import List, Optional, Sequence

import numpy as np

_POOL = None
_PROCS = 0


def _gpu_live() -> bool:
    torch = sys.modules.get('torch')
    try:
        if torch is not None and torch.cuda.is_initialized():
            return True
    except Exception:   # noqa: BLE001
        return True
    lib = sys.modules.get('pdeval._lib')
    return bool(lib is not None and getattr(lib, 'CONTEXTS_CREATED', 0))


def _init():
    # children: SymPy only (no GPU, no threads of their own); the SymPy side is imported here,
    # once per child, not inside the first batch that reaches it
    os.environ['OMP_NUM_THREADS'] = '1'
    from . import problem_defs   # noqa: F401  (sympy, the flattener, the problems' locals)
    from . import batch          # noqa: F401


def start(procs: Optional[int] = None):
    """Start the pool (idempotent).  Returns it, or None when the GPU is already live in this
    process (the caller then compiles declined strings in-process)."""
    global _POOL, _PROCS
    if _POOL is not None:
        return _POOL
    if _gpu_live():
        return None
    from .native import host_threads
    n = procs if procs is not None else max(1, host_threads() - 1)
    _POOL = mp.get_context('fork').Pool(n, initializer=_init)
    _PROCS = n
    return _POOL


def stop():
    global _POOL
    if _POOL is not None:
        _POOL.terminate()
        _POOL.join()
        _POOL = None


def run(fn, items, min_items: int = 8) -> list:
    """``[fn(x) for x in items]`` over the pool when it runs (order kept; ``fn`` a module-level
    function of picklable arguments), else in-process.  For the per-candidate SymPy checks
    of the host steps (pdeval.batch.symbolic_zero_gradient, the known-solution tagger)."""
    items = list(items)
    if _POOL is None or len(items) < min_items:
        return [fn(x) for x in items]
    return _POOL.map(fn, items, chunksize=max(1, len(items) // (_PROCS * 2)))


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
    if _POOL is None or len(strings) < 8:
        return P.compile_strings(pd_, strings)
    k = max(1, min(_PROCS * 2, len(strings) // 4))
    step = (len(strings) + k - 1) // k
    parts = _POOL.map(_compile_chunk, [(pd_.slug, strings[i:i + step]) for i in range(0, len(strings), step)])
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
