"""Native candidate compiler: candidate strings -> programs without SymPy.

The reference parses every normalized candidate with ``sp.sympify(s, locals=...)``
(``general_method_paper_reproduction.py:84-93, :1257, :1767``); this build then lowers the tree
with ``pdeval/flatten.py``.  Together that is ~1 ms per candidate on one core, far below what
one GPU validates.  ``pdeval_compile_batch`` (``csrc/pdcompile.cpp``, host C++ inside
libpdeval.so) restates the SymPy evaluation rules these strings exercise and the lowering, and
*declines* every string outside them; :func:`compile_strings` sends exactly the declined ones
through SymPy, so the result is the program set of ``problem_defs.compile_strings``.

Parity with SymPy is checked structurally (:func:`canonical` against :func:`sympy_canonical`
of ``sympify``'s tree) and by verdicts (tests/test_native_compile.py).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import sympy as sp

from ._lib import PdevalError, load

COMPILE_OK, COMPILE_DECLINED, COMPILE_PARSE = 0, 1, 2


def _pack_text(strings: Sequence[str]) -> Tuple[bytes, np.ndarray]:
    """All strings in one buffer and their byte offsets: one join + encode, the offsets from
    the separators' positions (a string holding the separator itself takes the slow path)."""
    strings = list(strings)
    off = np.zeros(len(strings) + 1, dtype=np.int64)
    if not strings:
        return b'', off
    text = '\n'.join(strings).encode()
    seps = np.flatnonzero(np.frombuffer(text, dtype=np.uint8) == 10)
    if len(seps) != len(strings) - 1:
        enc = [s.encode() for s in strings]
        np.cumsum([len(b) for b in enc], out=off[1:])
        return b''.join(enc), off
    # string i spans [start_i, sep_i): drop the separators from the buffer's offsets
    ends = np.append(seps, len(text))
    starts = np.concatenate([[0], seps + 1])
    lens = ends - starts
    np.cumsum(lens, out=off[1:])
    return text.replace(b'\n', b''), off


def host_threads() -> int:
    """Host threads for the native compile: PDEVAL_HOST_THREADS, else OMP_NUM_THREADS (16 on
    the GPU box, whose os.cpu_count() reports the whole machine), else the affinity mask."""
    for k in ('PDEVAL_HOST_THREADS', 'OMP_NUM_THREADS'):
        v = os.environ.get(k, '')
        if v.isdigit() and int(v) > 0:
            return min(int(v), 64)
    try:
        return max(1, min(len(os.sched_getaffinity(0)), 64))
    except AttributeError:
        return max(1, min(os.cpu_count() or 1, 64))


def compile_native(problem_id: int, strings: Sequence[str], threads: Optional[int] = None):
    """(ops int32, offsets int64[n+1], status int32[n]) from the C++ compiler alone; declined
    and unparsable strings get empty slots (status != COMPILE_OK).  ``threads`` host threads
    (pdeval_compile_batch_mt; default host_threads(), 1 = the single-threaded entry point)."""
    lib = load()
    text, soff = _pack_text(strings)
    n = len(strings)
    nt = host_threads() if threads is None else int(threads)
    cap = 8 * len(text) + 16 * n + 64
    while True:
        ops = np.empty(cap, dtype=np.int32)
        off = np.zeros(n + 1, dtype=np.int64)
        st = np.zeros(n, dtype=np.int32)
        nw = C.c_int64(0)
        tb = C.create_string_buffer(text, len(text) + 1)
        if nt == 1:
            rc = lib.pdeval_compile_batch(problem_id, C.cast(tb, C.c_void_p), soff.ctypes.data, n,
                                          ops.ctypes.data, cap, off.ctypes.data, st.ctypes.data,
                                          C.byref(nw))
        else:
            rc = lib.pdeval_compile_batch_mt(problem_id, C.cast(tb, C.c_void_p), soff.ctypes.data, n,
                                             ops.ctypes.data, cap, off.ctypes.data, st.ctypes.data,
                                             C.byref(nw), nt)
        if rc == 0:
            return ops[:nw.value], off, st
        if nw.value != -1:
            raise PdevalError(f'pdeval_compile_batch failed ({rc})')
        cap *= 2


def compile_strings(pd_, strings: Sequence[str], stats: Optional[dict] = None,
                    threads: Optional[int] = None):
    """Drop-in for ``problem_defs.compile_strings``: native compile, SymPy for the rest.
    Returns (ops, offsets, notes) with notes[i] = None or the reason a program is a stub.
    With a ``stats`` dict, ``stats['status']`` receives the native compiler's per-string
    status (COMPILE_PARSE marks the strings it could not parse)."""
    from .hostpool import compile_strings as sympy_compile   # (the SymPy pool when it runs)
    ops, off, st = compile_native(pd_.problem_id, strings, threads)
    host = np.flatnonzero(st != COMPILE_OK)
    if stats is not None:
        stats.update(n=len(strings), native=int(len(strings) - len(host)), host=int(len(host)), status=st)
    notes: List[Optional[str]] = [None] * len(strings)
    if len(host) == 0:
        return ops, off, notes
    h_ops, h_off, h_notes = sympy_compile(pd_, [strings[i] for i in host])
    for k, i in enumerate(host):
        notes[i] = h_notes[k]
    # splice: lengths per candidate, then one gather
    lens = np.diff(off)
    lens[host] = np.diff(h_off)
    new_off = np.zeros(len(strings) + 1, dtype=np.int64)
    np.cumsum(lens, out=new_off[1:])
    src = np.concatenate([ops, h_ops])
    starts = off[:-1].copy()
    starts[host] = h_off[:-1] + len(ops)
    idx = np.repeat(starts - new_off[:-1], lens) + np.arange(new_off[-1], dtype=np.int64)
    return src[idx].astype(np.int32), new_off, notes


def canonical(problem_id: int, s: str) -> Tuple[int, str]:
    """(status, canonical form of the natively evaluated tree)."""
    lib = load()
    b = s.encode()
    buf = C.create_string_buffer(1 << 16)
    st = lib.pdeval_canonical(problem_id, b, len(b), buf, len(buf))
    if st < 0:
        raise PdevalError('pdeval_canonical: bad argument')
    return st, buf.value.decode()


def sympy_canonical(e: sp.Basic) -> str:
    """The same canonical form computed from a SymPy tree (args sorted as strings)."""
    if e.is_Rational:
        return str(e.p) if e.q == 1 else f'{e.p}/{e.q}'
    if e.is_Symbol:
        return e.name
    if e is sp.E:
        return 'E(1)'
    if e is sp.I:
        return 'I'
    if e.is_Add or e.is_Mul:
        return ('A(' if e.is_Add else 'M(') + ','.join(sorted(sympy_canonical(a) for a in e.args)) + ')'
    if e.is_Pow:
        return f'P({sympy_canonical(e.base)},{sympy_canonical(e.exp)})'
    if isinstance(e, sp.exp):
        return f'E({sympy_canonical(e.args[0])})'
    if isinstance(e, sp.Abs):
        return f'B({sympy_canonical(e.args[0])})'
    return f'?{type(e).__name__}'
