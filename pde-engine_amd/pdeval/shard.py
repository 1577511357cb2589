"""Candidate sharding across GPUs and the one exchange step.

The reference's only parallelism is N validator processes pulling ``(expr_id, expr_str)``
from one ``multiprocessing.Queue`` (``general_method_paper_reproduction.py:773-823``).  Here a
batch is split into contiguous ranges, one per rank (one process per GPU), balanced by the
programs' FLOP model; every rank validates its range with no data-path communication, and the
packed verdict bitmaps are then assembled on every rank with a single all-gather: natively
through the C ABI (``pdeval_gather_bits``, RCCL over xGMI, :func:`gather_verdicts_native`) or
through ``torch.distributed`` (:func:`gather_verdicts`; gloo in the CPU tests).

What is gathered is the PLUGIN's final verdict, not the device bitmap: the host steps of
``pdeval.batch`` (``apply_host_steps``: the symbolic zero-gradient re-check, the Kerr
structural constant re-check, the Kerr exact point check, the symbolic modes) change verdicts
in BOTH directions -- the zero-gradient and constant re-checks turn True into False, the Kerr
exact point check turns a device point reject into an accept where only the fp64 range caused
it (a_value = 0, exp beyond +-708 at a reference point).  So every rank runs them on its own
shard (:func:`final_verdicts`; they need the candidate strings, which every rank has) and the
re-packed bits go into the one all-gather -- the reference's result is the plugin verdict of
each candidate (``general_method_paper_reproduction.py:1768-1816``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np


def shard_ranges(n: int, world: int, weights: Optional[Sequence[float]] = None) -> List[Tuple[int, int]]:
    """Contiguous [start, end) ranges, one per rank.

    Without weights the counts differ by at most one.  With weights (e.g. program lengths, a
    proxy for FLOPs) the cut points split the cumulative weight evenly instead.
    """
    if world < 1:
        raise ValueError('world must be >= 1')
    if n < 0:
        raise ValueError('n must be >= 0')
    if weights is None:
        base, extra = divmod(n, world)
        bounds = [0]
        for r in range(world):
            bounds.append(bounds[-1] + base + (1 if r < extra else 0))
    else:
        w = np.asarray(weights, dtype=np.float64)
        if w.shape != (n,):
            raise ValueError('weights must have one entry per candidate')
        cum = np.concatenate([[0.0], np.cumsum(w)])
        targets = cum[-1] * np.arange(1, world) / world
        cuts = np.searchsorted(cum, targets, side='left').tolist()
        bounds = [0] + [min(max(c, 0), n) for c in cuts] + [n]
        for i in range(1, len(bounds)):          # keep them monotone
            bounds[i] = max(bounds[i], bounds[i - 1])
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def slice_programs(ops: np.ndarray, offsets: np.ndarray, start: int, end: int):
    """Programs [start, end) of a packed batch as a new packed batch (offsets rebased to 0)."""
    lo, hi = int(offsets[start]), int(offsets[end])
    return ops[lo:hi], (offsets[start:end + 1] - lo).astype(np.int64)


def pack_bits(verdict: np.ndarray) -> np.ndarray:
    """bool[n] -> uint8[ceil(n/8)], bit i of the stream = candidate i (LSB first), as the
    kernel writes ``verdict_bits``."""
    return np.packbits(np.asarray(verdict, dtype=bool), bitorder='little')


def unpack_bits(bits: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(np.asarray(bits, dtype=np.uint8), bitorder='little')[:n].astype(bool)


def padded_nbytes(ranges: Sequence[Tuple[int, int]]) -> int:
    """Bytes each rank contributes to the all-gather: the largest shard's packed bitmap."""
    return max(max(((e - s) + 7) // 8 for s, e in ranges), 1) if ranges else 1


def assemble_bits(gathered: np.ndarray, ranges: Sequence[Tuple[int, int]]) -> np.ndarray:
    """Global bool verdicts from the all-gathered bitmaps (uint8 [world * nbytes], rank r's
    packed bits at r * nbytes, LSB first as the kernel writes them)."""
    nb = padded_nbytes(ranges)
    host = np.asarray(gathered, dtype=np.uint8).reshape(len(ranges), nb)
    return np.concatenate([unpack_bits(host[r], e - s) for r, (s, e) in enumerate(ranges)])


def gather_verdicts(local_bits, ranges: Sequence[Tuple[int, int]], group=None):
    """All-gather the per-rank verdict bitmaps and return the global bool[n] on every rank.

    ``local_bits`` is this rank's packed bitmap (a uint8 torch tensor, on the GPU for RCCL or
    on the CPU for gloo) of at least ceil(count/8) bytes.  Every rank pads to the largest
    shard's byte count so the collective has equal-sized inputs; one ``all_gather_into_tensor``
    (``all_gather`` for backends without it) is the only communication.
    """
    import torch
    import torch.distributed as dist
    world = len(ranges)
    nbytes = padded_nbytes(ranges)
    buf = torch.zeros(nbytes, dtype=torch.uint8, device=local_bits.device)
    k = min(nbytes, local_bits.numel())
    buf[:k] = local_bits.reshape(-1)[:k]
    out = torch.empty(world * nbytes, dtype=torch.uint8, device=local_bits.device)
    if hasattr(dist, 'all_gather_into_tensor') and dist.get_backend(group) != 'gloo':
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        out = torch.cat(parts)
    return assemble_bits(out.cpu().numpy(), ranges)


def init_native_comm(ctx, rank: int, world: int, group=None):
    """Join every rank's libpdeval context into one RCCL communicator: rank 0 draws the
    unique id, torch.distributed carries it to the others (a 128-byte broadcast, once)."""
    import torch.distributed as dist
    from ._lib import comm_unique_id
    box = [comm_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(box, src=0, group=group)
    ctx.comm_init(world, rank, box[0])


def gather_verdicts_native(ctx, local_bits, ranges: Sequence[Tuple[int, int]], stream: int = 0):
    """The same all-gather as :func:`gather_verdicts`, through ``pdeval_gather_bits`` (one
    ``ncclAllGather`` of the padded per-rank bitmaps on the context's communicator).
    ``local_bits`` is this rank's packed bitmap as a uint8 torch tensor on the context's GPU."""
    import torch
    world = len(ranges)
    nbytes = padded_nbytes(ranges)
    buf = torch.zeros(nbytes, dtype=torch.uint8, device=local_bits.device)
    k = min(nbytes, local_bits.numel())
    buf[:k] = local_bits.reshape(-1)[:k]
    out = torch.empty(world * nbytes, dtype=torch.uint8, device=local_bits.device)
    torch.cuda.synchronize(local_bits.device)
    ctx.gather_bits(buf.data_ptr(), nbytes, out.data_ptr(), stream)
    torch.cuda.synchronize(local_bits.device)
    return assemble_bits(out.cpu().numpy(), ranges)


def final_verdicts(pd, kerr, params, n_grid: int, items, r: dict, ops, off, keys=None,
                   symbolic: str = 'off', symbolic_timeout: Optional[float] = None,
                   omega: str = '0') -> np.ndarray:
    """This rank's final (plugin) verdicts: the device outputs ``r`` of its shard (host
    arrays) through ``pdeval.batch.apply_host_steps``; returns bool[n] (``r`` is updated in
    place: ``status``, ``verdict``, and the host steps' non-array entries -- the strict mode's
    ``reason_override`` and ``strict`` statistics).  ``omega`` and ``symbolic_timeout`` are the
    plugin's (``BatchValidator.omega`` / ``.symbolic_timeout``): the symbolic replay runs the
    reference's stage at the same Omega the device used.

    ``keys`` (optional, int[n]): a program id per candidate when the shard repeats programs (the
    bench's tiled batch).  The host steps then run once per distinct program, on its first
    occurrence, and the resulting class is given to every occurrence -- the device's outputs
    are a function of the program alone (bench.py checks that duplicates agree)."""
    from .batch import SYMBOLIC_TIMEOUT_S, apply_host_steps
    from .opcodes import CLS_ACCEPT
    tmo = SYMBOLIC_TIMEOUT_S if symbolic_timeout is None else symbolic_timeout
    st = np.asarray(r['status'])
    n = len(st)
    if 'verdict' not in r:
        r['verdict'] = st == CLS_ACCEPT
    if keys is None:
        apply_host_steps(pd, kerr, params, n_grid, items, r, ops, off, symbolic, tmo, omega)
        return np.asarray(r['verdict'], dtype=bool).copy()
    keys = np.asarray(keys)
    _, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    sub = {k: np.asarray(v)[first] for k, v in r.items() if isinstance(v, np.ndarray) and len(v) == n}
    sub_ops, sub_off = _gather(ops, off, first)
    apply_host_steps(pd, kerr, params, n_grid, [items[i] for i in first], sub, sub_ops, sub_off, symbolic,
                     tmo, omega)
    st[:] = sub['status'][inv]
    r['verdict'] = st == CLS_ACCEPT
    # the host steps' per-candidate extras, mapped back to every occurrence: the row-keyed dicts
    # (reason_override, Kerr evidence; keyed by position in the distinct-program list) and the
    # strict mode's statistics
    for k, v in sub.items():
        if k in ('status', 'verdict') or (isinstance(v, np.ndarray) and len(v) == len(first)):
            continue
        if isinstance(v, dict) and k in ('reason_override', 'evidence'):
            rows = np.nonzero(np.isin(inv, np.fromiter(v.keys(), dtype=np.int64)))[0] if v else []
            r[k] = {int(j): v[int(inv[j])] for j in rows}
        else:
            r[k] = v
    return np.asarray(r['verdict'], dtype=bool).copy()


def _gather(ops, off, idx):
    """Packed programs idx[...] of a packed batch (pdeval.workload.gather_programs)."""
    ops = np.asarray(ops)
    off = np.asarray(off, dtype=np.int64)
    idx = np.asarray(idx, dtype=np.int64)
    lens = off[idx + 1] - off[idx]
    new_off = np.zeros(len(idx) + 1, dtype=np.int64)
    np.cumsum(lens, out=new_off[1:])
    starts = np.repeat(off[idx] - new_off[:-1], lens) + np.arange(new_off[-1], dtype=np.int64)
    return ops[starts].astype(np.int32), new_off
