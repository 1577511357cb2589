"""Candidate sharding across GPUs and the one exchange step.

The reference's only parallelism is N validator processes pulling ``(expr_id, expr_str)``
from one ``multiprocessing.Queue`` (``general_method_paper_reproduction.py:773-823``).  Here a
batch is split into contiguous ranges, one per rank (one process per GPU), balanced by the
programs' FLOP model; every rank validates its range with no data-path communication, and the
packed verdict bitmaps are then assembled on every rank with a single all-gather: natively
through the C ABI (``pdeval_gather_bits``, RCCL over xGMI, :func:`gather_verdicts_native`) or
through ``torch.distributed`` (:func:`gather_verdicts`; gloo in the CPU tests).

The gathered bitmap is the DEVICE's verdict, before the host steps of ``pdeval.batch``
(``BatchValidator.host_steps``: the symbolic zero-gradient re-check, the Kerr structural
constant re-check and the Kerr exact point check).  Those steps change verdicts in BOTH
directions: the zero-gradient and constant re-checks turn True into False, but the Kerr exact
point check turns a device point reject into an accept where only fp64 range caused the reject
(a_value = 0, exp beyond +-708 at a reference point).  So the gathered bitmap under-accepts
such Kerr candidates relative to the plugin.  A caller that needs the plugin's verdicts runs
the host steps on its own shard (they need the candidate strings) and gathers the re-packed
bits after (:func:`pack_bits` of the host-stepped verdicts), as ``pdeval.worker`` does per
batch.
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
