"""The benchmark workloads of BASELINE.json's configs, built from the committed program tables
(SURVEY.md §8d), and the per-rank plan of the sharded run.

One code path for ``bench.py``, the full-size ``-m gpu`` config tests and the multi-rank CPU
tests, so that what the tests check is what the bench times:

* :func:`load_programs` -- a compiled program table under ``data/`` (the candidates of the
  reference's stream that reach ``validate``: ``general_method_paper_reproduction.py:1253-1294``);
* :func:`tiled_indices` -- the C3/C4 batches: the table tiled to ``total`` candidates and
  shuffled with seed 0 (C4, the depth-5-sized batch, is 2**24 candidates over 8 GPUs);
* :func:`gather_programs` -- the packed programs of an index list;
* :func:`flops_per_program` -- the FLOP model of every program (``pdeval_program_flops``),
  which balances the shards;
* :func:`rank_plan` -- this rank's contiguous shard of the batch (``shard.shard_ranges``);
* :func:`assemble_bits` -- the global verdict vector from the per-rank packed bitmaps as the
  all-gather leaves them (``world x nbytes``, each rank padded to the largest shard).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from .shard import assemble_bits, padded_nbytes, shard_ranges  # noqa: F401 (re-exported)

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DATA = os.path.join(ROOT, 'data')

C4_TOTAL = 1 << 24   # the depth-4 program set tiled to 2^24 over 8 GPUs


def load_programs(name: str):
    """(ops, offsets, exprs) of data/<name>.npz (no pickles)."""
    z = np.load(os.path.join(DATA, name if name.endswith('.npz') else name + '.npz'), allow_pickle=False)
    return z['ops'], z['offsets'], z['exprs']


def tiled_indices(nprog: int, total: int, seed: int = 0, shuffle: bool = True) -> np.ndarray:
    """Program index of every candidate of a batch of `total`: the table repeated in order and
    cut to `total`, then (C3/C4) shuffled with numpy's default_rng(seed)."""
    if nprog <= 0 or total < 0:
        raise ValueError('need nprog > 0 and total >= 0')
    idx = np.tile(np.arange(nprog, dtype=np.int64), (total + nprog - 1) // nprog)[:total]
    if shuffle:
        np.random.default_rng(seed).shuffle(idx)
    return idx


def gather_programs(ops: np.ndarray, offsets: np.ndarray, idx: np.ndarray):
    """Batch of programs idx[...] (contiguous, in order) from a program table."""
    idx = np.asarray(idx, dtype=np.int64)
    lens = (offsets[idx + 1] - offsets[idx]).astype(np.int64)
    new_off = np.zeros(len(idx) + 1, dtype=np.int64)
    np.cumsum(lens, out=new_off[1:])
    starts = np.repeat(offsets[idx] - new_off[:-1], lens)
    starts += np.arange(new_off[-1], dtype=np.int64)
    return ops[starts], new_off


def flops_per_program(problem_id: int, ops: np.ndarray, offsets: np.ndarray, hoisted: bool = False) -> np.ndarray:
    """pdeval_program_flops of every program of a table (FP64 flops per sample point), or with
    hoisted=True pdeval_program_hoist_flops: the part of it the lean passes evaluate once per
    grid row (the hoisted x-only prefix)."""
    from ._lib import load
    lib = load()
    fn = lib.pdeval_program_hoist_flops if hoisted else lib.pdeval_program_flops
    ops = np.ascontiguousarray(ops, dtype=np.int32)
    base = ops.ctypes.data
    return np.array([fn(problem_id, base + 4 * int(offsets[i]), int(offsets[i + 1] - offsets[i]))
                     for i in range(len(offsets) - 1)], dtype=np.float64)


@dataclass
class RankPlan:
    total: int                      # candidates of the global batch
    world: int
    rank: int
    ranges: List[Tuple[int, int]]   # every rank's [start, end) in the global batch
    idx: np.ndarray                 # program index of each of this rank's candidates

    @property
    def n(self) -> int:
        return len(self.idx)


def rank_plan(tiled: np.ndarray, world: int, rank: int, prog_weights=None) -> RankPlan:
    """This rank's contiguous shard of the global batch `tiled` (program indices), balanced by
    the programs' weights (FLOP model) when given, by count otherwise (world 1: everything)."""
    if not 0 <= rank < world:
        raise ValueError('rank out of range')
    w = None if (prog_weights is None or world == 1) else np.asarray(prog_weights)[tiled]
    ranges = shard_ranges(len(tiled), world, weights=w)
    s0, s1 = ranges[rank]
    return RankPlan(len(tiled), world, rank, ranges, tiled[s0:s1])
