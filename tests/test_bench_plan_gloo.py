"""bench.py's multi-GPU plan on the CPU (gloo, world 2 and 4): the C4 batch (the
depth-4 program set tiled and shuffled, seed 0, to 2^24 candidates), each rank's FLOP-balanced
contiguous shard (pdeval.workload.rank_plan, exactly as bench.py cuts it), a per-rank verdict
bitmap, and the one all-gather (pdeval.shard.gather_verdicts, the torch path bench.py checks
the RCCL gather against) assembled on every rank.

There is no GPU here, so the per-rank "engine" is a fixed function of the program index: the
test checks the index arithmetic, the padding of unequal shards and the assembly, which are
the parts of the sharded run that do not depend on the kernels.
"""
import os
import socket

import numpy as np
import pytest

from pdeval import workload as W
from pdeval.opcodes import PROBLEM_FORCE_FREE
from pdeval.shard import gather_verdicts, pack_bits


def _fake_verdict(nprog):
    return (np.arange(nprog, dtype=np.int64) * 2654435761 % 7) < 3


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, total, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        ops, off, _ = W.load_programs('force_free_d4_validated')
        nprog = len(off) - 1
        flops = W.flops_per_program(PROBLEM_FORCE_FREE, ops, off)
        tiled = W.tiled_indices(nprog, total, seed=0)
        plan = W.rank_plan(tiled, world, rank, flops)
        fake = _fake_verdict(nprog)
        local = torch.from_numpy(pack_bits(fake[plan.idx]))
        allv = gather_verdicts(local, plan.ranges)
        ok = bool(np.array_equal(allv, fake[tiled]))
        work = [float(flops[tiled[s:e]].sum()) for s, e in plan.ranges]
        np.save(os.path.join(out_dir, f'rank{rank}.npy'),
                np.array([ok, plan.n, max(work) / (sum(work) / world)], dtype=np.float64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_bench_c4_plan_gloo(tmp_path, world):
    import torch.multiprocessing as mp
    total = W.C4_TOTAL
    mp.spawn(_rank_main, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    rows = [np.load(tmp_path / f'rank{r}.npy') for r in range(world)]
    assert all(r[0] == 1.0 for r in rows)               # every rank assembled the global bitmap
    assert sum(int(r[1]) for r in rows) == total        # the shards cover the batch
    assert max(r[2] for r in rows) < 1.001              # FLOP balance within 0.1 %


def test_rank_plan_edges():
    tiled = W.tiled_indices(5, 13, seed=0)
    assert sorted(np.bincount(tiled).tolist()) == [2, 2, 3, 3, 3]
    p = [W.rank_plan(tiled, 4, r) for r in range(4)]
    assert [q.n for q in p] == [4, 3, 3, 3]
    assert np.array_equal(np.concatenate([q.idx for q in p]), tiled)
    # more ranks than candidates: empty shards, one padded byte each
    p = [W.rank_plan(tiled[:2], 4, r) for r in range(4)]
    assert [q.n for q in p] == [1, 1, 0, 0] and W.padded_nbytes(p[0].ranges) == 1
    v = np.array([1, 0], dtype=bool)
    g = np.zeros(4, dtype=np.uint8)
    g[0], g[1] = pack_bits(v[:1])[0], pack_bits(v[1:])[0]
    assert np.array_equal(W.assemble_bits(g, p[0].ranges), v)
    with pytest.raises(ValueError):
        W.rank_plan(tiled, 2, 2)
    # gather_programs keeps every program word in order
    ops = np.arange(20, dtype=np.int32)
    off = np.array([0, 3, 4, 10, 20], dtype=np.int64)
    o, f = W.gather_programs(ops, off, np.array([2, 0, 2, 3]))
    assert f.tolist() == [0, 6, 9, 15, 25]
    assert o.tolist() == list(range(4, 10)) + [0, 1, 2] + list(range(4, 10)) + list(range(10, 20))
