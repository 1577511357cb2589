"""Multi-rank path on the CPU: contiguous candidate shards + one all-gather of the verdict
bitmaps (bench.py runs the same code over RCCL, one process per GPU).

world_size 2 on gloo; each rank validates its shard with the CPU oracle (the per-rank engine
stand-in -- there is no GPU here) and the gathered bitmap must equal the one-rank bitmap.
"""
import os
import socket

import numpy as np
import pytest

from pdeval import problem_defs as P
from pdeval.shard import gather_verdicts, pack_bits, shard_ranges, slice_programs, unpack_bits

import golden_data as G


def test_shard_ranges_even():
    assert shard_ranges(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert shard_ranges(2, 4) == [(0, 1), (1, 2), (2, 2), (2, 2)]
    assert shard_ranges(0, 2) == [(0, 0), (0, 0)]
    r = shard_ranges(1 << 20, 8)
    assert r[0] == (0, 131072) and r[-1][1] == 1 << 20


def test_shard_ranges_weighted():
    w = np.array([10, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1], dtype=float)
    r = shard_ranges(len(w), 2, w)
    assert r[0][0] == 0 and r[-1][1] == len(w)
    assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
    assert r[0] == (0, 1)                      # the heavy program alone carries half the work
    with pytest.raises(ValueError):
        shard_ranges(3, 2, [1.0, 2.0])


def test_slice_and_bits_roundtrip():
    pd_ = P.force_free()
    ops, off, _ = P.compile_strings(pd_, ['rho', 'rho*z', 'exp(z)*rho**2', 'sqrt(rho + z**2)'])
    o2, f2 = slice_programs(ops, off, 1, 3)
    assert f2[0] == 0 and f2[-1] == o2.size and len(f2) == 3
    assert np.array_equal(o2, ops[off[1]:off[3]])
    v = np.array([1, 0, 1, 1, 0, 0, 0, 1, 1], dtype=bool)
    assert np.array_equal(unpack_bits(pack_bits(v), len(v)), v)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, strings, out_dir):
    import torch
    import torch.distributed as dist
    import oracle_lib as O
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        pd_ = P.force_free()
        ops, off, _ = P.compile_strings(pd_, strings)
        lens = np.diff(off)
        ranges = shard_ranges(len(strings), world, weights=lens)
        s, e = ranges[rank]
        o, f = slice_programs(ops, off, s, e)
        res = O.validate(0, o, f, O.params(full_grid=0))
        local = torch.from_numpy(pack_bits(res['status'] == 0))
        allv = gather_verdicts(local, ranges)
        np.save(os.path.join(out_dir, f'rank{rank}.npy'), allv)
    finally:
        dist.destroy_process_group()


def test_two_rank_gather_equals_single_rank(tmp_path):
    import torch.multiprocessing as mp
    import oracle_lib as O
    rows = G.ref_rows('ff_d2.jsonl', 'ff_edge.jsonl')
    strings = [r['expr'] for r in rows]
    pd_ = P.force_free()
    ops, off, _ = P.compile_strings(pd_, strings)
    single = O.validate(0, ops, off, O.params(full_grid=0))['status'] == 0
    mp.spawn(_rank_main, args=(2, _free_port(), strings, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        got = np.load(tmp_path / f'rank{r}.npy')
        assert np.array_equal(got, single), r
    assert single.any() and not single.all()


DEVICE_ROWS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'device')


def _device_rows(case):
    """The device's raw outputs for fixture rows, recorded on the MI355X
    (tests/golden/gen_device_outputs.py): the per-rank device results of this CPU test."""
    z = np.load(os.path.join(DEVICE_ROWS, f'{case}.npz'), allow_pickle=False)
    r = {k: z[k] for k in ('status', 'verdict', 'q_ref', 'res_ref', 'q_grid', 'n_bad', 'n_nonfinite', 'fingerprint')}
    return str(z['problem']), [float(v) for v in z['kerr']], [str(s) for s in z['strings']], z['ops'], z['off'], r, z['ref_ok']


def _kerr_of(pid, kerr):
    from pdeval import _lib
    if pid != 1:
        return None
    if kerr:
        k = [int(v) for v in kerr[:4]] + [kerr[4], kerr[5]] + [int(v) for v in kerr[6:]]
        return _lib.KerrConstants(*k)
    return _lib.default_kerr_constants()


def _final_rank_main(rank, world, port, case, out_dir):
    import torch
    import torch.distributed as dist
    from pdeval import _lib
    from pdeval.shard import final_verdicts, _gather
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        problem, kerr, strs, ops, off, r, _ = _device_rows(case)
        pd_ = P.get(problem)
        ranges = shard_ranges(len(strs), world)
        s, e = ranges[rank]
        sub = {k: v[s:e].copy() for k, v in r.items()}
        o, f = _gather(ops, off, np.arange(s, e))
        fin = final_verdicts(pd_, _kerr_of(pd_.problem_id, kerr), _lib.default_params(pd_.problem_id), 4096,
                             strs[s:e], sub, o, f)
        allv = gather_verdicts(torch.from_numpy(pack_bits(fin)), ranges)
        np.save(os.path.join(out_dir, f'{case}_rank{rank}.npy'), allv)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('case', ['kerr_a_value0', 'kerr_d4_range', 'ff_edge_d2'])
def test_two_rank_gather_of_final_verdicts(case, tmp_path):
    """every rank runs the host steps on its own shard of device results
    (pdeval.shard.final_verdicts) and the re-packed FINAL bits are what the all-gather carries.
    With device outputs recorded on the MI355X (tests/golden/gen_device_outputs.py) -- Kerr at
    a_value = 0, where the exact point check re-decides fp64-range point rejects; the Kerr
    depth-4 rows whose class the host steps decide; the force-free symbolic zero-gradient row --
    world 2 on gloo gives exactly the single-process plugin's verdicts (the same host steps over
    the whole batch), which equal the reference's on every decided row, while the raw device
    bitmap does not (force-free)."""
    import torch.multiprocessing as mp
    from pdeval import _lib
    from pdeval.shard import final_verdicts
    problem, kerr, strs, ops, off, r, ref_ok = _device_rows(case)
    pd_ = P.get(problem)
    raw = r['verdict'].astype(bool).copy()
    fin = {k: v.copy() for k, v in r.items()}
    single = final_verdicts(pd_, _kerr_of(pd_.problem_id, kerr), _lib.default_params(pd_.problem_id), 4096, strs,
                            fin, ops, off)
    mp.spawn(_final_rank_main, args=(2, _free_port(), case, str(tmp_path)), nprocs=2, join=True)
    for k in range(2):
        assert np.array_equal(np.load(tmp_path / f'{case}_rank{k}.npy'), single), k
    dec = ref_ok >= 0
    assert np.array_equal(single[dec], ref_ok[dec] == 1), [strs[i] for i in np.flatnonzero(dec & (single != (ref_ok == 1)))][:5]
    if case == 'kerr_a_value0':
        # the exact point check re-decides fp64-range point rejects (class changes; at these
        # constants the grid then rejects them too, so the bits stay)
        assert int((fin['status'] != r['status']).sum()) >= 3
    if case == 'ff_edge_d2':
        assert int((raw & ~single).sum()) >= 1                     # the symbolic zero gradient


_OMEGA_STRS = ['rho**2', 'rho**2*exp(-2*z)', 'z + log(1 - rho**2/9)', 'rho**2/(rho**2 + z**2)**(3/2)']


def _omega_rows(keys):
    """Device-style outputs for _OMEGA_STRS[keys]: every row a grid zero (ACCEPT), distinct
    fingerprint values (no zero-gradient re-check), as the strict / replay modes receive them."""
    from pdeval.opcodes import CLS_ACCEPT
    n = len(keys)
    strs = [_OMEGA_STRS[k] for k in keys]
    ops, off, _ = P.compile_strings(P.force_free(), strs)
    r = {'status': np.full(n, CLS_ACCEPT, dtype=np.uint8), 'verdict': np.ones(n, dtype=bool),
         'q_ref': np.zeros(n), 'res_ref': np.zeros((n, 1)), 'q_grid': np.zeros(n),
         'n_bad': np.zeros(n, dtype=np.int32), 'n_nonfinite': np.zeros(n, dtype=np.int32),
         'fingerprint': (np.arange(4 * n, dtype=np.float64).reshape(n, 4) + 1.0)}
    return strs, ops, off, r


def _omega_rank_main(rank, world, port, keys, out_dir):
    import torch
    import torch.distributed as dist
    from pdeval import _lib
    from pdeval.shard import final_verdicts, _gather
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        strs, ops, off, r = _omega_rows(keys)
        ranges = shard_ranges(len(strs), world)
        s, e = ranges[rank]
        sub = {k: v[s:e].copy() for k, v in r.items()}
        o, f = _gather(ops, off, np.arange(s, e))
        fin = final_verdicts(P.force_free(), None, _lib.default_params(0), 4096, strs[s:e], sub, o, f,
                             keys=np.asarray(keys[s:e]), symbolic='replay', omega='1/3')
        allv = gather_verdicts(torch.from_numpy(pack_bits(fin)), ranges)
        np.save(os.path.join(out_dir, f'omega_rank{rank}.npy'), allv)
    finally:
        dist.destroy_process_group()


def test_final_verdicts_forward_omega(tmp_path):
    """the multi-rank final verdicts replay the reference's symbolic stage at the
    plugin's Omega (BatchValidator.omega), not at 0.  Rotating solutions at Omega = 1/3
    (tests/golden/ref/ff_omega13_known.jsonl: the reference accepts them symbolically) stay
    accepted through final_verdicts(..., omega='1/3') on the keyed (duplicate-program) path,
    equal the single-process apply_host_steps, and the 2-rank gloo gather gives the same bits.
    Bent and Dipolar -- solutions at Omega = 0, rejected by the reference at 1/3 -- are
    rejected by the replay at 1/3 and accepted at 0 (the bug would have accepted them)."""
    import torch.multiprocessing as mp
    from pdeval import _lib
    from pdeval.batch import apply_host_steps
    from pdeval.shard import final_verdicts
    ref = {r['expr']: r['ok'] for r in G.ref_rows('ff_omega13_known.jsonl')}
    assert [ref[s] for s in _OMEGA_STRS] == [True, False, True, False]
    keys = [0, 1, 2, 3, 1, 0, 2, 1]
    prm = _lib.default_params(0)
    strs, ops, off, r = _omega_rows(keys)
    got = final_verdicts(P.force_free(), None, prm, 4096, strs, {k: v.copy() for k, v in r.items()}, ops, off,
                         keys=np.asarray(keys), symbolic='replay', omega='1/3')
    single = {k: v.copy() for k, v in r.items()}
    apply_host_steps(P.force_free(), None, prm, 4096, strs, single, ops, off, 'replay', omega='1/3')
    assert np.array_equal(got, single['verdict'])
    assert got.tolist() == [ref[_OMEGA_STRS[k]] for k in keys]
    at0 = final_verdicts(P.force_free(), None, prm, 4096, strs, {k: v.copy() for k, v in r.items()}, ops, off,
                         keys=np.asarray(keys), symbolic='replay')
    assert at0.all()
    mp.spawn(_omega_rank_main, args=(2, _free_port(), keys, str(tmp_path)), nprocs=2, join=True)
    for k in range(2):
        assert np.array_equal(np.load(tmp_path / f'omega_rank{k}.npy'), got), k
