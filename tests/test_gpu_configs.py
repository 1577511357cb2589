"""Every BASELINE.json config on the HIP path, at its full size.

  configs[1]  force_free --max-depth 3, 1 GPU: all 3,687 candidates that reach validate,
              device vs the CPU oracle class for class, and vs the reference's verdicts
  configs[2]  force_free --max-depth 4, 1 GPU: all 142,004 candidates; a seeded 2,000 sample
              vs the oracle, the 7 paper solutions recovered
  configs[3]  force_free --max-depth 5 over 8 GPUs: the C4 batch (the depth-4 program set tiled
              and shuffled, seed 0, to 2^24), cut into 8 FLOP-balanced shards, each shard through
              pdeval_validate_device as its rank runs it, the bitmap assembled the way the
              all-gather leaves it -- equal to the unsharded run, every copy of a program with
              the class of the program's own run, the paper solutions accepted everywhere
  configs[4]  kerr_magnetosphere --max-depth 4 over 8 GPUs: the 1,024,799-candidate stream, the
              same sharded/unsharded/shuffled properties, a seeded sample vs the oracle and the
              reference's depth-4 fixtures
configs[0] (CPU SymPy, depth 2) has no HIP path: the CPU suite and the bench's SymPy leg
cover it.  The shards run one after another on the one GPU of the test box; bench.py runs the
same plan (pdeval.workload) one rank per GPU.
"""
import numpy as np
import pytest

import golden_data as G
import oracle_lib as O
from pdeval import problem_defs as P
from pdeval import workload as W
from pdeval._lib import Context, Outputs
from pdeval.opcodes import CLS_ACCEPT, PROBLEM_FORCE_FREE, PROBLEM_KERR
from pdeval.shard import pack_bits

pytestmark = pytest.mark.gpu


def run_device(ctx, ops, off, want_status=True):
    """One pdeval_validate_device call on HBM-resident inputs: (status, packed verdict bits)."""
    import torch
    dev = torch.device('cuda:0')
    n = len(off) - 1
    d_ops = torch.from_numpy(np.ascontiguousarray(ops, dtype=np.int32)).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(off, dtype=np.int64)).to(dev)
    bits = torch.zeros(((n + 31) // 32) * 4, dtype=torch.uint8, device=dev)
    st = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev) if want_status else None
    d_out = Outputs(bits.data_ptr(), st.data_ptr() if st is not None else None, None, None, None,
                    None, None, None)
    torch.cuda.synchronize(dev)
    stream = torch.cuda.Stream(dev)
    ctx.validate_device(d_ops.data_ptr(), d_ops.numel(), d_off.data_ptr(), n, d_out,
                        stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    out_bits = bits.cpu().numpy()[:(n + 7) // 8]
    out_st = st.cpu().numpy()[:n] if st is not None else None
    del d_ops, d_off, bits, st
    torch.cuda.empty_cache()
    return out_st, out_bits


def sharded(ctx, ops_t, off_t, tiled, world, weights):
    """Run the batch `tiled` (indices into the program table) as `world` ranks would: each
    rank's FLOP-balanced shard through validate_device, then the all-gather's layout
    (world x padded bytes) assembled into the global verdicts.  Returns (status, verdicts)."""
    plans = [W.rank_plan(tiled, world, r, weights) for r in range(world)]
    ranges = plans[0].ranges
    assert ranges[0][0] == 0 and ranges[-1][1] == len(tiled)
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    nb = W.padded_nbytes(ranges)
    gathered = np.zeros(world * nb, dtype=np.uint8)
    status = []
    for p in plans:
        assert np.array_equal(p.idx, tiled[p.ranges[p.rank][0]:p.ranges[p.rank][1]])
        o, f = W.gather_programs(ops_t, off_t, p.idx)
        st, bits = run_device(ctx, o, f)
        gathered[p.rank * nb:p.rank * nb + len(bits)] = bits
        status.append(st)
    return np.concatenate(status), W.assemble_bits(gathered, ranges)


def known_rows(ctx, pd_, ops, off):
    """Indices (into the program table) of the accepted candidates whose fingerprint matches a
    known solution's, by name (pdeval.discovery's match)."""
    from pdeval.discovery import fingerprint_matches
    res = ctx.validate(ops, off)
    kops, koff, _ = P.compile_strings(pd_, list(pd_.known_solutions))
    kres = ctx.validate(kops, koff)
    acc = np.flatnonzero(res['status'] == CLS_ACCEPT)
    hits = fingerprint_matches(res['fingerprint'][acc], kres['fingerprint'])
    return res, {name: acc[hits[:, k]] for k, name in enumerate(pd_.known_solutions.values())}


# ---------------------------------------------------------------- configs[1]
def test_config1_ff_depth3_all_candidates():
    """configs[1]: the 3,687 candidates of the reference's depth<=3 stream that reach validate
    (tests/golden/streams/force_free_d3_validated.txt.gz), compiled by the product path (native
    compiler, SymPy for the strings it declines): device class == oracle class for every one;
    device verdict == reference verdict on every decided d1/d2/d3 fixture among them."""
    from pdeval import native
    from pdeval.batch import symbolic_zero_gradient
    pd_ = P.force_free()
    strings = [r[-1] for r in G.stream('force_free_d3_validated.txt.gz')]
    assert len(strings) == 3687
    ops, off, _ = native.compile_strings(pd_, strings)
    ctx = Context(PROBLEM_FORCE_FREE)
    dev = ctx.validate(ops, off)
    ora = O.validate_mt(PROBLEM_FORCE_FREE, ops, off)
    diff = np.flatnonzero(dev['status'] != ora['status'])
    assert not diff.size, [(strings[i], int(dev['status'][i]), int(ora['status'][i])) for i in diff[:10]]
    symbolic_zero_gradient(pd_, strings, dev)
    where = {s: i for i, s in enumerate(strings)}
    rows = [r for r in G.decided(G.ref_rows('ff_d1.jsonl', 'ff_d2.jsonl', 'ff_d3_s500.jsonl'))
            if r['expr'] in where]
    assert len(rows) == 470          # d1 + d2 + the decided rows of the d3 sample
    mism = [(r['expr'], r['reason']) for r in rows if bool(dev['verdict'][where[r['expr']]]) != r['ok']]
    assert not mism, mism[:10]
    ctx.close()


# ---------------------------------------------------------------- configs[2]
def test_config2_ff_depth4_all_candidates():
    """configs[2]: all 142,004 depth-4 candidates on one GPU: a seeded 2,000 sample equals the
    oracle class for class; the 6 streamable paper solutions are found in the stream and the 7th
    (Hyperbolic) by the direct known-solutions batch (discovery)."""
    from pdeval.discovery import find_known_solutions
    pd_ = P.force_free()
    ops, off, exprs = W.load_programs('force_free_d4_validated')
    assert len(off) - 1 == 142004
    ctx = Context(PROBLEM_FORCE_FREE)
    rec = find_known_solutions(ctx, pd_, ops, off, [str(s) for s in exprs])
    assert rec.n_found == 7, rec.found
    assert sum(1 for v in rec.found.values() if v == 'stream') == 6, rec.found
    sample = np.sort(np.random.default_rng(0).choice(len(off) - 1, 2000, replace=False))
    o, f = W.gather_programs(ops, off, sample)
    dev = ctx.validate(o, f)
    ora = O.validate_mt(PROBLEM_FORCE_FREE, o, f)
    diff = np.flatnonzero(dev['status'] != ora['status'])
    assert not diff.size, [(str(exprs[sample[i]]), int(dev['status'][i]), int(ora['status'][i])) for i in diff[:10]]
    ctx.close()


# ---------------------------------------------------------------- configs[3]
def test_config3_c4_batch_sharded_8_ways():
    """configs[3] (C4): 2^24 candidates, 8 FLOP-balanced shards, assembled
    bitmap == unsharded bitmap, per-program class consistency, paper solutions accepted."""
    pd_ = P.force_free()
    ops, off, _ = W.load_programs('force_free_d4_validated')
    nprog = len(off) - 1
    ctx = Context(PROBLEM_FORCE_FREE)
    uniq, kn = known_rows(ctx, pd_, ops, off)
    stream_names = [k for k, v in kn.items() if v.size]
    assert len(stream_names) == 6, {k: v.size for k, v in kn.items()}
    tiled = W.tiled_indices(nprog, W.C4_TOTAL, seed=0)
    weights = W.flops_per_program(PROBLEM_FORCE_FREE, ops, off)
    st8, v8 = sharded(ctx, ops, off, tiled, 8, weights)
    # every copy of a program has the class of the program's own run
    bad = np.flatnonzero(st8 != uniq['status'][tiled])
    assert not bad.size, (bad.size, [(int(tiled[i]), int(st8[i]), int(uniq['status'][tiled[i]])) for i in bad[:10]])
    assert np.array_equal(v8, st8 == CLS_ACCEPT)
    # the streamable paper solutions: accepted wherever they occur in the batch
    for name in stream_names:
        where = np.isin(tiled, kn[name])
        assert where.any() and v8[where].all(), name
    # the unsharded batch (one rank): the same bitmap
    o, f = W.gather_programs(ops, off, tiled)
    _, bits1 = run_device(ctx, o, f, want_status=False)
    del o, f
    assert np.array_equal(bits1, pack_bits(v8))
    ctx.close()


# ---------------------------------------------------------------- configs[4]
def test_config4_kerr_depth4_stream_sharded():
    """configs[4]: the Kerr depth<=4 stream (1,024,799 candidates) sharded 8 ways == unsharded
    == the stream shuffled (seed 0), class for class; a seeded 2,000 sample == the oracle; the
    reference's depth-4 fixtures (kerr_d4_s2000 + kerr_d4_accepts) get the reference verdict."""
    ops, off, exprs = W.load_programs('kerr_magnetosphere_d4_stream')
    nprog = len(off) - 1
    assert nprog == 1024799
    ctx = Context(PROBLEM_KERR)
    st1, bits1 = run_device(ctx, ops, off)
    weights = W.flops_per_program(PROBLEM_KERR, ops, off)
    st8, v8 = sharded(ctx, ops, off, np.arange(nprog, dtype=np.int64), 8, weights)
    assert np.array_equal(st8, st1)
    assert np.array_equal(pack_bits(v8), bits1)
    perm = W.tiled_indices(nprog, nprog, seed=0)
    o, f = W.gather_programs(ops, off, perm)
    stp, _ = run_device(ctx, o, f)
    del o, f
    assert np.array_equal(stp, st1[perm])
    sample = np.sort(np.random.default_rng(0).choice(nprog, 2000, replace=False))
    o, f = W.gather_programs(ops, off, sample)
    ora = O.validate_mt(PROBLEM_KERR, o, f)
    diff = np.flatnonzero(st1[sample] != ora['status'])
    assert not diff.size, [(str(exprs[sample[i]]), int(st1[sample[i]]), int(ora['status'][i])) for i in diff[:10]]
    where = {str(s): i for i, s in enumerate(exprs)}
    rows = [r for r in G.decided(G.ref_rows('kerr_d4_s2000.jsonl', 'kerr_d4_accepts.jsonl'))
            if r['expr'] in where]
    assert len(rows) == 2237
    mism = [(r['expr'], r['reason'][:60], int(st1[where[r['expr']]])) for r in rows
            if bool(st1[where[r['expr']]] == CLS_ACCEPT) != r['ok']]
    assert not mism, mism[:10]
    ctx.close()
