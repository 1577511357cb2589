#!/usr/bin/env python3
"""Where the worker's host time goes (GPU box): process_batches over the 142,004 validated
force-free d4 strings under cProfile, plus the stage totals of one un-pipelined pass."""
import cProfile
import gzip
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))


def main():
    import numpy as np
    from pdeval import hostpool
    hostpool.start()          # the SymPy pool, forked before the GPU is touched (as the worker does)
    from problems import load_problem
    from pdeval.worker import KnownSolutionTagger, filtered_kwargs, process_batches, _results
    with gzip.open(os.path.join(ROOT, 'tests', 'golden', 'streams', 'force_free_d4_validated.txt.gz'), 'rt') as f:
        strs = [l.rstrip('\n').split('\t')[-1] for l in f]
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger(prob, locs)
    kw = filtered_kwargs(prob.validator)
    items = [(i + 1, s) for i, s in enumerate(strs)]
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    list(process_batches([items[:4096]], prob.validator, kw, locs, tagger))   # warm
    # stage totals, one batch at a time
    bv = prob.validator._validator()
    st = {'prepare': 0.0, 'device': 0.0, 'finish': 0.0, 'results': 0.0}
    for k in range(0, len(items), b):
        c = items[k:k + b]
        t0 = time.perf_counter(); p = bv.prepare_strings([s for _, s in c]); t1 = time.perf_counter()
        r = bv.run_prepared(p); t2 = time.perf_counter()
        t = bv.finish(p, r); t3 = time.perf_counter()
        _results(c, p, t, locs, tagger); t4 = time.perf_counter()
        st['prepare'] += t1 - t0; st['device'] += t2 - t1; st['finish'] += t3 - t2; st['results'] += t4 - t3
    print('stage seconds (batch %d):' % b, {k: round(v, 4) for k, v in st.items()})
    # the host steps and the tuples alone (what holds the GIL in the pipeline), by function
    done = []
    for k in range(0, len(items), b):
        c = items[k:k + b]
        p = bv.prepare_strings([s for _, s in c])
        done.append((c, p, bv.run_prepared(p)))
    pr = cProfile.Profile()
    pr.enable()
    for c, p, r in done:
        _results(c, p, bv.finish(p, r), locs, tagger)
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(25)
    # pipeline shapes (depth, compile threads), no profiler; the first is process_batches' default
    for depth, comp in ((8, 4), (12, 6), (16, 8)):
        t0 = time.perf_counter()
        n = sum(len(r) for r in process_batches((items[k:k + b] for k in range(0, len(items), b)),
                                                prob.validator, kw, locs, tagger, depth=depth, compilers=comp))
        dt = time.perf_counter() - t0
        print(f'pipelined depth {depth} compilers {comp}: {n} rows in {dt:.3f} s = {n / dt:.0f} cand/s')
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    n = sum(len(r) for r in process_batches((items[k:k + b] for k in range(0, len(items), b)), prob.validator,
                                            kw, locs, tagger))
    pr.disable()
    dt = time.perf_counter() - t0
    print(f'pipelined: {n} rows in {dt:.3f} s = {n / dt:.0f} cand/s (under cProfile)')
    pstats.Stats(pr).sort_stats('cumulative').print_stats(30)


if __name__ == '__main__':
    main()
