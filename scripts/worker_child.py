#!/usr/bin/env python3
"""One process of a multi-process worker pool on one GPU (bench.py worker_pool leg): the
reference runs ``--validators N`` validator processes (general_method_paper_reproduction.py
:802-823), each draining the queue; here each process takes every P-th queue batch of the
validated force-free d4 stream and runs the worker's pipeline (pdeval.worker.process_batches)
over them.

Protocol: prints READY once its context, SymPy pool and tagger are warm; waits for one line
on stdin; then prints one JSON line {rows, seconds, t0, t1, digest} where digest is the SHA-256 of the
repr of its result tuples, batch by batch in its own order (over all --passes), computed after
the timed region."""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--part', type=int, required=True)
    ap.add_argument('--parts', type=int, required=True)
    ap.add_argument('--batch', type=int, default=4096)
    ap.add_argument('--passes', type=int, default=1,
                    help='run over its batches this many times (a continuous queue: the pipeline fill once)')
    a = ap.parse_args()
    from pdeval import hostpool
    hostpool.start(local_workers=a.parts)     # forked before this process touches the GPU
    from problems import load_problem
    from pdeval.worker import KnownSolutionTagger, filtered_kwargs, process_batches
    from pdeval.workload import load_programs
    _, _, exprs = load_programs('force_free_d4_validated')
    items = [(i + 1, str(s)) for i, s in enumerate(exprs)]
    mine = [items[k:k + a.batch] for k in range(0, len(items), a.batch)][a.part::a.parts]
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger(prob, locs)
    kw = filtered_kwargs(prob.validator)
    list(process_batches([items[:a.batch]], prob.validator, kw, locs, tagger))   # warm
    print('READY', flush=True)
    sys.stdin.readline()
    n = 0
    got = []
    t0 = time.perf_counter()
    for r in process_batches(iter(mine * a.passes), prob.validator, kw, locs, tagger):
        n += len(r)
        got.append(r)          # (the tuples are handed on, as a worker puts them on its queue)
    dt = time.perf_counter() - t0
    # the check of the tuples, after the timed region: SHA-256 of their repr, batch by batch
    # (round 5 hashed inside the loop -- ~4 ms per 4,096-row batch, a third of the process's time)
    h = hashlib.sha256()
    for r in got:
        h.update(repr(r).encode())
    # t0 / t1: time.perf_counter() (CLOCK_MONOTONIC, one clock for every process of the box), so
    # the parent times the pool from the first start to the last end, without this digest
    print(json.dumps({'rows': n, 'seconds': dt, 't0': t0, 't1': t0 + dt, 'digest': h.hexdigest()}), flush=True)
    hostpool.stop()


if __name__ == '__main__':
    main()
