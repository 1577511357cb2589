#!/usr/bin/env python3
"""The drop-in worker pool (bench.py worker_pool: N scripts/worker_child.py processes on one GPU,
each taking every N-th 4,096-row queue batch of the validated force-free d4 strings) under
host-thread settings: PDEVAL_HOST_THREADS (native compile threads per call) and the pipeline's
compile threads / depth (PDEVAL_PIPE_COMPILERS, PDEVAL_PIPE_DEPTH).  One JSON line per setting.
GPU box only.  Usage: python scripts/worker_pool_sweep.py [--procs 2,3,4]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))


def main():
    import bench
    from problems import load_problem
    from pdeval.worker import KnownSolutionTagger, filtered_kwargs, process_batch
    from pdeval.workload import load_programs
    _, _, exprs = load_programs('force_free_d4_validated')
    items = [(i + 1, str(s)) for i, s in enumerate(exprs)]
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger(prob, locs)
    kw = filtered_kwargs(prob.validator)
    ref = [process_batch(items[k:k + 4096], prob.validator, kw, locs, tagger) for k in range(0, len(items), 4096)]
    settings = [({}, 2), ({'PDEVAL_HOST_THREADS': '8'}, 2), ({'PDEVAL_HOST_THREADS': '4'}, 2),
                ({'PDEVAL_HOST_THREADS': '4', 'PDEVAL_PIPE_COMPILERS': '2'}, 2),
                ({'PDEVAL_HOST_THREADS': '8', 'PDEVAL_PIPE_DEPTH': '12'}, 2),
                ({'PDEVAL_HOST_THREADS': '4'}, 3), ({'PDEVAL_HOST_THREADS': '4'}, 4)]
    if '--pipe' in sys.argv:      # pipeline shapes at 2 processes
        settings = [({}, 2), ({'PDEVAL_PIPE_DEPTH': '16', 'PDEVAL_PIPE_COMPILERS': '8'}, 2),
                    ({'PDEVAL_PIPE_DEPTH': '16', 'PDEVAL_PIPE_COMPILERS': '8', 'PDEVAL_HOST_THREADS': '8'}, 2),
                    ({'PDEVAL_PIPE_DEPTH': '12', 'PDEVAL_PIPE_COMPILERS': '6'}, 2),
                    ({'PDEVAL_PIPE_DEPTH': '16', 'PDEVAL_PIPE_COMPILERS': '8'}, 3)]
    if '--procs' in sys.argv:     # only the default host settings, at these process counts
        settings = [({}, int(k)) for k in sys.argv[sys.argv.index('--procs') + 1].split(',')]
    for env, procs in settings:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            r = bench.worker_pool(ref, len(items), 4096, procs)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        print(json.dumps({'env': env, **r}), flush=True)


if __name__ == '__main__':
    main()
