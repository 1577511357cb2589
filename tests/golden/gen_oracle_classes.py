#!/usr/bin/env python3
"""Golden class vectors of the full-size workloads (test infrastructure; CPU only).

Runs the CPU oracle (oracle/jet_oracle.c, tests/oracle_lib.py) over every program of a
committed program table (data/<name>.npz) and stores, per candidate, its class, n_bad and
n_nonfinite, with the sha256 of the table they belong to:

    tests/golden/oracle/<name>.npz     status (u8), n_bad (i32), n_nonfinite (i32), table_sha256

The GPU tests (tests/test_gpu_configs.py) compare the device's classes with these for all
142,004 force-free depth-4 candidates (configs[2], and per program the 2^24 C4 batch of
configs[3]) and all 1,024,799 Kerr depth<=4 candidates (configs[4]) -- sizes the oracle
cannot run inside a test (~15 CPU-minutes for the Kerr stream on 7 threads).

    python tests/golden/gen_oracle_classes.py force_free_d4_validated 0
    python tests/golden/gen_oracle_classes.py kerr_magnetosphere_d4_stream 1
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def table_sha256(ops, offsets) -> str:
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(ops, dtype=np.int32).tobytes())
    h.update(np.ascontiguousarray(offsets, dtype=np.int64).tobytes())
    return h.hexdigest()


def main():
    import oracle_lib as O
    from pdeval import workload as W
    name, pid = sys.argv[1], int(sys.argv[2])
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    ops, off, _ = W.load_programs(name)
    t0 = time.time()
    r = O.validate_mt(pid, ops, off, threads=threads)
    out = os.path.join(HERE, 'oracle', name + '.npz')
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.savez_compressed(out, status=r['status'], n_bad=r['n_bad'], n_nonfinite=r['n_nonfinite'],
                        table_sha256=np.array(table_sha256(ops, off)))
    print(f'{name}: {len(off) - 1} candidates in {time.time() - t0:.0f} s, classes',
          np.bincount(r['status'], minlength=8).tolist(), '->', out)


if __name__ == '__main__':
    main()
