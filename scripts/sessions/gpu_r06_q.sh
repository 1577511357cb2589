#!/bin/bash
# Round 6, session q: where the worker's host time goes after the compiler speedup (stage
# totals, cProfile), and the pool timed from its children's own clocks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_q
timeout -k 10 300 python scripts/profile_worker.py 4096 > gpurun_out/${T}_profile_worker.log 2>&1 || exit 5
timeout -k 10 400 python scripts/worker_pool_sweep.py --procs 1,2,3,4 > gpurun_out/${T}_worker_sweep.log 2>&1 || exit 6
echo ALL_RC=0
