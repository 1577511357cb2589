#!/bin/bash
# Round 6, session r: pipeline shapes of the worker pool at 2 processes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python scripts/worker_pool_sweep.py --pipe > gpurun_out/r06_r_worker_sweep.log 2>&1 || exit 6
echo ALL_RC=0
