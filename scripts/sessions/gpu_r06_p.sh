#!/bin/bash
# Round 6, session p: the re-entry check (GPU tests, default bench line) after the native
# compiler's structural hash consing, then the worker pool sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit 5
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 6
timeout -k 10 500 python scripts/worker_pool_sweep.py > gpurun_out/${T}_worker_sweep.log 2>&1 || exit 7
echo ALL_RC=0
