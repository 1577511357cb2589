#!/bin/bash
# Round 6, session ab: the worker pipeline with two device lanes (two libpdeval contexts per
# process, PDEVAL_PIPE_DEVICES=2, the new default) against one; worker GPU tests first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_worker.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_worker.log 2>&1 || exit 5
for k in 1 2; do
  PDEVAL_PIPE_DEVICES=1 timeout -k 10 400 python scripts/worker_pool_sweep.py --procs 1,2,4 > gpurun_out/${T}_sweep_lanes1_$k.log 2>&1 || exit 6
  PDEVAL_PIPE_DEVICES=2 timeout -k 10 400 python scripts/worker_pool_sweep.py --procs 1,2,4 > gpurun_out/${T}_sweep_lanes2_$k.log 2>&1 || exit 7
done
PDEVAL_PIPE_DEVICES=3 timeout -k 10 400 python scripts/worker_pool_sweep.py --procs 1,2 > gpurun_out/${T}_sweep_lanes3.log 2>&1 || exit 8
echo ALL_RC=0
