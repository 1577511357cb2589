#!/bin/bash
# Round 6, session ac: the worker pipeline's GIL switch interval alone (PDEVAL_SWITCH_INTERVAL;
# the interpreter's default is 5 ms), one and two processes, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_ac
for k in 1 2; do
  for sw in 0 0.001 0.0002; do
    PDEVAL_SWITCH_INTERVAL=$sw timeout -k 10 400 python scripts/worker_pool_sweep.py --procs 1,2,4 > gpurun_out/${T}_sweep_sw${sw}_$k.log 2>&1 || exit 6
  done
done
echo ALL_RC=0
