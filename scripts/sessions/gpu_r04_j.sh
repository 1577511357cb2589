#!/bin/bash
# Round 4, session j: the worker's device call by batch size, the Kerr per-opcode costs, the
# worker pipeline shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_j}
timeout -k 10 300 python scripts/profile_device_batch.py > gpurun_out/${T}_device_batch.log 2>&1 || exit 3
timeout -k 10 300 python scripts/microbench.py --problem kerr_magnetosphere > gpurun_out/${T}_microbench_kerr.log 2>&1 || exit 4
timeout -k 10 400 python scripts/profile_worker.py 4096 > gpurun_out/${T}_worker_profile.log 2>&1 || exit 5
echo ALL_RC=0
