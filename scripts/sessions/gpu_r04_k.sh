#!/bin/bash
# Round 4, session k: the early double-double tier on a side stream (default) against one tier
# after the grid (PDEVAL_DD_EARLY=0): GPU tests, both benches, the device call by batch size,
# the inline split, the worker.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_k}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/${T}_ff.log 2>&1 || exit 5
PDEVAL_DD_EARLY=0 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/${T}_dd0_ff.log 2>&1 || exit 6
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_kerr.log 2>&1 || exit 7
timeout -k 10 300 python scripts/profile_device_batch.py > gpurun_out/${T}_device_batch.log 2>&1 || exit 8
timeout -k 10 300 python scripts/profile_inline.py --n 2000 > gpurun_out/${T}_inline.log 2>&1 || exit 9
timeout -k 10 400 python scripts/profile_worker.py 4096 > gpurun_out/${T}_worker_profile.log 2>&1 || exit 10
echo ALL_RC=0
