#!/bin/bash
# Round 6, session j: the speculative provisional double-double tier (PD_DD_SPEC) -- GPU tests,
# the worker batch's device call with it on / off, same-box bench A/B, the worker pool sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_j
timeout -k 10 700 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
for s in 1 0; do
  PDEVAL_DD_SPEC=$s timeout -k 10 300 python scripts/profile_device_batch.py --sizes 1024,4096,16384 --reps 9 > gpurun_out/${T}_device_batch_spec$s.log 2>&1 || exit 6
done
for k in 1 2; do
  for s in 1 0; do
    PDEVAL_DD_SPEC=$s timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_ff_spec${s}_$k.log 2>&1 || exit 7
  done
done
timeout -k 10 400 python scripts/worker_pool_sweep.py > gpurun_out/${T}_worker_sweep.log 2>&1 || exit 8
echo ALL_RC=0
