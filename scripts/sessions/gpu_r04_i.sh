#!/bin/bash
# Round 4, session i: GPU tests, worker pipeline shapes, A/B of the reciprocal-based scaled
# residual (fsc) on both problems, the inline split; then the PMC + kernel-trace chain.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_i}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 400 python scripts/profile_worker.py 4096 > gpurun_out/${T}_worker_profile.log 2>&1 || exit 7
timeout -k 10 300 python scripts/profile_inline.py --n 2000 > gpurun_out/${T}_inline.log 2>&1 || exit 9
TAG=${T} VARIANTS="fsc" KERR=1 bash scripts/gpu_ab_ff.sh || exit 8
TAG=r04_p bash scripts/gpu_r04_p.sh > gpurun_out/r04_p_chain.log 2>&1 || exit 10
echo ALL_RC=0
