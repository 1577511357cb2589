#!/bin/bash
# Round 4, session h: GPU tests, the worker stage profile at the default queue batch, and a
# same-box A/B of the prefetch-address select (presel = round-3 form), the one-hot group bits
# (oh0) and the epilogue's table reciprocal (erc0) on both problems; the inline per-call split.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_h}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 300 python scripts/profile_worker.py 4096 > gpurun_out/${T}_worker_profile.log 2>&1 || exit 7
timeout -k 10 300 python scripts/profile_inline.py --n 2000 > gpurun_out/${T}_inline.log 2>&1 || exit 9
TAG=${T} VARIANTS="presel oh0 erc0" KERR=1 bash scripts/gpu_ab_ff.sh || exit 8
echo ALL_RC=0
