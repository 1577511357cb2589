#!/bin/bash
# Round 4, session q: the rotating constraint in its own grid instances (Omega = 0 pass 1 must be
# back at ~134 ms); GPU tests; tier-2 at 2 waves/SIMD (t2w2) A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_q}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
TAG=${T} VARIANTS="t2w2" KERR=1 bash scripts/gpu_ab_ff.sh || exit 5
echo ALL_RC=0
