#!/bin/bash
# Round 5, session n: tier 2 re-checks only the points tier 1 failed, packed 64 to a batch (ESC_MASK;
# PDEVAL_TIER2_MASK=0 turns it off): the GPU tests, then same-box A/Bs at 2^21.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_n
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
ab() {  # tag problem mask
  PDEVAL_TIER2_MASK=$3 timeout -k 10 300 python bench.py --no-cpu --no-extras \
    --problem $2 --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab ff_m1_$r force_free 1 || exit 6
  ab ff_m0_$r force_free 0 || exit 6
  ab kerr_m1_$r kerr_magnetosphere 1 || exit 6
  ab kerr_m0_$r kerr_magnetosphere 0 || exit 6
done
echo ALL_RC=0
