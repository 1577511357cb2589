#!/bin/bash
# Round 5, session j: hoisted prefixes of x alone and of y alone (PD_HOIST): the GPU tests
# (with the hoist on / off equality test), then same-box A/Bs at 2^21, hoist on / off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_j}
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
ab() {  # tag problem hoist
  PDEVAL_HOIST=$3 timeout -k 10 300 python bench.py --no-cpu --no-extras \
    --problem $2 --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab ff_h1_$r force_free 1 || exit 6
  ab ff_h0_$r force_free 0 || exit 6
  ab kerr_h1_$r kerr_magnetosphere 1 || exit 6
  ab kerr_h0_$r kerr_magnetosphere 0 || exit 6
done
echo ALL_RC=0
