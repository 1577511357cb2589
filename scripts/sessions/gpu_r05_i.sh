#!/bin/bash
# Round 5, session i: x-only prefix hoisting (PD_HOIST, runtime PDEVAL_HOIST=0 turns it off):
# the GPU tests, then same-box A/Bs at 2^21: hoist on / off (force-free, Kerr), and the list
# schedule static vs queue chunks of 16.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_i}
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
ab() {  # tag problem hoist queue
  PDEVAL_HOIST=$3 PDEVAL_LIST_QUEUE=$4 timeout -k 10 300 python bench.py --no-cpu --no-extras \
    --problem $2 --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab ff_h1_$r force_free 1 0 || exit 6
  ab ff_h0_$r force_free 0 0 || exit 6
  ab kerr_h1_$r kerr_magnetosphere 1 0 || exit 6
  ab kerr_h0_$r kerr_magnetosphere 0 0 || exit 6
done
ab ff_h1_q16 force_free 1 16 || exit 6
ab kerr_h1_q16 kerr_magnetosphere 1 16 || exit 6
echo ALL_RC=0
