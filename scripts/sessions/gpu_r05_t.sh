#!/bin/bash
# Round 5, session t: the stack-8 lists split over waves (PD_DEEP_PARTS; PDEVAL_DEEP_PARTS=1 for
# one wave): the GPU tests, then same-box A/Bs at 2^21.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_t
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
ab() {  # tag problem parts
  PDEVAL_DEEP_PARTS=$3 timeout -k 10 300 python bench.py --no-cpu --no-extras \
    --problem $2 --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab kerr_p16_$r kerr_magnetosphere 16 || exit 6
  ab kerr_p1_$r kerr_magnetosphere 1 || exit 6
  ab ff_p16_$r force_free 16 || exit 6
  ab ff_p1_$r force_free 1 || exit 6
done
echo ALL_RC=0
