#!/bin/bash
# Round 5, session p: hoisted single-coordinate segments (PD_HOIST_SUB): the GPU tests, then
# same-box A/Bs at 2^21 -- the build with segments, the same build with PDEVAL_HOIST_SUB=0, and
# the build compiled without them (libpdeval_nosub.so).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_p
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
L=pde-engine_amd/lib
ab() {  # tag lib problem sub
  PDEVAL_LIB=$L/$2 PDEVAL_HOIST_SUB=$4 timeout -k 10 300 python bench.py --no-cpu --no-extras \
    --problem $3 --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab ff_seg_$r libpdeval.so force_free 1 || exit 6
  ab ff_seg0_$r libpdeval.so force_free 0 || exit 6
  ab ff_nosub_$r libpdeval_nosub.so force_free 1 || exit 6
  ab kerr_seg_$r libpdeval.so kerr_magnetosphere 1 || exit 6
  ab kerr_nosub_$r libpdeval_nosub.so kerr_magnetosphere 1 || exit 6
done
echo ALL_RC=0
