#!/bin/bash
# Round 5, session h: list checks of the hot list kernels moved to a sanitize pass (no spill);
# runtime list schedule (PDEVAL_LIST_QUEUE / _PARTS): the GPU tests, then same-box A/Bs at
# 2^21: static vs queue chunks of 16 / 64 items; Kerr W = 4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_h}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
L=pde-engine_amd/lib
ab() {  # tag lib problem queue parts
  PDEVAL_LIB=$L/$2 PDEVAL_LIST_QUEUE=$4 PDEVAL_LIST_PARTS=$5 timeout -k 10 300 python bench.py --no-cpu --no-extras \
    --problem $3 --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab ff_static_$r libpdeval.so force_free 0 1 || exit 6
  ab ff_q16_$r libpdeval.so force_free 16 1 || exit 6
  ab ff_q64_$r libpdeval.so force_free 64 1 || exit 6
  ab kerr_static_$r libpdeval.so kerr_magnetosphere 0 1 || exit 6
  ab kerr_q16_$r libpdeval.so kerr_magnetosphere 16 1 || exit 6
  ab kerr_q64_$r libpdeval.so kerr_magnetosphere 64 1 || exit 6
  ab kerr_kw4_$r libpdeval_kw4.so kerr_magnetosphere 0 1 || exit 6
done
echo ALL_RC=0
