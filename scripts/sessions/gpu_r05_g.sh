#!/bin/bash
# Round 5, session g: dynamic work queues + 4 parts per candidate in the list passes (pass 2,
# complex, tier 2): the GPU tests, then same-box A/Bs at the bench size (2^21): list parts 4
# (default) / 1 / 8, and Kerr W = 4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_g}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
L=pde-engine_amd/lib
ab() {  # tag lib problem
  PDEVAL_LIB=$L/$2 timeout -k 10 300 python bench.py --no-cpu --no-extras --problem $3 --steps 10 \
    > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab ff_def_$r libpdeval.so force_free || exit 6
  ab ff_lp1_$r libpdeval_lp1.so force_free || exit 6
  ab ff_lp8_$r libpdeval_lp8.so force_free || exit 6
  ab kerr_def_$r libpdeval.so kerr_magnetosphere || exit 6
  ab kerr_lp1_$r libpdeval_lp1.so kerr_magnetosphere || exit 6
  ab kerr_lp8_$r libpdeval_lp8.so kerr_magnetosphere || exit 6
  ab kerr_kw4_$r libpdeval_kw4.so kerr_magnetosphere || exit 6
done
echo ALL_RC=0
