#!/bin/bash
# Round 5, session f: list counters zeroed by a kernel (not a memset node): the GPU tests; the
# default bench; same-box A/Bs of the division-free zero test (FF, Kerr) and Kerr W = 4 / 8.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_f}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || exit 5
L=pde-engine_amd/lib
ab() {  # tag lib problem
  PDEVAL_LIB=$L/$2 timeout -k 10 300 python bench.py --no-cpu --no-extras --problem $3 --steps 10 --n 1048576 \
    > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab ff_def_$r libpdeval.so force_free || exit 6
  ab ff_nodiv_$r libpdeval_nodivfree.so force_free || exit 6
  ab kerr_def_$r libpdeval.so kerr_magnetosphere || exit 6
  ab kerr_nodiv_$r libpdeval_nodivfree.so kerr_magnetosphere || exit 6
  ab kerr_kw4_$r libpdeval_kw4.so kerr_magnetosphere || exit 6
  ab kerr_kw4w3_$r libpdeval_kw4w3.so kerr_magnetosphere || exit 6
  ab kerr_kw8_$r libpdeval_kw8.so kerr_magnetosphere || exit 6
done
echo ALL_RC=0
