#!/bin/bash
# Round 5, session s: force-free pass 1 at 4 / 5 (default) / 6 waves per SIMD with the hoisted
# prefixes in (same-box A/B at 2^21, libpdeval_w4.so / libpdeval_w6.so).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_s
L=pde-engine_amd/lib
ab() {  # tag lib
  PDEVAL_LIB=$L/$2 timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab ff_w5_$r libpdeval.so || exit 6
  ab ff_w4_$r libpdeval_w4.so || exit 6
  ab ff_w6_$r libpdeval_w6.so || exit 6
done
echo ALL_RC=0
