#!/bin/bash
# Microbench + bench of library variants (one process per variant, each time-limited).
set -o pipefail
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for v in "" ${VARS:-_c2 _c3 _w3}; do
  L=pde-engine_amd/lib/libpdeval$v.so
  [ -f $L ] || continue
  [ -n "$MICRO" ] && { PDEVAL_LIB=$L timeout -k 10 200 python scripts/microbench.py --n 262144 > gpurun_out/var/micro$v.log 2>&1 || exit 3; }
  PDEVAL_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/var/bench$v.log 2>&1 || exit 4
done
echo VAR_DONE
