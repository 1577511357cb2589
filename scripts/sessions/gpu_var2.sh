#!/bin/bash
# Bench (and optionally parity-test) library variants: VARS="_a _b" bash scripts/gpu_var2.sh
set -o pipefail
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for v in ${VARS}; do
  L=pde-engine_amd/lib/libpdeval$v.so
  [ -f $L ] || continue
  if [ -n "$TESTS" ]; then
    PDEVAL_LIB=$L timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/var/pytest$v.log 2>&1
    rc=$?; echo "PYTEST$v=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
  fi
  PDEVAL_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/var/bench$v.log 2>&1 || exit 5
  [ -n "$MICRO" ] && { PDEVAL_LIB=$L timeout -k 10 200 python scripts/microbench.py --n 262144 > gpurun_out/var/micro$v.log 2>&1 || exit 6; }
done
echo VAR_DONE
