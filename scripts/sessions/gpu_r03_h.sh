#!/bin/bash
# GPU tests on the default library, then same-box A/B: force-free + Kerr for the default and
# the no-inline variant (dd / tier-2 interpreters as calls), Kerr only for the pass-1 shape
# variants (kw*: grid rows per dispatch, waves per SIMD).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03_h}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; ok $rc || exit 4
for v in "" noinl; do
  for p in force_free kerr_magnetosphere; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras --problem $p > gpurun_out/${T}${v:+_$v}_$p.log 2>&1 || exit 5
  done
done
for v in ${KVARIANTS:-}; do
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval_$v.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_${v}_kerr_magnetosphere.log 2>&1 || exit 6
done
echo AB_DONE
