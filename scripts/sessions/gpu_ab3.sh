#!/bin/bash
# Same-box A/B of library builds: the GPU tests on the default library, then force-free and
# Kerr benches (2^20 candidates, 3 timed steps) for the default library and each variant named
# in VARIANTS (pde-engine_amd/lib/libpdeval_<v>.so, e.g. the previous commit's build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-ab}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; ok $rc || exit 4
for v in "" ${VARIANTS:-}; do
  lib=pde-engine_amd/lib/libpdeval${v:+_$v}.so
  for p in force_free kerr_magnetosphere; do
    PDEVAL_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras --problem $p > gpurun_out/${T}${v:+_$v}_$p.log 2>&1 || exit 5
  done
done
echo AB_DONE
