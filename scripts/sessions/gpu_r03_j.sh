#!/bin/bash
# GPU tests, same-box A/B of the default library against VARIANTS (force-free + Kerr, 2^20),
# the default bench with the drop-in-path extras (no CPU legs) and the worker's host profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03_j}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; ok $rc || exit 4
for v in "" ${VARIANTS:-}; do
  for p in force_free kerr_magnetosphere; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras --problem $p > gpurun_out/${T}${v:+_$v}_$p.log 2>&1 || exit 5
  done
done
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_bench.log 2>&1 || exit 6
timeout -k 10 300 python scripts/profile_worker.py > gpurun_out/${T}_worker_profile.log 2>&1 || exit 7
echo CHAIN_RC=0
