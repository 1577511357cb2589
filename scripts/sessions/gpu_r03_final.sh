#!/bin/bash
# Round-end session: GPU tests, smoke, the default bench (all legs), the Kerr bench, the
# worker's host profile, then a same-box A/B of the force-free bench against VARIANTS.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03_m}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; ok $rc || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 5
timeout -k 10 500 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 7
timeout -k 10 300 python scripts/profile_worker.py > gpurun_out/${T}_worker_profile.log 2>&1 || exit 8
for v in "" ${VARIANTS:-}; do
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras > gpurun_out/${T}_ab${v:+_$v}_force_free.log 2>&1 || exit 9
done
echo CHAIN_RC=0
