#!/bin/bash
# Parity tests, then the force-free and Kerr benches for the default library and each variant
# in VARS (pde-engine_amd/lib/libpdeval<v>.so), each step time-limited.
set -o pipefail
mkdir -p gpurun_out/k
export TMPDIR=/tmp
T=${TAG:-x}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/k/${T}_pytest.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
for v in "" ${VARS}; do
  L=pde-engine_amd/lib/libpdeval$v.so
  [ -f $L ] || continue
  PDEVAL_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/k/${T}_ff$v.log 2>&1 || exit 5
  PDEVAL_LIB=$L timeout -k 10 200 python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/k/${T}_kerr$v.log 2>&1 || exit 6
done
echo KERR_DONE
