#!/bin/bash
# Round 4, session o: rotating field lines (Omega != 0) through every tier; GPU tests; the
# benches (Omega = 0 must be unchanged).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_o}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/${T}_ff.log 2>&1 || exit 5
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_kerr.log 2>&1 || exit 6
echo ALL_RC=0
