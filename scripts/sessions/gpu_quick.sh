#!/bin/bash
# Quick GPU iteration: parity tests, the per-opcode microbenchmark, a short bench.
set -o pipefail
mkdir -p gpurun_out/q
export TMPDIR=/tmp
T=${TAG:-x}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q/${T}_pytest.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 200 python scripts/microbench.py --n 262144 > gpurun_out/q/${T}_micro.log 2>&1 || exit 5
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/q/${T}_bench.log 2>&1 || exit 6
echo QUICK_DONE
