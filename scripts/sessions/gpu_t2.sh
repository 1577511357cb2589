#!/bin/bash
# Parity tests (full, not -x), then the force-free and Kerr benches of the default library.
set -o pipefail
mkdir -p gpurun_out/t
export TMPDIR=/tmp
T=${TAG:-x}
timeout -k 10 400 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t/${T}_pytest.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/t/${T}_ff.log 2>&1 || exit 5
timeout -k 10 200 python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/t/${T}_kerr.log 2>&1 || exit 6
echo T2_DONE
