#!/bin/bash
# Round 4, last check of the shipped build: the GPU tests and smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04_check_pytest_gpu.log 2>&1 || exit 4
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_check_smoke.log 2>&1 || exit 3
echo ALL_RC=0
