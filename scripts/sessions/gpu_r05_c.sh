#!/bin/bash
# Round 5, session c: the division-free grid test build -- device-output fixtures, the GPU
# tests, the default bench (with stderr progress), a kernel trace of pass 1.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_c}
timeout -k 10 300 python -u tests/golden/gen_device_outputs.py > gpurun_out/${T}_devrows.log 2>&1 || exit 3
mkdir -p gpurun_out/device && cp tests/golden/device/*.npz gpurun_out/device/
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || exit 4
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || exit 5
echo ALL_RC=0
