#!/bin/bash
# Round 5, session e: the worker-test list-check failure with the call state in the message;
# device-output fixtures; then the GPU tests again.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_e}
timeout -k 10 300 python -u tests/golden/gen_device_outputs.py > gpurun_out/${T}_devrows.log 2>&1 || exit 3
mkdir -p gpurun_out/device && cp tests/golden/device/*.npz gpurun_out/device/
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
echo ALL_RC=0
