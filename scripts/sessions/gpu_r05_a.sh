#!/bin/bash
# Round 5, session a: device-output fixtures for the multi-rank final-verdict test, the GPU
# tests (new: Kerr constants vs the small-batch graph, the early double-double split), and the
# restructured bench (final-verdict gather, Kerr sub-record).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_a}
timeout -k 10 300 python -u tests/golden/gen_device_outputs.py > gpurun_out/${T}_devrows.log 2>&1 || exit 3
mkdir -p gpurun_out/device && cp tests/golden/device/*.npz gpurun_out/device/
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 5
echo ALL_RC=0
