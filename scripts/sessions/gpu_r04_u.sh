#!/bin/bash
# Round 4, session u: symmetric B and the FMA-accumulated A as the defaults: GPU tests and the default bench + Kerr bench;

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_u}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 3
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu --problem kerr_magnetosphere > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 6
echo ALL_RC=0
