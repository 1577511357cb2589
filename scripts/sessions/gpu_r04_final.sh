#!/bin/bash
# Round 4, final session: the shipped build (1/y pin, lean Kerr epilogue, 1-wave stack-2
# double-double kernel): the GPU tests, smoke, the default bench, the Kerr bench and kernel traces.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_final}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 3
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu --problem kerr_magnetosphere > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --no-cpu --no-extras > gpurun_out/${T}_prof.log 2>&1 || exit 10
echo ALL_RC=0
