#!/bin/bash
# Round-3 iteration session: GPU tests, smoke, the force-free bench with its drop-in-path
# extras (no CPU legs), and the Kerr bench.  Each GPU step has its own limit; a failing test
# (pytest rc 1) does not stop the chain, a crash / abort / time limit does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-x}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; ok $rc || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 5
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_bench.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 7
echo "CHAIN_RC=0"
