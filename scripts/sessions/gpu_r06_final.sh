#!/bin/bash
# Round 6, final: the shipped build -- GPU tests, smoke, the default bench line (the driver's
# command), then PMC passes + kernel traces of both benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_final
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 6
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { echo "BENCH failed"; exit 7; }
TAG=$T bash scripts/gpu_prof.sh > gpurun_out/${T}_prof_chain.log 2>&1
grep -q PROF_RC=0 gpurun_out/${T}_prof_chain.log || { echo "PROF failed"; exit 9; }
echo ALL_RC=0
