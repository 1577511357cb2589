#!/bin/bash
# Round 5, session r: the final build -- GPU tests, smoke, the default bench line, the Kerr
# bench, kernel-trace summaries of both benches and the PMC passes (scripts/gpu_prof.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_r
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 6
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || exit 7
timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu > gpurun_out/${T}_bench_kerr.log 2> gpurun_out/${T}_bench_kerr.err || exit 8
TAG=$T bash scripts/gpu_prof.sh > gpurun_out/${T}_prof_chain.log 2>&1
grep -q PROF_RC=0 gpurun_out/${T}_prof_chain.log || { echo "PROF failed"; exit 9; }
echo ALL_RC=0
