#!/bin/bash
# Round-end GPU session: parity tests, smoke, PMC passes (force-free and Kerr; the summaries
# go to profiles/ so the bench reports this build's traffic), the default bench (with the CPU
# baselines), the Kerr bench, and rocprofv3 kernel-trace summaries.  TAG names the outputs.
set -o pipefail
T=${TAG:-r02_z}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 5
TAG=$T bash scripts/gpu_prof.sh > gpurun_out/${T}_prof_chain.log 2>&1
grep -q PROF_RC=0 gpurun_out/${T}_prof_chain.log || exit 6
cp gpurun_out/${T}_ff_pmc.json profiles/${T}_ff_pmc.json && cp gpurun_out/${T}_kerr_pmc.json profiles/${T}_kerr_pmc.json || exit 7
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 8
timeout -k 10 200 python bench.py --problem kerr_magnetosphere --no-cpu > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 9
echo "FINAL_RC=0"
