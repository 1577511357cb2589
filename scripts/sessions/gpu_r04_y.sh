#!/bin/bash
# Round 4, session y: final evidence for the shipped build (1/y pinned, lean Kerr epilogue): the
# default bench, the Kerr bench, and rocprofv3 kernel-trace summaries of both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_y}
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 3
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu --problem kerr_magnetosphere > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --no-cpu --no-extras > gpurun_out/${T}_prof.log 2>&1 || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_kerr -o run -- python bench.py --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_prof_kerr.log 2>&1 || exit 11
echo ALL_RC=0
