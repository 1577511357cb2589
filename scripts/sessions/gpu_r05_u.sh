#!/bin/bash
# Round 5, session u: the final build's default bench line (as the driver runs it), smoke, the
# Kerr bench and kernel-trace summaries of both benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_u
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 6
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || exit 7
timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu > gpurun_out/${T}_bench_kerr.log 2> gpurun_out/${T}_bench_kerr.err || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ff -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/${T}_prof_ff.log 2>&1 || exit 9
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_kerr -o run -- python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/${T}_prof_kerr.log 2>&1 || exit 10
echo ALL_RC=0
