#!/bin/bash
# Round 6, session f: the default bench line (heartbeats in the long legs, smaller strict leg,
# recorded end-to-end time to the 7 solutions), then PMC passes + kernel traces of both benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_f
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH failed"; exit 7; }
TAG=$T bash scripts/gpu_prof.sh > gpurun_out/${T}_prof_chain.log 2>&1
grep -q PROF_RC=0 gpurun_out/${T}_prof_chain.log || { echo "PROF failed"; exit 9; }
echo ALL_RC=0
