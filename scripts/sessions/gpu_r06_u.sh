#!/bin/bash
# Round 6, session u: PMC passes and kernel traces of the shipped build (Kerr pass 1 at W = 3),
# then the default bench line reading the new PMC summaries.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_u
TAG=$T bash scripts/gpu_prof.sh > gpurun_out/${T}_prof_chain.log 2>&1
grep -q PROF_RC=0 gpurun_out/${T}_prof_chain.log || { echo "PROF failed"; exit 9; }
cp gpurun_out/${T}_ff_pmc.json gpurun_out/${T}_kerr_pmc.json profiles/ || exit 10
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { echo "BENCH failed"; exit 7; }
echo ALL_RC=0
