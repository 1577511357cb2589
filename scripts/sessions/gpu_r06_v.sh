#!/bin/bash
# Round 6, session v: Kerr PMC passes and kernel trace of the final build (pass 1 at W = 3 without
# power tables, pass 2 at W = 4); the summary sorts after r06_u, so the bench line reads it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_v
PMC_TAG=_${T}_kerr PROBLEM=kerr_magnetosphere bash scripts/gpu_pmc.sh > gpurun_out/${T}_pmc_kerr_chain.log 2>&1
grep -q PMC_RC=0 gpurun_out/${T}_pmc_kerr_chain.log || exit 8
python scripts/pmc_summary.py gpurun_out/pmc_${T}_kerr gpurun_out/${T}_kerr_pmc.json > gpurun_out/${T}_kerr_pmc_summary.log 2>&1 || exit 9
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_kerr -o run -- python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/${T}_prof_kerr.log 2>&1 || exit 11
cp gpurun_out/${T}_kerr_pmc.json profiles/ || exit 12
timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr_bench.log 2>&1 || exit 13
echo ALL_RC=0
