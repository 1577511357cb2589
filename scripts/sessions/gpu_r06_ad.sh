#!/bin/bash
# Round 6, session ad: kernel traces of both benches and the Kerr PMC passes on the shipped build
# (Kerr pass 2 at W = 3 since session u).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_ad
PMC_TAG=_${T}_kerr PROBLEM=kerr_magnetosphere bash scripts/gpu_pmc.sh > gpurun_out/${T}_pmc_kerr_chain.log 2>&1
grep -q PMC_RC=0 gpurun_out/${T}_pmc_kerr_chain.log || exit 8
python scripts/pmc_summary.py gpurun_out/pmc_${T}_kerr gpurun_out/${T}_kerr_pmc.json > gpurun_out/${T}_kerr_pmc_summary.log 2>&1 || exit 9
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ff -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/${T}_prof_ff.log 2>&1 || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_kerr -o run -- python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/${T}_prof_kerr.log 2>&1 || exit 11
echo ALL_RC=0
