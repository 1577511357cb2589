#!/bin/bash
# Round 4, session v: the final evidence for the shipped defaults (symmetric B, FMA-accumulated A):
# the default bench (worker pool over 3 passes), the Kerr bench, PMC passes for both problems and
# rocprofv3 kernel-trace summaries of both benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_v}
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu --problem kerr_magnetosphere > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --no-cpu --no-extras > gpurun_out/${T}_prof.log 2>&1 || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_kerr -o run -- python bench.py --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_prof_kerr.log 2>&1 || exit 11
bash scripts/gpu_pmc.sh > gpurun_out/${T}_pmc_chain.log 2>&1
grep -q PMC_RC=0 gpurun_out/${T}_pmc_chain.log || exit 7
python scripts/pmc_summary.py gpurun_out/pmc gpurun_out/${T}_pmc.json > gpurun_out/${T}_pmc_summary.log 2>&1 || exit 8
PMC_TAG=_kerr PROBLEM=kerr_magnetosphere bash scripts/gpu_pmc.sh > gpurun_out/${T}_pmc_kerr_chain.log 2>&1
grep -q PMC_RC=0 gpurun_out/${T}_pmc_kerr_chain.log || exit 9
python scripts/pmc_summary.py gpurun_out/pmc_kerr gpurun_out/${T}_kerr_pmc.json > gpurun_out/${T}_pmc_kerr_summary.log 2>&1 || exit 12
echo ALL_RC=0
