#!/bin/bash
# Round-4 profile session: PMC passes (force-free, Kerr) summarized into profiles/, and
# rocprofv3 kernel-trace summaries of the force-free and Kerr benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_p}
bash scripts/gpu_pmc.sh > gpurun_out/${T}_pmc_chain.log 2>&1
grep -q PMC_RC=0 gpurun_out/${T}_pmc_chain.log || exit 6
python scripts/pmc_summary.py gpurun_out/pmc gpurun_out/${T}_pmc.json > gpurun_out/${T}_pmc_summary.log 2>&1 || exit 7
PMC_TAG=_kerr PROBLEM=kerr_magnetosphere bash scripts/gpu_pmc.sh > gpurun_out/${T}_pmc_kerr_chain.log 2>&1
grep -q PMC_RC=0 gpurun_out/${T}_pmc_kerr_chain.log || exit 8
python scripts/pmc_summary.py gpurun_out/pmc_kerr gpurun_out/${T}_kerr_pmc.json > gpurun_out/${T}_pmc_kerr_summary.log 2>&1 || exit 9
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --no-cpu --no-extras > gpurun_out/${T}_prof.log 2>&1 || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_kerr -o run -- python bench.py --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_prof_kerr.log 2>&1 || exit 11
echo CHAIN_RC=0
