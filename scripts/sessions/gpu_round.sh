#!/bin/bash
# One GPU-box session in the order the bench needs: parity tests, smoke, the PMC passes
# (summary copied to profiles/ so bench.py reports this build's traffic), the bench, and a
# rocprofv3 kernel-trace summary.  TAG names the outputs (gpurun_out/<TAG>_*).
set -o pipefail
TAG=${TAG:-r01_x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 5
bash scripts/gpu_pmc.sh > gpurun_out/${TAG}_pmc_chain.log 2>&1
grep -q PMC_RC=0 gpurun_out/${TAG}_pmc_chain.log || exit 6
python scripts/pmc_summary.py gpurun_out/pmc gpurun_out/${TAG}_pmc.json > gpurun_out/${TAG}_pmc_summary.log 2>&1 || exit 7
cp gpurun_out/${TAG}_pmc.json profiles/
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python bench.py --no-cpu --no-extras > gpurun_out/${TAG}_prof.log 2>&1 || exit 9
echo "CHAIN_RC=0"
