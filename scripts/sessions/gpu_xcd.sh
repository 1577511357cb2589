#!/bin/bash
# pass-1 block order: benches (default and VARS) and the force-free PMC passes of the default.
set -o pipefail
mkdir -p gpurun_out/x
export TMPDIR=/tmp
for v in "" ${VARS}; do
  L=pde-engine_amd/lib/libpdeval$v.so
  PDEVAL_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/x/ff$v.log 2>&1 || exit 5
  PDEVAL_LIB=$L timeout -k 10 200 python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/x/kerr$v.log 2>&1 || exit 6
done
PMC_TAG=_xcd PROBLEM=force_free bash scripts/gpu_pmc.sh > gpurun_out/x/pmc_chain.log 2>&1
grep -q PMC_RC=0 gpurun_out/x/pmc_chain.log || exit 7
python scripts/pmc_summary.py gpurun_out/pmc_xcd gpurun_out/x/xcd_ff_pmc.json > gpurun_out/x/pmc_summary.log 2>&1 || exit 8
echo XCD_DONE
