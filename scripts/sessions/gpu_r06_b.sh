#!/bin/bash
# Round 6, session b: per-opcode executed FP64 counts (the FLOP model's calibration programs,
# scripts/microbench.py --set calib) and the PMC passes + kernel traces of both benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06_b}
for P in force_free kerr_magnetosphere; do
  TAG=_${T}_$P PROBLEM=$P SET=calib bash scripts/gpu_pmc_micro.sh > gpurun_out/${T}_pmcm_$P.log 2>&1
  grep -q PMCM_RC=0 gpurun_out/${T}_pmcm_$P.log || { echo "PMCM failed"; exit 10; }
  python scripts/pmc_micro.py gpurun_out/pmcm_${T}_$P $P calib gpurun_out/${T}_calib_$P.json > gpurun_out/${T}_calib_$P.txt 2>&1 || exit 11
done
TAG=$T bash scripts/gpu_prof.sh > gpurun_out/${T}_prof_chain.log 2>&1
grep -q PROF_RC=0 gpurun_out/${T}_prof_chain.log || { echo "PROF failed"; exit 9; }
echo ALL_RC=0
