#!/bin/bash
# Round 6, session d: GPU tests (streaming strict mode, range rows), the Kerr calibration
# programs under PMC (microbench output buffers fixed), PMC passes + kernel traces of both benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_d
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
timeout -k 10 120 python scripts/microbench.py --n 65536 --reps 1 --problem kerr_magnetosphere --set calib > gpurun_out/${T}_micro_kerr.log 2>&1 || exit 6
P=kerr_magnetosphere
TAG=_${T}_$P PROBLEM=$P SET=calib bash scripts/gpu_pmc_micro.sh > gpurun_out/${T}_pmcm_$P.log 2>&1
grep -q PMCM_RC=0 gpurun_out/${T}_pmcm_$P.log || { echo "PMCM failed"; exit 10; }
python scripts/pmc_micro.py gpurun_out/pmcm_${T}_$P $P calib gpurun_out/${T}_calib_$P.json > gpurun_out/${T}_calib_$P.txt 2>&1 || exit 11
TAG=$T bash scripts/gpu_prof.sh > gpurun_out/${T}_prof_chain.log 2>&1
grep -q PROF_RC=0 gpurun_out/${T}_prof_chain.log || { echo "PROF failed"; exit 9; }
echo ALL_RC=0
