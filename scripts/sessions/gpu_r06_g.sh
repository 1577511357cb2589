#!/bin/bash
# Round 6, session g: same-box A/B of the split ballots (lib/libpdeval_b0.so = PD_BALLOT_SPLIT=0),
# force-free pass-1 HBM traffic with the hoist slots on / off (WRITE_SIZE, FETCH_SIZE passes),
# the Kerr per-program calibration under PMC, then the GPU tests on the default build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_g
for k in 1 2; do
  for v in "" _b0; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_ff${v}_${k}.log 2>&1 || exit 7
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_kerr${v}_${k}.log 2>&1 || exit 8
  done
done
B="python bench.py --steps 1 --warmup 0 --n 262144 --no-cpu --no-extras"
for s in 1 0; do
  D=gpurun_out/pmc_${T}_slots$s
  mkdir -p $D
  PDEVAL_HOIST_SLOTS=$s timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $B > $D/write.log 2>&1 || exit 9
  PDEVAL_HOIST_SLOTS=$s timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $B > $D/fetch.log 2>&1 || exit 9
done
P=kerr_magnetosphere
TAG=_${T}_$P PROBLEM=$P SET=calib bash scripts/gpu_pmc_micro.sh > gpurun_out/${T}_pmcm_$P.log 2>&1
grep -q PMCM_RC=0 gpurun_out/${T}_pmcm_$P.log || { echo "PMCM failed"; exit 10; }
python scripts/pmc_micro.py gpurun_out/pmcm_${T}_$P $P calib gpurun_out/${T}_calib_$P.json > gpurun_out/${T}_calib_$P.txt 2>&1 || exit 11
timeout -k 10 300 python scripts/profile_device_batch.py --sizes 1024,4096,8192,16384 --reps 9 > gpurun_out/${T}_device_batch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_batch -o run -- python scripts/profile_device_batch.py --sizes 4096 --reps 5 > gpurun_out/${T}_prof_batch.log 2>&1 || exit 13
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
echo ALL_RC=0
