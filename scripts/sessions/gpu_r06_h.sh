#!/bin/bash
# Round 6, session h: GPU tests on the build with the pointer-walk interpreter, the uniform
# sparse-mask bitmap and the calibrated FLOP model; same-box A/B of the pointer walk
# (lib/libpdeval_p0.so = PD_LEAN_PTR=0); pass-1 traffic (WRITE_SIZE / FETCH_SIZE); the FF
# per-opcode calibration with the POWN programs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_h
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
for k in 1 2; do
  for v in "" _p0; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_ff${v}_${k}.log 2>&1 || exit 7
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_kerr${v}_${k}.log 2>&1 || exit 8
  done
done
B="python bench.py --steps 1 --warmup 0 --n 262144 --no-cpu --no-extras"
D=gpurun_out/pmc_${T}_traffic
mkdir -p $D
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $B > $D/write.log 2>&1 || exit 9
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $B > $D/fetch.log 2>&1 || exit 9
P=force_free
TAG=_${T}_$P PROBLEM=$P SET=calib bash scripts/gpu_pmc_micro.sh > gpurun_out/${T}_pmcm_$P.log 2>&1
grep -q PMCM_RC=0 gpurun_out/${T}_pmcm_$P.log || { echo "PMCM failed"; exit 10; }
python scripts/pmc_micro.py gpurun_out/pmcm_${T}_$P $P calib gpurun_out/${T}_calib_$P.json > gpurun_out/${T}_calib_$P.txt 2>&1 || exit 11
echo ALL_RC=0
