#!/bin/bash
# Round 6, session t: GPU tests with Kerr pass 1 at W = 3 (the new default), then Kerr pass 2
# variants (3 waves/SIMD without its spill, W = 3) against it, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit 5
for k in 1 2; do
  for v in "" _kd2s3 _kd3s3; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr${v}_$k.log 2>&1 || exit 7
  done
done
for v in "" _kd2s3; do
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ff${v}.log 2>&1 || exit 8
done
echo ALL_RC=0
