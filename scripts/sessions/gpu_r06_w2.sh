#!/bin/bash
# Round 6, session w2: Kerr pass 2 at W = 3 (4 waves, 128 B spill) and W = 4 (3 waves, 64 B spill)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_w2
for k in 1 2; do
  for v in "" _kd3s4 _kd4s3; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr${v}_$k.log 2>&1 || exit 7
  done
done
echo ALL_RC=0
