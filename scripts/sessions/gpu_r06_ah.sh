#!/bin/bash
# Round 6, session ah: Kerr without power tables -- pass 1 at W = 4 (4 waves/SIMD) and pass 2 at
# W = 4 (4 waves, 192 B spill) against the shipped W = 3 / W = 3, three alternations.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_ah
for k in 1 2 3; do
  for v in "" _kw4s4 _kd4; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr${v}_$k.log 2>&1 || exit 7
  done
done
echo ALL_RC=0
