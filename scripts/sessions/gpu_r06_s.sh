#!/bin/bash
# Round 6, session s: Kerr pass 1 with more grid rows per dispatch (W = 3 at 5 waves/SIMD,
# W = 4 at 4 waves/SIMD) against the shipped W = 2, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_s
for k in 1 2; do
  for v in "" _kw3s5 _kw4s4; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr${v}_$k.log 2>&1 || exit 7
  done
done
echo ALL_RC=0
