#!/bin/bash
# Round 6, session aa: force-free pass 1 switches re-measured on the current build: 4 waves/SIMD,
# wave-uniform epilogue constants, both power tables; against the shipped build, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_aa
for k in 1 2; do
  for v in "" _fs4 _feu1 _fpt1; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ff${v}_$k.log 2>&1 || exit 7
  done
done
echo ALL_RC=0
