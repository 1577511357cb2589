#!/bin/bash
# Round 6, session z: Kerr pass 1/2 switches re-measured at W = 3: opcode-frequency dispatch off,
# both power tables / none, 4 waves/SIMD; against the shipped build, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_z
for k in 1 2; do
  for v in "" _kdf0 _kpt1 _kpt0 _ks4; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr${v}_$k.log 2>&1 || exit 7
  done
done
echo ALL_RC=0
