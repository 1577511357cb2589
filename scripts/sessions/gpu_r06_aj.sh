#!/bin/bash
# Round 6, session aj: Kerr pass 2 at W = 5 and 6 against the shipped W = 4, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_aj
for k in 1 2; do
  for v in "" _kd5 _kd6; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr${v}_$k.log 2>&1 || exit 7
  done
done
echo ALL_RC=0
