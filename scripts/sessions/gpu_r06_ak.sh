#!/bin/bash
# Round 6, session ak: Kerr pass 1 at W = 2 / 6 waves without power tables against the shipped
# W = 3 / 5 waves, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_ak
for k in 1 2; do
  for v in "" _kw2s6; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr${v}_$k.log 2>&1 || exit 7
  done
done
echo ALL_RC=0
