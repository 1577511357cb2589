#!/bin/bash
# Round 6, session o: the round-5 build (ab_r05/, the tree of commit 6b2959f, built here) against
# the shipped round-6 build on one box, both benches, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_o
for k in 1 2; do
  (cd ab_r05 && timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5) > gpurun_out/${T}_ff_r05_$k.log 2>&1 || exit 7
  timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ff_r06_$k.log 2>&1 || exit 7
  (cd ab_r05 && timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5) > gpurun_out/${T}_kerr_r05_$k.log 2>&1 || exit 8
  timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr_r06_$k.log 2>&1 || exit 8
done
echo ALL_RC=0
