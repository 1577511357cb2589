#!/bin/bash
# Round 6, session c: the force-free guard maximum (PD_FF_GUARD_MAX; lib/libpdeval_g0.so = off)
# and the per-point counts before the fingerprint stores -- same-box A/B of both benches --,
# the worker pool leg (digest outside the timed region), then the PMC / calibration session.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_c
for k in 1 2; do
  for v in "" _g0; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_ff${v}_${k}.log 2>&1 || exit 7
  done
done
timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr.log 2>&1 || exit 8
T=r06_c bash scripts/sessions/gpu_r06_b.sh > gpurun_out/${T}_b_chain.log 2>&1 || { echo "B failed"; exit 9; }
echo ALL_RC=0
