#!/bin/bash
# Round 6, session m: the per-opcode opaque ordinate (PD_PIN_Y; lib/libpdeval_y0.so = off):
# same-box A/B of both benches (the GPU tests ran on this build in session l), pass-1 traffic (WRITE_SIZE / FETCH_SIZE).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_m
for k in 1 2; do
  for v in "" _y0; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_ff${v}_${k}.log 2>&1 || exit 7
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_kerr${v}_${k}.log 2>&1 || exit 8
  done
done
B="python bench.py --steps 1 --warmup 0 --n 262144 --no-cpu --no-extras"
D=gpurun_out/pmc_${T}_traffic
mkdir -p $D
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $B > $D/write.log 2>&1 || exit 9
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $B > $D/fetch.log 2>&1 || exit 9
echo ALL_RC=0
