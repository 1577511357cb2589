#!/bin/bash
# Round 4, session z: the stack-2 double-double point kernel at 1 wave/SIMD (PD_DD2_WAVES=1: its
# spill goes to AGPRs, scratch 0) against 2 waves (default): the 2^21 bench step and the device
# call of worker-sized batches, alternated twice on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in "" dd1; do
    L=pde-engine_amd/lib/libpdeval${v:+_$v}.so
    PDEVAL_LIB=$L timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r04_z${r}${v:+_$v}_ff.log 2>&1 || exit 5
    PDEVAL_LIB=$L timeout -k 10 200 python scripts/profile_device_batch.py --sizes 512,4096 --reps 15 > gpurun_out/r04_z${r}${v:+_$v}_batch.log 2>&1 || exit 6
  done
done
echo ALL_RC=0
