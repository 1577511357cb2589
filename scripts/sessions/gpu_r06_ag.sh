#!/bin/bash
# Round 6, session ag: force-free without the x power table (PD_PTAB=0, 80 B/lane spill) against
# the shipped x-table build, alternated twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_ag
for k in 1 2; do
  for v in "" _fpt0; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ff${v}_$k.log 2>&1 || exit 7
  done
done
echo ALL_RC=0
