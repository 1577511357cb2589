#!/bin/bash
# A/B of lean-interpreter variants in one box session (same clocks): the default library,
# no superinstructions (nofuse), and the round-2 interpreter (old: no superinstructions, both
# stack-3 operand slots in LDS).  Force-free and Kerr, 2^20 candidates, 3 timed steps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-ab}
for v in "" _nofuse _old; do
  for p in force_free kerr_magnetosphere; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras --problem $p > gpurun_out/${T}${v}_$p.log 2>&1 || exit 4
  done
done
echo AB_DONE
