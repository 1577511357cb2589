#!/bin/bash
# Same-box A/B of Kerr pass-1 shapes (W grid rows per dispatch, waves per SIMD): the default
# library and the variants named in VARIANTS, Kerr depth-4 bench at 2^20 candidates.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-abk}
for v in "" ${VARIANTS:-}; do
  lib=pde-engine_amd/lib/libpdeval${v:+_$v}.so
  PDEVAL_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}${v:+_$v}.log 2>&1 || exit 5
done
echo AB_DONE
