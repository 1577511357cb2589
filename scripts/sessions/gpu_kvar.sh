#!/bin/bash
# Kerr bench for the default library and each variant in VARS (no parity tests).
set -o pipefail
mkdir -p gpurun_out/k
export TMPDIR=/tmp
T=${TAG:-x}
for v in "" ${VARS}; do
  L=pde-engine_amd/lib/libpdeval$v.so
  [ -f $L ] || continue
  PDEVAL_LIB=$L timeout -k 10 200 python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/k/${T}_kerr$v.log 2>&1 || exit 6
done
echo KVAR_DONE
