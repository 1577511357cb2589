#!/bin/bash
# force-free and Kerr benches for the default library and each variant in VARS (no tests).
set -o pipefail
mkdir -p gpurun_out/v
export TMPDIR=/tmp
T=${TAG:-x}
for v in "" ${VARS}; do
  L=pde-engine_amd/lib/libpdeval$v.so
  [ -f $L ] || continue
  [ -n "$NOFF" ] || PDEVAL_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/v/${T}_ff$v.log 2>&1 || exit 5
  PDEVAL_LIB=$L timeout -k 10 200 python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/v/${T}_kerr$v.log 2>&1 || exit 6
done
echo VAR_DONE
