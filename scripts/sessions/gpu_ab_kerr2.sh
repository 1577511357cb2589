#!/bin/bash
# Same-box A/B of Kerr (2^20 candidates, 3 timed steps): the default library and each
# variant named in VARIANTS (pde-engine_amd/lib/libpdeval_<v>.so).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-abk2}
for v in "" ${VARIANTS:-}; do
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}${v:+_$v}_kerr_magnetosphere.log 2>&1 || exit 5
done
echo AB_DONE
