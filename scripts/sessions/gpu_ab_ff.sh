#!/bin/bash
# Same-box A/B of force-free pass 1 (2^21 candidates, 5 timed steps): the default library and
# each variant named in VARIANTS (pde-engine_amd/lib/libpdeval_<v>.so); KERR=1 adds Kerr runs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-abff}
for v in "" ${VARIANTS:-}; do
  [ "$v" = "-" ] && v=""
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/${T}${v:+_$v}_ff.log 2>&1 || exit 5
  if [ -n "${KERR:-}" ]; then
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}${v:+_$v}_kerr.log 2>&1 || exit 6
  fi
done
echo AB_DONE
