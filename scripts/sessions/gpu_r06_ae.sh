#!/bin/bash
# Round 6, session ae: Kerr without the x power table (PD_PTAB_KERR=0) against the shipped build,
# three alternations, then the Kerr GPU tests on the variant.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_ae
for k in 1 2 3; do
  for v in "" _kpt0; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr${v}_$k.log 2>&1 || exit 7
  done
done
PDEVAL_LIB=pde-engine_amd/lib/libpdeval_kpt0.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "kerr or Kerr or config4" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_kerr_kpt0.log 2>&1 || exit 5
echo ALL_RC=0
