#!/bin/bash
# Round 4, session b: GPU tests + smoke with the coordinate-power tables (PD_PTAB), then a
# same-box A/B: force-free and Kerr, tables off (nopt) / on (default) / force-free at 5 waves.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_b}
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 5
for v in nopt "" ff5; do
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/${T}${v:+_$v}_ff.log 2>&1 || exit 6
done
for v in nopt ""; do
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}${v:+_$v}_kerr.log 2>&1 || exit 7
done
echo ALL_RC=0
