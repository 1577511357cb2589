#!/bin/bash
# Round 4, session a: GPU tests + smoke on the closed-form fused Kerr push (no spill), a
# same-box Kerr A/B (round-3 grid unit, default, W=3 and W=4 variants), the force-free bench,
# and a kernel trace of the default Kerr bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_a}
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 5
for v in r03 "" kw3 kw4; do
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v:+_$v}.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}${v:+_$v}_kerr.log 2>&1 || exit 6
done
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${T}_bench.log 2>&1 || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_kerr -o run -- python3 bench.py --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_prof_kerr.log 2>&1 || exit 8
echo ALL_RC=0
