#!/bin/bash
# Round 6, session a: the slot-indexed hoist buffer and sparse tier-1 masks -- GPU tests, smoke and
# a same-box A/B of the bench (PDEVAL_HOIST_SLOTS=1 vs 0, force-free and Kerr; PDEVAL_DD_EARLY=0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_a
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 6
for k in 1 2; do
  for s in 1 0; do
    PDEVAL_HOIST_SLOTS=$s timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_ff_s${s}_${k}.log 2>&1 || exit 7
  done
  # the early double-double tier on its side stream, beside pass 1 (default) or after the grid
  PDEVAL_DD_EARLY=0 timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_ff_dd0_${k}.log 2>&1 || exit 7
done
for s in 1 0; do
  PDEVAL_HOIST_SLOTS=$s timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_kerr_s${s}.log 2>&1 || exit 8
done
echo ALL_RC=0
