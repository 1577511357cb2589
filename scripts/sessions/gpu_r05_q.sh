#!/bin/bash
# Round 5, session q: segments hoisted for Kerr only (force-free compiled without them): the
# GPU tests, a same-box A/B of PDEVAL_HOIST_SUB, then the default bench line and the Kerr bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_q
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
ab() {  # tag problem sub
  PDEVAL_HOIST_SUB=$3 timeout -k 10 300 python bench.py --no-cpu --no-extras \
    --problem $2 --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
for r in 1 2; do
  ab kerr_seg_$r kerr_magnetosphere 1 || exit 6
  ab kerr_seg0_$r kerr_magnetosphere 0 || exit 6
done
ab ff_1 force_free 1 || exit 6
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 7
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || exit 8
timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu > gpurun_out/${T}_bench_kerr.log 2> gpurun_out/${T}_bench_kerr.err || exit 9
echo ALL_RC=0
