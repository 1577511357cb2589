#!/bin/bash
# Round 5, session k: the GPU tests and a hoist on / off A/B of the shipped build, then the
# round's profiles of the shipped defaults -- PMC passes and kernel-trace summaries of both
# benches (scripts/gpu_prof.sh), and the force-free kernel trace with the double-double tier
# serialized after the grid (PDEVAL_DD_EARLY=0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_k
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
ab() {  # tag problem hoist
  PDEVAL_HOIST=$3 timeout -k 10 300 python bench.py --no-cpu --no-extras \
    --problem $2 --steps 10 > gpurun_out/${T}_ab_$1.log 2>&1 || return 1
  echo "$1 done" >> gpurun_out/${T}_ab_progress.txt
}
ab ff_h1 force_free 1 || exit 6
ab ff_h0 force_free 0 || exit 6
ab kerr_h1 kerr_magnetosphere 1 || exit 6
TAG=$T bash scripts/gpu_prof.sh > gpurun_out/${T}_prof_chain.log 2>&1
grep -q PROF_RC=0 gpurun_out/${T}_prof_chain.log || { echo "PROF failed"; exit 7; }
PDEVAL_DD_EARLY=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ff_dd0 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/${T}_prof_ff_dd0.log 2>&1 || exit 8
echo ALL_RC=0
