#!/bin/bash
# Re-entry session: GPU tests, smoke and bench on a freshly rebuilt tree, then a kernel-trace
# summary of the default bench command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03_p} bash scripts/gpu_r03_verify.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_p_prof -o run -- python3 bench.py --no-cpu --no-extras > gpurun_out/r03_p_prof.log 2>&1 || exit 10
echo ALL_RC=0
