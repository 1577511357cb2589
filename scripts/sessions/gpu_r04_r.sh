#!/bin/bash
# Round 4, session r: the symmetric jet square of B in the force-free epilogue (bsym), A/B twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04_r VARIANTS="bsym" bash scripts/gpu_ab_ff.sh || exit 5
TAG=r04_r2 VARIANTS="bsym" bash scripts/gpu_ab_ff.sh || exit 6
echo ALL_RC=0
