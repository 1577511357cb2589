#!/bin/bash
# Round 4, session t: same-box A/B of the force-free epilogue: default (symmetric B), nobsym
# (round-3 B), afma (A accumulated by FMAs), twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04_t VARIANTS="nobsym afma" bash scripts/gpu_ab_ff.sh || exit 5
TAG=r04_t2 VARIANTS="nobsym afma" bash scripts/gpu_ab_ff.sh || exit 6
echo ALL_RC=0
