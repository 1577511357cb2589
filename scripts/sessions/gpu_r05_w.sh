#!/bin/bash
# Round 5, session w: per-program costs of force-free pass 1 (one repeated program per batch):
# the fixed per-point work (the epilogue and the tests) against the opcodes, for DESIGN §10.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/microbench.py --problem force_free > gpurun_out/r05_w_microbench_ff.log 2>&1 || exit 5
echo ALL_RC=0
