#!/bin/bash
# Round 4, session w: the row's 1/x^2, 1/x^3 in SGPRs (PD_EPI_UNIFORM, the FF pass-1 spill 64 -> 32 B):
# GPU parity tests, then a same-box A/B against the VGPR build (nouni), twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_symbolic.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04_w_pytest.log 2>&1 || exit 4
TAG=r04_w VARIANTS="nouni" bash scripts/gpu_ab_ff.sh || exit 5
TAG=r04_w2 VARIANTS="nouni" bash scripts/gpu_ab_ff.sh || exit 6
echo ALL_RC=0
