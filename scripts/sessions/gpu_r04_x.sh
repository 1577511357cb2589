#!/bin/bash
# Round 4, session x: the lane's 1/y pinned outside the row loop (PD_INVY_PIN; the optimizer had
# moved the IEEE reciprocal into it): GPU parity tests, then a same-box A/B, force-free and Kerr,
# against the previous build (nopin), without the lean Kerr epilogue (noklean) and with the SGPR
# 1/x powers as well (pinuni), twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04_x_pytest.log 2>&1 || exit 4
TAG=r04_x KERR=1 VARIANTS="nopin noklean pinuni" bash scripts/gpu_ab_ff.sh || exit 5
TAG=r04_x2 KERR=1 VARIANTS="nopin noklean pinuni" bash scripts/gpu_ab_ff.sh || exit 6
echo ALL_RC=0
