#!/bin/bash
# Round 4, session s2: the per-point scaled residual as a select (PD_SCALED_SEL, variant ssel):
# the GPU parity tests on the variant library, then a same-box A/B (force-free and Kerr), twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PDEVAL_LIB=pde-engine_amd/lib/libpdeval_ssel.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04_s2_ssel_pytest.log 2>&1 || exit 4
TAG=r04_s2 KERR=1 VARIANTS="ssel" bash scripts/gpu_ab_ff.sh || exit 5
TAG=r04_s2b KERR=1 VARIANTS="ssel" bash scripts/gpu_ab_ff.sh || exit 6
echo ALL_RC=0
