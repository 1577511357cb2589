#!/bin/bash
# Round 6, session x: GPU tests and the Kerr bench with Kerr pass 2 at W = 3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_x
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_kerr.log 2>&1 || exit 7
echo ALL_RC=0
