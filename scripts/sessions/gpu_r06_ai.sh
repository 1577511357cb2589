#!/bin/bash
# Round 6, session ai: the final shipped build (Kerr pass 1 at W = 3, pass 2 at W = 4, without the power
# table) -- GPU tests, smoke, the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_ai
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit 5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 6
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 7
echo ALL_RC=0
