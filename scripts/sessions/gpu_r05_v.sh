#!/bin/bash
# Round 5, session v: the tree as committed at the end of the round -- GPU tests and smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05_v
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 10 > gpurun_out/${T}_bench_quick.log 2>&1 || exit 7
echo ALL_RC=0
