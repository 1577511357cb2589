#!/bin/bash
# One GPU-box session: parity tests, smoke, benches, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; steps are chained with && so the first failure ends it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${N:-262144}
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n 4096 --no-cpu > gpurun_out/bench_small.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python bench.py --early-exit --no-cpu > gpurun_out/bench_early.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --no-cpu > gpurun_out/prof.log 2>&1
echo "CHAIN_RC=$?"
