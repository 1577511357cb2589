#!/bin/bash
# One GPU-box session: parity tests, smoke, benches, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit.  A failing test (pytest rc 1) does not stop the
# chain; a crash, abort or time limit (any other non-zero rc) does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n 4096 --no-cpu > gpurun_out/${TAG:-x}_bench_small.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG:-x}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; ok $rc || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-x}_smoke.log 2>&1 || exit 5
timeout -k 10 300 python bench.py > gpurun_out/${TAG:-x}_bench.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG:-x}_prof -o run -- python bench.py --no-cpu --no-extras > gpurun_out/${TAG:-x}_prof.log 2>&1 || exit 7
echo "CHAIN_RC=0"
