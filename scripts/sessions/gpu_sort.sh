#!/bin/bash
# Parity tests, then force-free benches with and without the shape sort, and the Kerr bench.
set -o pipefail
mkdir -p gpurun_out/s
export TMPDIR=/tmp
T=${TAG:-x}
timeout -k 10 400 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s/${T}_pytest.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/s/${T}_ff.log 2>&1 || exit 5
PDEVAL_SORT=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/s/${T}_ff_nosort.log 2>&1 || exit 6
PD_BENCH_STREAM_ORDER=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/s/${T}_ff_stream.log 2>&1 || exit 7
timeout -k 10 200 python bench.py --problem kerr_magnetosphere --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/s/${T}_kerr.log 2>&1 || exit 8
echo SORT_DONE
