#!/bin/bash
# A/B of library variants on the bench workload (one process per variant, each time-limited).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${N:-262144}
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n 4096 --no-cpu > gpurun_out/ab_small.log 2>&1 || exit 3
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "PYTEST_RC=$?" >> gpurun_out/pytest_gpu.log
for v in "" _w3 _w4; do
  PDEVAL_LIB=pde-engine_amd/lib/libpdeval$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --n $N --no-cpu > gpurun_out/ab$v.log 2>&1 || exit 4
done
echo AB_DONE
