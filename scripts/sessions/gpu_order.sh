set -o pipefail
mkdir -p gpurun_out/o
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/o/shuf.log 2>&1 || exit 5
PD_BENCH_STREAM_ORDER=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/o/stream.log 2>&1 || exit 6
