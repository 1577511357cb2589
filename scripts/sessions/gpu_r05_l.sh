#!/bin/bash
# Round 5, session l: the default bench line of the shipped build (as the driver runs it), and
# smoke().
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_l_smoke.log 2>&1 || exit 5
timeout -k 10 900 python bench.py > gpurun_out/r05_l_bench.log 2> gpurun_out/r05_l_bench.err || exit 6
echo ALL_RC=0
