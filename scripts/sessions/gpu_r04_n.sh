#!/bin/bash
# Round 4, session n: the default bench (the driver's command) and the Kerr bench, smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_n}
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 3
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --no-cpu --problem kerr_magnetosphere > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 5
echo ALL_RC=0
