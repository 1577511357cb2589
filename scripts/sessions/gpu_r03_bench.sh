#!/bin/bash
# Round-3 bench session: smoke, the default bench (force-free, with the drop-in-path extras and
# both CPU baselines), the Kerr bench, and the worker's host-side profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03_g}
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 5
timeout -k 10 500 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --no-cpu --no-extras --problem kerr_magnetosphere > gpurun_out/${T}_bench_kerr.log 2>&1 || exit 7
timeout -k 10 300 python scripts/profile_worker.py > gpurun_out/${T}_worker_profile.log 2>&1 || exit 8
echo CHAIN_RC=0
