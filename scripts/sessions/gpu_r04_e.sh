#!/bin/bash
# Round 4, session e: GPU tests + smoke with the small-batch graph path, the inline split,
# the worker stage profile at the default queue batch, and the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_e}
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 5
timeout -k 10 300 python scripts/profile_inline.py --n 2000 > gpurun_out/${T}_inline.log 2>&1 || exit 6
PDEVAL_GRAPH=0 timeout -k 10 300 python scripts/profile_inline.py --n 1000 > gpurun_out/${T}_inline_nograph.log 2>&1 || exit 6
timeout -k 10 300 python scripts/profile_worker.py 4096 > gpurun_out/${T}_worker_profile.log 2>&1 || exit 7
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 8
echo ALL_RC=0
