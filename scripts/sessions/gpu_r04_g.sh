#!/bin/bash
# Round 4, session g: the whole GPU suite (graph path + split small-batch grid passes +
# symbolic modes), smoke, the inline split and the default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_g}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 5
timeout -k 10 300 python scripts/profile_inline.py --n 2000 > gpurun_out/${T}_inline.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${T}_bench.log 2>&1 || exit 8
echo ALL_RC=0
