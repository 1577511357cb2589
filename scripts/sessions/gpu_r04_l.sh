#!/bin/bash
# Round 4, session l: the worker's host steps by function; the inline split with the early
# double-double tier limited to batches of >= 1,024.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_l}
timeout -k 10 400 python scripts/profile_worker.py 4096 > gpurun_out/${T}_worker_profile.log 2>&1 || exit 3
timeout -k 10 300 python scripts/profile_inline.py --n 2000 > gpurun_out/${T}_inline.log 2>&1 || exit 4
echo ALL_RC=0
