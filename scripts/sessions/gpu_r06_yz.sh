#!/bin/bash
# Round 6, sessions y + z in one call: the shipped build's GPU tests, smoke and default bench
# line (gpu_r06_y.sh), then the Kerr switch sweep (gpu_r06_z.sh).
set -o pipefail
bash scripts/sessions/gpu_r06_y.sh || exit $?
bash scripts/sessions/gpu_r06_z.sh || exit $?
echo ALL_RC=0
