#!/bin/bash
# Round 6, session i: the streaming strict mode over a third of the validated d4 set (--part P)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${PART:-0}
timeout -k 10 1080 python bench.py --strict-full --part $P --parts 3 > gpurun_out/r06_i_strict_full_p$P.json 2> gpurun_out/r06_i_strict_full_p$P.log || { echo "STRICT failed"; exit 7; }
echo ALL_RC=0
