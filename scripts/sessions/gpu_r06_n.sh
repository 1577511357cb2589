#!/bin/bash
# Round 6, session n: streaming strict mode over sixths of the validated d4 set, one per run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in $PARTS; do
  timeout -k 10 ${LIMIT:-1100} python bench.py --strict-full --part $P --parts 6 > gpurun_out/r06_n_strict_full_6p$P.json 2> gpurun_out/r06_n_strict_full_6p$P.log || { echo "STRICT $P failed"; exit 7; }
done
echo ALL_RC=0
