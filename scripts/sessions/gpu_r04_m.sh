#!/bin/bash
# Round 4, session m: bench.py's worker leg alone (pipelined + the multi-process pool).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_m}
timeout -k 10 600 python - > gpurun_out/${T}_worker_leg.log 2>&1 <<'PY' || exit 3
import json, sys, os
sys.path.insert(0, os.getcwd())
import bench
from pdeval import hostpool
hostpool.start()
from pdeval.workload import load_programs
_, _, exprs = load_programs('force_free_d4_validated')
print(json.dumps(bench.worker_throughput(exprs)), flush=True)
PY
echo ALL_RC=0
