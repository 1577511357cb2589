#!/bin/bash
# Round 6, session k: streaming strict mode over two sixths of the validated d4 set (parts A, B
# of 6), and the native compiler's rate by host threads on the box's CPU share.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in $PARTS; do
  timeout -k 10 560 python bench.py --strict-full --part $P --parts 6 > gpurun_out/r06_k_strict_full_6p$P.json 2> gpurun_out/r06_k_strict_full_6p$P.log || { echo "STRICT $P failed"; exit 7; }
done
timeout -k 10 120 python -c "
import sys, time, json
sys.path.insert(0, 'pde-engine_amd')
from pdeval.workload import load_programs
from pdeval import native
_, _, ex = load_programs('force_free_d4_validated')
s = [str(x) for x in ex]
out = {}
for th in (1, 2, 4, 8, 16):
    t0 = time.perf_counter(); native.compile_native(0, s, threads=th); dt = time.perf_counter() - t0
    b0 = time.perf_counter()
    for k in range(0, len(s), 4096): native.compile_native(0, s[k:k + 4096], threads=th)
    db = time.perf_counter() - b0
    out[th] = {'whole_s': round(dt, 3), 'strings_per_s': round(len(s) / dt), 'batches4096_s': round(db, 3)}
print(json.dumps(out))
" > gpurun_out/r06_k_native_threads.json 2>&1 || exit 8
echo ALL_RC=0
