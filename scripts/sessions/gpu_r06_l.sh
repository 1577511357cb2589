#!/bin/bash
# Round 6, session l: same-box A/B of the frequency-ordered dispatch (lib/libpdeval_f0.so =
# PD_DISPATCH_FREQ=0), GPU tests on the default build, the native compiler by host threads.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06_l
for k in 1 2; do
  for v in "" _f0; do
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --problem kerr_magnetosphere --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_kerr${v}_${k}.log 2>&1 || exit 8
    PDEVAL_LIB=pde-engine_amd/lib/libpdeval${v}.so timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/${T}_ab_ff${v}_${k}.log 2>&1 || exit 7
  done
done
timeout -k 10 700 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "PYTEST_RC=$?"
grep -q " passed" gpurun_out/${T}_pytest_gpu.log || exit 5
grep -q " failed" gpurun_out/${T}_pytest_gpu.log && exit 5
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
" > gpurun_out/${T}_native_threads.json 2>&1 || exit 9
echo ALL_RC=0
