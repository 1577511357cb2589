#!/bin/bash
# Same-box A/B of the force-free complex pass: the GPU tests, then the bench (2^20 candidates)
# with the lean complex pass (default), its 1-wave/SIMD variant (libpdeval_c1.so) and the
# generic complex kernel (PDEVAL_LEAN_CPLX=0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-abc}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; ok $rc || exit 4
B="python bench.py --steps 3 --warmup 1 --n 1048576 --no-cpu --no-extras"
timeout -k 10 200 $B > gpurun_out/${T}_lean.log 2>&1 || exit 5
PDEVAL_LIB=pde-engine_amd/lib/libpdeval_c1.so timeout -k 10 200 $B > gpurun_out/${T}_lean_c1.log 2>&1 || exit 6
PDEVAL_LEAN_CPLX=0 timeout -k 10 200 $B > gpurun_out/${T}_generic.log 2>&1 || exit 7
echo AB_DONE
