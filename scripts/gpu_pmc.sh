#!/bin/bash
# PMC counter passes (each its own rocprofv3 run, kernel-trace only) on a short bench.
set -o pipefail
D=gpurun_out/pmc${PMC_TAG}
mkdir -p $D
export TMPDIR=/tmp
N=${N:-262144}
B="python bench.py --steps 1 --warmup 0 --n $N --no-cpu --no-extras --problem ${PROBLEM:-force_free}"
rocprofv3 -L > $D/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- $B > $D/trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $D/sq1 -o run -- $B > $D/sq1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $D/sq2 -o run -- $B > $D/sq2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $B > $D/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $B > $D/write.log 2>&1
echo "PMC_RC=$?"
