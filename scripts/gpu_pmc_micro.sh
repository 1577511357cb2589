#!/bin/bash
# PMC passes over the per-opcode microbenchmark (one validate call per program, --reps 1);
# each pass its own rocprofv3 run, kernel-trace only.  Summarize with scripts/pmc_micro.py.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmcm${TAG}
mkdir -p $O
M="python3 scripts/microbench.py --n ${N:-65536} --reps 1 --problem ${PROBLEM:-force_free} --set ${SET:-default}"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVE_CYCLES --output-format csv -d $O/p1 -o run -- $M > $O/p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_IFETCH SQ_ACTIVE_INST_ANY --output-format csv -d $O/p2 -o run -- $M > $O/p2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT --output-format csv -d $O/p3 -o run -- $M > $O/p3.log 2>&1
echo "PMCM_RC=$?"
