#!/bin/bash
# Round 4, session f: the graph-path equality test and the worker tag test with and without
# graphs, then the new symbolic-mode GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_f}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_symbolic.py::test_small_batch_graph_path_equals_direct > gpurun_out/${T}_graph.log 2>&1; echo "GRAPH_RC=$?"
PDEVAL_GRAPH=0 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_worker.py::test_worker_queue_protocol_and_tags > gpurun_out/${T}_tags_nograph.log 2>&1; echo "TAGS_NOGRAPH_RC=$?"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_symbolic.py > gpurun_out/${T}_symbolic.log 2>&1; echo "SYM_RC=$?"
echo ALL_DONE
