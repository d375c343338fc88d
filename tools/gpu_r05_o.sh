#!/bin/bash
# Round-5 GPU call O: lone in-launch queries at two K1 workgroups per CU (the new
# default, key 1 = 0) against one (key 1 = 1); single-query GPU tests.
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/host_call_bench.py --calls 3000 --modes 1 --coalesce 1 --variants 1 --gpcs 0,1,0,1 > $O/gpc_ab.jsonl 2> $O/gpc_ab.err || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_coalesce.py tests/test_gpu_robustness.py tests/test_gpu_parity.py tests/test_gpu_boundary.py > $O/tests.log 2>&1 || exit 2
