#!/bin/bash
# Round-5 GPU call AF: the coalescer with gathering after batches of >= 4 under
# 1-64 native callers, and the coalescer / robustness GPU tests.
set -o pipefail
O=gpurun_out/r05af
mkdir -p $O
export TMPDIR=/tmp
WVG_LIB=tools/libwvgpu_tools.so timeout -k 10 300 python -u tools/coalesce_probe.py --callers 1,2,3,4,16,32,64 > $O/coalesce.jsonl 2> $O/coalesce.err || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_coalesce.py tests/test_gpu_robustness.py > $O/tests.log 2>&1 || exit 2
