#!/bin/bash
# Round-5 GPU call S: the coalescer with batch gathering under 1-64 native callers,
# and the coalescer / robustness GPU tests.
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
WVG_LIB=tools/libwvgpu_tools.so timeout -k 10 300 python -u tools/coalesce_probe.py > $O/coalesce.jsonl 2> $O/coalesce.err || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_coalesce.py tests/test_gpu_robustness.py > $O/tests.log 2>&1 || exit 2
