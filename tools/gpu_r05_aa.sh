#!/bin/bash
# Round-5 GPU call AA: the coalescer GPU tests incl. the mixed-k prefix test.
set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_coalesce.py > $O/tests.log 2>&1 || exit 1
