#!/bin/bash
# Round-5 GPU call C: the full GPU suite on the product library (stream kernel
# with row-granular ranges + per-list hand-offs, filtered in-launch singles),
# the query-stream A/B (tuning key 25) on single-query host calls, and K3e
# (32x32x16 MFMA screen, tools build) timed and checked against the exact path.
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/host_call_bench.py --calls 3000 --modes 1 --coalesce 1 --variants 0,1,2,3 > $O/stream_ab.jsonl 2> $O/stream_ab.err || exit 2
WVG_LIB=tools/libwvgpu_tools.so WVG_SCREEN_VARIANT=0 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 0 > $O/screen_k3d.jsonl 2> $O/screen_k3d.err || exit 3
WVG_LIB=tools/libwvgpu_tools.so WVG_SCREEN_VARIANT=2 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 1 > $O/screen_k3e.jsonl 2> $O/screen_k3e.err || exit 4
WVG_LIB=tools/libwvgpu_tools.so WVG_SCREEN_VARIANT=2 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_screen.py > $O/screen_k3e_tests.log 2>&1 || exit 5
