#!/bin/bash
# Round-5 GPU call Y: K3g (two 4-wave workgroups of 64 queries per CU, each with its own
# ring and barrier; tools variant 4) checked bit for bit against the exact path on the
# config-2 batch, timed against K3d, the screen tests on K3g, and one counter pass set.
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
WVG_SCREEN_VARIANT=4 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 1 > $O/screen_k3g.jsonl 2> $O/screen_k3g.err || exit 1
WVG_SCREEN_VARIANT=0 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 0 > $O/screen_k3d.jsonl 2> $O/screen_k3d.err || exit 2
WVG_SCREEN_VARIANT=4 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 0 > $O/screen_k3g_b.jsonl 2> $O/screen_k3g_b.err || exit 3
WVG_SCREEN_VARIANT=4 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_screen.py > $O/screen_k3g_tests.log 2>&1 || exit 4
WVG_SCREEN_VARIANT=4 PMC_MFMA=1 timeout -k 10 900 bash tools/pmc_passes.sh $O/pmc_v4 screen_ar python3 tools/screen_bench.py --reps 1 --exact 0 > $O/pmc_v4.log 2>&1 || exit 5
