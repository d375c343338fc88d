#!/bin/bash
# Round-5 GPU call H: K3f (K3d at two waves per SIMD, tools build) checked bit for
# bit against the exact path on the config-2 batch, timed against K3d, the screen
# tests on K3f, and one counter pass set on K3f.
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
WVG_SCREEN_VARIANT=3 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 1 > $O/screen_k3f.jsonl 2> $O/screen_k3f.err || exit 1
WVG_SCREEN_VARIANT=0 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 0 > $O/screen_k3d.jsonl 2> $O/screen_k3d.err || exit 2
WVG_SCREEN_VARIANT=3 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 0 > $O/screen_k3f_b.jsonl 2> $O/screen_k3f_b.err || exit 3
WVG_SCREEN_VARIANT=3 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_screen.py > $O/screen_k3f_tests.log 2>&1 || exit 4
WVG_SCREEN_VARIANT=3 PMC_MFMA=1 timeout -k 10 900 bash tools/pmc_passes.sh $O/pmc_v3 screen_ar python3 tools/screen_bench.py --reps 1 --exact 0 > $O/pmc_v3.log 2>&1 || exit 5
