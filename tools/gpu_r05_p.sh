#!/bin/bash
# Round-5 GPU call P: the screen pilot (tuning key 26 / WVG_SCREEN_SP: tiles of a
# bf16-screen pilot + exact seed, replacing the 0.76 ms K3b pilot) on the config-2
# batch -- bit-identity against the exact path, timing by pilot size, screen tests.
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
WVG_SCREEN_SP=512 timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 1 > $O/sp512_exact.jsonl 2> $O/sp512_exact.err || exit 1
for sp in 0 512 2048 8192 0 512; do
  WVG_SCREEN_SP=$sp timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 0 > $O/sp$sp.jsonl 2> $O/sp$sp.err || exit 2
  echo "sp=$sp $(tail -1 $O/sp$sp.jsonl)" >> $O/summary.txt
done
WVG_SCREEN_SP=512 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_screen.py > $O/screen_tests_sp512.log 2>&1 || exit 3
