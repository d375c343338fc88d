#!/bin/bash
# Round-5 GPU call AE: config-2 batch time by K3b pilot size (tuning key 23, tiles),
# two alternating rounds (tools build, WVG_TUNING).
set -o pipefail
O=gpurun_out/r05ae
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
for t in 64 128 256 512 64 128 256 512; do
  WVG_TUNING=23:$t timeout -k 10 300 python -u tools/screen_bench.py --reps 3 --exact 0 > $O/t$t.jsonl 2>> $O/err.txt || exit 1
  echo "pilot=$t $(tail -1 $O/t$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin)["screen"]; print(d["batch_ms"], d["scoring_kernel_ms"])')" >> $O/summary.txt
done
