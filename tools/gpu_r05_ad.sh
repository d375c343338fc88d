#!/bin/bash
# Round-5 GPU call AD: the K3b pilot's cost by pilot size (tuning key 23 = tiles) on the
# config-2 batch, kernel-traced (tools build, WVG_TUNING).
set -o pipefail
O=gpurun_out/r05ad
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
for t in 64 512 2048; do
  WVG_TUNING=23:$t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$t -o run -- python3 tools/screen_bench.py --reps 2 --exact 0 > $O/t$t.log 2>&1 || exit 1
done
