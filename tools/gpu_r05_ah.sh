#!/bin/bash
# Round-5 GPU call AH: the coalescer's gathering window cap (tuning key 28: the last
# batch's run time / this) with K1Q batches, 1-64 native callers (tools build).
set -o pipefail
O=gpurun_out/r05ah
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
for dv in 8 2 4 8 2; do
  WVG_TUNING=28:$dv timeout -k 10 300 python -u tools/coalesce_probe.py --callers 1,4,16,64 > $O/div$dv.jsonl 2>> $O/err.txt || exit 1
  grep callers $O/div$dv.jsonl | python3 -c "
import json,sys
print('div$dv', [(d['callers'], d['qps'], d['p50_us'], d['p99_us'], d['mean_batch']) for d in map(json.loads, sys.stdin)])
" >> $O/summary.txt || exit 2
done
