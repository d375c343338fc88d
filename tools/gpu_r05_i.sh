#!/bin/bash
# Round-5 GPU call I: query-stream merge A/B on the device-pipelined path (tools
# build, WVG_STREAM_VARIANT: 1 = per-list hand-offs (default), 3 = arrival counter)
# -- the headline line (16 x 1M, k = 10) and config 5's 125M slab (8 queries, k = 100).
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
for v in 1 3 1 3; do
  WVG_STREAM_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --configs slab --scale-legs '' --no-cpu-baseline > $O/bench_v$v.json 2>> $O/bench.err || exit 1
  python3 -c "
import json,sys
d=[json.loads(l) for l in open('$O/bench_v$v.json') if l.startswith('{')][-1]
s=d['configs']['config5_slab_125m_x_128']
print('v$v', d['value'], d['roofline']['avg_launch_us'], s['scan_ms_per_query'], s['roofline']['frac'])
" >> $O/summary.txt || exit 2
done
