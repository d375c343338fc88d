#!/bin/bash
# Round-5 GPU call V: the K1 cache tail (WVG_K1_TAIL, /256 of each pass read with the
# default policy; 0 = auto = 160 at 1M x 128) on the headline at two workgroups per CU.
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
for t in 0 120 200 240 256 0; do
  WVG_K1_TAIL=$t timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --configs '' --scale-legs '' --no-cpu-baseline > $O/b$t.json 2>> $O/b.err || exit 1
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/b$t.json') if l.startswith('{')][-1]
print('tail$t', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])
" >> $O/summary.txt || exit 2
done
