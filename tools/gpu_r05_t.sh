#!/bin/bash
# Round-5 GPU call T: the headline 16-query stream launch at one vs two K1 workgroups
# per CU (tools build, WVG_GROUPS_PER_CU; 0 = auto = one).
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
for g in 0 2 0 2; do
  WVG_GROUPS_PER_CU=$g timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --configs '' --scale-legs '' --no-cpu-baseline > $O/b$g.json 2>> $O/b.err || exit 1
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/b$g.json') if l.startswith('{')][-1]
print('gpc$g', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['frac_no_reuse'])
" >> $O/summary.txt || exit 2
done
