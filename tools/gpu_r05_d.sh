#!/bin/bash
# Round-5 GPU call D: PQ ADC K8e -- timing of ring 4 (product) vs ring 8 at
# 100M codes, then counter passes of both at 25M codes (tools/pmc_passes.sh).
set -o pipefail
O=gpurun_out/r05e/pq
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
timeout -k 10 200 python -u tools/pq_scan_probe.py --rows 100000000 --variants 0,52,53,0 > $O/pq_timing_100m.jsonl 2> $O/pq_timing.err || exit 1
for v in 0 52; do
  PQV=$v timeout -k 10 900 bash tools/pmc_passes.sh $O/pmc_v$v scan_pq32_wide python3 tools/pq_scan_probe.py --rows 25000000 --queries 32 --variants $v > $O/pmc_v$v.log 2>&1 || exit 2
done
