#!/bin/bash
# Round-5 GPU call X: K8e at 16 waves per CU (variants 55 = ring 4, 56 = ring 2) against
# the product (8 waves, ring 4), 100M codes, single queries (tools build, key 7).
set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
timeout -k 10 400 python -u tools/pq_scan_probe.py --rows 100000000 --variants 0,55,56,0,55,56 > $O/pq16.jsonl 2> $O/pq16.err || exit 1
