#!/bin/bash
# Round-5 GPU call AB: host time of one caller's single-query path (tools build).
set -o pipefail
O=gpurun_out/r05ab
mkdir -p $O
export TMPDIR=/tmp
WVG_LIB=tools/libwvgpu_tools.so timeout -k 10 300 python -u tools/coalesce_probe.py --callers 1,1 > $O/single_host.jsonl 2> $O/single_host.err || exit 1
