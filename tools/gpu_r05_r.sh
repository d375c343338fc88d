#!/bin/bash
# Round-5 GPU call R: the coalescer under 1-64 native callers (batch counters).
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
timeout -k 10 300 python -u tools/coalesce_probe.py > $O/coalesce.jsonl 2> $O/coalesce.err || exit 1
