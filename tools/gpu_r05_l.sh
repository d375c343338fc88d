#!/bin/bash
# Round-5 GPU call L: BQ K5 scan (100M x 1536, top-200) by workgroups per CU, and
# the PQ K8e probe for comparison on the same box.
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
timeout -k 10 400 python -u tools/bq_scan_probe.py > $O/bq_gpc.jsonl 2> $O/bq_gpc.err || exit 1
