#!/bin/bash
# Round-5 GPU call N: single-query host calls by K1 workgroups per CU (tuning key 1)
# on the query-stream in-launch path (key 25 = 1, the product).
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/host_call_bench.py --calls 3000 --modes 1 --coalesce 1 --variants 1 --gpcs 0,2,3,4,0 > $O/gpc_ab.jsonl 2> $O/gpc_ab.err || exit 1
