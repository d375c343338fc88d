#!/bin/bash
# Round-5 GPU call B: single-query host-call cost split (wall vs kernel), a
# kernel trace of back-to-back single calls (gaps between launches), and the
# bench's host-API leg (latency percentiles, filtered legs) on the product library.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/host_call_bench.py --calls 3000 --modes 1 --coalesce 1,0 > $O/host_call.jsonl 2> $O/host_call.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o single -- python3 tools/host_call_bench.py --calls 400 --modes 1 --coalesce 1 > $O/trace.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
from oracle import wv_oracle as orc
from weaviate_amd.device import Context
torch.cuda.init()
ctx = Context(0)
print(json.dumps(bench.config_host_api(ctx, orc)), flush=True)
ctx.close()
" > $O/host_api.json 2> $O/host_api.err || exit 3
