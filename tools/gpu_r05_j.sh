#!/bin/bash
# Round-5 GPU call J: config-5 slab A/B (K1 workgroups per CU x k) on 125M x 128, then
# the host-API leg with native caller threads (tools/host_calls.c).
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
timeout -k 10 400 python -u tools/slab_ab.py > $O/slab_ab.jsonl 2> $O/slab_ab.err || exit 1
unset WVG_LIB
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
" > $O/host_api_native.json 2> $O/host_api_native.err || exit 2
