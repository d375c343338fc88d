#!/bin/bash
# Round-5 GPU call M: mixed-k coalescing -- the coalescer tests and the host-API leg
# (native callers, mixed-k 16-caller leg).
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_coalesce.py tests/test_gpu_robustness.py > $O/tests.log 2>&1 || exit 1
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
" > $O/host_api.json 2> $O/host_api.err || exit 2
