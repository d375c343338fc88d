#!/bin/bash
# Round-5 GPU call E (after the scratch fix): query-stream A/B on single-query
# host calls (tools build, key 25), the headline bench (no legs), the host-API
# leg (latency percentiles, filtered), then the PQ ADC K8e timing + counters.
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/host_call_bench.py --calls 3000 --modes 1 --coalesce 1 --variants 0,1,2,3,0 > $O/stream_ab.jsonl 2> $O/stream_ab.err || exit 1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --configs '' --scale-legs '' --no-cpu-baseline > $O/bench_headline.json 2> $O/bench_headline.err || exit 2
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
bash tools/gpu_r05_d.sh || exit 4
