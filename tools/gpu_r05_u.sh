#!/bin/bash
# Round-5 GPU call U: two K1 workgroups per CU as the auto rule for d <= 128 --
# headline, small co-scheduled batches and a 20M x 128 scan against one per CU
# (tools build, WVG_GROUPS_PER_CU=1), lone queries, and the flat GPU tests.
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --configs '' --scale-legs '' --no-cpu-baseline > $O/headline.json 2> $O/headline.err || exit 1
timeout -k 10 300 python -u tools/small_batch_bench.py --nqs 2,8,16,31 --fit 0 > $O/small_auto.jsonl 2> $O/small_auto.err || exit 2
WVG_LIB=tools/libwvgpu_tools.so WVG_GROUPS_PER_CU=1 timeout -k 10 300 python -u tools/small_batch_bench.py --nqs 2,8,16,31 --fit 0 > $O/small_one.jsonl 2> $O/small_one.err || exit 3
WVG_LIB=tools/libwvgpu_tools.so timeout -k 10 300 python -u tools/slab_ab.py --rows 20000000 --variants 0:10,1:10,0:10,1:10 > $O/scan20m.jsonl 2> $O/scan20m.err || exit 4
WVG_LIB=tools/libwvgpu_tools.so timeout -k 10 300 python -u tools/host_call_bench.py --calls 3000 --modes 1 --coalesce 1 --variants 1 --gpcs 0,1 > $O/single.jsonl 2> $O/single.err || exit 5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_coalesce.py tests/test_gpu_robustness.py tests/test_gpu_dist.py tests/test_gpu_boundary.py > $O/tests.log 2>&1 || exit 6
