#!/bin/bash
# Round-5 GPU call A: single-query tagged-records stress + A/B against the
# round-4 layout, the single-query GPU tests, then the bench's strong-scaling
# legs at N = 1 and as a 2-rank rehearsal on one GPU.
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 env WVG_LIB=tools/libwvgpu_tools.so python -u tools/single_query_stress.py --modes 0,2,4,6 \
    > $O/stress.jsonl 2> $O/stress.err || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_coalesce.py tests/test_gpu_robustness.py tests/test_gpu_boundary.py \
    "tests/test_gpu_reference_ports.py::test_concurrent_search_while_writing" > $O/tests.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --configs '' --no-cpu-baseline \
    > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
timeout -k 10 500 python -u bench.py --gpus 2 --share-gpu --steps 10 --warmup 2 \
    > $O/bench_n2_share.json 2> $O/bench_n2_share.err || exit 4
