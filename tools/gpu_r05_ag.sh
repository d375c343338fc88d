#!/bin/bash
# Round-5 GPU call AG: K1Q (co-scheduled batches, Q queries per workgroup; tuning key 27)
# -- small batches by Q (bit-identical to single calls), the coalescer under load, and
# the flat / coalescer / robustness GPU tests on the product build.
set -o pipefail
O=gpurun_out/r05ag
mkdir -p $O
export TMPDIR=/tmp
for q in 0 2 4; do
  WVG_LIB=tools/libwvgpu_tools.so WVG_TUNING=27:$q timeout -k 10 300 python -u tools/small_batch_bench.py --nqs 2,4,8,16,31 --fit 0 > $O/small_q$q.jsonl 2> $O/small_q$q.err || exit 1
  WVG_LIB=tools/libwvgpu_tools.so WVG_TUNING=27:$q timeout -k 10 300 python -u tools/small_batch_bench.py --nqs 4,16 --fit 0 --metric cosine --dim 768 --rows 200000 > $O/small_cos_q$q.jsonl 2> $O/small_cos_q$q.err || exit 2
done
WVG_LIB=tools/libwvgpu_tools.so timeout -k 10 300 python -u tools/coalesce_probe.py --callers 1,4,16,64 > $O/coalesce.jsonl 2> $O/coalesce.err || exit 3
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_coalesce.py tests/test_gpu_robustness.py tests/test_gpu_boundary.py tests/test_gpu_metrics.py > $O/tests.log 2>&1 || exit 4
