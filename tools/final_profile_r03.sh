#!/usr/bin/env bash
# Round-3 end measurement set (run on the GPU box through gpurun):
#   bench      bench.py default (the driver's command)                  -> $O/bench.json
#   trace      the same under rocprofv3 --kernel-trace --stats          -> $O/trace
#   pmc_fetch  a separate FETCH_SIZE counter pass of bench.py           -> $O/pmc_fetch
#   screen     K3c / K3b config-2 bench under the kernel trace          -> $O/screen_trace
#   configs    BQ / PQ / slab / rescore configs under the kernel trace  -> $O/configs_trace
#   encode     PQ encode 100M x 128 under the kernel trace              -> $O/encode_trace
#   small      co-scheduled K1 batches + KMeans.Fit under the trace     -> $O/small_trace
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_r03
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <limit> <name> <cmd...>
  local limit=$1 name=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 3 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step 300 bench python3 bench.py
grep '^{' $O/bench.log | tail -1 > $O/bench.json
step 300 trace rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 bench.py --profile-run
step 200 pmc_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -- python3 bench.py --steps 10 --warmup 2 --profile-run
step 240 screen rocprofv3 --kernel-trace --stats --output-format csv -d $O/screen_trace -- python3 tools/screen_bench.py
WVG_LIB=$PWD/tools/libwvgpu_tools.so step 400 configs rocprofv3 --kernel-trace --stats --output-format csv -d $O/configs_trace -- python3 tools/bench_configs.py --only bq,pq,slab,rescore
step 200 encode rocprofv3 --kernel-trace --stats --output-format csv -d $O/encode_trace -- python3 tools/encode_bench.py
step 200 small rocprofv3 --kernel-trace --stats --output-format csv -d $O/small_trace -- python3 tools/small_batch_bench.py
echo done
