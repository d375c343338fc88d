#!/usr/bin/env bash
# Round-5 end measurement set (run on the GPU box through gpurun):
#   bench      bench.py default (the driver's command)                   -> $O/bench.json
#   trace      bench.py under rocprofv3 --kernel-trace --stats: the line it
#              prints and the trace of the same process (every config's
#              kernels included), compared by tools/trace_launch_avg.py  -> $O/trace, trace_bench.json, trace_vs_events.json
#   pmc_fetch  a separate FETCH_SIZE counter pass of the headline          -> $O/pmc_fetch
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_r05
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
step 600 trace rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py
grep '^{"metric"' $O/trace.log | tail -1 > $O/trace_bench.json
python3 tools/trace_launch_avg.py "$(find $O/trace -name '*kernel_trace.csv' | head -1)" $O/trace_bench.json \
  --keep $O/trace_headline_dispatches.csv > $O/trace_vs_events.json
cat $O/trace_vs_events.json
step 200 pmc_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 10 --warmup 2 --profile-run --configs "" --no-cpu-baseline
python3 tools/pmc_summary.py $O/pmc_fetch --match scan_f32_stream > $O/pmc_fetch_summary.txt
find $O -name '*kernel_trace.csv' -size +4M -delete
echo done
