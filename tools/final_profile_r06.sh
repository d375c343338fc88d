#!/usr/bin/env bash
# Round-6 measurement set (run on the GPU box through gpurun; the tools library
# must travel with the tree for the counter passes):
#   bench      bench.py default (the driver's command)                  -> $O/bench.json
#   trace      bench.py under rocprofv3 --kernel-trace --stats, compared with
#              the line's own events by tools/trace_launch_avg.py        -> $O/trace, trace_vs_events.json
#   pmc_fetch  FETCH_SIZE of the headline (its own pass)                 -> $O/pmc_fetch_summary.txt
#   pmc_k5 / pmc_k8e / pmc_k3i   counter passes (tools/pmc_passes.sh) of
#              the BQ scan, the PQ ADC scan and the int8 screen           -> $O/pmc_*/summary.txt
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_r06
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
step 420 bench python3 bench.py
grep '^{' $O/bench.log | tail -1 > $O/bench.json
step 700 trace rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py
grep '^{"metric"' $O/trace.log | tail -1 > $O/trace_bench.json
python3 tools/trace_launch_avg.py "$(find $O/trace -name '*kernel_trace.csv' | head -1)" $O/trace_bench.json \
  --keep $O/trace_headline_dispatches.csv > $O/trace_vs_events.json
cat $O/trace_vs_events.json
step 200 pmc_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 10 --warmup 2 --profile-run --configs "" --no-cpu-baseline
python3 tools/pmc_summary.py $O/pmc_fetch --match scan_f32_stream > $O/pmc_fetch_summary.txt
export WVG_LIB=tools/libwvgpu_tools.so
timeout -k 10 400 tools/pmc_passes.sh $O/pmc_k5 scan_bq_kernel python3 tools/bq_scan_probe.py --gpc 0 --queries 8 > $O/pmc_k5.log 2>&1 || exit $?
timeout -k 10 400 tools/pmc_passes.sh $O/pmc_k8e scan_pq32_wide python3 tools/pq_scan_probe.py --variants 0 --queries 16 > $O/pmc_k8e.log 2>&1 || exit $?
PMC_MFMA=1 timeout -k 10 600 tools/pmc_passes.sh $O/pmc_k3i screen_i8_kernel python3 tools/screen_bench.py --screens int8 --exact 0 --reps 2 > $O/pmc_k3i.log 2>&1 || exit $?
find $O -name '*kernel_trace.csv' -size +4M -delete
echo done
