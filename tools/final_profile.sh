#!/usr/bin/env bash
# Round-end measurement set (run on the GPU box through gpurun):
#   1. bench.py default (the driver's command)            -> gpurun_out/final/bench.json
#   2. the same under rocprofv3 --kernel-trace --stats     -> gpurun_out/final/trace
#   3. a separate FETCH_SIZE counter pass of bench.py      -> gpurun_out/final/pmc_fetch
#   4. the other configs (batched MFMA, BQ, PQ, 1B slab) with kernel stats
#   5. a counter pass of the PQ ADC kernels (K8b vs K8) at 25M rows
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <limit> <name> <cmd...>
  local limit=$1 name=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 5 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step 300 bench python3 bench.py
grep '^{' $O/bench.log | tail -1 > $O/bench.json
step 300 trace rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 bench.py --no-cpu-baseline
step 300 pmc_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
step 600 configs rocprofv3 --kernel-trace --stats --output-format csv -d $O/configs_trace -- python3 tools/bench_configs.py
step 120 pmc_pq rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/pmc_pq -- python3 tools/bench_configs.py --only pq --scale 0.25
echo done
