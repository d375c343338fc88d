#!/bin/bash
# PMC passes for the headline kernel's fabric / DRAM traffic (tools/dram_probe.py),
# one counter set per rocprofv3 run.  Usage: bash tools/gpu_pmc_dram.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/pmc_dram}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, rows, reuse, counters...
    local name=$1 rows=$2 reuse=$3; shift 3
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o "$name" -- \
        python tools/dram_probe.py --rows "$rows" --reuse "$reuse" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run fetch_reuse1 1000000 1 FETCH_SIZE
run fetch_reuse0 1000000 0 FETCH_SIZE
run dram_reuse1 1000000 1 TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum
run dram_reuse0 1000000 0 TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum
run dram_64mb 125000 1 TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum
run fetch_64mb 125000 1 FETCH_SIZE
echo pmc done
