#!/bin/bash
# PMC passes over K3c (tools/screen_bench.py, 10M x 768 cosine, 1024 queries), one
# counter set per rocprofv3 run.  Usage: bash tools/gpu_pmc_screen.sh <outdir> [rows]
set -euo pipefail
OUT=${1:-gpurun_out/pmc_screen}
ROWS=${2:-10000000}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o "$name" -- \
        python tools/screen_bench.py --rows "$ROWS" --reps 2 --exact 0 > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_VALU
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
run tcc TCC_HIT_sum TCC_MISS_sum
run fetch FETCH_SIZE
echo pmc done
