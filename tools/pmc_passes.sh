#!/usr/bin/env bash
# Counter passes (one rocprofv3 run each, within the per-block slot limits)
# of one command, restricted to kernels matching a regex, plus a kernel trace.
# Usage (on the GPU box): [PMC_MFMA=1] tools/pmc_passes.sh <outdir> <kernel-regex> <cmd...>
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$1; RX=$2; shift 2
mkdir -p "$O"
run() {
  local name=$1; shift
  local ctr="$1"; shift
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" --output-format csv -d "$O/$name" -- "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -- "$@" > "$O/trace.log" 2>&1 || exit $?
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU" "$@" || exit $?
run p2 "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_LDS" "$@" || exit $?
run p3 "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE" "$@" || exit $?
run p4 "FETCH_SIZE" "$@" || exit $?
if [ "${PMC_MFMA:-0}" = 1 ]; then  # matrix-core kernels: MFMA busy / co-issue and the L2 hit rate
  run p5 "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "$@" || exit $?
  run p6 "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum" "$@" || exit $?
fi
if [ "${PMC_ICACHE:-0}" = 1 ]; then  # instruction-cache misses (large unrolled kernels)
  run p7 "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "$@" || exit $?
fi
python3 tools/pmc_summary.py "$O" > "$O/summary.txt"
cat "$O/summary.txt"
