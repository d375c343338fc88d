#!/usr/bin/env bash
# K3 profile passes (kernel trace + SQ / TCP / TCC counter passes) for one
# variant: tools/k3prof.sh <gemm_kernel variant> [scale]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=${1:-0}; S=${2:-0.2}
O=gpurun_out/k3v$V
mkdir -p $O
CMD="python3 tools/bench_configs.py --only batched --scale $S --gemm-kernel $V"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- $CMD > $O/trace.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-include-regex gemm --output-format csv -d $O/pmc1 -- $CMD > $O/pmc1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex gemm --output-format csv -d $O/pmc2 -- $CMD > $O/pmc2.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex gemm --output-format csv -d $O/pmc3 -- $CMD > $O/pmc3.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm --output-format csv -d $O/pmc4 -- $CMD > $O/pmc4.log 2>&1
