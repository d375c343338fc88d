# HBM bytes (FETCH_SIZE) and L2 hits of the K3b kernel per variant.
# Usage (on the GPU box): bash tools/fetch_ab.sh <gemm_kernel>:<lockstep_lag> ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "$@"; do
V="${spec%%:*}"; L="${spec#*:}"; tag="fab${V}_${L}"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-include-regex gemm --output-format csv -d gpurun_out/$tag -- python3 tools/bench_configs.py --only batched --gemm-kernel $V --gemm-lockstep $L > gpurun_out/$tag.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/$tag
grep tflops gpurun_out/$tag.log | cut -c1-200
done
