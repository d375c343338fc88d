#!/bin/bash
# Round-5 GPU call G: K3d vs K3e counter passes (MFMA busy, LDS activity, waits) on
# the config-2 batch (tools build; screen_bench over 10M x 768 cosine, one batch).
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
export WVG_LIB=tools/libwvgpu_tools.so
for v in 0 2; do
  WVG_SCREEN_VARIANT=$v PMC_MFMA=1 timeout -k 10 900 bash tools/pmc_passes.sh $O/pmc_v$v screen_ar python3 tools/screen_bench.py --reps 1 --exact 0 > $O/pmc_v$v.log 2>&1 || exit 1
done
