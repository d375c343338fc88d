#!/bin/bash
# Round-5 GPU call K: the in-process HBM read probe (wvg_measure_hbm_read) at
# 2, 16 and 64 GiB -- is config 5's 64 GB scan rate a buffer-size ceiling?
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "
import ctypes, json, sys
sys.path.insert(0, '.')
from weaviate_amd.device import Context
from weaviate_amd._lib import check
ctx = Context(0)
for gib in (2, 16, 64, 2):
    g = ctypes.c_double()
    check(ctx.lib.wvg_measure_hbm_read(ctx.handle, gib << 30, 3, ctypes.byref(g)))
    print(json.dumps({'bytes_gib': gib, 'GBps': round(g.value, 1)}), flush=True)
ctx.close()
" > $O/hbm_probe.jsonl 2> $O/hbm_probe.err || exit 1
