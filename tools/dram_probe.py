#!/usr/bin/env python3
"""Runs the headline kernel (query-stream K1, wvg_search_device_pipelined) on
one corpus for a fixed number of launches, for rocprofv3 PMC passes (tooling
only, not product): which bytes reach the fabric (FETCH_SIZE) and DRAM
(TCC_EA0_RDREQ_DRAM) with the Infinity-Cache reuse of the default context
(--reuse 1) and without it (--reuse 0: wvg_options.cache_reuse = 0).
--rows 125000 (64 MB, fits the 256 MiB Infinity Cache) calibrates whether a
counter sees Infinity-Cache hits.

    rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum --kernel-trace \
        -d gpurun_out/x -o x -- python tools/dram_probe.py --rows 1000000 --reuse 1
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--reuse", type=int, default=1)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--launches", type=int, default=12)
    a = ap.parse_args()
    import ctypes

    import torch

    torch.cuda.init()
    from weaviate_amd._lib import KIND_F32, METRIC_L2, check
    from weaviate_amd.device import Context, Corpus

    dev = torch.device("cuda:0")
    ctx = Context(0, cache_reuse=a.reuse)
    lib = ctx.lib
    n, d, B, k = a.rows, a.dim, a.batch, 10
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, (n + 63) // 64 * 64)
    c.fill_synthetic(42, n, 0)
    qs = torch.from_numpy(np.random.default_rng(43).uniform(-1, 1, (64, d)).astype(np.float32)).to(dev)
    wsb = lib.wvg_search_workspace_size(c.handle, B, k)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    oi = torch.empty((B, k), dtype=torch.int64, device=dev)
    od = torch.empty((B, k), dtype=torch.float32, device=dev)
    oc = torch.empty(B, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    check(lib.wvg_profile_start(ctx.handle))
    for s in range(a.launches):
        check(lib.wvg_search_device_pipelined(c.handle, qs[(s * B) % 64].data_ptr(), B, k, oi.data_ptr(),
                                              od.data_ptr(), oc.data_ptr(), ws.data_ptr(), wsb, st))
    ms, nl = ctypes.c_double(), ctypes.c_uint64()
    check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
    check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), st))
    per = ms.value / max(1, nl.value)
    print(json.dumps({"rows": n, "dim": d, "reuse": a.reuse, "batch": B, "launches": int(nl.value),
                      "avg_launch_ms": round(per, 4),
                      "algorithmic_GBps": round(n * d * 4 * B / (per / 1e3) / 1e9, 1)}), flush=True)
    c.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
