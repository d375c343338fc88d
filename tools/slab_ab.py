#!/usr/bin/env python3
"""Config-5 slab A/B (tools build): one 125M x 128 fp32 L2 corpus (64 GB),
8 single-query scans per query-stream launch (wvg_search_device_pipelined),
per variant (K1 workgroups per CU = tuning key 1, 0 = auto; k) the scan time
per query from HIP events bound to the launches, and the ids of query 0
compared with the first variant of the same k.  Prints one JSON line per
variant.  Usage: WVG_LIB=tools/libwvgpu_tools.so python tools/slab_ab.py [--rows 125000000]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("WVG_LIB", os.path.join(ROOT, "tools", "libwvgpu_tools.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=125_000_000)
    ap.add_argument("--variants", default="0:100,2:100,0:10,2:10,0:100")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch

    from oracle import wv_oracle as orc
    from weaviate_amd._lib import KIND_F32, METRIC_L2, check
    from weaviate_amd.device import Context, Corpus

    torch.cuda.init()
    dev = torch.device("cuda:0")
    ctx = Context(0)
    lib = ctx.lib
    lib.wvgx_set_tuning.restype = ctypes.c_int
    n, d, nq = a.rows, 128, 8
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.fill_synthetic(42, n, 0)
    tq = torch.from_numpy(orc.synth_rows(43, 0, nq, d, 0)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    ref = {}
    for spec in a.variants.split(","):
        gpc, k = (int(x) for x in spec.split(":"))
        prev = lib.wvgx_set_tuning(1, gpc)
        ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
        dd = torch.empty((nq, k), dtype=torch.float32, device=dev)
        cc = torch.empty(nq, dtype=torch.int32, device=dev)
        wsb = lib.wvg_search_workspace_size(c.handle, nq, k)
        ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)

        def run():
            check(lib.wvg_search_device_pipelined(c.handle, tq.data_ptr(), nq, k, ids.data_ptr(), dd.data_ptr(),
                                                  cc.data_ptr(), ws.data_ptr(), wsb, st))

        run()
        torch.cuda.synchronize(dev)
        check(lib.wvg_profile_start(ctx.handle))
        for _ in range(a.reps):
            run()
        torch.cuda.synchronize(dev)
        ms, nl = ctypes.c_double(), ctypes.c_uint64()
        check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
        check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), st))
        lib.wvgx_set_tuning(1, prev)
        scan_ms = ms.value / max(1, nl.value) / nq
        got = ids.cpu().numpy()[0].copy()
        same = bool(np.array_equal(ref.setdefault(k, got), got))
        print(json.dumps({"groups_per_cu": gpc, "k": k, "rows": n, "scan_ms_per_query": round(scan_ms, 3),
                          "GBps": round(n * d * 4 / scan_ms / 1e6, 1), "launches": int(nl.value),
                          "same_ids_as_first": same}), flush=True)
    c.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
