#!/usr/bin/env python3
"""A/B timing of K1 scan variants x resident workgroups per CU, interleaved
rounds in one process (cdna_hip_programming.md 5.4 rule 24).  Tooling only.

Usage: python tools/scan_ab.py [--rows 1000000 --dim 128 --k 10 --queries 64 --rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# A/B knobs (wvgx_set_tuning) exist only in the tools build: make -C weaviate_amd/csrc tools
os.environ.setdefault("WVG_LIB", os.path.join(ROOT, "tools", "libwvgpu_tools.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--gpcu", default="2,3,4,6")
    ap.add_argument("--metric", type=int, default=0)
    ap.add_argument("--pipelined", action="store_true")
    ap.add_argument("--modes", default="1", help="pipelined: 0 = launch per query, 1 = query-stream launch")
    args = ap.parse_args()
    import torch

    from weaviate_amd._lib import KIND_F32, check
    from weaviate_amd.device import Context, Corpus

    ctx = Context(0)
    lib = ctx.lib
    lib.wvgx_set_tuning.restype = ctypes.c_int
    lib.wvgx_set_tuning.argtypes = [ctypes.c_int, ctypes.c_int]
    n, d, k, Q = args.rows, args.dim, args.k, args.queries
    c = Corpus(ctx, KIND_F32, args.metric, d, n)
    c.fill_synthetic(42, n, 0)
    dev = torch.device("cuda:0")
    qs = torch.from_numpy(np.random.default_rng(43).uniform(-1, 1, (Q, d)).astype(np.float32)).to(dev)
    ids = torch.empty((Q, k), dtype=torch.int64, device=dev)
    dists = torch.empty((Q, k), dtype=torch.float32, device=dev)
    cnt = torch.empty(Q, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    ref_ids = None
    ref_d = None
    results = {}
    for rnd in range(args.rounds):
        for v in [int(x) for x in args.variants.split(",")]:
            for g, mode in [(int(x), int(y)) for x in args.gpcu.split(",") for y in args.modes.split(",")]:
                lib.wvgx_set_tuning(0, v)
                lib.wvgx_set_tuning(1, g)
                lib.wvgx_set_tuning(2, mode)
                wsb = lib.wvg_search_workspace_size(c.handle, 1, k)
                ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)

                wsb = lib.wvg_search_workspace_size(c.handle, Q, k)
                ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)

                def run():
                    if args.pipelined:
                        check(lib.wvg_search_device_pipelined(c.handle, qs.data_ptr(), Q, k, ids.data_ptr(),
                                                              dists.data_ptr(), cnt.data_ptr(), ws.data_ptr(), wsb,
                                                              stream))
                        return
                    for j in range(Q):
                        check(lib.wvg_search_device(c.handle, qs[j].data_ptr(), 1, k, ids[j].data_ptr(),
                                                    dists[j].data_ptr(), cnt[j].data_ptr(), ws.data_ptr(), wsb,
                                                    stream))

                run()
                torch.cuda.synchronize()
                check(lib.wvg_profile_start(ctx.handle))
                t0 = time.perf_counter()
                run()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                ms, nl = ctypes.c_double(), ctypes.c_uint64()
                check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
                got = ids.cpu().numpy()
                if ref_ids is None:
                    ref_ids = got.copy()
                    ref_d = dists.cpu().numpy().copy()
                ok = bool(np.array_equal(got, ref_ids))
                scan_us = ms.value * 1e3 / nl.value
                rec = {"round": rnd, "variant": v, "groups_per_cu": g, "mode": mode, "scan_us": round(scan_us, 2),
                       "GBps": round(n * d * 4 / (scan_us * 1e-6) / 1e9, 1),
                       "wall_us_per_query": round((t1 - t0) / Q * 1e6, 2),
                       "qps": round(Q / (t1 - t0), 1), "ids_equal": ok,
                       "dists_equal": bool(np.array_equal(dists.cpu().numpy(), ref_d)) if ref_d is not None else True}
                print(json.dumps(rec), flush=True)
                results.setdefault((v, g, mode), []).append(scan_us)
    best = min(results.items(), key=lambda kv: np.median(kv[1]))
    print(json.dumps({"best": {"variant": best[0][0], "groups_per_cu": best[0][1], "mode": best[0][2],
                               "median_scan_us": round(float(np.median(best[1])), 2)}}))


if __name__ == "__main__":
    main()
