#!/usr/bin/env python3
"""A/B of the single-query K1 scan at a given dimension: K1 resident
workgroups per CU (tuning key 1) on an N x d fp32 cosine corpus, scan time
from the HIP events bound to each scan dispatch.

Usage: python tools/k1_dim_ab.py [--rows 10000000] [--dim 768] [--gpc 1,2,3,4]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# A/B knobs (wvgx_set_tuning) exist only in the tools build: make -C weaviate_amd/csrc tools
os.environ.setdefault("WVG_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libwvgpu_tools.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--gpc", default="1,2,3,4")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--metric", default="cosine", choices=["cosine", "l2"])
    args = ap.parse_args()
    import torch

    torch.cuda.init()
    from weaviate_amd._lib import KIND_F32, METRIC_COSINE, METRIC_L2
    from weaviate_amd.device import Context, Corpus

    ctx = Context(0)
    lib = ctx.lib
    lib.wvgx_set_tuning.restype = ctypes.c_int
    lib.wvgx_set_tuning.argtypes = [ctypes.c_int, ctypes.c_int]
    n, d = args.rows, args.dim
    c = Corpus(ctx, KIND_F32, METRIC_COSINE if args.metric == "cosine" else METRIC_L2, d, n)
    c.fill_synthetic(42, n, 0)
    qs = np.random.default_rng(43).uniform(-1, 1, (args.reps, d)).astype(np.float32)
    ref = None
    for rnd in range(2):
        for g in [int(x) for x in args.gpc.split(",")]:
            old = lib.wvgx_set_tuning(1, g)
            c.search(qs[0], 10)
            lib.wvg_profile_start(ctx.handle)
            t0 = time.perf_counter()
            out = [c.search(q, 10) for q in qs]
            wall = (time.perf_counter() - t0) / len(qs)
            ms, nl = ctypes.c_double(), ctypes.c_uint64()
            lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl))
            lib.wvgx_set_tuning(1, old)
            scan_s = ms.value / 1e3 / max(1, nl.value)
            ids = np.stack([o[0][0] for o in out])
            same = True if ref is None else bool(np.array_equal(ids, ref))
            ref = ids if ref is None else ref
            print(json.dumps({"rows": n, "dim": d, "groups_per_cu": g, "round": rnd, "scan_ms": round(scan_s * 1e3, 3),
                              "GBps": round(n * d * 4 / scan_s / 1e9, 1), "qps": round(1 / wall, 1),
                              "ids_same_as_first": same}), flush=True)
    c.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
