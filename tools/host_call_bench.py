"""Latency of one single-query wvg_search call (1M x 128 L2, k = 10): wall
time per call against the scan kernel's own time (wvg_profile_*), for the
in-launch merge (tuning key 2 = 1, the product) and the scan + merge-kernel
pair (key 2 = 0), coalescer on and off.  Tools build (wvgx_set_tuning).
Usage: python tools/host_call_bench.py [--rows 1000000] [--calls 2000]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("WVG_LIB", os.path.join(ROOT, "tools", "libwvgpu_tools.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--gpcs", default="0", help="K1 workgroups per CU (tuning key 1; 0 = auto): comma list")
    ap.add_argument("--modes", default="1,0", help="tuning key 2: 1 = in-launch merge, 0 = scan + merge kernel")
    ap.add_argument("--coalesce", default="1,0")
    ap.add_argument("--variants", default="0", help="tuning key 25 (query-stream K1): bit 0 = tile-granular ranges, "
                                                   "bit 1 = arrival-counter merge (round 4); comma list")
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    from weaviate_amd._lib import KIND_F32, METRIC_L2, check, fptr, u32ptr, u64ptr
    from weaviate_amd.device import Context, Corpus

    out = {}
    for coalesce in (int(x) for x in a.coalesce.split(",")):
        ctx = Context(0, coalesce=coalesce)
        lib = ctx.lib
        lib.wvgx_set_tuning.restype = ctypes.c_int
        c = Corpus(ctx, KIND_F32, METRIC_L2, a.dim, a.rows)
        c.fill_synthetic(11, a.rows, 0)
        qs = np.random.default_rng(5).uniform(-1, 1, (64, a.dim)).astype(np.float32)
        ids = np.empty(10, np.uint64)
        d = np.empty(10, np.float32)
        cnt = np.empty(1, np.uint32)
        for mode, gpc, var in ((int(m), int(g), int(v)) for m in a.modes.split(",") for g in a.gpcs.split(",")
                               for v in a.variants.split(",")):
            prevv = lib.wvgx_set_tuning(25, var)
            prev = lib.wvgx_set_tuning(2, mode)
            prevg = lib.wvgx_set_tuning(1, gpc)
            for i in range(50):
                check(lib.wvg_search(c.handle, fptr(qs[i % 64]), 1, 10, None, 0, u64ptr(ids), fptr(d), u32ptr(cnt)))
            t0 = time.perf_counter()
            for i in range(a.calls):
                check(lib.wvg_search(c.handle, fptr(qs[i % 64]), 1, 10, None, 0, u64ptr(ids), fptr(d), u32ptr(cnt)))
            wall = (time.perf_counter() - t0) / a.calls
            check(lib.wvg_profile_start(ctx.handle))
            for i in range(200):
                check(lib.wvg_search(c.handle, fptr(qs[i % 64]), 1, 10, None, 0, u64ptr(ids), fptr(d), u32ptr(cnt)))
            ms = ctypes.c_double()
            nl = ctypes.c_uint64()
            check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
            kern_us = ms.value * 1e3 / max(1, nl.value)
            key = f"coalesce{coalesce}_inlaunch{mode}_gpc{gpc}_streamvar{var}"
            out[key] = {
                "us_per_call": round(wall * 1e6, 2), "scan_kernel_us": round(kern_us, 2),
                "host_and_gap_us": round(wall * 1e6 - kern_us, 2), "profiled_launches": nl.value,
                "frac_of_8TBs": round(a.rows * a.dim * 4 / wall / 8e12, 4)}
            lib.wvgx_set_tuning(2, prev)
            lib.wvgx_set_tuning(25, prevv)
            lib.wvgx_set_tuning(1, prevg)
            print(json.dumps({key: out[key]}), flush=True)
        c.destroy()
        ctx.close()


if __name__ == "__main__":
    main()
