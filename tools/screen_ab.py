#!/usr/bin/env python3
"""A/B of K3c (the bf16 screen of batched dot / cosine) through the tools
build (tools/libwvgpu_tools.so, -DWVG_TOOLS): row-range length (tuning key
17) and the diagnostics of key 18 (bit 0: no wait for the stage loads, bit 1:
no epilogue compare -- timing only, results are not distances).  10M x 768
cosine, 1024 queries, k = 10 by default; HIP events bound to the scoring
launch.  Usage: WVG_LIB=tools/libwvgpu_tools.so python tools/screen_ab.py
[--ranges 0,16,32,64,256] [--diags 0,1,2,3]"""
import argparse
import time
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ranges", default="0")
    ap.add_argument("--diags", default="0")
    ap.add_argument("--splits", default="1", help="K3c split launch (tuning key 19)")
    ap.add_argument("--variants", default="0", help="screen kernel (tuning key 20): 0 K3d where it applies, 1 K3c")
    ap.add_argument("--pilots", default="16", help="tiles of the exact pilot scan that seeds the bound (tuning key 21; 0 = none)")
    ap.add_argument("--gpilots", default="256", help="tiles of the K3b pilot (tuning keys 23 and 32; 0 = the K1 pilot)")
    ap.add_argument("--spilots", default="0", help="tiles of the screen pilot (tuning key 26; 0 = the K3b pilot)")
    ap.add_argument("--warms", default="32", help="K3i warm-up row blocks per first-phase range (tuning key 29; 0 = equal ranges)")
    ap.add_argument("--seeds", default="3", help="exact seeds (tuning key 22): bit 0 between phases, bit 1 before the final collect")
    ap.add_argument("--warm2s", default="0", help="K3i second-phase row blocks per range (tuning key 30; 0 = rest uniform)")
    ap.add_argument("--rounds", default="1", help="screen ranges in whole CU rounds (tuning key 33)")
    ap.add_argument("--set", default="", help="extra tuning keys for the whole run: key=value,key=value")
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    from weaviate_amd._lib import KIND_F32, METRIC_COSINE, check
    from weaviate_amd.device import Context, Corpus

    dev = torch.device("cuda:0")
    n, d, nq, k = a.rows, a.dim, a.nq, a.k
    q = np.random.default_rng(7).uniform(-1, 1, (nq, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True).astype(np.float32)
    tq = torch.from_numpy(q).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    ctx = Context(0)
    lib = ctx.lib
    lib.wvgx_set_tuning.restype = ctypes.c_int
    for kv in filter(None, a.set.split(",")):
        kk, vv = kv.split("=")
        lib.wvgx_set_tuning(int(kk), int(vv))
    c = Corpus(ctx, KIND_F32, METRIC_COSINE, d, n)
    c.fill_synthetic(42, n, 0)
    ctx.synchronize()
    oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
    od = torch.empty((nq, k), dtype=torch.float32, device=dev)
    oc = torch.empty(nq, dtype=torch.int32, device=dev)
    ref = None
    for rd, w2, wm, spl, gp, sd, pl, vr, sp, rb, dg in [(rd, w2, wm, spl, gp, sd, pl, vr, sp, rb, dg) for rd in [int(x) for x in a.rounds.split(",")] for w2 in [int(x) for x in a.warm2s.split(",")] for wm in [int(x) for x in a.warms.split(",")]
                                       for spl in [int(x) for x in a.spilots.split(",")]
                                       for gp in [int(x) for x in a.gpilots.split(",")]
                                       for sd in [int(x) for x in a.seeds.split(",")]
                                   for pl in [int(x) for x in a.pilots.split(",")]
                               for vr in [int(x) for x in a.variants.split(",")]
                               for sp in [int(x) for x in a.splits.split(",")]
                           for rb in [int(x) for x in a.ranges.split(",")] for dg in [int(x) for x in a.diags.split(",")]]:
        if True:
            lib.wvgx_set_tuning(33, rd)
            lib.wvgx_set_tuning(29, wm)
            lib.wvgx_set_tuning(30, w2)
            lib.wvgx_set_tuning(26, spl)
            lib.wvgx_set_tuning(23, gp)
            lib.wvgx_set_tuning(32, gp)
            lib.wvgx_set_tuning(22, sd)
            lib.wvgx_set_tuning(21, pl)
            lib.wvgx_set_tuning(20, vr)
            lib.wvgx_set_tuning(19, sp)
            lib.wvgx_set_tuning(17, rb)
            lib.wvgx_set_tuning(18, dg)
            wsb = lib.wvg_search_workspace_size(c.handle, nq, k)
            ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)

            def run():
                check(lib.wvg_search_device(c.handle, tq.data_ptr(), nq, k, oi.data_ptr(), od.data_ptr(),
                                            oc.data_ptr(), ws.data_ptr(), wsb, st))

            run()
            torch.cuda.synchronize()
            ctr = (ctypes.c_uint64 * 4)()
            lib.wvgx_screen_counters(ctr, 1)
            check(lib.wvg_profile_start(ctx.handle))
            t0 = time.perf_counter()
            for _ in range(a.reps):
                run()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3 / a.reps
            ms, nl = ctypes.c_double(), ctypes.c_uint64()
            check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
            kern = ms.value / max(1, nl.value)
            lib.wvgx_screen_counters(ctr, 1)
            cnt = [int(x) // a.reps for x in ctr[:4]]
            got = oi.cpu().numpy().copy()
            same = None
            if (dg & (1 | 2 | 4 | 8 | 32 | 64 | 128)) == 0:  # variants whose results are search results
                if ref is None:
                    ref = got
                same = bool(np.array_equal(got, ref))
            print(json.dumps({"round": rd, "warm": wm, "warm2": w2, "screen_pilot": spl, "gemm_pilot": gp, "seed": sd, "pilot": pl, "search_ms": round(wall, 3), "variant": vr, "split": sp, "range_blocks": rb, "diag": dg, "scoring_kernel_ms": round(kern, 3),
                              "tflops": round(2.0 * nq * n * d / (kern / 1e3) / 1e12, 1),
                              "ids_equal_first": same, "wave_row_blocks": cnt[0], "slow_path_blocks": cnt[1],
                              "insert_calls": cnt[2], "exact_groups": cnt[3]}), flush=True)
    lib.wvgx_set_tuning(33, 1)
    lib.wvgx_set_tuning(29, 32)
    lib.wvgx_set_tuning(30, 0)
    lib.wvgx_set_tuning(26, 0)
    lib.wvgx_set_tuning(17, 0)
    lib.wvgx_set_tuning(18, 0)
    lib.wvgx_set_tuning(19, 1)
    lib.wvgx_set_tuning(20, 0)
    lib.wvgx_set_tuning(21, 16)
    lib.wvgx_set_tuning(22, 3)
    lib.wvgx_set_tuning(23, 512)
    lib.wvgx_set_tuning(32, 256)
    c.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
