#!/usr/bin/env python3
"""PQ ADC scan probe (tools build): a PQ corpus of `--rows` random m = 32 x
ks = 256 codes and a synthetic codebook, then `--queries` single-query
searches (k = 10) per ADC variant (tuning key 7; 0 = the product choice, K8e
ring 4; 52 = K8e ring 8; 53 = ring 16), timed with HIP events bound to the
scan launches.  Used alone for timing and under rocprofv3 --pmc for counter
passes (tools/pmc_passes.sh).  Prints one JSON line per variant.
Usage: WVG_LIB=tools/libwvgpu_tools.so python tools/pq_scan_probe.py [--rows 25000000] [--variants 0,52]"""
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
    ap.add_argument("--rows", type=int, default=25_000_000)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--variants", default="0,52")
    ap.add_argument("--gpcs", default="0", help="workgroups per CU (tuning key 1; 0 = the product's choice)")
    a = ap.parse_args()
    from weaviate_amd._lib import KIND_PQ, METRIC_L2, check
    from weaviate_amd.device import Context, Corpus

    ctx = Context(0)
    lib = ctx.lib
    lib.wvgx_set_tuning.restype = ctypes.c_int
    m, ks, d, n = 32, 256, 128, a.rows
    rng = np.random.default_rng(44)
    centers = rng.uniform(-1, 1, (m, ks, d // m)).astype(np.float32)
    c = Corpus(ctx, KIND_PQ, METRIC_L2, d, n)
    c.set_codebook(centers)
    step = 5_000_000
    for r0 in range(0, n, step):
        cnt = min(step, n - r0)
        c.upsert_codes(np.arange(r0, r0 + cnt, dtype=np.uint64), rng.integers(0, ks, (cnt, m), dtype=np.uint8))
    qs = rng.uniform(-1, 1, (a.queries, d)).astype(np.float32)
    for g, v in ((int(g), int(x)) for g in a.gpcs.split(",") for x in a.variants.split(",")):
        prev = lib.wvgx_set_tuning(7, v)
        prev_g = lib.wvgx_set_tuning(1, g)
        ref = c.search(qs[0], 10)
        for i in range(8):
            c.search(qs[i % len(qs)], 10)
        check(lib.wvg_profile_start(ctx.handle))
        for i in range(a.queries):
            c.search(qs[i], 10)
        ms, nl = ctypes.c_double(), ctypes.c_uint64()
        check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
        lib.wvgx_set_tuning(7, prev)
        lib.wvgx_set_tuning(1, prev_g)
        same = bool(np.array_equal(ref[0], c.search(qs[0], 10)[0]))
        scan_ms = ms.value / max(1, nl.value)
        print(json.dumps({"variant": v, "groups_per_cu": g, "rows": n, "scan_ms": round(scan_ms, 4),
                          "GBps": round(n * m / scan_ms / 1e6, 1), "launches": int(nl.value),
                          "same_as_product": same}), flush=True)
    c.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
