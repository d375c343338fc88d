#!/usr/bin/env python3
"""BQ Hamming scan probe (tools build): a BQ corpus of `--rows` x 1536-bit
codes (fill_synthetic of cosine rows, configs[2]'s shape), single-query
Hamming top-R searches per variant (K1-family workgroups per CU, tuning key
1; 0 = auto), timed with HIP events bound to the scan launches; ids of the
first query compared with the first variant.  Prints one JSON line per variant.
Usage: WVG_LIB=tools/libwvgpu_tools.so python tools/bq_scan_probe.py [--rows 100000000] [--gpc 0,2,3,0]"""
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
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--queries", type=int, default=16)
    ap.add_argument("--r", type=int, default=200)
    ap.add_argument("--gpc", default="0,2,3,0")
    a = ap.parse_args()
    from oracle import wv_oracle as orc
    from weaviate_amd._lib import KIND_BQ, METRIC_COSINE, check
    from weaviate_amd.device import Context, Corpus

    ctx = Context(0)
    lib = ctx.lib
    lib.wvgx_set_tuning.restype = ctypes.c_int
    n, d = a.rows, 1536
    c = Corpus(ctx, KIND_BQ, METRIC_COSINE, d, n)
    c.fill_synthetic(42, n, 0)
    qs = orc.synth_rows(43, 0, a.queries, d, 0)
    ref = None
    for g in (int(x) for x in a.gpc.split(",")):
        prev = lib.wvgx_set_tuning(1, g)
        first = c.search(qs[0], a.r)[0][0].copy()
        for i in range(4):
            c.search(qs[i], a.r)
        check(lib.wvg_profile_start(ctx.handle))
        for i in range(a.queries):
            c.search(qs[i], a.r)
        ms, nl = ctypes.c_double(), ctypes.c_uint64()
        check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
        lib.wvgx_set_tuning(1, prev)
        ref = first if ref is None else ref
        scan_ms = ms.value / max(1, nl.value)
        print(json.dumps({"groups_per_cu": g, "rows": n, "R": a.r, "scan_ms": round(scan_ms, 4),
                          "GBps": round(n * 24 * 8 / scan_ms / 1e6, 1), "launches": int(nl.value),
                          "same_ids_as_first": bool(np.array_equal(ref, first))}), flush=True)
    c.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
