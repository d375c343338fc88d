#!/usr/bin/env python3
"""Coalescer under load (tools build): 1M x 128 L2, k = 10, T native caller
threads (bench.py's tools/host_calls.c loop) calling wvg_search with one query
each for `--seconds`; per T the QPS, latency percentiles and the coalescer's
batch counters (wvgx_coalesce_counters: batches, requests, time running
batches, largest batch), plus a direct nq-query call's time for reference;
at T = 1 also the host time inside the in-launch single-query path
(wvgx_single_timing).
Usage: WVG_LIB=tools/libwvgpu_tools.so python tools/coalesce_probe.py [--callers 1,16,32,64]"""
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
    ap.add_argument("--callers", default="1,16,32,64")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--allow-rate", type=float, default=0.0, help="calls carry one of 8 random allow lists of this rate")
    ap.add_argument("--zc", default="1", help="filtered batches' windows read from pinned staging (tuning key 31)")
    a = ap.parse_args()
    import bench
    from oracle import wv_oracle as orc
    from weaviate_amd._lib import KIND_F32, METRIC_L2
    from weaviate_amd.device import Context, Corpus, allow_bitmap

    ctx = Context(0)
    lib = ctx.lib
    n, d, k = 1_000_000, 128, 10
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.fill_synthetic(42, n, 0)
    qs = np.ascontiguousarray(orc.synth_rows(43, 0, 256, d, 0))
    hc = bench._host_calls_lib()
    cnt = (ctypes.c_uint64 * 4)()
    for nq in (16, 32, 64):
        c.search(qs[:nq], k)
        t0 = time.perf_counter()
        for _ in range(5):
            c.search(qs[:nq], k)
        print(json.dumps({"direct_call_nq": nq, "ms_per_call": round((time.perf_counter() - t0) / 5 * 1e3, 3)}),
              flush=True)
    st = (ctypes.c_uint64 * 5)()
    ft = (ctypes.c_uint64 * 5)()
    rng = np.random.default_rng(5)
    allows = [allow_bitmap(np.flatnonzero(rng.random(n) < a.allow_rate), n) for _ in range(8)] if a.allow_rate else None
    for zc, T in ((int(z), int(x)) for z in a.zc.split(",") for x in a.callers.split(",")):
        lib.wvgx_set_tuning(31, zc)
        lib.wvgx_coalesce_counters(cnt, 1)
        lib.wvgx_single_timing(st, 1)
        lib.wvgx_filtered_timing(ft, 1)
        qps, lat = bench._native_callers(hc, lib, c.handle, qs, k, T, a.seconds, allows=allows)
        lib.wvgx_coalesce_counters(cnt, 1)
        lib.wvgx_single_timing(st, 1)
        lib.wvgx_filtered_timing(ft, 1)
        if ft[4]:
            nb = int(ft[4])
            print(json.dumps({"zc": zc, "callers": T, "filtered_batch_host_us": {
                "entry_to_staged": round(ft[0] / nb / 1e3, 1), "fill_windows": round(ft[1] / nb / 1e3, 1),
                "launch_call": round(ft[2] / nb / 1e3, 1), "wait": round(ft[3] / nb / 1e3, 1), "batches": nb}}),
                  flush=True)
        if T == 1 and st[4]:  # host time inside search_batch of the in-launch single-query path
            n1 = int(st[4])
            print(json.dumps({"single_host_us": {"entry_to_launch": round(st[0] / n1 / 1e3, 2),
                                                 "launch_call": round(st[1] / n1 / 1e3, 2),
                                                 "poll_records": round(st[2] / n1 / 1e3, 2),
                                                 "copy_out": round(st[3] / n1 / 1e3, 2), "calls": n1}}),
                  flush=True)
        b, r, ns, mx = (int(x) for x in cnt)
        print(json.dumps({"zc": zc, "allow_rate": a.allow_rate, "callers": T, "qps": round(qps, 1), "p50_us": round(float(np.percentile(lat, 50)), 1),
                          "p99_us": round(float(np.percentile(lat, 99)), 1), "batches": b,
                          "mean_batch": round(r / max(1, b), 2), "max_batch": mx,
                          "mean_batch_run_us": round(ns / max(1, b) / 1e3, 1),
                          "busy_frac": round(ns / 1e9 / a.seconds, 3)}), flush=True)
    lib.wvgx_set_tuning(31, 1)
    c.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
