#!/usr/bin/env python3
"""Stress of concurrent single-query host calls (the coalescer, the query in
the kernel arguments, results written to coherent host memory and polled):
T reader threads issue k = 10 single-query wvg_search calls on one corpus
while a writer keeps upserting and deleting far-away rows, and every result
is compared with the oracle's top-k.  --modes: tuning key 24 (tools build):
bit 0 = query staged by copy, bit 1 = stream synchronization instead of
polling, bit 2 = round 4's untagged layout (ids / dists + a polled count).
Prints one JSON line per mode: calls, wrong results, and the library's
single-path counters (wvgx_single_counters): tagged calls, calls whose header
tag arrived before every entry's tag (out-of-order arrival seen), sync
fallbacks, and -- round-4 layout -- calls whose ids changed in host memory
after the polled count was seen.
--serial: first one thread alone (one stream slot), alternating queries with
8-query batch calls in between, the interleaving of the VERDICT r4 item 2.
Usage: WVG_LIB=tools/libwvgpu_tools.so python tools/single_query_stress.py [--modes 0,2,4,6]"""
import argparse
import ctypes
import json
import os
import sys
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,2,4,6")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--calls", type=int, default=400, help="calls per thread per mode")
    ap.add_argument("--coalesce", type=int, default=1)
    ap.add_argument("--serial", type=int, default=2000, help="single-thread interleaved calls per mode (0 = none)")
    a = ap.parse_args()
    from oracle import wv_oracle as orc
    from weaviate_amd._lib import KIND_F32, METRIC_L2
    from weaviate_amd.device import Context, Corpus

    rng = np.random.default_rng(7)
    n, d, k = 5_000, 64, 10
    stable = (rng.random((n, d), dtype=np.float32) * 2 - 1).astype(np.float32)
    far = (rng.random((1000, d), dtype=np.float32) * 2 - 1).astype(np.float32) + 100.0
    queries = (rng.random((32, d), dtype=np.float32) * 2 - 1).astype(np.float32)
    ids = np.arange(n, dtype=np.uint64)
    want = [orc.lex_topk(orc.dist_all(0, q, stable), ids, k)[0] for q in queries]
    ctx = Context(0) if a.coalesce else Context(0, coalesce=0)
    lib = ctx.lib
    lib.wvgx_set_tuning.restype = ctypes.c_int
    ctr = (ctypes.c_uint64 * 4)()
    corpus = Corpus(ctx, KIND_F32, METRIC_L2, d, n + len(far))
    corpus.upsert(ids, stable)

    def counters():
        lib.wvgx_single_counters(ctr, 1)
        return {"tagged": int(ctr[0]), "header_before_entries": int(ctr[1]), "sync_fallbacks": int(ctr[2]),
                "legacy_ids_changed_after_count": int(ctr[3])}

    for mode in [int(x) for x in a.modes.split(",")]:
        lib.wvgx_set_tuning(24, mode)
        counters()
        if a.serial:
            wrong = 0
            for r in range(a.serial):
                qi = (r * 5) % len(queries)
                got, _, cnt = corpus.search(queries[qi], k)
                wrong += int(int(cnt[0]) != k or not np.array_equal(got[0, :k], want[qi]))
                if r % 4 == 3:  # a batch call on the same slot between single calls
                    corpus.search(queries[:8], k)
            print(json.dumps({"mode": mode, "phase": "serial", "calls": a.serial, "wrong": wrong,
                              "counters": counters()}), flush=True)
        stop = threading.Event()
        bad = []

        def writer():
            far_ids = np.arange(n, n + len(far), dtype=np.uint64)
            while not stop.is_set():
                corpus.upsert(far_ids, far)
                corpus.delete(far_ids[::2])
                corpus.delete(far_ids[1::2])

        def reader(j):
            wrong = 0
            for r in range(a.calls):
                qi = (j * 7 + r) % len(queries)
                got, _, cnt = corpus.search(queries[qi], k)
                if int(cnt[0]) != k or not np.array_equal(got[0, :k], want[qi]):
                    wrong += 1
                    if len(bad) < 5:
                        hit = [i for i in range(len(queries)) if np.array_equal(got[0, :k], want[i])]
                        bad.append({"thread": j, "call": r, "query": qi, "count": int(cnt[0]),
                                    "result_is_query": hit})
            return wrong

        w = threading.Thread(target=writer)
        w.start()
        try:
            with ThreadPoolExecutor(a.threads) as ex:
                wrong = sum(ex.map(reader, range(a.threads)))
        finally:
            stop.set()
            w.join()
        print(json.dumps({"mode": mode, "phase": "concurrent", "calls": a.threads * a.calls, "wrong": wrong,
                          "examples": bad, "counters": counters()}), flush=True)
    lib.wvgx_set_tuning(24, 0)
    corpus.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
