#!/usr/bin/env python3
"""BASELINE configs[1]: batched 10-NN over 10M x 768 fp32 cosine, 1024-query
batches -- the K3i int8 screen and the K3d / K3c bf16 screen (+ exact rescore)
against the exact fp32 MFMA path (K3b), same corpus, same queries, results
compared bit for bit.
Device API (queries in HBM), HIP events bound to the scoring launch(es);
bf16_peak_frac = the batch's 2 Q N d FLOP / kernel time against the dense
bf16 peak (2.5 PFLOP/s; fp32 157.3 TFLOP/s for K3b); rescored_rows = the candidates
the exact fp32 rescore recomputed in the last batch.
Tooling only (product library; no tuning knobs)."""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def screen_nrr(n, nq, num_cus=256, whole_rounds=True):
    """The screen's row ranges for n rows and nq queries: screen_row_ranges
    (wvg_screen.hip), whole_rounds = its tuning screen_round."""
    nqb = (nq + 127) // 128
    nblk = ((n + 63) // 64 + 3) // 4
    want = max((num_cus + nqb - 1) // nqb, (nblk + 127) // 128)
    want = min((want + 7) // 8 * 8, 512)
    if whole_rounds:
        step = 8 * (num_cus // math.gcd(num_cus, nqb)) // math.gcd(8, num_cus // math.gcd(num_cus, nqb))
        w2 = (want + step - 1) // step * step
        if w2 <= 512 and w2 * 8 <= want * 9:
            want = w2
    return max(1, min(want, nblk))


def screen_offsets(n, nq, k, d, num_cus=256):
    """(candidate-array byte offset, candidates per query, flagged-count byte
    offset) in a K3c / K3d workspace (screen_ws in wvg_search.hip, after the
    256-byte status block); mirrors screen_row_ranges."""
    nrr = screen_nrr(n, nq, num_cus)
    ncand = nrr * 16
    part = (nq * ncand * 8 + 255) // 256 * 256
    return part, ncand, screen_nflag_offset(n, nq, k, d, num_cus)


def screen_nflag_offset(n, nq, k, d, num_cus=256):
    """Byte offset of the flagged-query count in a K3c workspace (screen_ws in
    wvg_search.hip, after the 256-byte status block); mirrors screen_row_ranges."""
    nrr = screen_nrr(n, nq, num_cus)
    off = 0

    def take(b):
        nonlocal off
        o = off
        off = (off + b + 255) // 256 * 256
        return o

    nq_pad, ncand, kbn = (nq + 127) // 128 * 128, nrr * 16, (d + 63) // 64 * 2
    for b in (nq * ncand * 8, nq * ncand * 8, nq * ncand * 8, nq * 4, nq_pad // 16 * kbn * 1024, nq_pad * 4,
              nq_pad * 4, nq_pad * 4, nq * 4):
        take(b)
    return take(4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--metric", default="cosine", choices=["cosine", "dot"])
    ap.add_argument("--exact", type=int, default=1, help="also time the exact path")
    ap.add_argument("--screens", default="int8,bf16", help="screens to time: int8 (K3i), bf16 (K3d / K3c)")
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    from weaviate_amd._lib import KIND_F32, METRIC_COSINE, METRIC_DOT, check
    from weaviate_amd.device import Context, Corpus

    metric = METRIC_COSINE if a.metric == "cosine" else METRIC_DOT
    dev = torch.device("cuda:0")
    n, d, nq, k = a.rows, a.dim, a.nq, a.k
    q = np.random.default_rng(7).uniform(-1, 1, (nq, d)).astype(np.float32)
    if metric == METRIC_COSINE:
        q /= np.linalg.norm(q, axis=1, keepdims=True).astype(np.float32)
    tq = torch.from_numpy(q).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    out = {}
    res = {}
    modes = [m for m in a.screens.split(",") if m] + (["exact"] if a.exact else [])
    for mode in modes:
        ctx = Context(0, batch_screen={"int8": 2, "bf16": 1, "exact": 0}[mode])
        lib = ctx.lib
        c = Corpus(ctx, KIND_F32, metric, d, n)
        t0 = time.time()
        c.fill_synthetic(42, n, 0)
        ctx.synchronize()
        gen_s = time.time() - t0
        wsb = lib.wvg_search_workspace_size(c.handle, nq, k)
        ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
        oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
        od = torch.empty((nq, k), dtype=torch.float32, device=dev)
        oc = torch.empty(nq, dtype=torch.int32, device=dev)

        def run():
            check(lib.wvg_search_device(c.handle, tq.data_ptr(), nq, k, oi.data_ptr(), od.data_ptr(), oc.data_ptr(),
                                        ws.data_ptr(), wsb, st))

        t0 = time.time()
        run()  # screen: builds the bf16 shadow
        torch.cuda.synchronize()
        first_s = time.time() - t0
        check(lib.wvg_profile_start(ctx.handle))
        t0 = time.time()
        for _ in range(a.reps):
            run()
        torch.cuda.synchronize()
        wall = (time.time() - t0) / a.reps
        ms, nl = ctypes.c_double(), ctypes.c_uint64()
        check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
        res[mode] = (oi.cpu().numpy().copy(), od.cpu().numpy().copy(), oc.cpu().numpy().copy())
        if mode != "exact":  # flagged (rescanned) queries of the last batch: the screen workspace's nflag word
            out[mode + "_flagged_queries"] = int(ws[256 + screen_nflag_offset(n, nq, k, d):][:4].cpu().numpy().view(np.uint32)[0])
            # candidates the exact fp32 rescore recomputed (keys the collect kept, K6's input)
            co, ncand, _ = screen_offsets(n, nq, k, d)
            cand = ws[256 + co:256 + co + nq * ncand * 8].cpu().numpy().view(np.uint64)
            out[mode + "_rescored_rows_per_query"] = round(int((cand != np.iinfo(np.uint64).max).sum()) / nq, 2)
        kern_ms = ms.value / max(1, nl.value)
        flop = 2.0 * nq * n * d
        out[mode] = {"batch_ms": round(wall * 1e3, 3), "qps": round(nq / wall, 1),
                     "scoring_kernel_ms": round(kern_ms, 3),
                     "tflops_kernel": round(flop / (kern_ms / 1e3) / 1e12, 1),
                     "bf16_peak_frac": round(flop / (kern_ms / 1e3) / 1e12 / (2500.0 if mode != "exact" else 157.3), 3),
                     "first_call_s": round(first_s, 3), "fill_s": round(gen_s, 2)}
        print(json.dumps({mode: out[mode]}), flush=True)
        c.destroy()
        ctx.close()
    first = modes[0]
    for m in modes[1:]:
        out[f"{m}_bit_identical_to_{first}"] = bool(all(
            np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8)) for x, y in zip(res[first], res[m])))
    print(json.dumps({"config": f"{n} x {d} {a.metric}, {nq} queries, k={k}", **out}), flush=True)


if __name__ == "__main__":
    main()
