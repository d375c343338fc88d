#!/usr/bin/env python3
"""PQ encode (K9) throughput on BASELINE configs[3]'s shape: 100M x 128 fp32
rows -> m = 32 codes of ks = 256 (ds = 4), codebook from wvg_pq_fit on the
first 100k rows.  Bulk compression of a resident corpus
(wvg_pq_encode_corpus), wall time around a synchronised call, best of --reps.
Peak: 5.5 VALU instructions per (row, segment, centroid) -- the reference's
unfused sub, mul, add per dimension, two centroids per packed op -- at one
wave64 VALU instruction per SIMD per 4 cycles, 1024 SIMDs, 2.4 GHz.
A sample of codes is compared with the oracle-free invariant that a second
encode gives the same bytes.  Tooling only (product library)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    from weaviate_amd._lib import KIND_F32, KIND_PQ, METRIC_L2, check, fptr, u32ptr, u64ptr
    from weaviate_amd.device import Context, Corpus

    n, d, m, ks = a.rows, 128, 32, 256
    ctx = Context(0)
    lib = ctx.lib
    f = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    f.fill_synthetic(42, n, 0)
    nt = min(n, 100_000)
    rows = np.empty((nt, d), np.float32)
    check(lib.wvg_synthetic_rows(ctx.handle, 42, u64ptr(np.arange(nt, dtype=np.uint64)), nt, d, 0, 0, fptr(rows)))
    centers = np.empty((m, ks, d // m), np.float32)
    passes = np.zeros(m, np.uint32)
    check(lib.wvg_pq_fit(ctx.handle, fptr(rows), nt, d, m, ks, 100_000, 7, fptr(centers), u32ptr(passes)))
    pq = Corpus(ctx, KIND_PQ, METRIC_L2, d, n)
    pq.set_codebook(centers)
    ctx.synchronize()
    sample = np.random.default_rng(5).integers(0, n, 4096).astype(np.uint64)
    times, codes = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        check(lib.wvg_pq_encode_corpus(pq.handle, f.handle))
        ctx.synchronize()
        times.append(time.perf_counter() - t0)
        codes.append(pq.get_batch(sample, pq_m=m)[0])
    best = min(times)
    peak_rows = 1024 * 2.4e9 / 4 * 64 / (m * ks * 5.5)
    print(json.dumps({"config": "pq/encode", "workload": f"{n} x {d} -> m={m} codes, ks={ks}",
                      "encode_s": [round(t, 4) for t in times], "rows_per_s": round(n / best, 1),
                      "frac_of_packed_op_peak": round(n / best / peak_rows, 3),
                      "peak_rows_per_s": round(peak_rows, 1),
                      "repeat_encodes_identical": all(np.array_equal(codes[0], c) for c in codes)}), flush=True)
    f.destroy()
    pq.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
