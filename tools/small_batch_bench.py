#!/usr/bin/env python3
"""Per-query throughput of small flat batches (1 < nq < the MFMA threshold):
one wvg_search_device call of nq queries (K1 COS: the nq queries of a row
range side by side on one XCD) against nq single-query calls, same queries,
results compared bit for bit; plus one KMeans.Fit (wvg_pq_fit) timing.
Tooling only (product library)."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--metric", default="l2", choices=["l2", "dot", "cosine"])
    ap.add_argument("--nqs", default="2,4,8,16,31")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--fit", type=int, default=1)
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    from weaviate_amd import _lib
    from weaviate_amd._lib import KIND_F32, METRIC_COSINE, METRIC_DOT, METRIC_L2, check
    from weaviate_amd.device import Context, Corpus

    metric = {"l2": METRIC_L2, "dot": METRIC_DOT, "cosine": METRIC_COSINE}[a.metric]
    dev = torch.device("cuda:0")
    ctx = Context(0)
    lib = ctx.lib
    n, d, k = a.rows, a.dim, a.k
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.fill_synthetic(42, n, 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    maxq = max(int(x) for x in a.nqs.split(","))
    q = np.random.default_rng(9).uniform(-1, 1, (maxq, d)).astype(np.float32)
    if metric == METRIC_COSINE:
        q /= np.linalg.norm(q, axis=1, keepdims=True)
    tq = torch.from_numpy(q).to(dev)

    def run(nq, q0=0):
        ws = torch.zeros(lib.wvg_search_workspace_size(c.handle, nq, k), dtype=torch.uint8, device=dev)
        oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
        od = torch.empty((nq, k), dtype=torch.float32, device=dev)
        oc = torch.empty(nq, dtype=torch.int32, device=dev)

        def go():
            check(lib.wvg_search_device(c.handle, tq[q0].data_ptr(), nq, k, oi.data_ptr(), od.data_ptr(),
                                        oc.data_ptr(), ws.data_ptr(), ws.numel(), st))

        go()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(a.reps):
            go()
        torch.cuda.synchronize()
        return (time.time() - t0) / a.reps, (oi.cpu().numpy(), od.cpu().numpy().view(np.uint32), oc.cpu().numpy())

    single = [run(1, i) for i in range(maxq)]
    t1 = sum(s[0] for s in single[:maxq]) / maxq
    out = {"config": f"{n} x {d} {a.metric}, k={k}", "single_query_ms": round(t1 * 1e3, 4),
           "single_qps": round(1 / t1, 1)}
    for nq in (int(x) for x in a.nqs.split(",")):
        tb, (bi, bd, bc) = run(nq)
        same = all(np.array_equal(bi[i], single[i][1][0][0]) and np.array_equal(bd[i], single[i][1][1][0])
                   for i in range(nq))
        out[f"nq{nq}"] = {"batch_ms": round(tb * 1e3, 4), "qps": round(nq / tb, 1),
                          "speedup_per_query": round(t1 * nq / tb, 2), "bit_identical_to_singles": bool(same)}
    print(json.dumps(out), flush=True)
    c.destroy()
    if a.fit:
        nt, dt, m, ks = 100_000, 128, 32, 256
        X = np.random.default_rng(3).uniform(-1, 1, (nt, dt)).astype(np.float32)
        cen = np.empty((m, ks, dt // m), np.float32)
        its = np.zeros(m, np.uint32)
        for rep in range(2):
            t0 = time.time()
            check(lib.wvg_pq_fit(ctx.handle, _lib.fptr(X), nt, dt, m, ks, 0, 7, _lib.fptr(cen), _lib.u32ptr(its)))
            el = time.time() - t0
        print(json.dumps({"pq_fit": f"{nt} x {dt}, m={m}, ks={ks}", "wall_s": round(el, 4),
                          "lloyd_passes": int(its.max()), "ms_per_pass_incl_host": round(el / max(1, its.max()) * 1e3, 3)}),
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
