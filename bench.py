#!/usr/bin/env python3
"""bench.py -- BASELINE metric: exact 10-NN QPS + achieved HBM GB/s,
1M x 128 fp32 L2 flat scan, 1/2/4/8-GPU scaling.

Workload (BASELINE.json configs[0] shape, on the GPU): every GPU holds a
1,000,000 x 128 fp32 shard (global docIDs rank*1M ..), generated in HBM by a
counter-based RNG.  A step is a batch of B single-query searches: each query
is one full scan of the shard (one K1 scan launch per query, flat.searchByVector
semantics; each launch also runs the previous query's top-k merge on one extra
workgroup -- wvg_search_device_pipelined), then -- for N > 1 -- one RCCL
all-gather of the B x k (dist, id) candidates and one device merge
(Index.objectVectorSearch's shard merge).  Weak scaling: value = query
scans of 1M rows per second over all GPUs = N * B * steps / time.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N > 1 via torch.distributed.run, one process per GPU, RCCL)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "exact 10-NN QPS + achieved HBM GB/s, 1M×128 L2 flat; 1/2/4/8 GPU scaling"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="single-query searches per step")
    ap.add_argument("--rows", type=int, default=1_000_000, help="rows per GPU")
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--cpu-queries", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(rows_n, d, k, qs, gpu_ids):
    """Weaviate's CPU flat path on this host: the reference's own l2_256
    (oracle/_ref, built from /root/reference) when this CPU can run it, else the
    oracle's bit-identical restatement; bounded max-heap top-k; one query per
    thread (CH/utils.go:25-42 Concurrently), plus a single-core sample."""
    from oracle import wv_oracle as orc

    flags = open("/proc/cpuinfo").read()
    can_ref = orc.ref() is not None and " avx512f" in flags and " fma" in flags
    rows = orc.synth_rows(42, 0, rows_n, d, 0)
    threads = max(1, min(16, os.cpu_count() or 1))
    nq = len(qs)
    secs, ids, dists, used_ref = orc.bench_flat(rows, qs, k, orc.L2, threads, use_ref_kernel=can_ref)
    n1 = min(8, nq)
    secs1, _, _, _ = orc.bench_flat(rows, qs[:n1], k, orc.L2, 1, use_ref_kernel=can_ref)
    match = bool(np.array_equal(ids[: len(gpu_ids)], gpu_ids))
    model = ""
    for line in flags.splitlines():
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    return {
        "value": round(nq / secs, 3),
        "unit": "queries/s",
        "cores": threads,
        "kind": "reference" if used_ref else "port",
        "sample": (f"{nq} queries over the same 1M x 128 rows (resident float32 matrix, no LSM cursor/decode), "
                   f"one query per thread on {threads} threads, {secs:.1f} s wall; kernel "
                   + ("l2_256 from the reference's C source (oracle/_ref)" if used_ref else
                      "oracle restatement of l2_256") + f"; cpu: {model}"),
        "single_core_qps": round(n1 / secs1, 3),
        "ids_match_gpu": match,
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from weaviate_amd import _lib
    from weaviate_amd._lib import KIND_F32, METRIC_L2, check
    from weaviate_amd.device import Context, Corpus

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    n, d, k, B = args.rows, args.dim, args.k, args.batch
    cap = (n + 63) // 64 * 64
    ctx = Context(local)
    lib = ctx.lib
    corpus = Corpus(ctx, KIND_F32, METRIC_L2, d, cap, id_base=rank * cap)
    corpus.fill_synthetic(42, n, 0)

    P = 64  # distinct queries cycled through the steps
    qs = np.random.default_rng(43).uniform(-1, 1, (P, d)).astype(np.float32)
    tq = torch.from_numpy(qs).to(dev)
    ids = torch.empty((B, k), dtype=torch.int64, device=dev)
    dists = torch.empty((B, k), dtype=torch.float32, device=dev)
    counts = torch.empty(B, dtype=torch.int32, device=dev)
    ws_bytes = lib.wvg_search_workspace_size(corpus.handle, B, k)
    ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
    if world > 1:
        g_d = torch.empty(world * B * k, dtype=torch.float32, device=dev)
        g_i = torch.empty(world * B * k, dtype=torch.int64, device=dev)
        m_ids = torch.empty((B, k), dtype=torch.int64, device=dev)
        m_d = torch.empty((B, k), dtype=torch.float32, device=dev)
        m_c = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    assert P % B == 0

    def step(s):
        # B single-query scans in one call = one query-stream launch (each query a full scan)
        q0 = (s * B) % P
        check(lib.wvg_search_device_pipelined(corpus.handle, tq[q0].data_ptr(), B, k, ids.data_ptr(),
                                              dists.data_ptr(), counts.data_ptr(), ws.data_ptr(), ws_bytes, stream))
        if world > 1:
            dist.all_gather_into_tensor(g_d, dists.view(-1))
            dist.all_gather_into_tensor(g_i, ids.view(-1))
            check(lib.wvg_topk_merge_device(ctx.handle, g_d.data_ptr(), g_i.data_ptr(), B, world, k, k,
                                            m_ids.data_ptr(), m_d.data_ptr(), m_c.data_ptr(), stream))

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    check(lib.wvg_profile_start(ctx.handle))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(args.warmup + s)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    import ctypes

    scan_ms, launches = ctypes.c_double(), ctypes.c_uint64()
    check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(scan_ms), ctypes.byref(launches)))
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_queries = world * B * args.steps  # 1M-row query scans over all GPUs
    value = total_queries / elapsed
    avg_launch_s = scan_ms.value / 1e3 / max(1, launches.value)
    # N*d*4 algorithmic bytes per query scan; one launch scans B queries
    bytes_per_launch = n * d * 4 * B
    achieved = bytes_per_launch / avg_launch_s / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf):
        try:
            rec = json.load(open(tf)).get("scan_f32_stream_l2_128", {})
            if rec.get("rows") == n and rec.get("dim") == d:
                traffic = int(round(rec["hbm_bytes_per_query_scan"] * B))  # per launch, like `achieved`
        except Exception:
            traffic = None

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: uniform[-1,1) rows from a counter RNG (seed 42) generated in HBM; "
                    "64 uniform[-1,1) queries (seed 43) cycled",
            "config": {
                "workload": "flat exact k-NN, 1M x 128 fp32 L2 per GPU, single-query scans "
                            "(BASELINE configs[0] shape on MI355X)",
                "rows_per_gpu": n, "dim": d, "k": k, "queries_per_step": B,
                "parallelism": f"shard rows by docID range over {world} GPU(s); RCCL all-gather of per-GPU top-k",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "wvg::scan_f32_stream_kernel<L2,128,1>",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "avg_launch_us": round(avg_launch_s * 1e6, 2),
                "queries_per_launch": B,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "launches": int(launches.value),
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            nq = args.cpu_queries
            cq = np.random.default_rng(43).uniform(-1, 1, (nq, d)).astype(np.float32)
            # GPU results for the first queries (host API) to cross-check at full size
            gids, _, _ = corpus.search(cq[:16], k)
            out["cpu_baseline"] = cpu_baseline(n, d, k, cq, gids)
        print(json.dumps(out), flush=True)
    corpus.destroy()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
