"""Per-call latency of the host C-ABI entry points an online caller hits
(flat SearchByVector, HNSW rescore / DistanceToNode by ids, BatchDist), at
BASELINE config 1's corpus (1M x 128 L2).  Prints one JSON line per entry.
Run under rocprofv3 --kernel-trace --stats to split a call into kernels."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    import torch

    torch.cuda.init()
    from weaviate_amd._lib import KIND_F32, METRIC_L2, check, fptr
    from weaviate_amd.device import Context, Corpus

    ctx = Context(0)
    lib = ctx.lib
    n, d = 1_000_000, 128
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.fill_synthetic(42, n, 0)
    ctx.synchronize()
    rng = np.random.default_rng(43)
    q1 = rng.uniform(-1, 1, (1, d)).astype(np.float32)
    q16 = rng.uniform(-1, 1, (16, d)).astype(np.float32)
    ids500 = rng.integers(0, n, 500).astype(np.uint64)
    X = rng.uniform(-1, 1, (1000, d)).astype(np.float32)
    out = np.empty(1000, np.float32)
    res = {
        "search_1q_k10_us": timed(lambda: c.search(q1, 10)),
        "search_16q_k10_us_per_call": timed(lambda: c.search(q16, 10), 50),
        "distance_by_ids_500_us": timed(lambda: c.distance_by_ids(q1[0], ids500)),
        "distance_batch_1000_us": timed(lambda: check(lib.wvg_distance_batch(ctx.handle, METRIC_L2, fptr(q1[0]), fptr(X),
                                                                              1000, d, fptr(out)))),
    }
    print(json.dumps({k: round(v, 1) for k, v in res.items()}))
    c.destroy()
    ctx.close()


if __name__ == "__main__":
    main()
