"""Times the host-rows rescore call (wvg_rescore, V/flat/index.go:347-389) and
the query normalize at BASELINE config 3's shape (R = 200 rows of d = 1536,
k = 10), per call; run under rocprofv3 --kernel-trace --stats to split the
call into its kernels and copies."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main():
    import torch

    torch.cuda.init()
    from weaviate_amd._lib import METRIC_COSINE, check, fptr, u32ptr, u64ptr
    from weaviate_amd.device import Context

    ctx = Context(0)
    lib = ctx.lib
    R, d, k, reps = 200, 1536, 10, 50
    ids = np.arange(1000, 1000 + R, dtype=np.uint64)
    rows = np.empty((R, d), np.float32)
    check(lib.wvg_synthetic_rows(ctx.handle, 42, u64ptr(ids), R, d, 0, 1, fptr(rows)))
    q = np.random.default_rng(43).uniform(-1, 1, d).astype(np.float32)
    qn = np.empty(d, np.float32)
    oi, od, oc = np.empty(k, np.uint64), np.empty(k, np.float32), np.zeros(1, np.uint32)
    for _ in range(5):
        check(lib.wvg_normalize_batch(ctx.handle, fptr(q), 1, d, fptr(qn)))
        check(lib.wvg_rescore(ctx.handle, METRIC_COSINE, fptr(qn), fptr(rows), u64ptr(ids), R, d, k, u64ptr(oi),
                              fptr(od), u32ptr(oc)))
    t0 = time.perf_counter()
    for _ in range(reps):
        check(lib.wvg_normalize_batch(ctx.handle, fptr(q), 1, d, fptr(qn)))
    t1 = time.perf_counter()
    for _ in range(reps):
        check(lib.wvg_rescore(ctx.handle, METRIC_COSINE, fptr(qn), fptr(rows), u64ptr(ids), R, d, k, u64ptr(oi),
                              fptr(od), u32ptr(oc)))
    t2 = time.perf_counter()
    print({"normalize_us": round((t1 - t0) / reps * 1e6, 1), "rescore_us": round((t2 - t1) / reps * 1e6, 1)})
    ctx.close()


if __name__ == "__main__":
    main()
