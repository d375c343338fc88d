#!/usr/bin/env python3
"""bench.py -- BASELINE metric: exact 10-NN QPS + achieved HBM GB/s,
1M x 128 fp32 L2 flat scan, 1/2/4/8-GPU scaling.

Default workload (``--workload flat1m``, BASELINE.json configs[0] shape on
the GPU): every GPU holds a 1,000,000 x 128 fp32 shard (global docIDs
rank*1M ..), generated in HBM by a counter-based RNG.  A step is a batch of B
single-query searches: each query is one full scan of the shard
(flat.searchByVector semantics; all B in one query-stream launch,
wvg_search_device_pipelined) written straight into this rank's packed result
block, then -- for N > 1 -- ONE RCCL all-gather of the blocks and one device
merge (Index.objectVectorSearch's shard merge, adapters/repos/db/index.go:
1567-1648).  Weak scaling: value = query scans of 1M rows per second over all
GPUs = N * B * steps / time.

``--workload slab1b`` (BASELINE.json configs[4]): the 1B x 128 fp32 L2 corpus
as 8 slabs of 125M rows, exact 100-NN.  The slabs are dealt to the N GPUs
(8/N each); a GPU holds one slab in HBM at a time, regenerated in place
between slabs (generation untimed), scans every step's B queries over it,
then the per-slab lists are merged on device and -- for N > 1 -- exchanged
with one all-gather per step.  Strong scaling: value = 1B-row queries per
second; at N = 1 this is the "8 sequential slabs" QPS_1 of SURVEY.md 8(d).

Run:  python bench.py [--gpus N --steps K --warmup W] [--workload flat1m|slab1b]
      N > 1: launched by the driver through torch.distributed.run (one
      process per GPU, RCCL); started directly with --gpus N it re-launches
      itself that way (before touching any GPU) and exits with its status.
      --dry-run: CPU-only rehearsal of the launch and the exchange (gloo).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "exact 10-NN QPS + achieved HBM GB/s, 1M×128 L2 flat; 1/2/4/8 GPU scaling"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["flat1m", "slab1b"], default="flat1m")
    ap.add_argument("--batch", type=int, default=0, help="single-query searches per step (default 16; slab1b 8)")
    ap.add_argument("--rows", type=int, default=0, help="flat1m: rows per GPU; slab1b: total rows (default 1e9)")
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=0, help="neighbours (default 10; slab1b 100)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target wall time of each multi-core CPU leg")
    ap.add_argument("--no-reuse-rows", type=int, default=4_000_000,
                    help="rows of the untimed no-reuse leg (frac_no_reuse); 8x the Infinity Cache at d = 128")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--configs", default="host_api,batched,bq,pq,slab",
                    help="N = 1: BASELINE configs 2-5 measured after the headline (comma list; '' = none)")
    ap.add_argument("--scale-legs", default="slab1b,pq,multi",
                    help="strong-scaling legs at every N (comma list; '' = none): slab1b = configs[4] 1B x 128 as 8 "
                         "slabs dealt to the N GPUs, pq = configs[3] 100M PQ sharded over the N GPUs")
    ap.add_argument("--s1b-rows", type=int, default=1_000_000_000, help="rows of the slab1b scale leg (tests: less)")
    ap.add_argument("--pq-rows", type=int, default=100_000_000, help="rows of the sharded PQ scale leg (tests: less)")
    ap.add_argument("--profile-run", action="store_true",
                    help="only the timed headline launches (no no-reuse leg, read probe or CPU baseline), so a "
                         "rocprofv3 --stats summary of the scan kernel covers exactly the launches `roofline` times")
    ap.add_argument("--dry-run", action="store_true", help="CPU-only rehearsal of the N-rank launch + exchange")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal: all ranks on cuda:0 with a gloo exchange (one-GPU boxes; not a measurement)")
    a = ap.parse_args(argv)
    slab = a.workload == "slab1b"
    a.batch = a.batch or (8 if slab else 16)
    a.k = a.k or (100 if slab else 10)
    a.rows = a.rows or (1_000_000_000 if slab else 1_000_000)
    return a


# ---------------------------------------------------------------------------
# N-rank launch
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def relaunch(n: int) -> int:
    """Runs this script under torch.distributed.run with n local ranks (a child
    process; this process has not touched a GPU) and returns its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the reference's CPU flat / BQ paths on this host
def cpu_share() -> tuple[int, int, str]:
    """(CPUs this process may use, CPUs of the machine, how it was determined):
    the affinity mask, capped by a cgroup CPU quota (the GPU box gives each
    job a share of a large host)."""
    total = os.cpu_count() or 1
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    how = "sched_getaffinity"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            if q < n:
                n, how = q, "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    v = os.environ.get("OMP_NUM_THREADS", "")  # the GPU box's declared per-job CPU share
    if v.isdigit() and 0 < int(v) < n and "TORCHELASTIC_RUN_ID" not in os.environ:  # (torchrun sets it to 1)
        n, how = int(v), f"OMP_NUM_THREADS={v} (job CPU share)"
    return n, total, how


def _sized(run_fn, per_query_probe: int, target_s: float, threads: int, cap: int) -> int:
    """Queries for about target_s seconds of wall time on `threads` threads."""
    t = run_fn(per_query_probe, 1)
    per_q = max(t / per_query_probe, 1e-5)
    return int(max(threads, min(cap, target_s * threads / per_q)))


def cpu_baseline(rows_n, d, k, gpu_ids, target_s, pq_check=None):
    """Weaviate's CPU flat path (findTopVectors: l2_256 + bounded max-heap,
    V/flat/index.go:411-452) and BQ path (findTopVectorsCached Hamming top-200
    + exact rescore, :347-389, 456-495) over the same 1M x 128 rows, with the
    reference's own l2_256 (oracle/_ref, built from /root/reference's C) when
    this CPU runs it, else the oracle's bit-identical restatement; one query
    per thread (CH/utils.go:25-42 Concurrently) on every CPU of this job's
    share, plus a single-core sample (Weaviate's flat scan of one query is
    single-threaded).  Resident float32 matrix: no LSM cursor / decode, so an
    upper bound on Weaviate's CPU QPS."""
    from oracle import wv_oracle as orc

    flags = open("/proc/cpuinfo").read()
    can_ref = orc.ref() is not None and " avx2" in flags and " fma" in flags
    model = next((ln.split(":", 1)[1].strip() for ln in flags.splitlines() if ln.startswith("model name")), "")
    threads, total, how = cpu_share()
    rows = orc.synth_rows(42, 0, rows_n, d, 0)
    qs = np.random.default_rng(43).uniform(-1, 1, (32768, d)).astype(np.float32)

    def flat(nq, th):
        return orc.bench_flat(rows, qs[:nq], k, orc.L2, th, use_ref_kernel=can_ref)[0]

    nq = _sized(flat, 4, target_s, threads, len(qs))
    secs, ids, _, used_ref = orc.bench_flat(rows, qs[:nq], k, orc.L2, threads, use_ref_kernel=can_ref)
    n1 = min(nq, max(4, int(nq / threads / 4)))
    secs1 = flat(n1, 1)
    match = bool(np.array_equal(ids[: len(gpu_ids)], gpu_ids))
    # BQ cache flow over the same rows (codes prebuilt, as the cache is at PostStartup)
    codes = orc.bq_encode_rows(rows)
    R = 200

    def bq(nqb, th):
        return orc.bench_flat_bq(rows, codes, qs[:nqb], k, R, orc.L2, th, use_ref_kernel=can_ref)[0]

    nqb = _sized(bq, 8, target_s, threads, len(qs))
    secs_b = bq(nqb, threads)
    nb1 = min(nqb, max(8, int(nqb / threads / 4)))
    secs_b1 = bq(nb1, 1)
    kernel = "l2_256 compiled from the reference's C source (oracle/_ref)" if used_ref else \
        "oracle restatement of l2_256"
    pq = cpu_pq_leg(target_s, threads, pq_check)
    return {
        "value": round(nq / secs, 3),
        "unit": "queries/s",
        "cores": threads,
        "kind": "reference" if used_ref else "port",
        "sample": (f"{nq} exact 10-NN queries over the same {rows_n:,} x {d} rows (resident float32 matrix, "
                   f"no LSM cursor/decode), one query per thread on {threads} threads ({how}; host has {total} "
                   f"CPUs), {secs:.1f} s wall; kernel {kernel}; cpu: {model}"),
        "single_core_qps": round(n1 / secs1, 3),
        "host_cpus": total,
        "ids_match_gpu": match,
        "bq": {
            "value": round(nqb / secs_b, 3),
            "unit": "queries/s",
            "cores": threads,
            "single_core_qps": round(nb1 / secs_b1, 3),
            "sample": (f"{nqb} flat BQ searches (Hamming top-{R} over prebuilt BQ codes with POPCNT, exact "
                       f"rescore of {R} rows, top-{k}; V/flat/index.go:347-389) over the same rows, "
                       f"{secs_b:.1f} s wall on {threads} threads"),
        },
        "pq": pq,
    }


PQ_CPU_ROWS = 10_000_000  # codes in the CPU PQ leg (320 MB at m = 32)


def pq_leg_data(n=PQ_CPU_ROWS, d=128, m=32, ks=256):
    """Synthetic PQ corpus of the configs[3] code shape: uniform random codes
    (seed 44), a synthetic codebook (counter RNG seed 45) and 64 queries."""
    codes = np.random.default_rng(44).integers(0, ks, (n, m), dtype=np.uint8)
    from oracle import wv_oracle as orc

    centers = orc.synth_rows(45, 0, m * ks, d // m, 0).reshape(m, ks, d // m)
    qs = np.random.default_rng(46).uniform(-1, 1, (64, d)).astype(np.float32)
    return codes, centers, qs


def cpu_pq_leg(target_s, threads, gpu_check):
    """BASELINE configs[3]'s CPU reference point: PQ ADC top-10 (the
    distancer's LUT, CH/product_quantization.go:85-104, sequential ADC sum +
    Wrap :352-361, flat heap) over PQ_CPU_ROWS m = 32 codes, one query per
    thread, restated in C (oracle/wv_oracle.c orc_bench_pq: the reference's
    PQ path is pure Go, so there is no compiled reference kernel).  The rate
    per 100M codes (configs[3]'s size) is the measured rate x rows / 1e8.
    `gpu_check(codes, centers, qs, k)` returns the GPU's ids for the same
    queries (K8e through the host API) for an ids cross-check."""
    from oracle import wv_oracle as orc

    codes, centers, qs = pq_leg_data()
    n, k = len(codes), 10
    nq = _sized(lambda q, th: orc.bench_pq(codes, centers, qs[:q], k, orc.L2, th)[0], 2, target_s, threads, 4096)
    qq = np.resize(qs, (nq, qs.shape[1]))
    secs, ids, _ = orc.bench_pq(codes, centers, qq, k, orc.L2, threads)
    n1 = min(nq, max(2, int(nq / threads / 4)))
    secs1 = orc.bench_pq(codes, centers, qq[:n1], k, orc.L2, 1)[0]
    match = None
    if gpu_check is not None:
        gids = gpu_check(codes, centers, qs[:4], k)
        match = bool(np.array_equal(ids[:4], gids))
    return {
        "value": round(nq / secs, 3),
        "unit": "queries/s",
        "cores": threads,
        "kind": "port",
        "single_core_qps": round(n1 / secs1, 3),
        "qps_per_100M_codes": round(nq / secs * n / 1e8, 3),
        "ids_match_gpu": match,
        "sample": (f"{nq} PQ ADC top-{k} queries over {n:,} synthetic m=32 x ks=256 codes (configs[3] code shape; "
                   f"LUT + sequential ADC + heap restated in C, oracle/wv_oracle.c orc_bench_pq), {secs:.1f} s wall "
                   f"on {threads} threads"),
    }


# ---------------------------------------------------------------------------
# BASELINE configs 2-5 on this GPU (rank 0, N = 1): the named shapes at full
# per-GPU size through the host C ABI (what the Go binding calls), each timed
# with HIP events bound to its dominant kernel and spot-checked afterwards.
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md; no 2:1 sparsity)
I8_PEAK_TOPS = 5000.0      # dense int8 MFMA: twice bf16 (cdna_hip_programming.md "MFMA rate per dtype")
# PQ encode: 5.5 VALU instructions per (row, segment, centroid) -- the reference's
# unfused sub, mul, add per dimension, two centroids per packed op -- at one wave64
# VALU instruction per SIMD per 4 cycles, 1024 SIMDs, 2.4 GHz
PQ_ENCODE_PEAK_ROWS = 1024 * 2.4e9 / 4 * 64 / (32 * 256 * 5.5)
# SURVEY.md 8(d)'s count for the same encode: N*m*ks*ds*3 fp32 ops (unfused sub, mul, add per
# dimension), against the packed non-FMA fp32 rate (2 ops per lane per v_pk_* instruction:
# 1024 SIMDs x 64 lanes x 2 / 4 cycles x 2.4 GHz = 78.6 Tops/s)
PQ_ENCODE_PEAK_OPS = 1024 * 64 * 2 / 4 * 2.4e9


def gpu_clock(dev, torch):
    """Lease identity next to the roofline: the GPU's current shader / memory
    clock levels from amdgpu's sysfs (read-only text), or None."""
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{getattr(p, 'pci_device_id', 0):02x}.0"
    except Exception:  # noqa: BLE001 -- no PCI location: no clock reading
        return None
    out = {"pci": bdf}
    for name in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk"):
        try:
            lines = open(f"/sys/bus/pci/devices/{bdf}/{name}").read().splitlines()
            cur = [ln.split(":", 1)[1].strip().rstrip("*").strip() for ln in lines if ln.rstrip().endswith("*")]
            out[name[7:]] = cur[0] if cur else None
        except (OSError, IndexError):
            out[name[7:]] = None
    return out


def _prof(lib, ctx):
    import ctypes

    from weaviate_amd._lib import check

    ms, nl = ctypes.c_double(), ctypes.c_uint64()
    check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
    return ms.value / 1e3, int(nl.value)


def _sorted_ok(orc, d):
    return bool(np.all(np.diff(orc.ord_key(np.asarray(d, np.float32)).astype(np.int64)) >= 0))


def _outside_ok(orc, sample_ids, sample_d, ids, dists):
    """No sampled row outside the result is ahead of the k-th in (distance, id) order."""
    outside = ~np.isin(sample_ids, np.asarray(ids).astype(np.int64))
    kd, kid = int(orc.ord_key(np.asarray(dists[-1:], np.float32))[0]), int(ids[-1])
    sk = orc.ord_key(np.asarray(sample_d, np.float32)[outside]).astype(np.int64)
    return bool(np.all((sk > kd) | ((sk == kd) & (sample_ids[outside] > kid))))


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def config_batched(ctx, orc, metric_name, metric, reps=3):
    """configs[1]: 10M x 768 fp32 dot / cosine, 1024-query batches (the int8
    MFMA screen K3i + exact fp32 rescore; results identical to the exact path);
    frac = 2 Q N d ops / the screen launches' time vs the dense int8 peak the
    kernel computes at, and bf16_equiv_frac the same rate against the dense bf16
    peak (the unit the bf16 screen of rounds 3-5 was quoted in)."""
    from weaviate_amd._lib import KIND_F32
    from weaviate_amd.device import Corpus

    n, d, Q, k = 10_000_000, 768, 1024, 10
    lib = ctx.lib
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.fill_synthetic(42, n, 0)
    qs = orc.synth_rows(43, 0, Q, d, 0)
    c.search(qs, k)  # untimed: builds the int8 shadow
    lib.wvg_profile_start(ctx.handle)
    t0 = time.perf_counter()
    for _ in range(reps):
        ids, dists, counts = c.search(qs, k)
    wall = (time.perf_counter() - t0) / reps
    ks, nl = _prof(lib, ctx)
    screen_s = ks / reps  # the screen launches of one batch (one event pair spans its phases)
    flop = 2.0 * Q * n * d
    # spot check (checker only): rows sampled at the start, middle and end
    starts = [0, n // 2 - 3, n - 10_000]
    sample_ids = np.concatenate([np.arange(s, s + 10_000, dtype=np.int64) for s in starts])
    srows = np.concatenate([orc.synth_rows(42, s, 10_000, d, 0) for s in starts])
    om = 2 if metric_name == "cosine" else 1
    if om == 2:
        srows = orc.normalize_rows(srows)
    ok = bool(np.all(counts == k))
    for qi in (0, Q - 1):
        q = orc.normalize(qs[qi]) if om == 2 else qs[qi]
        got = np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in ids[qi]])
        if om == 2:
            got = orc.normalize_rows(got)
        ok &= _sorted_ok(orc, dists[qi])
        ok &= bool(np.array_equal(_bits(orc.dist_all(om, q, got)), _bits(dists[qi])))
        ok &= _outside_ok(orc, sample_ids, orc.dist_all(om, q, srows), ids[qi], dists[qi])
    c.destroy()
    tflops = flop / screen_s / 1e12
    return {"workload": f"{n:,} x {d} fp32 {metric_name}, {Q}-query batches, exact {k}-NN (host API wvg_search)",
            "qps": round(Q / wall, 1), "batch_ms": round(wall * 1e3, 3), "batches": reps,
            "kernel": "int8 MFMA screen (K3i screen_i8_kernel<12, 0>, 2 x 2 waves per workgroup: exact int32 scores + a per-row "
                      "quantization-error bound) + exact fp32 AVX2-order rescore",
            "roofline": {"bound": "mfma", "achieved": round(tflops, 1), "peak": I8_PEAK_TOPS, "unit": "TOP/s (int8)",
                         "frac": round(tflops / I8_PEAK_TOPS, 4),
                         "bf16_equiv_frac": round(tflops / BF16_PEAK_TFLOPS, 4),
                         "screen_ms_per_batch": round(screen_s * 1e3, 3),
                         "frac_whole_batch_bf16_equiv": round(flop / wall / 1e12 / BF16_PEAK_TFLOPS, 4),
                         "ops_per_batch": flop},
            "check": {"ok": ok, "how": "queries 0 and 1023: results sorted, every distance a bit-exact oracle "
                                       "recomputation of its row, no row of 30k sampled (start / middle / end) "
                                       "ahead of the k-th; all counts = k"}}


def config_bq(ctx, orc, nq=8):
    """configs[2]: 100M x 1536 BQ (cosine) Hamming top-200 + exact fp32 rescore
    to 10 (flat.searchByVectorBQ, V/flat/index.go:347-389), exactly as
    Weaviate's heaps pick and order the candidates (wvg_search_bq_candidates:
    the K5 scan records the rows the heap could insert, the host replays the
    heap; wvg_rescore replays the k-heap in pop order).  The 614 GB of float
    rows do not fit one GPU: the R rows are regenerated by id into the
    caller's pinned gather buffer (stand-in for the LSM gets, timed apart) and
    rescored through wvg_rescore.  frac: 19.2 GB of codes per scan."""
    from weaviate_amd._lib import KIND_BQ, METRIC_COSINE, check, fptr, u32ptr, u64ptr
    from weaviate_amd.device import Corpus, search_bq_candidates

    n, d, k, R = 100_000_000, 1536, 10, 200
    w = (d + 63) // 64
    lib = ctx.lib
    c = Corpus(ctx, KIND_BQ, METRIC_COSINE, d, n)
    c.fill_synthetic(42, n, 0)
    qs = orc.synth_rows(43, 0, nq, d, 0)
    search_bq_candidates(c, qs[0], R)
    rows = ctx.host_array((R, d), np.float32)
    res, t_fetch = [], 0.0
    lib.wvg_profile_start(ctx.handle)
    t0 = time.perf_counter()
    for i in range(nq):
        ids, hd, cnt = search_bq_candidates(c, qs[i], R)  # pop order (descending Hamming, heap ties)
        t1 = time.perf_counter()
        cand = np.ascontiguousarray(ids[0, :cnt[0]])
        check(lib.wvg_synthetic_rows(ctx.handle, 42, u64ptr(cand), len(cand), d, 0, 1, fptr(rows)))
        t_fetch += time.perf_counter() - t1
        qn = np.empty(d, np.float32)
        check(lib.wvg_normalize_batch(ctx.handle, fptr(qs[i]), 1, d, fptr(qn)))
        oi, od, oc = np.empty(k, np.uint64), np.empty(k, np.float32), np.zeros(1, np.uint32)
        check(lib.wvg_rescore(ctx.handle, METRIC_COSINE, fptr(qn), fptr(rows), u64ptr(cand), len(cand), d, k,
                              u64ptr(oi), fptr(od), u32ptr(oc)))
        res.append((ids[0], hd[0], cand, oi.copy(), od.copy()))
    wall = (time.perf_counter() - t0) / nq
    scan_s, nl = _prof(lib, ctx)
    scan_s /= max(1, nl)
    # the cost of the exact heap: candidates call vs the plain lexicographic Hamming top-R
    # (the same K5 scan without the recording, one device merge)
    reps = 4
    t0 = time.perf_counter()
    for i in range(reps):
        search_bq_candidates(c, qs[i % nq], R)
    t_exact = (time.perf_counter() - t0) / reps
    c.search(qs[0], R)
    lib.wvg_profile_start(ctx.handle)
    t0 = time.perf_counter()
    for i in range(reps):
        c.search(qs[i % nq], R)
    t_lex = (time.perf_counter() - t0) / reps
    scan_lex_s, nl2 = _prof(lib, ctx)
    scan_lex_s /= max(1, nl2)
    # batch mode: nq queries per call (co-scheduled K5), Hamming top-R only
    c.search(qs, R)
    t0 = time.perf_counter()
    for _ in range(3):
        c.search(qs, R)
    wall_b = (time.perf_counter() - t0) / (3 * nq)
    search_bq_candidates(c, qs, R)
    t0 = time.perf_counter()
    for _ in range(2):
        search_bq_candidates(c, qs, R)
    wall_bx = (time.perf_counter() - t0) / (2 * nq)
    # check: sampled codes vs the oracle's encoder; query 0 EXACTLY against the
    # reference flow restated -- its Hamming heap over all 100M stored codes
    # (read back from the device), the pop order, the k-heap of the exact
    # distances; the last query: distances bit-exact, rescore = the k-heap
    starts = [0, n // 2 - 13, n - 10_000]
    sample_ids = np.concatenate([np.arange(s, s + 10_000, dtype=np.int64) for s in starts])
    scodes = np.concatenate([orc.bq_encode_rows(orc.normalize_rows(orc.synth_rows(42, s, 10_000, d, 0)))
                             for s in starts])
    got, okb = c.get_batch(sample_ids[::499].astype(np.uint64))
    ok = bool(okb.all() and np.array_equal(got, scodes[::499]))
    t_chk = time.perf_counter()
    for qi in (0, nq - 1):
        hid, hdist, cand, oi, od = res[qi]
        qc = orc.bq_encode(orc.normalize(qs[qi]))
        codes, okc = c.get_batch(hid.astype(np.uint64))
        ok &= bool(okc.all() and np.array_equal(_bits(orc.bq_dist_all(qc, codes.reshape(R, w))), _bits(hdist)))
        if qi == 0:
            alld = np.empty(n, np.float32)
            for r0 in range(0, n, 4_000_000):
                cc, okr = c.get_batch(np.arange(r0, min(n, r0 + 4_000_000), dtype=np.uint64))
                ok &= bool(okr.all())
                alld[r0:r0 + len(cc)] = orc.bq_dist_all(qc, cc)
                del cc
            pi, pd = orc.heap_pops(alld, R)
            del alld
            ok &= bool(np.array_equal(hid, pi) and np.array_equal(_bits(hdist), _bits(pd)))
        frows = orc.normalize_rows(np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in cand]))
        ed = orc.dist_all(2, orc.normalize(qs[qi]), frows)
        wi, wd = orc.heap_topk(ed, cand.astype(np.uint64), k)
        ok &= bool(np.array_equal(oi, wi) and np.array_equal(_bits(od), _bits(wd)))
    t_chk = time.perf_counter() - t_chk
    ctx.free_host_array(rows)
    c.destroy()
    by = n * w * 8
    gbps = by / scan_s / 1e9
    gbps_lex = by / scan_lex_s / 1e9
    return {"workload": f"{n:,} x {d} BQ (cosine, {w} words/row), Hamming top-{R} + exact fp32 rescore to {k}, "
                        f"Weaviate's heap order (heap_replay)",
            "qps": round(1 / wall, 2), "qps_without_row_fetch": round(1 / (wall - t_fetch / nq), 2),
            "row_fetch_stand_in_ms": round(t_fetch / nq * 1e3, 3), "scan_ms": round(scan_s * 1e3, 3),
            "heap_replay": {"candidates_call_ms": round(t_exact * 1e3, 3),
                            "lexicographic_top_r_call_ms": round(t_lex * 1e3, 3),
                            "cost_ms": round((t_exact - t_lex) * 1e3, 3),
                            "scan_ms_recording": round(scan_s * 1e3, 3),
                            "scan_ms_plain": round(scan_lex_s * 1e3, 3),
                            "batch_candidates_qps": round(1 / wall_bx, 2)},
            "batch_call_qps": round(1 / wall_b, 2), "batch_call_queries": nq,
            "kernel": "K5 scan_bq_kernel<..., EMIT> (XOR + popcount, fused top-200, heap-candidate recording)",
            "roofline": {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbps / HBM_PEAK_GBS, 4), "bytes_per_scan": by,
                         "frac_plain_scan": round(gbps_lex / HBM_PEAK_GBS, 4)},
            "check": {"ok": ok, "seconds": round(t_chk, 1),
                      "how": "sampled codes = oracle BQ encode; query 0: candidates (ids in pop order, Hamming "
                             "bits) = the oracle heap over all 100M stored codes; queries 0 and last: Hamming "
                             "distances bit-exact on the returned codes, rescore = the oracle k-heap of the exact "
                             "distances in pop order, ids and bits"}}


def config_pq(ctx, orc, nq=16):
    """configs[3]: 100M x 128 PQ (m = 32, ks = 256): ProductQuantizer.Fit on
    the first 100k rows, the bulk encode of all 100M rows (K9), then ADC
    top-10 (K8e; LUT in LDS).  frac: 3.2 GB of codes per scan (HBM); the
    encode against the packed-op peak of its instruction mix."""
    from weaviate_amd._lib import KIND_F32, KIND_PQ, METRIC_L2, check, fptr, u32ptr, u64ptr
    from weaviate_amd.device import Corpus

    n, d, m, ks, k = 100_000_000, 128, 32, 256, 10
    lib = ctx.lib
    f = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    f.fill_synthetic(42, n, 0)
    nt = 100_000
    trows = np.empty((nt, d), np.float32)
    check(lib.wvg_synthetic_rows(ctx.handle, 42, u64ptr(np.arange(nt, dtype=np.uint64)), nt, d, 0, 0, fptr(trows)))
    centers = np.empty((m, ks, d // m), np.float32)
    passes = np.zeros(m, np.uint32)
    t0 = time.perf_counter()
    check(lib.wvg_pq_fit(ctx.handle, fptr(trows), nt, d, m, ks, 100_000, 7, fptr(centers), u32ptr(passes)))
    fit_s = time.perf_counter() - t0
    pq = Corpus(ctx, KIND_PQ, METRIC_L2, d, n)
    pq.set_codebook(centers)
    ctx.synchronize()
    enc = []
    for _ in range(2):
        t0 = time.perf_counter()
        check(lib.wvg_pq_encode_corpus(pq.handle, f.handle))
        ctx.synchronize()
        enc.append(time.perf_counter() - t0)
    enc_s = min(enc)
    f.destroy()
    qs = orc.synth_rows(43, 0, nq, d, 0)
    for i in range(32):  # untimed: clocks settle after the encode
        pq.search(qs[i % nq], k)
    lib.wvg_profile_start(ctx.handle)
    res = []
    t0 = time.perf_counter()
    for i in range(nq):
        res.append(pq.search(qs[i], k))
    wall = (time.perf_counter() - t0) / nq
    scan_s, nl = _prof(lib, ctx)
    scan_s /= max(1, nl)
    pq.search(qs, k)
    t0 = time.perf_counter()
    for _ in range(4):
        pq.search(qs, k)
    wall_b = (time.perf_counter() - t0) / (4 * nq)
    # spot check: sampled codes vs the oracle encoder, ADC results on the returned codes
    starts = [0, n // 2 - 7, n - 20_000]
    sample_ids = np.concatenate([np.arange(s, s + 20_000, dtype=np.int64) for s in starts])
    scodes = orc.pq_encode(np.concatenate([orc.synth_rows(42, s, 20_000, d, 0) for s in starts]), centers)
    got, okb = pq.get_batch(sample_ids.astype(np.uint64), pq_m=m)
    ok = bool(okb.all() and np.array_equal(got, scodes))
    for qi in (0, nq - 1):
        ids, dists, counts = res[qi]
        lut = orc.pq_lut(0, qs[qi], centers)
        codes, okc = pq.get_batch(ids[0].astype(np.uint64), pq_m=m)
        ok &= bool(counts[0] == k and okc.all())
        ok &= bool(np.array_equal(_bits([orc.pq_adc(0, lut, cc) for cc in codes]), _bits(dists[0])))
        ok &= _sorted_ok(orc, dists[0])
        ok &= _outside_ok(orc, sample_ids, [orc.pq_adc(0, lut, cc) for cc in scodes], ids[0], dists[0])
    pq.destroy()
    gbps = n * m / scan_s / 1e9
    return {"workload": f"{n:,} x {d} fp32 -> PQ m={m} ks={ks}: fit (100k rows) + bulk encode + ADC top-{k}",
            "qps": round(1 / wall, 2), "scan_ms": round(scan_s * 1e3, 4), "batch_call_qps": round(1 / wall_b, 2),
            "batch_call_queries": nq, "fit_s": round(fit_s, 3), "lloyd_passes_mean": round(float(passes.mean()), 2),
            "encode_s": round(enc_s, 4), "encode_rows_per_s": round(n / enc_s, 1),
            "encode_frac_of_packed_op_peak": round(n / enc_s / PQ_ENCODE_PEAK_ROWS, 4),
            "encode_ops_8d": n * m * ks * (d // m) * 3,
            "encode_frac_8d_ops": round(n * m * ks * (d // m) * 3 / enc_s / PQ_ENCODE_PEAK_OPS, 4),
            "encode_frac_note": ("encode_frac_of_packed_op_peak prices the kernel's 5.5 VALU instructions per (row, "
                                 "segment, centroid) at full issue; encode_frac_8d_ops divides SURVEY.md 8(d)'s "
                                 "N*m*ks*ds*3 fp32 ops by the packed non-FMA rate (78.6 Tops/s)"),
            "kernel": "K8e scan_pq32_wide_kernel (LUT image in LDS); encode K9 pq_encode_kernel",
            "roofline": {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbps / HBM_PEAK_GBS, 4), "bytes_per_scan": n * m},
            "check": {"ok": ok, "how": "60k sampled codes (start / middle / end) = oracle encode; queries 0 and "
                                       "last: ADC distances bit-exact on the returned codes, sorted, no sampled "
                                       "row ahead of the k-th"}}


def config_slab(ctx, orc, dev, torch, nq=8):
    """configs[4], one GPU's share: a 125M x 128 fp32 L2 slab holding global
    docIDs [375M, 500M), exact 100-NN, nq single-query scans per
    query-stream launch (device API).  frac: 64 GB per query scan."""
    from weaviate_amd._lib import KIND_F32, METRIC_L2, check
    from weaviate_amd.device import Corpus

    n, d, k, base = 125_000_000, 128, 100, 375_000_000
    lib = ctx.lib
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n, id_base=base)
    c.fill_synthetic(42, n, 0)
    qs = orc.synth_rows(43, 0, nq, d, 0)
    tq = torch.from_numpy(qs).to(dev)
    ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
    dd = torch.empty((nq, k), dtype=torch.float32, device=dev)
    cc = torch.empty(nq, dtype=torch.int32, device=dev)
    wsb = lib.wvg_search_workspace_size(c.handle, nq, k)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    def run():
        check(lib.wvg_search_device_pipelined(c.handle, tq.data_ptr(), nq, k, ids.data_ptr(), dd.data_ptr(),
                                              cc.data_ptr(), ws.data_ptr(), wsb, st))

    run()
    torch.cuda.synchronize(dev)
    lib.wvg_profile_start(ctx.handle)
    t0 = time.perf_counter()
    reps = 2
    for _ in range(reps):
        run()
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / (reps * nq)
    ks_, nl = _prof(lib, ctx)
    check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), st))
    scan_s = ks_ / max(1, nl) / nq
    hi, hd, hc = ids.cpu().numpy().view(np.uint64), dd.cpu().numpy(), cc.cpu().numpy()
    starts = [base, base + n // 2 - 5, base + n - 20_000]
    sample_ids = np.concatenate([np.arange(s, s + 20_000, dtype=np.int64) for s in starts])
    srows = np.concatenate([orc.synth_rows(42, s, 20_000, d, 0) for s in starts])
    ok = bool(np.all(hc == k))
    for qi in (0, nq - 1):
        ok &= bool(np.all((hi[qi] >= base) & (hi[qi] < base + n))) and _sorted_ok(orc, hd[qi])
        got = np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in hi[qi]])
        ok &= bool(np.array_equal(_bits(orc.dist_all(0, qs[qi], got)), _bits(hd[qi])))
        ok &= _outside_ok(orc, sample_ids, orc.dist_all(0, qs[qi], srows), hi[qi], hd[qi])
    c.destroy()
    gbps = n * d * 4 / scan_s / 1e9
    return {"workload": f"{n:,} x {d} fp32 L2 slab (global docIDs [{base:,}, {base + n:,}): slab 3 of the 1B corpus), "
                        f"exact {k}-NN, {nq} single-query scans per query-stream launch",
            "qps_per_slab": round(1 / wall, 2), "scan_ms_per_query": round(scan_s * 1e3, 3),
            "note": "one slab of the 1B corpus; the measured 8-slab pass (all slabs scanned and merged at this "
                    "N) is configs.config5_1b_x_128",
            "kernel": "K1 scan_f32_stream_kernel<L2,128,2>",
            "roofline": {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbps / HBM_PEAK_GBS, 4), "bytes_per_scan": n * d * 4},
            "check": {"ok": ok, "how": "queries 0 and last: ids inside the slab, sorted, distances bit-exact "
                                       "recomputations, no row of 60k sampled ahead of the k-th; all counts = k"}}


def _callers(call, T, seconds):
    """T threads (goroutines) calling call(thread, i) back to back for about
    `seconds`; returns (calls per second, per-call latencies in us)."""
    import threading

    done = [0] * T
    lat = [[] for _ in range(T)]
    start = threading.Barrier(T + 1)
    stop_at = [0.0]

    def worker(t):
        i = t
        start.wait()
        pc = time.perf_counter
        while True:
            t0 = pc()
            if t0 >= stop_at[0]:
                break
            call(t, i)
            lat[t].append(pc() - t0)
            i += T
            done[t] += 1

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    [t.start() for t in th]
    stop_at[0] = time.perf_counter() + seconds + 0.2
    start.wait()
    t0 = time.perf_counter()
    [t.join() for t in th]
    el = time.perf_counter() - t0
    return sum(done) / el, np.concatenate([np.asarray(x) for x in lat]) * 1e6


_HOSTCALLS = []


def _host_calls_lib():
    """tools/libhostcalls.so (tools/host_calls.c, built by __graft_entry__.build()):
    native caller threads, or None when it was not built."""
    if not _HOSTCALLS:
        import ctypes

        path = os.path.join(ROOT, "tools", "libhostcalls.so")
        lib = None
        if os.path.exists(path):
            lib = ctypes.CDLL(path)
            lib.wvgb_call_loop.restype = ctypes.c_int
            lib.wvgb_call_loop.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] * 3 + [
                ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                ctypes.c_double, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        _HOSTCALLS.append(lib)
    return _HOSTCALLS[0]


def _native_callers(hc, lib, corpus, qs, k, T, seconds, allows=None, ks=None):
    """T native threads (tools/host_calls.c) calling wvg_search back to back for
    about `seconds` -- the goroutine shape without the interpreter; call i uses
    ks[i % len(ks)] when ks is given, else k: returns (calls per second,
    per-call latencies in us)."""
    import ctypes

    cap = 400_000
    lat = np.zeros(T * cap, np.float64)
    cnt = np.zeros(T, np.uint64)
    el = ctypes.c_double()
    qs = np.ascontiguousarray(qs, dtype=np.float32)
    if allows:
        arr = (ctypes.c_void_p * len(allows))(*[x.ctypes.data for x in allows])
        words = np.array([len(x) for x in allows], np.uint64)
        ap, wp, na = ctypes.cast(arr, ctypes.c_void_p), words.ctypes.data, len(allows)
    else:
        arr, words, ap, wp, na = None, None, None, None, 0
    fn = ctypes.cast(lib.wvg_search, ctypes.c_void_p).value
    kv = np.asarray(ks if ks else [], np.uint32)
    rc = hc.wvgb_call_loop(fn, corpus, qs.ctypes.data, qs.shape[0], qs.shape[1], k,
                           kv.ctypes.data if len(kv) else None, len(kv), ap, wp, na, T, seconds,
                           lat.ctypes.data, cap, cnt.ctypes.data, ctypes.byref(el))
    if rc != 0:
        raise RuntimeError(f"native caller loop failed: {rc}")
    got = np.concatenate([lat[t * cap:t * cap + int(cnt[t])] for t in range(T)])
    return float(cnt.sum()) / el.value, got


def _lat_rec(qps, lat_us, n, d, T):
    rec = {"qps": round(qps, 1), "calls": int(len(lat_us)),
           "latency_us": {"p50": round(float(np.percentile(lat_us, 50)), 1),
                          "p99": round(float(np.percentile(lat_us, 99)), 1),
                          "max": round(float(lat_us.max()), 1)}}
    if T == 1:
        rec["us_per_call"] = round(1e6 / qps, 2)
        rec["frac_of_8TBs"] = round(n * d * 4 * qps / 1e9 / HBM_PEAK_GBS, 4)
    return rec


def config_host_api(ctx, orc, callers=(1, 16), seconds=1.0):
    """The headline shape through the host API the Go binding calls: T caller
    threads (goroutines) each issuing single-query wvg_search calls (1M x 128
    L2, k = 10) for `seconds`; concurrent calls on one corpus are coalesced
    into shared launches inside the library (wvg_options.coalesce).  frac (one
    caller): N*d*4 bytes per call / the call's wall time vs 8 TB/s.  Per-call
    latency percentiles (the queries_durations_ms histogram's view,
    usecases/monitoring/prometheus.go:216) are taken around each call in the
    calling thread.  The callers are native threads (tools/host_calls.c: a
    goroutine's shape, whose cgo call adds ~0.1 us) when tools/libhostcalls.so
    was built; `python_caller_1` is the same single caller from a Python thread
    (~2-4 us more per call: interpreter + ctypes).  Filtered calls:
    every call carries one of 8 allow lists (helpers.AllowList bitmaps,
    V/flat/index.go:423-449) keeping 10 % or 1 % of the rows."""
    import threading

    from weaviate_amd._lib import KIND_F32, METRIC_L2, check, fptr, u32ptr, u64ptr
    from weaviate_amd.device import Context, Corpus, allow_bitmap

    n, d, k = 1_000_000, 128, 10
    qs = np.ascontiguousarray(orc.synth_rows(43, 0, 256, d, 0))
    out = {"workload": f"{n:,} x {d} fp32 L2 exact {k}-NN, one query per wvg_search call, T concurrent callers"}
    rng = np.random.default_rng(47)
    allows = {rate: [allow_bitmap(np.flatnonzero(rng.random(n) < rate), n) for _ in range(8)] for rate in (0.1, 0.01)}
    for coalesce in (1, 0):
        cx = ctx if coalesce else Context(ctx.device, coalesce=0)
        lib = cx.lib
        c = Corpus(cx, KIND_F32, METRIC_L2, d, n)
        c.fill_synthetic(42, n, 0)
        qp = [fptr(qs[i]) for i in range(len(qs))]

        def bufs_new():
            ids, ds, cnt = np.empty(k, np.uint64), np.empty(k, np.float32), np.empty(1, np.uint32)
            return (ids, ds, cnt), (u64ptr(ids), fptr(ds), u32ptr(cnt))

        bufs = [bufs_new() for _ in range(max(callers))]

        def call(t, i, allow=None):
            a = None if allow is None else allow[i % len(allow)]
            check(lib.wvg_search(c.handle, qp[i % len(qs)], 1, k, u64ptr(a) if a is not None else None,
                                 0 if a is None else len(a), *bufs[t][1]))

        # check: 16 concurrent calls return exactly what serial calls return
        serial = []
        for i in range(16):
            call(0, i)
            serial.append((bufs[0][0][0].copy(), bufs[0][0][1].copy()))
        got = [None] * 16

        def one(i):
            b = bufs_new()
            check(lib.wvg_search(c.handle, qp[i], 1, k, None, 0, *b[1]))
            got[i] = (b[0][0].copy(), b[0][1].copy())

        th = [threading.Thread(target=one, args=(i,)) for i in range(16)]
        [t.start() for t in th]
        [t.join() for t in th]
        same = all(np.array_equal(g[0], s[0]) and np.array_equal(g[1].view(np.uint32), s[1].view(np.uint32))
                   for g, s in zip(got, serial))
        tag = "coalesced" if coalesce else "uncoalesced"
        hc = _host_calls_lib()

        def drive(T, secs, allow=None):
            if hc is not None:
                return _native_callers(hc, lib, c.handle, qs, k, T, secs, allow)
            return _callers(call if allow is None else (lambda t, i: call(t, i, allow)), T, secs)

        for T in callers:
            qps, lat = drive(T, seconds)
            out[f"{tag}_callers_{T}"] = _lat_rec(qps, lat, n, d, T)
        if coalesce and hc is not None:  # the same single caller from a Python thread (ctypes + interpreter)
            qps, lat = _callers(call, 1, seconds / 2)
            out["python_caller_1"] = _lat_rec(qps, lat, n, d, 1)
        if coalesce and hc is not None:  # 64 callers: batches of up to 64 (the latency a caller pays under load)
            qps, lat = _native_callers(hc, lib, c.handle, qs, k, 64, seconds / 2)
            out["coalesced_callers_64"] = _lat_rec(qps, lat, n, d, 64)
        if hc is not None:  # 16 callers with k = 1 / 10 / 100 mixed (one coalesced batch runs at the largest k)
            qps, lat = _native_callers(hc, lib, c.handle, qs, k, 16, seconds / 2, ks=[10, 1, 100, 10])
            out[f"{tag}_mixed_k_callers_16"] = _lat_rec(qps, lat, n, d, 16)
        out[f"{tag}_16_concurrent_equal_serial"] = bool(same)
        if coalesce:  # filtered single queries, 10 % and 1 % allow lists
            for rate, al in allows.items():
                for T in callers:
                    qps, lat = drive(T, seconds / 2, al)
                    rec = _lat_rec(qps, lat, n, d, T)
                    rec.pop("frac_of_8TBs", None)  # a filtered scan skips tiles with no allowed row
                    out[f"filtered_{int(rate * 100)}pct_callers_{T}"] = rec
            # filtered concurrent calls = serial filtered calls
            fs = []
            for i in range(16):
                call(0, i, allows[0.01])
                fs.append(bufs[0][0][0].copy())
            fg = [None] * 16

            def onef(i):
                b = bufs_new()
                a = allows[0.01][i % 8]
                check(lib.wvg_search(c.handle, qp[i], 1, k, u64ptr(a), len(a), *b[1]))
                fg[i] = b[0][0].copy()

            th = [threading.Thread(target=onef, args=(i,)) for i in range(16)]
            [t.start() for t in th]
            [t.join() for t in th]
            out["filtered_16_concurrent_equal_serial"] = all(np.array_equal(x, y) for x, y in zip(fs, fg))
        c.destroy()
        if not coalesce:
            cx.close()
    return out


def run_configs(args, dev, torch):
    """The configs object of the bench line (N = 1): BASELINE configs 2-5."""
    from oracle import wv_oracle as orc  # the spot checks' checker only, never the measured path
    from weaviate_amd.device import Context

    want = [s for s in args.configs.split(",") if s]
    ctx = Context(dev.index)
    out = {}
    t_all = time.perf_counter()
    for name in want:
        t0 = time.perf_counter()
        try:
            if name == "batched":
                from weaviate_amd._lib import METRIC_COSINE, METRIC_DOT

                out["config2_batched_10m_x_768"] = {"cosine": config_batched(ctx, orc, "cosine", METRIC_COSINE),
                                                    "dot": config_batched(ctx, orc, "dot", METRIC_DOT)}
            elif name == "bq":
                out["config3_bq_100m_x_1536"] = config_bq(ctx, orc)
            elif name == "pq":
                out["config4_pq_100m_x_128"] = config_pq(ctx, orc)
            elif name == "slab":
                out["config5_slab_125m_x_128"] = config_slab(ctx, orc, dev, torch)
            elif name == "host_api":
                out["config1_host_api"] = config_host_api(ctx, orc)
        except Exception as e:  # noqa: BLE001 -- a failed leg is reported, the headline stands
            out[f"{name}_error"] = f"{type(e).__name__}: {e}"
        print(f"bench.py: config leg {name} {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    out["wall_s"] = round(time.perf_counter() - t_all, 1)
    ctx.close()
    return out


# ---------------------------------------------------------------------------
def _timed(fn, dist, world, dev, torch):
    """Barrier + synchronize on both sides of fn(); returns the max over ranks."""
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def stored_traffic(n, d, B):
    """HBM-side bytes per launch from the last rocprofv3 PMC pass over this
    exact workload (profiles/traffic.json, written by tools/traffic_from_pmc.py):
    FETCH_SIZE (x2, gfx950 half-count) counts Infinity-Cache hits as fetched,
    so it is the L2 -> fabric traffic, not DRAM traffic.  Not measured in this
    process (rocprofv3 cannot run inside the bench); labelled as stored."""
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        rec = json.load(open(tf)).get("scan_f32_stream_l2_128", {})
    except (OSError, ValueError):
        return None, None
    if rec.get("rows") != n or rec.get("dim") != d or "hbm_bytes_per_query_scan" not in rec:
        return None, None
    src = (f"stored, not measured in this run: profiles/traffic.json['scan_f32_stream_l2_128'] "
           f"({rec.get('source', '')}; {rec.get('method', '')})")
    return int(round(rec["hbm_bytes_per_query_scan"] * B)), src


def no_reuse_leg(args, dev, torch, n, d, k, B, tq, P, launches):
    """The headline kernel with nothing reused between scans: a context with
    wvg_options.cache_reuse = 0 (every scan walks upwards, every row load
    non-temporal) over n synthetic rows of the same shape -- n = 4M by default
    (2 GB, 8x the 256 MiB Infinity Cache; at 1M rows = 512 MB, about twice
    the cache, part of a streaming scan's rows may still be served on-die) -- same
    launch shape (B query scans per launch).  Returns the average launch time
    (s) from HIP events bound to each dispatch, and the context's HBM read
    ceiling (wvg_measure_hbm_read over 2 GiB)."""
    import ctypes

    from weaviate_amd._lib import KIND_F32, METRIC_L2, check
    from weaviate_amd.device import Context, Corpus

    cap = (n + 63) // 64 * 64
    ctx = Context(dev.index, cache_reuse=0)
    lib = ctx.lib
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, cap)
    c.fill_synthetic(42, n, 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    wsb = lib.wvg_search_workspace_size(c.handle, B, k)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    oi = torch.empty((B, k), dtype=torch.int64, device=dev)
    od = torch.empty((B, k), dtype=torch.float32, device=dev)
    oc = torch.empty(B, dtype=torch.int32, device=dev)

    def launch(s):
        check(lib.wvg_search_device_pipelined(c.handle, tq[(s * B) % P].data_ptr(), B, k, oi.data_ptr(),
                                              od.data_ptr(), oc.data_ptr(), ws.data_ptr(), wsb, stream))

    for s in range(2):
        launch(s)
    torch.cuda.synchronize(dev)
    check(lib.wvg_profile_start(ctx.handle))
    for s in range(launches):
        launch(s)
    ms, nl = ctypes.c_double(), ctypes.c_uint64()
    check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
    check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), stream))
    gbps = ctypes.c_double()
    check(lib.wvg_measure_hbm_read(ctx.handle, 2 << 30, 5, ctypes.byref(gbps)))
    c.destroy()
    ctx.close()
    return ms.value / 1e3 / max(1, nl.value), gbps.value


MERGE_CHECK_MAX_ROWS = 8_500_000  # the merged-result check's oracle regenerates every row on the host


def merge_check(ranges, d, k, qs, got_ids, got_d):
    """Rank 0's check of the (merged) top-k for the queries qs: the ids /
    distances equal the oracle's lexicographic top-k over every rank's or
    slab's rows, regenerated from the synthetic generator (at N = 1 the
    scan's own result; at N > 1 after the all-gather and the device merge,
    Index.objectVectorSearch, adapters/repos/db/index.go:1567-1648).  ranges:
    (first docID, rows) of each shard.  Checker only: runs after the timed
    region."""
    from oracle import wv_oracle as orc

    total = sum(r[1] for r in ranges)
    if total > MERGE_CHECK_MAX_ROWS:
        return {"ok": None, "skipped": f"{total:,} rows above the host oracle's {MERGE_CHECK_MAX_ROWS:,}"}
    best = [(np.empty(0, np.uint64), np.empty(0, np.float32)) for _ in qs]
    for base, nrows in ranges:
        for r0 in range(0, nrows, 1_000_000):
            m = min(1_000_000, nrows - r0)
            rows = orc.synth_rows(42, base + r0, m, d, 0)  # once per chunk, for every query
            ids = np.arange(base + r0, base + r0 + m, dtype=np.uint64)
            for qi in range(len(qs)):
                ci, cd = orc.lex_topk(orc.dist_all(0, qs[qi], rows), ids, k)
                bi, bd = best[qi]
                best[qi] = orc.lex_topk(np.concatenate([bd, cd]), np.concatenate([bi, ci]), k)
    ok = True
    for qi in range(len(qs)):
        bi, bd = best[qi]
        ok &= bool(np.array_equal(np.asarray(got_ids[qi]).view(np.uint64), bi)
                   and np.array_equal(np.asarray(got_d[qi], np.float32).view(np.uint32), bd.view(np.uint32)))
    return {"ok": ok, "queries": len(qs), "rows": total,
            "how": "ids and distance bits = the oracle's lexicographic top-k over every shard's rows"}


def run_flat1m(args, world, rank, dev, torch, dist):
    from weaviate_amd._lib import KIND_F32, METRIC_L2, check
    from weaviate_amd.device import Context, Corpus
    from weaviate_amd.shard import all_gather_packed

    n, d, k, B = args.rows, args.dim, args.k, args.batch
    cap = (n + 63) // 64 * 64
    ctx = Context(dev.index)
    lib = ctx.lib
    corpus = Corpus(ctx, KIND_F32, METRIC_L2, d, cap, id_base=rank * cap)
    corpus.fill_synthetic(42, n, 0)

    P = 64  # distinct queries cycled through the steps
    assert P % B == 0
    qs = np.random.default_rng(43).uniform(-1, 1, (P, d)).astype(np.float32)
    tq = torch.from_numpy(qs).to(dev)
    blk = lib.wvg_topk_packed_bytes(B, k)
    # two of each exchange buffer: step s's exchange + merge overlaps step s+1's scan
    send = [torch.empty(blk, dtype=torch.uint8, device=dev) for _ in range(2)]  # ids [B][k] then dists [B][k]
    counts = torch.empty(B, dtype=torch.int32, device=dev)
    ws_bytes = lib.wvg_search_workspace_size(corpus.handle, B, k)
    ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
    recv = [torch.empty(world * blk, dtype=torch.uint8, device=dev) for _ in range(2)]
    m_ids = [torch.empty((B, k), dtype=torch.int64, device=dev) for _ in range(2)]
    m_d = [torch.empty((B, k), dtype=torch.float32, device=dev) for _ in range(2)]
    m_c = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(2)]
    main_s = torch.cuda.current_stream(dev)
    stream = main_s.cuda_stream
    side = torch.cuda.Stream(dev) if world > 1 else None  # the exchange stream
    scanned = [torch.cuda.Event() for _ in range(2)]
    exchanged = [torch.cuda.Event() for _ in range(2)]

    def step(s):
        # B single-query scans in one call = one query-stream launch (each query a full scan)
        q0 = (s * B) % P
        b = s % 2
        if world > 1 and s >= 2:
            main_s.wait_event(exchanged[b])  # send[b] is free once step s-2's all-gather has read it
        check(lib.wvg_search_device_pipelined(corpus.handle, tq[q0].data_ptr(), B, k, send[b].data_ptr(),
                                              send[b].data_ptr() + B * k * 8, counts.data_ptr(), ws.data_ptr(),
                                              ws_bytes, stream))
        if world > 1:
            # ONE collective per step, on the exchange stream: RCCL moves step s's blocks and every
            # rank merges them while this rank's next scan runs on the main stream
            scanned[b].record(main_s)
            with torch.cuda.stream(side):
                side.wait_event(scanned[b])
                all_gather_packed(send[b], recv[b])
                check(lib.wvg_topk_merge_packed(ctx.handle, recv[b].data_ptr(), B, world, k, k, m_ids[b].data_ptr(),
                                                m_d[b].data_ptr(), m_c[b].data_ptr(), side.cuda_stream))
                exchanged[b].record(side)

    for s in range(args.warmup):
        step(s)
    check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), stream))
    import ctypes

    check(lib.wvg_profile_start(ctx.handle))
    elapsed = _timed(lambda: [step(args.warmup + s) for s in range(args.steps)], dist, world, dev, torch)
    scan_ms, launches = ctypes.c_double(), ctypes.c_uint64()
    check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(scan_ms), ctypes.byref(launches)))
    check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), stream))  # no merge gave up in the timed run
    # the last timed step's result against the oracle (untimed): at N = 1 the
    # query-stream launch's own packed block (every query of the step), at
    # N > 1 the exchanged + merged lists
    torch.cuda.synchronize(dev)
    last = args.warmup + args.steps - 1
    q0 = (last * B) % P
    mcheck = None
    if world > 1:
        if rank == 0:
            mcheck = merge_check([(r * cap, n) for r in range(world)], d, k, qs[q0:q0 + 2],
                                 m_ids[last % 2][:2].cpu().numpy(), m_d[last % 2][:2].cpu().numpy())
        dist.barrier()
    else:
        blk_h = send[last % 2].cpu().numpy()
        got_i = blk_h[:B * k * 8].view(np.uint64).reshape(B, k)
        got_d = blk_h[B * k * 8:B * k * 12].view(np.float32).reshape(B, k)
        mcheck = merge_check([(0, n)], d, k, qs[q0:q0 + B], got_i, got_d)
        mcheck["what"] = f"the last timed launch's {B} queries (scan_f32_stream_kernel's packed block)"

    total_queries = world * B * args.steps  # 1M-row query scans over all GPUs
    avg_launch_s = scan_ms.value / 1e3 / max(1, launches.value)
    bytes_per_launch = n * d * 4 * B  # N*d*4 algorithmic bytes per query scan
    achieved = bytes_per_launch / avg_launch_s / 1e9
    traffic, traffic_src = stored_traffic(n, d, B)  # per launch, like `achieved`
    # untimed: the same kernel with no reuse between scans, and the HBM read ceiling
    nr_rows = max(n, args.no_reuse_rows)
    if args.profile_run:
        nr_launch_s, ceiling, achieved_nr = float("nan"), float("nan"), float("nan")
    else:
        nr_launch_s, ceiling = no_reuse_leg(args, dev, torch, nr_rows, d, k, B, tq, P, max(4, min(args.steps, 10)))
        achieved_nr = nr_rows * d * 4 * B / nr_launch_s / 1e9
    out = {
        "metric": METRIC,
        "value": round(total_queries / elapsed, 3),
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
            "parallelism": (f"shard rows by docID range over {world} GPUs; one RCCL all-gather of packed "
                            f"per-GPU top-k blocks per step + device merge, on a second stream overlapping "
                            f"the next step's scan" if world > 1 else
                            "one GPU: no exchange (the scan's own top-k is the result)"),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": f"wvg::scan_f32_stream_kernel<L2,{d},1>",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "avg_launch_us": round(avg_launch_s * 1e6, 2),
            "queries_per_launch": B,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "launches": int(launches.value),
            "achieved_no_reuse": None if args.profile_run else round(achieved_nr, 1),
            "frac_no_reuse": None if args.profile_run else round(achieved_nr / HBM_PEAK_GBS, 4),
            "avg_launch_us_no_reuse": None if args.profile_run else round(nr_launch_s * 1e6, 2),
            "rows_no_reuse": nr_rows,
            "ceiling_GBps": None if args.profile_run else round(ceiling, 1),
            "frac_of_ceiling_no_reuse": (round(achieved_nr / ceiling, 4)
                                         if not args.profile_run and ceiling > 0 else None),
            "gpu_clock": gpu_clock(dev, torch),
            "note": ("`achieved` = ALGORITHMIC bytes (N*d*4 per query scan, every query a full scan) / the "
                     "kernel's average launch time, Infinity-Cache reuse included: consecutive scans alternate "
                     "direction and read the last ~320 MB of each pass with the default cache policy "
                     "(k1_cache_tail), so each scan starts on rows the previous one left in the 256 MiB "
                     "Infinity Cache -- it is not a DRAM rate and can exceed the DRAM read ceiling.  "
                     "`achieved_no_reuse` / `frac_no_reuse`: the same kernel and launch shape in a context with "
                     "wvg_options.cache_reuse = 0 (one direction, all loads non-temporal) over rows_no_reuse rows "
                     "(8x the Infinity Cache), measured in this run.  `ceiling_GBps`: wvg_measure_hbm_read (2 GiB non-temporal "
                     "streaming read) in this run.  `traffic`: see traffic_source"),
        },
        "cpu_baseline": None,
        "configs": None,
        "merge_check": mcheck,
    }
    legs = {}
    if args.scale_legs and not args.profile_run:
        # BASELINE configs[4] and configs[3] as strong scaling at this N (every rank takes part)
        for name in args.scale_legs.split(","):
            t0 = time.perf_counter()
            try:
                if name == "slab1b":
                    if 8 % world:  # the 8 slabs are dealt evenly (the driver's N = 1, 2, 4, 8)
                        legs["config5_1b_x_128"] = {"skipped": f"8 slabs do not deal evenly to {world} GPUs"}
                    else:
                        legs["config5_1b_x_128"] = slab1b_leg(world, rank, dev, torch, dist, total=args.s1b_rows)
                elif name == "pq":
                    legs["config4_pq_sharded"] = pq_sharded_leg(world, rank, dev, torch, dist, n=args.pq_rows)
                elif name == "multi":
                    r = multi_handle_leg(world, rank, dist)
                    if rank == 0:
                        legs["multi_gpu_one_process"] = r
            except Exception as e:  # noqa: BLE001 -- a failed leg is reported, the headline stands
                legs[f"{name}_error"] = f"{type(e).__name__}: {e}"
            if rank == 0:
                print(f"bench.py: scale leg {name} {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    if rank == 0 and world == 1 and args.configs and not args.profile_run:
        out["configs"] = run_configs(args, dev, torch)
    if legs:
        out["configs"] = dict(out["configs"] or {}, **legs)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_run:
        cq = np.random.default_rng(43).uniform(-1, 1, (16, d)).astype(np.float32)
        gids, _, _ = corpus.search(cq, k)  # GPU results of the baseline's first queries (full-size cross-check)

        def pq_check(codes, centers, pqs, kk):  # the same PQ queries on the GPU (K8e via wvg_search)
            from weaviate_amd._lib import KIND_PQ
            pc = Corpus(ctx, KIND_PQ, METRIC_L2, d, len(codes))
            try:
                pc.set_codebook(centers)
                pc.upsert_codes(np.arange(len(codes), dtype=np.uint64), codes)
                return pc.search(pqs, kk)[0]
            finally:
                pc.destroy()

        out["cpu_baseline"] = cpu_baseline(n, d, k, gids, args.cpu_seconds, pq_check)
    corpus.destroy()
    ctx.close()
    return out


SLAB_SAMPLE = 10_000  # rows sampled at the start, middle and end of every slab by the 1B property check


def sampled_check(total, per, S, d, k, qs, got_ids, got_d):
    """Rank 0's check of a merged result over a corpus too large for the host
    oracle (1B x 128): per query, the merged list is sorted in (distance,
    docID) order, holds k distinct ids inside the corpus, every distance is a
    bit-exact recomputation of its row (regenerated from the counter RNG), and
    no row of 3 x SLAB_SAMPLE sampled from every slab (start, middle, end) lies
    outside the result ahead of its k-th.  Checker only, after the timed region."""
    from oracle import wv_oracle as orc

    sample = []
    for s in range(S):
        n_s = max(0, min(per, total - s * per))
        for off in (0, n_s // 2 - SLAB_SAMPLE // 2, n_s - SLAB_SAMPLE):
            if n_s >= 3 * SLAB_SAMPLE:
                sample.append((s * per + off, SLAB_SAMPLE))
    sids = np.concatenate([np.arange(b, b + m, dtype=np.int64) for b, m in sample])
    srows = np.concatenate([orc.synth_rows(42, b, m, d, 0) for b, m in sample])
    ok = True
    for qi in range(len(qs)):
        gi = np.asarray(got_ids[qi]).view(np.uint64)
        gd = np.asarray(got_d[qi], np.float32)
        ok &= len(set(gi.tolist())) == k and bool(np.all(gi < total))
        ok &= _sorted_ok(orc, gd)
        rows = np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in gi])
        ok &= bool(np.array_equal(_bits(orc.dist_all(0, qs[qi], rows)), _bits(gd)))
        ok &= _outside_ok(orc, sids, orc.dist_all(0, qs[qi], srows), gi.astype(np.int64), gd)
    return {"ok": bool(ok), "queries": len(qs), "rows": total, "sampled_rows": int(len(sids)),
            "how": "merged lists sorted, k distinct ids, every distance a bit-exact recomputation of its row, no "
                   f"row of {len(sids):,} sampled (start / middle / end of each slab) ahead of the k-th"}


def multi_handle_leg(world, rank, dist, rows_per_gpu=1_000_000, d=128, k=10, B=16, calls=30):
    """The single-process multi-GPU design at this N (wvg_multi_*): rank 0
    opens all N GPUs of the job in ONE process -- one context and one RCCL
    communicator per device (ncclCommInitAll) -- deals N x 1M x 128 rows to
    them in docID slabs, and times host-API calls of B queries: per call every
    device scans its slab, one grouped RCCL all-gather moves the packed top-k
    blocks, device 0 merges (adapters/repos/db/index.go:1567-1648).  The other
    ranks wait at a barrier.  Rank 0's merged results are checked against the
    oracle over all N x 1M rows."""
    from weaviate_amd._lib import KIND_F32, METRIC_L2
    from weaviate_amd.device import Multi, MultiCorpus, device_count

    out = None
    if rank == 0:
        if device_count() < world:
            out = {"skipped": f"this process sees {device_count()} devices, fewer than {world}"}
        else:
            n = rows_per_gpu * world
            qs = np.random.default_rng(47).uniform(-1, 1, (64, d)).astype(np.float32)
            with Multi(list(range(world))) as m:
                mc = MultiCorpus(m, KIND_F32, METRIC_L2, d, n)
                try:
                    mc.fill_synthetic(42, n, 0)
                    for i in range(3):
                        mc.search(qs[(i * B) % 64:(i * B) % 64 + B], k)
                    t0 = time.perf_counter()
                    for i in range(calls):
                        q0 = (i * B) % 64
                        gi, gd, gc = mc.search(qs[q0:q0 + B], k)
                    wall = (time.perf_counter() - t0) / calls
                    slab = mc.shard(0)[2]
                    chk = merge_check([(s * slab, max(0, min(slab, n - s * slab))) for s in range(world)], d, k,
                                      qs[q0:q0 + 2], gi[:2], gd[:2])
                    out = {"workload": f"{world} x 1M x {d} fp32 L2 (docID slabs, one process), exact {k}-NN, "
                                       f"{B} queries per wvg_multi_search call",
                           "qps": round(B / wall, 1), "ms_per_call": round(wall * 1e3, 3), "ndev": m.ndev,
                           "exchange": "RCCL all-gather (ncclCommInitAll)" if m.uses_rccl else "peer copies",
                           "merge_check": chk}
                finally:
                    mc.destroy()
    if world > 1:
        dist.barrier()
    return out


def slab1b_leg(world, rank, dev, torch, dist, total=1_000_000_000, d=128, k=100, B=8, steps=2, W=1):
    """BASELINE configs[4] at N GPUs (strong scaling): the 1B x 128 fp32 L2
    corpus as 8 slabs of 125M rows dealt to the N ranks (8/N each).  A GPU
    holds one slab in HBM at a time, regenerated in place between slabs
    (generation untimed); every timed step scans B queries over it (one
    query-stream launch, exact 100-NN), then -- timed -- the per-slab lists
    are merged on device into this rank's packed block and exchanged with one
    RCCL all-gather + device merge (Index.objectVectorSearch's shard merge,
    adapters/repos/db/index.go:1567-1648).  At N = 1 all 8 slabs are scanned
    and merged: QPS_1 is measured, not derived.  Returns the measurements; rank
    0 checks the last step's merged lists on sampled rows."""
    import ctypes

    from weaviate_amd._lib import KIND_F32, METRIC_L2, check
    from weaviate_amd.device import Context, Corpus
    from weaviate_amd.shard import all_gather_packed

    S = 8  # slabs of the corpus
    per = (total + S - 1) // S
    per = (per + 63) // 64 * 64
    if S % world:
        raise ValueError(f"slab1b deals {S} slabs evenly, --gpus must divide {S}")
    mine = [s for s in range(S) if s % world == rank]
    L = len(mine)
    ctx = Context(dev.index)
    lib = ctx.lib
    qs = torch.from_numpy(np.random.default_rng(43).uniform(-1, 1, (steps * B, d)).astype(np.float32)).to(dev)
    # per (timed step, local slab) lists; warmup steps write into slot 0
    ids = torch.empty((steps, L, B, k), dtype=torch.int64, device=dev)
    dd = torch.empty((steps, L, B, k), dtype=torch.float32, device=dev)
    cc = torch.empty((steps, L, B), dtype=torch.int32, device=dev)
    blk = lib.wvg_topk_packed_bytes(B, k)
    send = torch.empty((steps, blk), dtype=torch.uint8, device=dev)
    recv = torch.empty((steps, world * blk), dtype=torch.uint8, device=dev)
    m_ids = torch.empty((steps, B, k), dtype=torch.int64, device=dev)
    m_d = torch.empty((steps, B, k), dtype=torch.float32, device=dev)
    m_c = torch.empty((steps, B), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    scan_s, gen_s, scan_ms_tot, launches_tot = 0.0, 0.0, 0.0, 0
    for j, s in enumerate(mine):
        n_s = max(0, min(per, total - s * per))
        t0 = time.perf_counter()
        c = Corpus(ctx, KIND_F32, METRIC_L2, d, per, id_base=s * per)
        if n_s:
            c.fill_synthetic(42, n_s, 0)  # untimed: the slab is (re)generated in place
        torch.cuda.synchronize(dev)
        gen_s += time.perf_counter() - t0
        wsb = lib.wvg_search_workspace_size(c.handle, B, k)
        ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)

        def scan(t, slot):
            check(lib.wvg_search_device_pipelined(c.handle, qs[(t % steps) * B].data_ptr(), B, k,
                                                  ids[slot, j].data_ptr(), dd[slot, j].data_ptr(),
                                                  cc[slot, j].data_ptr(), ws.data_ptr(), wsb, stream))

        for t in range(W):
            scan(t, 0)
        check(lib.wvg_profile_start(ctx.handle))
        scan_s += _timed(lambda: [scan(t, t) for t in range(steps)], dist, world, dev, torch)
        ms, nl = ctypes.c_double(), ctypes.c_uint64()
        check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
        check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), stream))
        scan_ms_tot += ms.value
        launches_tot += nl.value
        c.destroy()
        del ws

    def merge_all():
        for t in range(steps):
            # this GPU's slabs -> one list per query, straight into the packed block
            check(lib.wvg_topk_merge_device(ctx.handle, dd[t].data_ptr(), ids[t].data_ptr(), B, L, k, k,
                                            send[t].data_ptr(), send[t].data_ptr() + B * k * 8, m_c[t].data_ptr(),
                                            stream))
            if world > 1:
                all_gather_packed(send[t], recv[t])
                check(lib.wvg_topk_merge_packed(ctx.handle, recv[t].data_ptr(), B, world, k, k, m_ids[t].data_ptr(),
                                                m_d[t].data_ptr(), m_c[t].data_ptr(), stream))

    merge_s = _timed(merge_all, dist, world, dev, torch)
    elapsed = scan_s + merge_s
    mcheck = None
    if rank == 0:  # the last step's merged lists (untimed)
        if world > 1:
            gi, gd = m_ids[steps - 1][:2].cpu().numpy(), m_d[steps - 1][:2].cpu().numpy()
        else:  # one GPU: the local merge wrote the packed block (ids [B][k], then dists)
            blkh = send[steps - 1].cpu().numpy()
            gi = blkh[:B * k * 8].view(np.uint64).reshape(B, k)[:2]
            gd = blkh[B * k * 8:B * k * 12].view(np.float32).reshape(B, k)[:2]
        q2 = qs[(steps - 1) * B:(steps - 1) * B + 2].cpu().numpy()
        if total <= MERGE_CHECK_MAX_ROWS:
            mcheck = merge_check([(s * per, max(0, min(per, total - s * per))) for s in range(S)], d, k, q2, gi, gd)
        else:
            mcheck = sampled_check(total, per, S, d, k, q2, gi, gd)
    if world > 1:
        dist.barrier()
    avg_launch_s = scan_ms_tot / 1e3 / max(1, launches_tot)
    achieved = per * d * 4 * B / avg_launch_s / 1e9
    ctx.close()
    return {"qps": round(B * steps / elapsed, 3), "ms_per_step": round(elapsed / steps * 1e3, 3),
            "scan_ms_per_step": round(scan_s / steps * 1e3, 3), "merge_ms_per_step": round(merge_s / steps * 1e3, 3),
            "steps": steps, "warmup": W, "queries_per_step": B, "total_rows": total, "slabs": S,
            "slabs_per_gpu": L, "rows_per_slab": per, "k": k, "untimed_generation_s": round(gen_s, 2),
            "kernel": f"wvg::scan_f32_stream_kernel<L2,{d},2>",
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "avg_launch_us": round(avg_launch_s * 1e6, 2),
                         "algorithmic_bytes_per_launch": per * d * 4 * B, "launches": int(launches_tot),
                         "note": "per GPU (this rank's slab scans); the line's qps is over all GPUs"},
            "merge_check": mcheck}


def pq_sharded_leg(world, rank, dev, torch, dist, n=100_000_000, d=128, m=32, ks=256, k=10, B=16, steps=4, W=1):
    """BASELINE configs[3] "1 vs 8 GPUs" at N GPUs (strong scaling over one
    100M x 128 corpus): rank r holds docIDs shard_range(n, N, r) as fp32 rows;
    rank 0 fits the codebook (ProductQuantizer.Fit on the first 100k rows,
    CH/product_quantization.go:372-418) and broadcasts it once (RCCL), every
    rank encodes its own slab (K9, no collective; V/hnsw/compress.go:98-104
    per slab), then each step searches B queries: every rank's ADC scan of its
    codes (K8e, LUT in LDS) into its packed block, one all-gather, the device
    merge (ShardedFlatIndex.search_device).  Encode and search are timed with a
    barrier on both sides, max over ranks.  Rank 0 checks the last merged lists
    against the union of the gathered per-rank lists, and the ADC distances of
    the entries it owns against the oracle."""
    import ctypes

    from weaviate_amd._lib import KIND_F32, KIND_PQ, METRIC_L2, check, fptr, u32ptr, u64ptr
    from weaviate_amd.device import Context, Corpus
    from weaviate_amd.shard import ShardedFlatIndex, compress_slab, shard_range, unpack_blocks

    lo, cnt, per = shard_range(n, world, rank)
    ctx = Context(dev.index)
    lib = ctx.lib
    f = Corpus(ctx, KIND_F32, METRIC_L2, d, per, id_base=lo)
    if cnt:
        f.fill_synthetic(42, cnt, 0)
    centers = None
    fit_s = 0.0
    if rank == 0:
        nt = 100_000
        trows = np.empty((nt, d), np.float32)
        check(lib.wvg_synthetic_rows(ctx.handle, 42, u64ptr(np.arange(nt, dtype=np.uint64)), nt, d, 0, 0,
                                     fptr(trows)))
        centers = np.empty((m, ks, d // m), np.float32)
        passes = np.zeros(m, np.uint32)
        t0 = time.perf_counter()
        check(lib.wvg_pq_fit(ctx.handle, fptr(trows), nt, d, m, ks, nt, 7, fptr(centers), u32ptr(passes)))
        fit_s = time.perf_counter() - t0
    pq = Corpus(ctx, KIND_PQ, METRIC_L2, d, per, id_base=lo)
    grouped = world > 1
    cb = [None]

    def encode():
        if grouped:
            bdev = dev if dist.get_backend() == "nccl" else None  # gloo (one-GPU rehearsal): host tensors
            cb[0] = compress_slab(pq, f, centers, 0, None, bdev)
        else:
            pq.set_codebook(centers)
            check(lib.wvg_pq_encode_corpus(pq.handle, f.handle))
            cb[0] = centers

    encode()  # untimed first pass (codebook upload, encoder warm-up); the timed pass re-encodes
    enc_s = _timed(encode, dist, world, dev, torch)
    f.destroy()
    qs = torch.from_numpy(np.random.default_rng(46).uniform(-1, 1, (steps * B, d)).astype(np.float32)).to(dev)
    idx = ShardedFlatIndex(ctx, pq)
    res = [None]

    def search(t):
        res[0] = idx.search_device(qs[(t % steps) * B:(t % steps) * B + B], k)

    for t in range(W):
        search(t)
    check(lib.wvg_profile_start(ctx.handle))
    el = _timed(lambda: [search(t) for t in range(steps)], dist, world, dev, torch)
    ms, nl = ctypes.c_double(), ctypes.c_uint64()
    check(lib.wvg_profile_stop(ctx.handle, ctypes.byref(ms), ctypes.byref(nl)))
    idx.check()
    mcheck = None
    if rank == 0:
        from oracle import wv_oracle as orc

        gi, gd, gc = (x.cpu().numpy() for x in res[0])
        gi = gi.view(np.uint64)
        ok = bool(np.all(gc == k))
        if grouped:  # the merge: the lexicographic top-k of the union of every rank's gathered list
            b = next(iter(idx._bufs.values()))
            ui, ud = unpack_blocks(b.recv.cpu().numpy(), world, B, k)
            for qi in range(B):
                wi, wd = orc.lex_topk(ud[:, qi].reshape(-1), ui[:, qi].reshape(-1), k)
                ok &= bool(np.array_equal(gi[qi], wi) and np.array_equal(_bits(gd[qi]), _bits(wd)))
        q_last = qs[(steps - 1) * B:(steps - 1) * B + B].cpu().numpy()
        owned = 0
        for qi in (0, B - 1):  # the entries rank 0 owns: ADC distances bit-exact on their stored codes
            mine_ = (gi[qi] >= lo) & (gi[qi] < lo + cnt)
            ok &= _sorted_ok(orc, gd[qi])
            if mine_.any():
                codes, okc = pq.get_batch(gi[qi][mine_], pq_m=m)
                lut = orc.pq_lut(0, q_last[qi], cb[0])
                ok &= bool(okc.all() and np.array_equal(_bits([orc.pq_adc(0, lut, c) for c in codes]),
                                                        _bits(gd[qi][mine_])))
                owned += int(mine_.sum())
        mcheck = {"ok": bool(ok), "owned_entries_checked": owned,
                  "how": "merged lists = lexicographic top-k of the union of the gathered per-rank lists (N > 1); "
                         "sorted; rank 0's own entries' ADC distances bit-exact vs the oracle on their codes"}
    if world > 1:
        dist.barrier()
    pq.destroy()
    ctx.close()
    scan_s = ms.value / 1e3 / max(1, nl.value)  # one co-scheduled ADC launch of B queries on this rank
    return {"qps": round(B * steps / el, 2), "ms_per_step": round(el / steps * 1e3, 3), "queries_per_step": B,
            "steps": steps, "rows": n, "rows_per_gpu": per, "m": m, "ks": ks, "k": k,
            "fit_s_rank0": round(fit_s, 3), "encode_s": round(enc_s, 4), "encode_rows_per_s": round(n / enc_s, 1),
            "adc_launch_ms": round(scan_s * 1e3, 4),
            "kernel": "K8e scan_pq32_wide_kernel co-scheduled (B queries per launch, LUT images in LDS)",
            "note": "codebook fitted on rank 0 and broadcast; per-rank encode; per step one ADC launch per rank, "
                    "one all-gather of packed top-k blocks, device merge",
            "merge_check": mcheck}


def run_slab1b(args, world, rank, dev, torch, dist):
    if 8 % world:
        raise SystemExit(f"bench.py: slab1b deals 8 slabs evenly, --gpus must divide 8")
    r = slab1b_leg(world, rank, dev, torch, dist, args.rows, args.dim, args.k, args.batch, args.steps, args.warmup)
    total, d, k = args.rows, args.dim, args.k
    return {
        "metric": METRIC,
        "value": r["qps"],
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: uniform[-1,1) rows from a counter RNG (seed 42) generated in HBM slab by slab "
                "(generation untimed); uniform[-1,1) queries (seed 43)",
        "config": {
            "workload": f"flat exact {k}-NN over {total:,} x {d} fp32 L2 as {r['slabs']} slabs of "
                        f"{r['rows_per_slab']:,} rows (BASELINE configs[4]); {r['slabs_per_gpu']} slab(s) per GPU "
                        f"scanned in sequence",
            "total_rows": total, "dim": d, "k": k, "queries_per_step": args.batch, "slabs": r["slabs"],
            "slabs_per_gpu": r["slabs_per_gpu"],
            "parallelism": f"slabs dealt to {world} GPU(s); per step a device merge of the local slabs, one RCCL "
                           f"all-gather of packed top-{k} blocks and a device merge",
        },
        "roofline": dict(r["roofline"], traffic=None),
        "cpu_baseline": None,
        "merge_check": r["merge_check"],
    }


def dry_run(args, world, rank):
    """CPU rehearsal: the launch, the packed block and the one all-gather per
    step over gloo, with a plain numpy brute force standing in for the scan
    (no GPU, nothing timed against the metric)."""
    import torch
    import torch.distributed as dist

    from weaviate_amd.shard import all_gather_packed, pack_block, shard_range, unpack_blocks

    if world > 1:
        dist.init_process_group("gloo")
    n, d, k, B = 4096, 16, args.k, args.batch
    lo, cnt, _ = shard_range(n * world, world, rank)
    rng = np.random.default_rng(42)
    X = rng.uniform(-1, 1, (n * world, d)).astype(np.float32)[lo:lo + cnt]
    Q = np.random.default_rng(43).uniform(-1, 1, (B, d)).astype(np.float32)
    D = ((Q[:, None, :] - X[None]) ** 2).sum(-1)
    order = np.argsort(D, axis=1, kind="stable")[:, :k]
    ids = (order + lo).astype(np.uint64)
    send = torch.from_numpy(pack_block(ids, np.take_along_axis(D, order, 1).astype(np.float32)))
    recv = torch.empty(world * send.numel(), dtype=torch.uint8)
    if world > 1:
        all_gather_packed(send, recv)
    else:
        recv.copy_(send)
    gi, gd = unpack_blocks(recv.numpy(), world, B, k)
    assert gi.shape == (world, B, k)
    if world > 1:
        dist.destroy_process_group()
    return {"metric": METRIC, "value": None, "unit": "queries/s", "n_gpus": world, "steps": 0,
            "warmup": 0, "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "dry run (CPU, gloo): launch + packed all-gather rehearsal only",
            "config": {"workload": args.workload, "dry_run": True}, "roofline": None, "cpu_baseline": None}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus))  # nothing has touched a GPU in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        out = dry_run(args, world, rank)
    else:
        import torch
        import torch.distributed as dist

        if args.share_gpu:  # rehearsal on a one-GPU box: every rank on cuda:0, exchange over gloo
            local = 0
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            if args.share_gpu:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=dev)
        fn = run_slab1b if args.workload == "slab1b" else run_flat1m
        out = fn(args, world, rank, dev, torch, dist)
        if world > 1:
            dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
