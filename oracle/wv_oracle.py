"""ctypes wrapper of oracle/wv_oracle.c -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() (as the checker) and
bench.py's cpu_baseline leg.  The product (weaviate_amd/) never imports it.
Parity is pinned against the reference's own compiled C kernels
(oracle/_ref/libwvref.so, built by `make -C oracle ref` from /root/reference)
and against the known answers of the reference's Go tests (tests/golden/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_float, c_int, c_long, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "libwvoracle.so")
REF_SO = os.path.join(HERE, "_ref", "libwvref.so")

L2, DOT, COSINE, MANHATTAN, HAMMING = 0, 1, 2, 3, 4

_F = POINTER(c_float)
_U64 = POINTER(c_uint64)
_U8 = POINTER(c_uint8)
_REF_FN = ctypes.CFUNCTYPE(None, _F, _F, _F, POINTER(c_long))

_lib = None
_ref = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        l = ctypes.CDLL(ORACLE_SO)
        for n in ["orc_l2_256", "orc_dot_256", "orc_l2_512", "orc_dot_512", "orc_l2_step", "orc_dot_step",
                  "orc_manhattan", "orc_hamming_256", "orc_hamming_step"]:
            getattr(l, n).restype = c_float
            getattr(l, n).argtypes = [_F, _F, c_long]
        l.orc_single_dist.restype = c_float
        l.orc_single_dist.argtypes = [c_int, _F, _F, c_long]
        l.orc_step.restype = c_float
        l.orc_step.argtypes = [c_int, _F, _F, c_long]
        l.orc_normalize.argtypes = [_F, c_long, _F]
        l.orc_bq_encode.argtypes = [_F, c_long, _U64]
        l.orc_bq_distance.restype = c_float
        l.orc_bq_distance.argtypes = [_U64, _U64, c_long]
        l.orc_pq_lut.argtypes = [c_int, _F, _F, c_long, c_long, c_long, _F]
        l.orc_pq_adc.restype = c_float
        l.orc_pq_adc.argtypes = [c_int, _F, _U8, c_long, c_long]
        l.orc_pq_encode.argtypes = [_F, c_long, c_long, _F, c_long, c_long, _U8]
        l.orc_pq_fit.restype = c_long
        l.orc_pq_fit.argtypes = [_F, c_long, c_long, c_long, c_long, c_long, c_uint64, _F,
                                 ctypes.POINTER(c_uint32)]
        l.orc_pq_global_distances.argtypes = [c_int, _F, c_long, c_long, c_long, _F]
        l.orc_pq_sdc.restype = c_float
        l.orc_pq_sdc.argtypes = [c_int, _F, _U8, _U8, c_long, c_long]
        l.orc_kmeans_nearest.restype = c_uint32
        l.orc_kmeans_nearest.argtypes = [_F, _F, c_long, c_long]
        l.orc_heap_topk.restype = c_long
        l.orc_heap_topk.argtypes = [_F, _U64, _U8, c_long, c_long, _U64, _F]
        l.orc_flat_search.restype = c_long
        l.orc_flat_search.argtypes = [_F, c_long, c_long, c_long, _U8, _F, c_long, c_int, c_void_p, _U64, _F]
        l.orc_flat_search_bq.restype = c_long
        l.orc_flat_search_bq.argtypes = [_F, _U64, c_long, c_long, c_long, _U8, _F, c_long, c_long, c_int, _U64, _F,
                                         _U64]
        l.orc_heap_pops.restype = c_long
        l.orc_heap_pops.argtypes = [_F, c_long, _U8, c_long, _U64, _F]
        l.orc_synth_value.restype = c_float
        l.orc_synth_value.argtypes = [c_uint64, c_uint64, c_uint64, c_int]
        l.orc_synth_rows.argtypes = [c_uint64, c_uint64, c_long, c_long, c_long, c_int, _F]
        l.orc_dist_all.argtypes = [c_int, _F, _F, c_long, c_long, _F]
        l.orc_dist_all_512.argtypes = [c_int, _F, _F, c_long, c_long, _F]
        l.orc_bq_dist_all.argtypes = [_U64, _U64, c_long, c_long, _F]
        l.orc_bench_flat.restype = c_double
        l.orc_bench_flat.argtypes = [_F, c_long, c_long, c_long, _F, c_long, c_long, c_int, c_void_p, c_int, _U64, _F]
        l.orc_bench_flat_bq.restype = c_double
        l.orc_bench_flat_bq.argtypes = [_F, _U64, c_long, c_long, c_long, _F, c_long, c_long, c_long, c_int, c_void_p,
                                        c_int, _U64, _F]
        l.orc_bq_encode_rows.argtypes = [_F, c_long, c_long, _U64]
        l.orc_pq_search.restype = c_long
        l.orc_pq_search.argtypes = [_U8, c_long, c_long, c_long, c_long, _F, _F, c_long, c_int, _F, _U64, _F]
        l.orc_bench_pq.restype = c_double
        l.orc_bench_pq.argtypes = [_U8, c_long, c_long, c_long, c_long, _F, _F, c_long, c_long, c_int, c_int, _U64,
                                   _F]
        _lib = l
    return _lib


def ref():
    """The reference's own l2_256/l2_512/dot_256/dot_512/hamming_256/hamming_512
    (None if not built)."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        _ref = ctypes.CDLL(REF_SO)
    return _ref


def _f(a):
    return a.ctypes.data_as(_F)


def _u64(a):
    return a.ctypes.data_as(_U64)


def _u8(a):
    return a.ctypes.data_as(_U8)


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def l2_256(a, b):
    a, b = f32(a), f32(b)
    return np.float32(lib().orc_l2_256(_f(a), _f(b), len(a)))


def dot_256(a, b):
    a, b = f32(a), f32(b)
    return np.float32(lib().orc_dot_256(_f(a), _f(b), len(a)))


def ref_symbol(metric):
    """The reference C kernel behind a metric on an AVX2 host (None for
    manhattan, which is pure Go)."""
    return {L2: "l2_256", DOT: "dot_256", COSINE: "dot_256", HAMMING: "hamming_256"}.get(metric)


def manhattan(a, b):
    a, b = f32(a), f32(b)
    return np.float32(lib().orc_manhattan(_f(a), _f(b), len(a)))


def hamming_256(a, b):
    a, b = f32(a), f32(b)
    return np.float32(lib().orc_hamming_256(_f(a), _f(b), len(a)))


def single_dist(metric, a, b):
    a, b = f32(a), f32(b)
    return np.float32(lib().orc_single_dist(metric, _f(a), _f(b), len(a)))


def step(metric, a, b):
    a, b = f32(a), f32(b)
    return np.float32(lib().orc_step(metric, _f(a), _f(b), len(a)))


def dist_all(metric, q, rows):
    """SingleDist(q, row) for all rows (no normalization applied)."""
    q, rows = f32(q), f32(rows)
    out = np.empty(rows.shape[0], dtype=np.float32)
    lib().orc_dist_all(metric, _f(q), _f(rows), rows.shape[0], rows.shape[1], _f(out))
    return out


def dist_all_512(metric, q, rows):
    """SingleDist(q, row) for all rows with the AVX-512 kernels (AMX hosts)."""
    q, rows = f32(q), f32(rows)
    out = np.empty(rows.shape[0], dtype=np.float32)
    lib().orc_dist_all_512(metric, _f(q), _f(rows), rows.shape[0], rows.shape[1], _f(out))
    return out


def bq_dist_all(qcode, codes):
    qcode = np.ascontiguousarray(qcode, dtype=np.uint64)
    codes = np.ascontiguousarray(codes, dtype=np.uint64)
    out = np.empty(codes.shape[0], dtype=np.float32)
    lib().orc_bq_dist_all(_u64(qcode), _u64(codes), codes.shape[0], codes.shape[1], _f(out))
    return out


def normalize_rows(X):
    X = f32(X)
    return np.stack([normalize(r) for r in X]) if len(X) else X.copy()


def normalize(v):
    v = f32(v)
    out = np.empty_like(v)
    lib().orc_normalize(_f(v), len(v), _f(out))
    return out


def bq_encode(v):
    v = f32(v)
    out = np.empty((len(v) + 63) // 64, dtype=np.uint64)
    lib().orc_bq_encode(_f(v), len(v), _u64(out))
    return out


def bq_distance(x, y):
    x = np.ascontiguousarray(x, dtype=np.uint64)
    y = np.ascontiguousarray(y, dtype=np.uint64)
    return np.float32(lib().orc_bq_distance(_u64(x), _u64(y), len(x)))


def pq_lut(metric, q, centers):
    q, centers = f32(q), f32(centers)
    m, ks, ds = centers.shape
    out = np.empty((m, ks), dtype=np.float32)
    lib().orc_pq_lut(metric, _f(q), _f(centers), m, ks, ds, _f(out))
    return out


def pq_adc(metric, lut, code):
    lut = f32(lut)
    code = np.ascontiguousarray(code, dtype=np.uint8)
    m, ks = lut.shape
    return np.float32(lib().orc_pq_adc(metric, _f(lut), _u8(code), m, ks))


def pq_encode(X, centers):
    X, centers = f32(X), f32(centers)
    n, d = X.shape
    m, ks, _ = centers.shape
    out = np.empty((n, m), dtype=np.uint8)
    lib().orc_pq_encode(_f(X), n, d, _f(centers), m, ks, _u8(out))
    return out


def pq_fit(X, m, ks, training_limit=100_000, seed=0):
    """ProductQuantizer.Fit (k-means) restated: CH/product_quantization.go:372-418,
    CH/kmeans.go:146-250; returns (centers [m][ks][ds], passes per segment)."""
    X = f32(X)
    n, d = X.shape
    centers = np.empty((m, ks, d // m), dtype=np.float32)
    it = np.zeros(m, dtype=np.uint32)
    rc = lib().orc_pq_fit(_f(X), n, d, m, ks, training_limit, seed, _f(centers),
                          it.ctypes.data_as(ctypes.POINTER(c_uint32)))
    if rc != 0:
        raise ValueError("not enough data to fit kmeans")
    return centers, it


def pq_global_distances(metric, centers):
    centers = f32(centers)
    m, ks, ds = centers.shape
    out = np.empty((m, ks, ks), dtype=np.float32)
    lib().orc_pq_global_distances(metric, _f(centers), m, ks, ds, _f(out))
    return out


def pq_sdc(metric, table, x, y):
    table = f32(table)
    m, ks, _ = table.shape
    return lib().orc_pq_sdc(metric, _f(table), _u8(np.ascontiguousarray(x, np.uint8)),
                            _u8(np.ascontiguousarray(y, np.uint8)), m, ks)


def heap_topk(dists, ids, k, valid=None):
    dists = f32(dists)
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    oid = np.empty(max(k, 1), dtype=np.uint64)
    od = np.empty(max(k, 1), dtype=np.float32)
    v = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
    n = lib().orc_heap_topk(_f(dists), _u64(ids), _u8(v) if v is not None else None, len(dists), k, _u64(oid),
                            _f(od))
    return oid[:n], od[:n]


def flat_search(rows, q, k, metric, valid=None, use_ref_kernel=False):
    """flat.searchByVector restated over a dense matrix; q must be normalized for cosine."""
    rows, q = f32(rows), f32(q)
    n, d = rows.shape
    oid = np.empty(max(k, 1), dtype=np.uint64)
    od = np.empty(max(k, 1), dtype=np.float32)
    fn = None
    if use_ref_kernel and ref_symbol(metric):
        fn = ctypes.cast(getattr(ref(), ref_symbol(metric)), c_void_p)
    v = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
    cnt = lib().orc_flat_search(_f(rows), n, d, d, _u8(v) if v is not None else None, _f(q), k, metric, fn, _u64(oid),
                                _f(od))
    return oid[:cnt], od[:cnt]


def flat_search_bq(rows, q, k, rescore_limit, metric, valid=None):
    """flat.searchByVectorBQ restated; q must be normalized for cosine."""
    rows, q = f32(rows), f32(q)
    n, d = rows.shape
    codes = np.stack([bq_encode(r) for r in rows]) if n else np.zeros((0, (d + 63) // 64), np.uint64)
    codes = np.ascontiguousarray(codes)
    R = max(rescore_limit, k)
    oid = np.empty(max(k, 1), dtype=np.uint64)
    od = np.empty(max(k, 1), dtype=np.float32)
    cand = np.empty(max(R, 1), dtype=np.uint64)
    v = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
    cnt = lib().orc_flat_search_bq(_f(rows), _u64(codes), n, d, d, _u8(v) if v is not None else None, _f(q), k,
                                   rescore_limit, metric, _u64(oid), _f(od), _u64(cand))
    return oid[:cnt], od[:cnt]


def heap_pops(dists, rescore, valid=None):
    """findTopVectorsCached's heap of `rescore` over ids 0..n-1 with these
    distances, and the pop loop of searchByVectorBQ (V/flat/index.go:369-374):
    (ids, dists) in pop order."""
    dists = f32(dists)
    oid = np.empty(max(rescore, 1), dtype=np.uint64)
    od = np.empty(max(rescore, 1), dtype=np.float32)
    v = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
    cnt = lib().orc_heap_pops(_f(dists), len(dists), _u8(v) if v is not None else None, rescore, _u64(oid), _f(od))
    return oid[:cnt], od[:cnt]


def bq_heap_pops(codes, qcode, rescore, valid=None):
    """heap_pops over the Hamming distances of codes [n][w] to qcode."""
    return heap_pops(bq_dist_all(qcode, codes), rescore, valid)


def synth_rows(seed, row0, n, d, dist=0):
    out = np.empty((n, d), dtype=np.float32)
    lib().orc_synth_rows(seed, row0, n, d, d, dist, _f(out))
    return out


def bench_flat(rows, qs, k, metric, threads, use_ref_kernel=True):
    """Times nq flat searches, one query per thread at a time; returns seconds."""
    rows, qs = f32(rows), f32(qs)
    n, d = rows.shape
    nq = qs.shape[0]
    fn = None
    if use_ref_kernel and ref() is not None and ref_symbol(metric):
        fn = ctypes.cast(getattr(ref(), ref_symbol(metric)), c_void_p)
    oid = np.empty((nq, k), dtype=np.uint64)
    od = np.empty((nq, k), dtype=np.float32)
    secs = lib().orc_bench_flat(_f(rows), n, d, d, _f(qs), nq, k, metric, fn, threads, _u64(oid), _f(od))
    return secs, oid, od, fn is not None


def bq_encode_rows(rows):
    """BinaryQuantizer.Encode of every row -> codes [n][ceil(d/64)]."""
    rows = f32(rows)
    n, d = rows.shape
    codes = np.empty((n, (d + 63) // 64), dtype=np.uint64)
    lib().orc_bq_encode_rows(_f(rows), n, d, _u64(codes))
    return codes


def bench_flat_bq(rows, codes, qs, k, rescore_limit, metric, threads, use_ref_kernel=True):
    """Times nq flat BQ searches (Hamming top-R over the codes, exact rescore
    of R, top-k), one query per thread at a time; returns seconds."""
    rows, qs = f32(rows), f32(qs)
    codes = np.ascontiguousarray(codes, dtype=np.uint64)
    n, d = rows.shape
    nq = qs.shape[0]
    fn = None
    if use_ref_kernel and ref() is not None and ref_symbol(metric):
        fn = ctypes.cast(getattr(ref(), ref_symbol(metric)), c_void_p)
    oid = np.empty((nq, k), dtype=np.uint64)
    od = np.empty((nq, k), dtype=np.float32)
    secs = lib().orc_bench_flat_bq(_f(rows), _u64(codes), n, d, d, _f(qs), nq, k, rescore_limit, metric, fn, threads,
                                   _u64(oid), _f(od))
    return secs, oid, od, fn is not None


def pq_search(codes, centers, q, k, metric):
    """PQ ADC top-k of one query over codes [n][m] (LUT + sequential ADC sums +
    flat heap; CH/product_quantization.go:85-104,352-361)."""
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    centers, q = f32(centers), f32(q)
    n, m = codes.shape
    _, ks, ds = centers.shape
    lut = np.empty(m * ks, dtype=np.float32)
    oid = np.empty(max(k, 1), dtype=np.uint64)
    od = np.empty(max(k, 1), dtype=np.float32)
    cnt = lib().orc_pq_search(_u8(codes), n, m, ks, ds, _f(centers), _f(q), k, metric, _f(lut), _u64(oid), _f(od))
    return oid[:cnt], od[:cnt]


def bench_pq(codes, centers, qs, k, metric, threads):
    """Times nq PQ ADC searches, one query per thread at a time; returns
    (seconds, ids [nq][k], dists [nq][k])."""
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    centers, qs = f32(centers), f32(qs)
    n, m = codes.shape
    _, ks, ds = centers.shape
    nq = qs.shape[0]
    oid = np.empty((nq, k), dtype=np.uint64)
    od = np.empty((nq, k), dtype=np.float32)
    secs = lib().orc_bench_pq(_u8(codes), n, m, ks, ds, _f(centers), _f(qs), nq, k, metric, threads, _u64(oid),
                              _f(od))
    return secs, oid, od


def ord_key(dists):
    """Order-preserving u32 of float32 distances (weaviate_amd/csrc/wvg_common.hpp
    wvg_ord_f32): NaN -> +NaN (after +Inf); -0 sorts before +0."""
    u = f32(dists).view(np.uint32).copy()
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x007FFFFF) != 0)
    u[nan] = 0x7FC00000
    neg = (u & 0x80000000) != 0
    return np.where(neg, ~u, u | np.uint32(0x80000000)).astype(np.uint32)


def lex_topk(dists, ids, k):
    """Lexicographic (dist, id) top-k -- the GPU's documented tie rule."""
    dists = f32(dists)
    ids = np.asarray(ids, dtype=np.uint64)
    order = np.lexsort((ids, ord_key(dists)))[:k]
    return ids[order], dists[order]


def search_by_distance(search_fn, target, max_limit):
    """SearchByVectorDistance's growing-limit loop, restated from
    V/hnsw/search.go:85-151 (the loop V/flat/index.go:531-591 intends) with
    V/common/search_by_dist_params.go:14-83 (limits 100, then offset = total,
    limit *= 10) and floatcomp.InDelta (usecases/floatcomp/delta.go:16-19).
    search_fn(total) -> (ids, dists) ascending, as SearchByVector."""
    target = np.float32(target)
    offset, limit = 0, 100
    total = offset + limit
    res_i, res_d = [], []

    def recursive():
        ids, dist = search_fn(total)
        lo, hi = min(offset, len(ids)), min(total, len(ids))
        ids, dist = ids[lo:hi], dist[lo:hi]
        if len(ids) == 0:
            return False
        cont = bool(np.float32(dist[-1]) <= target)
        for i in range(len(ids)):
            if np.float32(dist[i]) <= target or abs(float(dist[i]) - float(target)) <= 1e-6:
                res_i.append(int(ids[i]))
                res_d.append(np.float32(dist[i]))
            else:
                break
        return cont

    cont = recursive()
    while cont:
        offset = total
        limit *= 10
        total = offset + limit
        if max_limit >= 0 and total > max_limit:
            break
        cont = recursive()
    return np.asarray(res_i, dtype=np.uint64), np.asarray(res_d, dtype=np.float32)


def search_by_distance_flat(search_fn, target, max_limit, max_iterations=1000):
    """flat.SearchByVectorDistance restated literally from V/flat/index.go:
    531-591 with V/common/search_by_dist_params.go:14-83.  search_fn(total) ->
    (ids, dists) ascending, as SearchByVector.  The loop's `for` has no post
    statement, so recursiveSearch runs once and later iterations only grow the
    limit (Iterate) until MaxLimitReached -- with max_limit < 0 and a first
    window that asks to continue, the reference never returns: that case is
    reported as nonterminating (after max_iterations) with the results so far.
    Returns (ids, dists, terminated)."""
    target = np.float32(target)
    offset, limit = 0, 100
    total = offset + limit
    res_i, res_d = [], []

    def recursive():
        ids, dist = search_fn(total)
        cont = not (len(ids) < total)
        lo, hi = min(offset, len(ids)), min(total, len(ids))
        if lo == hi:
            return False
        for i in range(lo, hi):
            if np.float32(dist[i]) <= target or abs(float(dist[i]) - float(target)) <= 1e-6:
                res_i.append(int(ids[i]))
                res_d.append(np.float32(dist[i]))
            else:
                cont = False
                break
        return cont

    cont = recursive()
    it = 0
    terminated = True
    while cont:
        offset = total  # searchParams.Iterate()
        limit *= 10
        total = offset + limit
        if max_limit >= 0 and total > max_limit:
            break
        it += 1
        if it >= max_iterations:
            terminated = False
            break
    return np.asarray(res_i, dtype=np.uint64), np.asarray(res_d, dtype=np.float32), terminated
