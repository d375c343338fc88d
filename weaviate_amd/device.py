"""Device context and device-resident corpora (handles of the C ABI).

One :class:`Context` per GPU.  Several GPUs serve one index either from one
process (:class:`Multi` / :class:`MultiCorpus`: wvg_multi_*, RCCL inside the
library) or with one process per GPU (weaviate_amd/shard.py, RCCL through
torch.distributed).
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_uint64, c_void_p

import numpy as np

from . import _lib
from ._lib import check, fptr, u32ptr, u64ptr


def device_count() -> int:
    lib = _lib.load()
    n = c_int(0)
    check(lib.wvg_device_count(byref(n)))
    return n.value


class Context:
    """wvg_open_ex / wvg_close.  Keyword options set the fields of
    wvg_options (mfma_min_queries, cache_reuse, merge_wait_us, batch_screen);
    the others keep wvg_options_default's values."""

    def __init__(self, device: int = 0, **options):
        self.lib = _lib.load()
        opts = _lib.Options()
        self.lib.wvg_options_default(byref(opts))
        for name, value in options.items():
            if name == "size" or name not in dict(_lib.Options._fields_):
                raise TypeError(f"unknown context option {name!r}")
            setattr(opts, name, int(value))
        h = c_void_p()
        check(self.lib.wvg_open_ex(device, byref(opts), byref(h)))
        self.handle = h
        self.device = device
        self.options = {name: getattr(opts, name) for name, _ in _lib.Options._fields_ if name != "size"}

    def close(self) -> None:
        if self.handle:
            self.lib.wvg_close(self.handle)
            self.handle = c_void_p()

    def synchronize(self) -> None:
        check(self.lib.wvg_synchronize(self.handle))

    def host_array(self, shape, dtype=np.float32):
        """wvg_host_alloc: a numpy array over page-locked host memory, which the
        entry points copy from / to without a staging copy; freed with
        free_host_array (the array must not be used afterwards)."""
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        p = c_void_p()
        check(self.lib.wvg_host_alloc(self.handle, max(n, 1), byref(p)))
        buf = (ctypes.c_uint8 * max(n, 1)).from_address(p.value)
        arr = np.frombuffer(buf, dtype=np.uint8, count=n).view(dt).reshape(shape)
        self._pinned = getattr(self, "_pinned", {})
        self._pinned[arr.ctypes.data] = p
        return arr

    def free_host_array(self, arr) -> None:
        p = self._pinned.pop(arr.ctypes.data)
        check(self.lib.wvg_host_free(self.handle, p))

    def set_distance_order(self, order: int) -> None:
        """wvg_set_distance_order: _lib.ORDER_AVX256 (default) or ORDER_AVX512
        (the kernels Weaviate dispatches on AMX + AVX-512 hosts)."""
        check(self.lib.wvg_set_distance_order(self.handle, order))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def allow_bitmap(ids, n_bits: int | None = None) -> np.ndarray:
    """helpers.AllowList -> bitmap over global docIDs (bit i of word i/64)."""
    ids = np.asarray(list(ids), dtype=np.uint64)
    top = int(ids.max()) + 1 if ids.size else 0
    n_bits = max(n_bits or 0, top)
    words = np.zeros((n_bits + 63) // 64, dtype=np.uint64)
    if ids.size:
        np.bitwise_or.at(words, (ids >> np.uint64(6)).astype(np.int64),
                         np.left_shift(np.uint64(1), ids & np.uint64(63)))
    return words


class Corpus:
    """A device-resident corpus (wvg_corpus_*): F32 rows, BQ codes or PQ codes."""

    def __init__(self, ctx: Context, kind: int, metric: int, dim: int, capacity: int, id_base: int = 0):
        self.ctx = ctx
        self.lib = ctx.lib
        self.kind, self.metric, self.dim, self.id_base = kind, metric, dim, id_base
        h = c_void_p()
        check(self.lib.wvg_corpus_create(ctx.handle, kind, metric, dim, id_base, capacity, byref(h)))
        self.handle = h

    def destroy(self) -> None:
        if self.handle:
            self.lib.wvg_corpus_destroy(self.handle)
            self.handle = c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    def info(self):
        cnt, hw, cap = c_uint64(), c_uint64(), c_uint64()
        check(self.lib.wvg_corpus_info(self.handle, byref(cnt), byref(hw), byref(cap)))
        return cnt.value, hw.value, cap.value

    def reserve(self, capacity: int) -> None:
        check(self.lib.wvg_corpus_reserve(self.handle, capacity))

    def upsert(self, ids, vectors) -> None:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        vectors = np.ascontiguousarray(vectors, dtype=np.float32)
        if vectors.ndim == 1:
            vectors = vectors[None, :]
        check(self.lib.wvg_corpus_upsert(self.handle, u64ptr(ids), fptr(vectors), len(ids),
                                         vectors.shape[1] if vectors.size else self.dim))

    def upsert_codes(self, ids, codes) -> None:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        codes = np.ascontiguousarray(codes)
        check(self.lib.wvg_corpus_upsert_codes(self.handle, u64ptr(ids), codes.ctypes.data_as(c_void_p), len(ids)))

    def load_kv(self, keys, values) -> None:
        """wvg_corpus_load_kv: an LSM cursor's (8-byte big-endian key, LE row) pairs."""
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, 8)
        values = np.ascontiguousarray(values, dtype=np.uint8).reshape(len(keys), -1)
        check(self.lib.wvg_corpus_load_kv(self.handle, keys.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                          values.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(keys),
                                          values.shape[1]))

    def distance_by_ids(self, query, ids):
        """wvg_corpus_distance_by_ids: (dists, ok) of the query to the rows with these docIDs."""
        q = np.ascontiguousarray(query, dtype=np.float32).reshape(-1)
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        out = np.empty(len(ids), dtype=np.float32)
        ok = np.empty(len(ids), dtype=np.uint8)
        check(self.lib.wvg_corpus_distance_by_ids(self.handle, fptr(q), u64ptr(ids), len(ids), fptr(out),
                                                  ok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out, ok.astype(bool)

    def distance_by_ids_batch(self, queries, id_lists):
        """wvg_corpus_distance_by_ids_batch: one launch for many queries' id lists;
        returns [(dists, ok)] per query."""
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(len(id_lists), -1)
        lists = [np.ascontiguousarray(x, dtype=np.uint64).reshape(-1) for x in id_lists]
        offsets = np.zeros(len(lists) + 1, dtype=np.uint64)
        offsets[1:] = np.cumsum([len(x) for x in lists])
        ids = np.concatenate(lists) if lists else np.empty(0, np.uint64)
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        out = np.empty(len(ids), dtype=np.float32)
        ok = np.empty(len(ids), dtype=np.uint8)
        check(self.lib.wvg_corpus_distance_by_ids_batch(self.handle, fptr(q), len(lists), u64ptr(offsets), u64ptr(ids),
                                                        fptr(out), ok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        res = []
        for i in range(len(lists)):
            a, b = int(offsets[i]), int(offsets[i + 1])
            res.append((out[a:b], ok[a:b].astype(bool)))
        return res

    def delete(self, ids) -> None:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        check(self.lib.wvg_corpus_delete(self.handle, u64ptr(ids), len(ids)))

    def get(self, id_: int, pq_m: int = 0) -> np.ndarray:
        if self.kind == _lib.KIND_F32:
            out = np.empty(self.dim, dtype=np.float32)
        elif self.kind == _lib.KIND_BQ:
            out = np.empty((self.dim + 63) // 64, dtype=np.uint64)
        else:
            out = np.empty(pq_m, dtype=np.uint8)
        check(self.lib.wvg_corpus_get(self.handle, id_, out.ctypes.data_as(c_void_p)))
        return out

    def get_batch(self, ids, pq_m: int = 0):
        """wvg_corpus_get_batch: (rows [n][...], ok [n]) for many docIDs in one call."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1)
        n = len(ids)
        if self.kind == _lib.KIND_F32:
            out = np.empty((n, self.dim), dtype=np.float32)
        elif self.kind == _lib.KIND_BQ:
            out = np.empty((n, (self.dim + 63) // 64), dtype=np.uint64)
        else:
            out = np.empty((n, pq_m), dtype=np.uint8)
        ok = np.empty(n, dtype=np.uint8)
        check(self.lib.wvg_corpus_get_batch(self.handle, u64ptr(ids), n, out.ctypes.data_as(c_void_p),
                                            ok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out, ok.astype(bool)

    def fill_synthetic(self, seed: int, n: int, distribution: int = 0) -> None:
        check(self.lib.wvg_corpus_fill_synthetic(self.handle, seed, n, distribution))

    def set_codebook(self, centers) -> None:
        centers = np.ascontiguousarray(centers, dtype=np.float32)
        m, ks, _ = centers.shape
        check(self.lib.wvg_pq_set_codebook(self.handle, fptr(centers), m, ks))

    def search(self, queries, k: int, allow=None):
        """wvg_search: returns (ids [nq][k], dists [nq][k], counts [nq])."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        ids = np.empty((nq, k), dtype=np.uint64)
        dists = np.empty((nq, k), dtype=np.float32)
        counts = np.empty(nq, dtype=np.uint32)
        aw, an = (None, 0) if allow is None else (np.ascontiguousarray(allow, dtype=np.uint64), len(allow))
        check(self.lib.wvg_search(self.handle, fptr(q), nq, k, u64ptr(aw) if aw is not None else None, an,
                                  u64ptr(ids), fptr(dists), u32ptr(counts)))
        return ids, dists, counts

    def search_by_distance(self, query, target: float, max_limit: int = -1, allow=None, capacity: int | None = None):
        """wvg_search_by_distance: (ids, dists) of every row within `target`
        (flat.SearchByVectorDistance, V/flat/index.go:531-591)."""
        q = np.ascontiguousarray(query, dtype=np.float32).reshape(-1)
        aw, an = (None, 0) if allow is None else (np.ascontiguousarray(allow, dtype=np.uint64), len(allow))
        cnt = c_uint64()
        cap = capacity if capacity is not None else max(1, self.info()[1])
        while True:
            ids = np.empty(cap, dtype=np.uint64)
            dists = np.empty(cap, dtype=np.float32)
            check(self.lib.wvg_search_by_distance(self.handle, fptr(q), float(target), int(max_limit),
                                                  u64ptr(aw) if aw is not None else None, an, u64ptr(ids),
                                                  fptr(dists), cap, byref(cnt)))
            if cnt.value <= cap:
                return ids[:cnt.value], dists[:cnt.value]
            cap = cnt.value

    def search_by_distance_window(self, query, target: float, window: int = 100, allow=None):
        """wvg_search_by_distance_window: the flat index's own range-search
        result (its first window, V/flat/index.go:531-591 as written)."""
        q = np.ascontiguousarray(query, dtype=np.float32).reshape(-1)
        aw, an = (None, 0) if allow is None else (np.ascontiguousarray(allow, dtype=np.uint64), len(allow))
        cnt = c_uint64()
        ids = np.empty(max(1, window), dtype=np.uint64)
        dists = np.empty(max(1, window), dtype=np.float32)
        check(self.lib.wvg_search_by_distance_window(self.handle, fptr(q), float(target), int(window),
                                                     u64ptr(aw) if aw is not None else None, an, u64ptr(ids),
                                                     fptr(dists), len(ids), byref(cnt)))
        return ids[:cnt.value], dists[:cnt.value]


def search_bq_candidates(bq: Corpus, queries, rescore_limit: int, allow=None):
    """wvg_search_bq_candidates: findTopVectorsCached's heap of rescore_limit and
    its pop order (V/flat/index.go:355-374): (ids [nq][R], dists [nq][R], counts)."""
    q = np.ascontiguousarray(queries, dtype=np.float32)
    if q.ndim == 1:
        q = q[None, :]
    nq, R = q.shape[0], rescore_limit
    ids = np.empty((nq, R), dtype=np.uint64)
    dists = np.empty((nq, R), dtype=np.float32)
    counts = np.empty(nq, dtype=np.uint32)
    aw, an = (None, 0) if allow is None else (np.ascontiguousarray(allow, dtype=np.uint64), len(allow))
    check(bq.lib.wvg_search_bq_candidates(bq.handle, fptr(q), nq, R, u64ptr(aw) if aw is not None else None, an,
                                          u64ptr(ids), fptr(dists), u32ptr(counts)))
    return ids, dists, counts


def search_bq_rescore(bq: Corpus, f32: Corpus, queries, k: int, rescore_limit: int, allow=None):
    q = np.ascontiguousarray(queries, dtype=np.float32)
    if q.ndim == 1:
        q = q[None, :]
    nq = q.shape[0]
    ids = np.empty((nq, k), dtype=np.uint64)
    dists = np.empty((nq, k), dtype=np.float32)
    counts = np.empty(nq, dtype=np.uint32)
    aw, an = (None, 0) if allow is None else (np.ascontiguousarray(allow, dtype=np.uint64), len(allow))
    check(bq.lib.wvg_search_bq_rescore(bq.handle, f32.handle, fptr(q), nq, k, rescore_limit,
                                       u64ptr(aw) if aw is not None else None, an,
                                       u64ptr(ids), fptr(dists), u32ptr(counts)))
    return ids, dists, counts


class Multi:
    """wvg_multi_open / wvg_multi_close: one context per device in this process
    and, for distinct devices, an RCCL communicator per device."""

    def __init__(self, devices, **options):
        self.lib = _lib.load()
        opts = _lib.Options()
        self.lib.wvg_options_default(byref(opts))
        for name, value in options.items():
            if name == "size" or name not in dict(_lib.Options._fields_):
                raise TypeError(f"unknown context option {name!r}")
            setattr(opts, name, int(value))
        devs = (c_int * len(devices))(*devices)
        h = c_void_p()
        check(self.lib.wvg_multi_open(devs, len(devices), byref(opts), byref(h)))
        self.handle = h
        nd, rc = c_int(), c_int()
        check(self.lib.wvg_multi_info(h, byref(nd), byref(rc)))
        self.ndev, self.uses_rccl = nd.value, bool(rc.value)

    def close(self) -> None:
        if self.handle:
            check(self.lib.wvg_multi_close(self.handle))
            self.handle = c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class MultiCorpus:
    """wvg_multi_corpus_*: docIDs dealt to the devices in contiguous slabs;
    search = every slab's scan on its device, one RCCL all-gather, the merge."""

    def __init__(self, multi: Multi, kind: int, metric: int, dim: int, rows: int):
        self.multi, self.lib = multi, multi.lib
        self.kind, self.metric, self.dim = kind, metric, dim
        h = c_void_p()
        check(self.lib.wvg_multi_corpus_create(multi.handle, kind, metric, dim, rows, byref(h)))
        self.handle = h

    def destroy(self) -> None:
        if self.handle:
            check(self.lib.wvg_multi_corpus_destroy(self.handle))
            self.handle = c_void_p()

    def shard(self, i: int):
        """(wvg_corpus handle, id_base, slab rows) of shard i."""
        h, base, slab = c_void_p(), c_uint64(), c_uint64()
        check(self.lib.wvg_multi_corpus_shard(self.handle, i, byref(h), byref(base), byref(slab)))
        return h, base.value, slab.value

    def upsert(self, ids, vectors) -> None:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        vectors = np.ascontiguousarray(vectors, dtype=np.float32).reshape(len(ids), -1)
        check(self.lib.wvg_multi_corpus_upsert(self.handle, u64ptr(ids), fptr(vectors), len(ids),
                                               vectors.shape[1] if vectors.size else self.dim))

    def delete(self, ids) -> None:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        check(self.lib.wvg_multi_corpus_delete(self.handle, u64ptr(ids), len(ids)))

    def fill_synthetic(self, seed: int, n: int, distribution: int = 0) -> None:
        check(self.lib.wvg_multi_corpus_fill_synthetic(self.handle, seed, n, distribution))

    def set_codebook(self, centers) -> None:
        centers = np.ascontiguousarray(centers, dtype=np.float32)
        m, ks, _ = centers.shape
        check(self.lib.wvg_multi_corpus_set_codebook(self.handle, fptr(centers), m, ks))

    def search(self, queries, k: int, allow=None):
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        ids = np.empty((nq, k), dtype=np.uint64)
        dists = np.empty((nq, k), dtype=np.float32)
        counts = np.empty(nq, dtype=np.uint32)
        aw, an = (None, 0) if allow is None else (np.ascontiguousarray(allow, dtype=np.uint64), len(allow))
        check(self.lib.wvg_multi_search(self.handle, fptr(q), nq, k, u64ptr(aw) if aw is not None else None, an,
                                        u64ptr(ids), fptr(dists), u32ptr(counts)))
        return ids, dists, counts
