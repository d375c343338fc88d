"""Mirror of Weaviate's flat vector index (``db.VectorIndex`` implemented by
``*flat``) with its scans on the GPU.

Reference: adapters/repos/db/vector/flat/index.go
  Add :247, AddBatch :197, Delete :276, SearchByVector :307,
  searchByVector :319, searchByVectorBQ :347, searchTimeRescore :297,
  SearchByVectorDistance :531; interface adapters/repos/db/vector_index.go:24-45.

The device-resident corpus replaces the LSM "vectors" / "vectors_compressed"
buckets for scoring (the LSM stays the source of truth in Weaviate; here the
caller owns persistence).  Results are ascending by (distance, docID).
"""
from __future__ import annotations

import numpy as np

from ._lib import KIND_BQ, KIND_F32, METRIC_BY_NAME, WVG_ERR_DIM_MISMATCH, WvgError
from .device import Corpus, allow_bitmap, search_bq_rescore
from .distancer import provider_for

DEFAULT_SEARCH_BY_DIST_INITIAL_LIMIT = 100  # V/common/search_by_dist_params.go:17
DEFAULT_SEARCH_BY_DIST_LIMIT_MULTIPLIER = 10  # :23


class AllowList:
    """helpers.AllowList (adapters/repos/db/helpers/allow_list.go:19-40) over docIDs."""

    def __init__(self, *ids):
        self.ids = set(int(i) for i in ids)

    def Insert(self, *ids):
        self.ids.update(int(i) for i in ids)

    def Contains(self, i):
        return int(i) in self.ids

    def IsEmpty(self):
        return not self.ids

    def Len(self):
        return len(self.ids)

    def bitmap(self):
        return allow_bitmap(sorted(self.ids))


# ---------------------------------------------------------------------------
# The flat index's user config (entities/vectorindex/flat/config.go) and its
# update rules (V/flat/index.go:593-606, 738-791): what the index is built
# from and what a schema update may change (only the rescore limit).
# ---------------------------------------------------------------------------
DEFAULT_VECTOR_CACHE_MAX_OBJECTS = int(1e12)  # config.go:24
DEFAULT_COMPRESSION_RESCORE = -1  # config.go:26 ("let Weaviate pick")


class CompressionUserConfig:
    def __init__(self, Enabled: bool = False, RescoreLimit: int = DEFAULT_COMPRESSION_RESCORE, Cache: bool = False):
        self.Enabled, self.RescoreLimit, self.Cache = Enabled, RescoreLimit, Cache


class UserConfig:
    """flatent.UserConfig with SetDefaults (config.go:53-62)."""

    def __init__(self, Distance: str = "cosine", PQ: CompressionUserConfig | None = None,
                 BQ: CompressionUserConfig | None = None,
                 VectorCacheMaxObjects: int = DEFAULT_VECTOR_CACHE_MAX_OBJECTS):
        self.Distance = Distance
        self.VectorCacheMaxObjects = VectorCacheMaxObjects
        self.PQ = PQ if PQ is not None else CompressionUserConfig()
        self.BQ = BQ if BQ is not None else CompressionUserConfig()

    def IndexType(self) -> str:
        return "flat"

    def DistanceName(self) -> str:
        return self.Distance


def _opt_int(m, name, set_fn):  # entities/vectorindex/common OptionalIntFromMap: json numbers arrive as float
    v = m.get(name)
    if isinstance(v, float) or (isinstance(v, int) and not isinstance(v, bool)):
        set_fn(int(v))


def _opt_typed(m, name, typ, set_fn):  # OptionalBoolFromMap / OptionalStringFromMap: other types are ignored
    v = m.get(name)
    if isinstance(v, typ):
        set_fn(v)


def ParseAndValidateConfig(input_) -> UserConfig:
    """config.go:64-148 then validate (:150-166).  Raises ValueError with the
    reference's messages."""
    uc = UserConfig()
    if input_ is None:
        return uc
    if not isinstance(input_, dict):
        raise ValueError("input must be a non-nil map")
    _opt_typed(input_, "distance", str, lambda v: setattr(uc, "Distance", v))
    _opt_int(input_, "vectorCacheMaxObjects", lambda v: setattr(uc, "VectorCacheMaxObjects", v))
    for key, cfg in (("pq", uc.PQ), ("bq", uc.BQ)):
        sub = input_.get(key)
        if isinstance(sub, dict):
            _opt_typed(sub, "enabled", bool, lambda v, c=cfg: setattr(c, "Enabled", v))
            _opt_typed(sub, "cache", bool, lambda v, c=cfg: setattr(c, "Cache", v))
            _opt_int(sub, "rescoreLimit", lambda v, c=cfg: setattr(c, "RescoreLimit", v))
    if uc.PQ.Enabled:
        raise ValueError("PQ is not currently supported for flat indices")
    if (uc.PQ.Cache and not uc.PQ.Enabled) or (uc.BQ.Cache and not uc.BQ.Enabled):
        raise ValueError("not possible to use the cache without compression")
    return uc


def extract_compression(uc: UserConfig) -> str | None:
    """V/flat/index.go:110-124 (both enabled = none)."""
    if uc.BQ.Enabled and uc.PQ.Enabled:
        return None
    return "bq" if uc.BQ.Enabled else ("pq" if uc.PQ.Enabled else None)


def extract_compression_rescore(uc: UserConfig) -> int:
    """V/flat/index.go:126-136."""
    c = extract_compression(uc)
    return uc.PQ.RescoreLimit if c == "pq" else (uc.BQ.RescoreLimit if c == "bq" else 0)


def ValidateUserConfigUpdate(initial: UserConfig, updated: UserConfig) -> None:
    """V/flat/index.go:751-791: distance, pq.cache, pq and bq are immutable."""
    for name, get in (("distance", lambda c: c.Distance), ("pq.cache", lambda c: c.PQ.Cache),
                      ("pq", lambda c: c.PQ.Enabled), ("bq", lambda c: c.BQ.Enabled)):
        old, new = get(initial), get(updated)
        if old != new:
            fmt = lambda v: str(v).lower() if isinstance(v, bool) else str(v)  # Go's %v of a bool
            raise ValueError(f'{name} is immutable: attempted change from "{fmt(old)}" to "{fmt(new)}"')


class FlatIndex:
    @classmethod
    def from_user_config(cls, ctx, dims: int, uc: UserConfig, capacity: int = 1 << 16, id_base: int = 0):
        """flat.New (V/flat/index.go:67-97): compression and rescore from the
        user config; PQ searches uncompressed (:311-313), so it keeps no code
        corpus here."""
        comp = extract_compression(uc)
        return cls(ctx, dims, uc.Distance or "cosine", "bq" if comp == "bq" else None,
                   extract_compression_rescore(uc), capacity, id_base)

    def UpdateUserConfig(self, updated: UserConfig, callback=None) -> None:
        """V/flat/index.go:593-606: only the rescore limit takes effect."""
        self.rescore = extract_compression_rescore(updated)
        if callback is not None:
            callback()

    def __init__(self, ctx, dims: int, distance: str = "cosine", compression: str | None = None,
                 rescore_limit: int = -1, capacity: int = 1 << 16, id_base: int = 0):
        self.ctx = ctx
        self.dims = dims
        self.distance = distance
        self.provider = provider_for(ctx, distance)
        self.metric = METRIC_BY_NAME[distance]
        self.compression = compression
        self.rescore = rescore_limit
        self.vectors = Corpus(ctx, KIND_F32, self.metric, dims, capacity, id_base)
        self.bq = Corpus(ctx, KIND_BQ, self.metric, dims, capacity, id_base) if compression == "bq" else None

    # --- writes ------------------------------------------------------------
    def _grow(self, max_id: int):
        _, _, cap = self.vectors.info()
        if max_id - self.vectors.id_base >= cap:
            new_cap = max(cap * 2, max_id - self.vectors.id_base + 1)
            self.vectors.reserve(new_cap)
            if self.bq is not None:
                self.bq.reserve(new_cap)

    def Add(self, id_: int, vector) -> None:
        self.AddBatch([id_], [vector])

    def AddBatch(self, ids, vectors) -> None:
        ids = np.asarray(ids, dtype=np.uint64)
        if len(ids) == 0:
            raise ValueError("insertBatch called with empty lists")  # index.go:205-206
        vectors = np.asarray(vectors, dtype=np.float32)
        if vectors.ndim != 2 or vectors.shape[0] != len(ids):
            raise ValueError("ids and vectors sizes does not match")  # index.go:202-203
        if vectors.shape[1] != self.dims:
            raise WvgError(WVG_ERR_DIM_MISMATCH, "insert called with a vector of the wrong size")
        self._grow(int(ids.max()))
        self.vectors.upsert(ids, vectors)
        if self.bq is not None:
            self.bq.upsert(ids, vectors)

    def PostStartup(self, vectors_bucket=None, compressed_bucket=None) -> None:
        """index.go:640-681: rebuild the device corpora from the LSM buckets --
        iterables of (8-byte big-endian key, little-endian value bytes)."""
        for corpus, bucket in ((self.vectors, vectors_bucket), (self.bq, compressed_bucket)):
            if corpus is None or bucket is None:
                continue
            kv = list(bucket)
            if not kv:
                continue
            keys = np.frombuffer(b"".join(k for k, _ in kv), dtype=np.uint8)
            vals = np.frombuffer(b"".join(v for _, v in kv), dtype=np.uint8)
            corpus.load_kv(keys, vals)

    def Delete(self, *ids) -> None:
        ids = np.asarray(ids, dtype=np.uint64)
        self.vectors.delete(ids)
        if self.bq is not None:
            self.bq.delete(ids)

    # --- reads -------------------------------------------------------------
    def DistancerProvider(self):
        return self.provider

    def searchTimeRescore(self, k: int) -> int:
        return self.rescore if self.rescore > k else k

    def SearchByVector(self, vector, k: int, allow: AllowList | None = None):
        if k < 0:
            raise ValueError("k must be >= 0")
        bm = allow.bitmap() if allow is not None else None
        if allow is not None and allow.IsEmpty():
            return np.empty(0, dtype=np.uint64), np.empty(0, dtype=np.float32)
        if self.bq is not None:
            ids, dists, counts = search_bq_rescore(self.bq, self.vectors, vector, k, self.searchTimeRescore(k), bm)
        else:
            ids, dists, counts = self.vectors.search(vector, k, bm)
        n = int(counts[0])
        return ids[0, :n], dists[0, :n]

    def SearchByVectorDistance(self, vector, target: float, max_limit: int, allow: AllowList | None = None,
                               semantics: str = "flat"):
        """index.go:531-591.  semantics="flat" (default): the flat index's own
        result as the reference computes it -- its loop calls recursiveSearch
        once (the `for` has no post statement; later iterations only grow the
        limit until max_limit, and never end for max_limit < 0 when the first
        window is full), so it returns the rows of the first window of 100
        (V/common/search_by_dist_params.go:17) up to the first beyond the
        target: wvg_search_by_distance_window, one fused top-100 scan.  Where
        the reference would not terminate this returns that window.
        semantics="hnsw": the re-searching loop HNSW runs
        (V/hnsw/search.go:85-151; limits 100, 1100, 11100, ...), as one GPU
        pass (wvg_search_by_distance)."""
        if semantics not in ("flat", "hnsw"):
            raise ValueError(f"unknown semantics {semantics!r}")
        if allow is not None and allow.IsEmpty():
            return np.empty(0, dtype=np.uint64), np.empty(0, dtype=np.float32)
        bm = allow.bitmap() if allow is not None else None
        if semantics == "flat":
            if self.bq is None:
                return self.vectors.search_by_distance_window(vector, target, DEFAULT_SEARCH_BY_DIST_INITIAL_LIMIT, bm)
            ids, dist = self.SearchByVector(vector, DEFAULT_SEARCH_BY_DIST_INITIAL_LIMIT, allow)
            keep = 0
            while keep < len(ids) and (dist[keep] <= target or abs(float(dist[keep]) - float(target)) <= 1e-6):
                keep += 1
            return np.asarray(ids[:keep], dtype=np.uint64), np.asarray(dist[:keep], dtype=np.float32)
        if self.bq is None:
            return self.vectors.search_by_distance(vector, target, max_limit, bm)
        # BQ: every window is a BQ search with rescoring (index.go:539 -> searchByVectorBQ),
        # so the loop runs as written, each SearchByVector one GPU call (any k).
        offset, limit = 0, DEFAULT_SEARCH_BY_DIST_INITIAL_LIMIT
        total = offset + limit
        res_ids, res_d = [], []
        while True:
            ids, dist = self.SearchByVector(vector, total, allow)
            lo, hi = min(offset, len(ids)), min(total, len(ids))
            if lo == hi:
                break
            cont = bool(dist[hi - 1] <= target)
            for i in range(lo, hi):
                if dist[i] <= target or abs(float(dist[i]) - float(target)) <= 1e-6:
                    res_ids.append(int(ids[i]))
                    res_d.append(float(dist[i]))
                else:
                    break
            if not cont:
                break
            offset = total
            limit *= DEFAULT_SEARCH_BY_DIST_LIMIT_MULTIPLIER
            total = offset + limit
            if max_limit >= 0 and total > max_limit:
                break
        return np.asarray(res_ids, dtype=np.uint64), np.asarray(res_d, dtype=np.float32)
