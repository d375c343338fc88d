"""Mirror of Weaviate's ``distancer.Provider`` backed by the HIP library.

Reference: adapters/repos/db/vector/hnsw/distancer/provider.go:14-24
(``New``, ``SingleDist``, ``Step``, ``Wrap``, ``Type``) and the concrete
providers in l2.go, dot_product.go, cosine_dist.go, manhattan.go and
hamming.go.  Every distance is computed on the GPU in the reference's AVX2
reduction order (bit-identical results; manhattan is the pure-Go loop, hamming
counts with hamming_256's comparisons); ``BatchDist`` is the new bulk entry point (``distancer.BatchProvider``)
the flat / HNSW rescore loops use instead of one call per row.

Errors follow the Go convention: ``SingleDist`` returns ``(dist, ok, err)``
with ``err`` set (not raised) on a length mismatch.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import METRIC_COSINE, METRIC_DOT, METRIC_HAMMING, METRIC_L2, METRIC_MANHATTAN, check, fptr


class _Provider:
    metric = METRIC_L2
    type_name = ""

    def __init__(self, ctx):
        self.ctx = ctx

    def Type(self) -> str:
        return self.type_name

    def BatchDist(self, q, X) -> np.ndarray:
        """Provider.SingleDist(q, X[i]) for every row (distancer.BatchProvider)."""
        q = np.ascontiguousarray(q, dtype=np.float32)
        X = np.ascontiguousarray(X, dtype=np.float32)
        if X.ndim == 1:
            X = X[None, :]
        if X.shape[1] != q.shape[0]:
            raise _lib.WvgError(_lib.WVG_ERR_DIM_MISMATCH,
                                f"vector lengths don't match: {q.shape[0]} vs {X.shape[1]}")
        out = np.empty(X.shape[0], dtype=np.float32)
        check(self.ctx.lib.wvg_distance_batch(self.ctx.handle, self.metric, fptr(q), fptr(X), X.shape[0],
                                              q.shape[0], fptr(out)))
        return out

    def SingleDist(self, a, b):
        a = np.asarray(a, dtype=np.float32)
        b = np.asarray(b, dtype=np.float32)
        if a.shape[0] != b.shape[0]:
            # D/l2.go:47-50 (same text in dot_product.go / cosine_dist.go)
            return 0.0, False, f"vector lengths don't match: {a.shape[0]} vs {b.shape[0]}"
        return float(self.BatchDist(a, b[None, :])[0]), True, None

    def New(self, a):
        return _Distancer(self, np.asarray(a, dtype=np.float32))

    def Step(self, a, b) -> float:
        """Un-wrapped partial sum in the pure-Go order (l2.go:79-88, dot_product.go:87-94,
        manhattan.go:68-78, hamming.go:76-86):
        a one-segment, one-centroid PQ lookup table is exactly Step(a, b)."""
        a = np.ascontiguousarray(a, dtype=np.float32)
        b = np.ascontiguousarray(b, dtype=np.float32).reshape(1, 1, -1)
        out = np.empty(1, dtype=np.float32)
        check(self.ctx.lib.wvg_pq_lut(self.ctx.handle, self.metric, fptr(b), 1, 1, a.shape[0], fptr(a), fptr(out)))
        return float(out[0])

    def Wrap(self, x: float) -> float:
        raise NotImplementedError


class _Distancer:
    def __init__(self, provider, a):
        self.p, self.a = provider, a

    def Distance(self, b):
        return self.p.SingleDist(self.a, b)


class L2SquaredProvider(_Provider):
    metric, type_name = METRIC_L2, "l2-squared"

    def Wrap(self, x):  # l2.go:90-92
        return np.float32(x)


class DotProductProvider(_Provider):
    metric, type_name = METRIC_DOT, "dot"

    def Wrap(self, x):  # dot_product.go:96-98
        return -np.float32(x)


class CosineDistanceProvider(_Provider):
    metric, type_name = METRIC_COSINE, "cosine-dot"

    def Wrap(self, x):  # cosine_dist.go:66-68
        return np.float32(1.0) - np.float32(x)


class ManhattanProvider(_Provider):
    metric, type_name = METRIC_MANHATTAN, "manhattan"

    def Wrap(self, x):  # manhattan.go:80-82
        return np.float32(x)


class HammingProvider(_Provider):
    metric, type_name = METRIC_HAMMING, "hamming"

    def Wrap(self, x):  # hamming.go:88-90
        return np.float32(x)


_BY_NAME = {"l2-squared": L2SquaredProvider, "dot": DotProductProvider, "cosine": CosineDistanceProvider,
            "cosine-dot": CosineDistanceProvider, "manhattan": ManhattanProvider, "hamming": HammingProvider}


def provider_for(ctx, name: str) -> _Provider:
    """Shard.initVectorIndex picks the provider by distance name (adapters/repos/db/shard.go:406-421);
    "" means cosine there."""
    if name == "":
        name = "cosine"
    if name not in _BY_NAME:
        raise ValueError(f'unrecognized distance metric "{name}",choose one of ["cosine", "dot", "l2-squared", '
                         f'"manhattan","hamming"]')
    return _BY_NAME[name](ctx)


def Normalize(ctx, v) -> np.ndarray:
    """distancer.Normalize (normalize.go:16-32) on the GPU; accepts one row or a matrix."""
    X = np.ascontiguousarray(v, dtype=np.float32)
    one = X.ndim == 1
    if one:
        X = X[None, :]
    out = np.empty_like(X)
    check(ctx.lib.wvg_normalize_batch(ctx.handle, fptr(X), X.shape[0], X.shape[1], fptr(out)))
    return out[0] if one else out
