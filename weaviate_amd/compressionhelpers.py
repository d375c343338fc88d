"""Mirror of Weaviate's ``compressionhelpers`` BQ / PQ quantizers on the GPU.

Reference:
  BinaryQuantizer      adapters/repos/db/vector/compressionhelpers/binary_quantization.go:24-56
  ProductQuantizer     .../compressionhelpers/product_quantization.go:155-442
  KMeans.Encode        .../compressionhelpers/kmeans.go:103-135
  quantizer[T]         .../compressionhelpers/quantizer.go:21-31

``ProductQuantizer`` is built from trained centers ([m][ks][ds] float32, the
layout of KMeans.ExposeDataForRestore, kmeans.go:85-93) or trained on the GPU
with :meth:`ProductQuantizer.fit` (KMeans.Fit per segment, kmeans.go:220-250).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import METRIC_BY_NAME, check, fptr, u8ptr, u32ptr, u64ptr

DEFAULT_TRAINING_LIMIT = 100_000  # DefaultPQTrainingLimit (entities/vectorindex/hnsw/pq_config.go)


class BinaryQuantizer:
    def __init__(self, ctx, distancer=None):
        self.ctx = ctx
        self.distancer = distancer

    def Encode(self, vec) -> np.ndarray:
        return self.EncodeBatch(np.asarray(vec, dtype=np.float32)[None, :])[0]

    def EncodeBatch(self, X) -> np.ndarray:
        X = np.ascontiguousarray(X, dtype=np.float32)
        out = np.empty((X.shape[0], (X.shape[1] + 63) // 64), dtype=np.uint64)
        check(self.ctx.lib.wvg_bq_encode(self.ctx.handle, fptr(X), X.shape[0], X.shape[1], u64ptr(out)))
        return out

    def DistanceBetweenCompressedVectors(self, x, y):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        y = np.ascontiguousarray(y, dtype=np.uint64)
        if x.shape[0] != y.shape[0]:
            return 0.0, "BinaryQuantizer.DistanceBetweenCompressedVectors: Both vectors should have the same len"
        return float(self.DistanceBatch(x, y[None, :])[0]), None

    def DistanceBatch(self, q, codes) -> np.ndarray:
        q = np.ascontiguousarray(q, dtype=np.uint64)
        codes = np.ascontiguousarray(codes, dtype=np.uint64)
        out = np.empty(codes.shape[0], dtype=np.float32)
        check(self.ctx.lib.wvg_bq_distance_batch(self.ctx.handle, u64ptr(q), u64ptr(codes), codes.shape[0],
                                                 q.shape[0], fptr(out)))
        return out

    def DistanceBetweenCompressedAndUncompressedVectors(self, x, y):
        """CH/quantizer.go:65-68: Encode(x), then the Hamming distance to y."""
        return self.DistanceBetweenCompressedVectors(self.Encode(x), y)

    def NewDistancer(self, a) -> "BQDistancer":
        """CH/quantizer.go:89-95."""
        a = np.asarray(a, dtype=np.float32)
        return BQDistancer(self, a, self.Encode(a))

    def NewCompressedQuantizerDistancer(self, code) -> "BQDistancer":
        """CH/quantizer.go:97-103."""
        return BQDistancer(self, None, np.asarray(code, dtype=np.uint64))


class BQDistancer:
    """CH/quantizer.go:83-117: Distance(code) = Hamming to the compressed
    query; DistanceToFloat(x) = the provider's exact SingleDist to the float
    query when there is one, else the Hamming distance to Encode(x)."""

    def __init__(self, bq, x, compressed):
        self.bq, self.x, self.compressed = bq, x, compressed

    def Distance(self, code):
        d, err = self.bq.DistanceBetweenCompressedVectors(self.compressed, code)
        return d, err is None, err

    def DistanceToFloat(self, x):
        if self.x is not None and len(self.x) > 0:
            return self.bq.distancer.SingleDist(self.x, x)
        d, err = self.bq.DistanceBetweenCompressedVectors(self.compressed, self.bq.Encode(x))
        return d, err is None, err


class ProductQuantizer:
    """k-means PQ with given centers [m][ks][ds]."""

    def __init__(self, ctx, centers, distance: str = "l2-squared"):
        self.ctx = ctx
        self.centers = np.ascontiguousarray(centers, dtype=np.float32)
        self.m, self.ks, self.ds = self.centers.shape
        self.dimensions = self.m * self.ds
        self.metric = METRIC_BY_NAME[distance]
        self.encoder_distribution = LOG_NORMAL_DISTRIBUTION  # DefaultPQEncoderDistribution (pq_config.go:32)
        self.fit_passes = None
        self._global = None

    @classmethod
    def fit(cls, ctx, data, segments: int, centroids: int = 256, distance: str = "l2-squared",
            training_limit: int = DEFAULT_TRAINING_LIMIT, seed: int = 0, encoder: str = "kmeans",
            distribution: str = "log-normal"):
        """NewProductQuantizer + Fit (CH/product_quantization.go:155-229, :372-418)
        with the k-means encoder, trained on the GPU (wvg_pq_fit)."""
        X = np.ascontiguousarray(data, dtype=np.float32)
        n, d = X.shape
        enc, dist = validate_pq_config(segments, centroids, d, encoder, distribution)
        if enc != USE_KMEANS_ENCODER:
            raise ValueError("tile encoder is out of scope: only the k-means encoder runs on the GPU")
        centers = np.empty((segments, centroids, d // segments if segments else 0), dtype=np.float32)
        passes = np.zeros(segments, dtype=np.uint32)
        check(ctx.lib.wvg_pq_fit(ctx.handle, fptr(X), n, d, segments, centroids, training_limit, seed,
                                 fptr(centers), u32ptr(passes)))
        pq = cls(ctx, centers, distance)
        pq.encoder_distribution = dist
        pq.fit_passes = passes
        return pq

    def globalDistances(self) -> np.ndarray:
        """buildGlobalDistances (CH/product_quantization.go:236-251), [m][ks][ks]."""
        if self._global is None:
            out = np.empty((self.m, self.ks, self.ks), dtype=np.float32)
            check(self.ctx.lib.wvg_pq_global_distances(self.ctx.handle, self.metric, fptr(self.centers), self.m,
                                                       self.ks, self.dimensions, fptr(out)))
            self._global = out
        return self._global

    def DistanceBetweenCompressedVectors(self, x, y):
        """:297-311 -- (distance, error)."""
        x = np.asarray(x, dtype=np.uint8)
        y = np.asarray(y, dtype=np.uint8)
        if x.shape[0] != self.m or y.shape[0] != self.m:
            return 0.0, "inconsistent compressed vectors lengths"
        return float(self.SDCBatch(x, y[None, :])[0]), None

    def SDCBatch(self, x, codes) -> np.ndarray:
        tab = self.globalDistances()
        x = np.ascontiguousarray(x, dtype=np.uint8)
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        out = np.empty(codes.shape[0], dtype=np.float32)
        check(self.ctx.lib.wvg_pq_sdc_batch(self.ctx.handle, self.metric, fptr(tab), self.m, self.ks, u8ptr(x),
                                            u8ptr(codes), codes.shape[0], fptr(out)))
        return out

    def DistanceBetweenCompressedAndUncompressedVectors(self, x, code):
        """:313-320: sum of Step(x_i, centroid_i[code_i]) in segment order == the
        ADC lookup of the same code (the LUT holds those Step values)."""
        return self.NewDistancer(x).Distance(code)[0], None

    def Decode(self, code) -> np.ndarray:
        """:428-434: concatenated centroids."""
        code = np.asarray(code, dtype=np.uint8)
        return np.concatenate([self.centers[i, code[i]] for i in range(self.m)])

    def Encode(self, vec) -> np.ndarray:
        return self.EncodeBatch(np.asarray(vec, dtype=np.float32)[None, :])[0]

    def EncodeBatch(self, X) -> np.ndarray:
        X = np.ascontiguousarray(X, dtype=np.float32)
        out = np.empty((X.shape[0], self.m), dtype=np.uint8)
        check(self.ctx.lib.wvg_pq_encode(self.ctx.handle, fptr(self.centers), self.m, self.ks, fptr(X), X.shape[0],
                                         X.shape[1], u8ptr(out)))
        return out

    def CenterAt(self, q) -> np.ndarray:
        """DistanceLookUpTable for q, fully materialized ([m][ks])."""
        q = np.ascontiguousarray(q, dtype=np.float32)
        out = np.empty((self.m, self.ks), dtype=np.float32)
        check(self.ctx.lib.wvg_pq_lut(self.ctx.handle, self.metric, fptr(self.centers), self.m, self.ks,
                                      self.dimensions, fptr(q), fptr(out)))
        return out

    def NewDistancer(self, q):
        return PQDistancer(self, np.asarray(q, dtype=np.float32), self.CenterAt(q))

    def NewCompressedQuantizerDistancer(self, code):
        """:339-346: no LUT; distances are SDC lookups against this code."""
        return PQDistancer(self, None, None, np.asarray(code, dtype=np.uint8))

    def ExposeFields(self) -> "PQData":
        """:285-295 -- the fields the HNSW commit log persists (compress.go:89)."""
        return PQData(Ks=self.ks, M=self.m, Dimensions=self.dimensions, EncoderType=USE_KMEANS_ENCODER,
                      EncoderDistribution=self.encoder_distribution, Centers=self.centers.copy())

    @classmethod
    def from_pq_data(cls, ctx, data: "PQData", distance: str = "l2-squared"):
        """NewProductQuantizerWithEncoders (:224-234) from a restored AddPQ record."""
        if data.EncoderType != USE_KMEANS_ENCODER:
            raise ValueError("tile encoder is out of scope: only the k-means encoder runs on the GPU")
        pq = cls(ctx, data.Centers, distance)
        pq.encoder_distribution = data.EncoderDistribution
        return pq


NORMAL_DISTRIBUTION, LOG_NORMAL_DISTRIBUTION = 0, 1  # CH/tile_encoder.go:89-90


def validate_pq_config(segments: int, centroids: int, dimensions: int, encoder: str = "kmeans",
                       distribution: str = "log-normal"):
    """The checks of NewProductQuantizer (CH/product_quantization.go:190-207),
    in the same order and with the same messages; parseEncoder /
    parseEncoderDistribution (:257-277; names from entities/vectorindex/hnsw/
    pq_config.go:21-24).  Returns (encoder type, distribution byte);
    raises WvgError(WVG_ERR_INVALID), as the C ABI does for the same checks."""
    if segments <= 0:
        raise _lib.WvgError(_lib.WVG_ERR_INVALID, "segments cannot be 0 nor negative")
    if centroids > 256:
        raise _lib.WvgError(_lib.WVG_ERR_INVALID, f"centroids should not be higher than 256. Attempting to use {centroids}")
    if dimensions % segments != 0:
        raise _lib.WvgError(_lib.WVG_ERR_INVALID, "segments should be an integer divisor of dimensions")
    enc = {"tile": USE_TILE_ENCODER, "kmeans": USE_KMEANS_ENCODER}.get(encoder)
    if enc is None:
        raise _lib.WvgError(_lib.WVG_ERR_INVALID, "invalid encoder type")
    dist = {"log-normal": LOG_NORMAL_DISTRIBUTION, "normal": NORMAL_DISTRIBUTION}.get(distribution)
    if dist is None:
        raise _lib.WvgError(_lib.WVG_ERR_INVALID, "invalid encoder distribution")
    # the reference accepts centroids <= 0 here and fails later; the device
    # path refuses it up front with the C ABI's message (pq_validate)
    if centroids <= 0:
        raise _lib.WvgError(_lib.WVG_ERR_INVALID, "centroids must be > 0")
    return enc, dist


# --- codebook persistence: the HNSW commit log's AddPQ record ------------------
# Writer: MemoryCondensor.AddPQ (V/hnsw/condensor.go:266-285).  Reader: the
# AddPQ case of Deserializer.Do (V/hnsw/deserializer.go:143-145) -> ReadPQ
# (:532-590) -> ReadKMeansEncoder (:509-530).  All integers little-endian; each
# k-means encoder's payload is KMeans.ExposeDataForRestore (CH/kmeans.go:85-93):
# ks*ds float32 LE, centroid-major.

ADD_PQ = 11  # HnswCommitType AddPQ (V/hnsw/commit_logger.go:266-280: iota, 12th value)
USE_TILE_ENCODER = 0  # CH/product_quantization.go:28-31
USE_KMEANS_ENCODER = 1


class PQData:
    """compressionhelpers.PQData (CH/product_quantization.go:170-179), with the
    k-means encoders held as one [m][ks][ds] float32 array."""

    def __init__(self, Ks, M, Dimensions, EncoderType=USE_KMEANS_ENCODER, EncoderDistribution=0,
                 UseBitsEncoding=False, Centers=None):
        self.Ks, self.M, self.Dimensions = int(Ks), int(M), int(Dimensions)
        self.EncoderType, self.EncoderDistribution = int(EncoderType), int(EncoderDistribution)
        self.UseBitsEncoding = bool(UseBitsEncoding)
        self.Centers = None if Centers is None else np.ascontiguousarray(Centers, dtype=np.float32)

    def __eq__(self, other):
        return (isinstance(other, PQData)
                and (self.Ks, self.M, self.Dimensions, self.EncoderType, self.EncoderDistribution,
                     self.UseBitsEncoding) == (other.Ks, other.M, other.Dimensions, other.EncoderType,
                                               other.EncoderDistribution, other.UseBitsEncoding)
                and self.Centers.shape == other.Centers.shape
                and np.array_equal(self.Centers.view(np.uint32), other.Centers.view(np.uint32)))


def add_pq_record(data: PQData) -> bytes:
    """MemoryCondensor.AddPQ: the full record, commit-type byte included."""
    if data.EncoderType != USE_KMEANS_ENCODER:
        raise ValueError("tile encoder is out of scope: only k-means codebooks are written")
    ds = data.Dimensions // data.M if data.M else 0
    c = np.ascontiguousarray(data.Centers, dtype="<f4")
    if c.shape != (data.M, data.Ks, ds):
        raise ValueError(f"centers shape {c.shape} != (m, ks, ds) = {(data.M, data.Ks, ds)}")
    head = np.zeros(10, np.uint8)
    head[0] = ADD_PQ
    head[1:3] = np.frombuffer(np.uint16(data.Dimensions).astype("<u2").tobytes(), np.uint8)
    head[3] = data.EncoderType
    head[4:6] = np.frombuffer(np.uint16(data.Ks).astype("<u2").tobytes(), np.uint8)
    head[6:8] = np.frombuffer(np.uint16(data.M).astype("<u2").tobytes(), np.uint8)
    head[8] = data.EncoderDistribution
    head[9] = 1 if data.UseBitsEncoding else 0
    return head.tobytes() + c.tobytes()


def read_pq_record(buf, offset: int = 0):
    """Deserializer.ReadPQ on `buf` starting after the commit-type byte.
    Returns (PQData, bytes consumed); raises ValueError with the reference's
    messages on a short read or an unknown encoder type."""
    mv = memoryview(bytes(buf))[offset:]
    if len(mv) < 9:
        what = "uint16" if len(mv) < 2 or 3 <= len(mv) < 7 else "byte"
        raise ValueError(f"failed to read {what}")
    dims, enc = int.from_bytes(mv[0:2], "little"), mv[2]
    ks, m = int.from_bytes(mv[3:5], "little"), int.from_bytes(mv[5:7], "little")
    dist, bits = mv[7], mv[8]
    if enc == USE_TILE_ENCODER:
        raise ValueError("tile encoder is out of scope: only k-means codebooks are restored")
    if enc != USE_KMEANS_ENCODER:
        raise ValueError("Unsuported encoder type")  # sic, deserializer.go:574
    ds = dims // m if m else 0
    need = 4 * m * ks * ds
    if len(mv) - 9 < need:
        raise ValueError("failed to read float32")
    centers = np.frombuffer(mv[9:9 + need], dtype="<f4").astype(np.float32).reshape(m, ks, ds)
    return PQData(ks, m, dims, enc, dist, bits != 0, centers), 9 + need


class PQDistancer:
    """CH/product_quantization.go:352-370.  From a float query: ADC through its
    LUT; from a code (NewCompressedQuantizerDistancer): SDC."""

    def __init__(self, pq, x, lut, compressed=None):
        self.pq, self.x, self.lut, self.compressed = pq, x, lut, compressed

    def Distance(self, code):
        code = np.asarray(code, dtype=np.uint8)
        if self.lut is None:
            d, err = self.pq.DistanceBetweenCompressedVectors(self.compressed, code)
            return d, err is None, err
        if code.shape[0] != self.pq.m:
            return 0.0, False, "inconsistent compressed vector length"  # product_quantization.go:357-358
        return float(self.DistanceBatch(code[None, :])[0]), True, None

    def DistanceToFloat(self, x):
        """:363-370: the exact distance to the query (the LUT's flatCenter), or SDC to Encode(x)."""
        if self.lut is not None:
            from .distancer import provider_for

            return provider_for(self.pq.ctx, _DIST_NAME[self.pq.metric]).SingleDist(x, self.x)
        d, err = self.pq.DistanceBetweenCompressedVectors(self.compressed, self.pq.Encode(x))
        return d, err is None, err

    def DistanceBatch(self, codes) -> np.ndarray:
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        out = np.empty(codes.shape[0], dtype=np.float32)
        check(self.pq.ctx.lib.wvg_pq_adc_batch(self.pq.ctx.handle, self.pq.metric, fptr(self.lut), self.pq.m,
                                               self.pq.ks, u8ptr(codes), codes.shape[0], fptr(out)))
        return out


_DIST_NAME = {_lib.METRIC_L2: "l2-squared", _lib.METRIC_DOT: "dot", _lib.METRIC_COSINE: "cosine-dot",
              _lib.METRIC_MANHATTAN: "manhattan", _lib.METRIC_HAMMING: "hamming"}


class QuantizedVectorsCompressor:
    """compressionhelpers.VectorCompressor (CH/compression.go:37-54, 56-200) with
    the compressed-vector cache held on the device: one BQ or PQ corpus of codes
    keyed by docID.  Preload encodes exactly as the reference does (the vector
    as given -- callers normalize for cosine -- through the quantizer's Encode,
    :87-94) and stores the code; Delete clears it.  Distances go through the
    quantizer's distancers, so they are the reference's bits."""

    def __init__(self, ctx, quantizer, capacity: int, dims: int | None = None):
        from ._lib import KIND_BQ, KIND_PQ
        from .device import Corpus

        self.ctx, self.quantizer = ctx, quantizer
        if isinstance(quantizer, BinaryQuantizer):
            metric = quantizer.distancer.metric if quantizer.distancer is not None else _lib.METRIC_L2
            self.kind, self.dims = KIND_BQ, int(dims)
            self.corpus = Corpus(ctx, KIND_BQ, metric, self.dims, capacity)
        else:
            self.kind, self.dims = KIND_PQ, quantizer.dimensions
            self.corpus = Corpus(ctx, KIND_PQ, quantizer.metric, self.dims, capacity)
            self.corpus.set_codebook(quantizer.centers)

    def Drop(self) -> None:
        self.corpus.destroy()

    def Preload(self, id_: int, vector) -> None:
        self.PreloadBatch(np.array([id_], np.uint64), np.asarray(vector, np.float32)[None, :])

    def PreloadBatch(self, ids, vectors) -> None:
        """Preload of many ids at once (the bulk path of V/hnsw/compress.go:98-104)."""
        codes = self.quantizer.EncodeBatch(np.ascontiguousarray(vectors, np.float32))
        self.corpus.upsert_codes(np.ascontiguousarray(ids, np.uint64), codes)

    def Delete(self, id_: int) -> None:
        self.corpus.delete(np.array([id_], np.uint64))

    def _codes(self, ids):
        m = self.quantizer.m if self.kind == _lib.KIND_PQ else 0
        return self.corpus.get_batch(np.ascontiguousarray(ids, np.uint64), pq_m=m)

    def compressedVectorFromID(self, id_: int):
        """:107-116: (code, error) -- an id never preloaded (or deleted) is an error."""
        codes, ok = self._codes([id_])
        if not ok[0]:
            return None, f"got a nil or zero-length vector at docID {id_}"
        return codes[0], None

    def DistanceBetweenCompressedVectorsFromIDs(self, x: int, y: int):
        """:118-131."""
        cx, err = self.compressedVectorFromID(x)
        if err:
            return 0.0, err
        cy, err = self.compressedVectorFromID(y)
        if err:
            return 0.0, err
        return self.quantizer.DistanceBetweenCompressedVectors(cx, cy)

    def DistanceBetweenCompressedAndUncompressedVectorsFromID(self, id_: int, vector):
        """:133-140."""
        c, err = self.compressedVectorFromID(id_)
        if err:
            return 0.0, err
        return self.quantizer.DistanceBetweenCompressedAndUncompressedVectors(np.asarray(vector, np.float32), c)

    def NewDistancer(self, vector):
        """:158-166: (CompressorDistancer, return function)."""
        return CompressorDistancer(self, self.quantizer.NewDistancer(vector)), (lambda: None)

    def NewDistancerFromID(self, id_: int):
        """:168-183: (CompressorDistancer, error)."""
        c, err = self.compressedVectorFromID(id_)
        if err:
            return None, err
        return CompressorDistancer(self, self.quantizer.NewCompressedQuantizerDistancer(c)), None

    def NewBag(self) -> "QuantizedDistanceBag":
        """:194-199."""
        return QuantizedDistanceBag(self)

    def ExposeFields(self):
        return self.quantizer.ExposeFields() if self.kind == _lib.KIND_PQ else PQData(0, 0, 0)


class CompressorDistancer:
    """quantizedCompressorDistancer (CH/compression.go:306-325): DistanceToNode
    reads the node's code from the device corpus; DistanceToNodes does a whole
    candidate list with one gather (the HNSW rescore batch)."""

    def __init__(self, compressor, distancer):
        self.c, self.d = compressor, distancer

    def DistanceToNode(self, id_: int):
        code, err = self.c.compressedVectorFromID(id_)
        if err:
            return 0.0, False, err
        return self.d.Distance(code)

    def DistanceToNodes(self, ids):
        """(dists, ok) for many nodes: one code gather, one batched distance."""
        codes, ok = self.c._codes(ids)
        out = np.zeros(len(ok), np.float32)
        if ok.any():
            live = codes[ok]
            if isinstance(self.d, PQDistancer) and self.d.lut is not None:
                out[ok] = self.d.DistanceBatch(live)
            elif isinstance(self.d, BQDistancer):
                out[ok] = self.c.quantizer.DistanceBatch(self.d.compressed, live)
            else:
                out[ok] = [self.d.Distance(cd)[0] for cd in live]
        return out, ok

    def DistanceToFloat(self, vector):
        return self.d.DistanceToFloat(np.asarray(vector, np.float32))


class QuantizedDistanceBag:
    """CompressionDistanceBag (CH/compression_distance_bag.go:19-45)."""

    def __init__(self, compressor):
        self.c = compressor
        self.elements = {}

    def Load(self, id_: int):
        code, err = self.c.compressedVectorFromID(id_)
        if err:
            return err
        self.elements[id_] = code
        return None

    def Distance(self, x: int, y: int):
        if x not in self.elements:
            return 0.0, f"missing id in bag: {x}"
        if y not in self.elements:
            return 0.0, f"missing id in bag: {y}"
        return self.c.quantizer.DistanceBetweenCompressedVectors(self.elements[x], self.elements[y])
