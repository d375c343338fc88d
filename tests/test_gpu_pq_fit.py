"""GPU parity of PQ codebook training (KMeans.Fit on the device, wvg_pq_fit)
and the symmetric-distance table (buildGlobalDistances / SDC), against the
oracle's line-by-line restatement of CH/kmeans.go:146-250 with the same random
stream; plus the reference's own statistical pins (CH/kmeans_test.go:26-53
nearest property, CH/product_quantization_test.go:63-116 recall > 0.99)."""
import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd.compressionhelpers import ProductQuantizer

pytestmark = pytest.mark.gpu


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("n,d,m,ks,limit,seed", [
    (3000, 32, 8, 16, 0, 1),          # ds = 4 (unfused scalar l2), converges
    (5000, 64, 4, 256, 0, 2),         # ds = 16 (l2_256 8-blocks), empty-cluster reseeds likely
    (2000, 48, 2, 64, 1500, 3),       # training limit truncates; ds = 24
    (700, 16, 16, 255, 0, 4),         # ks near n: many empty clusters -> reseeds every pass
])
def test_pq_fit_bitexact(ctx, orc, n, d, m, ks, limit, seed):
    X = orc.synth_rows(400 + seed, 0, n, d, 0)
    want_c, want_it = orc.pq_fit(X, m, ks, limit, seed)
    pq = ProductQuantizer.fit(ctx, X, m, ks, training_limit=limit, seed=seed)
    assert np.array_equal(pq.fit_passes, want_it)
    assert np.array_equal(bits(pq.centers), bits(want_c))


def test_pq_fit_sift_like_ties(ctx, orc):
    """Integer rows: exact distance ties in nNearest (ties -> highest index)."""
    X = np.floor(orc.synth_rows(410, 0, 4000, 16, 1) / 32).astype(np.float32)
    want_c, want_it = orc.pq_fit(X, 4, 32, 0, 9)
    pq = ProductQuantizer.fit(ctx, X, 4, 32, training_limit=0, seed=9)
    assert np.array_equal(pq.fit_passes, want_it)
    assert np.array_equal(bits(pq.centers), bits(want_c))


def test_pq_fit_errors(ctx, orc):
    X = orc.synth_rows(420, 0, 100, 8, 0)
    with pytest.raises(_lib.WvgError, match="not enough data to fit kmeans"):
        ProductQuantizer.fit(ctx, X, 2, 256)
    with pytest.raises(_lib.WvgError, match="segments should be an integer divisor"):
        ProductQuantizer.fit(ctx, X, 3, 16)


def test_kmeans_nearest_property(ctx, orc):
    """CH/kmeans_test.go:26-53 on the device-trained centers."""
    X = np.array([[0, 5], [0.1, 4.9], [0.01, 5.1], [10.1, 7], [5.1, 2], [5.0, 2.1]], np.float32)
    pq = ProductQuantizer.fit(ctx, X, 1, 3, seed=5)
    want_c, _ = orc.pq_fit(X, 1, 3, 0, 5)
    assert np.array_equal(bits(pq.centers), bits(want_c))
    codes = pq.EncodeBatch(X)[:, 0]
    for v in range(len(X)):
        mn = orc.l2_256(X[v], pq.centers[0, codes[v]])
        for c in codes:
            assert orc.l2_256(X[v], pq.centers[0, c]) >= mn


def test_pq_recall_dot(ctx, orc):
    """CH/product_quantization_test.go:63-116: 1000 x 128, dot, 128 segments,
    255 centroids; recall@100 of the ADC ranking > 0.99."""
    n, d, nq, k = 1000, 128, 100, 100
    X = orc.synth_rows(430, 0, n, d, 0)
    Q = orc.synth_rows(431, 0, nq, d, 0)
    pq = ProductQuantizer.fit(ctx, X, d, 255, distance="dot", seed=11)
    codes = pq.EncodeBatch(X)
    rel = 0
    for q in Q:
        truth = set(np.argsort(orc.dist_all(1, q, X), kind="stable")[:k].tolist())
        adc = pq.NewDistancer(q).DistanceBatch(codes)
        res = np.argsort(adc, kind="stable")[:k]
        rel += len(truth & set(res.tolist()))
    assert rel / (k * nq) > 0.99


@pytest.mark.parametrize("metric_name,metric", [("l2-squared", 0), ("dot", 1)])
def test_sdc_table_and_distance(ctx, orc, metric_name, metric):
    m, ks, ds = 8, 256, 4
    centers = orc.synth_rows(440, 0, m * ks, ds, 0).reshape(m, ks, ds)
    pq = ProductQuantizer(ctx, centers, metric_name)
    tab = pq.globalDistances()
    assert np.array_equal(bits(tab), bits(orc.pq_global_distances(metric, centers)))
    X = orc.synth_rows(441, 0, 500, m * ds, 0)
    codes = pq.EncodeBatch(X)
    got = pq.SDCBatch(codes[0], codes)
    want = [orc.pq_sdc(metric, tab, codes[0], c) for c in codes]
    assert np.array_equal(bits(got), bits(want))
    assert pq.DistanceBetweenCompressedVectors(codes[1], codes[2])[0] == np.float32(want[0] * 0 + got[0] * 0 +
                                                                                       orc.pq_sdc(metric, tab,
                                                                                                  codes[1],
                                                                                                  codes[2]))
    assert pq.DistanceBetweenCompressedVectors(codes[1], codes[2][:3])[1] == "inconsistent compressed vectors lengths"
    # Decode: concatenated centroids (CH/product_quantization.go:428-434)
    assert np.array_equal(pq.Decode(codes[3]), np.concatenate([centers[i, codes[3][i]] for i in range(m)]))


def test_pq_codebook_commitlog_restore(ctx, orc):
    """Fit on the GPU -> ExposeFields -> AddPQ record (V/hnsw/condensor.go:266-285)
    -> ReadPQ (V/hnsw/deserializer.go:532-590) -> NewProductQuantizerWithEncoders:
    the restored quantizer encodes and scores bit-identically to the trained one."""
    from weaviate_amd.compressionhelpers import add_pq_record, read_pq_record

    X = orc.synth_rows(430, 0, 4000, 64, 0)
    pq = ProductQuantizer.fit(ctx, X, 16, 64, training_limit=0, seed=11)
    data, used = read_pq_record(add_pq_record(pq.ExposeFields()), 1)
    back = ProductQuantizer.from_pq_data(ctx, data)
    codes = pq.EncodeBatch(X[:1000])
    assert np.array_equal(back.EncodeBatch(X[:1000]), codes)
    assert np.array_equal(codes, orc.pq_encode(X[:1000], pq.centers))
    q = X[1234]
    assert np.array_equal(bits(back.NewDistancer(q).DistanceBatch(codes)), bits(pq.NewDistancer(q).DistanceBatch(codes)))
    assert np.array_equal(bits(back.SDCBatch(codes[0], codes)), bits(pq.SDCBatch(codes[0], codes)))
