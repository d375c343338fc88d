"""The compressor facade on the device (compressionhelpers.VectorCompressor,
CH/compression.go:37-200): Preload / Delete, DistanceToNode, DistanceToFloat,
NewDistancerFromID, the distance bag -- ports of the reference's
Test_NoRaceQuantizedDistanceBag (CH/compression_distance_bag_test.go:26-52)
and the BQ / PQ compressor distance checks, against the oracle."""
import numpy as np
import pytest

from weaviate_amd.compressionhelpers import BinaryQuantizer, ProductQuantizer, QuantizedVectorsCompressor
from weaviate_amd.distancer import CosineDistanceProvider, L2SquaredProvider

pytestmark = pytest.mark.gpu


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def test_quantized_distance_bag_known_answers(ctx):
    """CH/compression_distance_bag_test.go:26-52 (BQ compressor, cosine)."""
    comp = QuantizedVectorsCompressor(ctx, BinaryQuantizer(ctx, CosineDistanceProvider(ctx)), capacity=64, dims=2)
    comp.Preload(1, [-0.5, 0.5])
    comp.Preload(2, [0.25, 0.7])
    comp.Preload(3, [0.5, 0.5])
    bag = comp.NewBag()
    d, err = bag.Distance(1, 2)  # "returns error when id has not been loaded"
    assert err is not None
    bag = comp.NewBag()
    for i in (1, 2, 3):
        assert bag.Load(i) is None
    d, err = bag.Distance(1, 2)
    assert err is None and d == np.float32(1)
    d, err = bag.Distance(2, 3)
    assert err is None and d == np.float32(0)
    assert bag.Load(9) is not None  # never preloaded
    comp.Drop()


def test_bq_compressor_distances(ctx, orc):
    n, d = 3000, 200
    rows = orc.synth_rows(1301, 0, n, d, 0)
    q = orc.synth_rows(1302, 0, 1, d, 0)[0]
    comp = QuantizedVectorsCompressor(ctx, BinaryQuantizer(ctx, L2SquaredProvider(ctx)), capacity=n, dims=d)
    comp.PreloadBatch(np.arange(n, dtype=np.uint64), rows)
    comp.Delete(17)
    codes = np.stack([orc.bq_encode(r) for r in rows])
    dist, _ = comp.NewDistancer(q)
    qc = orc.bq_encode(q)
    want = orc.bq_dist_all(qc, codes)
    for i in (0, 5, 2999):
        dd, ok, err = dist.DistanceToNode(i)
        assert ok and err is None and dd == want[i]
    dd, ok, err = dist.DistanceToNode(17)
    assert not ok and err is not None
    ds, oks = dist.DistanceToNodes(np.arange(0, n, 7, dtype=np.uint64))
    live = np.arange(0, n, 7) != 17
    assert np.array_equal(oks, live) and np.array_equal(bits(ds[oks]), bits(want[np.arange(0, n, 7)][live]))
    # DistanceToFloat with a float query = the provider's exact distance
    dd, ok, _ = dist.DistanceToFloat(rows[3])
    assert ok and bits(dd) == bits(orc.dist_all(orc.L2, q, rows[3:4])[0])
    d12, err = comp.DistanceBetweenCompressedVectorsFromIDs(1, 2)
    assert err is None and d12 == orc.bq_dist_all(codes[1], codes[2:3])[0]
    dfi, err = comp.NewDistancerFromID(4)
    assert err is None and dfi.DistanceToNode(9)[0] == orc.bq_dist_all(codes[4], codes[9:10])[0]
    assert comp.NewDistancerFromID(17)[1] is not None
    comp.Drop()


def test_pq_compressor_distances(ctx, orc):
    n, d, m, ks = 4000, 64, 16, 64
    rows = orc.synth_rows(1311, 0, n, d, 0)
    q = orc.synth_rows(1312, 0, 1, d, 0)[0]
    pq = ProductQuantizer.fit(ctx, rows, segments=m, centroids=ks, seed=3)
    comp = QuantizedVectorsCompressor(ctx, pq, capacity=n)
    comp.PreloadBatch(np.arange(n, dtype=np.uint64), rows)
    codes = orc.pq_encode(rows, pq.centers)
    lut = orc.pq_lut(0, q, pq.centers)
    dist, ret = comp.NewDistancer(q)
    for i in (0, 1, 3999):
        dd, ok, err = dist.DistanceToNode(i)
        assert ok and bits(dd) == bits(orc.pq_adc(0, lut, codes[i]))
    ds, oks = dist.DistanceToNodes(np.arange(n, dtype=np.uint64))
    want = np.array([orc.pq_adc(0, lut, c) for c in codes], np.float32)
    assert oks.all() and np.array_equal(bits(ds), bits(want))
    ret()
    dd, ok, _ = dist.DistanceToFloat(rows[8])  # exact L2 to the query (the LUT's flatCenter)
    assert ok and bits(dd) == bits(orc.dist_all(orc.L2, q, rows[8:9])[0])
    tab = orc.pq_global_distances(0, pq.centers)
    d12, err = comp.DistanceBetweenCompressedVectorsFromIDs(1, 2)
    assert err is None and bits(d12) == bits(orc.pq_sdc(0, tab, codes[1], codes[2]))
    dfi, err = comp.NewDistancerFromID(5)
    assert err is None and bits(dfi.DistanceToNode(6)[0]) == bits(orc.pq_sdc(0, tab, codes[5], codes[6]))
    bag = comp.NewBag()
    bag.Load(1)
    bag.Load(2)
    assert bits(bag.Distance(1, 2)[0]) == bits(d12)
    comp.Drop()
