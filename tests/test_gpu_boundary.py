"""GPU tests of the remaining drop-in entry points: the LSM bulk load
(PostStartup, V/flat/index.go:640-681; keys big-endian, values little-endian
as index.go:218-245 writes them) and the batched DistanceToNode by docID
(CH/compression.go:306-325; HNSW rescore, V/hnsw/search.go:564-581)."""
import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_BQ, KIND_F32, KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2
from weaviate_amd.device import Corpus

pytestmark = pytest.mark.gpu

ORC_METRIC = {METRIC_L2: 0, METRIC_DOT: 1, METRIC_COSINE: 2}


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def be_keys(ids):
    return np.asarray(ids, dtype=">u8").view(np.uint8)


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_COSINE])
def test_post_startup_from_buckets(ctx, orc, metric):
    from weaviate_amd.flat import FlatIndex

    n, d = 2500, 96
    rows = orc.synth_rows(501, 0, n, d, 0)
    q = orc.synth_rows(502, 0, 1, d, 0)[0]
    name = {METRIC_L2: "l2-squared", METRIC_COSINE: "cosine"}[metric]
    live = FlatIndex(ctx, d, name, compression="bq", rescore_limit=100, capacity=64)
    live.AddBatch(np.arange(n), rows)
    live.Delete(5, 17)
    # what the buckets hold: normalized float rows (index.go:258-260) and BQ words (:262-270)
    stored = orc.normalize_rows(rows) if metric == METRIC_COSINE else rows
    keep = [i for i in range(n) if i not in (5, 17)]
    order = np.random.default_rng(0).permutation(keep)  # cursor order is key order; any order must work
    vec_bucket = [(int(i).to_bytes(8, "big"), stored[i].astype("<f4").tobytes()) for i in order]
    bq_bucket = [(int(i).to_bytes(8, "big"), orc.bq_encode(stored[i]).astype("<u8").tobytes()) for i in order]
    restarted = FlatIndex(ctx, d, name, compression="bq", rescore_limit=100, capacity=64)
    restarted.PostStartup(vec_bucket, bq_bucket)
    for k in [10, 100]:
        a_ids, a_d = live.SearchByVector(q, k)
        b_ids, b_d = restarted.SearchByVector(q, k)
        assert np.array_equal(a_ids, b_ids) and np.array_equal(bits(a_d), bits(b_d))
    assert np.array_equal(restarted.vectors.get(3), stored[3])


def test_load_kv_errors_and_growth(ctx, orc):
    c = Corpus(ctx, KIND_F32, METRIC_L2, 8, 64)
    rows = orc.synth_rows(511, 0, 3, 8, 0)
    c.load_kv(be_keys([1000, 7, 64]), rows.view(np.uint8))
    _, hw, cap = c.info()
    assert cap >= 1001 and hw == 1001
    assert np.array_equal(c.get(1000), rows[0]) and np.array_equal(c.get(64), rows[2])
    with pytest.raises(_lib.WvgError, match="vector lengths don't match"):
        c.load_kv(be_keys([1]), np.zeros((1, 12), np.uint8))


@pytest.mark.parametrize("kind", [KIND_F32, KIND_BQ, KIND_PQ])
def test_distance_by_ids(ctx, orc, kind):
    n, d, m, ks = 3000, 64, 16, 256
    rows = orc.synth_rows(521, 0, n, d, 0)
    q = orc.synth_rows(522, 0, 1, d, 0)[0]
    metric = METRIC_DOT if kind == KIND_PQ else METRIC_L2
    base = 128
    c = Corpus(ctx, kind, metric, d, n, id_base=base)
    centers = None
    if kind == KIND_PQ:
        centers = orc.synth_rows(523, 0, m * ks, d // m, 0).reshape(m, ks, d // m)
        c.set_codebook(centers)
    c.upsert(np.arange(base, base + n, dtype=np.uint64), rows)
    c.delete(np.array([base + 10], np.uint64))
    ids = np.array([base + 10, base + 11, base + 2999, base, 5, base + n + 7, base + 1234], np.uint64)
    dists, ok = c.distance_by_ids(q, ids)
    assert ok.tolist() == [False, True, True, True, False, False, True]
    sl = (ids[ok] - base).astype(np.int64)
    if kind == KIND_F32:
        want = orc.dist_all(0, q, rows)[sl]
    elif kind == KIND_BQ:
        codes = np.stack([orc.bq_encode(r) for r in rows])
        want = orc.bq_dist_all(orc.bq_encode(q), codes)[sl]
    else:
        codes = orc.pq_encode(rows, centers)
        lut = orc.pq_lut(1, q, centers)
        want = np.array([orc.pq_adc(1, lut, codes[i]) for i in sl], np.float32)
    assert np.array_equal(bits(dists[ok]), bits(want))
    assert np.all(dists[~ok] == 0)
