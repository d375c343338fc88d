"""GPU parity of the HNSW / index-queue brute-force consumers (SURVEY.md §8f
row 1): hnsw.flatSearch over small allow lists (V/hnsw/flat_search.go:19-79),
the HNSW rescore loop (V/hnsw/search.go:564-597) and IndexQueue.bruteForce
(adapters/repos/db/index_queue.go:676-719).  Distances bit-exact against the
oracle; ids exact under the (distance, docID) rule."""
import numpy as np
import pytest

from weaviate_amd import hnsw, index_queue
from weaviate_amd._lib import KIND_BQ, KIND_F32, KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2
from weaviate_amd.device import Corpus
from weaviate_amd.distancer import provider_for
from weaviate_amd.flat import AllowList

pytestmark = pytest.mark.gpu

ORC = {METRIC_L2: 0, METRIC_DOT: 1, METRIC_COSINE: 2}
NAME = {METRIC_L2: "l2-squared", METRIC_DOT: "dot", METRIC_COSINE: "cosine-dot"}


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def _rows(orc, metric, X):
    return orc.normalize_rows(X) if metric == METRIC_COSINE else X


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
def test_flat_search_small_allow_list(ctx, orc, metric):
    rng = np.random.default_rng(19)
    n, d = 20_000, 96
    X = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal(d).astype(np.float32)
    c = Corpus(ctx, KIND_F32, metric, d, n)
    try:
        c.upsert(np.arange(n, dtype=np.uint64), X)
        tomb = np.arange(5, n, 97, dtype=np.uint64)  # tombstoned nodes are skipped
        c.delete(tomb)
        allow = rng.choice(n + 500, size=3_000, replace=False)  # some past the node count
        for limit in (1, 10, 100, 500):
            got_i, got_d = hnsw.flat_search(c, q, limit, allow)
            rows = _rows(orc, metric, X)
            qq = orc.normalize(q) if metric == METRIC_COSINE else q
            live = np.array(sorted(int(a) for a in allow if a < n and a not in set(tomb.tolist())), np.uint64)
            all_d = orc.dist_all(ORC[metric], qq, rows[live.astype(np.int64)])
            li, ld = orc.lex_topk(all_d, live, limit)
            assert np.array_equal(got_i, li)
            assert np.array_equal(bits(got_d), bits(ld))
        assert hnsw.flat_search(c, q, 10, [])[0].size == 0
        with pytest.raises(ValueError):
            hnsw.flat_search(c, q, -1, allow)
    finally:
        c.destroy()


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_COSINE])
def test_flat_search_compressed_nodes(ctx, orc, metric):
    """flatSearch on a compressed HNSW: distBetweenNodeAndVec is the BQ
    Hamming / PQ ADC distance of the node's code."""
    rng = np.random.default_rng(23)
    n, d = 6_000, 128
    X = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal(d).astype(np.float32)
    allow = rng.choice(n, size=800, replace=False)
    live = np.array(sorted(allow.tolist()), np.uint64)
    bq = Corpus(ctx, KIND_BQ, metric, d, n)
    try:
        bq.upsert(np.arange(n, dtype=np.uint64), X)
        got_i, got_d = hnsw.flat_search(bq, q, 50, allow)
        rows = _rows(orc, metric, X)
        qq = orc.normalize(q) if metric == METRIC_COSINE else q
        codes = np.stack([orc.bq_encode(r) for r in rows[live.astype(np.int64)]])
        li, ld = orc.lex_topk(orc.bq_dist_all(orc.bq_encode(qq), codes), live, 50)
        assert np.array_equal(got_i, li)
        assert np.array_equal(bits(got_d), bits(ld))
    finally:
        bq.destroy()
    if metric != METRIC_L2:
        return
    m, ks = 16, 256
    centers = rng.standard_normal((m, ks, d // m)).astype(np.float32)
    pq = Corpus(ctx, KIND_PQ, metric, d, n)
    try:
        pq.set_codebook(centers)
        pq.upsert(np.arange(n, dtype=np.uint64), X)
        got_i, got_d = hnsw.flat_search(pq, q, 50, allow)
        codes = orc.pq_encode(X[live.astype(np.int64)], centers)
        lut = orc.pq_lut(0, q, centers)
        adc = np.array([orc.pq_adc(0, lut, cd) for cd in codes], np.float32)
        li, ld = orc.lex_topk(adc, live, 50)
        assert np.array_equal(got_i, li)
        assert np.array_equal(bits(got_d), bits(ld))
    finally:
        pq.destroy()


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
def test_hnsw_rescore_loop(ctx, orc, metric):
    rng = np.random.default_rng(29)
    n, d = 10_000, 256
    X = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal(d).astype(np.float32)
    c = Corpus(ctx, KIND_F32, metric, d, n)
    try:
        c.upsert(np.arange(n, dtype=np.uint64), X)
        gone = np.array([7, 11], dtype=np.uint64)
        c.delete(gone)
        cand = np.concatenate([rng.choice(n, size=498, replace=False).astype(np.uint64), gone])
        got_i, got_d = hnsw.rescore(c, q, cand, k=10, ef=500)
        rows = _rows(orc, metric, X)
        qq = orc.normalize(q) if metric == METRIC_COSINE else q
        want_d = orc.dist_all(ORC[metric], qq, rows[cand.astype(np.int64)])
        want_d[np.isin(cand, gone)] = 0.0  # (0, false, nil) re-inserted at distance 0 (search.go:428-437)
        li, ld = orc.lex_topk(want_d, cand, 10)
        assert np.array_equal(got_i, li)
        assert np.array_equal(bits(got_d), bits(ld))
    finally:
        c.destroy()


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
def test_index_queue_brute_force(ctx, orc, metric):
    rng = np.random.default_rng(31)
    n, d = 4_000, 64
    ids = np.arange(1_000, 1_000 + n, dtype=np.uint64)
    V = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal(d).astype(np.float32)
    qq = orc.normalize(q) if metric == METRIC_COSINE else q
    prov = provider_for(ctx, NAME[metric])  # the caller passes the query normalized for cosine
    seen = set(range(1_000, 1_400))
    allow = AllowList(*range(1_000, 1_000 + n, 2))
    all_d = orc.dist_all(ORC[metric], qq, _rows(orc, metric, V))
    sel = np.array([(int(i) not in seen) and allow.Contains(int(i)) for i in ids])
    max_d = float(np.quantile(all_d[sel], 0.5))
    prior = (np.array([1, 2], np.uint64), np.array([np.float32(max_d) * 2, np.float32(-1e9)], np.float32))
    for k in (-1, 5, 50):
        got_i, got_d = index_queue.brute_force(prov, qq, ids, V, k, results=prior, allow=allow, max_distance=max_d,
                                               seen=seen)
        cid = np.concatenate([prior[0], ids[sel]])
        cd = np.concatenate([prior[1], all_d[sel]])
        # prior entries were in the heap already; new rows must pass the distance filter
        ok = np.concatenate([[True, True], all_d[sel] <= max_d])
        cid, cd = cid[ok], cd[ok]
        want_i, want_d = orc.lex_topk(cd, cid, len(cid) if k < 0 else k)
        assert np.array_equal(bits(got_d), bits(want_d))
        assert np.array_equal(got_i, want_i)


def _corpus_of(ctx, orc, kind, metric, n, d, m=32):
    rng = np.random.default_rng(29 + kind)
    X = rng.standard_normal((n, d)).astype(np.float32)
    c = Corpus(ctx, kind, metric, d, n)
    if kind == KIND_PQ:
        c.set_codebook(orc.synth_rows(31, 0, m * 256, d // m, 0).reshape(m, 256, d // m))
    c.upsert(np.arange(n, dtype=np.uint64), X)
    return c


@pytest.mark.parametrize("kind,metric,m", [(KIND_F32, METRIC_L2, 0), (KIND_F32, METRIC_DOT, 0),
                                           (KIND_F32, METRIC_COSINE, 0), (KIND_BQ, METRIC_COSINE, 0),
                                           (KIND_PQ, METRIC_L2, 32), (KIND_PQ, METRIC_DOT, 16)])
def test_distance_by_ids_batch_equals_per_query(ctx, orc, kind, metric, m):
    """wvg_corpus_distance_by_ids_batch == one wvg_corpus_distance_by_ids per
    query, bit for bit, for ragged lists (empty ones included), deleted and
    unknown ids; rescore_batch == rescore per query."""
    n, d, nq = 5_000, 128, 7
    c = _corpus_of(ctx, orc, kind, metric, n, d, m)
    try:
        c.delete(np.arange(3, n, 101, dtype=np.uint64))
        rng = np.random.default_rng(33)
        qs = rng.standard_normal((nq, d)).astype(np.float32)
        lists = [rng.choice(n + 40, size=sz, replace=False).astype(np.uint64) for sz in (0, 1, 17, 500, 0, 64, 333)]
        got = c.distance_by_ids_batch(qs, lists)
        for q, ids, (dg, okg) in zip(qs, lists, got):
            if ids.size == 0:
                assert dg.size == 0 and okg.size == 0
                continue
            dw, okw = c.distance_by_ids(q, ids)
            assert np.array_equal(okg, okw)
            assert np.array_equal(bits(dg), bits(dw))
        rb = hnsw.rescore_batch(c, qs, lists, 10, ef=200)
        for q, ids, (gi, gd) in zip(qs, lists, rb):
            wi, wd = hnsw.rescore(c, q, ids, 10, ef=200)
            assert np.array_equal(gi, wi) and np.array_equal(bits(gd), bits(wd))
    finally:
        c.destroy()


def test_distance_by_ids_batch_errors(ctx, orc):
    import ctypes

    from weaviate_amd import _lib
    from weaviate_amd._lib import fptr, u64ptr

    c = _corpus_of(ctx, orc, KIND_F32, METRIC_L2, 100, 16)
    try:
        lib = _lib.load()
        q = np.zeros((2, 16), np.float32)
        ids = np.arange(4, dtype=np.uint64)
        out = np.empty(4, np.float32)
        ok = np.empty(4, np.uint8)
        okp = ok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        bad = np.array([0, 3, 2], np.uint64)  # decreasing
        assert lib.wvg_corpus_distance_by_ids_batch(c.handle, fptr(q), 2, u64ptr(bad), u64ptr(ids), fptr(out), okp) < 0
        bad0 = np.array([1, 2, 4], np.uint64)  # offsets[0] != 0
        assert lib.wvg_corpus_distance_by_ids_batch(c.handle, fptr(q), 2, u64ptr(bad0), u64ptr(ids), fptr(out), okp) < 0
        good = np.array([0, 1, 4], np.uint64)
        assert lib.wvg_corpus_distance_by_ids_batch(c.handle, fptr(q), 2, u64ptr(good), u64ptr(ids), fptr(out), okp) == 0
        assert ok.all()
    finally:
        c.destroy()
