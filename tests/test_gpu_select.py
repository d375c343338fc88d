"""GPU parity of the unbounded selections (weaviate_amd/csrc/wvg_select.hip):
SearchByVector with k > 256 (radix select + sort in HBM), the BQ rescore flow
with a window above 256, wvg_rescore with k > 256, and SearchByVectorDistance
(V/flat/index.go:531-591) -- against the oracle on the same seeded inputs.
Distances bit-exact; ids exact under the lexicographic (distance, docID) rule."""
import ctypes

import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_BQ, KIND_F32, KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2
from weaviate_amd.device import Corpus, allow_bitmap, search_bq_rescore

pytestmark = pytest.mark.gpu

ORC_METRIC = {METRIC_L2: 0, METRIC_DOT: 1, METRIC_COSINE: 2}


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def _prep(orc, metric, rows, q):
    if metric == METRIC_COSINE:
        return orc.normalize_rows(rows), orc.normalize(q)
    return rows, q


def check_lex(orc, ids, dists, count, all_d, all_ids, k):
    li, ld = orc.lex_topk(all_d, all_ids, k)
    assert count == len(li)
    assert np.array_equal(ids[:count], li)
    assert np.array_equal(bits(dists[:count]), bits(ld))
    hi, hd = orc.heap_topk(all_d, all_ids, k)
    assert np.array_equal(bits(np.sort(hd)), bits(ld))  # the reference heap keeps the same distances


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
def test_large_k_flat(ctx, orc, metric):
    n, d = 7000 + 5, 96
    rows = orc.synth_rows(301, 0, n, d, 0)
    qs = orc.synth_rows(302, 0, 2, d, 0)
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    srows, _ = _prep(orc, metric, rows, qs[0])
    for k in [257, 1000, 4096, n, n + 100]:
        ids, dists, counts = c.search(qs, k)
        for qi in range(2):
            _, qn = _prep(orc, metric, rows[:1], qs[qi])
            all_d = orc.dist_all(ORC_METRIC[metric], qn, srows)
            check_lex(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k)
            if counts[qi] < k:
                assert np.all(ids[qi, counts[qi]:] == np.uint64(2**64 - 1))


def test_large_k_deletes_allow_ties(ctx, orc):
    """SIFT-like integer rows (heavy exact ties), deletes and an allow list, k > 256."""
    n, d = 9000, 8
    rows = np.floor(orc.synth_rows(311, 0, n, d, 1) / 64).astype(np.float32)
    q = np.floor(orc.synth_rows(312, 0, 1, d, 1)[0] / 64).astype(np.float32)
    base = 640
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n, id_base=base)
    ids_all = np.arange(base, base + n, dtype=np.uint64)
    c.upsert(ids_all, rows)
    dead = np.arange(base, base + n, 7, dtype=np.uint64)
    c.delete(dead)
    allow = np.arange(base + 100, base + 8000, 2, dtype=np.uint64)
    keep = np.isin(ids_all, allow) & ~np.isin(ids_all, dead)
    all_d = orc.dist_all(0, q, rows)
    for k in [300, 2000, 5000]:
        ids, dists, counts = c.search(q, k, allow_bitmap(allow))
        check_lex(orc, ids[0], dists[0], counts[0], all_d[keep], ids_all[keep], k)


def test_large_k_bq_and_pq(ctx, orc):
    n, d = 5000, 256
    rows = orc.synth_rows(321, 0, n, d, 0)
    q = orc.synth_rows(322, 0, 1, d, 0)[0]
    b = Corpus(ctx, KIND_BQ, METRIC_L2, d, n)
    b.upsert(np.arange(n, dtype=np.uint64), rows)
    codes = np.stack([orc.bq_encode(r) for r in rows])
    ham = orc.bq_dist_all(orc.bq_encode(q), codes)
    for k in [300, 3000]:
        ids, dists, counts = b.search(q, k)
        check_lex(orc, ids[0], dists[0], counts[0], ham, np.arange(n, dtype=np.uint64), k)
    # PQ
    m, ks, dd = 16, 256, 64
    centers = orc.synth_rows(323, 0, m * ks, dd // m, 0).reshape(m, ks, dd // m)
    prow = orc.synth_rows(324, 0, n, dd, 0)
    pq = Corpus(ctx, KIND_PQ, METRIC_DOT, dd, n)
    pq.set_codebook(centers)
    pq.upsert(np.arange(n, dtype=np.uint64), prow)
    pcodes = orc.pq_encode(prow, centers)
    qq = orc.synth_rows(325, 0, 1, dd, 0)[0]
    lut = orc.pq_lut(1, qq, centers)
    all_d = np.array([orc.pq_adc(1, lut, cd) for cd in pcodes], np.float32)
    ids, dists, counts = pq.search(qq, 500)
    check_lex(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), 500)


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_COSINE])
def test_bq_rescore_window_above_256(ctx, orc, metric):
    n, d, k, rescore = 6000, 128, 20, 700
    rows = orc.synth_rows(331, 0, n, d, 0)
    q = orc.synth_rows(332, 0, 1, d, 0)[0]
    f = Corpus(ctx, KIND_F32, metric, d, n)
    b = Corpus(ctx, KIND_BQ, metric, d, n)
    f.upsert(np.arange(n, dtype=np.uint64), rows)
    b.upsert(np.arange(n, dtype=np.uint64), rows)
    srows, qn = _prep(orc, metric, rows, q)
    codes = np.stack([orc.bq_encode(r) for r in srows])
    ham = orc.bq_dist_all(orc.bq_encode(qn), codes)
    cand, _ = orc.heap_pops(ham, rescore)  # the reference's Hamming heap of 700, in pop order
    exact = orc.dist_all(ORC_METRIC[metric], qn, srows[cand.astype(np.int64)])
    for kk in [k, 300]:
        ids, dists, counts = search_bq_rescore(b, f, q, kk, rescore)
        li, ld = orc.heap_topk(exact, cand, kk)
        assert counts[0] == kk
        assert np.array_equal(ids[0], li) and np.array_equal(bits(dists[0]), bits(ld))


def test_rescore_host_rows_large_k(ctx, orc):
    lib = _lib.load()
    n, d = 900, 64
    rows = orc.synth_rows(341, 0, n, d, 0)
    q = orc.synth_rows(342, 0, 1, d, 0)[0]
    ids = (5000 + np.arange(n)).astype(np.uint64)
    for k in [300, 1200]:
        oi = np.empty(k, np.uint64)
        od = np.empty(k, np.float32)
        cnt = ctypes.c_uint32()
        _lib.check(lib.wvg_rescore(ctx.handle, METRIC_L2, _lib.fptr(q), _lib.fptr(rows), _lib.u64ptr(ids), n, d, k,
                                   _lib.u64ptr(oi), _lib.fptr(od), ctypes.byref(cnt)))
        all_d = orc.dist_all(0, q, rows)
        hi, hd = orc.heap_topk(all_d, ids, k)  # the rescore loop's heap of k, input order
        assert cnt.value == min(k, n)
        assert np.array_equal(oi[:cnt.value], hi)
        assert np.array_equal(bits(od[:cnt.value]), bits(hd))
        assert np.all(oi[cnt.value:] == np.uint64(2**64 - 1)) and np.all(np.isinf(od[cnt.value:]))


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT])
def test_search_by_distance(ctx, orc, metric):
    """wvg_search_by_distance == the growing-limit loop over the exact sorted list."""
    n, d = 30000, 32
    rows = orc.synth_rows(351, 0, n, d, 0)
    q = orc.synth_rows(352, 0, 1, d, 0)[0]
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    all_d = orc.dist_all(ORC_METRIC[metric], q, rows)
    all_ids = np.arange(n, dtype=np.uint64)
    srt = np.sort(all_d)

    def search_fn(total):
        return orc.lex_topk(all_d, all_ids, total)

    targets = [srt[0] - 1.0, srt[0], srt[49], srt[99], srt[150], srt[1099], srt[1100], srt[5000], srt[-1] + 1,
               np.float32(np.inf)]
    # just below a row's distance: kept through InDelta(1e-6)
    targets.append(np.nextafter(srt[300], np.float32(-np.inf)))
    for t in targets:
        for max_limit in [-1, 50, 1100, 1101, 20000]:
            ei, ed = orc.search_by_distance(search_fn, t, max_limit)
            gi, gd = c.search_by_distance(q, t, max_limit)
            assert len(gi) == len(ei), (t, max_limit, len(gi), len(ei))
            assert np.array_equal(gi, ei)
            assert np.array_equal(bits(gd), bits(ed))
    # NaN target keeps nothing; an allow list restricts
    gi, _ = c.search_by_distance(q, np.float32(np.nan), -1)
    assert len(gi) == 0
    allow = np.arange(0, n, 3, dtype=np.uint64)
    sub = all_d[allow.astype(np.int64)]
    gi, gd = c.search_by_distance(q, srt[2000], -1, allow_bitmap(allow))
    ei, ed = orc.search_by_distance(lambda tot: orc.lex_topk(sub, allow, tot), srt[2000], -1)
    assert np.array_equal(gi, ei) and np.array_equal(bits(gd), bits(ed))


def test_flat_index_search_by_distance_and_large_limit(ctx, orc):
    """FlatIndex mirror: SearchByVector with a large limit and SearchByVectorDistance
    (plain and BQ-compressed) against the oracle loop."""
    from weaviate_amd.flat import AllowList, FlatIndex

    n, d = 3000, 64
    rows = orc.synth_rows(361, 0, n, d, 0)
    q = orc.synth_rows(362, 0, 1, d, 0)[0]
    idx = FlatIndex(ctx, d, "l2-squared", capacity=64)
    idx.AddBatch(np.arange(n), rows)
    all_d = orc.dist_all(0, q, rows)
    ids, dists = idx.SearchByVector(q, 1500)
    li, ld = orc.lex_topk(all_d, np.arange(n, dtype=np.uint64), 1500)
    assert np.array_equal(ids, li) and np.array_equal(bits(dists), bits(ld))
    t = np.sort(all_d)[400]
    gi, gd = idx.SearchByVectorDistance(q, t, -1, semantics="hnsw")
    ei, ed = orc.search_by_distance(lambda tot: orc.lex_topk(all_d, np.arange(n, dtype=np.uint64), tot), t, -1)
    assert np.array_equal(gi, ei) and np.array_equal(bits(gd), bits(ed))
    assert len(idx.SearchByVectorDistance(q, t, -1, AllowList(), semantics="hnsw")[0]) == 0
    # BQ-compressed index: every window is a rescored BQ search
    bidx = FlatIndex(ctx, d, "l2-squared", compression="bq", rescore_limit=400, capacity=64)
    bidx.AddBatch(np.arange(n), rows)
    gi, gd = bidx.SearchByVectorDistance(q, t, -1, semantics="hnsw")
    assert len(gi) > 0 and np.all(gd <= t + 1e-6)
    assert np.array_equal(bits(gd), bits(all_d[gi.astype(np.int64)]))  # rescored = exact distances
    ei, ed = orc.search_by_distance(lambda tot: bidx.SearchByVector(q, tot), t, -1)
    assert np.array_equal(gi, ei) and np.array_equal(bits(gd), bits(ed))


@pytest.mark.parametrize("compression", [None, "bq"])
def test_flat_search_by_distance_reference_semantics(ctx, orc, compression):
    """FlatIndex.SearchByVectorDistance default = the flat index's own result
    (V/flat/index.go:531-591 as written: one window of 100), against the
    literal restatement of that loop (oracle.search_by_distance_flat)."""
    from weaviate_amd.flat import AllowList, FlatIndex

    n, d = 4000, 48
    rows = orc.synth_rows(371, 0, n, d, 0)
    q = orc.synth_rows(372, 0, 1, d, 0)[0]
    kw = dict(compression="bq", rescore_limit=300) if compression else {}
    idx = FlatIndex(ctx, d, "l2-squared", capacity=64, **kw)
    idx.AddBatch(np.arange(n), rows)
    all_d = orc.dist_all(0, q, rows)
    srt = np.sort(all_d)
    for t in [srt[0] - 1, srt[10], srt[99], srt[100], srt[700], np.float32(np.inf),
              np.nextafter(srt[50], np.float32(-np.inf))]:
        for max_limit in [-1, 50, 1100, 100_000]:
            gi, gd = idx.SearchByVectorDistance(q, t, max_limit)
            ei, ed, done = orc.search_by_distance_flat(lambda tot: idx.SearchByVector(q, tot), t, max_limit)
            assert np.array_equal(gi, ei) and np.array_equal(bits(gd), bits(ed)), (t, max_limit)
            assert len(gi) <= 100
            if compression is None:  # and against the exact lexicographic search
                xi, xd, _ = orc.search_by_distance_flat(
                    lambda tot: orc.lex_topk(all_d, np.arange(n, dtype=np.uint64), tot), t, max_limit)
                assert np.array_equal(gi, xi) and np.array_equal(bits(gd), bits(xd))
    # a target past the 100th row: the flat result stops at the window, HNSW semantics go on
    t = srt[700]
    assert len(idx.SearchByVectorDistance(q, t, -1)[0]) == 100
    assert len(idx.SearchByVectorDistance(q, t, -1, semantics="hnsw")[0]) > 100
    allow = AllowList(*range(0, n, 7))
    gi, gd = idx.SearchByVectorDistance(q, srt[2000], -1, allow)
    assert len(gi) == 100 and np.all(gi % 7 == 0)
