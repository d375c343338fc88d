"""Full-size GPU tests (BASELINE.json configs 1-5 at their own per-GPU sizes).

This file collects LAST (the zz name) so that a fault in one of these
minutes-long tests cannot hide the quicker parity files under ``-x``.  The
oracle cannot scan 100M rows in seconds, so configs 2-5 check
size-independent properties: stored rows / codes bit-exact against the
oracle's generator on sampled tiles (start, middle, end and a stride over the
whole corpus), results sorted, every returned distance a bit-exact
recomputation of its row, and no sampled row outside the result ahead of the
k-th in (distance, docID) order.  Config 1 (1M x 128) is checked exactly:
every stored row, and the whole top-k against the oracle.
"""
import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_BQ, KIND_F32, KIND_PQ, METRIC_COSINE, METRIC_L2
from weaviate_amd.device import Corpus

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


# ---------------------------------------------------------------------------
# Full size (BASELINE config 1): 1M x 128 L2, created and filled back to back
# (a 512 MB allocation zero-filled on a pool stream, then written by the
# synthetic generator on another: round 1's fill raced the zeroing).
def test_full_size_1m_x_128_exact(ctx, orc):
    n, d, k = 1_000_000, 128, 10
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.fill_synthetic(42, n, 0)
    all_rows = orc.synth_rows(42, 0, n, d, 0)
    # every stored row, bit for bit
    got, ok = c.get_batch(np.arange(n, dtype=np.uint64))
    assert ok.all()
    bad = np.nonzero((got.view(np.uint32) != all_rows.view(np.uint32)).any(axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} stored rows differ, first {bad[:8]}"
    qs = orc.synth_rows(43, 0, 3, d, 0)
    ids, dists, counts = c.search(qs, k)
    for qi in range(len(qs)):
        assert counts[qi] == k
        all_d = orc.dist_all(0, qs[qi], all_rows)
        wi, wd = orc.lex_topk(all_d, np.arange(n, dtype=np.uint64), k)
        assert np.array_equal(ids[qi], wi)
        assert np.array_equal(bits(dists[qi]), bits(wd))
        for i, dv in zip(ids[qi], dists[qi]):  # the returned rows as stored
            assert bits(orc.dist_all(0, qs[qi], c.get(int(i))[None])) == bits(dv)
    c.destroy()


# The headline's own kernel on the headline's own shape:
# the query-stream launch (wvg_search_device_pipelined, 16 single-query scans
# per launch, as bench.py times it) three times in a row over 1M x 128 -- so
# the scans alternate direction and each starts on the default-policy tail
# the previous one left in the Infinity Cache -- and lone wvg_search calls
# (the in-launch merge into host memory), every result the oracle's exact
# top-10 over all 1M rows.
def test_full_size_headline_stream_and_lone_queries_exact(ctx, orc):
    import ctypes

    lib = _lib.load()
    n, d, k, nq, launches = 1_000_000, 128, 10, 16, 3
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.fill_synthetic(42, n, 0)
    rows = orc.synth_rows(42, 0, n, d, 0)
    all_ids = np.arange(n, dtype=np.uint64)
    h = ctx.handle

    def alloc(nbytes, zero=0):
        p = ctypes.c_void_p()
        _lib.check(lib.wvg_device_alloc(h, nbytes, zero, ctypes.byref(p)))
        return p

    s = ctypes.c_void_p()
    _lib.check(lib.wvg_stream_create(h, ctypes.byref(s)))
    wsb = lib.wvg_search_workspace_size(c.handle, nq, k)
    dq, di, dd, dc, ws = alloc(nq * d * 4), alloc(nq * k * 8), alloc(nq * k * 4), alloc(nq * 4), alloc(wsb, 1)
    try:
        results = []
        for L in range(launches):  # back to back on one stream, no host sync between launches
            qs = np.ascontiguousarray(orc.synth_rows(4300 + L, 0, nq, d, 0))
            _lib.check(lib.wvg_memcpy_h2d(h, dq, qs.ctypes.data_as(ctypes.c_void_p), qs.nbytes, s))
            _lib.check(lib.wvg_search_device_pipelined(c.handle, dq, nq, k, di, dd, dc, ws, wsb, s))
            gi, gd, gc = np.empty((nq, k), np.uint64), np.empty((nq, k), np.float32), np.empty(nq, np.uint32)
            for host, dev in ((gi, di), (gd, dd), (gc, dc)):
                _lib.check(lib.wvg_memcpy_d2h(h, host.ctypes.data_as(ctypes.c_void_p), dev, host.nbytes, s))
            results.append((qs, gi, gd, gc))
        _lib.check(lib.wvg_search_device_check(h, ws, s))
        for qs, gi, gd, gc in results:
            assert np.all(gc == k)
            for qi in range(nq):
                wi, wd = orc.lex_topk(orc.dist_all(0, qs[qi], rows), all_ids, k)
                assert np.array_equal(gi[qi], wi), qi
                assert np.array_equal(bits(gd[qi]), bits(wd)), qi
    finally:
        for p in (dq, di, dd, dc, ws):
            _lib.check(lib.wvg_device_free(h, p))
        _lib.check(lib.wvg_stream_destroy(h, s))
    lone = orc.synth_rows(4400, 0, 4, d, 0)
    for qi in range(len(lone)):  # one query per call: alternating directions between calls
        gi, gd, gc = c.search(lone[qi], k)
        wi, wd = orc.lex_topk(orc.dist_all(0, lone[qi], rows), all_ids, k)
        assert gc[0] == k and np.array_equal(gi[0], wi) and np.array_equal(bits(gd[0]), bits(wd)), qi
    c.destroy()


# Full size (BASELINE config 4): 100M x 128 L2, PQ m=32 ks=256 -- bulk encode on
# the device, then ADC top-10 over all 100M codes; checked by properties on
# sampled rows (the oracle cannot encode and scan 100M rows in seconds).
def test_full_size_pq_100m_properties(ctx, orc):
    n, d, m, ks, k = 100_000_000, 128, 32, 256, 10
    f = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    f.fill_synthetic(42, n, 0)
    centers = np.ascontiguousarray(orc.synth_rows(42, 0, ks, d, 0).reshape(ks, m, d // m).transpose(1, 0, 2))
    pq = Corpus(ctx, KIND_PQ, METRIC_L2, d, n)
    pq.set_codebook(centers)
    _lib.check(_lib.load().wvg_pq_encode_corpus(pq.handle, f.handle))
    f.destroy()
    # sampled rows at the start, the middle and the end: codes bit-exact vs the oracle
    starts = [0, n // 2 - 7, n - 20_000]
    sample_ids = np.concatenate([np.arange(s, s + 20_000, dtype=np.int64) for s in starts])
    srows = np.concatenate([orc.synth_rows(42, s, 20_000, d, 0) for s in starts])
    scodes = orc.pq_encode(srows, centers)
    for j in range(0, len(sample_ids), 997):
        assert np.array_equal(pq.get(int(sample_ids[j]), pq_m=m), scodes[j]), int(sample_ids[j])
    qs = orc.synth_rows(43, 0, 3, d, 0)
    ids, dists, counts = pq.search(qs, k)
    for qi in range(len(qs)):
        assert counts[qi] == k
        assert np.all(np.diff(orc.ord_key(dists[qi]).astype(np.int64)) >= 0)
        lut = orc.pq_lut(0, qs[qi], centers)
        # each returned distance is the sequential ADC sum of that row's stored code
        for i, dv in zip(ids[qi], dists[qi]):
            assert bits(orc.pq_adc(0, lut, pq.get(int(i), pq_m=m))) == bits(dv)
        # no sampled row outside the result beats the k-th result (lexicographic (dist, id))
        sd = np.array([orc.pq_adc(0, lut, c) for c in scodes], np.float32)
        outside = ~np.isin(sample_ids, ids[qi].astype(np.int64))
        kth = (int(orc.ord_key(dists[qi][-1:])[0]), int(ids[qi][-1]))
        sk = orc.ord_key(sd[outside]).astype(np.int64)
        assert np.all((sk > kth[0]) | ((sk == kth[0]) & (sample_ids[outside] > kth[1])))
    pq.destroy()


# Full size (BASELINE config 3): 100M x 1536 BQ (W = 24 words) cosine, Hamming
# top-200 over all 100M device-resident codes (the 614 GB of float rows do not
# fit, so the rescore stage is covered at small sizes above).
def test_full_size_bq_100m_x_1536_properties(ctx, orc):
    n, d, R = 100_000_000, 1536, 200
    w = (d + 63) // 64
    c = Corpus(ctx, KIND_BQ, METRIC_COSINE, d, n)
    c.fill_synthetic(42, n, 0)
    starts = [0, n // 2 - 13, n - 10_000]
    sample_ids = np.concatenate([np.arange(s, s + 10_000, dtype=np.int64) for s in starts])
    scodes = np.stack([orc.bq_encode(orc.normalize(r)) for s in starts for r in orc.synth_rows(42, s, 10_000, d, 0)])
    for j in range(0, len(sample_ids), 499):
        assert np.array_equal(c.get(int(sample_ids[j])), scodes[j]), int(sample_ids[j])
    qs = orc.synth_rows(43, 0, 2, d, 0)
    ids, dists, counts = c.search(qs, R)
    for qi in range(len(qs)):
        assert counts[qi] == R
        assert np.all(np.diff(dists[qi]) >= 0)
        qc = orc.bq_encode(orc.normalize(qs[qi]))
        got = np.stack([c.get(int(i)) for i in ids[qi]])
        assert got.shape == (R, w)
        assert np.array_equal(bits(orc.bq_dist_all(qc, got)), bits(dists[qi]))
        sd = orc.bq_dist_all(qc, scodes)
        outside = ~np.isin(sample_ids, ids[qi].astype(np.int64))
        kd, kid = float(dists[qi][-1]), int(ids[qi][-1])
        assert np.all((sd[outside] > kd) | ((sd[outside] == kd) & (sample_ids[outside] > kid)))
    # the reference heap's candidates exactly: findTopVectorsCached over all 100M
    # stored codes (streamed back from the device), its pop order, vs the library's
    from weaviate_amd.device import search_bq_candidates

    ci, cd, cc = search_bq_candidates(c, qs, R)
    for qi in range(len(qs)):
        qc = orc.bq_encode(orc.normalize(qs[qi]))
        pi, pd = orc.heap_pops(_bq_dists_chunked(orc, c, qc, n), R)
        assert cc[qi] == R
        assert np.array_equal(ci[qi], pi), qi
        assert np.array_equal(bits(cd[qi]), bits(pd)), qi
    c.destroy()


def _bq_dists_chunked(orc, c, qc, n, chunk=4_000_000):
    """Hamming distances of qc to every stored code of BQ corpus c (ids 0..n-1),
    read back chunk by chunk (wvg_corpus_get_batch)."""
    out = np.empty(n, np.float32)
    for r0 in range(0, n, chunk):
        codes, ok = c.get_batch(np.arange(r0, min(n, r0 + chunk), dtype=np.uint64))
        assert ok.all()
        out[r0:r0 + len(codes)] = orc.bq_dist_all(qc, codes)
    return out


# Full size (BASELINE config 2): 10M x 768 fp32 cosine, one 1024-query batch
# through the default batched path -- the K3d bf16 MFMA screen (a K3b exact
# fp32 MFMA pilot, exact seeds, the exact AVX2-order rescore of the kept
# candidates) -- properties on sampled rows and queries.
def test_full_size_batched_10m_x_768_cosine_properties(ctx, orc):
    n, d, nq, k = 10_000_000, 768, 1024, 10
    c = Corpus(ctx, KIND_F32, METRIC_COSINE, d, n)
    c.fill_synthetic(42, n, 0)
    starts = [0, n // 2 - 3, n - 10_000]
    sample_ids = np.concatenate([np.arange(s, s + 10_000, dtype=np.int64) for s in starts])
    srows = np.concatenate([orc.normalize_rows(orc.synth_rows(42, s, 10_000, d, 0)) for s in starts])
    for j in range(0, len(sample_ids), 997):
        assert np.array_equal(bits(c.get(int(sample_ids[j]))), bits(srows[j])), int(sample_ids[j])
    qs = orc.synth_rows(43, 0, nq, d, 0)
    ids, dists, counts = c.search(qs, k)
    assert np.all(counts == k)
    for qi in (0, 1, 511, 1023):
        q = orc.normalize(qs[qi])
        assert np.all(np.diff(orc.ord_key(dists[qi]).astype(np.int64)) >= 0)
        got = orc.normalize_rows(np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in ids[qi]]))
        assert np.array_equal(bits(orc.dist_all(2, q, got)), bits(dists[qi]))
        sd = orc.dist_all(2, q, srows)
        outside = ~np.isin(sample_ids, ids[qi].astype(np.int64))
        kth = (int(orc.ord_key(dists[qi][-1:])[0]), int(ids[qi][-1]))
        sk = orc.ord_key(sd[outside]).astype(np.int64)
        assert np.all((sk > kth[0]) | ((sk == kth[0]) & (sample_ids[outside] > kth[1])))
    c.destroy()


# Full size (BASELINE config 5, one GPU's share): a 125M x 128 fp32 L2 slab
# holding global docIDs [375M, 500M) (slab 3 of 8), exact 100-NN.
def test_full_size_slab_125m_global_ids_properties(ctx, orc):
    n, d, k, base = 125_000_000, 128, 100, 375_000_000
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n, id_base=base)
    c.fill_synthetic(42, n, 0)
    starts = [base, base + n // 2 - 5, base + n - 20_000]
    sample_ids = np.concatenate([np.arange(s, s + 20_000, dtype=np.int64) for s in starts])
    srows = np.concatenate([orc.synth_rows(42, s, 20_000, d, 0) for s in starts])
    for j in range(0, len(sample_ids), 997):
        assert np.array_equal(bits(c.get(int(sample_ids[j]))), bits(srows[j])), int(sample_ids[j])
    # whole tiles strided over the slab (every chunk of every lane of them)
    for t0 in range(0, n, 64 * 4000):
        tid = np.arange(base + t0, base + min(n, t0 + 64), dtype=np.uint64)
        got, ok = c.get_batch(tid)
        assert ok.all() and np.array_equal(bits(got), bits(orc.synth_rows(42, int(tid[0]), len(tid), d, 0)))
    qs = orc.synth_rows(43, 0, 2, d, 0)
    ids, dists, counts = c.search(qs, k)
    for qi in range(len(qs)):
        assert counts[qi] == k
        assert np.all((ids[qi] >= base) & (ids[qi] < base + n))
        assert np.all(np.diff(orc.ord_key(dists[qi]).astype(np.int64)) >= 0)
        got = np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in ids[qi]])
        assert np.array_equal(bits(orc.dist_all(0, qs[qi], got)), bits(dists[qi]))
        sd = orc.dist_all(0, qs[qi], srows)
        outside = ~np.isin(sample_ids, ids[qi].astype(np.int64))
        kth = (int(orc.ord_key(dists[qi][-1:])[0]), int(ids[qi][-1]))
        sk = orc.ord_key(sd[outside]).astype(np.int64)
        assert np.all((sk > kth[0]) | ((sk == kth[0]) & (sample_ids[outside] > kth[1])))
    c.destroy()


def _exact_topk_chunked(orc, metric, q, seed, n, d, k, chunk=1_000_000, normalize=False):
    """The oracle's lexicographic top-k of q over all n synthetic rows
    (generated chunk by chunk, so the whole corpus never sits in host memory)."""
    best_i = np.empty(0, np.uint64)
    best_d = np.empty(0, np.float32)
    for r0 in range(0, n, chunk):
        rows = orc.synth_rows(seed, r0, min(chunk, n - r0), d, 0)
        if normalize:
            rows = orc.normalize_rows(rows)
        dd = orc.dist_all(metric, q, rows)
        ci, cd = orc.lex_topk(dd, np.arange(r0, r0 + len(rows), dtype=np.uint64), k)
        best_i, best_d = orc.lex_topk(np.concatenate([best_d, cd]), np.concatenate([best_i, ci]), k)
    return best_i, best_d


# Full size (BASELINE config 2, dot): 10M x 768 fp32 dot, one 1024-query batch
# through the bf16 screen + exact rescore -- properties on sampled rows for four
# queries, and the whole 10M-row oracle top-k for two of them.
def test_full_size_batched_10m_x_768_dot_exact(ctx, orc):
    n, d, nq, k = 10_000_000, 768, 1024, 10
    c = Corpus(ctx, KIND_F32, _lib.METRIC_DOT, d, n)
    c.fill_synthetic(42, n, 0)
    qs = orc.synth_rows(43, 0, nq, d, 0)
    ids, dists, counts = c.search(qs, k)
    assert np.all(counts == k)
    starts = [0, n // 2 - 3, n - 10_000]
    sample_ids = np.concatenate([np.arange(s, s + 10_000, dtype=np.int64) for s in starts])
    srows = np.concatenate([orc.synth_rows(42, s, 10_000, d, 0) for s in starts])
    for qi in (0, 1, 511, 1023):
        assert np.all(np.diff(orc.ord_key(dists[qi]).astype(np.int64)) >= 0)
        got = np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in ids[qi]])
        assert np.array_equal(bits(orc.dist_all(1, qs[qi], got)), bits(dists[qi]))
        sd = orc.dist_all(1, qs[qi], srows)
        outside = ~np.isin(sample_ids, ids[qi].astype(np.int64))
        kth = (int(orc.ord_key(dists[qi][-1:])[0]), int(ids[qi][-1]))
        sk = orc.ord_key(sd[outside]).astype(np.int64)
        assert np.all((sk > kth[0]) | ((sk == kth[0]) & (sample_ids[outside] > kth[1])))
    for qi in (0, 1023):  # the exact answer over all 10M rows
        wi, wd = _exact_topk_chunked(orc, 1, qs[qi], 42, n, d, k)
        assert np.array_equal(ids[qi], wi), qi
        assert np.array_equal(bits(dists[qi]), bits(wd)), qi
    c.destroy()


# Config 3 at the largest size that fits with its float rows resident: 10M x
# 1536 fp32 (61 GB) + its BQ codes, flat.searchByVectorBQ with the exact
# rescore on the device (wvg_search_bq_rescore, R = 200, k = 10;
# V/flat/index.go:347-389), checked EXACTLY against the reference flow
# restated: the Hamming heap over all 10M stored codes (streamed back), its
# pop order, the exact cosine distances of those rows inserted into a heap of
# k in that order, extracted -- ids in order and distance bits equal.
def test_full_size_bq_rescore_10m_x_1536_resident(ctx, orc):
    from weaviate_amd.device import search_bq_candidates, search_bq_rescore

    n, d, R, k = 10_000_000, 1536, 200, 10
    f = Corpus(ctx, KIND_F32, METRIC_COSINE, d, n)
    f.fill_synthetic(42, n, 0)
    bq = Corpus(ctx, KIND_BQ, METRIC_COSINE, d, n)
    bq.fill_synthetic(42, n, 0)
    qs = orc.synth_rows(43, 0, 4, d, 0)
    ids, dists, counts = search_bq_rescore(bq, f, qs, k, R)
    ci, cd, cc = search_bq_candidates(bq, qs, R)
    for qi in range(len(qs)):
        qn = orc.normalize(qs[qi])
        pi, pd = orc.heap_pops(_bq_dists_chunked(orc, bq, orc.bq_encode(qn), n), R)
        assert cc[qi] == R and np.array_equal(ci[qi], pi) and np.array_equal(bits(cd[qi]), bits(pd)), qi
        rows = orc.normalize_rows(np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in pi]))
        wi, wd = orc.heap_topk(orc.dist_all(2, qn, rows), pi, k)
        assert counts[qi] == k
        assert np.array_equal(ids[qi], wi), qi
        assert np.array_equal(bits(dists[qi]), bits(wd)), qi
    f.destroy()
    bq.destroy()
