"""The reference heap's exact result on the GPU path (wvg_replay.hip).

flat.searchByVectorBQ (V/flat/index.go:347-389) keeps, of the rows tied at
the R-th Hamming distance, whichever its max-heap (priorityqueue/queue.go)
keeps, pops them in the heap's order, and inserts their exact distances into
a heap of k in that order.  With heap_replay (the default) the library
returns exactly that: every test here asserts ids in order and distance bits
equal to the oracle's restatement of the heap (oracle/wv_oracle.c
insert_to_heap / heap_pop / extract_heap), on inputs built to tie heavily --
small d (Hamming 0..64), integer rows (ties in the exact distances too),
batches (the co-scheduled K5 grid), allow lists, deletes, and a docID order
that overflows the per-wave buffers (the rerun path).
"""
import ctypes

import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_BQ, KIND_F32, METRIC_COSINE, METRIC_DOT, METRIC_L2
from weaviate_amd.device import Context, Corpus, allow_bitmap, search_bq_candidates, search_bq_rescore

pytestmark = pytest.mark.gpu

ORC_METRIC = {METRIC_L2: 0, METRIC_DOT: 1, METRIC_COSINE: 2}


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def stored(orc, metric, rows):
    return orc.normalize_rows(rows) if metric == METRIC_COSINE else np.asarray(rows, np.float32)


def prep(orc, metric, q):
    return orc.normalize(q) if metric == METRIC_COSINE else np.asarray(q, np.float32)


def assert_pops(orc, b, qs, codes, qcodes, R, valid=None, allow=None):
    ci, cd, cc = search_bq_candidates(b, qs, R, allow)
    for qi in range(len(qs)):
        pi, pd = orc.bq_heap_pops(codes, qcodes[qi], R, valid)
        assert cc[qi] == len(pi), (qi, cc[qi], len(pi))
        assert np.array_equal(ci[qi][:cc[qi]], pi), qi
        assert np.array_equal(bits(cd[qi][:cc[qi]]), bits(pd)), qi
        assert np.all(ci[qi][cc[qi]:] == np.uint64(0xFFFFFFFFFFFFFFFF))


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
@pytest.mark.parametrize("d,n", [(256, 6000), (64, 20000)])
def test_bq_rescore_flow_equals_reference_heap(ctx, orc, metric, d, n):
    k, R = 10, 200
    rows = orc.synth_rows(55 + d, 0, n, d, 0)
    qs = orc.synth_rows(56 + d, 0, 3, d, 0)
    f = Corpus(ctx, KIND_F32, metric, d, n)
    b = Corpus(ctx, KIND_BQ, metric, d, n)
    try:
        f.upsert(np.arange(n, dtype=np.uint64), rows)
        b.upsert(np.arange(n, dtype=np.uint64), rows)
        srows = stored(orc, metric, rows)
        codes = orc.bq_encode_rows(srows)
        for batch in (False, True):  # one query per call, and a co-scheduled batch
            sel = [qs] if batch else [qs[i] for i in range(len(qs))]
            got = [search_bq_rescore(b, f, q, k, R) for q in sel]
            gi = np.concatenate([g[0] for g in got])
            gd = np.concatenate([g[1] for g in got])
            gc = np.concatenate([g[2] for g in got])
            for qi in range(len(qs)):
                qn = prep(orc, metric, qs[qi])
                ri, rd = orc.flat_search_bq(srows, qn, k, R, ORC_METRIC[metric])
                assert gc[qi] == len(ri)
                assert np.array_equal(gi[qi][:gc[qi]], ri), (batch, qi, gi[qi], ri)
                assert np.array_equal(bits(gd[qi][:gc[qi]]), bits(rd)), (batch, qi)
        assert_pops(orc, b, qs, codes, [orc.bq_encode(prep(orc, metric, q)) for q in qs], R)
    finally:
        f.destroy()
        b.destroy()


def test_bq_candidates_heavy_ties_batches_allow_deletes(ctx, orc):
    """d = 64: Hamming distances 0..64 over 50k rows, so each R-th distance is
    shared by hundreds of rows; batches of 8 (co-scheduled grid), an allow list
    (30 %), deleted rows, R from 1 to 256."""
    n, d = 50_000, 64
    rows = orc.synth_rows(501, 0, n, d, 0)
    qs = orc.synth_rows(502, 0, 8, d, 0)
    b = Corpus(ctx, KIND_BQ, METRIC_L2, d, n)
    try:
        b.upsert(np.arange(n, dtype=np.uint64), rows)
        codes = orc.bq_encode_rows(rows)
        qcodes = [orc.bq_encode(q) for q in qs]
        for R in (1, 7, 64, 200, 256, 257, 700, 3000):  # above 256: the select-based superset
            assert_pops(orc, b, qs, codes, qcodes, R)
            assert_pops(orc, b, qs[:1], codes, qcodes[:1], R)
        rng = np.random.default_rng(7)
        gone = rng.choice(n, n // 20, replace=False).astype(np.uint64)
        b.delete(gone)
        valid = np.ones(n, np.uint8)
        valid[gone.astype(np.int64)] = 0
        assert_pops(orc, b, qs, codes, qcodes, 200, valid)
        assert_pops(orc, b, qs[:2], codes, qcodes[:2], 500, valid)
        allowed = np.sort(rng.choice(n, int(n * 0.3), replace=False)).astype(np.uint64)
        bm = allow_bitmap(allowed, n)
        av = np.zeros(n, np.uint8)
        av[allowed.astype(np.int64)] = 1
        assert_pops(orc, b, qs[:3], codes, qcodes[:3], 200, av & valid, bm)
        # an allow list over one narrow window (the scan plans only its tiles)
        win = np.arange(20_000, 20_700, dtype=np.uint64)
        av2 = np.zeros(n, np.uint8)
        av2[20_000:20_700] = 1
        assert_pops(orc, b, qs[:2], codes, qcodes[:2], 200, av2 & valid, allow_bitmap(win, n))
    finally:
        b.destroy()


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT])
def test_bq_rescore_integer_rows_ties_in_both_heaps(ctx, orc, metric):
    """Integer rows in [-128, 127] at d = 32: Hamming 0..32 and small-integer
    exact distances, so both the R-heap and the k-heap see ties at their
    boundary and among equal distances in their output order."""
    n, d, k, R = 30_000, 32, 10, 200
    rows = orc.synth_rows(601, 0, n, d, 1) - np.float32(128)
    qs = orc.synth_rows(602, 0, 4, d, 1) - np.float32(128)
    rows[5000:5100] = rows[17]  # exact duplicates: equal exact distances
    f = Corpus(ctx, KIND_F32, metric, d, n)
    b = Corpus(ctx, KIND_BQ, metric, d, n)
    try:
        f.upsert(np.arange(n, dtype=np.uint64), rows)
        b.upsert(np.arange(n, dtype=np.uint64), rows)
        for RR in (R, 600):  # 600: the select-based superset above 256
            gi, gd, gc = search_bq_rescore(b, f, qs, k, RR)
            for qi in range(len(qs)):
                ri, rd = orc.flat_search_bq(rows, qs[qi], k, RR, ORC_METRIC[metric])
                assert gc[qi] == len(ri)
                assert np.array_equal(gi[qi], ri), (RR, qi, gi[qi], ri)
                assert np.array_equal(bits(gd[qi]), bits(rd)), (RR, qi)
        gi, gd, gc = search_bq_rescore(b, f, qs, k, R)
        for qi in range(len(qs)):
            ri, rd = orc.flat_search_bq(rows, qs[qi], k, R, ORC_METRIC[metric])
            assert gc[qi] == len(ri)
            assert np.array_equal(gi[qi], ri), (qi, gi[qi], ri)
            assert np.array_equal(bits(gd[qi]), bits(rd)), qi
        # a query equal to the duplicated row: its 100 copies tie at distance 0 / -|x|^2
        gi, gd, gc = search_bq_rescore(b, f, rows[17], k, R)
        ri, rd = orc.flat_search_bq(rows, rows[17], k, R, ORC_METRIC[metric])
        assert np.array_equal(gi[0], ri) and np.array_equal(bits(gd[0]), bits(rd))
    finally:
        f.destroy()
        b.destroy()


def test_bq_candidates_overflow_rerun(ctx, orc):
    """Distances falling with the docID (1536 - id mod 1500 set bits against an
    all-zero query code): every row of a wave beats the wave's own running
    R-th, so the per-wave buffers overflow and the query is rerun with
    full-size buffers seeded from the first pass -- still the heap's result."""
    n, d = 400_000, 1536
    w = d // 64
    nb = (1536 - (np.arange(n) % 1500)).astype(np.int64)
    codes = np.zeros((n, w), np.uint64)
    for j in range(w):
        c = np.clip(nb - 64 * j, 0, 64)
        full = c >= 64
        codes[:, j] = np.where(full, np.uint64(0xFFFFFFFFFFFFFFFF),
                               (np.left_shift(np.uint64(1), np.minimum(c, 63).astype(np.uint64)) - np.uint64(1)))
    b = Corpus(ctx, KIND_BQ, METRIC_L2, d, n)
    try:
        b.upsert_codes(np.arange(n, dtype=np.uint64), codes)
        q = np.ones((2, d), np.float32)  # code 0: distance = set bits
        qc = [np.zeros(w, np.uint64)] * 2
        for R in (1, 4, 200, 600):
            assert_pops(orc, b, q, codes, qc, R)
            assert_pops(orc, b, q[:1], codes, qc[:1], R)
    finally:
        b.destroy()


def test_rescore_host_rows_is_the_k_heap(ctx, orc):
    """wvg_rescore inserts in input order into a heap of k and extracts it
    (V/flat/index.go:375-387): duplicate rows make equal distances whose
    output order is the heap's."""
    lib = _lib.load()
    n, d = 400, 64
    rows = orc.synth_rows(71, 0, n, d, 1) - np.float32(128)
    rows[50:90] = rows[3]
    q = rows[3] + np.float32(1)
    ids = (1000 + 3 * np.arange(n)[::-1]).astype(np.uint64)
    for metric in (METRIC_L2, METRIC_DOT):
        for k in (1, 10, 45, 300):
            oi = np.empty(k, np.uint64)
            od = np.empty(k, np.float32)
            cnt = ctypes.c_uint32()
            _lib.check(lib.wvg_rescore(ctx.handle, metric, _lib.fptr(q), _lib.fptr(rows), _lib.u64ptr(ids), n, d, k,
                                       _lib.u64ptr(oi), _lib.fptr(od), ctypes.byref(cnt)))
            hi, hd = orc.heap_topk(orc.dist_all(ORC_METRIC[metric], q, rows), ids, k)
            assert cnt.value == len(hi)
            assert np.array_equal(oi[:cnt.value], hi) and np.array_equal(bits(od[:cnt.value]), bits(hd))


def test_lexicographic_mode(orc):
    """heap_replay = 0 keeps the (distance, docID)-lexicographic candidates."""
    n, d, k, R = 20_000, 64, 10, 200
    rows = orc.synth_rows(801, 0, n, d, 0)
    q = orc.synth_rows(802, 0, 1, d, 0)[0]
    with Context(0, heap_replay=0) as c0:
        f = Corpus(c0, KIND_F32, METRIC_L2, d, n)
        b = Corpus(c0, KIND_BQ, METRIC_L2, d, n)
        f.upsert(np.arange(n, dtype=np.uint64), rows)
        b.upsert(np.arange(n, dtype=np.uint64), rows)
        gi, gd, gc = search_bq_rescore(b, f, q, k, R)
        ham = orc.bq_dist_all(orc.bq_encode(q), orc.bq_encode_rows(rows))
        cand, cd = orc.lex_topk(ham, np.arange(n, dtype=np.uint64), R)
        li, ld = orc.lex_topk(orc.dist_all(0, q, rows[cand.astype(np.int64)]), cand, k)
        assert np.array_equal(gi[0], li) and np.array_equal(bits(gd[0]), bits(ld))
        ci, cdd, cc = search_bq_candidates(b, q, R)
        assert cc[0] == R and np.array_equal(ci[0], cand[::-1]) and np.array_equal(bits(cdd[0]), bits(cd[::-1]))
        f.destroy()
        b.destroy()
