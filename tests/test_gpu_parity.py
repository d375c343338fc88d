import ctypes
"""GPU parity tests: the HIP path (through the C ABI) against the oracle on the
same seeded inputs, bit-exact for distances / codes / ids.

Tie rule: the GPU returns the lexicographic (distance, docID) top-k; the
reference's heap keeps an arbitrary member of a tie at the k-th distance.
Every test asserts (1) bit-exact equality with the lexicographic oracle and
(2) equality with the reference-heap oracle except inside the boundary tie.
"""
import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_BQ, KIND_F32, KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2
from weaviate_amd.device import Corpus, allow_bitmap, search_bq_rescore

pytestmark = pytest.mark.gpu

ORC_METRIC = {METRIC_L2: 0, METRIC_DOT: 1, METRIC_COSINE: 2}


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def stored_rows(orc, metric, rows):
    return orc.normalize_rows(rows) if metric == METRIC_COSINE else np.asarray(rows, np.float32)


def prep_query(orc, metric, q):
    return orc.normalize(q) if metric == METRIC_COSINE else np.asarray(q, np.float32)


def check_topk(orc, ids, dists, count, all_d, all_ids, k, valid=None):
    """GPU result vs lexicographic oracle (exact) and vs the reference heap (modulo ties)."""
    sel = np.ones(len(all_d), bool) if valid is None else valid.astype(bool)
    li, ld = orc.lex_topk(all_d[sel], all_ids[sel], k)
    assert count == len(li)
    assert np.array_equal(ids[:count], li)
    assert np.array_equal(bits(dists[:count]), bits(ld))
    hi, hd = orc.heap_topk(all_d, all_ids, k, valid)
    assert np.array_equal(bits(np.sort(hd)), bits(ld))  # same distance multiset
    if count:
        cut = ld[-1]
        assert set(hi[hd < cut].tolist()) == set(li[ld < cut].tolist())


# ---------------------------------------------------------------------------
def test_distance_batch_bitexact_vs_reference_kernels(ctx, orc):
    """Provider.SingleDist on the GPU == the reference's own l2_256 / dot_256 outputs
    (tests/golden/distances.npz), every length 1..1536."""
    import os
    from weaviate_amd.distancer import CosineDistanceProvider, DotProductProvider, L2SquaredProvider

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "distances.npz"))
    l2p, dp, cp = L2SquaredProvider(ctx), DotProductProvider(ctx), CosineDistanceProvider(ctx)
    off = 0
    got = {"l2": [], "dot": [], "cos": []}
    for n in g["lens"]:
        a, b = g["a"][off:off + n], g["b"][off:off + n]
        off += n
        got["l2"].append(l2p.BatchDist(a, b[None])[0])
        got["dot"].append(dp.BatchDist(a, b[None])[0])
        got["cos"].append(cp.BatchDist(a, b[None])[0])
    assert np.array_equal(bits(got["l2"]), bits(g["l2_256"]))
    assert np.array_equal(bits(got["dot"]), bits(-g["dot_256"]))
    assert np.array_equal(bits(got["cos"]), bits(np.float32(1) - g["dot_256"]))


def test_known_answers_on_gpu(ctx):
    from weaviate_amd.distancer import CosineDistanceProvider, DotProductProvider, L2SquaredProvider, Normalize

    l2p, dp, cp = L2SquaredProvider(ctx), DotProductProvider(ctx), CosineDistanceProvider(ctx)
    assert l2p.SingleDist([3, 4, 5], [1.5, 2, 2.5])[0] == 12.5  # D/l2_test.go:37-50
    assert l2p.SingleDist([10, 11], [13, 15])[0] == 25  # :52-65
    assert dp.SingleDist([3, 4, 5], [-3, -4, -5])[0] == 50  # D/dot_product_test.go:50-63
    d, ok, err = l2p.SingleDist([1, 2], [1, 2, 3])
    assert not ok and err == "vector lengths don't match: 2 vs 3"
    a, b = Normalize(ctx, [0.1, 0.3, 0.7]), Normalize(ctx, [0.2, 0.2, 0.2])
    assert abs(cp.SingleDist(a, b)[0] - 0.173) < 0.01  # D/cosine_dist_test.go:51-65
    assert cp.SingleDist([0.1, -0.2], [0.8, -0.2])[0] == np.float32(0.88)  # CH/compression_test.go:84-86
    # Step-by-step equals SingleDist (D/l2_test.go:68-88)
    s = np.float32(0)
    for x, y in zip([3, 4, 5], [1.5, 2, 2.5]):
        s = np.float32(s + l2p.Step([x], [y]))
    assert s == 12.5


@pytest.mark.parametrize("d", [1, 63, 64, 65, 77, 128, 1536])
def test_normalize_bitexact(ctx, orc, d):
    """normalize_rows_kernel (one wave per row, the sum folded in element order
    through v_readlane) = Normalize's sequential fp32 sum (D/normalize.go:16-32),
    for dims around the 64-element block, zero rows and non-finite elements."""
    from weaviate_amd.distancer import Normalize

    X = orc.synth_rows(11 + d, 0, 300, d, 0) * np.float32(3e3)
    X[3] = 0
    X[5, d // 2] = np.inf
    X[7, d - 1] = np.nan
    X[9] = np.float32(1e-30)  # squares underflow: a zero norm
    assert np.array_equal(bits(Normalize(ctx, X)), bits(orc.normalize_rows(X)))


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
@pytest.mark.parametrize("d", [3, 37, 128, 200, 768])
def test_flat_search_parity(ctx, orc, metric, d):
    n = 4000 + 17  # ragged: not a multiple of the 64-row tile
    rows = orc.synth_rows(100 + d, 0, n, d, 0)
    qs = orc.synth_rows(200 + d, 0, 3, d, 0)
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    srows = stored_rows(orc, metric, rows)
    for k in [1, 10, 64, 65, 100, 256]:
        ids, dists, counts = c.search(qs, k)
        for qi in range(len(qs)):
            all_d = orc.dist_all(ORC_METRIC[metric], prep_query(orc, metric, qs[qi]), srows)
            check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k)


def test_flat_search_sift_like_ties(ctx, orc):
    """Integer-valued rows (SIFT-like): exact sums and many distance ties."""
    n, d = 20000, 16
    rows = np.floor(orc.synth_rows(7, 0, n, d, 1) / 64)  # values 0..3 -> heavy ties
    rows = rows.astype(np.float32)
    q = np.floor(orc.synth_rows(8, 0, 1, d, 1)[0] / 64).astype(np.float32)
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    for k in [10, 100, 200]:
        ids, dists, counts = c.search(q, k)
        all_d = orc.dist_all(0, q, rows)
        check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), k)


def test_delete_allow_list_and_edge_cases(ctx, orc):
    n, d, k = 3000, 64, 10
    rows = orc.synth_rows(21, 0, n, d, 0)
    q = orc.synth_rows(22, 0, 1, d, 0)[0]
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, 4096)
    # empty corpus -> empty result (not an error)
    ids, dists, counts = c.search(q, k)
    assert counts[0] == 0
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    all_d = orc.dist_all(0, q, rows)
    all_ids = np.arange(n, dtype=np.uint64)
    # deletes (V/flat/index.go:276-295)
    top = c.search(q, k)[0][0]
    c.delete(top[:5])
    valid = np.ones(n, np.uint8)
    valid[top[:5].astype(np.int64)] = 0
    ids, dists, counts = c.search(q, k)
    check_topk(orc, ids[0], dists[0], counts[0], all_d, all_ids, k, valid)
    assert c.info()[0] == n - 5
    # re-add one deleted id
    c.upsert(top[:1], rows[top[:1].astype(np.int64)])
    valid[int(top[0])] = 1
    ids, dists, counts = c.search(q, k)
    check_topk(orc, ids[0], dists[0], counts[0], all_d, all_ids, k, valid)
    # allow lists (sparse, ranged) restrict candidates (V/flat/index.go:423-449)
    rng = np.random.default_rng(5)
    allowed = np.sort(rng.choice(np.arange(100, 2000), 57, replace=False)).astype(np.uint64)
    am = np.zeros(n, np.uint8)
    am[allowed.astype(np.int64)] = 1
    ids, dists, counts = c.search(q, k, allow_bitmap(allowed))
    check_topk(orc, ids[0], dists[0], counts[0], all_d, all_ids, k, am & valid)
    # empty allow list -> empty result
    ids, dists, counts = c.search(q, k, np.zeros(10, np.uint64))
    assert counts[0] == 0
    # k larger than live rows
    small = Corpus(ctx, KIND_F32, METRIC_L2, d, 64)
    small.upsert(np.arange(7, dtype=np.uint64), rows[:7])
    ids, dists, counts = small.search(q, 50)
    assert counts[0] == 7
    check_topk(orc, ids[0], dists[0], counts[0], orc.dist_all(0, q, rows[:7]), np.arange(7, dtype=np.uint64), 50)
    # k above the fused register top-k runs the select path with the same result rule
    ids, dists, counts = c.search(q, 257)
    check_topk(orc, ids[0], dists[0], counts[0], all_d, all_ids, 257, valid)
    # dimension mismatch on insert
    with pytest.raises(_lib.WvgError) as e:
        c.upsert(np.array([1], np.uint64), np.zeros((1, d + 1), np.float32))
    assert e.value.code == _lib.WVG_ERR_DIM_MISMATCH
    # get by id
    assert np.array_equal(bits(c.get(int(top[0]))), bits(rows[int(top[0])]))
    with pytest.raises(_lib.WvgError):
        c.get(int(top[1]))


def test_id_base_and_reserve(ctx, orc):
    n, d = 1000, 32
    rows = orc.synth_rows(31, 0, n, d, 0)
    q = orc.synth_rows(32, 0, 1, d, 0)[0]
    base = 64 * 1000
    c = Corpus(ctx, KIND_F32, METRIC_DOT, d, 128, id_base=base)
    c.reserve(n)  # grow keeps contents
    c.upsert(np.arange(base, base + 100, dtype=np.uint64), rows[:100])
    c.reserve(2 * n)
    c.upsert(np.arange(base + 100, base + n, dtype=np.uint64), rows[100:])
    ids, dists, counts = c.search(q, 20)
    all_d = orc.dist_all(1, q, rows)
    check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(base, base + n, dtype=np.uint64), 20)


def test_synthetic_fill_matches_oracle_generator(ctx, orc):
    for metric in [METRIC_L2, METRIC_COSINE]:
        c = Corpus(ctx, KIND_F32, metric, 100, 512)
        c.fill_synthetic(42, 300, 0)
        want = orc.synth_rows(42, 0, 300, 100, 0)
        if metric == METRIC_COSINE:
            want = orc.normalize_rows(want)
        for i in [0, 1, 63, 64, 299]:
            assert np.array_equal(bits(c.get(i)), bits(want[i]))


def test_multi_query_batch(ctx, orc):
    n, d, k, nq = 5000, 128, 10, 37
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.fill_synthetic(1, n, 0)
    rows = orc.synth_rows(1, 0, n, d, 0)
    qs = orc.synth_rows(2, 0, nq, d, 0)
    ids, dists, counts = c.search(qs, k)
    for qi in range(nq):
        check_topk(orc, ids[qi], dists[qi], counts[qi], orc.dist_all(0, qs[qi], rows),
                   np.arange(n, dtype=np.uint64), k)


# ---------------------------------------------------------------------------
# K3: batched dot / cosine on fp32 MFMA (nq >= 32 routes there by default)
@pytest.mark.parametrize("metric", [METRIC_DOT, METRIC_COSINE])
@pytest.mark.parametrize("d", [32, 96, 128, 160, 768])
def test_batched_mfma_parity(ctx, orc, metric, d):
    n, nq = 3000 + 29, 40  # ragged rows; 40 queries = one full and one partial 32-query block
    rows = orc.synth_rows(500 + d, 0, n, d, 0)
    qs = orc.synth_rows(501 + d, 0, nq, d, 0)
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    srows = stored_rows(orc, metric, rows)
    valid = np.ones(n, np.uint8)
    c.delete(np.array([3, 64, 65, 2000], np.uint64))
    valid[[3, 64, 65, 2000]] = 0
    for k in [1, 10, 100]:
        ids, dists, counts = c.search(qs, k)
        for qi in range(nq):
            all_d = orc.dist_all(ORC_METRIC[metric], prep_query(orc, metric, qs[qi]), srows)
            check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k, valid)


def test_batched_mfma_sift_like_ties_and_allow(ctx, orc):
    n, d, nq, k = 9000, 128, 33, 50
    rows = (orc.synth_rows(61, 0, n, d, 1) - 128.0).astype(np.float32)  # integers: exact dots, ties
    qs = (orc.synth_rows(62, 0, nq, d, 1) - 128.0).astype(np.float32)
    c = Corpus(ctx, KIND_F32, METRIC_DOT, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    allowed = np.arange(100, 7000, 3, dtype=np.uint64)
    am = np.zeros(n, np.uint8)
    am[allowed.astype(np.int64)] = 1
    ids, dists, counts = c.search(qs, k, allow_bitmap(allowed))
    for qi in range(nq):
        all_d = orc.dist_all(1, qs[qi], rows)
        check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k, am)


# ---------------------------------------------------------------------------
# BQ
def test_bq_encode_and_distance_bitexact(ctx, orc):
    from weaviate_amd.compressionhelpers import BinaryQuantizer

    bq = BinaryQuantizer(ctx)
    for d in [2, 63, 64, 65, 130, 1536]:
        X = orc.synth_rows(40 + d, 0, 200, d, 0)
        X[0, :] = -0.0
        codes = bq.EncodeBatch(X)
        want = np.stack([orc.bq_encode(r) for r in X])
        assert np.array_equal(codes, want)
        got = bq.DistanceBatch(codes[1], codes)
        assert np.array_equal(bits(got), bits(orc.bq_dist_all(want[1], want)))
    # known answers (CH/compression_test.go:44-60)
    c = bq.EncodeBatch(np.array([[-0.5, 0.5], [0.25, 0.7], [0.5, 0.5]], np.float32))
    assert bq.DistanceBetweenCompressedVectors(c[0], c[1])[0] == 1
    assert bq.DistanceBetweenCompressedVectors(c[0], c[2])[0] == 1
    assert bq.DistanceBetweenCompressedVectors(c[1], c[2])[0] == 0


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_COSINE])
@pytest.mark.parametrize("d", [128, 1536])
def test_bq_scan_parity(ctx, orc, metric, d):
    n = 3000 + 5
    rows = orc.synth_rows(300 + d, 0, n, d, 0)
    q = orc.synth_rows(301 + d, 0, 1, d, 0)[0]
    c = Corpus(ctx, KIND_BQ, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    srows = stored_rows(orc, metric, rows)
    codes = np.stack([orc.bq_encode(r) for r in srows])
    qc = orc.bq_encode(prep_query(orc, metric, q))
    all_d = orc.bq_dist_all(qc, codes)
    for k in [10, 200]:
        ids, dists, counts = c.search(q, k)
        check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), k)


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
def test_bq_rescore_flow(ctx, orc, metric):
    """flat.searchByVectorBQ: Hamming top-R then exact rescore (V/flat/index.go:347-389)."""
    n, d, k, rescore = 6000, 256, 10, 200
    rows = orc.synth_rows(55, 0, n, d, 0)
    q = orc.synth_rows(56, 0, 1, d, 0)[0]
    f = Corpus(ctx, KIND_F32, metric, d, n)
    b = Corpus(ctx, KIND_BQ, metric, d, n)
    f.upsert(np.arange(n, dtype=np.uint64), rows)
    b.upsert(np.arange(n, dtype=np.uint64), rows)
    ids, dists, counts = search_bq_rescore(b, f, q, k, rescore)
    srows = stored_rows(orc, metric, rows)
    qn = prep_query(orc, metric, q)
    # the reference flow restated (its Hamming heap, pop order, k-heap): ids and bits equal
    ri, rd = orc.flat_search_bq(srows, qn, k, rescore, ORC_METRIC[metric])
    assert counts[0] == k == len(ri)
    assert np.array_equal(ids[0], ri) and np.array_equal(bits(dists[0]), bits(rd))


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
def test_rescore_host_rows(ctx, orc, metric):
    """wvg_rescore == exact SingleDist over host-fetched candidate rows, inserted
    into a heap of k in input order (the reference inserts in its pop order,
    V/flat/index.go:375-387) -- the heap oracle exactly, ties included."""
    import ctypes

    lib = _lib.load()
    n, d, k = 500, 1536, 10
    rows = orc.synth_rows(71, 0, n, d, 0)
    q = orc.synth_rows(72, 0, 1, d, 0)[0]
    if metric == METRIC_COSINE:
        rows, q = orc.normalize_rows(rows), orc.normalize(q)
    rows[7] = rows[3]  # an exact tie
    ids = (1000 + 3 * np.arange(n)[::-1]).astype(np.uint64)
    oi = np.empty(k, np.uint64)
    od = np.empty(k, np.float32)
    cnt = ctypes.c_uint32()
    _lib.check(lib.wvg_rescore(ctx.handle, metric, _lib.fptr(q), _lib.fptr(rows), _lib.u64ptr(ids), n, d, k,
                               _lib.u64ptr(oi), _lib.fptr(od), ctypes.byref(cnt)))
    all_d = orc.dist_all(ORC_METRIC[metric], q, rows)
    hi, hd = orc.heap_topk(all_d, ids, k)
    assert cnt.value == k
    assert np.array_equal(oi, hi) and np.array_equal(bits(od), bits(hd))


@pytest.mark.parametrize("d", [96, 1, 65, 1536])
def test_synthetic_rows_helper(ctx, orc, d):
    lib = _lib.load()
    ids = np.array([5, 0, 999_999, 123_456_789, 7, 8, 9], np.uint64)  # 7 rows: two workgroups of 4 waves
    for norm in [0, 1]:
        out = np.empty((len(ids), d), np.float32)
        _lib.check(lib.wvg_synthetic_rows(ctx.handle, 42, _lib.u64ptr(ids), len(ids), d, 0, norm, _lib.fptr(out)))
        want = np.stack([orc.synth_rows(42, int(i), 1, d, 0)[0] for i in ids])
        if norm:
            want = orc.normalize_rows(want)
        assert np.array_equal(bits(out), bits(want))


# ---------------------------------------------------------------------------
# PQ
def _codebook(orc, m, ks, ds, seed):
    return orc.synth_rows(seed, 0, m * ks, ds, 0).reshape(m, ks, ds)


@pytest.mark.parametrize("m,ks,d", [(32, 256, 128), (8, 16, 24), (16, 256, 256), (32, 16, 128), (32, 24, 128),
                                     (16, 6, 64)])
def test_pq_encode_lut_adc_bitexact(ctx, orc, m, ks, d):
    from weaviate_amd.compressionhelpers import ProductQuantizer

    centers = _codebook(orc, m, ks, d // m, 900 + m)
    X = orc.synth_rows(901, 0, 500, d, 0)
    X[:5] = centers[np.arange(m)[None, :], np.array([[1] * m] * 5)].reshape(5, d)  # exact hits
    pq = ProductQuantizer(ctx, centers)
    codes = pq.EncodeBatch(X)
    assert np.array_equal(codes, orc.pq_encode(X, centers))
    for metric, name in [(0, "l2-squared"), (1, "dot")]:
        pqm = ProductQuantizer(ctx, centers, name)
        lut = pqm.CenterAt(X[7])
        assert np.array_equal(bits(lut), bits(orc.pq_lut(metric, X[7], centers)))
        got = pqm.NewDistancer(X[7]).DistanceBatch(codes)
        want = [orc.pq_adc(metric, lut, cd) for cd in codes]
        assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT])
def test_pq_scan_parity(ctx, orc, metric):
    m, ks, d, n = 32, 256, 128, 5000
    centers = _codebook(orc, m, ks, d // m, 77)
    rows = orc.synth_rows(78, 0, n, d, 0)
    q = orc.synth_rows(79, 0, 1, d, 0)[0]
    c = Corpus(ctx, KIND_PQ, metric, d, n)
    c.set_codebook(centers)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    codes = orc.pq_encode(rows, centers)
    assert np.array_equal(c.get(17, pq_m=m), codes[17])
    lut = orc.pq_lut(ORC_METRIC[metric], q, centers)
    all_d = np.array([orc.pq_adc(ORC_METRIC[metric], lut, cd) for cd in codes], np.float32)
    for k in [10, 100]:
        ids, dists, counts = c.search(q, k)
        check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), k)
    # restart path: load codes as stored (V/flat/index.go:640-681 analogue)
    c2 = Corpus(ctx, KIND_PQ, metric, d, n)
    c2.set_codebook(centers)
    c2.upsert_codes(np.arange(n, dtype=np.uint64), codes)
    ids2, dists2, _ = c2.search(q, 10)
    ids1, dists1, _ = c.search(q, 10)
    assert np.array_equal(ids1, ids2)


def test_pq_encode_argmin_ties_and_nonfinite(ctx, orc):
    """nNearest's rule (CH/kmeans.go:126-130: replace on !(minD < d)) on both
    encoder paths -- the min3 pair argmin (NaN-free codebooks) and the
    reference's compare-and-select loop (a codebook holding a NaN, or a row
    with NaN in the segment): exact ties inside a centroid pair and across
    pairs go to the highest index, rows with NaN take the reference loop, rows
    whose every distance overflows to +inf keep centroid 0."""
    from weaviate_amd.compressionhelpers import ProductQuantizer

    m, ks, d = 32, 256, 128
    centers = _codebook(orc, m, ks, d // m, 910)
    centers[:, 9] = centers[:, 8]      # a tie inside pair 4
    centers[:, 201] = centers[:, 8]    # ... and with a later pair
    centers[:, 130] = centers[:, 131]  # a tie inside pair 65 only
    centers[:, 16] = centers[:, 15]    # ties across the first two 16-centroid argmin groups
    centers[:, 30] = centers[:, 15]    # ... and inside the second group (30 wins)
    X = orc.synth_rows(911, 0, 700, d, 0)
    X[:4] = centers[np.arange(m)[None, :], np.array([[8] * m] * 4)].reshape(4, d)   # d = 0 at 8, 9, 201
    X[4:8] = centers[np.arange(m)[None, :], np.array([[131] * m] * 4)].reshape(4, d)  # d = 0 at 130, 131
    X[11:14] = centers[np.arange(m)[None, :], np.array([[15] * m] * 3)].reshape(3, d)  # d = 0 at 15, 16, 30
    X[8, 5] = np.nan                   # segment 1 of row 8: NaN distances
    X[70, 127] = np.nan                # a NaN in the second wave of the batch
    X[9, 12:16] = np.float32(3e38)     # segment 3: every distance overflows to +inf
    X[10, 0:4] = np.inf                # segment 0: +inf distances
    for cb in (centers, None):
        if cb is None:  # NaN in the codebook: the pair path must not use min3 (the loop sees the same ties)
            cb = centers.copy()
            cb[2, 17, 1] = np.nan
        want = orc.pq_encode(X, cb)
        pq = ProductQuantizer(ctx, cb)
        assert np.array_equal(pq.EncodeBatch(X), want)
        c = Corpus(ctx, KIND_PQ, METRIC_L2, d, len(X))
        c.set_codebook(cb)
        c.upsert(np.arange(len(X), dtype=np.uint64), X)
        got = c.get_batch(np.arange(len(X), dtype=np.uint64), pq_m=m)[0]
        assert np.array_equal(got, want)
        c.destroy()


def test_pq_encode_corpus(ctx, orc):
    """Bulk compression of a resident float corpus == per-row Encode."""
    lib = _lib.load()
    m, ks, d, n = 32, 256, 128, 3000
    centers = _codebook(orc, m, ks, d // m, 81)
    f = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    f.fill_synthetic(82, n, 0)
    f.delete(np.array([5, 6], np.uint64))
    pq = Corpus(ctx, KIND_PQ, METRIC_L2, d, n)
    pq.set_codebook(centers)
    _lib.check(lib.wvg_pq_encode_corpus(pq.handle, f.handle))
    rows = orc.synth_rows(82, 0, n, d, 0)
    codes = orc.pq_encode(rows, centers)
    for i in [0, 1, 63, 64, 2999]:
        assert np.array_equal(pq.get(i, pq_m=m), codes[i])
    assert pq.info()[0] == n - 2
    q = orc.synth_rows(83, 0, 1, d, 0)[0]
    lut = orc.pq_lut(0, q, centers)
    all_d = np.array([orc.pq_adc(0, lut, cd) for cd in codes], np.float32)
    valid = np.ones(n, np.uint8)
    valid[[5, 6]] = 0
    ids, dists, counts = pq.search(q, 10)
    check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), 10, valid)


def test_pq_invalid_config(ctx):
    c = Corpus(ctx, KIND_PQ, METRIC_L2, 128, 64)
    with pytest.raises(_lib.WvgError, match="segments should be an integer divisor"):
        c.set_codebook(np.zeros((3, 4, 42), np.float32))
    with pytest.raises(_lib.WvgError, match="centroids should not be higher than 256"):
        c.set_codebook(np.zeros((4, 257, 32), np.float32))


# ---------------------------------------------------------------------------
# Multi-shard merge (device) -- the RCCL all-gather's consumer
def test_topk_merge_device(ctx, orc):
    import torch

    dev = torch.device("cuda:0")
    G, nq, k = 8, 5, 100
    rng = np.random.default_rng(9)
    d = np.floor(rng.uniform(0, 50, (G, nq, k))).astype(np.float32)  # ties across shards
    ids = rng.permutation(G * nq * k).reshape(G, nq, k).astype(np.uint64)
    ids[0, 0, :3] = np.iinfo(np.uint64).max  # missing entries (short shard)
    td = torch.from_numpy(d).to(dev)
    ti = torch.from_numpy(ids.view(np.int64)).to(dev)
    oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
    od = torch.empty((nq, k), dtype=torch.float32, device=dev)
    oc = torch.empty(nq, dtype=torch.int32, device=dev)
    lib = _lib.load()
    _lib.check(lib.wvg_topk_merge_device(ctx.handle, td.data_ptr(), ti.data_ptr(), nq, G, k, k, oi.data_ptr(),
                                         od.data_ptr(), oc.data_ptr(), None))
    torch.cuda.synchronize()
    oi = oi.cpu().numpy().view(np.uint64)
    od = od.cpu().numpy()
    for qi in range(nq):
        live = ids[:, qi, :] != np.iinfo(np.uint64).max
        wi, wd = orc.lex_topk(d[:, qi, :][live], ids[:, qi, :][live], k)
        assert np.array_equal(oi[qi], wi) and np.array_equal(bits(od[qi]), bits(wd))


def test_search_device_matches_host_api(ctx, orc):
    """Device API; one workspace reused by many calls."""
    import torch

    n, d, k = 20000, 128, 10
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.fill_synthetic(3, n, 0)
    lib = _lib.load()
    dev = torch.device("cuda:0")
    for nq in [4, 1, 3]:
        ws = torch.zeros(lib.wvg_search_workspace_size(c.handle, nq, k), dtype=torch.uint8, device=dev)
        for rep in range(3):
            qs = orc.synth_rows(4 + rep, 0, nq, d, 0)
            hid, hd, hc = c.search(qs, k)
            tq = torch.from_numpy(qs).to(dev)
            oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
            od = torch.empty((nq, k), dtype=torch.float32, device=dev)
            oc = torch.empty(nq, dtype=torch.int32, device=dev)
            _lib.check(lib.wvg_search_device(c.handle, tq.data_ptr(), nq, k, oi.data_ptr(), od.data_ptr(),
                                             oc.data_ptr(), ws.data_ptr(), ws.numel(),
                                             torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            assert np.array_equal(oi.cpu().numpy().view(np.uint64), hid)
            assert np.array_equal(bits(od.cpu().numpy()), bits(hd))
            assert np.array_equal(oc.cpu().numpy(), hc.astype(np.int32))


def test_search_device_pipelined_matches_host_api(ctx, orc):
    """nq single-query scans in one query-stream launch (the merge workgroup
    merges each query while the scan moves on) == the host API."""
    import torch

    n, d = 30000 + 7, 128
    lib = _lib.load()
    dev = torch.device("cuda:0")
    for metric in [METRIC_L2, METRIC_DOT]:
        c = Corpus(ctx, KIND_F32, metric, d, n)
        c.fill_synthetic(5, n, 0)
        c.delete(np.array([0, 1, 77, 30000], np.uint64))
        for nq, k in [(1, 10), (2, 10), (5, 100), (16, 10), (3, 256)]:
            ws = torch.zeros(lib.wvg_search_workspace_size(c.handle, nq, k), dtype=torch.uint8, device=dev)
            outs = []
            for rep in range(2):  # two calls back to back on one workspace, no sync between them
                qs = orc.synth_rows(9 + nq + 100 * rep, 0, nq, d, 0)
                tq = torch.from_numpy(qs).to(dev)
                oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
                od = torch.empty((nq, k), dtype=torch.float32, device=dev)
                oc = torch.empty(nq, dtype=torch.int32, device=dev)
                _lib.check(lib.wvg_search_device_pipelined(c.handle, tq.data_ptr(), nq, k, oi.data_ptr(),
                                                           od.data_ptr(), oc.data_ptr(), ws.data_ptr(),
                                                           ws.numel(), torch.cuda.current_stream().cuda_stream))
                outs.append((qs, tq, oi, od, oc))
            torch.cuda.synchronize()
            for qs, _, oi, od, oc in outs:
                hid, hd, hc = c.search(qs, k)  # host API (nq concurrent scans in one launch)
                assert np.array_equal(oi.cpu().numpy().view(np.uint64), hid)
                assert np.array_equal(bits(od.cpu().numpy()), bits(hd))
                assert np.array_equal(oc.cpu().numpy(), hc.astype(np.int32))
        c.destroy()


@pytest.mark.parametrize("screen", [0, 1])
@pytest.mark.parametrize("metric,d", [(METRIC_COSINE, 768), (METRIC_DOT, 256), (METRIC_COSINE, 1536), (METRIC_DOT, 512),
                                      (METRIC_DOT, 128), (METRIC_COSINE, 96)])
def test_batched_mfma_variants(ctx, orc, screen, metric, d):
    """Batched dot / cosine on the matrix cores against the oracle: ragged
    rows, deletes, an allow list, partial query blocks, SIFT-like ties.
    screen 0: the exact fp32 MFMA kernels -- K3b (queries resident in LDS,
    rows streamed into MFMA operands) for k <= 64 and d in {256 .. 1536}, K3
    otherwise (k = 100, d = 128 / 96); screen 1: the context default, where
    the bf16 screen + exact rescore takes the batches it applies to."""
    from weaviate_amd.device import Context

    cx = ctx if screen else Context(0, batch_screen=0)
    try:
        n, nq = 4000 + 45, 70
        rows = orc.synth_rows(700 + d, 0, n, d, 0)
        qs = orc.synth_rows(701 + d, 0, nq, d, 0)
        if metric == METRIC_DOT:  # integer values: exact dots and many ties
            rows = np.floor(rows * 3).astype(np.float32)
            qs = np.floor(qs * 3).astype(np.float32)
        c = Corpus(cx, KIND_F32, metric, d, n)
        c.upsert(np.arange(n, dtype=np.uint64), rows)
        srows = stored_rows(orc, metric, rows)
        valid = np.ones(n, np.uint8)
        dead = [0, 63, 64, 1000, 4044]
        c.delete(np.array(dead, np.uint64))
        valid[dead] = 0
        allowed = np.arange(5, 3900, 2, dtype=np.uint64)
        am = np.zeros(n, np.uint8)
        am[allowed.astype(np.int64)] = 1
        for k, allow in [(1, None), (10, None), (64, None), (10, allowed), (100, None)]:
            ids, dists, counts = c.search(qs, k, None if allow is None else allow_bitmap(allow))
            vm = valid if allow is None else valid & am
            for qi in range(0, nq, 3):
                all_d = orc.dist_all(ORC_METRIC[metric], prep_query(orc, metric, qs[qi]), srows)
                check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k, vm)
        c.destroy()
    finally:
        if cx is not ctx:
            cx.close()



@pytest.mark.parametrize("screen", [0, 1])
def test_batched_mfma_nonfinite_zero_and_ranges(ctx, orc, screen):
    """The batched kernels' float-distance rejection (!(dist > tau) before any
    key is built) against the oracle on rows that give NaN, +-inf, -0.0 and
    +0.0 dot products and exact ties; 94 tiles over 94 row ranges, so lists
    restart often and the K2 merge sees many partial lists.  screen 0: exact
    fp32 MFMA only; 1: the bf16 screen, whose error bound is infinite for the
    non-finite rows (always rescored exactly)."""
    from weaviate_amd.device import Context

    def check_lex(orc, ids, dists, count, all_d, k, valid):  # NaN sorts last (no heap comparison with NaN rows)
        sel = valid.astype(bool)
        li, ld = orc.lex_topk(all_d[sel], np.arange(len(all_d), dtype=np.uint64)[sel], k)
        assert count == len(li) and np.array_equal(ids[:count], li)
        assert np.array_equal(bits(dists[:count]), bits(ld))

    cx = ctx if screen else Context(0, batch_screen=0)
    try:
        n, nq, d = 6000 + 13, 48, 256
        rows = np.floor(orc.synth_rows(900, 0, n, d, 0) * 2).astype(np.float32)
        qs = np.floor(orc.synth_rows(901, 0, nq, d, 0) * 2).astype(np.float32)
        rows[100, 5] = np.nan
        rows[200, 7] = np.inf
        rows[300, 9] = -np.inf
        rows[[400, 401, 5000]] = 0.0        # dot = +0 -> dist -0 under DOT
        rows[402] = -0.0
        rows[[403, 404]] = rows[405]        # exact ties
        qs[3, 5] = 0.0
        c = Corpus(cx, KIND_F32, METRIC_DOT, d, n)
        c.upsert(np.arange(n, dtype=np.uint64), rows)
        valid = np.ones(n, np.uint8)
        c.delete(np.array([64, 3000], np.uint64))
        valid[[64, 3000]] = 0
        for k in (1, 10, 64):
            ids, dists, counts = c.search(qs, k)
            for qi in range(nq):
                all_d = orc.dist_all(1, qs[qi], rows)
                check_lex(orc, ids[qi], dists[qi], counts[qi], all_d, k, valid)
        # large-positive query: NaN / -inf rows rank first and last
        q = np.full((40, d), 1.0, np.float32)
        ids, dists, counts = c.search(q, 10)
        all_d = orc.dist_all(1, q[0], rows)
        check_lex(orc, ids[0], dists[0], counts[0], all_d, 10, valid)
        c.destroy()
    finally:
        if cx is not ctx:
            cx.close()


@pytest.mark.parametrize("reuse", [0, 1])
def test_flat_scan_load_policies(ctx, orc, reuse):
    """K1's row loads: the default context (reuse 1: default-policy loads at
    this size, alternating directions) and a streaming context
    (wvg_options.cache_reuse = 0: non-temporal loads, one direction), through
    the host search and the query-stream device search: same bits as the
    oracle."""
    import torch

    from weaviate_amd.device import Context

    lib = _lib.load()
    cx = ctx if reuse else Context(0, cache_reuse=0)
    try:
        n, d, k, nq = 20_000 + 7, 128, 10, 5
        c = Corpus(cx, KIND_F32, METRIC_L2, d, n)
        c.fill_synthetic(71, n, 0)
        c.delete(np.array([3, 640], np.uint64))
        valid = np.ones(n, np.uint8)
        valid[[3, 640]] = 0
        rows = orc.synth_rows(71, 0, n, d, 0)
        qs = orc.synth_rows(72, 0, nq, d, 0)
        ids, dists, counts = c.search(qs, k)
        dev = torch.device("cuda:0")
        ws = torch.zeros(lib.wvg_search_workspace_size(c.handle, nq, k), dtype=torch.uint8, device=dev)
        tq = torch.from_numpy(qs).to(dev)
        oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
        od = torch.empty((nq, k), dtype=torch.float32, device=dev)
        oc = torch.empty(nq, dtype=torch.int32, device=dev)
        _lib.check(lib.wvg_search_device_pipelined(c.handle, tq.data_ptr(), nq, k, oi.data_ptr(), od.data_ptr(),
                                                   oc.data_ptr(), ws.data_ptr(), ws.numel(),
                                                   torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        assert np.array_equal(oi.cpu().numpy().view(np.uint64), ids)
        for qi in range(nq):
            all_d = orc.dist_all(orc.L2, qs[qi], rows)
            check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k, valid)
        c.destroy()
    finally:
        if cx is not ctx:
            cx.close()
