"""GPU parity for the "manhattan" and "hamming" distances of the vector index
config (entities/vectorindex/common/config.go:26-27; picked by name in
adapters/repos/db/shard.go:406-421 and handed to the flat index like the
others).  Every path that takes a metric runs them: the flat scan (K1, fixed
and generic dimensions, allow lists, deletes), batched queries (K1: the MFMA
kernel is dot / cosine only), the query-stream device search, the unbounded
selection (k > 256) and range search, BQ rescoring, DistanceToNode, the
distance batch and the PQ lookup table / ADC scan / SDC table (their Step is
the pure-Go loop).

Oracle: manhattan is the pure-Go loop (D/manhattan.go:20-30); hamming is the
reference's own hamming_256 (D/c/hamming_avx256_amd64.c), whose outputs are
pinned in tests/golden/hamming.npz.  Bit-exact throughout.
"""
import os

import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_BQ, KIND_F32, KIND_PQ, METRIC_HAMMING, METRIC_MANHATTAN
from weaviate_amd.device import Corpus, allow_bitmap, search_bq_rescore

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ORC = {METRIC_MANHATTAN: 3, METRIC_HAMMING: 4}
METRICS = [METRIC_MANHATTAN, METRIC_HAMMING]


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def _rows(orc, metric, seed, n, d):
    """Hamming wants repeated values (equal elements are what it counts):
    integers 0..3; manhattan the uniform [-1, 1) rows."""
    if metric == METRIC_HAMMING:
        return np.floor(orc.synth_rows(seed, 0, n, d, 1) / 64).astype(np.float32)
    return orc.synth_rows(seed, 0, n, d, 0)


def check_topk(orc, ids, dists, count, all_d, all_ids, k, valid=None):
    sel = np.ones(len(all_d), bool) if valid is None else valid.astype(bool)
    li, ld = orc.lex_topk(all_d[sel], all_ids[sel], k)
    assert count == len(li)
    assert np.array_equal(ids[:count], li)
    assert np.array_equal(bits(dists[:count]), bits(ld))


def _pairs(g):
    off = 0
    for n in g["lens"]:
        yield g["a"][off:off + n], g["b"][off:off + n]
        off += n


def test_distance_batch_vs_reference_kernels(ctx, orc):
    """HammingProvider on the GPU == the reference's hamming_256 outputs
    (NaN in blocks and tails, signed zeros, lengths 1..1536); ManhattanProvider
    == the Go loop on the same pairs and on the float golden pairs."""
    from weaviate_amd.distancer import HammingProvider, ManhattanProvider

    hp, mp = HammingProvider(ctx), ManhattanProvider(ctx)
    g = np.load(os.path.join(GOLDEN, "hamming.npz"))
    got = [hp.BatchDist(a, b[None])[0] for a, b in _pairs(g)]
    assert np.array_equal(bits(got), bits(g["hamming_256"]))
    f = np.load(os.path.join(GOLDEN, "distances.npz"))
    for src in (g, f):
        got = [mp.BatchDist(a, b[None])[0] for a, b in _pairs(src)]
        want = [orc.manhattan(a, b) for a, b in _pairs(src)]
        assert np.array_equal(bits(got), bits(want))


def test_known_answers_and_provider_names(ctx):
    """D/manhattan_test.go:21-68, D/hamming_test.go:23-82; Type() names and
    the shard's by-name selection with its error text."""
    from weaviate_amd.distancer import HammingProvider, ManhattanProvider, provider_for

    mp, hp = ManhattanProvider(ctx), HammingProvider(ctx)
    assert mp.SingleDist([3, 4, 5], [3, 4, 5])[0] == 0
    assert mp.SingleDist([3, 4, 5], [1.5, 2, 2.5])[0] == 6
    assert mp.SingleDist([10, 11], [13, 15])[0] == 7
    assert hp.SingleDist([3, 4, 5], [1.5, 2, 2.5])[0] == 3
    assert hp.SingleDist([10, 11], [10, 15])[0] == 1
    assert hp.SingleDist([10, 11, 15, 25, 31], [10, 15, 16, 25, 30])[0] == 3
    # Step by step (D/manhattan_test.go:70-90, D/hamming_test.go:85-103)
    a, b = [10, 11, 15, 25, 31], [10, 15, 16, 25, 30]
    assert sum(np.float32(hp.Step([x], [y])) for x, y in zip(a, b)) == 3
    assert sum(np.float32(mp.Step([x], [y])) for x, y in zip([3, 4, 5], [1.5, 2, 2.5])) == 6
    d, ok, err = hp.SingleDist([1, 2], [1, 2, 3])
    assert not ok and err == "vector lengths don't match: 2 vs 3"
    assert mp.Type() == "manhattan" and hp.Type() == "hamming"
    assert provider_for(ctx, "manhattan").Type() == "manhattan"
    assert provider_for(ctx, "").Type() == "cosine-dot"
    with pytest.raises(ValueError, match='unrecognized distance metric "foo"'):
        provider_for(ctx, "foo")


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("d", [3, 37, 128, 200, 768])
def test_flat_search_parity(ctx, orc, metric, d):
    n = 3000 + 17
    rows = _rows(orc, metric, 500 + d, n, d)
    qs = _rows(orc, metric, 600 + d, 3, d)
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    for k in [1, 10, 100, 256]:
        ids, dists, counts = c.search(qs, k)
        for qi in range(len(qs)):
            all_d = orc.dist_all(ORC[metric], qs[qi], rows)
            check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k)
    c.destroy()


def test_hamming_nan_rows(ctx, orc):
    """NaNs in stored rows and the query, in the SIMD blocks and in the
    scalar tail (d = 37: elements 32..36 are the tail), where hamming_256
    counts them differently."""
    n, d = 700, 37
    rows = _rows(orc, METRIC_HAMMING, 31, n, d)
    rng = np.random.default_rng(3)
    for r in range(0, n, 3):
        rows[r, rng.integers(0, d)] = np.nan
    q = _rows(orc, METRIC_HAMMING, 32, 1, d)[0]
    q[[1, 33]] = np.nan
    c = Corpus(ctx, KIND_F32, METRIC_HAMMING, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    all_d = orc.dist_all(4, q, rows)
    assert len(set(all_d.tolist())) > 5
    for k in [10, 300]:
        ids, dists, counts = c.search(q, k)
        check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), k)


@pytest.mark.parametrize("metric", METRICS)
def test_deletes_allow_list_and_order512(ctx, orc, metric):
    n, d, k = 2500, 64, 10
    rows = _rows(orc, metric, 41, n, d)
    q = _rows(orc, metric, 42, 1, d)[0]
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    dead = np.arange(0, n, 7, dtype=np.uint64)
    c.delete(dead)
    valid = np.ones(n, bool)
    valid[dead.astype(np.int64)] = False
    all_d = orc.dist_all(ORC[metric], q, rows)
    ids, dists, counts = c.search(q, k)
    check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), k, valid)
    allow_ids = np.arange(100, 1900, 5, dtype=np.uint64)
    am = np.zeros(n, bool)
    am[allow_ids.astype(np.int64)] = True
    ids, dists, counts = c.search(q, k, allow_bitmap(allow_ids, n))
    check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), k, valid & am)
    # AVX-512 hosts: manhattan has no SIMD kernel, hamming_512 counts alike -> same results
    ctx.set_distance_order(1)
    try:
        ids2, dists2, _ = c.search(q, k)
    finally:
        ctx.set_distance_order(0)
    ids1, dists1, _ = c.search(q, k)
    assert np.array_equal(ids1, ids2) and np.array_equal(bits(dists1), bits(dists2))
    c.destroy()


@pytest.mark.parametrize("metric", METRICS)
def test_batched_queries_and_device_stream(ctx, orc, metric):
    """48 queries in one wvg_search (the batched MFMA kernel is not used for
    these metrics) and the query-stream device search at d = 128."""
    import torch

    n, d, k = 5000 + 3, 128, 10
    rows = _rows(orc, metric, 51, n, d)
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    qs = _rows(orc, metric, 52, 48, d)
    ids, dists, counts = c.search(qs, k)
    for qi in range(0, 48, 7):
        all_d = orc.dist_all(ORC[metric], qs[qi], rows)
        check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k)
    lib = _lib.load()
    dev = torch.device("cuda:0")
    nq = 16
    ws = torch.zeros(lib.wvg_search_workspace_size(c.handle, nq, k), dtype=torch.uint8, device=dev)
    tq = torch.from_numpy(np.ascontiguousarray(qs[:nq])).to(dev)
    oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
    od = torch.empty((nq, k), dtype=torch.float32, device=dev)
    oc = torch.empty(nq, dtype=torch.int32, device=dev)
    _lib.check(lib.wvg_search_device_pipelined(c.handle, tq.data_ptr(), nq, k, oi.data_ptr(), od.data_ptr(),
                                               oc.data_ptr(), ws.data_ptr(), ws.numel(),
                                               torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert np.array_equal(oi.cpu().numpy().view(np.uint64), ids[:nq])
    assert np.array_equal(bits(od.cpu().numpy()), bits(dists[:nq]))
    c.destroy()


@pytest.mark.parametrize("metric", METRICS)
def test_unbounded_selection_and_range_search(ctx, orc, metric):
    """k > 256 (radix select; hamming has huge ties) and SearchByVectorDistance
    in both callers' semantics."""
    n, d = 6000, 24
    rows = _rows(orc, metric, 61, n, d)
    q = _rows(orc, metric, 62, 1, d)[0]
    c = Corpus(ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    all_d = orc.dist_all(ORC[metric], q, rows)
    all_ids = np.arange(n, dtype=np.uint64)
    for k in [300, 1000]:
        ids, dists, counts = c.search(q, k)
        check_topk(orc, ids[0], dists[0], counts[0], all_d, all_ids, k)
    target = float(np.sort(all_d)[250])

    def search_fn(total):
        return orc.lex_topk(all_d, all_ids, total)

    wi, wd = orc.search_by_distance(search_fn, target, -1)
    gi, gd = c.search_by_distance(q, target, -1)
    assert np.array_equal(gi, wi) and np.array_equal(bits(gd), bits(wd))
    fi, fd, _ = orc.search_by_distance_flat(search_fn, target, -1, max_iterations=3)
    gi, gd = c.search_by_distance_window(q, target)
    assert np.array_equal(gi, fi) and np.array_equal(bits(gd), bits(fd))
    c.destroy()


@pytest.mark.parametrize("metric", METRICS)
def test_bq_rescore_and_distance_to_node(ctx, orc, metric):
    """flat.searchByVectorBQ with these metrics (Hamming-bit top-R, exact
    rescore with the metric) and DistanceToNode by docID."""
    n, d, k, rescore = 4000, 256, 10, 200
    rows = orc.synth_rows(71, 0, n, d, 0)
    q = orc.synth_rows(72, 0, 1, d, 0)[0]
    f = Corpus(ctx, KIND_F32, metric, d, n)
    b = Corpus(ctx, KIND_BQ, metric, d, n)
    f.upsert(np.arange(n, dtype=np.uint64), rows)
    b.upsert(np.arange(n, dtype=np.uint64), rows)
    ids, dists, counts = search_bq_rescore(b, f, q, k, rescore)
    codes = np.stack([orc.bq_encode(r) for r in rows])
    # the reference flow: Hamming heap, pop order, exact distances into a k-heap in that order
    cand, _ = orc.bq_heap_pops(codes, orc.bq_encode(q), rescore)
    exact = orc.dist_all(ORC[metric], q, rows[cand.astype(np.int64)])
    li, ld = orc.heap_topk(exact, cand, k)
    assert counts[0] == k
    assert np.array_equal(ids[0], li) and np.array_equal(bits(dists[0]), bits(ld))
    probe = np.array([0, 5, 63, 64, 3999, 4000], np.uint64)
    f.delete(np.array([5], np.uint64))
    dd, ok = f.distance_by_ids(q, probe)
    assert ok.tolist() == [True, False, True, True, True, False]
    want = orc.dist_all(ORC[metric], q, rows[[0, 63, 64, 3999]])
    assert np.array_equal(bits(dd[ok]), bits(want))
    f.destroy()
    b.destroy()


@pytest.mark.parametrize("metric_name,metric", [("manhattan", METRIC_MANHATTAN), ("hamming", METRIC_HAMMING)])
def test_pq_lut_adc_scan_and_sdc(ctx, orc, metric_name, metric):
    """PQ with these metrics: LUT[i][c] = Step(q_i, C_i[c]) in the pure-Go
    loop (hamming: Go's !=), the ADC sum, the K8c / K8b scans (m = 32) and
    the SDC table (CH/product_quantization.go:62-104, 236-311)."""
    from weaviate_amd.compressionhelpers import ProductQuantizer

    m, ks, d, n = 32, 256, 128, 5000
    centers = np.floor(orc.synth_rows(81, 0, m * ks, d // m, 1) / 64).astype(np.float32).reshape(m, ks, d // m) \
        if metric == METRIC_HAMMING else orc.synth_rows(81, 0, m * ks, d // m, 0).reshape(m, ks, d // m)
    rows = _rows(orc, metric, 82, n, d)
    q = _rows(orc, metric, 83, 1, d)[0]
    if metric == METRIC_HAMMING:
        q[5] = np.nan  # Step counts a NaN (Go's !=)
    pq = ProductQuantizer(ctx, centers, metric_name)
    lut = pq.CenterAt(q)
    assert np.array_equal(bits(lut), bits(orc.pq_lut(ORC[metric], q, centers)))
    codes = orc.pq_encode(rows, centers)
    all_d = np.array([orc.pq_adc(ORC[metric], lut, cd) for cd in codes], np.float32)
    assert np.array_equal(bits(pq.NewDistancer(q).DistanceBatch(codes)), bits(all_d))
    c = Corpus(ctx, KIND_PQ, metric, d, n)
    c.set_codebook(centers)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    for k in [10, 100]:
        ids, dists, counts = c.search(q, k)  # K8c (dense)
        check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), k)
    allow_ids = np.arange(0, n, 3, dtype=np.uint64)
    am = np.zeros(n, bool)
    am[allow_ids.astype(np.int64)] = True
    ids, dists, counts = c.search(q, 10, allow_bitmap(allow_ids, n))  # K8b (allow list)
    check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), 10, am)
    tab = pq.globalDistances()
    assert np.array_equal(bits(tab), bits(orc.pq_global_distances(ORC[metric], centers)))
    got = pq.SDCBatch(codes[0], codes[:300])
    want = [orc.pq_sdc(ORC[metric], tab, codes[0], cd) for cd in codes[:300]]
    assert np.array_equal(bits(got), bits(want))
    c.destroy()
