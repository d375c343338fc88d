"""Ports of the reference's own tests for this path, run through the C ABI:

* Test_NoRaceFlatIndex (V/flat/index_test.go:150-230, `run` :48-137): 12k x 256
  normalized cosine vectors, 100 queries, k = 10; no compression and BQ with
  RescoreLimit = 100 * k; plain, with 5k added-then-deleted vectors, filtered
  to ids [0, 3000), filtered with deletes; queries issued concurrently
  (compressionhelpers.Concurrently) and checked for duplicates.  Recall
  targets as the reference (> 0.99 none, > 0.8 BQ); without compression we
  also require the exact top-k.
* TestBinaryQuantizerRecall (CH/binary_quantization_test.go:31-84): 10k x 1536
  normalized vectors, the true top-10 must be in the Hamming top-200 with
  recall > 0.7.
* A concurrency test in the spirit of the `NoRace` suites: searches from many
  threads while a writer adds and deletes rows on the same corpus.

The reference draws its vectors from Go's math/rand (an unseeded stream,
testinghelpers/helpers.go:111-133: r.Float32()*2-1); here numpy draws the same
distribution from a fixed seed.  Ground truth comes from the oracle."""
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from weaviate_amd._lib import KIND_BQ, KIND_F32, METRIC_COSINE, METRIC_L2
from weaviate_amd.compressionhelpers import BinaryQuantizer
from weaviate_amd.device import Corpus, allow_bitmap
from weaviate_amd.flat import AllowList, FlatIndex

pytestmark = pytest.mark.gpu


def random_vecs(rng, n, d):
    return (rng.random((n, d), dtype=np.float32) * 2 - 1).astype(np.float32)


def matches(truth, results):
    return len(set(int(x) for x in truth) & set(int(x) for x in results))


@pytest.fixture(scope="module")
def flat_data(orc):
    rng = np.random.default_rng(150)
    vectors = orc.normalize_rows(random_vecs(rng, 12_000, 256))
    queries = orc.normalize_rows(random_vecs(rng, 100, 256))
    extra = random_vecs(rng, 5_000, 256)
    return vectors, queries, extra


def _truths(orc, vectors, queries, k):
    ids = np.arange(len(vectors), dtype=np.uint64)
    return [orc.lex_topk(orc.dist_all(2, q, vectors), ids, k)[0] for q in queries]


def _run(ctx, compression, vectors, queries, k, truths, extra=None, allow_ids=None):
    """V/flat/index_test.go:48-137 `run`: build the index (Add per vector,
    concurrently), add + delete the extra vectors, search concurrently."""
    idx = FlatIndex(ctx, 256, "cosine", compression=compression, rescore_limit=100 * k,
                    capacity=len(vectors) + (len(extra) if extra is not None else 0))
    n = len(vectors)
    with ThreadPoolExecutor(8) as ex:  # compressionhelpers.ConcurrentlyWithError
        list(ex.map(lambda lo: idx.AddBatch(np.arange(lo, min(lo + 1000, n)), vectors[lo:lo + 1000]),
                    range(0, n, 1000)))
    if extra is not None:
        for i in range(len(extra)):
            idx.Add(n + i, extra[i])
        for i in range(len(extra)):
            idx.Delete(n + i)
    allow = AllowList(*allow_ids) if allow_ids is not None else None

    def one(i):
        res, dists = idx.SearchByVector(queries[i], k, allow)
        return res, dists

    with ThreadPoolExecutor(8) as ex:  # compressionhelpers.Concurrently
        out = list(ex.map(one, range(len(queries))))
    relevant = retrieved = 0
    for i, (res, _) in enumerate(out):
        assert len(set(res.tolist())) == len(res), "results have duplicates"
        relevant += matches(truths[i], res)
        retrieved += len(res)
    return relevant / retrieved, out


@pytest.mark.parametrize("compression", [None, "bq"])
@pytest.mark.parametrize("deletes", [False, True])
@pytest.mark.parametrize("filtered", [False, True])
def test_no_race_flat_index(ctx, orc, flat_data, compression, deletes, filtered):
    vectors, queries, extra = flat_data
    k = 10
    if filtered:
        allow_ids = list(range(0, 3_000))
        truths = _truths(orc, vectors[:3_000], queries, k)
    else:
        allow_ids = None
        truths = _truths(orc, vectors, queries, k)
    recall, out = _run(ctx, compression, vectors, queries, k, truths, extra if deletes else None, allow_ids)
    target = 0.99 if compression is None else 0.8
    assert recall > target, recall
    if compression is None:  # exact search: the exact top-k, not just the recall
        for i, (res, _) in enumerate(out):
            assert np.array_equal(res, truths[i]), i
    if deletes or filtered:
        for res, _ in out:
            assert res.size == 0 or int(res.max()) < (3_000 if filtered else len(vectors))


def test_binary_quantizer_recall(ctx, orc):
    """CH/binary_quantization_test.go:31-84."""
    k, corrected_k = 10, 200
    rng = np.random.default_rng(31)
    vectors = orc.normalize_rows(random_vecs(rng, 10_000, 1536))
    queries = orc.normalize_rows(random_vecs(rng, 100, 1536))
    ids = np.arange(len(vectors), dtype=np.uint64)
    neighbors = [orc.lex_topk(orc.dist_all(2, q, vectors), ids, k)[0] for q in queries]
    bq = BinaryQuantizer(ctx)
    codes = bq.EncodeBatch(vectors)
    corpus = Corpus(ctx, KIND_BQ, METRIC_L2, 1536, len(vectors))
    try:
        corpus.upsert_codes(ids, codes)
        got, _, counts = corpus.search(queries, corrected_k)
        assert np.all(counts == corrected_k)
        hits = sum(matches(neighbors[i][:k], got[i]) for i in range(len(queries)))
        # the device Hamming scan equals the oracle's for every query
        for i in range(0, len(queries), 10):
            hd = orc.bq_dist_all(orc.bq_encode(queries[i]), codes)
            li, _ = orc.lex_topk(hd, ids, corrected_k)
            assert np.array_equal(got[i], li)
    finally:
        corpus.destroy()
    recall = hits / (k * len(queries))
    assert recall > 0.7, recall


def test_binary_quantizer_checks_size(ctx):
    """CH/binary_quantization_test.go:86-90."""
    bq = BinaryQuantizer(ctx)
    _, err = bq.DistanceBetweenCompressedVectors(np.zeros(3, np.uint64), np.zeros(4, np.uint64))
    assert err is not None


def test_concurrent_search_while_writing(ctx, orc):
    """Readers (k = 10 fused top-k and k = 300 select path) on many threads
    while a writer keeps adding and deleting far-away rows on the same corpus:
    every search must return exactly the oracle's top-k of the stable rows."""
    rng = np.random.default_rng(7)
    n, d = 5_000, 64
    stable = random_vecs(rng, n, d)
    far = random_vecs(rng, 1_000, d) + 100.0  # never enters a top-k of the stable queries
    queries = random_vecs(rng, 32, d)
    corpus = Corpus(ctx, KIND_F32, METRIC_L2, d, n + len(far))
    try:
        corpus.upsert(np.arange(n, dtype=np.uint64), stable)
        ids = np.arange(n, dtype=np.uint64)
        want = {}
        for k in (10, 300):
            want[k] = [orc.lex_topk(orc.dist_all(0, q, stable), ids, k) for q in queries]
        stop = threading.Event()
        errors = []

        def writer():
            far_ids = np.arange(n, n + len(far), dtype=np.uint64)
            try:
                while not stop.is_set():
                    corpus.upsert(far_ids, far)
                    corpus.delete(far_ids[::2])
                    corpus.delete(far_ids[1::2])
            except Exception as e:  # pragma: no cover - reported below
                errors.append(e)

        def reader(j):
            k = 10 if j % 2 == 0 else 300
            for r in range(6):
                qi = (j * 7 + r) % len(queries)
                got, dists, counts = corpus.search(queries[qi], k)
                wi, wd = want[k][qi]
                assert int(counts[0]) == k
                assert np.array_equal(got[0, :k], wi)
                assert np.array_equal(dists[0, :k].view(np.uint32), wd.view(np.uint32))

        w = threading.Thread(target=writer)
        w.start()
        try:
            with ThreadPoolExecutor(8) as ex:
                list(ex.map(reader, range(16)))
        finally:
            stop.set()
            w.join()
        assert not errors, errors
    finally:
        corpus.destroy()


def test_flat_from_user_config_and_rescore_update(ctx, orc):
    """flat.New from a parsed user config (BQ, rescoreLimit 20) and
    UpdateUserConfig raising the rescore limit (V/flat/index.go:67-97,
    297-305, 593-606): the search-time rescore window follows the update."""
    from oracle import wv_oracle
    from weaviate_amd.flat import ParseAndValidateConfig, ValidateUserConfigUpdate

    n, d, k = 5000, 128, 10
    rows = orc.synth_rows(91, 0, n, d, 0)
    q = orc.synth_rows(92, 0, 1, d, 0)[0]
    uc = ParseAndValidateConfig({"distance": "l2-squared", "bq": {"enabled": True, "rescoreLimit": 20}})
    idx = FlatIndex.from_user_config(ctx, d, uc, capacity=n)
    assert idx.bq is not None and idx.searchTimeRescore(k) == 20
    idx.AddBatch(np.arange(n, dtype=np.uint64), rows)
    codes = orc.bq_encode_rows(rows)
    ham = orc.bq_dist_all(orc.bq_encode(q), codes)
    exact = orc.dist_all(wv_oracle.L2, q, rows)
    for R in (20, 400):
        if R == 400:
            upd = ParseAndValidateConfig({"distance": "l2-squared", "bq": {"enabled": True, "rescoreLimit": 400}})
            ValidateUserConfigUpdate(uc, upd)
            idx.UpdateUserConfig(upd)
        assert idx.searchTimeRescore(k) == R
        ids, dists = idx.SearchByVector(q, k)
        cand, _ = orc.heap_pops(ham, R)  # the reference's Hamming heap, in pop order
        li, ld = orc.heap_topk(exact[cand.astype(np.int64)], cand, k)
        assert np.array_equal(ids, li)
        assert np.array_equal(dists.view(np.uint32), ld.view(np.uint32))
