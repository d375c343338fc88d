"""The m = 32, ks = 256 ADC scans against the oracle and against each other,
bit for bit: K8e (dense corpora, no allow list; one query per call), K8e COS
(co-scheduled batches), K8b (the rotated-segment scan that skips dead /
disallowed tiles: allow lists, thin corpora) and K8 (segment-order gather,
any m: here m = 16 on the same rows' codes' first half is not comparable, so
K8 is pinned to the oracle in test_gpu_parity).

K8b reads a different segment on every lane and keeps two rows in flight per
lane, so these cases aim at its pipeline: many tiles per wave, fully deleted
tiles between live ones, ragged tails, allow lists, several queries per
launch, every top-k width (E = 1, 2, 4) and non-finite LUT entries.
PQDistancer.Distance: CH/product_quantization.go:352-361 (LookUp :85-104).
"""
import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2
from weaviate_amd.device import Corpus, allow_bitmap

from test_gpu_parity import ORC_METRIC, bits, check_topk

pytestmark = pytest.mark.gpu

M, KS, D = 32, 256, 128


def _paths(c, qs, k, allow=None):
    """The same searches through every product path: one batch call (K8e COS
    when dense and no allow list), one call per query (K8e), and with an
    allow list admitting every row (K8b, which skips dead tiles)."""
    n = c.info()[1]
    batch = c.search(qs, k, allow=allow)
    singles = [c.search(qs[i], k, allow=allow) for i in range(len(qs))]
    single = tuple(np.concatenate([x[j] for x in singles]) for j in range(3))
    every = allow if allow is not None else allow_bitmap(np.arange(n, dtype=np.uint64))
    k8b = c.search(qs, k, allow=every)
    return batch, single, k8b


def _same(a, b):
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


def adc_all(metric, lut, codes):
    """Sequential fp32 sum over segments for every row (vectorised over rows; the
    per-row order is the reference's) + Wrap."""
    s = np.zeros(len(codes), np.float32)
    for i in range(lut.shape[0]):
        s = (s + lut[i, codes[:, i]]).astype(np.float32)
    if metric == 1:
        return (-s).astype(np.float32)
    if metric == 2:
        return (np.float32(1.0) - s).astype(np.float32)
    return s


@pytest.fixture(scope="module")
def big(ctx, orc):
    n = 600_000  # 9375 tiles: several per wave at 256 x 16 waves
    rng = np.random.default_rng(5)
    codes = rng.integers(0, KS, (n, M), dtype=np.uint8)
    codes[100:164] = codes[100]  # a tile of identical rows (ties)
    centers = orc.synth_rows(61, 0, M * KS, D // M, 0).reshape(M, KS, D // M)
    deleted = np.concatenate([np.arange(64 * 10, 64 * 40), np.arange(64 * 7000, 64 * 7300), rng.choice(n, 5000, replace=False)])
    deleted = np.unique(deleted).astype(np.uint64)
    valid = np.ones(n, np.uint8)
    valid[deleted] = 0
    return n, codes, centers, deleted, valid


def _corpus(ctx, metric, big):
    n, codes, centers, deleted, _ = big
    c = Corpus(ctx, KIND_PQ, metric, D, n)
    c.set_codebook(centers)
    c.upsert_codes(np.arange(n, dtype=np.uint64), codes)
    c.delete(deleted)
    return c


def test_adc_all_matches_oracle_rowwise(orc, big):
    _, codes, centers, _, _ = big
    q = orc.synth_rows(62, 0, 1, D, 0)[0]
    for metric in (0, 1):
        lut = orc.pq_lut(metric, q, centers)
        got = adc_all(metric, lut, codes[:200])
        want = np.array([orc.pq_adc(metric, lut, cd) for cd in codes[:200]], np.float32)
        assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT])
def test_rot_scan_vs_oracle(ctx, orc, big, metric):
    n, codes, centers, _, valid = big
    c = _corpus(ctx, metric, big)
    qs = orc.synth_rows(63, 0, 3, D, 0)
    try:
        for k in (10, 100, 200):
            paths = _paths(c, qs, k)
            for p in paths[1:]:
                _same(paths[0], p)
            ids, dists, counts = paths[0]
            for qi in range(len(qs)):
                lut = orc.pq_lut(ORC_METRIC[metric], qs[qi], centers)
                all_d = adc_all(ORC_METRIC[metric], lut, codes)
                check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k, valid)
    finally:
        c.destroy()


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
def test_rot_paths_agree(ctx, orc, big, metric):
    """K8e, K8e COS and K8b give the same bits, with and without a real allow
    list (an allow list sends every call to K8b, so then the three calls
    differ only in batching)."""
    n = big[0]
    c = _corpus(ctx, metric, big)
    qs = orc.synth_rows(64, 0, 2, D, 0)
    allow = allow_bitmap(np.arange(0, n, 3, dtype=np.uint64))
    try:
        for k, al in [(10, None), (64, allow), (150, None), (256, None)]:
            paths = _paths(c, qs, k, al)
            for p in paths[1:]:
                _same(paths[0], p)
    finally:
        c.destroy()


def test_rot_nonfinite_lut(ctx, orc, big):
    """Queries far outside the codebook overflow LUT entries to +inf; rows that
    hit them must tie at inf on every path, the others stay exact."""
    n, codes, centers, _, valid = big
    c = _corpus(ctx, METRIC_L2, big)
    q = orc.synth_rows(65, 0, 1, D, 0)[0].copy()
    q[:4] = 3e19  # segment 0: (3e19 - c)^2 -> inf for every centroid
    q2 = orc.synth_rows(66, 0, 1, D, 0)[0].copy()
    q2[64:66] = 2e19  # one segment: inf once the squares are summed
    qs = np.stack([q, q2])
    try:
        paths = _paths(c, qs, 20)
        for p in paths[1:]:
            _same(paths[0], p)
        ids, dists, counts = paths[0]
        for qi in range(2):
            all_d = adc_all(0, orc.pq_lut(0, qs[qi], centers), codes)
            check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), 20, valid)
    finally:
        c.destroy()


def test_rot_small_and_ragged(ctx, orc):
    """Corpora smaller than one tile per wave, ragged last tile, single live row."""
    centers = orc.synth_rows(67, 0, M * KS, D // M, 0).reshape(M, KS, D // M)
    rng = np.random.default_rng(68)
    for n in (1, 63, 65, 1000, 4097):
        codes = rng.integers(0, KS, (n, M), dtype=np.uint8)
        c = Corpus(ctx, KIND_PQ, METRIC_L2, D, n)
        c.set_codebook(centers)
        c.upsert_codes(np.arange(n, dtype=np.uint64), codes)
        q = orc.synth_rows(69, 0, 1, D, 0)[0]
        lut = orc.pq_lut(0, q, centers)
        all_d = adc_all(0, lut, codes)
        ids, dists, counts = c.search(q, 10)
        check_topk(orc, ids[0], dists[0], counts[0], all_d, np.arange(n, dtype=np.uint64), 10)
        if n > 1:
            c.delete(np.arange(1, n, dtype=np.uint64))
            ids, dists, counts = c.search(q, 10)
            assert counts[0] == 1 and ids[0][0] == 0
            assert np.array_equal(bits(dists[0][:1]), bits(all_d[:1]))
        c.destroy()
