"""K8b (rotated-segment ADC scan, m = 32, ks = 256) against the oracle and
against K8 (segment-order gather), bit for bit.

K8b reads a different segment on every lane and keeps two rows in flight per
lane, so these cases aim at its pipeline: many tiles per wave, fully deleted
tiles between live ones, ragged tails, allow lists, several queries per
launch, every top-k width (E = 1, 2, 4) and non-finite LUT entries.
PQDistancer.Distance: CH/product_quantization.go:352-361 (LookUp :85-104).
"""
import ctypes

import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2
from weaviate_amd.device import Corpus, allow_bitmap

from test_gpu_parity import ORC_METRIC, bits, check_topk

pytestmark = pytest.mark.gpu

M, KS, D = 32, 256, 128


def _variant(v):
    lib = _lib.load()
    lib.wvgx_set_tuning.restype = ctypes.c_int
    lib.wvgx_set_tuning.argtypes = [ctypes.c_int, ctypes.c_int]
    return lib.wvgx_set_tuning(7, v)


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
    old = _variant(0)
    try:
        for k in (10, 100, 200):
            ids, dists, counts = c.search(qs, k)
            for qi in range(len(qs)):
                lut = orc.pq_lut(ORC_METRIC[metric], qs[qi], centers)
                all_d = adc_all(ORC_METRIC[metric], lut, codes)
                check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k, valid)
    finally:
        _variant(old)
        c.destroy()


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
def test_rot_equals_gather_variant(ctx, orc, big, metric):
    n = big[0]
    c = _corpus(ctx, metric, big)
    qs = orc.synth_rows(64, 0, 2, D, 0)
    allow = allow_bitmap(np.arange(0, n, 3, dtype=np.uint64))
    old = _variant(0)
    try:
        for k, al in [(10, None), (64, allow), (150, None)]:
            _variant(1)
            b = c.search(qs, k, allow=al)
            for v in (0, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 29, 30, 31, 32, 33, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49):
                # K8b: ring 6, ring 4, interleaved waves, LDS batches 32 / 8, dense (no tile skip) rings 6 / 4 / 8;
                # K8c rings 8 / 4 / 8; K8b forced; K8d (buffer / global loads); K8c one-v_perm addresses; K8e
                _variant(v)
                a = c.search(qs, k, allow=al)
                for x, y in zip(a, b):
                    assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8)), v
    finally:
        _variant(old)
        c.destroy()


def test_rot_nonfinite_lut(ctx, orc, big):
    """Queries far outside the codebook overflow LUT entries to +inf; rows that
    hit them must tie at inf in both variants, the others stay exact."""
    n = big[0]
    c = _corpus(ctx, METRIC_L2, big)
    q = orc.synth_rows(65, 0, 1, D, 0)[0].copy()
    q[:4] = 3e19  # segment 0: (3e19 - c)^2 -> inf for every centroid
    q2 = orc.synth_rows(66, 0, 1, D, 0)[0].copy()
    q2[64:66] = 2e19  # one segment: inf once the squares are summed
    old = _variant(0)
    try:
        for qq in (q, q2):
            _variant(1)
            b = c.search(qq, 20)
            for v in (0, 6, 10, 14, 17, 18, 20, 22, 29, 31, 35, 36, 38, 41, 42, 46):
                _variant(v)
                a = c.search(qq, 20)
                for x, y in zip(a, b):
                    assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    finally:
        _variant(old)
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
