"""K3c / K3d -- the bf16 MFMA screen -- and K3i -- the int8 MFMA screen (the
default for d = 512 / 768 / 1024, wvg_options.batch_screen = 2) -- each with a
per-row error bound + the exact fp32 rescore of every row the bound cannot rule
out (weaviate_amd/csrc/wvg_screen.hip) -- return exactly what the exact path returns: the same ids, the same
distance bits, the same counts, for batched dot and cosine searches
(Q flat.searchByVector calls, V/flat/index.go:319; SingleDist = dot_256,
D/dot_product.go:68-98, D/cosine_dist.go:38-68).  The exact path here is a
context with wvg_options.batch_screen = 0 (K3b / K3 fp32 MFMA), itself pinned
to the oracle in test_gpu_parity; a few queries are also checked against the
oracle directly."""
import numpy as np
import pytest

from weaviate_amd._lib import KIND_F32, METRIC_COSINE, METRIC_DOT
from weaviate_amd.device import Context, Corpus, allow_bitmap

from test_gpu_parity import ORC_METRIC, bits, check_topk, prep_query, stored_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def exact_ctx(ctx):
    c = Context(0, batch_screen=0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def bf16_ctx(ctx):
    c = Context(0, batch_screen=1)  # the bf16 screen (K3c / K3d) for every d
    yield c
    c.close()


def _pair(ctx, exact_ctx, metric, d, rows, ids=None):
    ids = np.arange(len(rows), dtype=np.uint64) if ids is None else ids
    cap = int(ids.max()) + 1 if len(ids) else 64
    a = Corpus(ctx, KIND_F32, metric, d, cap)
    b = Corpus(exact_ctx, KIND_F32, metric, d, cap)
    if len(ids):
        a.upsert(ids, rows)
        b.upsert(ids, rows)
    return a, b


def _same(x, y):
    ai, ad, ac = x
    bi, bd, bc = y
    assert np.array_equal(ac, bc)
    assert np.array_equal(ai, bi)
    assert np.array_equal(bits(ad), bits(bd))


@pytest.mark.parametrize("metric,d", [(METRIC_COSINE, 768), (METRIC_DOT, 768), (METRIC_COSINE, 128), (METRIC_DOT, 256),
                                      (METRIC_COSINE, 96), (METRIC_DOT, 1536), (METRIC_DOT, 512), (METRIC_COSINE, 512)])
def test_screen_equals_exact(ctx, exact_ctx, orc, metric, d):
    n = 30_000 + 77
    rows = orc.synth_rows(1000 + d, 0, n, d, 0)
    qs = orc.synth_rows(1001 + d, 0, 300, d, 0)
    a, b = _pair(ctx, exact_ctx, metric, d, rows)
    dead = np.array([0, 5, 64, 255, 256, 20_000, n - 1], np.uint64)
    a.delete(dead)
    b.delete(dead)
    try:
        for nq, k in [(32, 10), (300, 10), (40, 1), (129, 16), (64, 7)]:
            _same(a.search(qs[:nq], k), b.search(qs[:nq], k))
        ids, dists, counts = a.search(qs[:32], 10)
        srows = stored_rows(orc, metric, rows)
        valid = np.ones(n, np.uint8)
        valid[dead.astype(np.int64)] = 0
        for qi in (0, 31):
            all_d = orc.dist_all(ORC_METRIC[metric], prep_query(orc, metric, qs[qi]), srows)
            check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), 10, valid)
    finally:
        a.destroy()
        b.destroy()


@pytest.mark.parametrize("d", [256, 768])  # K3c, K3d
def test_screen_ties_overflow_rescan(ctx, exact_ctx, orc, d):
    """3000 copies of one row and a query equal to it: every copy ties at the
    k-th distance, the range lists fill below tau, the queries are flagged
    and rescanned exactly -- still the lexicographic (distance, docID) top-k."""
    n = 20_000
    rows = orc.synth_rows(1100, 0, n, d, 0)
    dup = np.arange(1000, 4000)
    rows[dup] = rows[1000]
    qs = orc.synth_rows(1101, 0, 40, d, 0)
    qs[::3] = rows[1000]
    for metric in (METRIC_DOT, METRIC_COSINE):
        a, b = _pair(ctx, exact_ctx, metric, d, rows)
        try:
            for k in (1, 10, 16):
                _same(a.search(qs, k), b.search(qs, k))
        finally:
            a.destroy()
            b.destroy()


@pytest.mark.parametrize("d", [128, 768])  # K3c, K3d
def test_screen_nonfinite_and_zero(ctx, exact_ctx, orc, d):
    """Rows and queries with inf / NaN / zero components: their bound is
    infinite (always rescored) or their distance exact; NaN sorts last."""
    n = 8000
    rows = np.floor(orc.synth_rows(1200, 0, n, d, 0) * 3).astype(np.float32)
    rows[10, 3] = np.nan
    rows[11, 4] = np.inf
    rows[12, 5] = -np.inf
    rows[[13, 14]] = 0.0
    rows[15] = 1e30
    qs = np.floor(orc.synth_rows(1201, 0, 48, d, 0) * 3).astype(np.float32)
    qs[1] = 0.0
    qs[2, 7] = np.inf
    qs[3] = 1e-30
    for metric in (METRIC_DOT, METRIC_COSINE):
        a, b = _pair(ctx, exact_ctx, metric, d, rows)
        try:
            for k in (1, 10):
                _same(a.search(qs, k), b.search(qs, k))
        finally:
            a.destroy()
            b.destroy()


def test_screen_large_finite_magnitudes(ctx, exact_ctx, orc):
    """Large finite rows and queries on both sides of the fast check's limits
    (row norm bound 2^60, query K1 2^50: beyond them every element takes the
    exact per-element test, inside them u - sigma must stay finite): dot
    products up to ~1e38, products that overflow bf16 / fp32 accumulation."""
    n, d = 6000, 768
    rows = orc.synth_rows(1250, 0, n, d, 0)
    rows[100:110] *= np.float32(1e10)     # norm ~1e11: fast-eligible
    rows[200:210] *= np.float32(1e19)     # norm ~1e20 > 2^60: forced exact
    rows[300] = np.float32(3e38)          # bf16 rounds it to inf
    qs = orc.synth_rows(1251, 0, 40, d, 0)
    qs[1] *= np.float32(1e10)             # K1 ~1e9: fast-eligible
    qs[2] *= np.float32(1e17)             # K1 > 2^50: forced exact
    qs[3] *= np.float32(1e25)
    for metric in (METRIC_DOT, METRIC_COSINE):
        a, b = _pair(ctx, exact_ctx, metric, d, rows)
        try:
            for k in (1, 10, 16):
                _same(a.search(qs, k), b.search(qs, k))
        finally:
            a.destroy()
            b.destroy()


@pytest.mark.parametrize("d", [128, 768])  # K3c, K3d
def test_screen_allow_sparse_small(ctx, exact_ctx, orc, d):
    """Allow lists, a corpus smaller than k, ragged tails, a sparse id space."""
    qs = orc.synth_rows(1301, 0, 64, d, 0)
    for n in (5, 63, 300, 4097):
        rows = orc.synth_rows(1300 + n, 0, n, d, 0)
        a, b = _pair(ctx, exact_ctx, METRIC_DOT, d, rows)
        try:
            _same(a.search(qs, 10), b.search(qs, 10))
            if n > 60:
                al = allow_bitmap(np.arange(1, n, 3, dtype=np.uint64))
                _same(a.search(qs, 10, al), b.search(qs, 10, al))
        finally:
            a.destroy()
            b.destroy()
    ids = np.sort(np.random.default_rng(1302).choice(200_000, 5000, replace=False)).astype(np.uint64)
    rows = orc.synth_rows(1303, 0, len(ids), d, 0)
    a, b = _pair(ctx, exact_ctx, METRIC_COSINE, d, rows, ids)
    try:
        _same(a.search(qs, 10), b.search(qs, 10))
    finally:
        a.destroy()
        b.destroy()


def test_screen_shadow_follows_writes(ctx, exact_ctx, orc):
    """The bf16 shadow is rebuilt over the tiles written since the last
    screened search (upsert, restart load) and dropped on growth (reserve)."""
    n, d = 12_000, 256
    rows = orc.synth_rows(1400, 0, n, d, 0)
    qs = orc.synth_rows(1401, 0, 40, d, 0)
    a, b = _pair(ctx, exact_ctx, METRIC_DOT, d, rows)
    try:
        _same(a.search(qs, 10), b.search(qs, 10))  # builds the shadow
        # overwrite rows so that new ones win: the query itself, scaled up
        ids = np.array([7, 4000, 11_999], np.uint64)
        new = (qs[:3] * 4).astype(np.float32)
        a.upsert(ids, new)
        b.upsert(ids, new)
        got = a.search(qs, 10)
        _same(got, b.search(qs, 10))
        assert got[0][0][0] == 7 and got[0][1][0] == 4000 and got[0][2][0] == 11_999
        a.reserve(20_000)  # realloc: the shadow is rebuilt from scratch
        b.reserve(20_000)
        more = orc.synth_rows(1402, 0, 5000, d, 0)
        mids = np.arange(15_000, 20_000, dtype=np.uint64)
        a.upsert(mids, more)
        b.upsert(mids, more)
        _same(a.search(qs, 10), b.search(qs, 10))
        a.fill_synthetic(1403, 9000, 0)
        b.fill_synthetic(1403, 9000, 0)
        _same(a.search(qs, 10), b.search(qs, 10))
    finally:
        a.destroy()
        b.destroy()


def test_screen_device_path(ctx, exact_ctx, orc):
    """wvg_search_device (queries in HBM, async on a stream) takes the screen
    for batches too, and returns the host API's exact results."""
    import torch

    from weaviate_amd import _lib

    n, d, nq, k = 25_000, 768, 200, 10
    rows = orc.synth_rows(1500, 0, n, d, 0)
    a, b = _pair(ctx, exact_ctx, METRIC_COSINE, d, rows)
    try:
        raw = orc.synth_rows(1501, 0, nq, d, 0)
        # the device API takes normalized queries; the host API normalizes raw ones (Normalize, the same bits)
        qs = np.stack([orc.normalize(q) for q in raw]).astype(np.float32)
        lib = ctx.lib
        dev = torch.device("cuda:0")
        ws = torch.zeros(lib.wvg_search_workspace_size(a.handle, nq, k), dtype=torch.uint8, device=dev)
        tq = torch.from_numpy(qs).to(dev)
        oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
        od = torch.empty((nq, k), dtype=torch.float32, device=dev)
        oc = torch.empty(nq, dtype=torch.int32, device=dev)
        for _ in range(2):
            _lib.check(lib.wvg_search_device(a.handle, tq.data_ptr(), nq, k, oi.data_ptr(), od.data_ptr(),
                                             oc.data_ptr(), ws.data_ptr(), ws.numel(),
                                             torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            _same((oi.cpu().numpy().view(np.uint64), od.cpu().numpy(), oc.cpu().numpy().astype(np.uint32)),
                  b.search(raw, k))
        # d_counts = NULL (allowed by the header): the pilot and the merges keep their own counts
        oi.fill_(0)
        _lib.check(lib.wvg_search_device(a.handle, tq.data_ptr(), nq, k, oi.data_ptr(), od.data_ptr(), None,
                                         ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        ei, ed, _ = b.search(raw, k)
        assert np.array_equal(oi.cpu().numpy().view(np.uint64), ei)
        assert np.array_equal(od.cpu().numpy().view(np.uint32), ed.view(np.uint32))
    finally:
        a.destroy()
        b.destroy()


@pytest.mark.parametrize("d", [512, 768, 1024])
@pytest.mark.parametrize("metric", [METRIC_COSINE, METRIC_DOT])
def test_screen_int8_and_bf16_equal_exact(ctx, bf16_ctx, exact_ctx, orc, metric, d):
    """The int8 screen (default context) and the bf16 one (batch_screen = 1) on
    the same rows: both bit-identical to the exact path, over batch sizes that
    take one or several 128-query blocks, k = 1 .. 16, deletes and an allow list."""
    n = 40_000 + 13
    rows = orc.synth_rows(1600 + d, 0, n, d, 0)
    qs = orc.synth_rows(1601 + d, 0, 260, d, 0)
    a, b = _pair(ctx, exact_ctx, metric, d, rows)
    c = Corpus(bf16_ctx, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    dead = np.arange(0, n, 97, dtype=np.uint64)
    for x in (a, b, c):
        x.delete(dead)
    try:
        al = allow_bitmap(np.arange(2, n, 5, dtype=np.uint64))
        for nq, k, allow in [(32, 10, None), (260, 16, None), (33, 1, None), (64, 10, al)]:
            want = b.search(qs[:nq], k, allow)
            _same(a.search(qs[:nq], k, allow), want)
            _same(c.search(qs[:nq], k, allow), want)
    finally:
        for x in (a, b, c):
            x.destroy()


def test_screen_int8_scale_outliers_and_saturation(ctx, exact_ctx, orc):
    """The int8 shadow's one corpus scale S is set at its first build: rows with
    one huge element (S large, every other row coarsely coded), rows written
    later that exceed 127 S (clamped codes, large error bounds), rows of equal
    maximal codes (|int32 score| = d 127^2 near 2^24 at d = 1024), heavy ties
    and zero rows -- the bound stays valid, results exact."""
    for d in (768, 1024):
        n = 20_000
        rows = orc.synth_rows(1700 + d, 0, n, d, 0)
        rows[5, 3] = 40.0                      # one outlier: S = 40 / 127
        rows[6:9] = 1.0                        # all codes at the clamp value after scaling
        rows[9] = -1.0
        rows[10:14] = 0.0
        rows[100:400] = rows[100]              # 300 exact ties
        qs = orc.synth_rows(1701 + d, 0, 48, d, 0)
        qs[0] = 1.0                            # |q8 . x8| = d 127^2 against rows 6..8
        qs[1] = rows[100]
        qs[2] = 0.0
        qs[3, :] = 1e-30                       # a scale near the underflow guard
        qs[4, 7] = np.nan
        for metric in (METRIC_DOT, METRIC_COSINE):
            a, b = _pair(ctx, exact_ctx, metric, d, rows)
            try:
                for k in (1, 10, 16):
                    _same(a.search(qs, k), b.search(qs, k))  # first build: S from these rows
                big = (orc.synth_rows(1702 + d, 0, 50, d, 0) * 1000).astype(np.float32)
                bids = np.arange(15_000, 15_050, dtype=np.uint64)
                a.upsert(bids, big)                # beyond 127 S: clamped codes
                b.upsert(bids, big)
                for k in (1, 10):
                    _same(a.search(qs, k), b.search(qs, k))
                qs2 = big[:40] / 1000
                _same(a.search(qs2, 10), b.search(qs2, 10))
            finally:
                a.destroy()
                b.destroy()


def test_screen_int8_varied_norms_dot(ctx, exact_ctx, orc):
    """Dot products over rows whose norms span six orders of magnitude (the
    corpus scale codes small rows with few levels: wide bounds, many
    candidates, the flag path) -- exact."""
    n, d = 30_000, 768
    rows = orc.synth_rows(1800, 0, n, d, 0)
    scale = (10.0 ** np.random.default_rng(1801).uniform(-3, 3, n)).astype(np.float32)
    rows *= scale[:, None]
    qs = orc.synth_rows(1802, 0, 128, d, 0)
    a, b = _pair(ctx, exact_ctx, METRIC_DOT, d, rows)
    try:
        for k in (1, 10, 16):
            _same(a.search(qs, k), b.search(qs, k))
    finally:
        a.destroy()
        b.destroy()
