"""Concurrent single-query wvg_search calls (one goroutine per Weaviate query:
adapters/repos/db/index_queue.go:575-586, V/flat/index.go:307-334) are
coalesced inside the library into shared batched launches
(wvg_options.coalesce, wvg_search.hip search_coalesced).  Every caller must
get exactly what a call of its own returns: ids, distance bits and counts,
whatever batch it lands in -- K1 co-scheduled batches (L2, manhattan), the
bf16 screen for dot / cosine batches of 32 or more, K5 / K8e batches for BQ /
PQ corpora -- and with different k values in flight at once."""
import threading

import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import (KIND_BQ, KIND_F32, KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2, METRIC_MANHATTAN,
                               fptr, u32ptr, u64ptr)
from weaviate_amd.device import Context, Corpus

pytestmark = pytest.mark.gpu


def one_search(lib, c, q, k):
    ids = np.empty(k, np.uint64)
    d = np.empty(k, np.float32)
    cnt = np.empty(1, np.uint32)
    _lib.check(lib.wvg_search(c.handle, fptr(q), 1, k, None, 0, u64ptr(ids), fptr(d), u32ptr(cnt)))
    return ids, d, int(cnt[0])


def concurrent(lib, c, qs, ks, threads):
    """Every thread searches its share of the queries, one call each, all
    threads released together."""
    out = [None] * len(qs)
    errs = []
    start = threading.Barrier(threads)

    def worker(t):
        try:
            start.wait()
            for i in range(t, len(qs), threads):
                out[i] = one_search(lib, c, qs[i], ks[i])
        except Exception as e:  # noqa: BLE001 -- reported by the test
            errs.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    assert all(o is not None for o in out)
    return out


def make_corpus(ctx, orc, kind, metric, n, d):
    rows = orc.synth_rows(701, 0, n, d, 0)
    c = Corpus(ctx, kind, metric, d, n)
    if kind == KIND_PQ:
        c.set_codebook(np.ascontiguousarray(rows[:256].reshape(256, d // 4, 4).transpose(1, 0, 2)))
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    c.delete(np.arange(5, n, 97, dtype=np.uint64))
    return c


@pytest.mark.parametrize("kind,metric,d,threads", [
    (KIND_F32, METRIC_L2, 128, 16),
    (KIND_F32, METRIC_MANHATTAN, 96, 16),
    (KIND_F32, METRIC_COSINE, 256, 48),   # batches of >= 32 take the bf16 screen
    (KIND_F32, METRIC_DOT, 768, 40),
    (KIND_BQ, METRIC_COSINE, 512, 16),
    (KIND_PQ, METRIC_L2, 128, 16),
])
def test_concurrent_calls_equal_serial_calls(ctx, orc, kind, metric, d, threads):
    n = 20_000
    c = make_corpus(ctx, orc, kind, metric, n, d)
    lib = _lib.load()
    nq = 6 * threads
    qs = np.ascontiguousarray(orc.synth_rows(702, 0, nq, d, 0))
    ks = [(10, 1, 16, 10, 64, 10)[i % 6] for i in range(nq)]  # different k in flight together
    serial = [one_search(lib, c, qs[i], ks[i]) for i in range(nq)]
    for rep in range(2):
        got = concurrent(lib, c, qs, ks, threads)
        for i in range(nq):
            si, sd, sc = serial[i]
            gi, gd, gc = got[i]
            assert gc == sc, (rep, i)
            assert np.array_equal(gi, si), (rep, i, gi, si)
            assert np.array_equal(gd.view(np.uint32), sd.view(np.uint32)), (rep, i)
    c.destroy()


@pytest.mark.parametrize("kind,metric,n", [
    (KIND_F32, METRIC_L2, 20_000),
    (KIND_F32, METRIC_L2, 150),    # fewer live rows than the batch's k: counts = min(live, k)
    (KIND_BQ, METRIC_COSINE, 20_000),
    (KIND_PQ, METRIC_L2, 20_000),
])
def test_mixed_k_batches_give_each_caller_its_prefix(ctx, orc, kind, metric, n):
    """Round 5: a coalesced batch runs at the largest k of its requests (up to
    256) and hands each caller the first k of its rows -- exactly what a call
    of its own returns, counts and the entries past the count included."""
    d = 128
    c = make_corpus(ctx, orc, kind, metric, n, d)
    lib = _lib.load()
    threads = 16
    nq = 4 * threads
    qs = np.ascontiguousarray(orc.synth_rows(711, 0, nq, d, 0))
    ks = [(1, 256, 10, 100)[i % 4] for i in range(nq)]
    live = n - len(range(5, n, 97))  # make_corpus deletes every 97th row from 5
    serial = [one_search(lib, c, qs[i], ks[i]) for i in range(nq)]
    for rep in range(3):
        got = concurrent(lib, c, qs, ks, threads)
        for i in range(nq):
            si, sd, sc = serial[i]
            gi, gd, gc = got[i]
            assert gc == sc == min(ks[i], live), (rep, i)
            assert np.array_equal(gi, si), (rep, i)
            assert np.array_equal(gd.view(np.uint32), sd.view(np.uint32)), (rep, i)
    c.destroy()


def test_coalescing_can_be_switched_off(ctx, orc):
    """wvg_options.coalesce = 0: every call launches alone -- same results."""
    n, d = 5000, 64
    off = Context(0, coalesce=0)
    try:
        c0 = make_corpus(off, orc, KIND_F32, METRIC_L2, n, d)
        c1 = make_corpus(ctx, orc, KIND_F32, METRIC_L2, n, d)
        qs = np.ascontiguousarray(orc.synth_rows(703, 0, 64, d, 0))
        a = concurrent(off.lib, c0, qs, [10] * 64, 8)
        b = concurrent(ctx.lib, c1, qs, [10] * 64, 8)
        for x, y in zip(a, b):
            assert np.array_equal(x[0], y[0]) and np.array_equal(x[1].view(np.uint32), y[1].view(np.uint32))
        c0.destroy()
        c1.destroy()
    finally:
        off.close()


def test_coalesced_results_match_oracle(ctx, orc):
    n, d, k = 8000, 128, 10
    rows = orc.synth_rows(704, 0, n, d, 0)
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    qs = np.ascontiguousarray(orc.synth_rows(705, 0, 32, d, 0))
    got = concurrent(_lib.load(), c, qs, [k] * 32, 16)
    for qi in range(32):
        wi, wd = orc.lex_topk(orc.dist_all(0, qs[qi], rows), np.arange(n, dtype=np.uint64), k)
        assert np.array_equal(got[qi][0], wi)
        assert np.array_equal(got[qi][1].view(np.uint32), wd.view(np.uint32))
    c.destroy()


def test_back_to_back_single_queries_on_one_slot(ctx, orc):
    """The interleaving behind round 4's polled-path failure (What's
    weak #1): one thread = one stream slot, so consecutive single-query calls
    reuse the slot's host result buffer, its partial lists and its arrival
    counter, and the previous call's complete result sits in that buffer when
    the next call starts.  Each call's results arrive as tagged records
    (StreamJob::records); a call may only return entries carrying its own tag.
    Alternating queries with 8-query batches (other partial lists on the slot)
    in between, every result must be its own query's oracle top-k -- never the
    previous call's."""
    n, d, k = 5000, 64, 10
    rows = orc.synth_rows(708, 0, n, d, 0)
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    lib = _lib.load()
    qs = np.ascontiguousarray(orc.synth_rows(709, 0, 7, d, 0))
    want = [orc.lex_topk(orc.dist_all(0, q, rows), np.arange(n, dtype=np.uint64), k) for q in qs]
    for r in range(700):
        qi = (r * 3) % len(qs)
        kk = k if r % 5 else 7  # a shorter result than the slot's previous one
        gi, gd, gc = one_search(lib, c, qs[qi], kk)
        assert gc == kk, r
        assert np.array_equal(gi, want[qi][0][:kk]), (r, qi)
        assert np.array_equal(gd.view(np.uint32), want[qi][1][:kk].view(np.uint32)), (r, qi)
        if r % 4 == 3:
            c.search(qs[:5], k)
    c.destroy()


def test_coalesced_calls_with_concurrent_writes(ctx, orc):
    """Single-query searches keep coalescing while another thread upserts and
    deletes (writers take the corpus exclusively; queued searches wait, none
    deadlocks); afterwards the corpus answers exactly as the oracle on its
    final rows."""
    n, d, k = 6000, 64, 10
    rows = orc.synth_rows(706, 0, n, d, 0)
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    lib = _lib.load()
    qs = np.ascontiguousarray(orc.synth_rows(707, 0, 48, d, 0))
    stop = threading.Event()
    errs = []

    def writer():
        try:
            for i in range(20):
                ids = np.arange(i * 50, i * 50 + 50, dtype=np.uint64)
                c.upsert(ids, rows[ids.astype(np.int64)] * np.float32(1.0))
                c.delete(ids[::7])
            stop.set()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            stop.set()

    def reader(t):
        try:
            while not stop.is_set():
                ids, dd, cnt = one_search(lib, c, qs[t], k)
                assert cnt == k
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=reader, args=(t,)) for t in range(12)] + [threading.Thread(target=writer)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a thread did not finish"
    assert not errs, errs
    valid = np.ones(n, bool)
    for i in range(20):
        valid[np.arange(i * 50, i * 50 + 50)[::7]] = False
    live = np.flatnonzero(valid).astype(np.uint64)
    for qi in (0, 47):
        gi, gd, gc = one_search(lib, c, qs[qi], k)
        wi, wd = orc.lex_topk(orc.dist_all(0, qs[qi], rows[live.astype(np.int64)]), live, k)
        assert np.array_equal(gi, wi)
        assert np.array_equal(gd.view(np.uint32), wd.view(np.uint32))
    c.destroy()


@pytest.mark.parametrize("metric,d", [(METRIC_L2, 128), (METRIC_COSINE, 96)])
def test_filtered_calls_coalesce_equal_serial(ctx, orc, metric, d):
    """Filtered single queries (every Weaviate query with a where-filter carries
    its own allow list: adapters/repos/db/shard_read.go:341, the scan
    restriction V/flat/index.go:423-449) join coalesced batches too: one
    co-scheduled K1 launch over the union of their allow windows, each query
    masked by its own (ScanArgs::allow_qstride).  16 threads with mixed lists
    -- 10 %, 1 %, a narrow id range, a single id, an empty list, none -- and
    mixed k must get exactly what serial calls return."""
    _filtered_vs_serial(ctx, orc, metric, d)


def test_filtered_calls_coalesce_with_mfma_min_queries_1(orc):
    """with mfma_min_queries = 1 a filtered cosine batch used to be
    planned onto the MFMA path, which takes no per-query allow windows, and
    every caller of the batch failed.  Filtered batches never go to MFMA."""
    with Context(0, mfma_min_queries=1) as c1:
        _filtered_vs_serial(c1, orc, METRIC_COSINE, 96)


def test_filtered_batches_stay_within_the_byte_budget(ctx, orc):
    """80 concurrent callers with wide allow lists over 1.2M rows: one batch of
    all of them would hold 80 x 150 KB of allow words, above the 8 MB budget
    (ADVICE r5), so the coalescer splits them -- every caller still gets its
    own call's result."""
    _filtered_vs_serial(ctx, orc, METRIC_L2, 32, n=1_200_000, nq=160, threads=80, wide=True)


def _filtered_vs_serial(ctx, orc, metric, d, n=30_000, nq=96, threads=16, wide=False):
    from weaviate_amd.device import allow_bitmap

    c = make_corpus(ctx, orc, KIND_F32, metric, n, d)
    lib = _lib.load()
    rng = np.random.default_rng(710)
    qs = np.ascontiguousarray(orc.synth_rows(711, 0, nq, d, 0))
    allows = []
    for i in range(nq):
        kind = 0 if wide else i % 6
        if wide:
            allows.append(allow_bitmap(np.flatnonzero(rng.random(n) < 0.5), n))
        elif kind == 0:
            allows.append(allow_bitmap(np.flatnonzero(rng.random(n) < 0.10), n))
        elif kind == 1:
            allows.append(allow_bitmap(np.flatnonzero(rng.random(n) < 0.01), n))
        elif kind == 2:
            lo = int(rng.integers(0, n - 3000))
            allows.append(allow_bitmap(range(lo, lo + 2500), n))
        elif kind == 3:
            allows.append(allow_bitmap([int(rng.integers(0, n))], n))
        elif kind == 4:
            allows.append(np.zeros((n + 63) // 64, np.uint64))  # non-nil, empty: no results
        else:
            allows.append(None)
    ks = [(10, 3, 10, 64, 10, 1)[(i // 6) % 6] for i in range(nq)]

    def call(i):
        ids = np.empty(ks[i], np.uint64)
        dd = np.empty(ks[i], np.float32)
        cnt = np.empty(1, np.uint32)
        a = allows[i]
        _lib.check(lib.wvg_search(c.handle, fptr(qs[i]), 1, ks[i], u64ptr(a) if a is not None else None,
                                  0 if a is None else len(a), u64ptr(ids), fptr(dd), u32ptr(cnt)))
        return ids, dd, int(cnt[0])

    serial = [call(i) for i in range(nq)]
    for rep in range(3):
        out = [None] * nq
        errs = []
        start = threading.Barrier(threads)

        def worker(t):
            try:
                start.wait()
                for i in range(t, nq, threads):
                    out[i] = call(i)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errs, errs
        for i in range(nq):
            si, sd, sc = serial[i]
            gi, gd, gc = out[i]
            assert gc == sc, (rep, i)
            assert np.array_equal(gi[:sc], si[:sc]), (rep, i)
            assert np.array_equal(gd[:sc].view(np.uint32), sd[:sc].view(np.uint32)), (rep, i)
    # and the serial results are the oracle's: the filtered lexicographic top-k
    rows = orc.synth_rows(701, 0, n, d, 0)
    live = np.ones(n, bool)
    live[np.arange(5, n, 97)] = False
    om = 2 if metric == METRIC_COSINE else 0
    for i in range(0, nq, 7):
        a = allows[i]
        ok = live.copy()
        if a is not None:
            bitsv = np.unpackbits(a.view(np.uint8), bitorder="little")[:n].astype(bool)
            ok &= bitsv
        ids = np.flatnonzero(ok).astype(np.uint64)
        want = min(ks[i], len(ids))
        assert serial[i][2] == want
        if want:
            r = rows[ids.astype(np.int64)]
            q = qs[i]
            if om == 2:
                r = orc.normalize_rows(r)
                q = orc.normalize(q)
            wi, wd = orc.lex_topk(orc.dist_all(om, q, r), ids, ks[i])
            assert np.array_equal(serial[i][0][:want], wi[:want]), i
    c.destroy()
