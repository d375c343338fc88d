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
