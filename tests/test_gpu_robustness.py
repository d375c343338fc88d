"""GPU tests of the boundary's failure and edge behaviour: stored data right
after creation, empty corpora on the device path, the query-stream merge
timeout (surfaced, never stale), allow lists over a docID space far larger
than the corpus, PQ codebook / code validation, batched row fetch and the
packed all-gather merge."""
import ctypes

import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_BQ, KIND_F32, KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2
from weaviate_amd.device import Corpus, allow_bitmap

pytestmark = pytest.mark.gpu

NONE = np.iinfo(np.uint64).max


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def test_create_then_fill_stored_rows_exact(ctx, orc):
    """Round 1's fault: the allocation's zero fill (null stream) could land
    after rows written on a pool stream.  Create + fill + reserve-grow
    repeatedly and compare chunk 0 of every tile and a stride of all rows."""
    n, d = 300_000, 128  # 153.6 MB of rows
    want = orc.synth_rows(42, 0, n, d, 0)
    for rep in range(3):
        c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
        c.fill_synthetic(42, n, 0)
        firsts = np.arange(0, n, 64, dtype=np.uint64)  # lane 0 of every tile
        got, ok = c.get_batch(firsts)
        assert ok.all() and np.array_equal(bits(got), bits(want[firsts.astype(np.int64)]))
        strided = np.arange(rep, n, 7, dtype=np.uint64)
        got, ok = c.get_batch(strided)
        assert ok.all() and np.array_equal(bits(got), bits(want[strided.astype(np.int64)]))
        # a grow copies the rows and zero-fills the rest on the same stream
        c.reserve(2 * n)
        got, ok = c.get_batch(firsts)
        assert ok.all() and np.array_equal(bits(got), bits(want[firsts.astype(np.int64)]))
        c.destroy()


@pytest.mark.parametrize("kind", [KIND_F32, KIND_BQ, KIND_PQ])
def test_get_batch_matches_get(ctx, orc, kind):
    n, d, m, ks = 1000, 64, 32, 256
    c = Corpus(ctx, kind, METRIC_L2, d, n, id_base=640)
    if kind == KIND_PQ:
        c.set_codebook(orc.synth_rows(5, 0, m * ks, d // m, 0).reshape(m, ks, d // m))
    c.upsert(np.arange(640, 640 + n, dtype=np.uint64), orc.synth_rows(6, 0, n, d, 0))
    c.delete(np.array([641, 700], np.uint64))
    ids = np.array([640, 641, 700, 701, 640 + n - 1, 5, 640 + n + 3, 1000], np.uint64)
    rows, ok = c.get_batch(ids, pq_m=m)
    assert ok.tolist() == [True, False, False, True, True, False, False, True]
    for i, good in zip(ids, ok):
        if good:
            assert np.array_equal(rows[list(ids).index(i)], c.get(int(i), pq_m=m))
    assert not rows[~ok].any()


def test_device_search_on_empty_corpus_writes_empty_results(ctx):
    import torch

    lib = _lib.load()
    dev = torch.device("cuda:0")
    for cap in (0, 640):
        c = Corpus(ctx, KIND_F32, METRIC_L2, 32, cap, id_base=64)
        nq, k = 3, 10
        ws = torch.zeros(max(256, lib.wvg_search_workspace_size(c.handle, nq, k)), dtype=torch.uint8, device=dev)
        q = torch.zeros((nq, 32), dtype=torch.float32, device=dev)
        for fn in (lib.wvg_search_device, lib.wvg_search_device_pipelined):
            ids = torch.full((nq, k), 7, dtype=torch.int64, device=dev)  # garbage that must be overwritten
            dd = torch.full((nq, k), -1.0, dtype=torch.float32, device=dev)
            cc = torch.full((nq,), 5, dtype=torch.int32, device=dev)
            _lib.check(fn(c.handle, q.data_ptr(), nq, k, ids.data_ptr(), dd.data_ptr(), cc.data_ptr(),
                          ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            assert (ids.cpu().numpy().view(np.uint64) == NONE).all()
            assert np.isinf(dd.cpu().numpy()).all()
            assert (cc.cpu().numpy() == 0).all()
        c.destroy()


def test_query_stream_merge_timeout_is_reported(ctx, orc):
    """A merge workgroup that gives up (a context with a 1 us merge wait,
    wvg_options.merge_wait_us) makes wvg_search_device_check fail, and the
    unmerged queries come back empty, never with a previous call's results;
    the default wait then succeeds."""
    import torch

    from weaviate_amd.device import Context

    lib = _lib.load()
    n, d, k, nq = 1_000_000, 128, 10, 4
    short = Context(0, merge_wait_us=1)
    assert short.options["merge_wait_us"] == 1
    c = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
    cs = Corpus(short, KIND_F32, METRIC_L2, d, n)
    cs.fill_synthetic(42, n, 0)
    c.fill_synthetic(42, n, 0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.zeros(lib.wvg_search_workspace_size(c.handle, nq, k), dtype=torch.uint8, device=dev)
    tq = torch.from_numpy(orc.synth_rows(43, 0, nq, d, 0)).to(dev)
    ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
    dd = torch.empty((nq, k), dtype=torch.float32, device=dev)
    cc = torch.empty(nq, dtype=torch.int32, device=dev)

    def run(corpus):
        _lib.check(lib.wvg_search_device_pipelined(corpus.handle, tq.data_ptr(), nq, k, ids.data_ptr(),
                                                   dd.data_ptr(), cc.data_ptr(), ws.data_ptr(), ws.numel(), st))

    try:
        run(c)
        _lib.check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), st))
        good = ids.cpu().numpy().copy()
        assert (cc.cpu().numpy() == k).all()
        run(cs)  # the same rows and workspace, the 1 us merge bound
        rc = lib.wvg_search_device_check(short.handle, ws.data_ptr(), st)
        assert rc == _lib.WVG_ERR_DEVICE
        assert b"timed out" in lib.wvg_last_error()
        got_c = cc.cpu().numpy()
        got_i = ids.cpu().numpy()
        for qi in range(nq):  # each query is either fully merged or empty -- never stale
            if got_c[qi] == 0:
                assert (got_i[qi].view(np.uint64) == NONE).all()
            else:
                assert np.array_equal(got_i[qi], good[qi])
        assert (got_c == 0).any()
        # the check cleared the sticky word; a normal call passes again
        run(c)
        _lib.check(lib.wvg_search_device_check(ctx.handle, ws.data_ptr(), st))
        assert np.array_equal(ids.cpu().numpy(), good)
    finally:
        c.destroy()
        cs.destroy()
        short.close()


@pytest.mark.parametrize("kind", [KIND_F32, KIND_BQ])
def test_allow_list_over_large_docid_space(ctx, orc, kind):
    """The allow bitmap spans docIDs far beyond this corpus (a 1B-id index
    whose rank holds [id_base, id_base + n)); only the corpus's window is read."""
    n, d, k = 5000, 128, 10
    base = 64 * 1_000_000
    rows = orc.synth_rows(91, 0, n, d, 0)
    q = orc.synth_rows(92, 0, 1, d, 0)[0]
    c = Corpus(ctx, kind, METRIC_L2, d, n, id_base=base)
    c.upsert(np.arange(base, base + n, dtype=np.uint64), rows)
    rng = np.random.default_rng(1)
    inside = np.sort(rng.choice(np.arange(base + 100, base + 4900), 300, replace=False)).astype(np.uint64)
    outside = np.array([0, 5, base - 1, base + n, base + n + 64, 3 * base], np.uint64)
    bm = allow_bitmap(np.concatenate([inside, outside]), n_bits=4 * base)
    ids, dists, counts = c.search(q, k, bm)
    if kind == KIND_F32:
        all_d = orc.dist_all(0, q, rows)
    else:
        all_d = orc.bq_dist_all(orc.bq_encode(q), np.stack([orc.bq_encode(r) for r in rows]))
    sl = (inside - base).astype(np.int64)
    wi, wd = orc.lex_topk(all_d[sl], inside, k)
    assert counts[0] == k and np.array_equal(ids[0], wi) and np.array_equal(bits(dists[0]), bits(wd))
    # ids only outside this corpus -> empty; a bitmap that ends before the corpus -> empty
    for bm2 in (allow_bitmap(outside, n_bits=4 * base), allow_bitmap([3, 64], n_bits=128)):
        assert c.search(q, k, bm2)[2][0] == 0
    # k > 256 (select path) with the same window
    ids, dists, counts = c.search(q, 290, bm)
    wi, wd = orc.lex_topk(all_d[sl], inside, 290)
    assert counts[0] == 290 and np.array_equal(ids[0], wi)


def test_pq_codebook_shape_and_code_validation(ctx, orc):
    d, m, ks = 64, 16, 16
    c = Corpus(ctx, KIND_PQ, METRIC_L2, d, 640)
    centers = orc.synth_rows(7, 0, m * ks, d // m, 0).reshape(m, ks, d // m)
    c.set_codebook(centers)
    codes = (np.arange(10 * m) % ks).astype(np.uint8).reshape(10, m)
    c.upsert_codes(np.arange(10, dtype=np.uint64), codes)
    with pytest.raises(_lib.WvgError, match="cannot change centroids"):
        c.set_codebook(orc.synth_rows(8, 0, m * 8, d // m, 0).reshape(m, 8, d // m))
    bad = codes.copy()
    bad[3, 5] = ks  # indexes past the m x ks LUT
    with pytest.raises(_lib.WvgError, match="not below centroids"):
        c.upsert_codes(np.arange(20, 30, dtype=np.uint64), bad)
    assert c.info()[0] == 10  # the rejected call stored nothing
    c.set_codebook(centers)  # same shape: allowed


def test_merge_packed_equals_merge_device(ctx, orc):
    import torch

    from weaviate_amd.shard import pack_block

    lib = _lib.load()
    dev = torch.device("cuda:0")
    G, nq, k = 8, 5, 100
    rng = np.random.default_rng(11)
    d = np.floor(rng.uniform(0, 40, (G, nq, k))).astype(np.float32)
    ids = rng.permutation(G * nq * k).reshape(G, nq, k).astype(np.uint64)
    ids[2, 1, 50:] = NONE
    d[2, 1, 50:] = np.inf
    packed = torch.from_numpy(np.concatenate([pack_block(ids[g], d[g]) for g in range(G)])).to(dev)
    outs = []
    for packed_call in (False, True):
        oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
        od = torch.empty((nq, k), dtype=torch.float32, device=dev)
        oc = torch.empty(nq, dtype=torch.int32, device=dev)
        if packed_call:
            _lib.check(lib.wvg_topk_merge_packed(ctx.handle, packed.data_ptr(), nq, G, k, k, oi.data_ptr(),
                                                 od.data_ptr(), oc.data_ptr(), None))
        else:
            td = torch.from_numpy(d).to(dev)
            ti = torch.from_numpy(ids.view(np.int64)).to(dev)
            _lib.check(lib.wvg_topk_merge_device(ctx.handle, td.data_ptr(), ti.data_ptr(), nq, G, k, k,
                                                 oi.data_ptr(), od.data_ptr(), oc.data_ptr(), None))
        torch.cuda.synchronize()
        outs.append((oi.cpu().numpy().view(np.uint64), od.cpu().numpy(), oc.cpu().numpy()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(bits(outs[0][1]), bits(outs[1][1]))
    for qi in range(nq):
        live = ids[:, qi, :] != NONE
        wi, wd = orc.lex_topk(d[:, qi, :][live], ids[:, qi, :][live], k)
        assert np.array_equal(outs[1][0][qi], wi) and np.array_equal(bits(outs[1][1][qi]), bits(wd))


def test_cache_reuse_scan_order_does_not_change_results(ctx, orc):
    """With wvg_options.cache_reuse (the default) consecutive scans alternate
    direction and read their tail with the default cache policy; with it off
    every scan walks upwards with non-temporal loads.  The lexicographic top-k
    does not depend on the order rows are visited, so every call gives the
    same bits in both contexts -- K1 (host API, query-stream kernel), K8e
    (PQ m = 32) and the BQ scan, three calls in a row each."""
    import torch

    from weaviate_amd.device import Context

    lib = _lib.load()
    n, d, k = 70_000 + 13, 128, 10
    qs = orc.synth_rows(77, 0, 5, d, 0)
    dev = torch.device("cuda:0")
    tq = torch.from_numpy(qs).to(dev)

    def build(cx):
        f = Corpus(cx, KIND_F32, METRIC_L2, d, n)
        f.fill_synthetic(76, n, 0)
        f.delete(np.array([3, 64, 69_999], np.uint64))
        pq = Corpus(cx, KIND_PQ, METRIC_DOT, d, n)
        pq.set_codebook(orc.synth_rows(78, 0, 32 * 256, 4, 0).reshape(32, 256, 4))
        _lib.check(lib.wvg_pq_encode_corpus(pq.handle, f.handle))
        bq = Corpus(cx, KIND_BQ, METRIC_COSINE, d, n)
        bq.fill_synthetic(76, n, 0)
        return f, pq, bq

    def run_all(f, pq, bq):
        ws = torch.zeros(lib.wvg_search_workspace_size(f.handle, 5, k), dtype=torch.uint8, device=dev)

        def device_stream():
            oi = torch.empty((5, k), dtype=torch.int64, device=dev)
            od = torch.empty((5, k), dtype=torch.float32, device=dev)
            oc = torch.empty(5, dtype=torch.int32, device=dev)
            _lib.check(lib.wvg_search_device_pipelined(f.handle, tq.data_ptr(), 5, k, oi.data_ptr(),
                                                       od.data_ptr(), oc.data_ptr(), ws.data_ptr(), ws.numel(),
                                                       torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            return oi.cpu().numpy(), od.cpu().numpy()

        out = []
        for rep in range(3):  # consecutive calls: directions alternate between them
            out.append(f.search(qs, k))
            out.append(pq.search(qs[rep], 20))
            out.append(bq.search(qs[rep], 30))
            out.append(device_stream())
        return out

    streaming = Context(0, cache_reuse=0)
    try:
        cs = build(streaming)
        want = run_all(*cs)
        for c in cs:
            c.destroy()
        cr = build(ctx)
        got = run_all(*cr)
        got2 = run_all(*cr)
        for c in cr:
            c.destroy()
    finally:
        streaming.close()
    for a_, b_, c_ in zip(want, got, got2):
        for x, y, z in zip(a_, b_, c_):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(z).view(np.uint8))


def test_pinned_host_buffers(ctx, orc):
    """wvg_host_alloc buffers go straight to the copies (no staging copy); the
    results equal those from ordinary (pageable) host memory."""
    import ctypes as ct

    from weaviate_amd._lib import METRIC_COSINE, METRIC_L2, check, fptr, u32ptr, u64ptr

    lib = ctx.lib
    R, d, k = 200, 1536, 10
    ids = np.arange(7000, 7000 + R, dtype=np.uint64)
    rows = np.empty((R, d), np.float32)
    check(lib.wvg_synthetic_rows(ctx.handle, 42, u64ptr(ids), R, d, 0, 1, fptr(rows)))
    pinned = ctx.host_array((R, d), np.float32)
    try:
        check(lib.wvg_synthetic_rows(ctx.handle, 42, u64ptr(ids), R, d, 0, 1, fptr(pinned)))  # D2H into it
        assert np.array_equal(pinned.view(np.uint32), rows.view(np.uint32))
        q = orc.normalize(orc.synth_rows(43, 0, 1, d, 0)[0])
        outs = []
        for src in (rows, pinned):
            oi, od, oc = np.empty(k, np.uint64), np.empty(k, np.float32), np.zeros(1, np.uint32)
            check(lib.wvg_rescore(ctx.handle, METRIC_COSINE, fptr(q), fptr(src), u64ptr(ids), R, d, k, u64ptr(oi),
                                  fptr(od), u32ptr(oc)))
            outs.append((oi.copy(), od.view(np.uint32).copy(), int(oc[0])))
        assert outs[0][2] == k and np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
        d1, d2 = np.empty(R, np.float32), np.empty(R, np.float32)
        check(lib.wvg_distance_batch(ctx.handle, METRIC_L2, fptr(q), fptr(rows), R, d, fptr(d1)))
        check(lib.wvg_distance_batch(ctx.handle, METRIC_L2, fptr(q), fptr(pinned), R, d, fptr(d2)))
        assert np.array_equal(d1.view(np.uint32), d2.view(np.uint32))
        want = orc.dist_all(orc.L2, q, rows)
        assert np.array_equal(d1.view(np.uint32), np.asarray(want, np.float32).view(np.uint32))
    finally:
        ctx.free_host_array(pinned)
    check(lib.wvg_host_free(ctx.handle, None))  # null is a no-op
    p = ct.c_void_p()
    check(lib.wvg_host_alloc(ctx.handle, 0, ct.byref(p)))
    assert not p.value


@pytest.mark.parametrize("kind", [KIND_F32, KIND_BQ, KIND_PQ])
def test_cosched_batches_equal_single_queries(ctx, orc, kind):
    """Co-scheduled batches (K1 / K5 / K8e COS: the nq queries of a row range on one
    XCD, workgroup id -> (range, query)) return exactly what one query per
    call returns.  nq = 2 .. 300 covers the range-count floor of
    pq_cosched_groups (8 ranges once nq >= num_cus / 8, where the queries of
    a range are no longer all resident together), k = 256 the E = 4 top-k
    (where the 16-wave PQ image does not fit and 8 waves run), and the BQ
    batch also goes through searchByVectorBQ's rescore flow."""
    from weaviate_amd.device import search_bq_rescore

    n, d = 50_000 + 37, 128
    rows = orc.synth_rows(600, 0, n, d, 0)
    c = Corpus(ctx, kind, METRIC_L2, d, n)
    f = None
    if kind == KIND_PQ:
        centers = orc.synth_rows(601, 0, 32 * 256, d // 32, 0).reshape(32, 256, d // 32)
        c.set_codebook(centers)
    elif kind == KIND_BQ:
        f = Corpus(ctx, KIND_F32, METRIC_L2, d, n)
        f.upsert(np.arange(n, dtype=np.uint64), rows)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    dead = np.arange(5, n, 97, dtype=np.uint64)
    c.delete(dead)
    if f is not None:
        f.delete(dead)
    qs_all = orc.synth_rows(602, 0, 300, d, 0)
    allow = allow_bitmap(np.arange(3, n, 5, dtype=np.uint64)) if kind == KIND_F32 else None
    try:
        for nq, ks in [(2, (10, 256)), (12, (10, 100, 200)), (40, (10, 256)), (300, (10,))]:
            qs = qs_all[:nq]
            for k in ks:
                for al in ((None, allow) if allow is not None and nq <= 12 else (None,)):
                    singles = [c.search(qs[i], k, al) for i in range(nq)]
                    ids, dists, counts = c.search(qs, k, al)
                    for i, (si, sd, sc) in enumerate(singles):
                        assert counts[i] == sc[0]
                        assert np.array_equal(ids[i], si[0]) and np.array_equal(bits(dists[i]), bits(sd[0]))
            if f is not None and nq <= 40:
                single = [search_bq_rescore(c, f, qs[i], 10, 200) for i in range(nq)]
                bi, bd, bc = search_bq_rescore(c, f, qs, 10, 200)
                for i, (si, sd, sc) in enumerate(single):
                    assert bc[i] == sc[0] and np.array_equal(bi[i], si[0]) and np.array_equal(bits(bd[i]), bits(sd[0]))
    finally:
        c.destroy()
        if f is not None:
            f.destroy()
