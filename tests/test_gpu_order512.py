"""The AVX-512 reduction-order mode (wvg_set_distance_order): on hosts with
AMX-BF16 + AVX-512 Weaviate's init() dispatches l2_512 / dot_512
(D/l2_amd64.go:19-25, D/dot_product_amd64.go:19-25; kernels
D/c/l2_avx512_amd64.c, D/c/dot_avx512_amd64.c).  With the mode on, every fp32
distance of the context must equal those kernels' outputs bit for bit:
checked against the reference's own compiled l2_512 / dot_512 outputs
(tests/golden/distances.npz, lengths 1..1536) and, through the scans, the
rescore and DistanceToNode, against the oracle's 512 restatement (itself
pinned to the same golden outputs in tests/test_oracle.py)."""
import os

import numpy as np
import pytest

from weaviate_amd import _lib
from weaviate_amd._lib import KIND_BQ, KIND_F32, METRIC_COSINE, METRIC_DOT, METRIC_L2, ORDER_AVX256, ORDER_AVX512
from weaviate_amd.device import Corpus, allow_bitmap, search_bq_rescore

from test_gpu_parity import ORC_METRIC, bits, check_topk, prep_query, stored_rows

pytestmark = pytest.mark.gpu


@pytest.fixture
def ctx512(ctx):
    ctx.set_distance_order(ORDER_AVX512)
    yield ctx
    ctx.set_distance_order(ORDER_AVX256)


def test_distance_batch_bitexact_vs_reference_512_kernels(ctx512):
    from weaviate_amd.distancer import CosineDistanceProvider, DotProductProvider, L2SquaredProvider

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "distances.npz"))
    l2p, dp, cp = L2SquaredProvider(ctx512), DotProductProvider(ctx512), CosineDistanceProvider(ctx512)
    off = 0
    got = {"l2": [], "dot": [], "cos": []}
    for n in g["lens"]:
        a, b = g["a"][off:off + n], g["b"][off:off + n]
        off += n
        got["l2"].append(l2p.BatchDist(a, b[None])[0])
        got["dot"].append(dp.BatchDist(a, b[None])[0])
        got["cos"].append(cp.BatchDist(a, b[None])[0])
    assert np.array_equal(bits(got["l2"]), bits(g["l2_512"]))
    assert np.array_equal(bits(got["dot"]), bits(-g["dot_512"]))
    assert np.array_equal(bits(got["cos"]), bits(np.float32(1) - g["dot_512"]))
    # and the orders really differ somewhere (the mode is not a no-op)
    assert not np.array_equal(bits(g["dot_512"]), bits(g["dot_256"]))


def test_invalid_order_rejected(ctx):
    with pytest.raises(_lib.WvgError, match="unknown distance order"):
        ctx.set_distance_order(7)


@pytest.mark.parametrize("metric", [METRIC_L2, METRIC_DOT, METRIC_COSINE])
@pytest.mark.parametrize("d", [100, 128, 300, 768])
def test_flat_search_512_order(ctx512, orc, metric, d):
    n, nq = 3000 + 11, 40  # 40 queries: the batched path (K1 here, not the MFMA kernel)
    rows = orc.synth_rows(800 + d, 0, n, d, 0)
    qs = orc.synth_rows(801 + d, 0, nq, d, 0)
    c = Corpus(ctx512, KIND_F32, metric, d, n)
    c.upsert(np.arange(n, dtype=np.uint64), rows)
    c.delete(np.array([5, 64, 3000], np.uint64))
    valid = np.ones(n, np.uint8)
    valid[[5, 64, 3000]] = 0
    srows = stored_rows(orc, metric, rows)
    for k in (10, 300):  # fused top-k and the select path
        ids, dists, counts = c.search(qs if k == 10 else qs[:2], k)
        for qi in range(0, len(ids), 7):
            all_d = orc.dist_all_512(ORC_METRIC[metric], prep_query(orc, metric, qs[qi]), srows)
            check_topk(orc, ids[qi], dists[qi], counts[qi], all_d, np.arange(n, dtype=np.uint64), k, valid)
    # DistanceToNode by docID
    q = prep_query(orc, metric, qs[0])
    dd, ok = c.distance_by_ids(qs[0], np.array([0, 5, 17, 2999], np.uint64))
    want = orc.dist_all_512(ORC_METRIC[metric], q, srows[[0, 17, 2999]])
    assert ok.tolist() == [True, False, True, True]
    assert np.array_equal(bits(dd[ok]), bits(want))
    c.destroy()


def test_bq_rescore_and_host_rescore_512_order(ctx512, orc):
    import ctypes

    n, d, k, R = 5000, 768, 10, 200
    rows = orc.synth_rows(811, 0, n, d, 0)
    q = orc.synth_rows(812, 0, 1, d, 0)[0]
    f = Corpus(ctx512, KIND_F32, METRIC_DOT, d, n)
    b = Corpus(ctx512, KIND_BQ, METRIC_DOT, d, n)
    f.upsert(np.arange(n, dtype=np.uint64), rows)
    b.upsert(np.arange(n, dtype=np.uint64), rows)
    ids, dists, counts = search_bq_rescore(b, f, q, k, R)
    codes = np.stack([orc.bq_encode(r) for r in rows])
    cand, _ = orc.bq_heap_pops(codes, orc.bq_encode(q), R)  # the reference heap's pop order
    exact = orc.dist_all_512(1, q, rows[cand.astype(np.int64)])
    li, ld = orc.heap_topk(exact, cand, k)
    assert counts[0] == k and np.array_equal(ids[0], li) and np.array_equal(bits(dists[0]), bits(ld))
    # wvg_rescore (candidate rows from the host)
    lib = _lib.load()
    sub = rows[:300]
    oi = np.empty(k, np.uint64)
    od = np.empty(k, np.float32)
    cnt = ctypes.c_uint32()
    _lib.check(lib.wvg_rescore(ctx512.handle, METRIC_DOT, _lib.fptr(q), _lib.fptr(sub),
                               _lib.u64ptr(np.arange(300, dtype=np.uint64)), 300, d, k, _lib.u64ptr(oi),
                               _lib.fptr(od), ctypes.byref(cnt)))
    wi, wd = orc.heap_topk(orc.dist_all_512(1, q, sub), np.arange(300, dtype=np.uint64), k)
    assert np.array_equal(oi, wi) and np.array_equal(bits(od), bits(wd))
    f.destroy()
    b.destroy()


def test_device_stream_search_512_order(ctx512, orc):
    import torch

    lib = _lib.load()
    n, d, k, nq = 20_000 + 5, 256, 10, 6
    c = Corpus(ctx512, KIND_F32, METRIC_L2, d, n)
    c.fill_synthetic(61, n, 0)
    rows = orc.synth_rows(61, 0, n, d, 0)
    qs = orc.synth_rows(62, 0, nq, d, 0)
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
    ids = oi.cpu().numpy().view(np.uint64)
    dd = od.cpu().numpy()
    for qi in range(nq):
        all_d = orc.dist_all_512(0, qs[qi], rows)
        wi, wd = orc.lex_topk(all_d, np.arange(n, dtype=np.uint64), k)
        assert np.array_equal(ids[qi], wi) and np.array_equal(bits(dd[qi]), bits(wd))
    c.destroy()
