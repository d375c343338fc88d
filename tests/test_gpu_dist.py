"""Multi-process GPU test of the sharded path: two ranks on cuda:0 over a gloo
group (the box has one GPU; the product path uses nccl = RCCL), each holding
its docID slab in HBM.  Every rank runs the HIP scan into its packed block,
the blocks are all-gathered once, and every rank merges them with
wvg_topk_merge_packed -- the device restatement of Index.objectVectorSearch's
shard merge (adapters/repos/db/index.go:1644-1648).  Checked against the
oracle over the whole corpus (lexicographic (distance, docID) top-k)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, d, k, nq, dead, pipelined, side, out, backend="gloo"):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist

    torch.cuda.init()
    from weaviate_amd._lib import KIND_F32, METRIC_L2
    from weaviate_amd.device import Context, Corpus
    from weaviate_amd.shard import ShardedFlatIndex, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":  # RCCL: the device all-gather of the product path (one rank per GPU)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, cnt, per = shard_range(n, world, rank)
        ctx = Context(0)
        c = Corpus(ctx, KIND_F32, METRIC_L2, d, max(cnt, 0), id_base=lo)
        if cnt:
            c.fill_synthetic(42, cnt, 0)  # rows of global docIDs lo .. lo+cnt-1
            mine = np.array([i for i in dead if lo <= i < lo + cnt], np.uint64)
            if len(mine):
                c.delete(mine)
        rng = np.random.default_rng(43)
        qs = torch.from_numpy(rng.uniform(-1, 1, (nq, d)).astype(np.float32)).cuda()
        idx = ShardedFlatIndex(ctx, c)
        res = []
        st = torch.cuda.Stream() if side else None
        for rep in range(2):  # the cached workspace / send / recv buffers are reused
            # side: every step on the caller's own stream -- a raw hipStream_t,
            # then the torch.cuda.Stream -- while torch's current stream stays
            # the default one (the all-gather and merge must order on it too)
            s_arg = None if st is None else (st.cuda_stream if rep == 0 else st)
            ids, dists, counts = idx.search_device(qs, k, stream=s_arg, pipelined=pipelined)
            if st is not None:
                st.synchronize()
            torch.cuda.synchronize()
            res.append((ids.cpu().numpy().view(np.uint64).copy(), dists.cpu().numpy().copy(),
                        counts.cpu().numpy().copy()))
        idx.check()
        assert np.array_equal(res[0][0], res[1][0])
        out.put((rank, res[0]))
        c.destroy()
        ctx.close()
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("n,pipelined,side", [(20_000 + 37, False, False), (20_000 + 37, True, False), (50, False, False),
                                             (50, True, False), (20_000 + 37, False, True), (20_000 + 37, True, True)])
def test_two_ranks_packed_allgather_device_merge(orc, n, pipelined, side):
    """n = 50: rank 1's slab is empty (empty results from the device path)."""
    _run_sharded(orc, 2, n, pipelined, side, "gloo")


@pytest.mark.parametrize("pipelined,side", [(False, False), (True, True)])
def test_rccl_group_of_one_packed_allgather(orc, pipelined, side):
    """The nccl (RCCL) backend on the box's one GPU: a process group of one
    rank still takes the exchange path (ShardedFlatIndex exchanges whenever a
    group is initialised), so the device all-gather of the packed block over
    RCCL and wvg_topk_merge_packed run on hardware -- with torch's current
    stream and with a caller side stream -- and equal the oracle."""
    _run_sharded(orc, 1, 20_000 + 37, pipelined, side, "nccl")


def _run_sharded(orc, world, n, pipelined, side, backend):
    d, k, nq = 64, 10, 5
    dead = [0, 3, 777, 10_111, 20_036]
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_worker, args=(r, world, port, n, d, k, nq, dead, pipelined, side, q, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, v = q.get(timeout=240)
        got[r] = v
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rows = orc.synth_rows(42, 0, n, d, 0)
    qs = np.random.default_rng(43).uniform(-1, 1, (nq, d)).astype(np.float32)
    valid = np.ones(n, np.uint8)
    valid[[i for i in dead if i < n]] = 0
    for r in range(world):
        ids, dists, counts = got[r]
        for qi in range(nq):
            all_d = orc.dist_all(orc.L2, qs[qi], rows)
            sel = valid.astype(bool)
            wi, wd = orc.lex_topk(all_d[sel], np.arange(n, dtype=np.uint64)[sel], k)
            assert counts[qi] == len(wi)
            assert np.array_equal(ids[qi][:len(wi)], wi)
            assert np.array_equal(dists[qi][:len(wi)].view(np.uint32), wd.view(np.uint32))
            assert np.all(ids[qi][len(wi):] == np.iinfo(np.uint64).max)


def _pq_worker(rank, world, port, n, d, m, ks, k, nq, out):
    try:
        _pq_worker_body(rank, world, port, n, d, m, ks, k, nq, out)
    except BaseException as e:  # report instead of leaving the parent waiting on the queue
        import traceback

        out.put((rank, "error", traceback.format_exc()))
        raise


def _pq_worker_body(rank, world, port, n, d, m, ks, k, nq, out):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist

    torch.cuda.init()
    from weaviate_amd import _lib
    from weaviate_amd._lib import KIND_F32, KIND_PQ, METRIC_L2
    from weaviate_amd.device import Context, Corpus
    from weaviate_amd.shard import ShardedFlatIndex, compress_slab, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, cnt, per = shard_range(n, world, rank)
        ctx = Context(0)
        f = Corpus(ctx, KIND_F32, METRIC_L2, d, cnt, id_base=lo)
        f.fill_synthetic(52, cnt, 0)
        centers = None
        if rank == 0:  # rank 0 trains on its own slab (KMeans.Fit on the device)
            rows0 = f.get_batch(np.arange(lo, lo + cnt, dtype=np.uint64))[0]
            centers = np.empty((m, ks, d // m), np.float32)
            passes = np.zeros(m, np.uint32)  # [m] Lloyd passes per segment
            _lib.check(ctx.lib.wvg_pq_fit(ctx.handle, _lib.fptr(rows0), cnt, d, m, ks, 0, 7, _lib.fptr(centers),
                                          _lib.u32ptr(passes)))
        pq = Corpus(ctx, KIND_PQ, METRIC_L2, d, cnt, id_base=lo)
        cb = compress_slab(pq, f, centers)
        rng = np.random.default_rng(53)
        qs = torch.from_numpy(rng.uniform(-1, 1, (nq, d)).astype(np.float32)).cuda()
        ids, dists, counts = ShardedFlatIndex(ctx, pq).search_device(qs, k)
        torch.cuda.synchronize()
        codes = pq.get_batch(np.arange(lo, lo + cnt, dtype=np.uint64), pq_m=m)[0]
        out.put((rank, cb, codes, ids.cpu().numpy().view(np.uint64).copy(), dists.cpu().numpy().copy(),
                 counts.cpu().numpy().copy()))
        pq.destroy()
        f.destroy()
        ctx.close()
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_two_ranks_pq_codebook_broadcast_encode_search(orc):
    """Config 4 sharded: rank 0 fits the codebook, one broadcast,
    every rank encodes its slab on the GPU, then the sharded ADC search with
    the packed all-gather + device merge equals the single-corpus oracle."""
    world, n, d, m, ks, k, nq = 2, 6000 + 17, 32, 8, 32, 10, 4
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_pq_worker, args=(r, world, port, n, d, m, ks, k, nq, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        v = q.get(timeout=240)
        assert not (len(v) == 3 and v[1] == "error"), v[2]
        got[v[0]] = v[1:]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    cb = got[0][0]
    assert np.array_equal(got[1][0].view(np.uint32), cb.view(np.uint32))  # the same codebook on every rank
    rows = orc.synth_rows(52, 0, n, d, 0)
    codes = orc.pq_encode(rows, cb)
    assert np.array_equal(np.concatenate([got[0][1], got[1][1]]), codes)  # each slab encoded on its own GPU
    qs = np.random.default_rng(53).uniform(-1, 1, (nq, d)).astype(np.float32)
    for r in range(world):
        ids, dists, counts = got[r][2:]
        for qi in range(nq):
            lut = orc.pq_lut(0, qs[qi], cb)
            all_d = np.array([orc.pq_adc(0, lut, c) for c in codes], np.float32)
            wi, wd = orc.lex_topk(all_d, np.arange(n, dtype=np.uint64), k)
            assert counts[qi] == k and np.array_equal(ids[qi], wi)
            assert np.array_equal(dists[qi].view(np.uint32), wd.view(np.uint32))


def test_sharded_workspace_follows_slab_growth(ctx, orc):
    """ShardedFlatIndex asks for the workspace size on every call: a batch
    (nq >= the MFMA threshold) on a small slab, then the slab grows by 30x,
    then the same batch again -- the grown plan (more K3b row ranges) must
    get a grown workspace, not 'workspace too small'."""
    import torch

    from weaviate_amd._lib import KIND_F32, METRIC_DOT
    from weaviate_amd.device import Corpus
    from weaviate_amd.shard import ShardedFlatIndex

    d, k, nq = 128, 10, 40
    c = Corpus(ctx, KIND_F32, METRIC_DOT, d, 2048)
    try:
        c.fill_synthetic(61, 2048, 0)
        qs = np.random.default_rng(62).uniform(-1, 1, (nq, d)).astype(np.float32)
        idx = ShardedFlatIndex(ctx, c)
        tq = torch.from_numpy(qs).cuda()
        for n in (2048, 60_000):
            if n > 2048:
                c.reserve(n)
                c.fill_synthetic(61, n, 0)
            ids, dists, counts = idx.search_device(tq, k)
            torch.cuda.synchronize()
            ids = ids.cpu().numpy().view(np.uint64)
            dists = dists.cpu().numpy()
            rows = orc.synth_rows(61, 0, n, d, 0)
            for qi in (0, nq - 1):
                wi, wd = orc.lex_topk(orc.dist_all(orc.DOT, qs[qi], rows), np.arange(n, dtype=np.uint64), k)
                assert np.array_equal(ids[qi], wi)
                assert np.array_equal(dists[qi].view(np.uint32), wd.view(np.uint32))
        idx.check()
    finally:
        c.destroy()
