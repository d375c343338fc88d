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


def _worker(rank, world, port, n, d, k, nq, dead, pipelined, out):
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
        for rep in range(2):  # the cached workspace / send / recv buffers are reused
            ids, dists, counts = idx.search_device(qs, k, pipelined=pipelined)
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


@pytest.mark.parametrize("n,pipelined", [(20_000 + 37, False), (20_000 + 37, True), (50, False), (50, True)])
def test_two_ranks_packed_allgather_device_merge(orc, n, pipelined):
    """n = 50: rank 1's slab is empty (empty results from the device path)."""
    world, d, k, nq = 2, 64, 10, 5
    dead = [0, 3, 777, 10_111, 20_036]
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_worker, args=(r, world, port, n, d, k, nq, dead, pipelined, q))
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
