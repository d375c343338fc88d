"""CPU tests of the N > 1 path with world_size 2 over gloo: docID-range
sharding, the all-gather layout [world][nq][k] and the lexicographic merge
reproduce the single-corpus result (the GPU scan and merge kernels are
covered by tests/test_gpu_parity.py; here the oracle stands in for the
per-rank scan, as a checker)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, d, k, nq, out):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import wv_oracle as orc
    from weaviate_amd.shard import all_gather_topk, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, cnt, per = shard_range(n, world, rank)
    assert lo % 64 == 0
    rows = orc.synth_rows(42, lo, cnt, d, 0)  # the slab generated from global ids
    qs = orc.synth_rows(43, 0, nq, d, 0)
    ld = np.full((nq, k), np.inf, np.float32)
    li = np.full((nq, k), np.iinfo(np.uint64).max, np.uint64)
    for qi in range(nq):
        all_d = orc.dist_all(orc.L2, qs[qi], rows)
        ids, dd = orc.lex_topk(all_d, np.arange(lo, lo + cnt, dtype=np.uint64), k)
        li[qi, :len(ids)] = ids
        ld[qi, :len(ids)] = dd
    g = all_gather_topk(torch.from_numpy(ld), torch.from_numpy(li.view(np.int64)))
    assert tuple(g.dists.shape) == (world, nq, k)
    gd = g.dists.numpy()
    gi = g.ids.numpy().view(np.uint64)
    res = []
    for qi in range(nq):
        live = gi[:, qi, :] != np.iinfo(np.uint64).max
        ids, dd = orc.lex_topk(gd[:, qi, :][live], gi[:, qi, :][live], k)
        res.append((ids.tolist(), dd.tolist()))
    if rank == 0:
        out.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 10_007), (2, 130)])
def test_sharded_search_equals_single_corpus(world, n):
    from oracle import wv_oracle as orc

    d, k, nq = 32, 10, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, d, k, nq, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rows = orc.synth_rows(42, 0, n, d, 0)
    qs = orc.synth_rows(43, 0, nq, d, 0)
    for qi in range(nq):
        wi, wd = orc.lex_topk(orc.dist_all(orc.L2, qs[qi], rows), np.arange(n, dtype=np.uint64), k)
        assert res[qi][0] == wi.tolist()
        assert np.array_equal(np.asarray(res[qi][1], np.float32), wd)


def test_shard_range_partitions_exactly():
    from weaviate_amd.shard import shard_range

    for n in [1, 63, 64, 1000, 1_000_000]:
        for world in [1, 2, 4, 8]:
            covered = 0
            prev_end = 0
            for r in range(world):
                lo, cnt, _ = shard_range(n, world, r)
                assert lo % 64 == 0 or cnt == 0
                if cnt:
                    assert lo == prev_end
                    prev_end = lo + cnt
                covered += cnt
            assert covered == n
