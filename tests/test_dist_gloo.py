"""CPU tests of the N > 1 path with world_size 2 over gloo: docID-range
sharding, the packed per-rank block (ids then dists, one all-gather per
batch) and the lexicographic merge reproduce the single-corpus result.  Here
the oracle stands in for the per-rank scan and for the merge, as checkers;
tests/test_gpu_dist.py runs the same exchange with the HIP scan and the
device merge (wvg_topk_merge_packed) on the GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

NONE = np.iinfo(np.uint64).max


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
    from weaviate_amd.shard import all_gather_packed, pack_block, packed_bytes, shard_range, unpack_blocks

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, cnt, per = shard_range(n, world, rank)
    assert lo % 64 == 0
    rows = orc.synth_rows(42, lo, cnt, d, 0)  # the slab generated from global ids
    qs = orc.synth_rows(43, 0, nq, d, 0)
    ld = np.full((nq, k), np.inf, np.float32)
    li = np.full((nq, k), NONE, np.uint64)
    for qi in range(nq):
        if cnt == 0:
            continue
        all_d = orc.dist_all(orc.L2, qs[qi], rows)
        ids, dd = orc.lex_topk(all_d, np.arange(lo, lo + cnt, dtype=np.uint64), k)
        li[qi, :len(ids)] = ids
        ld[qi, :len(ids)] = dd
    send = torch.from_numpy(pack_block(li, ld))
    assert send.numel() == packed_bytes(nq, k) and send.numel() % 16 == 0
    recv = torch.empty(world * send.numel(), dtype=torch.uint8)
    all_gather_packed(send, recv)  # ONE collective per batch
    gi, gd = unpack_blocks(recv.numpy(), world, nq, k)
    assert gi.shape == (world, nq, k)
    assert np.array_equal(gi[rank], li) and np.array_equal(gd[rank].view(np.uint32), ld.view(np.uint32))
    res = []
    for qi in range(nq):
        live = gi[:, qi, :] != NONE
        ids, dd = orc.lex_topk(gd[:, qi, :][live], gi[:, qi, :][live], k)
        res.append((ids.tolist(), dd.tolist()))
    if rank == 0:
        out.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 10_007), (2, 130), (2, 63)])
def test_sharded_search_equals_single_corpus(world, n):
    """n = 63: rank 1 holds no rows and contributes an all-empty block."""
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


def test_pack_roundtrip():
    from weaviate_amd.shard import pack_block, packed_bytes, unpack_blocks

    rng = np.random.default_rng(3)
    for nq, k in [(1, 1), (3, 10), (16, 10), (5, 7)]:
        ids = rng.integers(0, 2**63, (nq, k)).astype(np.uint64)
        ids[0, -1] = NONE
        dd = rng.standard_normal((nq, k)).astype(np.float32)
        blocks = np.concatenate([pack_block(ids, dd), pack_block(ids[::-1].copy(), dd[::-1].copy())])
        assert len(blocks) == 2 * packed_bytes(nq, k)
        gi, gd = unpack_blocks(blocks, 2, nq, k)
        assert np.array_equal(gi[0], ids) and np.array_equal(gi[1], ids[::-1])
        assert np.array_equal(gd[0], dd) and np.array_equal(gd[1], dd[::-1])


def test_packed_bytes_matches_library():
    from weaviate_amd import _lib
    from weaviate_amd.shard import packed_bytes

    lib = _lib.load()
    for nq, k in [(1, 1), (16, 10), (8, 100), (3, 7)]:
        assert lib.wvg_topk_packed_bytes(nq, k) == packed_bytes(nq, k)


def test_shard_range_partitions_exactly():
    from weaviate_amd.shard import shard_range

    for n in [1, 63, 64, 1000, 1_000_000]:
        for world in [1, 2, 4, 8]:
            covered = 0
            prev_end = 0
            for r in range(world):
                lo, cnt, _ = shard_range(n, world, r)
                assert lo % 64 == 0
                if cnt:
                    assert lo == prev_end
                    prev_end = lo + cnt
                covered += cnt
            assert covered == n


def _bcast_worker(rank, world, port, out):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from weaviate_amd.shard import broadcast_codebook

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    centers = np.random.default_rng(5).standard_normal((32, 256, 4)).astype(np.float32) if rank == 1 else None
    cb = broadcast_codebook(centers, src=1)
    out.put((rank, cb))
    dist.barrier()
    dist.destroy_process_group()


def test_codebook_broadcast():
    """The PQ codebook of the source rank reaches every rank bit for bit (shape included)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = np.random.default_rng(5).standard_normal((32, 256, 4)).astype(np.float32)
    for r in range(world):
        assert got[r].shape == (32, 256, 4) and np.array_equal(got[r].view(np.uint32), want.view(np.uint32))
