"""CPU (gloo, world size 2) test of ShardedFlatIndex.search_device's stream
ordering with an explicit caller stream (adapters/repos/db/index.go:1567-1648
restated in weaviate_amd/shard.py).  The caller's scan, the all-gather (with
its gloo staging copies), the merge and the result allocations must all be
issued on the caller's stream -- not on torch's current stream -- so a side
stream needs no extra synchronisation.  The C ABI is replaced by a recording
stand-in (no GPU here): its "scan" writes a deterministic per-rank block and
its "merge" reads the all-gathered blocks, so the test also checks that the
exchange moved what the scan wrote.  tests/test_gpu_dist.py runs the same
side-stream case through the HIP library on the GPU."""
import contextlib
import ctypes
import os
import socket

import numpy as np
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


class _FakeStream:
    def __init__(self, handle):
        self.cuda_stream = handle


class _Recorder:
    """torch.cuda.stream / ExternalStream stand-ins that record the active stream."""

    def __init__(self):
        self.active = [_FakeStream(0)]  # torch's current stream: handle 0
        self.log = []

    def external(self, handle, device=None):
        return _FakeStream(int(handle))

    @contextlib.contextmanager
    def stream(self, s):
        self.active.append(s)
        try:
            yield
        finally:
            self.active.pop()

    def cur(self):
        return self.active[-1].cuda_stream


def _view(ptr, n, dtype):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dtype))), (n,))


class _FakeLib:
    def __init__(self, rec, rank):
        self.rec, self.rank = rec, rank

    def wvg_search_workspace_size(self, h, nq, k):
        return 4096

    def wvg_topk_packed_bytes(self, nq, k):
        return (nq * k * 12 + 15) // 16 * 16

    def wvg_search_device(self, h, q, nq, k, ids, dd, cnt, ws, wsn, stream):
        self.rec.log.append(("scan", stream, self.rec.cur()))
        _view(ids, nq * k, np.uint64)[:] = np.arange(nq * k, dtype=np.uint64) * 2 + self.rank  # rank r: ids = r mod 2
        _view(dd, nq * k, np.float32)[:] = np.arange(nq * k, dtype=np.float32) + 0.5 * self.rank
        return 0

    wvg_search_device_pipelined = wvg_search_device

    def wvg_topk_merge_packed(self, ctx, packed, nq, nlists, k_in, k, ids, dd, cnt, stream):
        self.rec.log.append(("merge", stream, self.rec.cur()))
        blk = self.wvg_topk_packed_bytes(nq, k_in)
        raw = _view(packed, nlists * blk, np.uint8).copy()
        ri = np.stack([raw[r * blk:r * blk + nq * k_in * 8].view(np.uint64) for r in range(nlists)])
        rd = np.stack([raw[r * blk + nq * k_in * 8:r * blk + nq * k_in * 12].view(np.float32) for r in range(nlists)])
        out_i, out_d = _view(ids, nq * k, np.uint64), _view(dd, nq * k, np.float32)
        for qi in range(nq):
            cand = sorted(zip(rd[:, qi * k_in:(qi + 1) * k_in].ravel(), ri[:, qi * k_in:(qi + 1) * k_in].ravel()))
            for j in range(k):
                out_d[qi * k + j], out_i[qi * k + j] = cand[j]
        _view(cnt, nq, np.int32)[:] = k
        return 0


class _Ctx:
    def __init__(self, lib):
        self.lib, self.handle = lib, 1


class _Corpus:
    handle = 2


def _worker(rank, world, port, out):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from weaviate_amd import shard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rec = _Recorder()
        shard.torch.cuda.stream = rec.stream
        shard.torch.cuda.ExternalStream = rec.external
        orig_ag = shard.all_gather_packed

        def ag(send, recv, group=None):
            rec.log.append(("all_gather", None, rec.cur()))
            return orig_ag(send, recv, group)

        shard.all_gather_packed = ag
        idx = shard.ShardedFlatIndex(_Ctx(_FakeLib(rec, rank)), _Corpus())
        nq, k = 3, 4
        q = torch.zeros((nq, 8), dtype=torch.float32)
        ids, dists, counts = idx.search_device(q, k, stream=0xABC)
        out.put((rank, rec.log, ids.numpy().view(np.uint64).copy(), dists.numpy().copy()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_side_stream_orders_scan_allgather_merge():
    world = 2
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, log, ids, dists = q.get(timeout=120)
        got[r] = (log, ids, dists)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        log, ids, dists = got[r]
        assert [e[0] for e in log] == ["scan", "all_gather", "merge"]
        for name, passed, active in log:
            assert active == 0xABC, (name, active)  # every step issued inside the caller's stream
            if passed is not None:
                assert passed == 0xABC, (name, passed)  # the raw handle handed to the C ABI
        # the merge saw both ranks' blocks: for query 0 the k smallest of
        # {2i + r | dist i + r/2} interleave the two ranks
        assert ids[0].tolist() == [0, 1, 2, 3] and dists[0].tolist() == [0.0, 0.5, 1.0, 1.5]
