"""One-process-per-GPU sharding of a flat index.

Rows are partitioned by contiguous docID range, one slab per GPU; every rank
scans its slab with the fused K1 scan + top-k and writes its (id, dist) lists
straight into ONE packed block (ids [nq][k] uint64, then dists [nq][k]
float32; ``wvg_topk_packed_bytes``).  A single all-gather per query batch
(RCCL over xGMI when the process group is "nccl") moves every rank's block,
and every rank merges the [world] blocks on device (``wvg_topk_merge_packed``).
This is the device restatement of Index.objectVectorSearch's shard fan-out
and merge (adapters/repos/db/index.go:1567-1648: per-shard top-limit,
concatenate, sort by distance, truncate).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import check

KEY_NONE = np.iinfo(np.uint64).max


def shard_range(n_total: int, world: int, rank: int, align: int = 64):
    """Contiguous docID range [id_base, id_base + count) of `rank`; id_base is a
    multiple of `align` (the 64-row tile) so bitmaps stay word-aligned."""
    per = (n_total + world - 1) // world
    per = (per + align - 1) // align * align
    lo = rank * per  # aligned even for a rank past the end (count 0)
    hi = min(n_total, lo + per)
    return lo, max(0, hi - lo), per


def packed_bytes(nq: int, k: int) -> int:
    """Size of one rank's packed result block (wvg_topk_packed_bytes)."""
    return (nq * k * 12 + 15) // 16 * 16


def pack_block(ids: np.ndarray, dists: np.ndarray) -> np.ndarray:
    """Host packing of [nq][k] ids / dists into the block layout (tests, tools)."""
    nq, k = ids.shape
    blk = np.zeros(packed_bytes(nq, k), np.uint8)
    blk[:nq * k * 8] = np.ascontiguousarray(ids, np.uint64).view(np.uint8).reshape(-1)
    blk[nq * k * 8:nq * k * 12] = np.ascontiguousarray(dists, np.float32).view(np.uint8).reshape(-1)
    return blk


def unpack_blocks(buf: np.ndarray, nlists: int, nq: int, k: int):
    """[nlists] consecutive packed blocks -> (ids [nlists][nq][k], dists [nlists][nq][k])."""
    blk = packed_bytes(nq, k)
    b = np.ascontiguousarray(buf, np.uint8).reshape(nlists, blk)
    ids = np.ascontiguousarray(b[:, :nq * k * 8]).view(np.uint64).reshape(nlists, nq, k)
    dists = np.ascontiguousarray(b[:, nq * k * 8:nq * k * 12]).view(np.float32).reshape(nlists, nq, k)
    return ids, dists


def all_gather_packed(send: torch.Tensor, recv: torch.Tensor, group=None) -> None:
    """One all-gather of the packed blocks: recv[r * len(send):] = rank r's send.
    With a gloo group and device tensors the exchange is staged through host
    memory (test rehearsals on one GPU); with nccl it is RCCL over xGMI."""
    if send.is_cuda and dist.get_backend(group) == "gloo":
        hr = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_gather_into_tensor(hr, send.cpu(), group=group)
        recv.copy_(hr)
    else:
        dist.all_gather_into_tensor(recv, send, group=group)


def broadcast_codebook(centers, src: int = 0, group=None, device=None) -> np.ndarray:
    """The PQ codebook fitted on rank `src` (ProductQuantizer.Fit,
    CH/product_quantization.go:372-418) sent once to every rank of the group:
    a 3-word shape header then the m*ks*ds float32 centres (32 KiB at m = 32,
    ks = 256, ds = 4) -- two broadcasts per index, RCCL over xGMI with nccl.
    `centers` [m][ks][ds] is read on `src` only; every rank returns the host
    copy.  `device`: where the broadcast tensors live (a GPU for nccl; None =
    host, for gloo)."""
    rank = dist.get_rank(group)
    dev = device if device is not None else torch.device("cpu")
    hdr = torch.zeros(3, dtype=torch.int64, device=dev)
    if rank == src:
        c = np.ascontiguousarray(centers, np.float32)
        if c.ndim != 3:
            raise ValueError("centers must be [m][ks][ds]")
        hdr.copy_(torch.tensor(c.shape, dtype=torch.int64))
    dist.broadcast(hdr, src, group=group)
    m, ks, ds = (int(v) for v in hdr.cpu().tolist())
    buf = (torch.from_numpy(c).to(dev) if rank == src else torch.empty((m, ks, ds), dtype=torch.float32, device=dev))
    dist.broadcast(buf, src, group=group)
    return buf.cpu().numpy()


def compress_slab(pq_corpus, f32_corpus, centers, src: int = 0, group=None, device=None) -> np.ndarray:
    """Sharded PQ compression: the codebook of rank
    `src` is broadcast once, then every rank encodes its own docID slab on its
    GPU (wvg_pq_encode_corpus; V/hnsw/compress.go:98-104 restated per slab) --
    no collective on the encode itself.  Returns the codebook every rank used."""
    cb = broadcast_codebook(centers, src, group, device)
    pq_corpus.set_codebook(cb)
    check(pq_corpus.ctx.lib.wvg_pq_encode_corpus(pq_corpus.handle, f32_corpus.handle))
    return cb


@dataclass
class _Buffers:
    ws: torch.Tensor      # search workspace (zero-filled when allocated)
    send: torch.Tensor    # this rank's packed block
    recv: torch.Tensor    # [world] packed blocks
    counts: torch.Tensor  # local counts


def _stream_obj(stream, dev):
    """(torch stream object, raw hipStream_t) of the caller's stream: torch's
    current stream when `stream` is None, else the raw handle wrapped so torch
    ops (the all-gather, its staging copies, allocations) can run on it."""
    if stream is None:
        s = torch.cuda.current_stream(dev)
        return s, s.cuda_stream
    if isinstance(stream, torch.cuda.Stream):
        return stream, stream.cuda_stream
    return torch.cuda.ExternalStream(int(stream), device=dev), int(stream)


class ShardedFlatIndex:
    """The local slab of a flat index sharded over the ranks of a process group."""

    def __init__(self, ctx, corpus, group=None):
        self.ctx, self.corpus, self.group = ctx, corpus, group
        self.lib = ctx.lib
        self._bufs: dict = {}

    def _buffers(self, nq: int, k: int, dev, world: int) -> _Buffers:
        # The workspace size depends on the corpus's current state (its tile
        # count, how many rows are live), so it is asked for on every call --
        # a host-only computation -- and the cached workspace grows when a
        # grown (or thinned) slab needs more.
        ws_bytes = max(256, self.lib.wvg_search_workspace_size(self.corpus.handle, nq, k))
        key = (nq, k, str(dev), world)
        b = self._bufs.get(key)
        if b is None:
            blk = self.lib.wvg_topk_packed_bytes(nq, k)
            b = _Buffers(ws=torch.zeros(ws_bytes, dtype=torch.uint8, device=dev),
                         send=torch.empty(blk, dtype=torch.uint8, device=dev),
                         recv=torch.empty(world * blk, dtype=torch.uint8, device=dev),
                         counts=torch.empty(nq, dtype=torch.int32, device=dev))
            self._bufs[key] = b
        elif b.ws.numel() < ws_bytes:
            b.ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
        return b

    def search_device(self, q: torch.Tensor, k: int, stream=None, pipelined: bool = False):
        """q: [nq][dim] float32 on this rank's GPU (normalized for cosine).
        Returns (ids int64 [nq][k] global docIDs, dists [nq][k], counts [nq]).
        stream: the stream every step runs on (a torch.cuda.Stream or a raw
        hipStream_t; None = torch's current stream): the scan, the all-gather
        (and, over gloo, its host staging copies), the merge and the result
        allocations are all ordered on it, so a caller's side stream needs no
        extra synchronisation.  pipelined: nq independent single-query scans
        in one launch (wvg_search_device_pipelined) instead of one batched
        search."""
        nq = q.shape[0]
        dev = q.device
        s_obj, s_raw = _stream_obj(stream, dev)
        grouped = dist.is_initialized()  # a group of any size (one included) exchanges through it
        world = dist.get_world_size(self.group) if grouped else 1
        fn = self.lib.wvg_search_device_pipelined if pipelined else self.lib.wvg_search_device
        with torch.cuda.stream(s_obj):
            b = self._buffers(nq, k, dev, world)
            if not grouped:
                ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
                dists = torch.empty((nq, k), dtype=torch.float32, device=dev)
                counts = torch.empty(nq, dtype=torch.int32, device=dev)
                check(fn(self.corpus.handle, q.data_ptr(), nq, k, ids.data_ptr(), dists.data_ptr(),
                         counts.data_ptr(), b.ws.data_ptr(), b.ws.numel(), s_raw))
                return ids, dists, counts
            # local lists straight into the packed block: ids at byte 0, dists at nq*k*8
            check(fn(self.corpus.handle, q.data_ptr(), nq, k, b.send.data_ptr(), b.send.data_ptr() + nq * k * 8,
                     b.counts.data_ptr(), b.ws.data_ptr(), b.ws.numel(), s_raw))
            all_gather_packed(b.send, b.recv, self.group)  # ordered after the scan on s_obj
            m_ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
            m_d = torch.empty((nq, k), dtype=torch.float32, device=dev)
            m_c = torch.empty(nq, dtype=torch.int32, device=dev)
            check(self.lib.wvg_topk_merge_packed(self.ctx.handle, b.recv.data_ptr(), nq, world, k, k,
                                                 m_ids.data_ptr(), m_d.data_ptr(), m_c.data_ptr(), s_raw))
            return m_ids, m_d, m_c

    def check(self, stream=None) -> None:
        """wvg_search_device_check over every workspace this index used."""
        for (nq, k, dev, world), b in self._bufs.items():
            st = stream if stream is not None else torch.cuda.current_stream(b.ws.device).cuda_stream
            check(self.lib.wvg_search_device_check(self.ctx.handle, b.ws.data_ptr(), st))


__all__ = ["shard_range", "packed_bytes", "pack_block", "unpack_blocks", "all_gather_packed", "broadcast_codebook",
           "compress_slab", "ShardedFlatIndex", "_lib"]
