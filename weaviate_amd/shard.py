"""One-process-per-GPU sharding of a flat index.

Rows are partitioned by contiguous docID range, one slab per GPU; every rank
scans its slab with the fused K1 scan + top-k, the per-rank (dist, id) lists
are exchanged with ONE all-gather per query batch (RCCL over xGMI when the
process group is "nccl"), and every rank merges them on device.  This is the
device restatement of Index.objectVectorSearch's shard fan-out and merge
(adapters/repos/db/index.go:1567-1648: per-shard top-limit, concatenate,
sort by distance, truncate).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check


def shard_range(n_total: int, world: int, rank: int, align: int = 64):
    """Contiguous docID range [id_base, id_base + count) of `rank`; id_base is a
    multiple of `align` (the 64-row tile) so bitmaps stay word-aligned."""
    per = (n_total + world - 1) // world
    per = (per + align - 1) // align * align
    lo = min(n_total, rank * per)
    hi = min(n_total, lo + per)
    return lo, hi - lo, per


@dataclass
class GatherBuffers:
    dists: torch.Tensor
    ids: torch.Tensor


def all_gather_topk(dists: torch.Tensor, ids: torch.Tensor, group=None) -> GatherBuffers:
    """[nq][k] local lists -> [world][nq][k] (one collective per tensor)."""
    world = dist.get_world_size(group)
    gd = torch.empty((world,) + tuple(dists.shape), dtype=dists.dtype, device=dists.device)
    gi = torch.empty((world,) + tuple(ids.shape), dtype=ids.dtype, device=ids.device)
    dist.all_gather_into_tensor(gd.view(-1), dists.contiguous().view(-1), group=group)
    dist.all_gather_into_tensor(gi.view(-1), ids.contiguous().view(-1), group=group)
    return GatherBuffers(gd, gi)


class ShardedFlatIndex:
    """The local slab of a flat index sharded over the ranks of a process group."""

    def __init__(self, ctx, corpus, group=None):
        self.ctx, self.corpus, self.group = ctx, corpus, group
        self.lib = ctx.lib

    def search_device(self, q: torch.Tensor, k: int, stream=None):
        """q: [nq][dim] float32 on this rank's GPU (normalized for cosine).
        Returns (ids int64 [nq][k] global docIDs, dists [nq][k], counts [nq])."""
        nq = q.shape[0]
        dev = q.device
        stream = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
        dists = torch.empty((nq, k), dtype=torch.float32, device=dev)
        counts = torch.empty(nq, dtype=torch.int32, device=dev)
        ws_bytes = self.lib.wvg_search_workspace_size(self.corpus.handle, nq, k)
        ws = torch.zeros(max(1, ws_bytes), dtype=torch.uint8, device=dev)
        check(self.lib.wvg_search_device(self.corpus.handle, q.data_ptr(), nq, k, ids.data_ptr(), dists.data_ptr(),
                                         counts.data_ptr(), ws.data_ptr(), ws_bytes, stream))
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return ids, dists, counts
        g = all_gather_topk(dists, ids, self.group)
        world = g.dists.shape[0]
        m_ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
        m_d = torch.empty((nq, k), dtype=torch.float32, device=dev)
        m_c = torch.empty(nq, dtype=torch.int32, device=dev)
        check(self.lib.wvg_topk_merge_device(self.ctx.handle, g.dists.data_ptr(), g.ids.data_ptr(), nq, world, k, k,
                                             m_ids.data_ptr(), m_d.data_ptr(), m_c.data_ptr(), stream))
        return m_ids, m_d, m_c


__all__ = ["shard_range", "all_gather_topk", "ShardedFlatIndex", "_lib"]
