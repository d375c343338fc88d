"""``IndexQueue.bruteForce`` (adapters/repos/db/index_queue.go:676-719) with the
distances on the GPU.

While vectors wait in the async indexing queue (up to ~100k), a search scores
them by brute force and merges them into the index's result heap.  The
per-vector ``DistanceBetweenVectors`` calls become one ``wvg_normalize_batch``
(cosine-dot only, index_queue.go:696-700) and one ``wvg_distance_batch`` over
the snapshot; the selection keeps the reference's rules:

* ids already in ``seen`` (indexed meanwhile) and ids outside the allow list
  are skipped;
* ``max_distance > 0`` drops rows with ``dist > max_distance``;
* ``k < 0`` keeps everything; otherwise the result heap holds the k best --
  a row enters a full heap only if strictly closer than its current top
  (``dist < results.Top().Dist``).  Which member of an exact tie at the k-th
  distance survives a pop depends on the heap's insertion history in the
  reference; here the latest inserted goes first.

``results`` is the (ids, dists) content of the heap passed in by the caller
(the index's own hits); the merged content is returned ascending.
"""
from __future__ import annotations

import heapq

import numpy as np

from .distancer import Normalize


def brute_force(provider, vector, snapshot_ids, snapshot_vectors, k: int, results=None, allow=None,
                max_distance: float = 0.0, seen=None):
    ids = np.asarray(snapshot_ids, dtype=np.uint64)
    X = np.ascontiguousarray(snapshot_vectors, dtype=np.float32)
    keep = np.ones(len(ids), dtype=bool)
    if seen:
        keep &= np.array([int(i) not in seen for i in ids], dtype=bool)
    if allow is not None:
        keep &= np.array([allow.Contains(int(i)) for i in ids], dtype=bool)
    ids, X = ids[keep], X[keep]
    dists = np.empty(0, dtype=np.float32)
    if len(ids):
        if provider.Type() == "cosine-dot":
            X = Normalize(provider.ctx, X)
        dists = provider.BatchDist(np.asarray(vector, dtype=np.float32), X)

    # max-heap of (dist, insertion order, id) via negation; mirrors
    # priorityqueue.NewMax + the insert/pop rule of index_queue.go:710-716
    heap: list = []
    order = 0
    if results is not None:
        for i, d in zip(*results):
            heapq.heappush(heap, (-float(d), -order, int(i)))
            order += 1
    for i, d in zip(ids.tolist(), dists.tolist()):
        if max_distance > 0 and d > max_distance:
            continue
        if k < 0 or len(heap) < k or d < -heap[0][0]:
            heapq.heappush(heap, (-d, -order, i))
            order += 1
            if k > 0:
                while len(heap) > k:
                    heapq.heappop(heap)
    out = sorted(((-nd, -no, i) for nd, no, i in heap))
    return (np.asarray([i for _, _, i in out], dtype=np.uint64),
            np.asarray([d for d, _, _ in out], dtype=np.float32))
