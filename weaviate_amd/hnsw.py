"""The HNSW index's brute-force consumers of the scoring path, on the GPU
(SURVEY.md §8f row 1).  The graph walk itself stays in Go; these are the
loops in it that score many stored vectors against one query:

* ``flat_search`` -- ``hnsw.flatSearch`` (V/hnsw/flat_search.go:19-79), taken
  when the allow list is small (< flatSearchCutoff, V/hnsw/search.go:70): the
  exact top-``limit`` of the allowed, live nodes.  One ``wvg_search`` with the
  allow list as a docID bitmap; nodes past the corpus (``candidate >=
  nodeSize``) and tombstoned / deleted nodes are skipped by the validity
  bitmap, as the reference skips them.
* ``rescore`` -- the rescore block of ``searchByVectorDistance`` / ``knnSearchByVector``
  (V/hnsw/search.go:564-597): exact float distances of the ef candidates the
  compressed walk found (``distanceFromBytesToFloatNode``), keep ef, then k.
  One ``wvg_corpus_distance_by_ids`` over the candidates' device rows;
  ``rescore_batch`` does the loop for many concurrent queries in one launch
  (``wvg_corpus_distance_by_ids_batch``).

Both work on a ``Corpus`` that mirrors the HNSW node vectors (F32), or its
compressed codes (BQ / PQ: ``distBetweenNodeAndVec`` with the compressor's
distancer).  Results are ascending by (distance, docID).
"""
from __future__ import annotations

import numpy as np

from .device import Corpus, allow_bitmap


def _lex_smallest(ids: np.ndarray, dists: np.ndarray, k: int):
    """Ascending (distance, id) order of the k smallest; distances compare as
    float32 with -0 == +0 and NaN last, as the device keys order them."""
    order = np.lexsort((ids, np.where(np.isnan(dists), np.inf, dists), np.isnan(dists)))[:k]
    return ids[order], dists[order]


def flat_search(corpus: Corpus, query, limit: int, allow_ids):
    """hnsw.flatSearch (V/hnsw/flat_search.go:19-79)."""
    if limit < 0:
        raise ValueError("k must be >= 0")  # V/hnsw/search.go:486-488
    ids = np.asarray(sorted(int(i) for i in allow_ids), dtype=np.uint64)
    if limit == 0 or ids.size == 0:
        return np.empty(0, dtype=np.uint64), np.empty(0, dtype=np.float32)
    got, dists, counts = corpus.search(query, limit, allow_bitmap(ids))
    n = int(counts[0])
    return got[0, :n], dists[0, :n]


def rescore(corpus: Corpus, query, candidate_ids, k: int, ef: int | None = None):
    """The HNSW rescore loop (V/hnsw/search.go:564-597): exact distances of the
    candidates from the float rows (``DistanceToFloat`` = SingleDist of the
    query and the stored, normalized-for-cosine row, search.go:428-444), the
    best ef kept (``res.Len() > ef`` pops), then the best k, ascending.

    A candidate whose object is gone comes back from
    ``distanceFromBytesToFloatNode`` as ``(0, false, nil)`` and the loop
    ignores ``ok``, so the reference re-inserts it at distance 0; the mirror
    does the same (``ok == false`` -> 0.0)."""
    cand = np.asarray(candidate_ids, dtype=np.uint64)
    if cand.size == 0 or k <= 0:
        return np.empty(0, dtype=np.uint64), np.empty(0, dtype=np.float32)
    dists, ok = corpus.distance_by_ids(query, cand)
    dists = np.where(ok, dists, np.float32(0.0)).astype(np.float32)
    keep = min(k, ef if ef is not None else cand.size)
    return _lex_smallest(cand, dists, keep)


def rescore_batch(corpus: Corpus, queries, candidate_lists, k: int, ef: int | None = None):
    """``rescore`` for many queries (each with its own candidate list) with ONE
    device launch: the serving shape, where concurrent HNSW searches reach
    their rescore step together.  Same per-query semantics as ``rescore``."""
    lists = [np.asarray(c, dtype=np.uint64).reshape(-1) for c in candidate_lists]
    q = np.asarray(queries, dtype=np.float32).reshape(len(lists), -1)
    empty = (np.empty(0, dtype=np.uint64), np.empty(0, dtype=np.float32))
    if k <= 0:
        return [empty for _ in lists]
    out = []
    for cand, (dists, ok) in zip(lists, corpus.distance_by_ids_batch(q, lists)):
        if cand.size == 0:
            out.append(empty)
            continue
        dists = np.where(ok, dists, np.float32(0.0)).astype(np.float32)
        keep = min(k, ef if ef is not None else cand.size)
        out.append(_lex_smallest(cand, dists, keep))
    return out
