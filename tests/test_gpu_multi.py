"""Several GPUs in one process behind the C ABI (wvg_multi_*, wvg_multi.hip).

Weaviate fans a search out over the shards of one process and merges their
results by distance (adapters/repos/db/index.go:1567-1648).  A multi corpus
deals docIDs to devices in slabs; a search runs each slab's scan on its
device, ONE grouped RCCL all-gather of the packed top-k blocks (or peer
copies when a device repeats), and the merge.  Every result must equal one
plain corpus holding all the rows, bit for bit: ids, distance bits, counts.
The box has one GPU, so devices = [0] exercises the RCCL path (a
one-rank communicator from ncclCommInitAll, the grouped all-gather) and
devices = [0, 0, 0] three slabs with the peer-copy exchange.
"""
import numpy as np
import pytest

from weaviate_amd._lib import (KIND_BQ, KIND_F32, KIND_PQ, METRIC_COSINE, METRIC_DOT, METRIC_L2, WVG_ERR_CAPACITY,
                               WvgError)
from weaviate_amd.device import Corpus, Multi, MultiCorpus, allow_bitmap

pytestmark = pytest.mark.gpu


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def same(a, b):
    (ai, ad, ac), (bi, bd, bc) = a, b
    assert np.array_equal(ac, bc)
    for q in range(len(ac)):
        n = int(ac[q])
        assert np.array_equal(ai[q][:n], bi[q][:n]), q
        assert np.array_equal(bits(ad[q][:n]), bits(bd[q][:n])), q


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
@pytest.mark.parametrize("kind,metric,d", [(KIND_F32, METRIC_L2, 128), (KIND_F32, METRIC_COSINE, 768),
                                           (KIND_BQ, METRIC_COSINE, 256), (KIND_PQ, METRIC_L2, 128)])
def test_multi_search_equals_one_corpus(ctx, orc, devices, kind, metric, d):
    n = 100_000 + 37
    rows = orc.synth_rows(901, 0, n, d, 0)
    qs = orc.synth_rows(902, 0, 40, d, 0)  # 40 queries: the cosine batch takes the bf16 screen
    ref = Corpus(ctx, kind, metric, d, n)
    with Multi(devices) as m:
        assert m.ndev == len(devices)
        assert m.uses_rccl == (len(set(devices)) == len(devices))
        mc = MultiCorpus(m, kind, metric, d, n)
        try:
            if kind == KIND_PQ:
                cb = np.ascontiguousarray(rows[:256].reshape(256, d // 4, 4).transpose(1, 0, 2))
                ref.set_codebook(cb)
                mc.set_codebook(cb)
            ids = np.arange(n, dtype=np.uint64)
            ref.upsert(ids, rows)
            mc.upsert(ids[::-1], rows[::-1])  # any order: routed to the owning slab
            gone = np.arange(3, n, 89, dtype=np.uint64)
            ref.delete(gone)
            mc.delete(gone)
            for k in (1, 10, 100):
                same(mc.search(qs, k), ref.search(qs, k))
            same(mc.search(qs[:1], 10), ref.search(qs[:1], 10))
            # filtered: a 20 % allow list, and one window inside a single slab
            allow = allow_bitmap(np.flatnonzero(np.random.default_rng(3).random(n) < 0.2), n)
            same(mc.search(qs[:5], 10, allow), ref.search(qs[:5], 10, allow))
            win = allow_bitmap(range(n - 500, n), n)
            same(mc.search(qs[:3], 10, win), ref.search(qs[:3], 10, win))
            if len(devices) > 1:
                _, base1, slab = mc.shard(1)
                assert base1 == slab and slab % 64 == 0
        finally:
            mc.destroy()
    ref.destroy()


def test_multi_synthetic_slabs_and_errors(ctx, orc):
    n, d, k = 300_000, 128, 10
    qs = orc.synth_rows(903, 0, 4, d, 0)
    with Multi([0, 0]) as m:
        mc = MultiCorpus(m, KIND_F32, METRIC_DOT, d, n)
        mc.fill_synthetic(42, n, 0)  # every slab keyed by its global docIDs
        ref = Corpus(ctx, KIND_F32, METRIC_DOT, d, n)
        ref.fill_synthetic(42, n, 0)
        same(mc.search(qs, k), ref.search(qs, k))
        with pytest.raises(WvgError) as e:  # beyond the last slab
            mc.upsert(np.array([2 * mc.shard(1)[2]], np.uint64), qs[:1])
        assert e.value.code == WVG_ERR_CAPACITY
        with pytest.raises(WvgError):  # corpora still open
            m.close()
        mc.destroy()
        ref.destroy()
