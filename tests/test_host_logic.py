"""CPU tests of host-side logic that needs no GPU: the selection rules of
IndexQueue.bruteForce (adapters/repos/db/index_queue.go:676-719) driven by a
stand-in provider whose distances come from the oracle."""
import numpy as np

from weaviate_amd import index_queue
from weaviate_amd.flat import AllowList


class _OracleProvider:
    """Test double for distancer.Provider: Type() + BatchDist from the oracle."""

    def __init__(self, orc, metric, name):
        self.orc, self.metric, self.name = orc, metric, name
        self.ctx = None

    def Type(self):
        return self.name

    def BatchDist(self, q, X):
        return self.orc.dist_all(self.metric, q, X)


def test_brute_force_selection_rules(orc):
    prov = _OracleProvider(orc, 0, "l2-squared")
    ids = np.arange(10, 20, dtype=np.uint64)
    V = np.arange(10, dtype=np.float32)[:, None] * np.ones((1, 4), np.float32)  # dist = 4 * i^2
    q = np.zeros(4, np.float32)
    # k < 0 keeps everything that passes the filters
    got_i, got_d = index_queue.brute_force(prov, q, ids, V, -1)
    assert got_i.tolist() == list(range(10, 20))
    assert got_d.tolist() == [4.0 * i * i for i in range(10)]
    # seen and allow list skip rows; max_distance drops rows beyond it
    got_i, _ = index_queue.brute_force(prov, q, ids, V, -1, allow=AllowList(*range(10, 20, 2)),
                                       max_distance=64.0, seen={12})
    assert got_i.tolist() == [10, 14]
    # k bounds the heap; existing results take part
    got_i, got_d = index_queue.brute_force(prov, q, ids, V, 3, results=([99], [2.0]))
    assert got_i.tolist() == [10, 99, 11]
    assert got_d.tolist() == [0.0, 2.0, 4.0]
    # a row tied with the top of a full heap does not enter it (strict <)
    got_i, _ = index_queue.brute_force(prov, q, ids[1:2], V[1:2], 1, results=([77], [4.0]))
    assert got_i.tolist() == [77]
    # max_distance <= 0 disables the filter
    assert len(index_queue.brute_force(prov, q, ids, V, -1, max_distance=0.0)[0]) == 10
