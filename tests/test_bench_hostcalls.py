"""bench.py's native caller loop (tools/host_calls.c) on CPU: a ctypes callback
stands in for wvg_search; every call gets one query, k, and the allow list of
its index (pointer and word count), latencies are recorded per call, and a
nonzero return code ends the loop and is reported."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEARCH = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)


@pytest.fixture(scope="module")
def bench_mod():
    so = os.path.join(ROOT, "tools", "libhostcalls.so")
    if not os.path.exists(so):
        subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-pthread", os.path.join(ROOT, "tools", "host_calls.c"),
                        "-o", so], check=True)
    import bench

    assert bench._host_calls_lib() is not None
    return bench


class _Lib:
    pass


def test_native_caller_loop_passes_queries_and_allow_lists(bench_mod):
    qs = np.arange(4 * 8, dtype=np.float32).reshape(4, 8)
    allows = [np.full(w, w, np.uint64) for w in (3, 5, 7)]
    seen = []

    def fake(corpus, q, nq, k, allow, words, ids, dists, cnt):
        row = np.ctypeslib.as_array(ctypes.cast(q, ctypes.POINTER(ctypes.c_float)), (8,))
        first = int(np.ctypeslib.as_array(ctypes.cast(allow, ctypes.POINTER(ctypes.c_uint64)), (1,))[0])
        seen.append((int(row[0]) // 8, nq, k, int(words), first))
        return 0

    lib = _Lib()
    lib.wvg_search = SEARCH(fake)
    qps, lat = bench_mod._native_callers(bench_mod._host_calls_lib(), lib, None, qs, 10, 1, 0.05, allows)
    assert len(seen) == len(lat) > 10 and qps > 0 and np.all(lat > 0)
    for i, (qi, nq, k, words, first) in enumerate(seen):
        assert (qi, nq, k) == (i % 4, 1, 10)
        assert words == first == (3, 5, 7)[i % 3]


def test_native_caller_loop_mixed_k(bench_mod):
    seen = []

    def fake(corpus, q, nq, k, allow, words, ids, dists, cnt):
        seen.append(int(k))
        return 0

    lib = _Lib()
    lib.wvg_search = SEARCH(fake)
    bench_mod._native_callers(bench_mod._host_calls_lib(), lib, None, np.zeros((2, 4), np.float32), 5, 1, 0.02,
                              ks=[10, 1, 100])
    assert len(seen) > 6 and seen == [(10, 1, 100)[i % 3] for i in range(len(seen))]


def test_native_caller_loop_reports_errors(bench_mod):
    lib = _Lib()
    lib.wvg_search = SEARCH(lambda *a: -3)
    with pytest.raises(RuntimeError, match="-3"):
        bench_mod._native_callers(bench_mod._host_calls_lib(), lib, None, np.zeros((2, 4), np.float32), 5, 4, 0.02)
