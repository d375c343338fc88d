"""Generates the golden fixtures in tests/golden/ (run in the build container,
where /root/reference exists; the committed outputs travel, the reference
does not).

distances.npz       seeded random vector pairs of many lengths (uniform [-1,1)
                    and SIFT-like integers) with the outputs of the
                    reference's OWN C kernels l2_256 / dot_256 / l2_512 /
                    dot_512 (adapters/repos/db/vector/hnsw/distancer/c/*.c),
                    compiled in place by `make -C oracle ref` into
                    oracle/_ref/libwvref.so.
hamming.npz         seeded vector pairs (lengths 1..1536) with equal elements,
                    NaNs and signed zeros placed in the SIMD blocks and in the
                    scalar tail, with the outputs of the reference's own
                    hamming_256 / hamming_512 (D/c/hamming_avx{256,512}_amd64.c).
known_answers.json  the hand-vector known answers of the reference's Go
                    tests (values transcribed as data, file:line cited).

Usage:  make -C oracle ref && python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import wv_oracle  # noqa: E402

LENGTHS = list(range(1, 41)) + [63, 64, 65, 96, 127, 128, 129, 200, 255, 256, 257, 384, 511, 512, 768, 777, 1024,
                                 1536]
PAIRS_PER_LEN = 4


def ref_call(lib, sym, a, b):
    P = ctypes.POINTER(ctypes.c_float)
    r = ctypes.c_float()
    n = ctypes.c_long(len(a))
    getattr(lib, sym)(a.ctypes.data_as(P), b.ctypes.data_as(P), ctypes.byref(r), ctypes.byref(n))
    return np.float32(r.value)


def make_distances():
    ref = wv_oracle.ref()
    if ref is None:
        raise SystemExit("oracle/_ref/libwvref.so missing: run `make -C oracle ref` where /root/reference exists")
    rng = np.random.default_rng(20241015)
    a_all, b_all, lens, dist_kind = [], [], [], []
    for n in LENGTHS:
        for p in range(PAIRS_PER_LEN):
            if p % 2 == 0:
                a = rng.uniform(-1, 1, n).astype(np.float32)
                b = rng.uniform(-1, 1, n).astype(np.float32)
            else:
                a = rng.integers(0, 256, n).astype(np.float32)
                b = rng.integers(0, 256, n).astype(np.float32)
            a_all.append(a)
            b_all.append(b)
            lens.append(n)
            dist_kind.append(p % 2)
    out = {s: [] for s in ["l2_256", "dot_256", "l2_512", "dot_512"]}
    for a, b in zip(a_all, b_all):
        for s in out:
            out[s].append(ref_call(ref, s, a, b))
    np.savez_compressed(os.path.join(HERE, "distances.npz"), a=np.concatenate(a_all), b=np.concatenate(b_all),
                        lens=np.asarray(lens, np.int64), kind=np.asarray(dist_kind, np.int8),
                        **{s: np.asarray(v, np.float32) for s, v in out.items()})


def make_hamming():
    """Float-vector Hamming (the "hamming" distance of the vector index config):
    pairs share ~half their elements, and NaN / -0.0 / +0.0 land in the 32-
    and 8-blocks (compared with _CMP_NEQ_OQ) and in the tail (compared with
    !=), where the two comparisons disagree about NaN."""
    ref = wv_oracle.ref()
    if ref is None or not hasattr(ref, "hamming_256"):
        raise SystemExit("oracle/_ref/libwvref.so without hamming_256: run `make -C oracle ref`")
    rng = np.random.default_rng(20261016)
    a_all, b_all, lens = [], [], []
    for n in LENGTHS:
        for p in range(PAIRS_PER_LEN):
            a = rng.integers(0, 4, n).astype(np.float32)
            b = np.where(rng.random(n) < 0.5, a, rng.integers(0, 4, n).astype(np.float32)).astype(np.float32)
            if p >= 1:  # NaNs: one in a, one in b, one in both (block or tail)
                for arr in (a, b):
                    arr[rng.integers(0, n)] = np.nan
                i = rng.integers(0, n)
                a[i] = b[i] = np.nan
            if p >= 2:  # a NaN in the scalar tail when there is one
                t = n - (n % 8) if n >= 8 else 0
                if t < n:
                    a[rng.integers(t, n)] = np.nan
            if p == 3:  # -0.0 vs +0.0 compares equal under both comparisons
                i = rng.integers(0, n)
                a[i], b[i] = np.float32(-0.0), np.float32(0.0)
            a_all.append(a)
            b_all.append(b)
            lens.append(n)
    out = {s: [ref_call(ref, s, a, b) for a, b in zip(a_all, b_all)] for s in ["hamming_256", "hamming_512"]}
    np.savez_compressed(os.path.join(HERE, "hamming.npz"), a=np.concatenate(a_all), b=np.concatenate(b_all),
                        lens=np.asarray(lens, np.int64), **{s: np.asarray(v, np.float32) for s, v in out.items()})


KNOWN = {
    "source": "reference Go tests, transcribed as data",
    "l2": [  # D/l2_test.go:21-66
        {"a": [3, 4, 5], "b": [3, 4, 5], "expected": 0.0},
        {"a": [3, 4, 5], "b": [1.5, 2, 2.5], "expected": 12.5},
        {"a": [10, 11], "b": [13, 15], "expected": 25.0},
    ],
    "dot": [  # D/dot_product_test.go:21-66
        {"a": [3, 4, 5], "b": [3, 4, 5], "expected": -50.0},
        {"a": [0, 1, 0, 2, 0, 3], "b": [1, 0, 2, 0, 3, 0], "expected": 0.0},
        {"a": [3, 4, 5], "b": [-3, -4, -5], "expected": 50.0},
    ],
    "cosine": [  # D/cosine_dist_test.go:21-82 (inputs normalized first); tol = assert.InDelta
        {"a": [0.1, 0.3, 0.7], "b": [0.1, 0.3, 0.7], "expected": 0.0, "tol": 0.0},
        {"a": [0.1, 0.3, 0.7], "b": [0.2, 0.6, 1.4], "expected": 0.0, "tol": 0.0},
        {"a": [0.1, 0.3, 0.7], "b": [0.2, 0.2, 0.2], "expected": 0.173, "tol": 0.01},
        {"a": [0.1, 0.3, 0.7], "b": [-0.1, -0.3, -0.7], "expected": 2.0, "tol": 0.01},
    ],
    "bq_pairs": [  # CH/compression_test.go:44-60 (cosine provider, vectors not normalized)
        {"vecs": [[-0.5, 0.5], [0.25, 0.7], [0.5, 0.5]], "pairs": [[0, 1, 1.0], [0, 2, 1.0], [1, 2, 0.0]]},
    ],
    "bq_query": {  # CH/compression_test.go:62-87
        "vecs": [[-0.5, 0.5], [0.25, 0.7], [0.5, 0.5]], "query": [0.1, -0.2], "hamming": [2.0, 1.0, 1.0],
        "float_vec": [0.8, -0.2], "distance_to_float": 0.88,
    },
    "bq_from_id": {  # CH/compression_test.go:89-113
        "vecs": [[-0.5, 0.5], [0.25, 0.7], [0.5, 0.5]], "from": 0, "hamming": [0.0, 1.0, 1.0],
        "float_vec": [0.8, -0.2], "distance_to_float": 2.0,
    },
    "manhattan": [  # D/manhattan_test.go:21-68
        {"a": [3, 4, 5], "b": [3, 4, 5], "expected": 0.0},
        {"a": [3, 4, 5], "b": [1.5, 2, 2.5], "expected": 6.0},
        {"a": [10, 11], "b": [13, 15], "expected": 7.0},
    ],
    "hamming": [  # D/hamming_test.go:23-82
        {"a": [3, 4, 5], "b": [3, 4, 5], "expected": 0.0},
        {"a": [3, 4, 5], "b": [1.5, 2, 2.5], "expected": 3.0},
        {"a": [10, 11], "b": [10, 15], "expected": 1.0},
        {"a": [10, 11, 15, 25, 31], "b": [10, 15, 16, 25, 30], "expected": 3.0},
    ],
    "pq_code_bytes": list(range(100)),  # CH/product_quantization_test.go:118-130, 235-247
}


def main():
    make_distances()
    make_hamming()
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(KNOWN, f, indent=1)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
