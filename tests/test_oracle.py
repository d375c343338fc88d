"""CPU tests: the oracle (CPU restatement) pinned against the reference's own
outputs -- the golden vectors produced by the reference's C kernels and the
hand-vector known answers of the reference's Go tests."""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "distances.npz"))


@pytest.fixture(scope="module")
def known():
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        return json.load(f)


def _pairs(g):
    off = 0
    for i, n in enumerate(g["lens"]):
        yield i, g["a"][off:off + n], g["b"][off:off + n]
        off += n


@pytest.mark.parametrize("fn,key", [("orc_l2_256", "l2_256"), ("orc_dot_256", "dot_256"),
                                    ("orc_l2_512", "l2_512"), ("orc_dot_512", "dot_512")])
def test_oracle_matches_reference_kernels_bitwise(orc, golden, fn, key):
    """D/c/{l2,dot}_avx{256,512}_amd64.c outputs, all lengths 1..1536."""
    f = getattr(orc.lib(), fn)
    got, want = [], golden[key]
    for i, a, b in _pairs(golden):
        got.append(f(orc._f(np.ascontiguousarray(a)), orc._f(np.ascontiguousarray(b)), len(a)))
    assert np.array_equal(_bits(got), _bits(want))


def test_l2_known_answers(orc, known):
    for c in known["l2"]:
        assert orc.single_dist(orc.L2, c["a"], c["b"]) == np.float32(c["expected"])
        # Step-by-step equals SingleDist (D/l2_test.go:68-88)
        s = np.float32(0)
        for x, y in zip(c["a"], c["b"]):
            s = np.float32(s + orc.step(orc.L2, [x], [y]))
        assert s == np.float32(c["expected"])


def test_dot_known_answers(orc, known):
    for c in known["dot"]:
        assert orc.single_dist(orc.DOT, c["a"], c["b"]) == np.float32(c["expected"])


def test_cosine_known_answers(orc, known):
    for c in known["cosine"]:
        a, b = orc.normalize(c["a"]), orc.normalize(c["b"])
        d = orc.single_dist(orc.COSINE, a, b)
        if c["tol"] == 0.0:
            assert abs(float(d) - c["expected"]) <= 1e-6
        else:
            assert abs(float(d) - c["expected"]) <= c["tol"]


@pytest.mark.parametrize("key", ["hamming_256", "hamming_512"])
def test_oracle_hamming_matches_reference_kernels(orc, key):
    """D/c/hamming_avx{256,512}_amd64.c outputs (tests/golden/hamming.npz):
    equal elements, NaN in the SIMD blocks (_CMP_NEQ_OQ: not counted) and in
    the scalar tail (!=: counted), -0.0 vs +0.0; lengths 1..1536."""
    g = np.load(os.path.join(GOLDEN, "hamming.npz"))
    got = [orc.hamming_256(a, b) for _, a, b in _pairs(g)]
    assert np.array_equal(_bits(got), _bits(g[key]))
    # the NaN rule matters: some pairs differ from a plain count of a != b
    plain = [np.float32(np.count_nonzero(a != b)) for _, a, b in _pairs(g)]
    assert not np.array_equal(_bits(plain), _bits(g[key]))


@pytest.mark.parametrize("metric,key", [("MANHATTAN", "manhattan"), ("HAMMING", "hamming")])
def test_manhattan_hamming_known_answers(orc, known, metric, key):
    """D/manhattan_test.go:21-90, D/hamming_test.go:23-103: SingleDist and the
    step-by-step sum of Step over single elements."""
    m = getattr(orc, metric)
    for c in known[key]:
        assert orc.single_dist(m, c["a"], c["b"]) == np.float32(c["expected"])
        s = np.float32(0)
        for x, y in zip(c["a"], c["b"]):
            s = np.float32(s + orc.step(m, [x], [y]))
        assert s == np.float32(c["expected"])


def test_manhattan_is_the_sequential_go_loop(orc):
    """manhattanImpl (D/manhattan.go:20-30) adds |a_i - b_i| in element order
    in fp32: compare with a numpy loop in the same order."""
    rng = np.random.default_rng(5)
    for n in [1, 7, 8, 33, 128, 777]:
        a = rng.uniform(-1, 1, n).astype(np.float32)
        b = rng.uniform(-1, 1, n).astype(np.float32)
        s = np.float32(0)
        for x, y in zip(a, b):
            s = np.float32(s + np.abs(np.float32(x - y)))
        assert orc.manhattan(a, b).view(np.uint32) == s.view(np.uint32)


def test_normalize_zero_vector(orc):
    assert np.all(orc.normalize(np.zeros(7)) == 0)


def test_bq_known_answers(orc, known):
    kp = known["bq_pairs"][0]
    codes = [orc.bq_encode(v) for v in kp["vecs"]]
    for i, j, want in kp["pairs"]:
        assert orc.bq_distance(codes[i], codes[j]) == np.float32(want)
    kq = known["bq_query"]
    qc = orc.bq_encode(kq["query"])
    for v, want in zip(kq["vecs"], kq["hamming"]):
        assert orc.bq_distance(orc.bq_encode(v), qc) == np.float32(want)
    # DistanceToFloat with the raw query: cosine SingleDist = 1 - dot (CH/quantizer.go:109-115)
    assert orc.single_dist(orc.COSINE, kq["query"], kq["float_vec"]) == np.float32(kq["distance_to_float"])
    kf = known["bq_from_id"]
    base = orc.bq_encode(kf["vecs"][kf["from"]])
    for v, want in zip(kf["vecs"], kf["hamming"]):
        assert orc.bq_distance(base, orc.bq_encode(v)) == np.float32(want)
    assert orc.bq_distance(base, orc.bq_encode(kf["float_vec"])) == np.float32(kf["distance_to_float"])


def test_bq_encode_bit_layout(orc):
    v = np.ones(130, dtype=np.float32)
    v[[0, 63, 64, 129]] = -1.0
    v[5] = -0.0  # -0 is not < 0
    code = orc.bq_encode(v)
    assert code.tolist() == [1 | (1 << 63), 1, 2]


def test_pq_lut_adc_and_encode_tie_rule(orc):
    rng = np.random.default_rng(3)
    m, ks, ds = 4, 16, 3
    centers = rng.integers(-3, 4, (m, ks, ds)).astype(np.float32)
    centers[:, 7] = centers[:, 2]  # duplicate centroid: ties must go to the higher index (kmeans.go:122-132)
    X = centers[np.arange(m)[None, :], rng.integers(0, ks, (50, m))].reshape(50, m * ds)
    codes = orc.pq_encode(X, centers)
    for s in range(m):
        assert not np.any(codes[:, s] == 2), "tie must resolve to the later centroid 7"
    q = rng.uniform(-1, 1, m * ds).astype(np.float32)
    lut = orc.pq_lut(orc.L2, q, centers)
    code = codes[0]
    s = np.float32(0)
    for i in range(m):
        s = np.float32(s + lut[i, code[i]])
    assert orc.pq_adc(orc.L2, lut, code) == s


def test_pq_search_is_lut_adc_plus_heap(orc):
    """orc_pq_search / orc_bench_pq (the CPU PQ-ADC leg of bench.py) equal the
    per-row LookUp sums fed through the flat heap."""
    rng = np.random.default_rng(11)
    n, m, ks, ds = 3000, 32, 256, 4
    codes = rng.integers(0, ks, (n, m), dtype=np.uint8)
    centers = orc.synth_rows(45, 0, m * ks, ds, 0).reshape(m, ks, ds)
    qs = rng.uniform(-1, 1, (3, m * ds)).astype(np.float32)
    _, bi, bd = orc.bench_pq(codes, centers, qs, 10, orc.L2, 2)
    for j, q in enumerate(qs):
        lut = orc.pq_lut(orc.L2, q, centers)
        d = np.array([orc.pq_adc(orc.L2, lut, c) for c in codes], np.float32)
        wi, wd = orc.heap_topk(d, np.arange(n, dtype=np.uint64), 10)
        i, dd = orc.pq_search(codes, centers, q, 10, orc.L2)
        assert np.array_equal(i, wi) and np.array_equal(dd.view(np.uint32), wd.view(np.uint32))
        assert np.array_equal(bi[j], wi) and np.array_equal(bd[j].view(np.uint32), wd.view(np.uint32))


def test_heap_topk_matches_lexicographic_modulo_ties(orc):
    rng = np.random.default_rng(7)
    d = rng.integers(0, 20, 2000).astype(np.float32)  # many ties
    ids = np.arange(2000, dtype=np.uint64)
    hi, hd = orc.heap_topk(d, ids, 37)
    li, ld = orc.lex_topk(d, ids, 37)
    assert np.array_equal(hd, ld)  # distances identical
    cut = ld[-1]
    assert set(hi[hd < cut].tolist()) == set(li[ld < cut].tolist())  # ids identical below the boundary tie


def test_synthetic_generator_is_stable(orc):
    # pinned values of the counter-based generator (shared with the device kernel)
    r = orc.synth_rows(42, 0, 2, 4, 0)
    assert r.dtype == np.float32 and np.all(r >= -1) and np.all(r < 1)
    r2 = orc.synth_rows(42, 1, 1, 4, 0)
    assert np.array_equal(r[1], r2[0])
    ints = orc.synth_rows(42, 0, 100, 8, 1)
    assert np.all(ints == np.floor(ints)) and ints.max() <= 255 and ints.min() >= 0


def test_flat_search_oracle_with_reference_kernel(orc):
    """The oracle's flat search gives the same results whether it calls its own
    restated l2_256 or the reference's compiled l2_256 (when available)."""
    if orc.ref() is None:
        pytest.skip("oracle/_ref not built here")
    rows = orc.synth_rows(5, 0, 3000, 128, 0)
    q = orc.synth_rows(6, 0, 1, 128, 0)[0]
    a = orc.flat_search(rows, q, 10, orc.L2)
    b = orc.flat_search(rows, q, 10, orc.L2, use_ref_kernel=True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(_bits(a[1]), _bits(b[1]))


def test_oracle_kmeans_fit_properties():
    """The k-means restatement (CH/kmeans.go:146-250): deterministic for a seed,
    centers are means of their members (nearest-property pin, kmeans_test.go:26-53)."""
    from oracle import wv_oracle as orc

    X = np.array([[0, 5], [0.1, 4.9], [0.01, 5.1], [10.1, 7], [5.1, 2], [5.0, 2.1]], np.float32)
    c1, it1 = orc.pq_fit(X, 1, 3, 0, 5)
    c2, it2 = orc.pq_fit(X, 1, 3, 0, 5)
    assert np.array_equal(c1, c2) and np.array_equal(it1, it2)
    codes = orc.pq_encode(X, c1)[:, 0]
    for v in range(len(X)):
        mn = orc.l2_256(X[v], c1[0, codes[v]])
        assert all(orc.l2_256(X[v], c1[0, c]) >= mn for c in codes)
    # seed 3 starts in the three separated groups -> each center the mean of its group
    c3, _ = orc.pq_fit(X, 1, 3, 0, 3)
    got = np.array(sorted(map(tuple, c3[0].tolist())))
    assert np.allclose(got, sorted([(0.11 / 3, 5.0), (5.05, 2.05), (10.1, 7.0)]), atol=1e-5)
    with pytest.raises(ValueError):
        orc.pq_fit(X, 1, 7, 0, 5)


def test_oracle_search_by_distance_loop():
    """The growing-limit loop restated from V/hnsw/search.go:85-151."""
    from oracle import wv_oracle as orc

    d = np.arange(5000, dtype=np.float32)
    ids = np.arange(5000, dtype=np.uint64)
    fn = lambda tot: (ids[:tot], d[:tot])  # noqa: E731
    assert len(orc.search_by_distance(fn, 49.0, -1)[0]) == 50
    assert len(orc.search_by_distance(fn, 99.0, -1)[0]) == 100     # window's last <= target: one more search
    assert len(orc.search_by_distance(fn, 3000.0, -1)[0]) == 3001
    assert len(orc.search_by_distance(fn, 3000.0, 1100)[0]) == 1100  # next limit 11100 > max_limit
    assert len(orc.search_by_distance(fn, 3000.0, 50)[0]) == 100     # the first search always runs
    assert len(orc.search_by_distance(fn, 1e9, -1)[0]) == 5000
    assert len(orc.search_by_distance(fn, np.float32(10.0) - np.float32(5e-7), -1)[0]) == 11  # InDelta 1e-6


def test_oracle_selftest_under_asan_ubsan():
    """The checker itself under AddressSanitizer + UBSan (oracle/selftest.c):
    every entry point over empty, ragged and block-boundary sizes, k = 0 and
    k > n, deleted rows -- a buffer overrun in the oracle would otherwise show
    up as a spurious (or hidden) parity difference."""
    import shutil
    import subprocess

    here = os.path.join(os.path.dirname(GOLDEN), "..", "oracle")
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    b = subprocess.run(["make", "-s", "-C", here, "asan"], capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in (b.stderr or ""):
        pytest.skip("sanitizer runtime unavailable: " + b.stderr[-200:])
    assert b.returncode == 0, b.stderr
    r = subprocess.run([os.path.join(here, "_build", "selftest_asan")], capture_output=True, text=True,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"), timeout=300)
    assert r.returncode == 0 and "selftest ok" in r.stdout, r.stderr[-2000:]


def test_dist_all_512_matches_reference_kernels(orc):
    """The oracle's AVX-512-order SingleDist (used by the 512-mode GPU tests)
    equals the reference's compiled l2_512 / dot_512 outputs, with Wrap."""
    import os

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "distances.npz"))
    off = 0
    for n, l5, d5 in zip(g["lens"], g["l2_512"], g["dot_512"]):
        a, b = g["a"][off:off + n], g["b"][off:off + n]
        off += n
        assert orc.dist_all_512(0, a, b[None])[0].view(np.uint32) == np.float32(l5).view(np.uint32)
        assert orc.dist_all_512(1, a, b[None])[0].view(np.uint32) == np.float32(-d5).view(np.uint32)
        assert orc.dist_all_512(2, a, b[None])[0].view(np.uint32) == (np.float32(1) - d5).view(np.uint32)
