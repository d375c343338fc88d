"""CPU tests of the PQ codebook persistence format: the HNSW commit log's AddPQ
record (writer MemoryCondensor.AddPQ, V/hnsw/condensor.go:266-285; reader
Deserializer.ReadPQ / ReadKMeansEncoder, V/hnsw/deserializer.go:509-590).

The known-answer record uses the PQData of the reference's own test
(V/hnsw/condensor_integration_test.go:590-621: ks=4, m=3, dims=6, k-means
encoders); the expected bytes are that record laid out by hand from the
writer's field order, and the test asserts the reader gives back the same
PQData the reference test asserts (:650-660)."""
import struct

import numpy as np
import pytest

from weaviate_amd.compressionhelpers import ADD_PQ, PQData, add_pq_record, read_pq_record

CENTERS = np.array([[[1, 2], [3, 4], [5, 6], [7, 8]],
                    [[8, 7], [6, 5], [4, 3], [2, 1]],
                    [[1, 2], [3, 4], [5, 6], [7, 8]]], np.float32)


def _golden():
    head = bytes([11]) + struct.pack("<H", 6) + bytes([1]) + struct.pack("<HH", 4, 3) + bytes([0, 0])
    return head + struct.pack("<24f", *CENTERS.ravel().tolist())


def test_add_pq_record_known_answer():
    data = PQData(Ks=4, M=3, Dimensions=6, EncoderType=1, EncoderDistribution=0, UseBitsEncoding=False,
                  Centers=CENTERS)
    rec = add_pq_record(data)
    assert rec == _golden()
    assert rec[0] == ADD_PQ == 11
    got, used = read_pq_record(rec, 1)
    assert used == len(rec) - 1
    assert got == data


def test_add_pq_record_round_trip_bits():
    rng = np.random.default_rng(5)
    c = rng.standard_normal((32, 256, 4)).astype(np.float32)
    c.ravel()[:3] = [-0.0, np.inf, np.nan]  # raw float32 bits survive
    data = PQData(256, 32, 128, 1, 1, True, c)
    rec = add_pq_record(data)
    assert len(rec) == 10 + 32 * 256 * 4 * 4
    assert rec[9] == 1 and rec[8] == 1
    got, used = read_pq_record(rec + b"\x05trailing", 1)  # the next record is left alone
    assert used == len(rec) - 1
    assert np.array_equal(got.Centers.view(np.uint32), c.view(np.uint32))
    assert got.UseBitsEncoding and got.EncoderDistribution == 1


def test_read_pq_record_errors():
    rec = _golden()[1:]
    for cut, what in [(0, "uint16"), (1, "uint16"), (2, "byte"), (4, "uint16"), (6, "uint16"),
                      (7, "byte"), (8, "byte"), (9, "float32"), (len(rec) - 1, "float32")]:
        with pytest.raises(ValueError, match=f"failed to read {what}"):
            read_pq_record(rec[:cut])
    bad = bytearray(rec)
    bad[2] = 7
    with pytest.raises(ValueError, match="Unsuported encoder type"):
        read_pq_record(bytes(bad))
    bad[2] = 0
    with pytest.raises(ValueError, match="tile encoder is out of scope"):
        read_pq_record(bytes(bad))
    with pytest.raises(ValueError, match="centers shape"):
        add_pq_record(PQData(4, 3, 6, 1, 0, False, CENTERS[:2]))


def test_pq_config_errors():
    """NewProductQuantizer's checks (CH/product_quantization.go:190-207) in the
    order and with the messages of CH/product_quantization_test.go:132-233."""
    from weaviate_amd import _lib
    from weaviate_amd.compressionhelpers import validate_pq_config

    for args, msg in [((4, 256, 128, "kmeans-x", "log-normal"), "invalid encoder type"),
                      ((4, 256, 128, "kmeans", "normal-x"), "invalid encoder distribution"),
                      ((0, 256, 128), "segments cannot be 0 nor negative"),
                      ((-2, 256, 128), "segments cannot be 0 nor negative"),
                      ((3, 256, 128), "segments should be an integer divisor of dimensions"),
                      ((4, 512, 128), "centroids should not be higher than 256. Attempting to use 512"),
                      ((4, 0, 128), "centroids must be > 0"),
                      ((4, -3, 128), "centroids must be > 0")]:
        with pytest.raises(_lib.WvgError, match=msg):
            validate_pq_config(*args)
    assert validate_pq_config(4, 256, 128) == (1, 1)  # defaults: kmeans, log-normal
    assert validate_pq_config(4, 256, 128, "tile", "normal") == (0, 0)
