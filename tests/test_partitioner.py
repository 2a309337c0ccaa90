"""Repartition routing (oracle rule R8): Kafka's default partitioner over the KAFKA-format key.

Pinned by Kafka's own murmur2 known-answer vectors (tests/golden/kafka_murmur2.json).  The
partition of a BIGINT / INT key is toPositive(murmur2(big-endian 8 / 4 bytes)) % n — checked
here against a pure-Python restatement on the same bytes.
"""
import json
import os
import struct

import numpy as np
import pytest

from ksql_amd import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kafka_murmur2.json")


def _murmur2_py(data):
    m = 0x5BD1E995
    h = (0x9747B28C ^ len(data)) & 0xFFFFFFFF
    n4 = len(data) // 4
    for i in range(n4):
        k = int.from_bytes(data[4 * i:4 * i + 4], "little")
        k = (k * m) & 0xFFFFFFFF
        k ^= k >> 24
        k = (k * m) & 0xFFFFFFFF
        h = ((h * m) & 0xFFFFFFFF) ^ k
    tail = data[4 * n4:]
    if len(tail) == 3:
        h ^= tail[2] << 16
    if len(tail) >= 2:
        h ^= tail[1] << 8
    if len(tail) >= 1:
        h ^= tail[0]
        h = (h * m) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= h >> 15
    return h - (1 << 32) if h >= 1 << 31 else h


def test_murmur2_known_answers():
    orc = abi.load_oracle()
    cases = json.load(open(GOLDEN))["cases"]
    assert len(cases) == 6
    for c in cases:
        b = c["bytes"].encode()
        assert orc.dll.oracle_murmur2(b, len(b)) == c["murmur2"], c
        assert _murmur2_py(b) == c["murmur2"], c


@pytest.mark.parametrize("width", [4, 8])
@pytest.mark.parametrize("n_parts", [1, 2, 3, 8, 256])
def test_kafka_partition_of_kafka_format_keys(width, n_parts):
    orc = abi.load_oracle()
    rng = np.random.default_rng(width * 1000 + n_parts)
    lo, hi = (-(1 << 31), 1 << 31) if width == 4 else (-(1 << 63), 1 << 63)
    keys = rng.integers(lo, hi, size=500, dtype=np.int64)
    keys[:4] = [0, -1, 1, lo]
    out = np.zeros(len(keys), np.int32)
    orc.dll.oracle_kafka_partition(keys.ctypes.data, len(keys), width, n_parts, out.ctypes.data)
    fmt = ">i" if width == 4 else ">q"
    for k, p in zip(keys.tolist(), out.tolist()):
        assert p == (_murmur2_py(struct.pack(fmt, k)) & 0x7FFFFFFF) % n_parts
