"""ABI 7 shuffle entry points, through the C ABI, against the oracle partitioner (shuffle_ref):

1. khip_shuffle_pack_v (the one-pass multi-destination pack): destination d's rows at
   offsets[d] are exactly the rows the oracle routes to d, in arrival order, bit-exact words —
   for INT32 / INT64 keys, 2..256 destinations, ragged sizes (one row, a tile ± 1, many tiles).
2. Skew: a batch whose largest destination overflows its region is packed again with the exact
   stride (when the buffer holds it) or contiguously (when not) — the same rows either way.
3. KHIP_SHUFFLE_STREAM_TIME: rows carry the batch's stream_time word before the validity word
   (pack, pack_v, the one-destination pack) and khip_shuffle_unpack_stream_time returns it.
4. khip_comm_alltoall_v on one rank (RCCL): the regions arrive back-to-back by source.
Reference: the repartition topic of S/StreamGroupByBuilderBase.java:101-103, Kafka's default
partitioner (kafka-clients Utils.murmur2, pinned by tests/golden/kafka_murmur2.json).
"""
import numpy as np
import pytest
import torch

from ksql_amd import abi
from shuffle_ref import expected_pack
from test_gpu_shuffle import _device_batch, _random_source

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def _split(exp_rows, exp_counts):
    out, off = [], 0
    for c in exp_counts:
        out.append(exp_rows[off:off + c])
        off += c
    return out


def _check_regions(send, counts, offs, exp_rows, exp_counts):
    assert counts == exp_counts
    got = send.cpu().numpy()
    for d, rows in enumerate(_split(exp_rows, exp_counts)):
        np.testing.assert_array_equal(got[offs[d]:offs[d] + counts[d]], rows)
    # regions never overlap
    spans = sorted((o, o + c) for o, c in zip(offs, counts) if c)
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))


@pytest.mark.parametrize("key_type", ["INT64", "INT32"])
@pytest.mark.parametrize("n_parts", [2, 3, 8, 64, 256])
@pytest.mark.parametrize("n", [1, 4095, 4097, 70_001])
def test_pack_v_matches_oracle_partitioner(prod, orc, key_type, n_parts, n):
    cols, types, cv, rv, ts = _random_source(n, key_type, seed=n_parts * 7 + n)
    sh = abi.ShuffleHandle(prod, n_parts, 0, types)
    send, counts, offs = sh.pack_v(_device_batch(cols, cv, rv, ts))
    exp_rows, exp_counts = expected_pack(orc, 0, cols, cv, rv, ts, n_parts)
    _check_regions(send, counts, offs, exp_rows, exp_counts)
    sh.close()


def test_pack_v_large_many_tiles(prod, orc):
    """2^22 + 5 rows over 8 destinations (1025 tiles of look-back) and key column 1."""
    n = (1 << 22) + 5
    cols, types, cv, rv, ts = _random_source(n, "INT64", seed=11)
    types[1] = "INT64"
    cols[1] = cols[1].astype(np.int64)
    sh = abi.ShuffleHandle(prod, 8, 1, types)
    send, counts, offs = sh.pack_v(_device_batch(cols, cv, rv, ts))
    exp_rows, exp_counts = expected_pack(orc, 1, cols, cv, rv, ts, 8)
    _check_regions(send, counts, offs, exp_rows, exp_counts)
    sh.close()


@pytest.mark.parametrize("room", ["exact_stride", "contiguous"])
def test_pack_v_skewed_batch(prod, orc, room):
    """60 % of the rows carry one key: its destination overflows the even-share region.  With room
    for N x the largest destination the batch is packed again with that stride; without, it is
    packed contiguously (offsets = prefix of counts).  The rows are the oracle's either way."""
    n, n_parts = 200_000, 4
    cols, types, cv, rv, ts = _random_source(n, "INT64", seed=5, null_frac=0.0)
    hot = np.random.default_rng(1).random(n) < 0.6
    cols[0] = np.where(hot, 424242, cols[0])
    sh = abi.ShuffleHandle(prod, n_parts, 0, types)
    cap = 3 * n if room == "exact_stride" else sh.pack_capacity(n)
    buf = torch.empty((cap, sh.row_words), dtype=torch.int64, device="cuda")
    send, counts, offs = sh.pack_v(_device_batch(cols, cv, rv, ts), send=buf)
    exp_rows, exp_counts = expected_pack(orc, 0, cols, cv, rv, ts, n_parts)
    _check_regions(send, counts, offs, exp_rows, exp_counts)
    mx = max(counts)
    if room == "exact_stride":
        assert offs == [d * mx for d in range(n_parts)]
    else:
        assert offs == [sum(counts[:d]) for d in range(n_parts)]
    sh.close()


def test_pack_v_buffer_too_small(prod):
    n = 10_000
    cols, types, cv, rv, ts = _random_source(n, "INT64", seed=3)
    sh = abi.ShuffleHandle(prod, 4, 0, types)
    assert sh.pack_capacity(n) >= n
    buf = torch.empty((n, sh.row_words), dtype=torch.int64, device="cuda")
    b = _device_batch(cols, cv, rv, ts)
    counts = (abi.i64 * 4)()
    offs = (abi.i64 * 4)()
    import ctypes as C
    st = prod.shuffle_pack_v(sh.h, C.byref(b.struct), buf.data_ptr(), n, counts, offs)
    assert st == abi.KHIP_E_BUFFER
    sh.close()


@pytest.mark.parametrize("n_parts", [1, 3, 8])
@pytest.mark.parametrize("entry", ["pack", "pack_v"])
def test_stream_time_word(prod, orc, n_parts, entry):
    n = 30_011
    cols, types, cv, rv, ts = _random_source(n, "INT64", seed=n_parts)
    st = np.maximum.accumulate(np.where(ts >= 0, ts, -1))
    sh = abi.ShuffleHandle(prod, n_parts, 0, types, stream_time=True)
    assert sh.row_words == 2 + len(cols) + 1
    b = abi.DeviceBatch(torch.from_numpy(ts).cuda(), row_valid=abi.bitmap_torch(torch.from_numpy(rv).cuda()),
                        cols=[torch.from_numpy(c).cuda() for c in cols],
                        col_valid=[abi.bitmap_torch(torch.from_numpy(v).cuda()) for v in cv],
                        stream_time=torch.from_numpy(st).cuda())
    exp_rows, exp_counts = expected_pack(orc, 0, cols, cv, rv, ts, n_parts, stream_time=st)
    if entry == "pack":
        buf = torch.empty((n, sh.row_words), dtype=torch.int64, device="cuda")
        send, counts = sh.pack(b, send=buf)
        offs = [sum(counts[:d]) for d in range(n_parts)]
    else:
        send, counts, offs = sh.pack_v(b)
    _check_regions(send, counts, offs, exp_rows, exp_counts)
    rows = torch.cat([send[o:o + c] for o, c in zip(offs, counts)])
    got = sh.unpack_stream_time(rows, rows.shape[0]).cpu().numpy()
    np.testing.assert_array_equal(got, exp_rows[:, -2])
    # the column is required
    plain = _device_batch(cols, cv, rv, ts)
    with pytest.raises(abi.KsqlHipError):
        sh.pack_v(plain)
    sh.close()


def test_alltoall_v_single_rank(prod):
    uid = abi.comm_unique_id(prod)
    comm = abi.Comm(prod, 1, 0, uid, 0)
    rows = torch.arange(3 * 40, dtype=torch.int64, device="cuda").reshape(40, 3)
    recv, rc = comm.alltoall(rows, [7], 3, send_offsets=[20])
    assert rc == [7]
    assert torch.equal(recv[:7], rows[20:27])
    assert comm.allgather_i64(12345) == [12345]
    comm.close()
