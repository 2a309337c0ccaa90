"""The windowed COUNT(*) pipeline (ksql_amd/csrc/khip_agg_c1.hip) against the oracle.

The pipeline takes a push of `COUNT(*) ... WINDOW TUMBLING ... GROUP BY k` when no step of 4096
records can hold a late record and every ts lies within 2^31 ms of the push's time base; otherwise
it declines and the general path runs on the same batch.  Every case checks
the final table, the batch statistics and the maintained HAVING count against the oracle (the
sequential restatement of KStreamWindowAggregate as called from S/StreamAggregateBuilder.java:
287-294), and which path the pushes took (khip_kernel_times.c1_pushes / c1_declined, ABI 5):
- the bench shape scaled down (dense ids, default grace, HAVING > 3);
- several pushes with windows closing between them (resident rows merged, closed rows evicted)
  and the per-push changelog (EMIT CHANGES with HAVING tombstones);
- a key range past 31 - window bits (the 64-bit group identity);
- null keys, null rows and negative timestamps (sentinel records);
- UTF-8 keys (dictionary ids);
- more groups per partition than one LDS table takes (sub-pass retries) and than a region holds
  (region growth);
- keys spread over 2^53 (the wide records: 64-bit key hashes and u32 ts words);
- pushes the pipeline must decline: late records, a ts span past 2^31 ms.
"""
import numpy as np
import pytest

from ksql_amd import abi
from test_gpu_parity import assert_snap_equal

pytestmark = pytest.mark.gpu

HAVING = {"agg": 0, "op": "GT", "value": 3}


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def _desc(size=5000, grace=-1, hint=0, flags=0, key_type="INT64", having=HAVING):
    return abi.make_agg_desc(window_kind="TUMBLING", key_type=key_type, size_ms=size, advance_ms=size, grace_ms=grace,
                             aggs=[("COUNT_STAR", -1)], capacity_hint=hint, flags=flags, having=having)


def _run(prod, orc, batches, changes=False, **kw):
    """Push every batch through the product (profiled) and the oracle; compare after each push
    (statistics, and the changelog when asked) and at the end (table, HAVING count).  Returns the
    product's kernel_times counters."""
    flags = abi.FLAG_CHANGELOG if changes else 0
    gd, od = _desc(flags=flags | abi.FLAG_PROFILE, **kw), _desc(flags=flags, **kw)
    g, o = abi.AggHandle(prod, gd), abi.AggHandle(orc, od)
    for b in batches:
        gs, os_ = g.push(b), o.push(b)
        assert gs == os_, (gs, os_)
        if changes:
            gc, oc = g.changes(), o.changes()
            assert_snap_equal(gc, oc, gd)
            assert np.array_equal(gc["tombstone"], oc["tombstone"])
    gsnap, osnap = g.snapshot(), o.snapshot()
    assert_snap_equal(gsnap, osnap, gd)
    if kw.get("having", HAVING) is not None:
        assert g.count_rows(HAVING) == o.snapshot(HAVING)["n"]
    kt = g.kernel_times()
    g.close()
    o.close()
    return kt


def _fraud(rng, n, keys, span=10_000, disorder=500, t0=0, kbase=0):
    k = kbase + rng.integers(0, keys, n)
    ts = t0 + (np.arange(n) * span) // n + rng.integers(0, disorder, n)
    return k, ts


def test_c1_bench_shape(prod, orc):
    rng = np.random.default_rng(1)
    k, ts = _fraud(rng, 2_000_000, 200_000)
    kt = _run(prod, orc, [abi.HostBatch(ts, keys=k)], hint=400_000 * 8)
    assert kt["c1_pushes"] == 1 and kt["c1_declined"] == 0, kt


def test_c1_pushes_close_windows_and_changelog(prod, orc):
    """Grace 1 s, disorder 100 ms: no record is late, but each push's stream time closes the
    previous pushes' windows (evicted to the closed store by the merge)."""
    rng = np.random.default_rng(2)
    batches = []
    for p in range(5):
        k, ts = _fraud(rng, 300_000, 40_000, span=20_000, disorder=100, t0=p * 20_000)
        batches.append(abi.HostBatch(ts, keys=k))
    kt = _run(prod, orc, batches, changes=True, grace=1000, hint=1 << 22)
    assert kt["c1_pushes"] == 5, kt


def test_c1_wide_key_identity(prod, orc):
    """Key range 2^30: (key - kmin) << window bits does not fit 31 bits → 64-bit identities."""
    rng = np.random.default_rng(3)
    pool = (1 << 40) + rng.integers(0, 1 << 30, 100_000)
    k = pool[rng.integers(0, len(pool), 1_000_000)]
    _, ts = _fraud(rng, 1_000_000, 1)
    kt = _run(prod, orc, [abi.HostBatch(ts, keys=k)], hint=1 << 22)
    assert kt["c1_pushes"] == 1, kt


def test_c1_invalid_records(prod, orc):
    rng = np.random.default_rng(4)
    n = 1_000_000
    k, ts = _fraud(rng, n, 50_000, t0=10_000)
    ts[rng.random(n) < 0.01] = -1  # failed timestamps: dropped
    kv = rng.random(n) > 0.02
    rv = rng.random(n) > 0.02
    kt = _run(prod, orc, [abi.HostBatch(ts, keys=k, key_valid=kv, row_valid=rv)], hint=1 << 22)
    assert kt["c1_pushes"] == 1, kt


def test_c1_utf8_keys(prod, orc):
    rng = np.random.default_rng(5)
    n = 500_000
    ids = rng.integers(0, 60_000, n)
    keys = ["%016d" % (4000000000000000 + int(i)) for i in ids]
    _, ts = _fraud(rng, n, 1)
    kt = _run(prod, orc, [abi.HostBatch(ts, utf8_keys=keys)], key_type="UTF8", hint=1 << 22)
    assert kt["c1_pushes"] == 1, kt


def test_c1_utf8_dictionary_growth(prod, orc):
    """The key dictionary is sized from the keys the last map added (twice that, at least n / 16),
    not from the batch size: a push bringing far more new keys than that fails its probes and is
    mapped again into a larger table (khip_agg.hip dict_map); a reset gives back a table sized by
    the first map's every-row estimate.  Rounds (a reset after each): [100 keys] (the reset shrinks
    the table), [100 keys, 150K new keys] (the second push is mapped again twice), the same again."""
    rng = np.random.default_rng(15)
    b1 = ["k%07d" % int(i) for i in rng.integers(0, 100, 20_000)]
    b2 = ["n%09d" % int(i) for i in rng.permutation(150_000)]
    _, t1 = _fraud(rng, len(b1), 1, span=5_000)
    _, t2 = _fraud(rng, len(b2), 1, span=5_000, t0=5_000)
    batches = [abi.HostBatch(t1, utf8_keys=b1), abi.HostBatch(t2, utf8_keys=b2)]
    gd, od = _desc(key_type="UTF8", hint=1 << 20), _desc(key_type="UTF8", hint=1 << 20)
    g = abi.AggHandle(prod, gd)
    for rnd in ([batches[0]], batches, batches):  # the oracle has no reset: a fresh handle per round
        o = abi.AggHandle(orc, od)
        for b in rnd:
            assert g.push(b) == o.push(b)
        assert_snap_equal(g.snapshot(), o.snapshot(), gd)
        assert g.count_rows(HAVING) == o.snapshot(HAVING)["n"]
        g.reset()
        o.close()
    g.close()


def test_c1_sub_passes_and_region_growth(prod, orc):
    """4096 partitions (from the hint) and ~4150 groups each: over the 3072 an LDS table takes
    (retried with 2 sub-passes) and, for some, over the 4096-row regions (grown)."""
    rng = np.random.default_rng(6)
    n = 17_000_000
    k = rng.permutation(n)[: n // 2]
    k = np.concatenate([k, k])  # 8M keys, each twice: once per window
    ts = np.concatenate([rng.integers(0, 5000, n // 2), rng.integers(5000, 10_000, n // 2)])
    kt = _run(prod, orc, [abi.HostBatch(ts, keys=k)], hint=1 << 22, having=None)
    assert kt["c1_pushes"] == 1, kt


def test_c1_wide_records(prod, orc):
    """Keys spread over 2^53 (a bijection of dense card ids): the key range needs the wide records
    (64-bit key hash + u32 ts word); the first push declines the compact format and is redone with
    them in the same call, later pushes start wide."""
    rng = np.random.default_rng(8)
    batches = []
    for p in range(3):
        k, ts = _fraud(rng, 700_000, 60_000, span=15_000, disorder=300, t0=p * 15_000)
        k = (k * 0x5DEECE66D) & ((1 << 53) - 1)  # a bijection on [0, 2^53) (odd multiplier)
        batches.append(abi.HostBatch(ts, keys=k))
    kt = _run(prod, orc, batches, changes=True, grace=2000, hint=1 << 22)
    assert kt["c1_pushes"] == 3 and kt["c1_declined"] == 0, kt


@pytest.mark.parametrize("case", ["late", "ts_span"])
def test_c1_declined_pushes(prod, orc, case):
    rng = np.random.default_rng(7)
    n = 400_000
    k, ts = _fraud(rng, n, 30_000)
    grace = -1
    if case == "late":
        grace = 0
        ts = rng.permutation(ts)  # heavy disorder, no grace: late records
    else:
        ts[-1000:] += 1 << 32
    kt = _run(prod, orc, [abi.HostBatch(ts, keys=k)], grace=grace, hint=1 << 22)
    assert kt["c1_pushes"] == 0 and kt["c1_declined"] == 1, kt
