"""The oracle's key-sharded P-thread restatement (oracle_agg_push_sharded) equals the sequential
oracle bit for bit: same stats, same rows, same DOUBLE sums (each group sees its records in the
same order).  It is the checker of the full-size GPU parity tests and the multi-core CPU
baseline, so it is pinned here against the sequential restatement (itself pinned by the QTT
goldens in test_oracle_golden.py), including late records, null keys/values, negative
timestamps and micro-batch boundaries.  CPU only."""
import numpy as np
import pytest

import qtt
from ksql_amd import abi
from test_gpu_parity import ALL_AGGS, WINDOWS, _random_batch


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def _same(a, b):
    assert a["n"] == b["n"]
    if isinstance(a["key"], list):
        assert a["key"] == b["key"]
    else:
        assert np.array_equal(a["key"], b["key"])
    for f in ("ws", "we", "rowtime"):
        assert np.array_equal(a[f], b[f]), f
    for x, y in zip(a["values"], b["values"]):
        assert np.array_equal(x.view(np.int64) if x.dtype == np.float64 else x,
                              y.view(np.int64) if y.dtype == np.float64 else y)
    for x, y in zip(a["nulls"], b["nulls"]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("shards", [1, 3, 8])
@pytest.mark.parametrize("key_type", ["INT64", "UTF8"])
@pytest.mark.parametrize("win", range(len(WINDOWS)))
def test_sharded_equals_sequential(orc, win, key_type, shards):
    rng = np.random.default_rng(31 * win + shards)
    batches = [_random_batch(rng, 6000, key_type, 300, 200_000, 40_000, t0=b * 150_000, neg_ts=0.01)
               for b in range(3)]
    desc = abi.make_agg_desc(**dict(WINDOWS[win], key_type=key_type,
                                    col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"], aggs=ALL_AGGS))
    seq = abi.AggHandle(orc, desc)
    par = abi.ShardedOracleAgg(orc, desc, shards)
    assert [seq.push(b) for b in batches] == [par.push(b) for b in batches]
    _same(seq.snapshot(), par.snapshot())
    having = {"agg": 0, "op": "GT", "value": 3}
    _same(seq.snapshot(having), par.snapshot(having))
    seq.close()
    par.close()


@pytest.mark.parametrize("case", qtt.load_cases("agg")[:12], ids=lambda c: c["name"])
def test_sharded_passes_qtt_goldens(orc, case):
    par = abi.ShardedOracleAgg(orc, qtt.case_desc(case), 4)
    par.push(qtt.case_batch(case))
    assert qtt.compare_agg(case, par.snapshot(case["desc"]["having"])) == []
    par.close()


SESSIONS = [dict(window_kind="SESSION", size_ms=20_000, grace_ms=-1),
            dict(window_kind="SESSION", size_ms=5_000, grace_ms=10_000),
            dict(window_kind="SESSION", size_ms=30_000, grace_ms=0, retention_ms=100_000)]


@pytest.mark.parametrize("shards", [1, 4])
@pytest.mark.parametrize("win", range(len(SESSIONS)))
def test_sharded_sessions_and_changes(orc, win, shards):
    """SESSION windows (R11) and the per-push changelog (R10) of the sharded restatement equal the
    sequential one: merges, tombstones, late drops, expiry."""
    rng = np.random.default_rng(71 * win + shards)
    batches = [_random_batch(rng, 5000, "INT64", 200, 300_000, 60_000, t0=b * 250_000, neg_ts=0.01)
               for b in range(4)]
    desc = abi.make_agg_desc(**dict(SESSIONS[win], key_type="INT64", col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"],
                                    aggs=ALL_AGGS, having={"agg": 0, "op": "GT", "value": 2}))
    seq = abi.AggHandle(orc, desc)
    par = abi.ShardedOracleAgg(orc, desc, shards)
    tombs = 0
    for b in batches:
        assert seq.push(b) == par.push(b)
        c1, c2 = seq.changes(), par.changes()
        _same(c1, c2)
        assert np.array_equal(c1["tombstone"], c2["tombstone"])
        tombs += int(c1["tombstone"].sum())
    assert tombs > 0 or win == 1  # 5 s gap over sparse keys: no merges
    _same(seq.snapshot(), par.snapshot())
    seq.close()
    par.close()
