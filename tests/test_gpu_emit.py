"""Emission and retention on the HIP path (khip_agg_changes, include/ksqldb_hip.h), against the
oracle's rules R9 (retention) and R10 (emission), themselves pinned by the QTT goldens
(test_oracle_golden.py: output sequences of having.json, suppress.json, ...).

1. EMIT CHANGES: after every push, the rows the push emitted (deduplicated per (key, window),
   sorted) and their tombstone flags equal the oracle's — random micro-batches with late
   records, hopping fan-out, UTF-8 keys, HAVING on integer and DOUBLE aggregates, both
   partitioned-engine claim modes (packed identity / claim protocol) and many partitions.
2. EMIT FINAL: windows closed by each push, minus those that expired before the record that
   closed them (stream-time jumps inside a push), both engines, default and explicit RETENTION.
3. Retention: the window store (snapshot, pull query, row count) drops expired windows exactly
   like the oracle's store, across pushes that evict and purge the closed store.
"""
import numpy as np
import pytest

from ksql_amd import abi
from test_gpu_parity import ABS_SUM, ALL_AGGS, CNT_DBL, WINDOWS, _random_batch, assert_snap_equal

pytestmark = pytest.mark.gpu

COLS = ["INT32", "INT64", "DOUBLE", "DOUBLE"]


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def _assert_changes_equal(g, o, desc):
    assert_snap_equal(g, o, desc, ABS_SUM, CNT_DBL)
    assert np.array_equal(g["tombstone"], o["tombstone"])


def _batches(rng, nb, n, key_type, nkeys, span, disorder, jump=0):
    out = []
    t0 = 0
    for b in range(nb):
        out.append(_random_batch(rng, n, key_type, nkeys, span, disorder, t0=t0, neg_ts=0.005))
        t0 += span * 3 // 4 + (jump if b % 2 else 0)
    return out


HAVINGS = [None, {"agg": 0, "op": "GT", "value": 3}, {"agg": 13, "op": "LE", "value": 10.5}]


@pytest.mark.parametrize("engine", [0, abi.FLAG_PART_CLAIM])
@pytest.mark.parametrize("having", range(len(HAVINGS)))
@pytest.mark.parametrize("win", range(len(WINDOWS)))
def test_changes_vs_oracle(prod, orc, win, having, engine):
    rng = np.random.default_rng(300 + 10 * win + having)
    hv = HAVINGS[having]
    kw = dict(WINDOWS[win], key_type="INT64", col_types=COLS, aggs=ALL_AGGS, having=hv)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=engine | abi.FLAG_CHANGELOG)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    emitted = 0
    for batch in _batches(rng, 5, 6000, "INT64", 400, 120_000, 30_000):
        assert g.push(batch) == o.push(batch)
        gc, oc = g.changes(), o.changes()
        _assert_changes_equal(gc, oc, g.desc)
        emitted += gc["n"]
    assert emitted > 0 or (win == 2 and having == 1)  # sparse tumbling windows: no count above 3
    assert_snap_equal(g.snapshot(hv), o.snapshot(hv), g.desc, ABS_SUM, CNT_DBL)
    g.close()
    o.close()


def test_changes_utf8_and_many_partitions(prod, orc):
    rng = np.random.default_rng(7)
    hv = {"agg": 0, "op": "GE", "value": 2}
    for key_type, hint, nkeys in (("UTF8", 0, 500), ("INT64", 30_000_000, 40_000)):
        kw = dict(WINDOWS[3], key_type=key_type, col_types=COLS, aggs=ALL_AGGS, having=hv, capacity_hint=hint)
        g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=abi.FLAG_CHANGELOG)))
        o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
        for batch in _batches(rng, 3, 60_000, key_type, nkeys, 200_000, 20_000):
            assert g.push(batch) == o.push(batch)
            _assert_changes_equal(g.changes(), o.changes(), g.desc)
        g.close()
        o.close()


def test_changes_one_record_pushes_match_sequence(prod, orc):
    """Tiny pushes (1-3 records) exercise the cache-off sequence with tombstones."""
    rng = np.random.default_rng(9)
    hv = {"agg": 3, "op": "GT", "value": 0}  # SUM(BIGINT) > 0 flips back and forth
    kw = dict(WINDOWS[4], key_type="INT64", col_types=COLS, aggs=ALL_AGGS, having=hv)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=abi.FLAG_CHANGELOG)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    big = _random_batch(rng, 300, "INT64", 5, 100_000, 20_000)
    i = 0
    tombs = 0
    while i < 300:
        k = int(rng.integers(1, 4))
        sl = slice(i, min(i + k, 300))
        b = abi.HostBatch(big.ts[sl], keys=big.keys[sl], cols=[c[sl] for c in big.cols],
                          col_valid=[None if v is None else np.unpackbits(v, bitorder="little")[:300][sl].astype(bool)
                                     for v in big.col_valid])
        assert g.push(b) == o.push(b)
        gc, oc = g.changes(), o.changes()
        _assert_changes_equal(gc, oc, g.desc)
        tombs += int(gc["tombstone"].sum())
        i = sl.stop
    assert tombs > 0
    g.close()
    o.close()


@pytest.mark.parametrize("engine", [0, abi.FLAG_PART_CLAIM, abi.FLAG_ENGINE_ATOMIC])
@pytest.mark.parametrize("retention", [-1, 200_000])
@pytest.mark.parametrize("win", [2, 3, 4])
def test_emit_final_vs_oracle(prod, orc, win, retention, engine):
    """EMIT FINAL with stream-time jumps inside pushes (windows that expire before they close are
    lost, as in Q/suppress.json 'tumbling windows'), HAVING on COUNT(*)."""
    rng = np.random.default_rng(500 + win)
    w = WINDOWS[win]
    hv = {"agg": 0, "op": "GT", "value": 1}
    kw = dict(w, key_type="INT64", col_types=COLS, aggs=ALL_AGGS, having=hv, emit="FINAL", retention_ms=retention)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=engine)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    emitted = 0
    for b in range(6):
        n = 5000
        ts = b * 100_000 + np.sort(rng.integers(0, 80_000, n)) + rng.integers(0, 5_000, n)
        jump = rng.random(n) < 0.002  # single records far ahead: close + expire in one step
        ts = np.where(jump, ts + rng.integers(50_000, 400_000, n), ts)
        ts = np.maximum.accumulate(ts) if b % 2 else ts
        keys = rng.integers(0, 200, n)
        cols = [rng.integers(-9, 9, n).astype(np.int32), rng.integers(-9, 9, n), rng.random(n), rng.random(n)]
        batch = abi.HostBatch(ts, keys=keys, cols=cols)
        assert g.push(batch) == o.push(batch)
        gc, oc = g.changes(), o.changes()
        _assert_changes_equal(gc, oc, g.desc)
        emitted += gc["n"]
    assert emitted > 0
    assert_snap_equal(g.snapshot(), o.snapshot(), g.desc, ABS_SUM, CNT_DBL)
    g.close()
    o.close()


@pytest.mark.parametrize("engine", [0, abi.FLAG_ENGINE_ATOMIC])
@pytest.mark.parametrize("retention", [-1, 90_000])
def test_retention_store_vs_oracle(prod, orc, retention, engine):
    """The store after each push: snapshot, HAVING count, pull queries (keys + window bounds)."""
    rng = np.random.default_rng(17)
    hv = {"agg": 0, "op": "GT", "value": 2}
    kw = dict(window_kind="HOPPING", size_ms=30_000, advance_ms=10_000, grace_ms=5_000, retention_ms=retention,
              key_type="INT64", col_types=COLS, aggs=ALL_AGGS, having=hv, capacity_hint=20_000)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=engine)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    for batch in _batches(rng, 6, 8000, "INT64", 300, 100_000, 10_000, jump=150_000):
        assert g.push(batch) == o.push(batch)
        gs, os_ = g.snapshot(), o.snapshot()
        assert_snap_equal(gs, os_, g.desc, ABS_SUM, CNT_DBL)
        assert g.snapshot_size() == os_["n"]
        assert g.count_rows(hv) == o.snapshot(hv)["n"]
        keys = rng.choice(os_["key"], 10) if os_["n"] else np.array([1])
        q = g.get(keys=keys)
        sel = np.isin(os_["key"], keys)
        assert np.array_equal(q["key"], os_["key"][sel]) and np.array_equal(q["ws"], os_["ws"][sel])
    g.close()
    o.close()


def test_changes_need_the_flag(prod):
    h = abi.AggHandle(prod, abi.make_agg_desc(**dict(WINDOWS[1], key_type="INT64", aggs=[("COUNT_STAR", -1)])))
    h.push(abi.HostBatch(np.arange(10), keys=np.arange(10)))
    with pytest.raises(abi.KsqlHipError):
        h.changes()
    h.close()
    with pytest.raises(abi.KsqlHipError):  # the atomic engine keeps no EMIT CHANGES changelog
        abi.AggHandle(prod, abi.make_agg_desc(**dict(WINDOWS[1], key_type="INT64", aggs=[("COUNT_STAR", -1)],
                                                     flags=abi.FLAG_ENGINE_ATOMIC | abi.FLAG_CHANGELOG)))


# ------------------------------------------------------------------ SESSION windows (R11)

SESSIONS = [dict(window_kind="SESSION", size_ms=20_000, grace_ms=-1),
            dict(window_kind="SESSION", size_ms=5_000, grace_ms=10_000),
            dict(window_kind="SESSION", size_ms=30_000, grace_ms=0, retention_ms=100_000)]


@pytest.mark.parametrize("key_type", ["INT64", "UTF8"])
@pytest.mark.parametrize("having", [None, {"agg": 0, "op": "GT", "value": 2}])
@pytest.mark.parametrize("win", range(len(SESSIONS)))
def test_sessions_vs_oracle(prod, orc, win, having, key_type):
    """Session merges (tombstones of merged-away sessions), late drops against
    streamTime - grace - gap, expiry by session end; per-push changes, the store, pull queries."""
    rng = np.random.default_rng(900 + 10 * win + (having is not None) + (5 if key_type == "UTF8" else 0))
    kw = dict(SESSIONS[win], key_type=key_type, col_types=COLS, aggs=ALL_AGGS, having=having)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=abi.FLAG_CHANGELOG)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    tombs = 0
    for batch in _batches(rng, 5, 5000, key_type, 200, 300_000, 60_000):
        assert g.push(batch) == o.push(batch)
        gc, oc = g.changes(), o.changes()
        _assert_changes_equal(gc, oc, g.desc)
        tombs += int(gc["tombstone"].sum())
        gs, os_ = g.snapshot(having), o.snapshot(having)
        assert_snap_equal(gs, os_, g.desc, ABS_SUM, CNT_DBL)
        assert g.count_rows(having) == os_["n"]
    assert tombs > 0 or win == 1
    if key_type == "INT64":
        s = o.snapshot()
        keys = s["key"][::7][:20]
        q = g.get(keys=keys, ws=(50_000, None))
        sel = np.isin(s["key"], keys) & (s["ws"] >= 50_000)
        assert np.array_equal(q["key"], s["key"][sel]) and np.array_equal(q["we"], s["we"][sel])
    g.close()
    o.close()


def test_sessions_hot_key_and_big_batch(prod, orc):
    """One key with many sessions and many records (sequential replay of a hot key), plus
    100k keys in one push."""
    rng = np.random.default_rng(4242)
    kw = dict(SESSIONS[0], key_type="INT64", col_types=COLS, aggs=ALL_AGGS)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=abi.FLAG_CHANGELOG)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    n = 40_000
    ts = np.sort(rng.integers(0, 4_000_000, n)) + rng.integers(0, 50_000, n)
    keys = np.where(rng.random(n) < 0.3, 7, rng.integers(0, 100_000, n))
    cols = [rng.integers(-9, 9, n).astype(np.int32), rng.integers(-9, 9, n), rng.random(n), rng.random(n)]
    for lo in range(0, n, 20_000):
        b = abi.HostBatch(ts[lo:lo + 20_000], keys=keys[lo:lo + 20_000], cols=[c[lo:lo + 20_000] for c in cols])
        assert g.push(b) == o.push(b)
        _assert_changes_equal(g.changes(), o.changes(), g.desc)
    assert_snap_equal(g.snapshot(), o.snapshot(), g.desc, ABS_SUM, CNT_DBL)
    g.close()
    o.close()


def test_sessions_bench_shape_vs_oracle(prod, orc):
    """bench.py --config session's shape (C2's records, COUNT(*) WINDOW SESSION (1 SECOND)) at
    4M records / 400k card numbers in two pushes: the store, row count and drop counters equal
    the oracle's."""
    from ksql_amd import synth
    n, keys = 4_000_000, 400_000
    card, ts = synth.possible_fraud(0, n, n, keys=keys)
    kw = dict(window_kind="SESSION", size_ms=1000, key_type="INT64", aggs=[("COUNT_STAR", -1)])
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, capacity_hint=3 * keys)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    for lo in (0, n // 2):
        b = abi.HostBatch(ts[lo:lo + n // 2], keys=card[lo:lo + n // 2])
        assert g.push(b) == o.push(b)
    s = o.snapshot()
    assert_snap_equal(g.snapshot(), s, g.desc, ABS_SUM, CNT_DBL)
    assert g.count_rows(None) == s["n"]
    g.close()
    o.close()


def test_sessions_key_range_edges(prod, orc):
    """The session sort runs over key - kmin on the bits of the push's key range: keys at both
    ends of BIGINT (the full 64-bit range, no sentinel key for dropped rows), a push whose
    records are all dropped, a single-key push, dropped rows mixed with the largest key."""
    kw = dict(SESSIONS[0], key_type="INT64", col_types=COLS, aggs=ALL_AGGS)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=abi.FLAG_CHANGELOG)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    rng = np.random.default_rng(77)
    lo64, hi64 = np.iinfo(np.int64).min, np.iinfo(np.int64).max

    def batch(keys, ts, key_valid=None):
        m = len(keys)
        cols = [rng.integers(-9, 9, m).astype(np.int32), rng.integers(-9, 9, m), rng.random(m), rng.random(m)]
        return abi.HostBatch(np.asarray(ts, np.int64), keys=np.asarray(keys, np.int64), key_valid=key_valid, cols=cols)

    pushes = [
        batch([lo64, hi64, 0, lo64, hi64, -1, 1], [10, 20, 30, 40, 50, -5, 60]),
        batch([5, 6, 7], [100, 110, 120], key_valid=[False, False, False]),
        batch([hi64] * 5, [200, 30_000, 30_100, 90_000, 95_000]),
        batch([hi64, 3, hi64, 4], [96_000, 96_500, 97_000, -1], key_valid=[True, False, True, True]),
        batch([lo64 + 1, lo64 + 2, lo64 + 1], [98_000, 98_000, 99_000]),
    ]
    for b in pushes:
        assert g.push(b) == o.push(b)
        _assert_changes_equal(g.changes(), o.changes(), g.desc)
        assert_snap_equal(g.snapshot(), o.snapshot(), g.desc, ABS_SUM, CNT_DBL)
    g.close()
    o.close()


@pytest.mark.parametrize("count_only", [True, False])
def test_sessions_time_span_edges(prod, orc, count_only):
    """Replay records are packed to 8 bytes relative to the push's time base (smallest accepted ts,
    or the stream time before the push when smaller) when the push's times span < 2^32 - 16 ms,
    and kept at 16 bytes otherwise: pushes on both sides of that boundary, a push entirely below
    the stream time (late), dropped rows before the first accepted one, with and without argument
    columns (the sort carries the packed record itself, or row indices and a gather)."""
    rng = np.random.default_rng(78)
    aggs = [("COUNT_STAR", -1)] if count_only else ALL_AGGS
    kw = dict(window_kind="SESSION", size_ms=5_000, grace_ms=2 ** 40, key_type="INT64",
              col_types=[] if count_only else COLS, aggs=aggs)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=abi.FLAG_CHANGELOG)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    edge = 2 ** 32 - 17

    def batch(ts, keys=None, key_valid=None):
        ts = np.asarray(ts, np.int64)
        m = len(ts)
        keys = rng.integers(0, 6, m) if keys is None else np.asarray(keys, np.int64)
        cols = [] if count_only else [rng.integers(-9, 9, m).astype(np.int32), rng.integers(-9, 9, m),
                                        rng.random(m), rng.random(m)]
        return abi.HostBatch(ts, keys=keys, key_valid=key_valid, cols=cols)

    base = 1_000_000
    pushes = [
        batch([base + 5, base, base + 3, -1, base + 7000]),                     # packed, base = tmin
        batch([base + 1000, base + edge - 1000, base + 2000]),                   # span just inside
        batch([base, base + edge + 1000, base + 10]),                            # span just outside
        batch(rng.integers(base, base + 3 * 2 ** 32, 3000)),                     # wide, many records
        batch([7, 3, 9, 5, 1]),                                                  # all below stream time
        batch([base + 3 * 2 ** 32 + 1, base + 3 * 2 ** 32 + 9], key_valid=[False, True]),  # dropped first
        batch(rng.integers(base + 3 * 2 ** 32, base + 3 * 2 ** 32 + 60_000, 2000)),
    ]
    for b in pushes:
        assert g.push(b) == o.push(b)
        _assert_changes_equal(g.changes(), o.changes(), g.desc)
        assert_snap_equal(g.snapshot(), o.snapshot(), g.desc, ABS_SUM, CNT_DBL)
    g.close()
    o.close()


# ------------------------------------------------------------------ SESSION + EMIT FINAL
# VERDICT r05 missing #2 (S/StreamAggregateBuilder.java:310-312, sessionWindowedKStream.emitStrategy(
# onWindowClose())).  The oracle restates Kafka 3.4's per-record check (R11: after every record,
# sessions whose END lies in [max(0, lastClose), close - 1], close = streamTime - grace - gap; pinned
# by Q/suppress.json "should support final results for session windows", test_oracle_golden.py and
# test_gpu_parity.py).  The device derives a push's emissions from that rule (sess_push): sessions
# in the store after the push whose end the push's close passed, plus sessions a record merged away
# after the close before it had passed their end (possible only with RETENTION > gap + grace).

SESSIONS_FINAL = [dict(window_kind="SESSION", size_ms=5_000, grace_ms=10_000),
                  dict(window_kind="SESSION", size_ms=20_000, grace_ms=0),
                  dict(window_kind="SESSION", size_ms=3_000, grace_ms=2_000, retention_ms=60_000)]


@pytest.mark.parametrize("key_type", ["INT64", "UTF8"])
@pytest.mark.parametrize("having", [None, {"agg": 0, "op": "GT", "value": 2}])
@pytest.mark.parametrize("win", range(len(SESSIONS_FINAL)))
def test_sessions_emit_final_vs_oracle(prod, orc, win, having, key_type):
    rng = np.random.default_rng(1200 + 10 * win + (having is not None) + (5 if key_type == "UTF8" else 0))
    kw = dict(SESSIONS_FINAL[win], key_type=key_type, col_types=COLS, aggs=ALL_AGGS, having=having, emit="FINAL")
    g = abi.AggHandle(prod, abi.make_agg_desc(**kw))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    emitted = 0
    for batch in _batches(rng, 6, 4000, key_type, 150, 200_000, 40_000, jump=60_000):
        assert g.push(batch) == o.push(batch)
        gc, oc = g.changes(), o.changes()
        _assert_changes_equal(gc, oc, g.desc)
        assert not gc["tombstone"].any()
        emitted += gc["n"]
        assert_snap_equal(g.snapshot(having), o.snapshot(having), g.desc, ABS_SUM, CNT_DBL)
    assert emitted > 0
    g.close()
    o.close()


@pytest.mark.parametrize("retention", [-1, 40_000])
def test_sessions_emit_final_small_pushes(prod, orc, retention):
    """1-4-record pushes (the reference's emit-at-every-record run), boundary records that merge
    with a session right at the close time, a session extended after it was emitted (RETENTION
    beyond gap + grace keeps it visible)."""
    rng = np.random.default_rng(1300 + (retention > 0))
    kw = dict(window_kind="SESSION", size_ms=5, grace_ms=6, key_type="INT64", col_types=COLS, aggs=ALL_AGGS,
              emit="FINAL", retention_ms=retention)
    g = abi.AggHandle(prod, abi.make_agg_desc(**kw))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    n = 600
    ts = np.cumsum(rng.integers(0, 4, n)) + rng.integers(-15, 3, n)
    ts[rng.random(n) < 0.05] += 25  # jumps: closes several sessions at once
    keys = rng.integers(0, 4, n)
    cols = [rng.integers(-9, 9, n).astype(np.int32), rng.integers(-9, 9, n), rng.random(n), rng.random(n)]
    i = emitted = 0
    while i < n:
        sl = slice(i, min(i + int(rng.integers(1, 5)), n))
        b = abi.HostBatch(ts[sl], keys=keys[sl], cols=[c[sl] for c in cols])
        assert g.push(b) == o.push(b)
        gc, oc = g.changes(), o.changes()
        _assert_changes_equal(gc, oc, g.desc)
        emitted += gc["n"]
        i = sl.stop
    assert emitted > 0
    g.close()
    o.close()


def test_sessions_emit_final_one_push_equals_record_by_record(prod, orc):
    """The same records as ONE push and as one-record pushes: the device's batched rule emits the
    union of what the oracle's per-record checks emit (rows keyed by session)."""
    rng = np.random.default_rng(1400)
    kw = dict(window_kind="SESSION", size_ms=50, grace_ms=30, key_type="INT64", col_types=COLS, aggs=ALL_AGGS,
              emit="FINAL", retention_ms=400)
    n = 3000
    ts = np.cumsum(rng.integers(0, 6, n)) + rng.integers(-60, 5, n)
    keys = rng.integers(0, 40, n)
    cols = [rng.integers(-9, 9, n).astype(np.int32), rng.integers(-9, 9, n), rng.random(n), rng.random(n)]
    g = abi.AggHandle(prod, abi.make_agg_desc(**kw))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    assert g.push(abi.HostBatch(ts, keys=keys, cols=cols)) is not None
    gc = g.changes()
    rows = []
    for r in range(n):
        o.push(abi.HostBatch(ts[r:r + 1], keys=keys[r:r + 1], cols=[c[r:r + 1] for c in cols]))
        oc = o.changes()
        rows += [(int(k), int(s), int(e), int(c)) for k, s, e, c in zip(oc["key"], oc["ws"], oc["we"], oc["values"][0])]
    got = sorted((int(k), int(s), int(e), int(c)) for k, s, e, c in zip(gc["key"], gc["ws"], gc["we"], gc["values"][0]))
    assert got == sorted(rows) and len(rows) > 0
    g.close()
    o.close()
