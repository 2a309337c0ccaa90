"""Pull queries against the HBM-resident table (khip_agg_get) — SURVEY §8(f)-3.

Reference: KsMaterializedWindowTable.get(key, partition, windowStartBounds, windowEndBounds)
and the all-keys scan get(partition, ...) (ksqldb-streams/.../materialization/ks/
KsMaterializedWindowTable.java:70-165): rows of the key whose WINDOWSTART is in the start
bounds and WINDOWEND (= start + size) in the end bounds; unwindowed tables ignore bounds
(KsMaterializedTable.get).  The checker is the oracle's full snapshot filtered in numpy with
the same predicate; the product path filters on the device.  Integer work: bit-exact.
"""
import ctypes as C

import numpy as np
import pytest

from ksql_amd import abi
from test_gpu_parity import ALL_AGGS, ABS_SUM, CNT_DBL, ENGINES, WINDOWS, _random_batch, assert_snap_equal

pytestmark = pytest.mark.gpu

COLS = ["INT32", "INT64", "DOUBLE", "DOUBLE"]
I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


@pytest.fixture(params=list(ENGINES), scope="module")
def engine(request):
    return ENGINES[request.param]


def _filter(o, keys, ws, we, windowed):
    m = np.ones(o["n"], bool)
    if keys is not None and isinstance(o["key"], list):
        ks = set(keys)
        m &= np.array([k in ks for k in o["key"]], bool)
    elif keys is not None:
        m &= np.isin(o["key"], np.asarray(keys, np.int64))
    if windowed:
        lo, hi = ws
        m &= (o["ws"] >= (I64_MIN if lo is None else lo)) & (o["ws"] <= (I64_MAX if hi is None else hi))
        lo, hi = we
        m &= (o["we"] >= (I64_MIN if lo is None else lo)) & (o["we"] <= (I64_MAX if hi is None else hi))
    out = {"n": int(m.sum()), "key": o["key"][m] if not isinstance(o["key"], list) else
           [k for k, t in zip(o["key"], m) if t]}
    for f in ("ws", "we", "rowtime"):
        out[f] = o[f][m]
    out["values"] = [v[m] for v in o["values"]]
    out["nulls"] = [v[m] for v in o["nulls"]]
    return out


def _tables(prod, orc, kw, batches, engine):
    hs = []
    for lib in (prod, orc):
        desc = abi.make_agg_desc(**dict(kw, flags=engine if lib is prod else 0))
        h = abi.AggHandle(lib, desc)
        for b in batches:
            h.push(b)
        hs.append((h, desc))
    return hs


@pytest.mark.parametrize("win", range(len(WINDOWS)))
def test_pull_by_keys_and_bounds(prod, orc, win, engine):
    rng = np.random.default_rng(77 + win)
    batches = [_random_batch(rng, 6000, "INT64", 400, 200_000, 40_000, t0=b * 150_000) for b in range(3)]
    kw = dict(WINDOWS[win], key_type="INT64", col_types=COLS, aggs=ALL_AGGS)
    (g, desc), (o, _) = _tables(prod, orc, kw, batches, engine)
    full = o.snapshot()
    windowed = WINDOWS[win]["window_kind"] != "NONE"
    keys_all = np.unique(full["key"])
    queries = [
        (None, (None, None), (None, None)),                                # scan: the whole table
        (keys_all[:1], (None, None), (None, None)),                        # one key, every window
        (rng.choice(keys_all, 25), (100_000, 300_000), (None, None)),       # WINDOWSTART range
        (rng.choice(keys_all, 25), (None, None), (150_000, 400_000)),       # WINDOWEND range
        (keys_all[::3], (200_000, 200_000), (None, None)),                  # WINDOWSTART = x
        (np.array([123456789, -5, keys_all[0]]), (None, None), (None, None)),  # missing keys
        (None, (10**12, None), (None, None)),                              # empty result
    ]
    for keys, ws, we in queries:
        got = g.get(keys, ws, we)
        exp = _filter(full, keys, ws, we, windowed)
        assert_snap_equal(got, exp, desc, ABS_SUM, CNT_DBL)
    assert g.get([], (None, None), (None, None))["n"] == 0
    g.close()
    o.close()


def test_pull_with_having(prod, orc, engine):
    rng = np.random.default_rng(9)
    batches = [_random_batch(rng, 20000, "INT64", 2000, 100_000, 5_000)]
    kw = dict(WINDOWS[1], key_type="INT64", col_types=COLS, aggs=ALL_AGGS)
    (g, desc), (o, _) = _tables(prod, orc, kw, batches, engine)
    having = {"agg": 0, "op": "GT", "value": 3}
    exp_all = o.snapshot(having)
    keys = np.unique(exp_all["key"])[:50]
    got = g.get(keys, (0, 50_000), (None, None), having=having)
    assert_snap_equal(got, _filter(exp_all, keys, (0, 50_000), (None, None), True), desc, ABS_SUM, CNT_DBL)
    g.close()
    o.close()


def test_pull_sees_closed_windows(prod, orc):
    """Windows evicted to the closed store (grace passed) stay queryable (the reference keeps
    them until retention)."""
    rng = np.random.default_rng(3)
    batches = [_random_batch(rng, 5000, "INT64", 300, 100_000, 1_000, t0=b * 100_000) for b in range(8)]
    kw = dict(window_kind="TUMBLING", size_ms=5000, grace_ms=0, key_type="INT64", col_types=COLS, aggs=ALL_AGGS)
    (g, desc), (o, _) = _tables(prod, orc, kw, batches, 0)
    full = o.snapshot()
    keys = np.unique(full["key"])[:40]
    for ws in [(0, 99_999), (400_000, 800_000), (None, None)]:
        assert_snap_equal(g.get(keys, ws), _filter(full, keys, ws, (None, None), True), desc, ABS_SUM, CNT_DBL)
    g.close()
    o.close()


def test_pull_utf8_keys(prod, orc, engine):
    """`SELECT * FROM hourly_metrics WHERE url = … AND WINDOWSTART = …` over a VARCHAR-keyed table
    (README.md:45-46): key bytes are mapped to dictionary ids by a read-only device probe; keys
    never pushed (and the empty string) match nothing; bounds-only scans work too."""
    rng = np.random.default_rng(4)
    batches = [_random_batch(rng, 5000, "UTF8", 200, 100_000, 5_000) for _ in range(2)]
    kw = dict(WINDOWS[1], key_type="UTF8", col_types=COLS, aggs=ALL_AGGS)
    (g, desc), (o, _) = _tables(prod, orc, kw, batches, engine)
    full = o.snapshot()
    uk = sorted(set(full["key"]))
    queries = [
        (None, (50_000, 50_000)),
        (uk[:1], (None, None)),
        ([uk[i] for i in rng.choice(len(uk), 30)], (20_000, 80_000)),
        ([uk[3], "never-pushed", "", "éè-7", uk[3]], (None, None)),
        (["never-pushed"], (None, None)),
    ]
    for keys, ws in queries:
        assert_snap_equal(g.get(keys, ws), _filter(full, keys, ws, (None, None), True), desc, ABS_SUM, CNT_DBL)
    g.close()
    o.close()


def test_pull_null_arguments_rejected(prod):
    h = abi.AggHandle(prod, abi.make_agg_desc(window_kind="TUMBLING", size_ms=1000))
    q = abi.Pull(3, None, 0, 0, 0, 0)  # keys missing
    s = abi.Snapshot()
    assert prod.agg_get(h.h, C.byref(q), None, C.byref(s)) == -1
    assert prod.agg_get(h.h, None, None, C.byref(s)) == -1
    h.close()


def test_pull_point_lookup_many_partitions(prod, orc):
    """Partition-directed point lookups (≤ 256 keys read only their partitions) on a table large
    enough for many partitions, vs the oracle snapshot; plus a > 256-key lookup (scan path)."""
    rng = np.random.default_rng(11)
    n = 3_000_000
    keys = rng.integers(0, 1_500_000, n)
    ts = np.sort(rng.integers(0, 20_000, n))
    b = abi.HostBatch(ts, keys=keys)
    kw = dict(window_kind="TUMBLING", size_ms=5000, key_type="INT64", aggs=[("COUNT_STAR", -1)])
    (g, desc), (o, _) = _tables(prod, orc, kw, [b], 0)
    full = o.snapshot()
    uk = np.unique(full["key"])
    for q in [uk[:1], rng.choice(uk, 100), np.concatenate([rng.choice(uk, 200), [-1, 10**9]]), rng.choice(uk, 5000)]:
        for ws in [(None, None), (5000, 10_000)]:
            assert_snap_equal(g.get(q, ws), _filter(full, q, ws, (None, None), True), desc)
    g.close()
    o.close()
