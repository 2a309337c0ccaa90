"""Parity of the HIP path (libksqldb_hip.so, through the C ABI) with the reference.

1. The reference's own QTT golden vectors (tests/golden/qtt_*.json), pushed as one
   batch and split into 1-row and 3-row micro-batches (cross-batch state).
2. Seeded random differential tests against the CPU oracle: integer aggregates,
   keys, windows and row times bit-exact; DOUBLE SUM/AVG within the north-star
   relative tolerance 1e-12 (scaled by the sum of |x| to stay meaningful under
   cancellation); DOUBLE MIN/MAX bit-exact (NaN compared as NaN: payload unpinned).
3. Edge cases the reference tests: empty batches, null keys / values / inputs,
   negative timestamps, late records, hot keys, table growth, deletes in joins.
"""
import numpy as np
import pytest

import qtt
from ksql_amd import abi

pytestmark = pytest.mark.gpu

AGG_CASES = qtt.load_cases("agg")
JOIN_CASES = qtt.load_cases("join")
DOUBLE_RTOL = 1e-12  # north_star: DOUBLE SUM/AVG relative tolerance


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


ENGINES = {"part": 0, "part_claim": abi.FLAG_PART_CLAIM, "atomic": abi.FLAG_ENGINE_ATOMIC}


@pytest.fixture(params=list(ENGINES), scope="module")
def engine(request):
    return ENGINES[request.param]


def _emits(case, engine):
    """The global-atomic engine keeps no per-push changelog (EMIT CHANGES); EMIT FINAL it has."""
    return engine != abi.FLAG_ENGINE_ATOMIC or case["desc"].get("emit") == "FINAL"


@pytest.mark.parametrize("split", [None, 1, 3])
@pytest.mark.parametrize("case", AGG_CASES, ids=["%s %s" % (c["source"], c["name"]) for c in AGG_CASES])
def test_qtt_aggregate_golden(prod, orc, case, split, engine):
    """The final table the query emitted (fold of khip_agg_changes over the pushes) equals the
    reference's (last output per (key, window)); and the window store equals the oracle's."""
    if _emits(case, engine):
        assert qtt.compare_agg(case, qtt.run_agg_case(prod, case, split, flags=engine)) == []
    desc = qtt.case_desc(case)
    assert_snap_equal(qtt.run_agg_store(prod, case, split, flags=engine), qtt.run_agg_store(orc, case, split), desc)


@pytest.mark.parametrize("case", AGG_CASES, ids=["%s %s" % (c["source"], c["name"]) for c in AGG_CASES])
def test_qtt_output_sequence(prod, case, engine):
    """Every output record of the reference, in order (HAVING tombstones, EMIT FINAL), from
    one-record pushes (the reference's cache-off run)."""
    if not _emits(case, engine):
        pytest.skip("EMIT CHANGES changelog: partitioned engine only")
    assert qtt.compare_outputs(case, qtt.run_agg_outputs(prod, case, 1, flags=engine)) == []


@pytest.mark.parametrize("case", JOIN_CASES, ids=["%s %s" % (c["source"], c["name"]) for c in JOIN_CASES])
def test_qtt_join_golden(prod, case):
    rows = qtt.run_join_case(prod, case)
    assert qtt.compare_join(case, rows) == []


# ----------------------------------------------------------------- differential

def _nan_eq(a, b):
    return (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)


def assert_snap_equal(g, o, desc, abs_sum_agg=None, count_agg=None):
    """Integer results, keys, windows, row times, null flags and DOUBLE MIN/MAX bit-exact.
    DOUBLE-input SUM/AVG within DOUBLE_RTOL (north star 1e-12) relative to the magnitude the
    summation error is bounded by: for SUM max(|sum|, sum|x|), for AVG max(|avg|, sum|x| / n)
    — sum|x| from the abs_sum_agg column (SUM over |x|), n from count_agg (COUNT(x)).  Without
    them (non-negative inputs) the bound is the plain relative error.  AVG of an integer
    column is an exact int sum divided once, so it is compared bit-exact."""
    assert g["n"] == o["n"], (g["n"], o["n"])
    if isinstance(g["key"], list):
        assert g["key"] == o["key"]
    else:
        assert np.array_equal(g["key"], o["key"])
    assert np.array_equal(g["ws"], o["ws"])
    assert np.array_equal(g["we"], o["we"])
    assert np.array_equal(g["rowtime"], o["rowtime"])
    rts = abi.result_types(desc)
    for a in range(desc.n_aggs):
        assert np.array_equal(g["nulls"][a], o["nulls"][a]), "nulls of agg %d" % a
        kind = desc.aggs[a].kind
        gv, ov = g["values"][a], o["values"][a]
        in_dbl = kind != abi.AGG["COUNT_STAR"] and desc.col_types[desc.aggs[a].arg_col] == abi.TYPE["DOUBLE"]
        dbl_sum = in_dbl and kind in (abi.AGG["SUM"], abi.AGG["AVG"])
        if dbl_sum:
            scale = np.abs(ov)
            if abs_sum_agg is not None:
                bound = np.abs(o["values"][abs_sum_agg])
                if kind == abi.AGG["AVG"]:
                    assert count_agg is not None, "AVG bound needs the non-null count"
                    bound = bound / np.maximum(o["values"][count_agg], 1)
                scale = np.maximum(scale, bound)
            err = np.abs(gv - ov)
            ok = (err <= DOUBLE_RTOL * scale + 1e-300) | (np.isnan(gv) & np.isnan(ov))
            assert ok.all(), "agg %d max rel err %g" % (a, np.max(err / np.maximum(scale, 1e-300)))
        else:
            assert _nan_eq(gv, ov).all(), "agg %d" % a


def _random_batch(rng, n, key_type, nkeys, span, disorder, null_frac=0.05, t0=0, neg_ts=0.0):
    ts = t0 + np.sort(rng.integers(0, span, n)) + rng.integers(0, max(disorder, 1), n)
    if neg_ts:
        ts = np.where(rng.random(n) < neg_ts, -rng.integers(1, 100, n), ts)
    kv = rng.random(n) > null_frac
    rv = rng.random(n) > null_frac
    c_i32 = rng.integers(-2**31, 2**31, n).astype(np.int32)
    c_i64 = rng.integers(-2**62, 2**62, n) * rng.integers(-1, 2, n)  # wraps on SUM
    c_dbl = rng.uniform(-1e3, 1e3, n) * np.where(rng.random(n) < 0.01, 1e6, 1.0)
    c_abs = np.abs(c_dbl)
    vals = [rng.random(n) > null_frac for _ in range(4)]
    vals[3] = vals[2]  # |x| null iff x null
    cols = [c_i32, c_i64, c_dbl, c_abs]
    if key_type == "UTF8":
        ids = rng.integers(0, nkeys, n)
        # dictionary keys and digit keys (inline ids, khip_dict.hpp; "00.." keeps leading zeros apart)
        keys = ["%d" % k if k % 3 == 0 else "00%d" % k if k % 5 == 0 else "k%d" % k if k % 7 else "éè-%d" % k
                for k in ids]
        return abi.HostBatch(ts, utf8_keys=keys, key_valid=kv, row_valid=rv, cols=cols, col_valid=vals)
    keys = rng.integers(-nkeys, nkeys, n) * 1_000_003
    return abi.HostBatch(ts, keys=keys, key_valid=kv, row_valid=rv, cols=cols, col_valid=vals)


ALL_AGGS = [("COUNT_STAR", -1), ("COUNT", 0), ("SUM", 0), ("SUM", 1), ("SUM", 2), ("MIN", 0), ("MAX", 0),
            ("MIN", 1), ("MAX", 1), ("MIN", 2), ("MAX", 2), ("AVG", 0), ("AVG", 1), ("AVG", 2), ("COUNT", 2),
            ("SUM", 3)]
ABS_SUM = len(ALL_AGGS) - 1  # SUM(|x|) of the DOUBLE column: the summation error bound
CNT_DBL = len(ALL_AGGS) - 2  # COUNT(x) of the DOUBLE column: AVG's divisor

WINDOWS = [
    dict(window_kind="NONE"),
    dict(window_kind="TUMBLING", size_ms=5000, grace_ms=-1),
    dict(window_kind="TUMBLING", size_ms=5000, grace_ms=1000),
    dict(window_kind="HOPPING", size_ms=60_000, advance_ms=10_000, grace_ms=30_000),
    dict(window_kind="HOPPING", size_ms=30_000, advance_ms=7_000, grace_ms=0),
]


def _run_both(prod, orc, desc_kw, batches, having=None, engine=0):
    out = []
    for lib in (prod, orc):
        desc = abi.make_agg_desc(**dict(desc_kw, flags=engine if lib is prod else 0))
        h = abi.AggHandle(lib, desc)
        stats = [h.push(b) for b in batches]
        out.append((h.snapshot(having), stats, desc))
        h.close()
    return out


@pytest.mark.parametrize("key_type", ["INT64", "UTF8"])
@pytest.mark.parametrize("win", range(len(WINDOWS)))
@pytest.mark.parametrize("nbatches", [1, 4])
def test_random_vs_oracle(prod, orc, key_type, win, nbatches, engine):
    rng = np.random.default_rng(1000 * win + nbatches + (7 if key_type == "UTF8" else 0))
    batches = [_random_batch(rng, 4000, key_type, 300, 200_000, 40_000, t0=b * 150_000, neg_ts=0.01)
               for b in range(nbatches)]
    kw = dict(WINDOWS[win], key_type=key_type, col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"], aggs=ALL_AGGS)
    (g, gs, desc), (o, os_, _) = _run_both(prod, orc, kw, batches, engine=engine)
    assert gs == os_
    assert_snap_equal(g, o, desc, ABS_SUM, CNT_DBL)


@pytest.mark.parametrize("having", [{"agg": 0, "op": "GT", "value": 3}, {"agg": 4, "op": "LE", "value": 10.5},
                                    {"agg": 5, "op": "NE", "value": 0}])
def test_having_vs_oracle(prod, orc, having, engine):
    rng = np.random.default_rng(5)
    batches = [_random_batch(rng, 20000, "INT64", 2000, 100_000, 5_000)]
    kw = dict(WINDOWS[1], key_type="INT64", col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"], aggs=ALL_AGGS)
    (g, _, desc), (o, _, _) = _run_both(prod, orc, kw, batches, having, engine=engine)
    assert_snap_equal(g, o, desc, ABS_SUM, CNT_DBL)
    h = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=engine)))
    h.push(batches[0])
    assert h.count_rows(having) == o["n"]
    h.close()
    # the query's own HAVING in the descriptor: the count the aggregate kernel maintains
    h = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=engine, having=having)))
    h.push(batches[0])
    assert h.count_rows(having) == o["n"]
    h.close()


@pytest.mark.parametrize("win", [1, 3, 4])
def test_maintained_having_count_across_pushes(prod, orc, win, engine):
    """HAVING counts kept per partition (and for evicted closed windows) across micro-batches
    with late records and eviction, checked after every push against the oracle's table."""
    rng = np.random.default_rng(50 + win)
    having = {"agg": 0, "op": "GT", "value": 3}
    kw = dict(WINDOWS[win], key_type="INT64", col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"], aggs=ALL_AGGS,
              capacity_hint=200_000)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=engine, having=having)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    for b in range(5):
        batch = _random_batch(rng, 30_000, "INT64", 3000, 120_000, 20_000, t0=b * 100_000)
        assert g.push(batch) == o.push(batch)
        assert g.count_rows(having) == o.snapshot(having)["n"]
    g.close()
    o.close()


def test_empty_and_all_null_batches(prod, orc, engine):
    kw = dict(WINDOWS[3], key_type="INT64", col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"], aggs=ALL_AGGS)
    empty = abi.HostBatch(np.zeros(0, np.int64), keys=np.zeros(0, np.int64),
                          cols=[np.zeros(0, np.int32), np.zeros(0, np.int64), np.zeros(0), np.zeros(0)])
    n = 1000
    allnull = abi.HostBatch(np.arange(n), keys=np.arange(n), key_valid=np.zeros(n, bool),
                            cols=[np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n), np.zeros(n)])
    nullvals = abi.HostBatch(np.arange(n), keys=np.arange(n) % 10,
                             cols=[np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n), np.zeros(n)],
                             col_valid=[np.zeros(n, bool)] * 4)
    (g, gs, desc), (o, os_, _) = _run_both(prod, orc, kw, [empty, allnull, nullvals, empty], engine=engine)
    assert gs == os_
    assert gs[1]["dropped_null_key"] == n
    assert_snap_equal(g, o, desc, ABS_SUM, CNT_DBL)
    assert g["n"] > 0 and g["nulls"][5].all()  # MIN over only-null inputs is NULL (entry exists)


def test_hot_key_contention(prod, orc, engine):
    n = 200_000
    rng = np.random.default_rng(3)
    b = abi.HostBatch(np.arange(n) // 10, keys=np.zeros(n, np.int64),
                      cols=[rng.integers(-100, 100, n).astype(np.int32), rng.integers(-2**40, 2**40, n),
                            rng.random(n), rng.random(n)])
    kw = dict(WINDOWS[3], key_type="INT64", col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"], aggs=ALL_AGGS)
    (g, gs, desc), (o, os_, _) = _run_both(prod, orc, kw, [b], engine=engine)
    assert gs == os_
    assert_snap_equal(g, o, desc, ABS_SUM, CNT_DBL)


def test_table_growth_and_resume(prod, orc, engine):
    # capacity hint far too small: forces resume passes after probe exhaustion + rehash
    rng = np.random.default_rng(11)
    batches = [_random_batch(rng, 60000, "INT64", 50_000, 1_000_000, 10, null_frac=0.0, t0=i * 1_000_000)
               for i in range(3)]
    kw = dict(WINDOWS[3], key_type="INT64", col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"], aggs=ALL_AGGS,
              capacity_hint=16)
    (g, gs, desc), (o, os_, _) = _run_both(prod, orc, kw, batches, engine=engine)
    assert gs == os_
    assert_snap_equal(g, o, desc, ABS_SUM, CNT_DBL)


@pytest.mark.parametrize("win", [0, 1, 3])
def test_many_partitions_vs_oracle(prod, orc, win, engine):
    # a large capacity hint gives 2^14 partitions: two-level scatter (buckets → partitions)
    # and, while the window range fits, the packed-identity CAS; 3 pushes with eviction
    rng = np.random.default_rng(77 + win)
    batches = [_random_batch(rng, 150_000, "INT64", 40_000, 300_000, 20_000, t0=b * 200_000) for b in range(3)]
    kw = dict(WINDOWS[win], key_type="INT64", col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"], aggs=ALL_AGGS,
              capacity_hint=30_000_000)
    (g, gs, desc), (o, os_, _) = _run_both(prod, orc, kw, batches, engine=engine)
    assert gs == os_
    assert_snap_equal(g, o, desc, ABS_SUM, CNT_DBL)


@pytest.mark.parametrize("win", [1, 3])
def test_max_partitions_vs_oracle(prod, orc, win):
    # a hint past 2^14 x 0.7 LDS tables of groups gives 2^15 partitions (128 KB LDS histogram)
    rng = np.random.default_rng(91 + win)
    batches = [_random_batch(rng, 200_000, "INT64", 60_000, 300_000, 20_000, t0=b * 200_000) for b in range(2)]
    kw = dict(WINDOWS[win], key_type="INT64", col_types=["INT32", "INT64", "DOUBLE", "DOUBLE"],
              aggs=[("COUNT_STAR", -1), ("SUM", 1), ("MAX", 0)],
              capacity_hint=60_000_000)
    (g, gs, desc), (o, os_, _) = _run_both(prod, orc, kw, batches)
    assert gs == os_
    assert_snap_equal(g, o, desc)


def test_special_doubles(prod, orc):
    vals = np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 1e-310, -1e-310, 5.0, np.nan, -0.0])
    n = len(vals)
    b = abi.HostBatch(np.arange(n), keys=np.zeros(n, np.int64), cols=[vals])
    kw = dict(window_kind="NONE", key_type="INT64", col_types=["DOUBLE"],
              aggs=[("MIN", 0), ("MAX", 0), ("COUNT", 0)])
    for split in (1, n):
        res = []
        for lib in (prod, orc):
            h = abi.AggHandle(lib, abi.make_agg_desc(**kw))
            for lo in range(0, n, split):
                h.push(abi.HostBatch(np.arange(lo, min(lo + split, n)), keys=np.zeros(min(split, n - lo), np.int64),
                                     cols=[vals[lo:lo + split]]))
            res.append(h.snapshot())
            h.close()
        g, o = res
        assert g["values"][0][0] == -np.inf and np.isnan(g["values"][1][0])
        assert g["values"][2][0] == o["values"][2][0] == n


def test_device_batch_equals_host_batch(prod):
    torch = pytest.importorskip("torch")
    n = 50_000
    card, ts = (x for x in __import__("ksql_amd.synth", fromlist=["x"]).possible_fraud(0, n, n, keys=5000))
    kw = dict(window_kind="TUMBLING", size_ms=5000, key_type="INT64", aggs=[("COUNT_STAR", -1)])
    h1 = abi.AggHandle(prod, abi.make_agg_desc(**kw))
    h1.push(abi.HostBatch(ts, keys=card))
    s1 = h1.snapshot()
    dk = torch.from_numpy(card).cuda()
    dt = torch.from_numpy(ts).cuda()
    torch.cuda.synchronize()
    h2 = abi.AggHandle(prod, abi.make_agg_desc(**kw))
    h2.push(abi.DeviceBatch(dt, keys=dk))
    s2 = h2.snapshot()
    for f in ("key", "ws", "rowtime"):
        assert np.array_equal(s1[f], s2[f])
    assert np.array_equal(s1["values"][0], s2["values"][0])


# ----------------------------------------------------------------------- join

def _join_events(rng, nkeys, rounds):
    ev = []
    for r in range(rounds):
        m = int(rng.integers(1, 3000))
        keys = rng.integers(0, nkeys, m)
        ev.append(("T", keys, rng.random(m) > 0.02, rng.random(m) > 0.1,
                   [rng.integers(0, 3, m).astype(np.int32), rng.uniform(-5, 5, m), rng.integers(-9, 9, m)],
                   [rng.random(m) > 0.05 for _ in range(3)]))
        m = int(rng.integers(1, 5000))
        ev.append(("S", rng.integers(-5, nkeys + 50, m), rng.random(m) > 0.02, rng.random(m) > 0.02,
                   np.where(rng.random(m) < 0.01, -1, rng.integers(0, 10**6, m))))
    return ev


@pytest.mark.parametrize("join_type", ["LEFT", "INNER"])
@pytest.mark.parametrize("where", [None, {"col": 0, "op": "EQ", "i64": 2, "f64": 2.0},
                                   {"col": 1, "op": "GT", "i64": 0, "f64": 0.5}])
def test_join_random_vs_oracle(prod, orc, join_type, where):
    rng = np.random.default_rng(21)
    events = _join_events(rng, 4000, 6)
    res = []
    for lib in (prod, orc):
        t = abi.TableHandle(lib, ["INT32", "DOUBLE", "INT64"], capacity_hint=64)
        outs = []
        for e in events:
            if e[0] == "T":
                _, keys, kv, rv, cols, cv = e
                t.upsert(abi.HostBatch(np.zeros(len(keys), np.int64), keys=keys, key_valid=kv, row_valid=rv,
                                       cols=cols, col_valid=cv))
            else:
                _, keys, kv, rv, ts = e
                outs.append(t.probe(abi.HostBatch(ts, keys=keys, key_valid=kv, row_valid=rv), join_type, where))
        outs.append(t.size())
        res.append(outs)
        t.close()
    g, o = res
    assert g[-1] == o[-1]
    for a, b in zip(g[:-1], o[:-1]):
        assert a["n"] == b["n"]
        assert np.array_equal(a["stream_row"], b["stream_row"])
        assert np.array_equal(a["matched"], b["matched"])
        for c in range(3):
            assert np.array_equal(a["nulls"][c], b["nulls"][c])
            assert np.array_equal(a["cols"][c][~a["nulls"][c]], b["cols"][c][~b["nulls"][c]])


@pytest.mark.parametrize("layout", ["dense", "quarter", "spread"])
@pytest.mark.parametrize("ctype", ["INT32", "INT64"])
def test_join_dense_index_vs_oracle(prod, orc, ctype, layout):
    """One value column: the probe index (khip_join.hip) — dense keys: the dense cell index
    ("quarter": three values and no NULL, so 2-bit cells, until a NULL value (step 5) moves it to
    byte cells);
    keys spread far past 4x their count: the hashed index (8-byte words, one 16-byte read per
    probe) — is built on the first probe, kept in step by upserts (deletes, NULL values), dropped
    when a key or a value leaves its ranges and rebuilt by the next probe (or the slot table probed
    when no index fits) — host and device probe outputs equal the oracle's after every step."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng((31 if ctype == "INT32" else 32) + (layout == "spread") + 7 * (layout == "quarter"))
    tables = [abi.TableHandle(lib, [ctype], capacity_hint=64) for lib in (prod, orc)]
    dt = np.int32 if ctype == "INT32" else np.int64
    spread = (lambda k: k * 1000003 + 7) if layout == "spread" else (lambda k: k)
    for step in range(8):
        m = int(rng.integers(500, 3000))
        keys = spread(rng.integers(0, 5000, m))
        vals = rng.integers(0, 3, m).astype(dt)
        if step == 4:
            keys[0] = 10**9 if layout != "spread" else -(2**62)  # a key far outside the index range: index dropped, then rebuilt
        if step == 6:
            vals[0] = dt(2**30) if ctype == "INT32" else dt(2**50)  # a value outside the cell width
        rv = rng.random(m) > 0.1
        cv = rng.random(m) > 0.05
        if layout == "quarter":
            cv = np.ones(m, bool)
            cv[0] = step != 5
        for t in tables:
            t.upsert(abi.HostBatch(np.zeros(m, np.int64), keys=keys, row_valid=rv, cols=[vals], col_valid=[cv]))
        k = int(rng.integers(1000, 9000))
        pk = spread(rng.integers(-10, 5200, k))
        pk[::17] += 1  # (spread: keys between the table's)
        pts = np.where(rng.random(k) < 0.01, -1, rng.integers(0, 10**6, k))
        pkv, prv = rng.random(k) > 0.02, rng.random(k) > 0.02
        where = {"col": 0, "op": "EQ", "i64": 2, "f64": 2.0} if step % 2 else None
        for jt in ("LEFT", "INNER"):
            g, o = (t.probe(abi.HostBatch(pts, keys=pk, key_valid=pkv, row_valid=prv), jt, where) for t in tables)
            assert g["n"] == o["n"]
            assert np.array_equal(g["stream_row"], o["stream_row"]) and np.array_equal(g["matched"], o["matched"])
            assert np.array_equal(g["nulls"][0], o["nulls"][0])
            assert np.array_equal(g["cols"][0][~g["nulls"][0]], o["cols"][0][~o["nulls"][0]])
            # device probe: row-aligned bitmaps and column
            dk, dts = torch.from_numpy(pk).cuda(), torch.from_numpy(pts).cuda()
            kvb = abi.bitmap_torch(torch.from_numpy(pkv).cuda())
            rvb = abi.bitmap_torch(torch.from_numpy(prv).cuda())
            nb = (k + 7) // 8
            emit = torch.zeros(nb, dtype=torch.uint8, device="cuda")
            matched = torch.zeros(nb, dtype=torch.uint8, device="cuda")
            col = torch.zeros(k, dtype=torch.int32 if ctype == "INT32" else torch.int64, device="cuda")
            null = torch.zeros(nb, dtype=torch.uint8, device="cuda")
            n_emit = tables[0].probe_device(abi.DeviceBatch(dts, keys=dk, key_valid=kvb, row_valid=rvb), jt, where,
                                            emit, matched, [col], [null])
            assert n_emit == o["n"]
            e = np.unpackbits(emit.cpu().numpy(), bitorder="little")[:k].astype(bool)
            assert np.array_equal(np.nonzero(e)[0], o["stream_row"])
            mt = np.unpackbits(matched.cpu().numpy(), bitorder="little")[:k].astype(bool)
            assert np.array_equal(mt[o["stream_row"]], o["matched"].astype(bool))
            nl = np.unpackbits(null.cpu().numpy(), bitorder="little")[:k].astype(bool)
            assert np.array_equal(nl[o["stream_row"]], o["nulls"][0])
            cv_ = col.cpu().numpy()[o["stream_row"]]
            assert np.array_equal(cv_[~o["nulls"][0]], o["cols"][0][~o["nulls"][0]])
    for t in tables:
        t.close()
