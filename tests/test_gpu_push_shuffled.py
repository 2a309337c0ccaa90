"""khip_agg_push_shuffled (ABI 6): the rows a shuffle packed / received go straight into the
GROUP BY's aggregation (the repartition topic read back by StreamAggregateBuilder,
S/StreamGroupByBuilderBase.java:101-103).  Every case pushes the same packed rows through
khip_agg_push_shuffled and through khip_shuffle_unpack + khip_agg_push on the product, and the
rows' source records through the oracle (re-keyed by the GROUP BY column, null keys / rows and
negative ts dropped as the shuffle does); tables, batch statistics and (where asked) changelogs
agree.  Cases: the value pipeline reading the rows where they lie (SUM / AVG / MIN / MAX / COUNT,
TUMBLING and HOPPING, INT32 / INT64 / DOUBLE arguments with nulls, the GROUP BY column before or
after the argument), pushes it declines (late records: the unpacked general path), aggregates it
does not take (COUNT(*) alone, several argument columns), and schema mismatches (errors)."""
import zlib

import numpy as np
import pytest

from ksql_amd import abi
from test_gpu_parity import assert_snap_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def _source(rng, n, groups, span, t0, types, disorder=300, late=0.0):
    ts = t0 + (np.arange(n) * span) // n + rng.integers(0, disorder, n)
    if late:
        ts[rng.random(n) < late] -= 4 * span
    cols, valid = [], []
    for t in types:
        if t == "INT32":
            c = rng.integers(-2**31, 2**31, n).astype(np.int32)
        elif t == "INT64":
            c = rng.integers(-10**12, 10**12, n)
        else:  # non-negative: DOUBLE sums are compared relative to the sum (the paths add in other orders)
            c = rng.uniform(0, 1e3, n)
        cols.append(c)
        valid.append(rng.random(n) > 0.05)
    return ts, cols, valid


def _dev(ts, cols, valid, types):
    import torch
    tdt = {"INT32": torch.int32, "INT64": torch.int64, "DOUBLE": torch.float64}
    tc = [torch.as_tensor(c, dtype=tdt[t], device="cuda") for c, t in zip(cols, types)]
    tv = [abi.bitmap_torch(torch.as_tensor(v, device="cuda")) for v in valid]
    return abi.DeviceBatch(torch.as_tensor(ts, dtype=torch.int64, device="cuda"), cols=tc, col_valid=tv)


def _run(prod, orc, types, key_col, aggs, win, pushes, changes=False, late=0.0, expect_rows_path=None):
    rng = np.random.default_rng(zlib.crc32(repr((types, key_col, aggs, win, late)).encode()))
    kw = dict(key_type="INT64", col_types=types, aggs=aggs, capacity_hint=1 << 22, **win)
    flags = (abi.FLAG_CHANGELOG if changes else 0)
    g = abi.AggHandle(prod, abi.make_agg_desc(flags=flags | abi.FLAG_PROFILE, **kw))
    u = abi.AggHandle(prod, abi.make_agg_desc(flags=flags, **kw))
    o = abi.AggHandle(orc, abi.make_agg_desc(flags=flags, **kw))
    sh = abi.ShuffleHandle(prod, 1, key_col, types)
    span = 30_000
    for p in range(pushes):
        n = 300_000
        ts, cols, valid = _source(rng, n, 20_000, span, p * span, types, late=late)
        cols[key_col] = rng.integers(0, 20_000, n).astype(cols[key_col].dtype)  # the new GROUP BY key
        send, counts = sh.pack(_dev(ts, cols, valid, types))
        m = int(sum(counts))
        gs = g.push_shuffled(sh, send, m)
        key, kts, ucols, uvalid = sh.unpack(send, m)
        us = u.push(abi.DeviceBatch(kts, keys=key, cols=ucols, col_valid=uvalid))
        keep = valid[key_col] & (ts >= 0)  # the shuffle drops null new keys and negative ts
        os_ = o.push(abi.HostBatch(ts[keep], keys=cols[key_col][keep].astype(np.int64),
                                   cols=[c[keep] for c in cols], col_valid=[v[keep] for v in valid]))
        assert gs == us == os_, (gs, us, os_)
        if changes:
            gc, oc = g.changes(), o.changes()
            assert_snap_equal(gc, oc, g.desc)
    assert_snap_equal(g.snapshot(), o.snapshot(), g.desc)
    assert_snap_equal(u.snapshot(), o.snapshot(), u.desc)
    kt = g.kernel_times()
    for h in (g, u, o):
        h.close()
    sh.close()
    if expect_rows_path is not None:
        assert (kt["c1_pushes"] == pushes) == expect_rows_path, kt
    return kt


TUMBLING = dict(window_kind="TUMBLING", size_ms=5000)
HOPPING = dict(window_kind="HOPPING", size_ms=6000, advance_ms=2000, grace_ms=30_000)


@pytest.mark.parametrize("win", [TUMBLING, HOPPING], ids=["tumbling", "hopping"])
@pytest.mark.parametrize("types,key_col,aggs", [
    (["INT64", "INT64"], 0, [("SUM", 1)]),                                   # C5's query
    (["DOUBLE", "INT32"], 1, [("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0)]),  # key after the argument
    (["INT64", "INT32", "INT64"], 0, [("COUNT", 1), ("SUM", 1), ("COUNT_STAR", -1)]),
], ids=["sum_i64", "f64_key_after", "i32_three_cols"])
def test_push_shuffled_value_pipeline(prod, orc, types, key_col, aggs, win):
    _run(prod, orc, types, key_col, aggs, win, 3, expect_rows_path=True)


def test_push_shuffled_changelog(prod, orc):
    _run(prod, orc, ["INT64", "INT64"], 0, [("SUM", 1)], TUMBLING, 2, changes=True, expect_rows_path=True)


def test_push_shuffled_declined_and_unpacked(prod, orc):
    """Late records (grace 0): the value pipeline declines, the rows are unpacked and take the
    general path; COUNT(*) alone and two argument columns never take the rows path."""
    late = dict(window_kind="TUMBLING", size_ms=5000, grace_ms=0)
    _run(prod, orc, ["INT64", "INT64"], 0, [("SUM", 1)], late, 2, late=0.02, expect_rows_path=False)
    _run(prod, orc, ["INT64", "INT64"], 0, [("COUNT_STAR", -1)], TUMBLING, 2, expect_rows_path=None)
    _run(prod, orc, ["INT64", "INT64", "DOUBLE"], 0, [("SUM", 1), ("SUM", 2)], TUMBLING, 2, expect_rows_path=None)


def test_push_shuffled_schema_errors(prod):
    sh = abi.ShuffleHandle(prod, 1, 0, ["INT64", "INT64"])
    bad = [abi.make_agg_desc(key_type="INT64", col_types=["INT64"], aggs=[("SUM", 0)], window_kind="TUMBLING",
                             size_ms=1000),
           abi.make_agg_desc(key_type="INT64", col_types=["INT64", "DOUBLE"], aggs=[("SUM", 1)],
                             window_kind="TUMBLING", size_ms=1000),
           abi.make_agg_desc(key_type="UTF8", col_types=["INT64", "INT64"], aggs=[("SUM", 1)],
                             window_kind="TUMBLING", size_ms=1000)]
    for d in bad:
        h = abi.AggHandle(prod, d)
        with pytest.raises(abi.KsqlHipError):
            h.push_shuffled(sh, None, 0)
        h.close()
    sh.close()
