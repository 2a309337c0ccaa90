"""Pane aggregation in the partitioned engine's merge (k_part_merge, HOPPING windows whose size is a
multiple of the advance): a record whose windows are all open updates its pane (key, advance slice)
once, and each pane is folded into its F windows after the records; records with closed (late)
windows update their open windows directly, in the same LDS table.  Panes need partitions with at
least one full chunk of records (thousands), so these pushes are large and the keys few.  Checked
against the oracle: snapshots, EMIT CHANGES rows and tombstones, pull queries; DOUBLE sums within
the tolerance of a reordered sum (1e-12 x sum |x|)."""
import numpy as np
import pytest

from ksql_amd import abi
from test_gpu_parity import ABS_SUM, ALL_AGGS, CNT_DBL, _random_batch, assert_snap_equal

pytestmark = pytest.mark.gpu

COLS = ["INT32", "INT64", "DOUBLE", "DOUBLE"]


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


@pytest.mark.parametrize("win", [dict(size_ms=60_000, advance_ms=10_000, grace_ms=30_000),
                                 dict(size_ms=30_000, advance_ms=5_000, grace_ms=0),
                                 dict(size_ms=20_000, advance_ms=10_000, grace_ms=-1)])
def test_panes_vs_oracle(prod, orc, win):
    rng = np.random.default_rng(41 + win["advance_ms"] + win["grace_ms"])
    kw = dict(window_kind="HOPPING", key_type="INT64", col_types=COLS, aggs=ALL_AGGS, **win)
    g = abi.AggHandle(prod, abi.make_agg_desc(**dict(kw, flags=abi.FLAG_CHANGELOG)))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    t0 = 0
    for b in range(3):
        batch = _random_batch(rng, 600_000, "INT64", 24, 400_000, 45_000, t0=t0)
        t0 += 300_000
        assert g.push(batch) == o.push(batch)
        gc, oc = g.changes(), o.changes()
        assert_snap_equal(gc, oc, g.desc, ABS_SUM, CNT_DBL)
        assert np.array_equal(gc["tombstone"], oc["tombstone"])
        assert_snap_equal(g.snapshot(), o.snapshot(), g.desc, ABS_SUM, CNT_DBL)
    s = o.snapshot()
    keys = s["key"][::5][:10]
    q = g.get(keys=keys)
    sel = np.isin(s["key"], keys)
    assert np.array_equal(q["key"], s["key"][sel]) and np.array_equal(q["ws"], s["ws"][sel])
    g.close()
    o.close()


def test_panes_c3_shape_vs_oracle(prod, orc):
    """C3's query shape (SUM / AVG / MIN / MAX of one DOUBLE with nulls, HOPPING 60 s / 10 s,
    grace 60 s) over in-order micro-batches with disorder: the one-column update path."""
    rng = np.random.default_rng(7)
    kw = dict(window_kind="HOPPING", size_ms=60_000, advance_ms=10_000, grace_ms=60_000, key_type="INT64",
              col_types=["DOUBLE"], aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0), ("COUNT", 0)])
    g = abi.AggHandle(prod, abi.make_agg_desc(**kw))
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    abs_sum = 0.0
    for b in range(3):
        n = 500_000
        ts = b * 200_000 + np.sort(rng.integers(0, 200_000, n)) + rng.integers(0, 20_000, n)
        val = rng.normal(0, 100, n)
        abs_sum += float(np.abs(val).sum())
        batch = abi.HostBatch(ts, keys=rng.integers(0, 40, n), cols=[val], col_valid=[rng.random(n) > 0.01])
        assert g.push(batch) == o.push(batch)
    gs, os_ = g.snapshot(), o.snapshot()
    assert gs["n"] == os_["n"] and np.array_equal(gs["key"], os_["key"]) and np.array_equal(gs["ws"], os_["ws"])
    assert np.array_equal(gs["rowtime"], os_["rowtime"])
    for a in (2, 3, 4):  # MIN, MAX, COUNT: exact
        assert np.array_equal(gs["values"][a], os_["values"][a]), a
    np.testing.assert_allclose(gs["values"][0], os_["values"][0], rtol=0, atol=1e-12 * abs_sum)
    np.testing.assert_allclose(gs["values"][1], os_["values"][1], rtol=0, atol=1e-12 * abs_sum)
    g.close()
    o.close()
