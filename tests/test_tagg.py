"""Table aggregation (CREATE TABLE .. AS SELECT .. FROM <TABLE> GROUP BY ..): khip_agg_push_table
against the QTT table-source cases (tests/golden/qtt_tagg.json, extracted from count.json,
average-udaf.json and group-by.json) and against the oracle's R12 restatement on random source-table
changelogs (updates that move keys between groups, deletes, NULL GROUP BY values and arguments,
repeated keys inside one push, INT wrap-around, STRING and BIGINT keys on both sides).

Comparison: integers exact; DOUBLE SUM/AVG within 1e-12 relative to the sum of |x| the group's
updates touched (the device folds a push's adds/undos per group in no fixed order — LDS atomics on
the delta path, agent-scope atomics on the atomic path — and nets each source key's changes inside
one push: an intermediate row's +x / -x are not applied)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import qtt
from ksql_amd import abi

CASES = qtt.load_cases("tagg")


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


@pytest.mark.parametrize("case", CASES, ids=[c["source"] for c in CASES])
@pytest.mark.parametrize("split", [None, 1, 2])
def test_oracle_tagg_golden(orc, case, split):
    errs = qtt.compare_agg(case, qtt.run_tagg_case(orc, case, split))
    assert not errs, errs


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["source"] for c in CASES])
@pytest.mark.parametrize("split", [None, 1, 2])
def test_tagg_golden(prod, case, split):
    errs = qtt.compare_agg(case, qtt.run_tagg_case(prod, case, split))
    assert not errs, errs


def _changelog(rng, n, nsrc, ngroups, utf8_src, utf8_group):
    pk = rng.integers(0, nsrc, n)
    grp = rng.integers(0, ngroups, n)
    gvalid = rng.random(n) > 0.05
    rvalid = rng.random(n) > 0.12  # tombstones
    ts = rng.integers(0, 10**6, n)
    ts[rng.random(n) < 0.01] = -1
    pkv = rng.random(n) > 0.01
    c0 = rng.integers(-2**31, 2**31, n).astype(np.int32)  # INT: sums wrap
    c1 = rng.integers(-10**15, 10**15, n)
    c2 = rng.uniform(-100, 100, n)
    cv = [rng.random(n) > 0.07 for _ in range(3)]
    # (digit keys take inline ids, the others the dictionary: khip_dict.hpp)
    ka = {"utf8_keys": ["%d" % g if g % 2 else "g%d" % g for g in grp]} if utf8_group else {"keys": grp}
    b = abi.HostBatch(ts, key_valid=gvalid, row_valid=rvalid, cols=[c0, c1, c2], col_valid=cv, **ka)
    sa = {"src_utf8_keys": [("%d" % k if k % 3 == 0 else "pk-%d" % k) if v else None for k, v in zip(pk, pkv)]} \
        if utf8_src else {"src_keys": pk, "src_key_valid": pkv}
    return b, sa, np.abs(c2)


AGGS = [("COUNT_STAR", -1), ("COUNT", 0), ("SUM", 0), ("SUM", 1), ("SUM", 2), ("AVG", 2), ("AVG", 1), ("COUNT", 2)]


def _run(lib, batches, utf8_group, having=None):
    desc = abi.make_agg_desc("NONE", "UTF8" if utf8_group else "INT64", col_types=["INT32", "INT64", "DOUBLE"],
                             aggs=AGGS, flags=abi.FLAG_TABLE_SOURCE)
    h = abi.AggHandle(lib, desc)
    stats = [h.push_table(b, **sa) for b, sa, _ in batches]
    snap = h.snapshot(having)
    h.close()
    return snap, stats


def _assert_same(g, o, scale):
    assert g["n"] == o["n"]
    assert list(g["key"]) == list(o["key"])
    assert np.array_equal(g["rowtime"], o["rowtime"])
    for a, (kind, col) in enumerate(AGGS):
        assert np.array_equal(g["nulls"][a], o["nulls"][a]), a
        if col == 2 and kind in ("SUM", "AVG"):
            np.testing.assert_allclose(g["values"][a], o["values"][a], rtol=0, atol=1e-12 * scale)
        elif kind == "AVG":  # AVG(BIGINT): (double)sum / count of exact integers
            np.testing.assert_allclose(g["values"][a], o["values"][a], rtol=1e-15)
        else:
            assert np.array_equal(g["values"][a], o["values"][a]), (kind, col)


@pytest.mark.gpu
@pytest.mark.parametrize("utf8_src,utf8_group", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("pushes", [1, 5])
def test_tagg_random_vs_oracle(prod, orc, utf8_src, utf8_group, pushes):
    rng = np.random.default_rng(100 + 10 * pushes + 2 * utf8_src + utf8_group)
    batches = [_changelog(rng, int(rng.integers(20000, 60000)), 8000, 300, utf8_src, utf8_group)
               for _ in range(pushes)]
    scale = sum(float(x.sum()) for _, _, x in batches) * 4  # every row can be added and undone twice
    (g, gs), (o, os_) = (_run(lib, batches, utf8_group) for lib in (prod, orc))
    for a, b in zip(gs, os_):
        for f in ("rows_in", "rows_accepted", "dropped_null_key", "dropped_bad_ts", "windows_applied", "stream_time"):
            assert a[f] == b[f], f
    _assert_same(g, o, scale)
    having = {"agg": 0, "op": "GT", "value": 0}  # HAVING COUNT(*) > 0: emptied groups disappear
    (g, _), (o, _) = (_run(lib, batches, utf8_group, having) for lib in (prod, orc))
    assert 0 < o["n"] <= 300
    _assert_same(g, o, scale)


@pytest.mark.gpu
def test_tagg_many_updates_per_key(prod, orc):
    """A handful of PRIMARY KEYs updated thousands of times inside one push: one device thread
    replays each key's rows in arrival order."""
    rng = np.random.default_rng(9)
    batches = [_changelog(rng, 50000, 7, 20, False, False) for _ in range(2)]
    scale = sum(float(x.sum()) for _, _, x in batches) * 4
    (g, _), (o, _) = (_run(lib, batches, False) for lib in (prod, orc))
    _assert_same(g, o, scale)


@pytest.mark.gpu
def test_tagg_reset_and_errors(prod, orc):
    rng = np.random.default_rng(3)
    b, sa, _ = _changelog(rng, 5000, 500, 50, False, False)
    desc = abi.make_agg_desc("NONE", "INT64", col_types=["INT32", "INT64", "DOUBLE"], aggs=AGGS,
                             flags=abi.FLAG_TABLE_SOURCE)
    h = abi.AggHandle(prod, desc)
    h.push_table(b, **sa)
    first = h.snapshot()
    with pytest.raises(abi.KsqlHipError):
        h.push(b)  # a table-source handle takes source-table changes only
    prod.check(prod.agg_reset(h.h), "agg_reset")
    assert h.snapshot()["n"] == 0
    h.push_table(b, **sa)
    again = h.snapshot()
    assert again["n"] == first["n"] and np.array_equal(again["values"][0], first["values"][0])
    h.close()
    for lib in (prod, orc):  # MIN/MAX are not undoable: rejected like the reference's KsqlException
        bad = abi.make_agg_desc("NONE", "INT64", col_types=["INT64"], aggs=[("MIN", 0)], flags=abi.FLAG_TABLE_SOURCE)
        with pytest.raises(abi.KsqlHipError):
            abi.AggHandle(lib, bad)


@pytest.mark.gpu
def test_tagg_key_range_edges(prod, orc):
    """The PRIMARY KEY sort runs over id − kmin on the bits of the push's key range: keys at both
    ends of BIGINT (the full 64-bit range: no sentinel for dropped rows), a push with every row
    dropped, negative keys, one key updated across pushes."""
    lo, hi = np.iinfo(np.int64).min, np.iinfo(np.int64).max

    def batch(pk, grp, ts, pkv=None, rv=None):
        m = len(pk)
        b = abi.HostBatch(np.asarray(ts, np.int64), keys=np.asarray(grp, np.int64),
                          row_valid=rv if rv is not None else [True] * m,
                          cols=[np.arange(m, dtype=np.int32), np.arange(m, dtype=np.int64) * 7, np.linspace(0, 1, m)])
        return b, {"src_keys": np.asarray(pk, np.int64), "src_key_valid": pkv}, np.ones(m)

    batches = [
        batch([lo, hi, 0, lo, -5, hi], [1, 2, 3, 2, 1, 1], [1, 2, 3, 4, 5, 6]),
        batch([1, 2, 3], [1, 1, 1], [7, 8, 9], pkv=[False, False, False]),
        batch([-5, -6, -5, -7], [4, 4, 5, 4], [10, -1, 12, 13], rv=[True, True, False, True]),
        batch([hi, hi, lo], [3, 1, 1], [14, 15, 16], pkv=[True, False, True]),
    ]
    (g, gs), (o, os_) = (_run(lib, batches, False) for lib in (prod, orc))
    for a, b in zip(gs, os_):
        for f in ("rows_in", "rows_accepted", "dropped_null_key", "dropped_bad_ts", "windows_applied", "stream_time"):
            assert a[f] == b[f], f
    _assert_same(g, o, 100.0)


@pytest.mark.gpu
def test_tagg_group_capacity_growth(prod, orc):
    """The group table grows ahead of a push by min(rows, span of the push's GROUP BY keys) new
    groups (8 slots per group): pushes whose groups are mostly new — a narrow span with many rows,
    a wide random span, distinct dense keys with both BIGINT extremes — from a tiny initial table."""
    rng = np.random.default_rng(11)
    lo, hi = np.iinfo(np.int64).min, np.iinfo(np.int64).max
    batches = []
    for p in range(12):
        m = 3000
        if p % 3 == 0:
            grp = 100_000 * p + rng.integers(0, 500, m)
        elif p % 3 == 1:
            grp = rng.integers(lo, hi, m)
        else:
            grp = np.concatenate([[lo, hi], 1_000_000 * p + np.arange(m - 2)])
        c2 = rng.normal(size=m)
        b = abi.HostBatch(np.arange(m, dtype=np.int64) + p * m, keys=np.asarray(grp, np.int64),
                          row_valid=rng.random(m) > 0.05,
                          cols=[rng.integers(-9, 9, m).astype(np.int32), rng.integers(-9, 9, m), c2])
        batches.append((b, {"src_keys": rng.integers(0, 5000, m)}, np.abs(c2)))
    scale = sum(float(x.sum()) for _, _, x in batches) * 4
    (g, _), (o, _) = (_run(lib, batches, False) for lib in (prod, orc))
    assert o["n"] > 10_000
    _assert_same(g, o, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("ncols", [0, 1, 2])
@pytest.mark.parametrize("utf8_src", [False, True])
def test_tagg_narrow_rows_vs_oracle(prod, orc, ncols, utf8_src):
    """Narrow handles (0-2 argument columns, INT and DOUBLE; each column count is its own replay
    kernel instantiation) against the oracle, BIGINT and STRING PRIMARY KEYs."""
    rng = np.random.default_rng(500 + 10 * ncols + utf8_src)
    types = ["INT32", "DOUBLE"][:ncols]
    aggs = [("COUNT_STAR", -1)] + [a for c in range(ncols) for a in (("SUM", c), ("COUNT", c), ("AVG", c))]
    batches, scale = [], 0.0
    for _ in range(4):
        n = int(rng.integers(20000, 50000))
        pk = rng.integers(0, 6000, n)
        grp = rng.integers(0, 200, n)
        ts = rng.integers(0, 10**6, n)
        ts[rng.random(n) < 0.01] = -1
        cols = [rng.integers(-2**31, 2**31, n).astype(np.int32), rng.uniform(-100, 100, n)][:ncols]
        cv = [rng.random(n) > 0.07 for _ in range(ncols)]
        b = abi.HostBatch(ts, keys=grp, key_valid=rng.random(n) > 0.05, row_valid=rng.random(n) > 0.12, cols=cols,
                          col_valid=cv)
        pkv = rng.random(n) > 0.01
        sa = {"src_utf8_keys": ["pk-%d" % k if v else None for k, v in zip(pk, pkv)]} if utf8_src else \
            {"src_keys": pk, "src_key_valid": pkv}
        batches.append((b, sa))
        if ncols == 2:
            scale += float(np.abs(cols[1]).sum()) * 4
    res = []
    for lib in (prod, orc):
        h = abi.AggHandle(lib, abi.make_agg_desc("NONE", "INT64", col_types=types, aggs=aggs, flags=abi.FLAG_TABLE_SOURCE))
        st = [h.push_table(b, **sa) for b, sa in batches]
        res.append((h.snapshot(), st))
        h.close()
    (g, gs), (o, os_) = res
    for a, b in zip(gs, os_):
        for f in ("rows_in", "rows_accepted", "dropped_null_key", "dropped_bad_ts", "windows_applied", "stream_time"):
            assert a[f] == b[f], f
    assert g["n"] == o["n"] and list(g["key"]) == list(o["key"])
    assert np.array_equal(g["rowtime"], o["rowtime"])
    for a, (kind, col) in enumerate(aggs):
        assert np.array_equal(g["nulls"][a], o["nulls"][a]), a
        if col >= 0 and types[col] == "DOUBLE" and kind in ("SUM", "AVG"):
            np.testing.assert_allclose(g["values"][a], o["values"][a], rtol=0, atol=1e-12 * scale)
        elif kind == "AVG":
            np.testing.assert_allclose(g["values"][a], o["values"][a], rtol=1e-15)
        else:
            assert np.array_equal(g["values"][a], o["values"][a]), (kind, col)


@pytest.mark.gpu
def test_tagg_source_layout_transitions(prod, orc):
    """The source table's dense layout (slot = id − base) grows its window when a push's ids fall
    below or above it, and moves to the hash layout when the ids spread past the dense bound; keys
    updated and deleted before each move must be found after it."""
    rng = np.random.default_rng(21)
    ranges = [(1000, 2000), (500, 3000), (400, 2600), None, (0, 3000), (2**40, 2**40 + 50)]
    batches = []
    for p, r in enumerate(ranges):
        n = 20000
        if r is None:  # far ids mixed with old ones: the dense window would be too large
            pk = np.where(rng.random(n) < 0.3, rng.integers(10**12, 10**12 + 10**6, n), rng.integers(400, 3000, n))
        else:
            pk = rng.integers(r[0], r[1], n)
        b, sa, x = _changelog(rng, n, 1, 300, False, False)
        sa = {"src_keys": pk, "src_key_valid": sa["src_key_valid"]}
        batches.append((b, sa, x))
    scale = sum(float(x.sum()) for _, _, x in batches) * 4
    (g, gs), (o, os_) = (_run(lib, batches, False) for lib in (prod, orc))
    for a, b in zip(gs, os_):
        for f in ("rows_in", "rows_accepted", "dropped_null_key", "dropped_bad_ts", "windows_applied", "stream_time"):
            assert a[f] == b[f], f
    _assert_same(g, o, scale)


@pytest.mark.gpu
def test_tagg_hash_layout_tuning_build():
    """KHIP_TAGG_DENSE=0 on the tuning build: the hash layout for every source table (the layout
    sparse and STRING PRIMARY KEYs take) on the dense-id workloads, against the oracle."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, KSQL_AMD_LIB_VARIANT="tune", KHIP_TAGG_DENSE="0",
               PYTHONPATH=os.pathsep.join([repo, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def _child():
    prod, orc = abi.load_product(), abi.load_oracle()
    assert prod.path.endswith("libksqldb_hip_tune.so"), prod.path
    for utf8_group in (False, True):
        test_tagg_random_vs_oracle(prod, orc, False, utf8_group, 5)
    test_tagg_many_updates_per_key(prod, orc)
    test_tagg_group_capacity_growth(prod, orc)
    print("OK")


if __name__ == "__main__" and "--child" in sys.argv:
    _child()
