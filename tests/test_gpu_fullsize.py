"""Full-size parity of every path bench.py times, through the C ABI, against the oracle.

Each test runs the bench leg's own configuration (same generator, descriptor, capacity hint
and micro-batch structure) and compares the HIP result with the CPU restatement on the same
records — the key-sharded P-thread oracle (oracle_agg_push_sharded), itself pinned bit for bit
to the sequential oracle in test_oracle_sharded.py:

  C2 possible_fraud   100M records / 10M BIGINT card numbers, TUMBLING 5 s COUNT(*), HAVING > 3:
                      the full table, the stats and the HAVING row count (the numbers the bench
                      line prints: 22,054,808 groups, 14,333,273 HAVING rows)
  C2 --utf8           the same with 16-byte VARCHAR card numbers through the device dictionary
  C1 hourly_metrics   1M page views, VARCHAR url keys, TUMBLING 1 HOUR COUNT(*)
  C3 hopping_double   5e7 records pushed as 8 event-time micro-batches (closed windows are
                      evicted between pushes), HOPPING 60 s / 10 s GRACE 60 s SUM/AVG/MIN/MAX
  C4 clickstream      khip_table_probe_device (the C4 bench kernel): emit / matched / null
                      bitmaps, the gathered column and n_emitted, 1e7-row table, 1e8 + 37 probes
  C5 repartition_sum  2^24 records over 8 simulated source tasks: pack → all-to-all (emulated)
                      → unpack → SUM(amount) TUMBLING 1 MINUTE per destination task

Integers, keys, windows, row times and DOUBLE MIN/MAX are bit-exact; DOUBLE SUM/AVG (inputs are
non-negative here) within the north star's 1e-12 relative tolerance.
"""
import os
import sys
import threading

import numpy as np
import pytest
import torch

from ksql_amd import abi, synth
from test_gpu_parity import assert_snap_equal

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


@pytest.fixture
def say(capsys):
    def _say(msg):
        with capsys.disabled():
            sys.stderr.write("  [fullsize] %s\n" % msg)
            sys.stderr.flush()
    return _say


# ------------------------------------------------------------------------ C2

C2_DESC = dict(window_kind="TUMBLING", size_ms=5000, aggs=[("COUNT_STAR", -1)])
C2_HAVING = {"agg": 0, "op": "GT", "value": 3}
C2_N, C2_KEYS = 100_000_000, 10_000_000


SPARSE_MULT = 0x5DEECE66D  # bench.py --sparse-keys: id -> (id * SPARSE_MULT) mod 2^53, a bijection


def _c2_oracle(orc, key_type, say, sparse=False):
    card, ts = synth.possible_fraud(0, C2_N, C2_N, keys=C2_KEYS)
    if sparse:
        card = (card * SPARSE_MULT) & ((1 << 53) - 1)
    o = abi.ShardedOracleAgg(orc, abi.make_agg_desc(key_type=key_type, **C2_DESC), THREADS)
    if key_type == "UTF8":
        offs, kb = synth.card_utf8(card)
        b = abi.HostBatch(ts, key_offsets=offs, key_bytes=kb)
    else:
        b = abi.HostBatch(ts, keys=card)
    st = o.push(b)
    say("C2 %s oracle pushed (%d threads)" % (key_type, THREADS))
    exp = o.snapshot(raw_keys=True)
    o.close()
    return st, exp


@pytest.mark.timeout(900)
def test_c2_possible_fraud_full(prod, orc, say):
    card, ts = synth.possible_fraud(0, C2_N, C2_N, xp="torch", device="cuda", keys=C2_KEYS)
    # bench.py: capacity_hint = min(3 * keys, 2 * n) → 2^14 partitions, two-level scatter
    desc = abi.make_agg_desc(key_type="INT64", capacity_hint=min(3 * C2_KEYS, 2 * C2_N), **C2_DESC)
    h = abi.AggHandle(prod, desc)
    st = h.push(abi.DeviceBatch(ts, keys=card))
    n_having = h.count_rows(C2_HAVING)
    got = h.snapshot()
    h.close()
    del card, ts
    say("C2 product: %d groups, %d HAVING rows" % (got["n"], n_having))
    ost, exp = _c2_oracle(orc, "INT64", say)
    assert st == ost
    assert st["rows_accepted"] == st["windows_applied"] == C2_N
    assert_snap_equal(got, exp, desc)
    assert n_having == int((exp["values"][0] > 3).sum())
    # the counts the round-1 bench line printed are the oracle's
    assert (exp["n"], n_having) == (22_054_808, 14_333_273)


@pytest.mark.timeout(900)
def test_c2_possible_fraud_sparse_full(prod, orc, say):
    """bench.py --sparse-keys: the same records with the card ids spread over 2^53 (the COUNT(*)
    pipeline's wide records: 64-bit key hashes)."""
    card, ts = synth.possible_fraud(0, C2_N, C2_N, xp="torch", device="cuda", keys=C2_KEYS)
    card = (card * SPARSE_MULT) & ((1 << 53) - 1)
    desc = abi.make_agg_desc(key_type="INT64", capacity_hint=min(3 * C2_KEYS, 2 * C2_N), flags=abi.FLAG_PROFILE,
                             **C2_DESC)
    h = abi.AggHandle(prod, desc)
    st = h.push(abi.DeviceBatch(ts, keys=card))
    n_having = h.count_rows(C2_HAVING)
    got = h.snapshot()
    kt = h.kernel_times()
    h.close()
    del card, ts
    say("C2 sparse product: %d groups, %d HAVING rows" % (got["n"], n_having))
    ost, exp = _c2_oracle(orc, "INT64", say, sparse=True)
    assert st == ost
    assert_snap_equal(got, exp, desc)
    assert n_having == int((exp["values"][0] > 3).sum())
    assert (exp["n"], n_having) == (22_054_808, 14_333_273)  # a bijection of the keys: the same table shape
    assert kt["c1_pushes"] == 1, kt


@pytest.mark.timeout(900)
def test_c2_possible_fraud_utf8_full(prod, orc, say):
    card, ts = synth.possible_fraud(0, C2_N, C2_N, xp="torch", device="cuda", keys=C2_KEYS)
    offs, kb = synth.card_utf8(card, xp="torch")
    del card
    desc = abi.make_agg_desc(key_type="UTF8", capacity_hint=min(3 * C2_KEYS, 2 * C2_N), **C2_DESC)
    h = abi.AggHandle(prod, desc)
    st = h.push(abi.DeviceBatch(ts, key_offsets=offs, key_bytes=kb))
    n_having = h.count_rows(C2_HAVING)
    got = h.snapshot(raw_keys=True)
    h.close()
    del offs, kb, ts
    say("C2 utf8 product: %d groups" % got["n"])
    ost, exp = _c2_oracle(orc, "UTF8", say)
    assert st == ost
    assert got["n"] == exp["n"]
    assert np.array_equal(got["key_offsets"], exp["key_offsets"])
    assert np.array_equal(got["key_bytes"], exp["key_bytes"])
    for f in ("ws", "we", "rowtime"):
        assert np.array_equal(got[f], exp[f]), f
    assert np.array_equal(got["values"][0], exp["values"][0])
    assert n_having == int((exp["values"][0] > 3).sum())


# ------------------------------------------------------------------------ C1

def test_c1_hourly_metrics_full(prod, orc):
    n = synth.CONFIGS["hourly_metrics"]["n"]
    offs, kb, ts = synth.hourly_metrics_utf8(0, n, n)
    kw = dict(window_kind="TUMBLING", size_ms=3_600_000, key_type="UTF8", aggs=[("COUNT_STAR", -1)])
    h = abi.AggHandle(prod, abi.make_agg_desc(**kw, capacity_hint=40_000))
    dev = lambda a: torch.from_numpy(a).cuda()
    st = h.push(abi.DeviceBatch(dev(ts), key_offsets=dev(offs), key_bytes=dev(kb)))
    got = h.snapshot()
    h.close()
    urls, ts2 = synth.hourly_metrics(0, n, n)
    o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
    ost = o.push(abi.HostBatch(ts2, utf8_keys=urls))
    exp = o.snapshot()
    o.close()
    assert st == ost
    assert got["n"] == exp["n"] == 30_000  # 10,000 urls x 3 hour windows (10,000 s of page views)
    assert got["key"] == exp["key"]
    for f in ("ws", "we", "rowtime"):
        assert np.array_equal(got[f], exp[f]), f
    assert np.array_equal(got["values"][0], exp["values"][0])


# ------------------------------------------------------------------------ C3

@pytest.mark.timeout(900)
def test_c3_hopping_double_microbatches(prod, orc, say):
    n = 50_000_000
    S = n // 8  # eight event-time micro-batches: windows close and are evicted between pushes
    cfg = synth.CONFIGS["hopping_double"]
    kw = dict(window_kind="HOPPING", size_ms=cfg["size_ms"], advance_ms=cfg["advance_ms"], grace_ms=cfg["grace_ms"],
              key_type="INT64", col_types=["DOUBLE"], aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0)])
    key, ts, val, valid = synth.hopping_double(0, n, n, xp="torch", device="cuda")
    vb = abi.bitmap_torch(valid)
    del valid
    span_push = cfg["span_ms"] * S / n  # bench.py's live-group hint
    live = int(cfg["keys"] * (span_push + cfg["size_ms"] + cfg["grace_ms"] + cfg["disorder_ms"]) / cfg["advance_ms"])
    desc = abi.make_agg_desc(**kw, capacity_hint=live)
    h = abi.AggHandle(prod, desc)
    stats = [h.push(abi.DeviceBatch(ts[lo:lo + S], keys=key[lo:lo + S], cols=[val[lo:lo + S]],
                                    col_valid=[vb[lo // 8:(lo + S) // 8]])) for lo in range(0, n, S)]
    got = h.snapshot()
    h.close()
    del key, ts, val, vb
    say("C3 product: %d groups over %d pushes" % (got["n"], len(stats)))
    keyh, tsh, valh, validh = synth.hopping_double(0, n, n)
    o = abi.ShardedOracleAgg(orc, abi.make_agg_desc(**kw), THREADS)
    ostats = [o.push(abi.HostBatch(tsh[lo:lo + S], keys=keyh[lo:lo + S], cols=[valh[lo:lo + S]],
                                   col_valid=[validh[lo:lo + S]])) for lo in range(0, n, S)]
    exp = o.snapshot()
    o.close()
    assert stats == ostats
    assert sum(s["rows_accepted"] for s in stats) == n
    assert_snap_equal(got, exp, desc)


@pytest.mark.timeout(1100)
def test_c3_bench_push_size(prod, orc, say):
    """The timed configuration itself: bench.py's hopping_double pushes (2^27-record event-time
    micro-batches of the 1e9-record workload, its capacity hint), two of them — the first two pushes
    of a bench step, bit-exact integer state and DOUBLE within tolerance against the oracle."""
    n_total = 1_000_000_000
    S = 1 << 27
    m = 2 * S
    cfg = synth.CONFIGS["hopping_double"]
    kw = dict(window_kind="HOPPING", size_ms=cfg["size_ms"], advance_ms=cfg["advance_ms"], grace_ms=cfg["grace_ms"],
              key_type="INT64", col_types=["DOUBLE"], aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0)])
    key, ts, val, valid = synth.hopping_double(0, m, n_total, xp="torch", device="cuda")
    vb = abi.bitmap_torch(valid)
    del valid
    span_push = cfg["span_ms"] * S / n_total  # bench.py:bench_hopping_double's live-group hint
    live = int(cfg["keys"] * (span_push + cfg["size_ms"] + cfg["grace_ms"] + cfg["disorder_ms"]) / cfg["advance_ms"])
    desc = abi.make_agg_desc(**kw, capacity_hint=live)
    h = abi.AggHandle(prod, desc)
    stats = [h.push(abi.DeviceBatch(ts[lo:lo + S], keys=key[lo:lo + S], cols=[val[lo:lo + S]],
                                    col_valid=[vb[lo // 8:(lo + S) // 8]])) for lo in range(0, m, S)]
    got = h.snapshot()
    h.close()
    del key, ts, val, vb
    say("C3 at the bench's push size: %d groups after %d pushes of %d records" % (got["n"], len(stats), S))
    keyh, tsh, valh, validh = synth.hopping_double(0, m, n_total)
    o = abi.ShardedOracleAgg(orc, abi.make_agg_desc(**kw), THREADS)
    ostats = [o.push(abi.HostBatch(tsh[lo:lo + S], keys=keyh[lo:lo + S], cols=[valh[lo:lo + S]],
                                   col_valid=[validh[lo:lo + S]])) for lo in range(0, m, S)]
    del keyh, tsh, valh, validh
    exp = o.snapshot()
    o.close()
    assert stats == ostats
    assert sum(s["rows_accepted"] for s in stats) == m
    assert_snap_equal(got, exp, desc)


@pytest.mark.timeout(900)
def test_c3_signed_cancellation(prod, orc, say):
    """DOUBLE SUM / AVG under cancellation.  C3's query shape (HOPPING 60 s /
    10 s, grace 60 s, SUM/AVG/MIN/MAX of a DOUBLE, eight event-time micro-batches) with SIGNED
    values U[-1000, 1000) and 1e4 keys (~33 records per window), against the oracle's sequential
    `aggregateValue + valueToAdd` (DoubleSumKudaf.java:26-31) per (key, window).
    The device adds a window's records in LDS-atomic order, panes first, so the two sums round
    differently.  Any order of n additions is within (n-1)·eps·Σ|x| of the exact sum; so
      - every group: |device - reference| <= 1e-12 · Σ|x|  (asserted);
      - plain relative 1e-12 wherever Σ|x| <= 50·|sum| (condition number <= 50: the bound above,
        with n <= 60 records a window, is below 1e-12·|sum|)  (asserted);
      - below that (near-total cancellation) no reordered summation meets a plain relative bound —
        the reference's own sequential sum is off from the exact one by more — the worst observed
        plain relative error and the share of groups past 1e-12 are reported (bench.py's C3 line
        quotes them)."""
    n = 40_000_000
    S = n // 8
    cfg = synth.CONFIGS["hopping_double"]
    win = dict(window_kind="HOPPING", size_ms=cfg["size_ms"], advance_ms=cfg["advance_ms"], grace_ms=cfg["grace_ms"],
               key_type="INT64")
    kw = dict(win, col_types=["DOUBLE"], aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0)])
    # the error bound's Σ|x| and n per group: a second oracle query over |x| (the same groups)
    kabs = dict(win, col_types=["DOUBLE"], aggs=[("SUM", 0), ("COUNT", 0)])
    keyh, tsh, valh, validh = synth.hopping_double(0, n, n, keys=10_000)
    valh = valh * 2.0 - 1000.0  # U[-1000, 1000)
    absh = np.abs(valh)
    desc = abi.make_agg_desc(**kw, capacity_hint=4_000_000, flags=abi.FLAG_PROFILE)  # >= 2^11 partitions: the pipeline
    h = abi.AggHandle(prod, desc)
    o = abi.ShardedOracleAgg(orc, abi.make_agg_desc(**kw), THREADS)
    oa = abi.ShardedOracleAgg(orc, abi.make_agg_desc(**kabs), THREADS)
    for lo in range(0, n, S):
        b = abi.HostBatch(tsh[lo:lo + S], keys=keyh[lo:lo + S], cols=[valh[lo:lo + S]], col_valid=[validh[lo:lo + S]])
        assert h.push(b) == o.push(b)
        oa.push(abi.HostBatch(tsh[lo:lo + S], keys=keyh[lo:lo + S], cols=[absh[lo:lo + S]],
                              col_valid=[validh[lo:lo + S]]))
    assert h.kernel_times()["c1_pushes"] == 8  # the value pipeline (C3's), not the general engine
    got, exp, ab = h.snapshot(), o.snapshot(), oa.snapshot()
    h.close()
    o.close()
    oa.close()
    assert np.array_equal(ab["key"], exp["key"]) and np.array_equal(ab["ws"], exp["ws"])
    for d in (got, exp):  # compare through assert_snap_equal's Σ|x| bound: append SUM(|x|), COUNT(x)
        d["values"] = list(d["values"]) + list(ab["values"])
        d["nulls"] = list(d["nulls"]) + list(ab["nulls"])
    d6 = abi.make_agg_desc(**win, col_types=["DOUBLE", "DOUBLE"],
                           aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0), ("SUM", 1), ("COUNT", 1)])
    assert_snap_equal(got, exp, d6, abs_sum_agg=4, count_agg=5)
    g, r, sabs = got["values"][0], exp["values"][0], exp["values"][4]
    ok = ~exp["nulls"][0]
    g, r, sabs = g[ok], r[ok], sabs[ok]
    rel = np.abs(g - r) / np.maximum(np.abs(r), 1e-300)
    cond = sabs / np.maximum(np.abs(r), 1e-300)
    well = cond <= 50
    assert well.sum() > 0.8 * len(r)
    assert rel[well].max() <= 1e-12, rel[well].max()
    bad = rel > 1e-12
    say("C3 signed SUM: %d groups; plain relative error max %.3g (median %.3g); %d groups (%.4f%%) past 1e-12, "
        "all at condition number > 50 (min %.3g); max over cond <= 50: %.3g"
        % (len(r), rel.max(), np.median(rel), bad.sum(), 100.0 * bad.mean(), cond[bad].min() if bad.any() else 0,
           rel[well].max()))


@pytest.mark.timeout(900)
def test_c3_changelog_per_push(prod, orc, say):
    """C3's micro-batch structure with EMIT CHANGES kept (KHIP_FLAG_CHANGELOG): the rows every
    push emits equal the oracle's, push by push (the changelog a downstream topic receives)."""
    n = 50_000_000
    S = n // 8
    cfg = synth.CONFIGS["hopping_double"]
    kw = dict(window_kind="HOPPING", size_ms=cfg["size_ms"], advance_ms=cfg["advance_ms"], grace_ms=cfg["grace_ms"],
              key_type="INT64", col_types=["DOUBLE"], aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0)],
              having={"agg": 1, "op": "GT", "value": 500.0})
    key, ts, val, valid = synth.hopping_double(0, n, n, xp="torch", device="cuda")
    vb = abi.bitmap_torch(valid)
    del valid
    span_push = cfg["span_ms"] * S / n
    live = int(cfg["keys"] * (span_push + cfg["size_ms"] + cfg["grace_ms"] + cfg["disorder_ms"]) / cfg["advance_ms"])
    desc = abi.make_agg_desc(**kw, capacity_hint=live, flags=abi.FLAG_CHANGELOG)
    keyh, tsh, valh, validh = synth.hopping_double(0, n, n)
    h = abi.AggHandle(prod, desc)
    o = abi.ShardedOracleAgg(orc, abi.make_agg_desc(**kw), THREADS)
    total = tombs = 0
    for lo in range(0, n, S):
        st = h.push(abi.DeviceBatch(ts[lo:lo + S], keys=key[lo:lo + S], cols=[val[lo:lo + S]],
                                    col_valid=[vb[lo // 8:(lo + S) // 8]]))
        ost = o.push(abi.HostBatch(tsh[lo:lo + S], keys=keyh[lo:lo + S], cols=[valh[lo:lo + S]],
                                   col_valid=[validh[lo:lo + S]]))
        assert st == ost
        gc, oc = h.changes(), o.changes()
        assert_snap_equal(gc, oc, desc)
        assert np.array_equal(gc["tombstone"], oc["tombstone"])
        total += gc["n"]
        tombs += int(gc["tombstone"].sum())
    say("C3 changelog: %d rows emitted over 8 pushes (%d tombstones)" % (total, tombs))
    assert total > 0 and tombs > 0
    h.close()
    o.close()


# ------------------------------------------------------------------------ C4

def _probe_oracle(orc_table, keys, ts, kv, rv, join_type, where, threads=THREADS):
    """oracle_table_probe over `threads` chunks of the stream (the table is read-only while
    probing, and ctypes releases the GIL): emitted rows (global index), matched, cols, nulls."""
    n = len(ts)
    bounds = np.linspace(0, n, threads + 1).astype(np.int64)
    res = [None] * threads

    def run(k):
        lo, hi = int(bounds[k]), int(bounds[k + 1])
        b = abi.HostBatch(ts[lo:hi], keys=keys[lo:hi], key_valid=None if kv is None else kv[lo:hi],
                          row_valid=None if rv is None else rv[lo:hi])
        r = orc_table.probe(b, join_type, where)
        r["stream_row"] = r["stream_row"] + lo
        res[k] = r

    th = [threading.Thread(target=run, args=(k,)) for k in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    out = {"stream_row": np.concatenate([r["stream_row"] for r in res]),
           "matched": np.concatenate([r["matched"] for r in res]),
           "cols": [np.concatenate([r["cols"][c] for r in res]) for c in range(len(res[0]["cols"]))],
           "nulls": [np.concatenate([r["nulls"][c] for r in res]) for c in range(len(res[0]["nulls"]))]}
    return out


def _bits(mask_bool):
    return np.packbits(mask_bool, bitorder="little")


def _check_probe_device(prod_table, orc_table, keys, ts, kv, rv, join_type, where, col_types):
    """khip_table_probe_device vs the oracle: row-aligned bitmaps and gathered columns."""
    n = len(ts)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    dkv = None if kv is None else abi.bitmap_torch(dev(kv))
    drv = None if rv is None else abi.bitmap_torch(dev(rv))
    batch = abi.DeviceBatch(dev(ts), keys=dev(keys), key_valid=dkv, row_valid=drv)
    nb = (n + 7) // 8
    emit = torch.full((nb + 8,), 0xAB, dtype=torch.uint8, device="cuda")  # guard bytes past the batch
    matched = torch.full((nb + 8,), 0xAB, dtype=torch.uint8, device="cuda")
    tdt = {"INT32": torch.int32, "INT64": torch.int64, "DOUBLE": torch.float64}
    cols = [torch.zeros(n, dtype=tdt[t], device="cuda") for t in col_types]
    nulls = [torch.full((nb + 8,), 0xAB, dtype=torch.uint8, device="cuda") for _ in col_types]
    n_emit = prod_table.probe_device(batch, join_type, where, emit, matched, cols, nulls)
    torch.cuda.synchronize()
    exp = _probe_oracle(orc_table, keys, ts, kv, rv, join_type, where)
    hit_all = _probe_oracle(orc_table, keys, ts, kv, rv, "LEFT", None)  # every accepted row: table hit?
    e = np.zeros(n, bool)
    e[exp["stream_row"]] = True
    hit = np.zeros(n, bool)
    hit[hit_all["stream_row"]] = hit_all["matched"]
    assert n_emit == len(exp["stream_row"])
    em, mt = emit.cpu().numpy(), matched.cpu().numpy()
    assert np.array_equal(em[:nb], _bits(e)), "emit bitmap"
    assert np.array_equal(mt[:nb], _bits(hit)), "matched bitmap"
    assert (em[nb:] == 0xAB).all() and (mt[nb:] == 0xAB).all(), "wrote past the batch"
    # right columns: null bit = no hit or NULL value; values where hit and non-null
    for c in range(len(col_types)):
        isnull = np.ones(n, bool)
        isnull[hit_all["stream_row"]] = hit_all["nulls"][c]
        nm = nulls[c].cpu().numpy()
        assert np.array_equal(nm[:nb], _bits(isnull)), "null bitmap of column %d" % c
        assert (nm[nb:] == 0xAB).all()
        val = np.zeros(n, hit_all["cols"][c].dtype)
        val[hit_all["stream_row"]] = hit_all["cols"][c]
        g = cols[c].cpu().numpy()
        sel = ~isnull
        assert np.array_equal(g[sel].view(np.int64) if g.dtype == np.float64 else g[sel],
                              val[sel].view(np.int64) if val.dtype == np.float64 else val[sel]), "column %d" % c


def _table_pair(prod, orc, col_types, batches, capacity_hint):
    tp = abi.TableHandle(prod, col_types, capacity_hint=capacity_hint)
    to = abi.TableHandle(orc, col_types, capacity_hint=capacity_hint)
    for b in batches:
        tp.upsert(b)
        to.upsert(b)
    assert tp.size() == to.size()
    return tp, to


@pytest.mark.parametrize("join_type", ["LEFT", "INNER"])
@pytest.mark.parametrize("where", [None, {"col": 0, "op": "EQ", "i64": 2}, {"col": 1, "op": "GT", "f64": 0.5}])
def test_c4_probe_device_vs_oracle(prod, orc, join_type, where):
    """Table with deletes and NULL columns (several upsert batches, repeated keys), stream with
    null keys / values / negative timestamps and n not a multiple of 64 (tail bytes)."""
    rng = np.random.default_rng(4 + (where is None) + 10 * (join_type == "INNER"))
    U = 1_000_000
    batches = []
    for r in range(3):
        m = U if r == 0 else U // 4
        k = np.arange(1, U + 1) if r == 0 else rng.integers(1, U + 1, m)
        cols = [rng.integers(0, 3, m).astype(np.int32), rng.random(m)]
        batches.append(abi.HostBatch(np.zeros(m, np.int64), keys=k, row_valid=rng.random(m) > (0 if r == 0 else 0.2),
                                     cols=cols, col_valid=[rng.random(m) > 0.05, rng.random(m) > 0.05]))
    tp, to = _table_pair(prod, orc, ["INT32", "DOUBLE"], batches, U)
    n = 3_000_013
    keys = rng.integers(-5, int(U * 1.2), n)
    ts = np.arange(n, dtype=np.int64)
    ts[rng.random(n) < 0.01] = -1
    kv, rv = rng.random(n) > 0.01, rng.random(n) > 0.01
    _check_probe_device(tp, to, keys, ts, kv, rv, join_type, where, ["INT32", "DOUBLE"])
    tp.close()
    to.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("sparse", [False, True], ids=["dense-ids", "sparse-ids"])
def test_c4_clickstream_probe_device_full(prod, orc, say, sparse):
    """The bench's C4 step (LEFT JOIN users WHERE level = 'Platinum', one INT32 level column)
    on a 1e7-row users table and 1e8 + 37 clicks: user ids 1..U (the dense direct-map index) and
    spread over 2^40 (bench.py --sparse-ids: the hash-probe kernel)."""
    U, n = 10_000_000, 100_000_037
    uid, level = synth.users_table(0, U)
    if sparse:
        uid = synth.sparse_ids(uid)
    b = abi.HostBatch(np.zeros(U, np.int64), keys=uid, cols=[level.astype(np.int32)])
    tp, to = _table_pair(prod, orc, ["INT32"], [b], U)
    cu, cts = synth.clicks(0, n, U, seed_clicks=5)
    if sparse:
        cu = synth.sparse_ids(cu)
    where = {"col": 0, "op": "EQ", "i64": synth.LEVELS.index("Platinum")}
    say("C4 table built, probing %d clicks" % n)
    _check_probe_device(tp, to, cu, cts, None, None, "LEFT", where, ["INT32"])
    tp.close()
    to.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("sparse", [False, True], ids=["dense-ids", "sparse-ids"])
def test_c4_clickstream_full_table(prod, say, sparse):
    """BASELINE configs[3] at its stated size: the 1e8-row users table built on
    the device (synth.users_table, 2^28 slots of 16 B = 4 GB; a 100 MB dense index, or the hashed
    index for ids spread over 2^40) and the bench's 1e9 clicks probed in ONE khip_table_probe_device
    (8 GB of keys: byte offsets past 2^32).  Expected, computed exactly on the device from the
    generator (StreamTableJoinBuilder.java:38-88 LEFT join, KsqlValueJoiner.java:41-63, the WHERE
    level = 'Platinum' filter StreamFilterBuilder.java:44-69):
      matched  <=> the click's dense user id u <= U (ids 1..U are the table's keys),
      level    =  users_table level at u - 1 (never NULL),
      emit     <=> matched and level = Platinum;
    the emit / matched / null bitmaps, the gathered column and the emitted count bit for bit."""
    U, n = 100_000_000, 1_000_000_000
    uid, level = synth.users_table(0, U, xp="torch", device="cuda")
    level = level.to(torch.int32)
    keys = synth.sparse_ids(uid) if sparse else uid
    t = abi.TableHandle(prod, ["INT32"], capacity_hint=U)
    t.upsert(abi.DeviceBatch(torch.zeros(U, dtype=torch.int64, device="cuda"), keys=keys, cols=[level]))
    t.sync()
    del keys, uid
    assert t.size() == U
    say("C4 full table built (%d rows), probing %d clicks" % (U, n))
    cu, cts = synth.clicks(0, n, U, xp="torch", device="cuda", seed_clicks=5)  # the bench's clicks
    probe_keys = synth.sparse_ids(cu) if sparse else cu
    nb = (n + 7) // 8
    guard = lambda: torch.full((nb + 8,), 0xAB, dtype=torch.uint8, device="cuda")
    emit, matched, null = guard(), guard(), guard()
    col = torch.zeros(n, dtype=torch.int32, device="cuda")
    plat = synth.LEVELS.index("Platinum")
    n_emit = t.probe_device(abi.DeviceBatch(cts, keys=probe_keys), "LEFT", {"col": 0, "op": "EQ", "i64": plat},
                            emit, matched, [col], [null])
    torch.cuda.synchronize()
    del probe_keys, cts
    hit = cu <= U
    lev = level[(cu - 1).clamp_(max=U - 1)]
    del cu
    e = hit & (lev == plat)
    assert n_emit == int(e.sum()) > 0
    assert torch.equal(emit[:nb], abi.bitmap_torch(e)), "emit bitmap"
    assert torch.equal(matched[:nb], abi.bitmap_torch(hit)), "matched bitmap"
    assert torch.equal(null[:nb], abi.bitmap_torch(~hit)), "null bitmap (a hit's level is never NULL)"
    for g in (emit, matched, null):
        assert bool((g[nb:] == 0xAB).all()), "wrote past the batch"
    assert torch.equal(col[hit], lev[hit]), "gathered level column"
    say("C4 full: %d clicks, %d matched, %d emitted" % (n, int(hit.sum()), n_emit))
    t.close()


@pytest.mark.timeout(900)
def test_c4_full_table_vs_oracle(prod, orc, say):
    """The 1e8-row users table against the oracle's own table (ids 1..U, built from the same rows)
    with 1e8 + 37 clicks: the device probe vs oracle R-join rows bit for bit."""
    U, n = 100_000_000, 100_000_037
    uid, level = synth.users_table(0, U)
    b = abi.HostBatch(np.zeros(U, np.int64), keys=uid, cols=[level.astype(np.int32)])
    tp, to = _table_pair(prod, orc, ["INT32"], [b], U)
    del b, uid, level
    cu, cts = synth.clicks(0, n, U, seed_clicks=9)
    where = {"col": 0, "op": "EQ", "i64": synth.LEVELS.index("Platinum")}
    say("C4 oracle table built (%d rows), probing %d clicks" % (U, n))
    _check_probe_device(tp, to, cu, cts, None, None, "LEFT", where, ["INT32"])
    tp.close()
    to.close()


# ------------------------------------------------------------------------ C5

def _kafka_partition(orc, keys, n_parts):
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    out = np.zeros(len(keys), np.int32)
    orc.dll.oracle_kafka_partition(keys.ctypes.data, len(keys), 8, n_parts, out.ctypes.data)
    return out


@pytest.mark.timeout(900)
def test_c5_repartition_2p24(prod, orc, say):
    W, n_src = 8, (1 << 24) // 8
    kw = dict(window_kind="TUMBLING", size_ms=60_000, key_type="INT64", col_types=["INT64", "INT64"],
              aggs=[("SUM", 1)])
    srcs = [synth.repartition_sum(0, n_src, n_src, xp="torch", device="cuda", rank=r, world=W) for r in range(W)]
    sends = []
    for eid, ts, region, amount in srcs:
        sh = abi.ShuffleHandle(prod, W, 0, ["INT64", "INT64"])
        sends.append(sh.pack(abi.DeviceBatch(ts, cols=[region, amount])))
        sh.close()
    host = [tuple(t.cpu().numpy() for t in s) for s in srcs]
    dests = [_kafka_partition(orc, h_[2], W) for h_ in host]
    total = 0
    for d in range(W):
        parts = []
        for send, counts in sends:
            off = sum(counts[:d])
            parts.append(send[off:off + counts[d]])
        recv = torch.cat(parts)
        sh = abi.ShuffleHandle(prod, W, 0, ["INT64", "INT64"])
        key, ts, cols, valid = sh.unpack(recv, recv.shape[0])
        h = abi.AggHandle(prod, abi.make_agg_desc(**kw, capacity_hint=60 * 1_000_000 // W))
        st = h.push(abi.DeviceBatch(ts, keys=key, cols=cols, col_valid=valid))
        got = h.snapshot()
        h.close()
        sh.close()
        rk = np.concatenate([h_[2][dd == d] for h_, dd in zip(host, dests)])
        rts = np.concatenate([h_[1][dd == d] for h_, dd in zip(host, dests)])
        ra = np.concatenate([h_[3][dd == d] for h_, dd in zip(host, dests)])
        o = abi.AggHandle(orc, abi.make_agg_desc(**kw))
        ost = o.push(abi.HostBatch(rts, keys=rk, cols=[rk, ra]))
        exp = o.snapshot()
        o.close()
        assert st == ost
        assert_snap_equal(got, exp, abi.make_agg_desc(**kw))
        total += int(recv.shape[0])
    say("C5: %d rows routed to %d tasks" % (total, W))
    assert total == 1 << 24
