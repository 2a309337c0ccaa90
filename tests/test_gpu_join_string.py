"""STRING-keyed tables for the stream-table join (VARCHAR primary key, S/JoinParamsFactory.java:65-84:
both sides' key types match; identity = byte equality of the serialized KAFKA STRING key).

The HIP path maps key bytes to ids with the device key dictionary (insert on upsert, read-only
probe) and then runs the INT64 slot table; the oracle interns the bytes on the CPU
(oracle/oracle.c table_key).  No QTT stream-table case has STRING keys in the replayable shape
(tests/golden/make_fixtures.py), so parity for the key mapping is pinned to the oracle, whose
INT64 join path is pinned by the QTT goldens (test_oracle_golden.py); the CPU test below checks the
oracle's STRING path against its own INT64 path through a key bijection."""
import numpy as np
import pytest

from ksql_amd import abi


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def _skey(k):
    # a bijection onto ASCII, multi-byte UTF-8, digit keys (inline ids, khip_dict.hpp: with and
    # without leading zeros; 18 digits: too long to inline) and the empty key (lengths 0..~24)
    if k == 0:
        return ""
    if k % 13 == 0:
        return "usér-%d-ünïcødé" % k
    if k % 7 == 0:
        return "%d" % k
    if k % 11 == 0:
        return "%018d" % k
    if k % 17 == 0:
        return "0%d" % k
    return "user_%d" % k


def _events(rng, nkeys, rounds):
    ev = []
    for _ in range(rounds):
        m = int(rng.integers(1, 3000))
        ev.append(("T", rng.integers(0, nkeys, m), rng.random(m) > 0.02, rng.random(m) > 0.1,
                   [rng.integers(0, 3, m).astype(np.int32), rng.uniform(-5, 5, m)],
                   [rng.random(m) > 0.05 for _ in range(2)]))
        m = int(rng.integers(1, 5000))
        ev.append(("S", rng.integers(0, nkeys + 300, m), rng.random(m) > 0.02, rng.random(m) > 0.02,
                   np.where(rng.random(m) < 0.01, -1, rng.integers(0, 10**6, m))))
    return ev


def _replay(lib, events, join_type, where, utf8):
    t = abi.TableHandle(lib, ["INT32", "DOUBLE"], capacity_hint=64, key_type="UTF8" if utf8 else "INT64")
    outs = []
    for e in events:
        kk = e[1]
        ka = {"utf8_keys": [_skey(int(k)) for k in kk]} if utf8 else {"keys": kk}
        if e[0] == "T":
            _, _, kv, rv, cols, cv = e
            t.upsert(abi.HostBatch(np.zeros(len(kk), np.int64), key_valid=kv, row_valid=rv, cols=cols, col_valid=cv,
                                   **ka))
        else:
            _, _, kv, rv, ts = e
            outs.append(t.probe(abi.HostBatch(ts, key_valid=kv, row_valid=rv, **ka), join_type, where))
    outs.append(t.size())
    t.close()
    return outs


def _same(g, o):
    assert g[-1] == o[-1]
    for a, b in zip(g[:-1], o[:-1]):
        assert a["n"] == b["n"]
        assert np.array_equal(a["stream_row"], b["stream_row"])
        assert np.array_equal(a["matched"], b["matched"])
        for c in range(2):
            assert np.array_equal(a["nulls"][c], b["nulls"][c])
            assert np.array_equal(a["cols"][c][~a["nulls"][c]], b["cols"][c][~b["nulls"][c]])


WHERES = [None, {"col": 0, "op": "EQ", "i64": 2, "f64": 2.0}, {"col": 1, "op": "GT", "i64": 0, "f64": 0.5}]


@pytest.mark.parametrize("join_type", ["LEFT", "INNER"])
def test_oracle_string_table_equals_int_table(orc, join_type):
    """Oracle self-check: STRING keys through a bijection give the INT64 table's output."""
    rng = np.random.default_rng(5)
    ev = _events(rng, 3000, 4)
    _same(_replay(orc, ev, join_type, WHERES[1], True), _replay(orc, ev, join_type, WHERES[1], False))


@pytest.mark.gpu
@pytest.mark.parametrize("join_type", ["LEFT", "INNER"])
@pytest.mark.parametrize("where", WHERES)
def test_string_join_vs_oracle(prod, orc, join_type, where):
    rng = np.random.default_rng(77)
    ev = _events(rng, 4000, 6)
    _same(_replay(prod, ev, join_type, where, True), _replay(orc, ev, join_type, where, True))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 4097, 100_003])
def test_string_join_probe_device_vs_oracle(prod, orc, n):
    """khip_table_probe_device with a device STRING-key batch: row-aligned emit / matched / null
    bitmaps and the gathered column equal the oracle's compacted output (n not a multiple of 64)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(n)
    tk = rng.integers(0, 20000, 30000)
    tv = rng.integers(0, 3, tk.size).astype(np.int32)
    trv = rng.random(tk.size) > 0.05
    tcv = rng.random(tk.size) > 0.05
    tb = abi.HostBatch(np.zeros(tk.size, np.int64), utf8_keys=[_skey(int(k)) for k in tk], row_valid=trv,
                       cols=[tv], col_valid=[tcv])
    tables = [abi.TableHandle(lib, ["INT32"], key_type="UTF8") for lib in (prod, orc)]
    for t in tables:
        t.upsert(tb)
    pk = rng.integers(0, 22000, n)
    pts = np.where(rng.random(n) < 0.01, -1, rng.integers(0, 10**6, n))
    pkv = rng.random(n) > 0.02
    hb = abi.HostBatch(pts, utf8_keys=[_skey(int(k)) for k in pk], key_valid=pkv)
    for jt in ("LEFT", "INNER"):
        for where in (None, {"col": 0, "op": "EQ", "i64": 2, "f64": 2.0}):
            o = tables[1].probe(hb, jt, where)
            g = tables[0].probe(hb, jt, where)
            assert g["n"] == o["n"] and np.array_equal(g["stream_row"], o["stream_row"])
            koff = torch.from_numpy(hb.key_offsets).cuda()
            kb = torch.from_numpy(hb.key_bytes).cuda()
            dts = torch.from_numpy(pts).cuda()
            kvb = abi.bitmap_torch(torch.from_numpy(pkv).cuda())
            nb = (n + 7) // 8
            emit = torch.zeros(nb, dtype=torch.uint8, device="cuda")
            matched = torch.zeros(nb, dtype=torch.uint8, device="cuda")
            col = torch.zeros(n, dtype=torch.int32, device="cuda")
            null = torch.zeros(nb, dtype=torch.uint8, device="cuda")
            n_emit = tables[0].probe_device(abi.DeviceBatch(dts, key_offsets=koff, key_bytes=kb, key_valid=kvb), jt,
                                            where, emit, matched, [col], [null])
            assert n_emit == o["n"]
            e = np.unpackbits(emit.cpu().numpy(), bitorder="little")[:n].astype(bool)
            assert np.array_equal(np.nonzero(e)[0], o["stream_row"])
            mt = np.unpackbits(matched.cpu().numpy(), bitorder="little")[:n].astype(bool)
            assert np.array_equal(mt[o["stream_row"]], o["matched"].astype(bool))
            nl = np.unpackbits(null.cpu().numpy(), bitorder="little")[:n].astype(bool)
            assert np.array_equal(nl[o["stream_row"]], o["nulls"][0])
            cv = col.cpu().numpy()[o["stream_row"]]
            assert np.array_equal(cv[~o["nulls"][0]], o["cols"][0][~o["nulls"][0]])
    assert tables[0].size() == tables[1].size()
    for t in tables:
        t.close()
