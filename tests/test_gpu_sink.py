"""Sink serializers on the HIP path (khip_sink_*, include/ksqldb_hip.h "serialization").

1. Every byte the device writes equals tests/sink_ref.py (the CPU restatement of GenericKeySerDe /
   GenericRowSerDe's output side): Double.toString over random bit patterns, decimal-looking values
   and the special values; Long.toString at the extremes; KAFKA / JSON / DELIMITED keys with the
   time- and session-windowed suffixes; JSON / DELIMITED / KAFKA values with NULLs and tombstones.
2. GROUP BY columns → serialized composite keys (khip_sink_key), host and device batches, with NULLs.
3. The QTT output sequences as bytes: every extracted aggregate case whose sink formats the device
   writes, replayed one record per push; each emitted record's key bytes equal the key the QTT case
   expects, serialized (windowed suffix included), and its value equals the expected value (JSON:
   the same fields in output-column order, integers exact, doubles within the reference comparator's
   1e-6; DELIMITED: the expected text field by field) — and is byte-identical to sink_ref's encoding
   of the row.  Composite GROUP BY keys are built on the device from the group columns.
"""
import json
import math
import struct

import numpy as np
import pytest

import qtt
import sink_ref
from ksql_amd import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


def _rows(n, keys=None, ws=None, we=None, values=(), nulls=()):
    return {"n": n, "key": keys if keys is not None else np.zeros(n, np.int64),
            "ws": np.zeros(n, np.int64) if ws is None else ws, "we": np.zeros(n, np.int64) if we is None else we,
            "values": list(values), "nulls": list(nulls)}


def _special_doubles(rng, n):
    bits = rng.integers(0, 2**63, n, dtype=np.int64).astype(np.uint64) | (
        rng.integers(0, 2, n).astype(np.uint64) << np.uint64(63))
    rand_bits = bits.view(np.float64)
    dec = np.array([float("%de%d" % (rng.integers(1, 10 ** int(rng.integers(1, 17))), rng.integers(-330, 310)))
                    for _ in range(n)])
    specials = np.array([0.0, -0.0, 1.0, -1.0, 0.1, 0.001, 9.999e-4, 1e7, 9999999.0, 1e-3, 1e22, 1e23,
                         5e-324, 1e-323, 2.2250738585072014e-308, 1.7976931348623157e308, 2.82879384806159e17,
                         123456.789, 1.0 / 3, float("nan"), float("inf"), float("-inf"), 2.0 ** 63, -2.0 ** 52])
    return np.concatenate([rand_bits, dec, specials])


@pytest.mark.parametrize("vfmt", ["JSON", "DELIMITED"])
@pytest.mark.parametrize("dev_out", [False, True])
def test_doubles_and_longs(prod, vfmt, dev_out):
    rng = np.random.default_rng(11)
    d = _special_doubles(rng, 4000)
    n = len(d)
    ints = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    ints[:4] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1]
    dn = rng.random(n) < 0.05
    s = abi.SinkHandle(prod, "KAFKA", [("K", "INT64")], vfmt, [("D", "DOUBLE", 0), ("L", "INT64", 1)])
    keys, vals = s.encode(_rows(n, keys=np.arange(n, dtype=np.int64), values=[d, ints],
                                nulls=[dn, np.zeros(n, bool)]), device_out=dev_out, align=5)
    bad = []
    for i in range(n):
        exp = sink_ref.encode_value(vfmt, [("D", "DOUBLE"), ("L", "INT64")], [None if dn[i] else float(d[i]), int(ints[i])])
        if vals[i] != exp:
            bad.append((i, d[i], vals[i], exp))
        assert keys[i] == struct.pack(">q", i)
    assert not bad, bad[:5]
    s.close()


WINDOWS = ["NONE", "TUMBLING", "SESSION"]


@pytest.mark.parametrize("window", WINDOWS)
@pytest.mark.parametrize("kfmt,ktype", [("KAFKA", "INT64"), ("KAFKA", "INT32"), ("KAFKA", "STRING"),
                                        ("JSON", "INT64"), ("JSON", "STRING"), ("DELIMITED", "STRING")])
@pytest.mark.parametrize("dev_out", [False, True])
def test_keys_windows_tombstones(prod, window, kfmt, ktype, dev_out):
    rng = np.random.default_rng(hash((window, kfmt, ktype)) % 1000)
    n = 3000
    if ktype == "STRING":
        pool = ["a", "", "x,y", 'q"u', " lead", "trail ", "#h", "é", "tab\there", "nl\nx", "ctl\x01", "\\back"]
        keys = [pool[i % len(pool)] + str(i // len(pool)) if i % 7 else pool[i % len(pool)] for i in range(n)]
    else:
        lim = 2**31 if ktype == "INT32" else 2**63
        keys = rng.integers(-lim, lim - 1, n, dtype=np.int64)
    ws = rng.integers(0, 2**40, n, dtype=np.int64)
    we = ws + rng.integers(0, 10**6, n, dtype=np.int64)
    cnt = rng.integers(0, 10**9, n, dtype=np.int64)
    tomb = (rng.random(n) < 0.1).astype(np.uint8)
    vcols = [("COUNT", "INT64", 0), ("WSTART", "INT64", "WS"), ("WEND", "INT64", "WE")]
    for vfmt in ("JSON", "DELIMITED", "KAFKA"):
        vc = vcols[:1] if vfmt == "KAFKA" else vcols
        s = abi.SinkHandle(prod, kfmt, [("K", ktype)], vfmt, vc, window_kind=window)
        kb, vb = s.encode(_rows(n, keys=keys, ws=ws, we=we, values=[cnt], nulls=[np.zeros(n, bool)]), tombstone=tomb,
                          device_out=dev_out, align=len(vfmt) % 16)
        for i in range(n):
            kv = keys[i] if ktype == "STRING" else int(keys[i])
            exp_k = sink_ref.encode_key(kfmt, [("K", ktype)], [kv]) + sink_ref.window_suffix(window, int(ws[i]), int(we[i]))
            assert kb[i] == exp_k, (i, kb[i], exp_k)
            exp_v = sink_ref.encode_value(vfmt, [(c[0], c[1]) for c in vc],
                                          [int(cnt[i]), int(ws[i]), int(we[i])][:len(vc)], tombstone=bool(tomb[i]))
            assert vb[i] == exp_v, (i, vb[i], exp_v)
        s.close()


@pytest.mark.parametrize("n", [1, 255, 256, 257, 70_000])
def test_device_outputs_long_rows(prod, n):
    """Device outputs (offsets, bytes and nulls written in place) against host outputs and the CPU
    restatement: keys of 0..300 bytes, JSON values of five columns (most NULL in some rows),
    tombstones (empty values), several tiles of rows, every output alignment, guard bytes either
    side of the outputs untouched."""
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 300, n)
    short = rng.random(n) < 0.5
    lens[short] = rng.integers(0, 60, int(short.sum()))
    keys = ["".join(chr(97 + (i + j) % 26) for j in range(int(lens[i]))) for i in range(n)]
    names = ["C%d_" % c + "X" * int(rng.integers(1, 12)) for c in range(5)]
    vc = [(nm, "INT64" if c % 2 else "DOUBLE", c) for c, nm in enumerate(names)]
    cols = [rng.uniform(-1e9, 1e9, n) if c % 2 == 0 else rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
            for c in range(5)]
    few = rng.random(n) < 0.3  # short values: most columns NULL
    nulls = [few & (c > 0) for c in range(5)]
    tomb = (rng.random(n) < 0.1).astype(np.uint8)
    ws = rng.integers(0, 2**40, n, dtype=np.int64)
    s = abi.SinkHandle(prod, "KAFKA", [("K", "STRING")], "JSON", vc, window_kind="TUMBLING")
    snap = _rows(n, keys=keys, ws=ws, we=ws + 1000, values=cols, nulls=nulls)
    host = s.encode(snap, tombstone=tomb)
    for align in (0, 7, 13) if n < 1000 else (3,):
        assert s.encode(snap, tombstone=tomb, device_out=True, align=align) == host
    for i in range(0, n, max(1, n // 300)):
        exp_k = sink_ref.encode_key("KAFKA", [("K", "STRING")], [keys[i]]) + sink_ref.window_suffix(
            "TUMBLING", int(ws[i]), int(ws[i]) + 1000)
        assert host[0][i] == exp_k
        exp_v = sink_ref.encode_value("JSON", [(c[0], c[1]) for c in vc],
                                      [None if nulls[c][i] else (float(cols[c][i]) if c % 2 == 0 else int(cols[c][i]))
                                       for c in range(5)], tombstone=bool(tomb[i]))
        assert host[1][i] == exp_v, (i, host[1][i], exp_v)
    if n >= 255:
        assert any(len(k) > 52 for k in host[0]) and any(len(k) <= 52 for k in host[0])
        assert any(v and len(v) > 116 for v in host[1]) and any(v and len(v) <= 116 for v in host[1])
    s.close()


@pytest.mark.parametrize("dev_out", [False, True])
def test_json_column_names_escaped(prod, dev_out):
    """JSON object columns print '{' / ',' + the escaped name + ':' from text built once on the
    host by the device escaper; a name whose escaped text passes 72 bytes (64 control characters:
    384) is escaped per row instead.  Both against sink_ref, for value and composite-key objects."""
    names = ['a"b', "back\\slash", "ctl\x01x\x1f", "tab\there", "é", "\x02" * 64, "K" * 64, "Z"]
    n = 700
    rng = np.random.default_rng(9)
    cols = [rng.integers(-10**6, 10**6, n, dtype=np.int64) for _ in names]
    vc = [(nm, "INT64", c) for c, nm in enumerate(names)]
    kc = [(nm, "INT64") for nm in names[:4]] + [(names[5], "INT32")]
    s = abi.SinkHandle(prod, "KAFKA", [("K", "INT64")], "JSON", vc)
    kb, vb = s.encode(_rows(n, values=cols, nulls=[np.zeros(n, bool)] * len(names)), device_out=dev_out, align=1)
    for i in range(n):
        exp = sink_ref.encode_value("JSON", [(c[0], c[1]) for c in vc], [int(cols[c][i]) for c in range(len(names))])
        assert vb[i] == exp, (i, vb[i], exp)
    s.close()
    s = abi.SinkHandle(prod, "JSON", kc, "JSON", [])  # composite keys: khip_sink_key
    hb = abi.HostBatch(np.arange(n, dtype=np.int64), keys=np.zeros(n, np.int64))
    kcols = [cols[0], cols[1], cols[2], cols[3], cols[4].astype(np.int32)]
    got = s.key_bytes(s.key(hb, kcols))
    for i in range(n):
        exp = sink_ref.encode_key("JSON", kc, [int(kcols[c][i]) for c in range(len(kc))])
        assert got[i] == exp, (i, got[i], exp)
    s.close()


def test_value_null_kafka_and_empty(prod):
    s = abi.SinkHandle(prod, "KAFKA", [("K", "INT64")], "KAFKA", [("V", "DOUBLE", 0)])
    kb, vb = s.encode(_rows(3, keys=np.array([1, 2, 3], np.int64), values=[np.array([1.5, 0.0, -2.0])],
                            nulls=[np.array([False, True, False])]))
    assert vb == [struct.pack(">d", 1.5), None, struct.pack(">d", -2.0)]
    kb, vb = s.encode(_rows(0, keys=np.zeros(0, np.int64), values=[np.zeros(0)], nulls=[np.zeros(0, bool)]))
    assert kb == [] and vb == []
    s.close()


@pytest.mark.parametrize("vfmt", ["JSON", "DELIMITED"])
def test_value_sources_with_gap(prod, vfmt):
    """Value columns read rows columns 0 and 2; column 1 (an INT32 column no value column reads,
    n * 4 bytes of host memory) sits in the gap and must not be staged or read."""
    rng = np.random.default_rng(5)
    n = 5000
    a = rng.integers(-2**40, 2**40, n, dtype=np.int64)
    gap = rng.integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype(np.int32)
    b = rng.uniform(-1e6, 1e6, n)
    bn = rng.random(n) < 0.1
    s = abi.SinkHandle(prod, "KAFKA", [("K", "INT64")], vfmt, [("A", "INT64", 0), ("B", "DOUBLE", 2)])
    kb, vb = s.encode(_rows(n, keys=np.arange(n, dtype=np.int64), values=[a, gap, b],
                            nulls=[np.zeros(n, bool), np.zeros(n, bool), bn]))
    for i in range(n):
        exp = sink_ref.encode_value(vfmt, [("A", "INT64"), ("B", "DOUBLE")], [int(a[i]), None if bn[i] else float(b[i])])
        assert vb[i] == exp, (i, vb[i], exp)
    s.close()


@pytest.mark.parametrize("kfmt", ["JSON", "DELIMITED"])
@pytest.mark.parametrize("device", [False, True])
def test_composite_keys(prod, kfmt, device):
    import torch
    rng = np.random.default_rng(5)
    n = 5000
    a = rng.integers(-2**31, 2**31 - 1, n).astype(np.int32)
    b = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    strs = [None if rng.random() < 0.03 else "s%d%s" % (i % 97, ',"' if i % 13 == 0 else "") for i in range(n)]
    av = rng.random(n) > 0.02
    cols_t = [("A", "INT32"), ("B", "INT64"), ("S", "STRING")]
    s = abi.SinkHandle(prod, kfmt, cols_t, "JSON", [])
    ts = np.arange(n, dtype=np.int64)
    if device:
        enc = [b"" if x is None else x.encode() for x in strs]
        offs = np.concatenate([[0], np.cumsum([len(e) for e in enc])]).astype(np.int64)
        dev = {k: torch.from_numpy(v).cuda() for k, v in dict(
            a=a, b=b, offs=offs, bytes=np.frombuffer(b"".join(enc) + b"\0", np.uint8).copy(),
            av=abi.bitmap(av), sv=abi.bitmap([x is not None for x in strs]), ts=ts).items()}
        batch = abi.Batch()
        batch.n_rows, batch.mem = n, abi.MEM_DEVICE
        batch.ts = dev["ts"].data_ptr()

        class _B:
            pass
        bb = _B()
        bb.struct = batch
        keyed = s.key(bb, [{"data": dev["a"].data_ptr(), "valid": dev["av"].data_ptr()}, {"data": dev["b"].data_ptr()},
                           {"offsets": dev["offs"].data_ptr(), "bytes": dev["bytes"].data_ptr(),
                            "valid": dev["sv"].data_ptr()}])
        kb = keyed.struct
        torch.cuda.synchronize()
        offs_d = torch.empty(n + 1, dtype=torch.int64)
        abi._hip_copy(offs_d.numpy(), kb.key_offsets, (n + 1) * 8)
        tot = int(offs_d[n])
        data = np.zeros(max(tot, 1), np.uint8)
        abi._hip_copy(data, kb.key_bytes, tot)
        vbits = np.zeros((n + 7) // 8, np.uint8)
        abi._hip_copy(vbits, kb.key_valid, len(vbits))
        valid = np.unpackbits(vbits, bitorder="little")[:n].astype(bool)
        o = offs_d.numpy()
        got = [bytes(data[o[i]:o[i + 1]]) if valid[i] else None for i in range(n)]
    else:
        hb = abi.HostBatch(ts, keys=np.zeros(n, np.int64))
        keyed = s.key(hb, [(a, av), b, strs])
        got = s.key_bytes(keyed)
    for i in range(n):
        vals = [int(a[i]) if av[i] else None, int(b[i]), strs[i]]
        exp = None if any(v is None for v in vals) else sink_ref.encode_key(kfmt, cols_t, vals)
        assert got[i] == exp, (i, got[i], exp)
    s.close()


# ------------------------------------------------------------------ QTT output sequences as bytes

def _sink_cases():
    out = []
    for c in qtt.load_cases("agg"):
        if c.get("sink") and c["desc"].get("emit", "CHANGES") == "CHANGES" and not c["desc"]["repartition"]:
            out.append(c)
    return out


SINK_CASES = _sink_cases()


def _result_type(case, a):
    ag = case["desc"]["aggs"][a]
    if ag["kind"] in ("COUNT", "COUNT_STAR"):
        return "INT64"
    if ag["kind"] == "AVG":
        return "DOUBLE"
    return case["desc"]["col_types"][ag["arg_col"]]


def _close(a, b):
    if isinstance(a, float) or isinstance(b, float):
        if isinstance(a, str) or isinstance(b, str):
            return str(a) == str(b)
        if math.isnan(float(a)) and math.isnan(float(b)):
            return True
        return abs(float(a) - float(b)) < 1e-6
    return a == b


def _expected_key(case, o):
    sk = case["sink"]
    if case["desc"].get("group"):
        inner = o["key"].encode()  # the fixture's composite key is already the serialized key
    else:
        (name, typ), = sk["key_cols"]
        inner = sink_ref.encode_key(sk["key_format"], [(name, typ)], [o["key"]])
    return inner + sink_ref.window_suffix(case["desc"]["window_kind"], o["ws"], o["we"])


@pytest.mark.parametrize("case", SINK_CASES, ids=[c["name"] for c in SINK_CASES])
def test_qtt_output_bytes(prod, case):
    sk = case["sink"]
    d = case["desc"]
    vcols = []
    for vc in sk["value_cols"]:
        if vc["src"] == "AGG":
            vcols.append((vc["name"], _result_type(case, vc["agg"]), vc["agg"]))
        else:
            vcols.append((vc["name"], "INT64", vc["src"]))
    group = d.get("group")
    kcols = [tuple(k) for k in sk["key_cols"]]
    if group:
        kcols = [tuple(k) for k in group["cols"]]
    s = abi.SinkHandle(prod, sk["key_format"], kcols, sk["value_format"], vcols, window_kind=d["window_kind"])
    h = abi.AggHandle(prod, qtt.case_desc(case))
    got = []
    for i in range(len(case["input"])):
        batch = qtt.case_batch(case, i, i + 1)
        if group:  # the composite key, built on the device from the GROUP BY columns
            gv = case["input"][i]["gvals"]
            cols = []
            for (name, typ), v in zip(kcols, gv):
                if typ == "STRING":
                    cols.append([v])
                else:
                    cols.append((np.array([0 if v is None else v], np.int32 if typ == "INT32" else np.int64),
                                 [v is not None]))
            keyed = s.key(batch, cols)
            kb = s.key_bytes(keyed)[0]
            exp_k = None if case["input"][i]["key"] is None else case["input"][i]["key"].encode()
            assert kb == exp_k, (i, kb, exp_k)
            h.push(keyed)
        else:
            h.push(batch)
        chg = h.changes()
        if chg["n"] == 0:
            continue
        keys, vals = s.encode(chg, tombstone=chg["tombstone"], key_serialized=bool(group))
        for r in range(chg["n"]):
            got.append((keys[r], vals[r], chg, r))
    h.close()
    exp = case["outputs"]
    assert len(got) == len(exp), (len(got), len(exp))
    names = [v[0] for v in vcols]
    for i, ((kb, vb, chg, r), o) in enumerate(zip(got, exp)):
        assert kb == _expected_key(case, o), (i, kb, _expected_key(case, o))
        if o["tombstone"]:
            assert vb is None, (i, vb)
            continue
        assert vb is not None, i
        # the row's bytes are exactly sink_ref's serialization of the row the device emitted
        row_vals = []
        for (name, typ, src) in vcols:
            if src == "WS":
                row_vals.append(int(chg["ws"][r]))
            elif src == "WE":
                row_vals.append(int(chg["we"][r]))
            else:
                row_vals.append(None if chg["nulls"][src][r] else chg["values"][src][r].item())
        assert vb == sink_ref.encode_value(sk["value_format"], [(v[0], v[1]) for v in vcols], row_vals), i
        # ... and equal to the reference's expected record
        rv = o["raw_value"]
        if sk["value_format"] == "JSON":
            gv = json.loads(vb)
            assert list(gv.keys()) == names, (list(gv.keys()), names)
            ev = {k.upper(): x for k, x in rv.items()} if isinstance(rv, dict) else {names[0]: rv}
            for nm in names:
                if o.get("present") is not None and nm not in ev:
                    continue
                assert _close(gv[nm], ev[nm]) or (gv[nm] is None and ev[nm] is None), (i, nm, gv[nm], ev[nm])
        else:
            gf, ef = vb.decode().split(","), str(rv).split(",")
            assert len(gf) == len(ef), (i, vb, rv)
            for (nm, typ, _), g, e in zip(vcols, gf, ef):
                if typ == "DOUBLE" and g and e:
                    assert abs(float(g) - float(e)) < 1e-6, (i, nm, g, e)
                else:
                    assert g == e, (i, nm, g, e)
    s.close()
