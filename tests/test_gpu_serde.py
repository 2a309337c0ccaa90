"""khip_serde_decode (KAFKA / DELIMITED / JSON record bytes → device columns) against the CPU
restatement of ksqlDB's deserializers (tests/serde_ref.py), and end to end: the reference's own
QTT inputs as raw record bytes → decode → aggregate → the reference's expected outputs."""
import json
import random
import struct

import numpy as np
import pytest

import avro_ref
import qtt
import serde_ref
from ksql_amd import abi

pytestmark = pytest.mark.gpu

FIELDS = [("ID", "INT64", -1), ("V32", "INT32", 0), ("V64", "INT64", 1), ("D", "DOUBLE", 2), ("NAME", "STRING", 3),
          ("SKIPPED", "INT32", -1)]
OUT_TYPES = ["INT32", "INT64", "DOUBLE", "STRING"]


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


def _num_text(rng, t):
    r = rng.random()
    if t == "DOUBLE":
        if r < 0.3:
            return repr(rng.uniform(-1e6, 1e6))
        if r < 0.45:  # more than 19 significant digits (big-integer rounding path)
            return str(rng.randrange(1, 10)) + "".join(str(rng.randrange(10)) for _ in range(rng.randrange(19, 30))) + \
                "e" + str(rng.randrange(-320, 300))
        if r < 0.55:
            return rng.choice(["NaN", "Infinity", "-Infinity", " 1.5 ", "2.5e-310", "1e400", "7d", "abc", "1..2"])
        return "%d.%d" % (rng.randrange(-10 ** 6, 10 ** 6), rng.randrange(1000))
    bits = 32 if t == "INT32" else 64
    if r < 0.7:
        return str(rng.randrange(-(1 << (bits - 1)), 1 << (bits - 1)))
    return rng.choice([str(1 << bits), "-0", "+5", " 3", "1.0", "x", "99999999999999999999"])


def _delimited(rng):
    parts = []
    for name, t, _ in FIELDS:
        if rng.random() < 0.08:
            parts.append("")
            continue
        if t == "STRING":
            s = rng.choice(["alice", "b,ob", 'q"uote', "", "x y"])
            parts.append('"%s"' % s.replace('"', '""') if ("," in s or '"' in s or rng.random() < 0.2) else s)
        else:
            v = _num_text(rng, t)
            parts.append('"%s"' % v if rng.random() < 0.1 else v)
    if rng.random() < 0.03:
        parts.append("extra")  # arity mismatch
    if rng.random() < 0.03:
        parts = parts[:-1]
    line = ",".join(parts)
    return (line + ("\n" if rng.random() < 0.05 else "")).encode()


def _json(rng):
    obj = []
    for name, t, _ in FIELDS:
        r = rng.random()
        if r < 0.07:
            continue  # missing
        key = name if rng.random() < 0.7 else name.lower()
        if r < 0.12:
            val = "null"
        elif t == "STRING":
            val = json.dumps(rng.choice(["alice", "é", "a\"b"])) if rng.random() < 0.8 else rng.choice(["12", "true", "[1,2]"])
        else:
            k = rng.random()
            if k < 0.5:
                txt = _num_text(rng, t)
                try:
                    json.loads(txt)
                    val = txt  # a JSON number token
                except ValueError:
                    val = json.dumps(txt)
            elif k < 0.7:
                val = json.dumps(_num_text(rng, t))  # numbers as strings
            elif k < 0.8:
                val = rng.choice(["true", "{\"a\":1}", "[1]"])
            elif k < 0.9:  # float token into an integer column (BigDecimal truncation)
                val = repr(rng.uniform(-3e9, 3e9)) if rng.random() < 0.6 else rng.choice(DECIMAL_TOKENS)
            else:
                val = str(rng.randrange(-(1 << 70), 1 << 70))  # BigInteger token
        obj.append('"%s": %s' % (key, val))
    if rng.random() < 0.1 and obj:
        obj.append(obj[0])  # duplicate field: the last wins
    body = "{" + ", ".join(obj) + "}"
    if rng.random() < 0.03:
        body = body[:-1]  # truncated
    if rng.random() < 0.05:
        body = "  " + body + "  trailing"
    return body.encode()


# JSON float tokens (Jackson BigDecimal) whose int / long value differs from a saturating double
# conversion: above 2^31, above 2^53 (digits a double loses), 1e20 (low 64 bits), huge exponents
DECIMAL_TOKENS = ["3000000000.5", "-3000000000.5", "1e20", "-1e20", "9007199254740993.7", "1.5e300", "-0.9",
                  "123456789012345678901234.9", "4.2E1", "1e-5", "0.0", "-0e0", "18446744073709551617.25",
                  "2147483648.0", "-2147483649.99", "1E+19", "12345678901234567890e-3"]


def test_json_decimal_into_integer_columns(prod):
    """USE_BIG_DECIMAL_FOR_FLOATS (KsqlJsonDeserializer.java:68-70): intValue() / longValue() of a
    BigDecimal keep the low bits of the truncated integer part, exactly."""
    fields = [("V32", "INT32", 0), ("V64", "INT64", 1), ("D", "DOUBLE", 2)]
    vals = [('{"V32": %s, "V64": %s, "D": %s}' % (t, t, t)).encode() for t in DECIMAL_TOKENS]
    keys = [struct.pack(">q", i) for i in range(len(vals))]
    sd = abi.SerdeHandle(prod, "JSON", fields, key_type="INT64")
    d, nerr = sd.decode(np.arange(len(vals), dtype=np.int64), keys, vals)
    exp, experr = serde_ref.decode("JSON", fields, "INT64", keys, vals)
    assert nerr == experr == 0
    got = sd.columns(d, ["INT32", "INT64", "DOUBLE"])
    _check(got, exp, fields, ["INT32", "INT64", "DOUBLE"])
    assert int(got["cols"][0][0]) == -1294967296 and int(got["cols"][1][2]) == 7766279631452241920
    assert int(got["cols"][1][4]) == 9007199254740993
    sd.close()


def _kafka_value(rng):
    return struct.pack(">q", rng.randrange(-(1 << 63), 1 << 63)) if rng.random() < 0.95 else b"\x01\x02"


def _records(rng, fmt, n):
    keys, vals = [], []
    for _ in range(n):
        r = rng.random()
        keys.append(None if r < 0.03 else (b"\x00\x01" if r < 0.05 else struct.pack(">q", rng.randrange(-1000, 1000))))
        if rng.random() < 0.05:
            vals.append(None)
        elif fmt == "DELIMITED":
            vals.append(_delimited(rng))
        elif fmt == "JSON":
            vals.append(_json(rng))
        else:
            vals.append(_kafka_value(rng))
    return keys, vals


def _check(got, exp, fields, out_types):
    n = len(exp)
    for i, (kv, key, rv, row) in enumerate(exp):
        assert got["key_valid"][i] == kv, (i, kv)
        assert got["row_valid"][i] == rv, i
        if kv and key is not None and "key" in got:
            assert got["key"][i] == key, i
        if not rv or row is None:
            continue
        for name, t, c in fields:
            if c < 0:
                continue
            v = row[name]
            assert got["valid"][c][i] == (v is not None), (i, name, v)
            if v is None or t == "STRING":
                continue
            g = got["cols"][c][i]
            if t == "DOUBLE":
                assert struct.pack("<d", g) == struct.pack("<d", v) or (np.isnan(g) and np.isnan(v)), (i, name, g, v)
            else:
                assert int(g) == v, (i, name, g, v)


@pytest.mark.parametrize("fmt", ["DELIMITED", "JSON", "KAFKA"])
def test_decode_vs_reference(prod, fmt):
    rng = random.Random({"DELIMITED": 1, "JSON": 2, "KAFKA": 3}[fmt])
    fields = FIELDS if fmt != "KAFKA" else [("V64", "INT64", 0)]
    out_types = OUT_TYPES if fmt != "KAFKA" else ["INT64"]
    sd = abi.SerdeHandle(prod, fmt, fields, key_type="INT64")
    for n in (1, 63, 4000):
        keys, vals = _records(rng, fmt, n)
        ts = np.arange(n, dtype=np.int64)
        d, nerr = sd.decode(ts, keys, vals)
        exp, experr = serde_ref.decode(fmt, fields, "INT64", keys, vals)
        assert nerr == experr
        _check(sd.columns(d, out_types), exp, fields, out_types)
    sd.close()


def test_decode_string_keys_feed_aggregate(prod):
    """UTF-8 keys straight from the records into the aggregate: COUNT(*) / SUM by card."""
    rng = random.Random(9)
    n = 5000
    cards = ["4000%012d" % rng.randrange(300) for _ in range(n)]
    amounts = [rng.randrange(-100, 100) for _ in range(n)]
    vals = [("%d,%s" % (a, "x")).encode() for a in amounts]
    sd = abi.SerdeHandle(prod, "DELIMITED", [("AMOUNT", "INT64", 0), ("TAG", "STRING", -1)], key_type="STRING")
    ts = np.arange(n, dtype=np.int64) * 10
    d, nerr = sd.decode(ts, [c.encode() for c in cards], vals)
    assert nerr == 0
    desc = abi.make_agg_desc(window_kind="TUMBLING", size_ms=20_000, key_type="UTF8", col_types=["INT64"],
                             aggs=[("COUNT_STAR", -1), ("SUM", 0)])
    g = abi.AggHandle(prod, desc)
    g.push(d)
    got = g.snapshot()
    g.close()
    o = abi.AggHandle(abi.load_oracle(), desc)
    o.push(abi.HostBatch(ts, utf8_keys=cards, cols=[np.array(amounts, np.int64)]))
    exp = o.snapshot()
    o.close()
    assert got["key"] == exp["key"]
    assert np.array_equal(got["ws"], exp["ws"]) and np.array_equal(got["values"][1], exp["values"][1])
    sd.close()


# ---- QTT inputs as the raw record bytes the reference consumed

RAW_CASES = [c for c in qtt.load_cases("agg") if c.get("raw")]


@pytest.mark.parametrize("case", RAW_CASES, ids=["%s %s" % (c["source"], c["name"]) for c in RAW_CASES])
def test_qtt_raw_records_end_to_end(prod, case):
    """Serialized QTT inputs (DELIMITED / JSON values, KAFKA keys) → khip_serde_decode →
    khip_agg_push (one record per push) → the reference's expected output sequence."""
    raw = case["raw"]
    fields = [(f["name"], f["type"], f["out"]) for f in raw["fields"]]
    key_type = raw["key_type"]
    writer = avro_ref.ksql_writer_schema(fields) if raw["format"] == "AVRO" else None
    sd = abi.SerdeHandle(prod, raw["format"], fields, key_type="STRING" if key_type == "STRING" else key_type,
                         avro_schema=writer)
    h = abi.AggHandle(prod, qtt.case_desc(case))
    rows = []
    for rec in raw["records"]:
        k = rec["key"]
        if k is None:
            kb = None
        elif key_type == "STRING":
            kb = k.encode()
        else:
            kb = struct.pack(">q" if key_type == "INT64" else ">i", int(k))
        v = rec["value"]
        if v is None:
            vb = None
        elif writer:  # the QTT harness serializes the spec's JSON object with the source's AVRO schema
            vb = avro_ref.encode(writer, _avro_spec(v, fields))
        else:
            vb = (v if isinstance(v, str) else json.dumps(v)).encode()
        d, nerr = sd.decode(np.array([rec["ts"]], np.int64), [kb], [vb])
        h.push(d)
        rows += qtt._rows_of(h.changes())
    h.close()
    sd.close()
    assert qtt.compare_outputs(case, rows) == []


def _avro_spec(value, fields):
    """A QTT input value (JSON object) as the Avro record of the source's schema: the field of the
    column's name (any case), coerced to the column's type."""
    up = {k.upper(): x for k, x in value.items()}
    rec = {}
    for name, t, _ in fields:
        x = up.get(name)
        if x is None:
            rec[name] = None
        elif t == "STRING":
            rec[name] = x if isinstance(x, str) else json.dumps(x)
        elif t == "DOUBLE":
            rec[name] = float(x)
        else:
            rec[name] = int(x)
    return rec


@pytest.mark.parametrize("narrow", [False, True])
@pytest.mark.parametrize("fmt", ["DELIMITED", "JSON"])
def test_decode_device_batches_staged_and_long(prod, fmt, narrow):
    """khip_serde_decode on a device-resident raw batch (bench.py's serde_json path): the
    kernel stages each wave's record bytes in LDS when they fit (unaligned record offsets, partial
    first/last dwords) and reads HBM directly when a wave's records are too long (padding makes
    every 7th wave's records exceed the stage).  narrow: a 4-field schema (the kernel variant
    whose field-token arrays live in registers)."""
    torch = pytest.importorskip("torch")
    fields = FIELDS[1:5] if narrow else FIELDS
    rng = random.Random({"DELIMITED": 11, "JSON": 12}[fmt])
    n = 3000
    keys, vals = _records(rng, fmt, n)
    if fmt == "JSON":
        vals = [v if (v is None or (i // 64) % 7) else v[:1] + b" " * 90 + v[1:] for i, v in enumerate(vals)]
    else:
        vals = [v if (v is None or (i // 64) % 7) else v + b"\r\n" + b"x" * 90 for i, v in enumerate(vals)]
    if narrow and fmt == "DELIMITED":  # the narrow schema's records: fields 1..4 of each row
        vals = [v if v is None else _narrow_delimited(v) for v in vals]
    exp, experr = serde_ref.decode(fmt, fields, "INT64", keys, vals)

    def pack(items):
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum([0 if x is None else len(x) for x in items])
        data = np.frombuffer(b"".join(b"" if x is None else x for x in items) + b"\0", np.uint8).copy()
        valid = np.array([x is not None for x in items])
        return offs, data, valid
    koff, kb, kvld = pack(keys)
    voff, vb, vvld = pack(vals)
    dev = lambda a: torch.from_numpy(a).cuda()
    ts = dev(np.arange(n, dtype=np.int64))
    sd = abi.SerdeHandle(prod, fmt, fields, key_type="INT64")
    d, nerr = sd.decode_device(ts, dev(koff), dev(kb), dev(voff), dev(vb), key_valid=dev(abi.bitmap(kvld)),
                               value_valid=dev(abi.bitmap(vvld)))
    assert nerr == experr
    _check(sd.columns(d, OUT_TYPES), exp, fields, OUT_TYPES)
    sd.close()


def _narrow_delimited(v):
    """Drop a DELIMITED record's first and last field (the ID / SKIPPED columns) when it is a plain
    6-field row; other records (quoted, malformed) stay as they are: errors on both sides."""
    parts = v.split(b",")
    return b",".join(parts[1:5]) if len(parts) == 6 and b'"' not in v and b"\n" not in v else v


# ---- AVRO (Confluent wire format + Avro binary of the writer schema; tests/avro_ref.py)

AVRO_FIELDS = [("ID", "INT64", -1), ("V32", "INT32", 0), ("V64", "INT64", 1), ("D", "DOUBLE", 2), ("NAME", "STRING", 3),
               ("F", "DOUBLE", 4), ("W", "INT64", 5)]
# the writer's record: lower-case names matched through upper-casing, a float into a DOUBLE column,
# an int into a BIGINT column, both union orders, plain fields, fields no column reads
AVRO_WRITER = [("id", "long", 1), ("extra", "string", 1), ("V32", "int", 2), ("v64", "long", 0), ("D", "double", 1),
               ("flag", "boolean", 0), ("NAME", "boolean", 1), ("F", "float", 1), ("w", "int", 1),
               ("blob", "bytes", 0)]


def _avro_record(rng):
    rec = {"id": rng.randrange(-(1 << 63), 1 << 63), "extra": rng.choice([None, "", "xyz", "é" * 40]),
           "V32": rng.randrange(-(1 << 31), 1 << 31), "v64": rng.randrange(-(1 << 63), 1 << 63),
           "D": rng.choice([rng.uniform(-1e9, 1e9), float("nan"), -0.0, 1e-310]), "flag": rng.random() < 0.5,
           "NAME": rng.random() < 0.5, "F": rng.uniform(-1e6, 1e6), "w": rng.randrange(-(1 << 31), 1 << 31),
           "blob": bytes(rng.randrange(256) for _ in range(rng.randrange(0, 20)))}
    for k in ("id", "extra", "V32", "D", "NAME", "F", "w"):
        if rng.random() < 0.1:
            rec[k] = None
    return rec


def _avro_corrupt(rng, b):
    k = rng.randrange(7)
    if k == 0:
        return b"\x01" + b[1:]  # unknown magic byte
    if k == 1:
        return b[:rng.randrange(0, len(b))]  # truncated
    if k == 2:
        return b[:5] + b"\x04" + b[6:]  # union branch index 2
    if k == 3:
        return b[:5] + b"\x02" + b"\xff" * 10 + b"\x01"  # long varint over 10 bytes
    if k == 4:
        return b[:1] + b"\x00\x00\x00\x09" + b[5:]  # another schema id
    if k == 5:
        return b + b"trailing bytes"  # ignored: not an error
    return b"\x00"  # shorter than the header


def test_avro_decode_vs_reference(prod):
    rng = random.Random(21)
    fields = AVRO_FIELDS
    out_types = ["INT32", "INT64", "DOUBLE", "STRING", "DOUBLE", "INT64"]
    sd = abi.SerdeHandle(prod, "AVRO", fields, key_type="INT64", avro_schema=AVRO_WRITER, avro_schema_id=7)
    for n in (1, 64, 5000):
        keys, vals = [], []
        for _ in range(n):
            r = rng.random()
            keys.append(None if r < 0.03 else struct.pack(">q", rng.randrange(-1000, 1000)))
            if rng.random() < 0.05:
                vals.append(None)
                continue
            b = avro_ref.encode(AVRO_WRITER, _avro_record(rng), schema_id=7)
            vals.append(_avro_corrupt(rng, b) if rng.random() < 0.1 else b)
        ts = np.arange(n, dtype=np.int64)
        d, nerr = sd.decode(ts, keys, vals)
        exp, experr = avro_ref.decode(fields, AVRO_WRITER, "INT64", keys, vals, schema_id=7)
        assert nerr == experr
        _check(sd.columns(d, out_types), exp, fields, out_types)
    sd.close()


def test_avro_incompatible_writer_type_fails_every_record(prod):
    """validateSchema (ConnectDataTranslator.java:123-146): a long field for an INT column fails
    each record, even where that field is null; null values (tombstones) stay null."""
    fields = [("A", "INT32", 0), ("B", "INT64", 1)]
    writer = [("A", "long", 1), ("B", "long", 1)]
    vals = [avro_ref.encode(writer, {"A": None, "B": 5}), None, avro_ref.encode(writer, {"A": 3, "B": 4})]
    keys = [struct.pack(">q", i) for i in range(3)]
    sd = abi.SerdeHandle(prod, "AVRO", fields, key_type="INT64", avro_schema=writer)
    d, nerr = sd.decode(np.arange(3, dtype=np.int64), keys, vals)
    exp, experr = avro_ref.decode(fields, writer, "INT64", keys, vals)
    assert nerr == experr == 2
    _check(sd.columns(d, ["INT32", "INT64"]), exp, fields, ["INT32", "INT64"])
    sd.close()


# ---- case-insensitive field names beyond ASCII (Java's String.toUpperCase: full Unicode mapping)

UNI_FIELDS = [("STRASSE", "INT64", 0), ("ǄX", "INT64", 1), ("ΣΊΣΥΦΟΣ", "INT64", 2), ("CAFÉ", "DOUBLE", 3),
              ("𐐀B", "INT64", 4), ("FFʼN", "INT32", 5)]
UNI_NAMES = {"STRASSE": ["STRASSE", "straße", "Strasse", "STRAßE", "strasse"],
             "ǄX": ["ǄX", "ǆx", "ǅX", "ǆX"], "ΣΊΣΥΦΟΣ": ["ΣΊΣΥΦΟΣ", "σίσυφος", "Σίσυφος", "σίσυφοσ"],
             "CAFÉ": ["CAFÉ", "café", "Café", "cafe"], "𐐀B": ["𐐀B", "𐐨b", "𐐨B"], "FFʼN": ["FFʼN", "ﬀŉ", "ffŉ"]}


def test_json_field_names_unicode_upper_case(prod):
    """A JSON field matches its column exactly, else through toUpperCase (KsqlJsonDeserializer.java:
    301-306): "straße" → STRASSE, "ǆx" → ǄX, Greek final sigma, "ﬀŉ" → FFʼN (length-changing maps),
    a supplementary-plane letter; "cafe" is not "CAFÉ".  Checked against tests/serde_ref.py, whose
    matching is Python's str.upper() (the same unconditional Unicode mapping)."""
    rng = random.Random(31)
    vals = []
    for i in range(300):
        parts = []
        for name, t, _ in UNI_FIELDS:
            if rng.random() < 0.15:
                continue
            v = "%.3f" % rng.uniform(-9, 9) if t == "DOUBLE" else str(rng.randrange(-1000, 1000))
            parts.append('%s: %s' % (json.dumps(rng.choice(UNI_NAMES[name]), ensure_ascii=rng.random() < 0.3), v))
        rng.shuffle(parts)
        vals.append(("{" + ", ".join(parts) + "}").encode())
    keys = [struct.pack(">q", i) for i in range(len(vals))]
    out_types = ["INT64", "INT64", "INT64", "DOUBLE", "INT64", "INT32"]
    sd = abi.SerdeHandle(prod, "JSON", UNI_FIELDS, key_type="INT64")
    d, nerr = sd.decode(np.arange(len(vals), dtype=np.int64), keys, vals)
    exp, experr = serde_ref.decode("JSON", UNI_FIELDS, "INT64", keys, vals)
    assert nerr == experr == 0
    got = sd.columns(d, out_types)
    _check(got, exp, UNI_FIELDS, out_types)
    assert got["valid"][0].any() and not all(got["valid"][3])  # matches through upper case; "cafe" misses
    sd.close()

