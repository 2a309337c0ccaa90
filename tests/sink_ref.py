"""CPU restatement of the sink-side serializers (TEST INFRASTRUCTURE: the checker of
khip_sink_*, never shipped, never on a product path).

What the reference does when an aggregate's changelog row becomes a Kafka record:
  key   GenericKeySerDe (ksqldb-serde/.../serde/GenericKeySerDe.java:95-117): the inner key
        serializer, then for a windowed table Kafka Streams' TimeWindowedSerializer (inner key
        bytes ++ 8-byte big-endian window start) or SessionWindowedSerializer / SessionKeySchema
        (inner key ++ 8-byte big-endian end ++ 8-byte big-endian start).
        KAFKA key format (kafka/KafkaSerdeFactory.java:42-46): INT 4-byte / BIGINT 8-byte big
        endian, DOUBLE 8-byte IEEE big endian, STRING UTF-8 — one column only.
        JSON: one key column unwrapped (the bare JSON value), several as an object in schema order.
        DELIMITED: the CSV record of the key columns.
  value GenericRowSerDe: JSON through Kafka Connect's JsonConverter (json/KsqlJsonSerdeFactory.java:
        158-161, schemas off) → Jackson: compact object, fields in schema order, a single field
        wrapped; DELIMITED through KsqlDelimitedSerializer (delimited/KsqlDelimitedSerializer.java:
        59-71: commons-csv printRecord, the trailing CRLF cut off, null = empty field); KAFKA: the
        one column's primitive bytes.  A tombstone (the row left the table) is a null value.
Numbers print as Long.toString / Double.toString.  Double.toString here is the JDK 19+
specification (shortest decimal that rounds back, Schubfach; computerized scientific notation
outside [1e-3, 1e7)); JDK <= 18's FloatingDecimal prints a longer digit string for a few values
(e.g. 2.82879384806159E17) — those values are parity-unpinned.  Non-finite doubles follow
Jackson's default QUOTE_NON_NUMERIC_NUMBERS ("NaN", "Infinity", "-Infinity" as JSON strings).
"""
import json
import math
import os
import struct
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
import gen_dtoa  # noqa: E402

M64 = (1 << 64) - 1
MASK_63 = (1 << 63) - 1
P, Q_MIN, C_MIN, C_TINY, H = 53, -1074, 1 << 52, 3, 17
K_MIN = gen_dtoa.K_MIN
_G = gen_dtoa.table()


def flog10pow2(e):
    return (e * 661_971_961_083) >> 41


def flog10_three_quarters_pow2(e):
    return (e * 661_971_961_083 - 274_743_187_321) >> 41


def _mulhi(a, b):
    return (a * b) >> 64  # operands are non-negative here


def _rop(g1, g0, cp):
    x1 = _mulhi(g0, cp)
    y0 = (g1 * cp) & M64
    y1 = _mulhi(g1, cp)
    z = ((y0 >> 1) + x1) & M64
    vbp = (y1 + (z >> 63)) & M64
    return vbp | ((((z & MASK_63) + MASK_63) & M64) >> 63)


def _to_decimal(q, c, dk):
    """(f, e): the shortest decimal f * 10^e that rounds to c * 2^q (Schubfach)."""
    out = c & 1
    cb = c << 2
    cbr = cb + 2
    if c != C_MIN or q == Q_MIN:
        cbl = cb - 2
        k = flog10pow2(q)
    else:
        cbl = cb - 1
        k = flog10_three_quarters_pow2(q)
    h = q + gen_dtoa.flog2pow10(-k) + 2
    g1, g0 = _G[k - K_MIN]  # 10^-k
    vb = _rop(g1, g0, cb << h)
    vbl = _rop(g1, g0, cbl << h)
    vbr = _rop(g1, g0, cbr << h)
    s = vb >> 2
    if s >= 100:
        sp10 = 10 * _mulhi(s, 115_292_150_460_684_698 << 4)
        tp10 = sp10 + 10
        upin = vbl + out <= sp10 << 2
        wpin = (tp10 << 2) + out <= vbr
        if upin != wpin:
            return (sp10 if upin else tp10), k
    t = s + 1
    uin = vbl + out <= s << 2
    win = (t << 2) + out <= vbr
    if uin != win:
        return (s if uin else t), k + dk
    cmp = vb - ((s + t) << 1)
    return (s if cmp < 0 or (cmp == 0 and (s & 1) == 0) else t), k + dk


def _chars(f, e):
    """Java's layout of f * 10^e (DoubleToDecimal.toChars)."""
    d = str(f)
    e10 = e + len(d)  # value = 0.d * 10^e10
    d = d.rstrip("0") or "0"
    if 0 < e10 <= 7:
        ip = d[:e10].ljust(e10, "0")
        fp = d[e10:] or "0"
        return ip + "." + fp
    if -3 < e10 <= 0:
        return "0." + "0" * (-e10) + d
    return d[0] + "." + (d[1:] or "0") + "E" + str(e10 - 1)


def java_double_str(v):
    """java.lang.Double.toString(v) (JDK 19+)."""
    bits = struct.unpack("<Q", struct.pack("<d", v))[0]
    t = bits & ((1 << 52) - 1)
    bq = (bits >> 52) & 0x7FF
    sign = "-" if bits >> 63 else ""
    if bq < 0x7FF:
        if bq != 0:
            mq = -Q_MIN + 1 - bq
            c = C_MIN | t
            if 0 < mq < P:
                f = c >> mq
                if f << mq == c:
                    return sign + _chars(f, 0)
            return sign + _chars(*_to_decimal(-mq, c, 0))
        if t != 0:
            return sign + _chars(*(_to_decimal(Q_MIN, 10 * t, -1) if t < C_TINY else _to_decimal(Q_MIN, t, 0)))
        return sign + "0.0"
    if t != 0:
        return "NaN"
    return sign + "Infinity"


# ------------------------------------------------------------------------------ encoders

def json_string(s):
    """Jackson's string escaping: quote, backslash, control characters; UTF-8 otherwise as is."""
    out = ['"']
    short = {'"': '\\"', "\\": "\\\\", "\n": "\\n", "\r": "\\r", "\t": "\\t", "\b": "\\b", "\f": "\\f"}
    for ch in s:
        if ch in short:
            out.append(short[ch])
        elif ord(ch) < 0x20:
            out.append("\\u%04X" % ord(ch))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def json_value(typ, v):
    if v is None:
        return "null"
    if typ in ("INT32", "INT64"):
        return str(int(v))
    if typ == "DOUBLE":
        if math.isnan(v) or math.isinf(v):
            return '"' + java_double_str(v) + '"'
        return java_double_str(float(v))
    if typ == "STRING":
        return json_string(v)
    raise ValueError(typ)


def csv_text(t, first, delim=","):
    """commons-csv 1.4 CSVFormat.printAndQuote, QuoteMode.MINIMAL (the delimited serializer's
    CSVPrinter): quote an empty first field, a first field starting outside RFC 4180 TEXTDATA, any
    field starting with a character <= '#', holding CR / LF / quote / delimiter, or ending <= ' '."""
    if t == "":
        quote = first
    else:
        c = ord(t[0])
        if first and (c < 0x20 or 0x21 < c < 0x23 or 0x2B < c < 0x2D or c > 0x7E):
            quote = True
        elif c <= ord("#"):
            quote = True
        else:
            quote = any(x in t for x in ("\n", "\r", '"', delim)) or ord(t[-1]) <= 0x20
    return '"' + t.replace('"', '""') + '"' if quote else t


def csv_field(typ, v, first=True, delim=","):
    if v is None:
        return ""  # CSVPrinter.print(null) with no null string: nothing, unquoted
    if typ in ("INT32", "INT64"):
        return csv_text(str(int(v)), first, delim)
    if typ == "DOUBLE":
        return csv_text(java_double_str(float(v)), first, delim)
    if typ == "STRING":
        return csv_text(v, first, delim)
    raise ValueError(typ)


def kafka_bytes(typ, v):
    if v is None:
        return None
    if typ == "INT32":
        return struct.pack(">i", int(v))
    if typ == "INT64":
        return struct.pack(">q", int(v))
    if typ == "DOUBLE":
        return struct.pack(">d", float(v))
    if typ == "STRING":
        return v.encode()
    raise ValueError(typ)


def encode_key(fmt, cols, vals):
    """cols: [(name, type)], vals: python values (never null: a null group-by value drops the row)."""
    if fmt == "KAFKA":
        assert len(cols) == 1
        return kafka_bytes(cols[0][1], vals[0])
    if fmt == "JSON":
        if len(cols) == 1:
            return json_value(cols[0][1], vals[0]).encode()
        return ("{" + ",".join(json_string(n) + ":" + json_value(t, v) for (n, t), v in zip(cols, vals)) + "}").encode()
    if fmt == "DELIMITED":
        return ",".join(csv_field(t, v, i == 0) for i, ((n, t), v) in enumerate(zip(cols, vals))).encode()
    raise ValueError(fmt)


def window_suffix(kind, ws, we):
    if kind in ("TUMBLING", "HOPPING"):
        return struct.pack(">q", ws)
    if kind == "SESSION":
        return struct.pack(">qq", we, ws)
    return b""


def encode_value(fmt, cols, vals, tombstone=False):
    """cols: [(name, type)]; returns bytes or None (null value)."""
    if tombstone:
        return None
    if fmt == "KAFKA":
        assert len(cols) == 1
        return kafka_bytes(cols[0][1], vals[0])
    if fmt == "JSON":
        return ("{" + ",".join(json_string(n) + ":" + json_value(t, v) for (n, t), v in zip(cols, vals)) + "}").encode()
    if fmt == "DELIMITED":
        return ",".join(csv_field(t, v, i == 0) for i, ((n, t), v) in enumerate(zip(cols, vals))).encode()
    raise ValueError(fmt)


def python_java_str(v):
    """Independent check of java_double_str from Python's repr (shortest round trip, closest):
    the same digits except where JDK 19 prefers a closer 2-digit decimal to a 1-digit one (only
    the smallest subnormals)."""
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "-Infinity" if v < 0 else "Infinity"
    sign = "-" if math.copysign(1.0, v) < 0 else ""
    r = repr(abs(v))
    if "e" in r:
        mant, exp = r.split("e")
        exp = int(exp)
    else:
        mant, exp = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # value = 0.digits * 10^e10
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    e10 = len(ip) - lead_zeros + exp
    if not digits:
        return sign + "0.0"
    return sign + _chars(int(digits), e10 - len(digits))


if __name__ == "__main__":
    for v in (1.0, 0.1, 1e7, 1e-3, 9.999e-4, 123456.789, 2.82879384806159e17, 5e-324, 1.7976931348623157e308):
        print(v, java_double_str(v), python_java_str(v))
    print(json.dumps(None))
