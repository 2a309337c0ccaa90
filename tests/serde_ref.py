"""CPU restatement of ksqlDB's deserializers for the types on the hot path (test infrastructure,
small batches): the checker of khip_serde_decode.

  KAFKA      ksqldb-serde/.../kafka/KafkaSerdeFactory.java:42-46 (Kafka's Integer / Long / Double /
             String deserializers: big-endian, exact lengths)
  DELIMITED  ksqldb-serde/.../delimited/KsqlDelimitedDeserializer.java (Apache Commons CSV
             CSVFormat.DEFAULT with the delimiter: a quote starts an encapsulated token only at the
             token start, "" escapes a quote, the first record only, empty field = NULL,
             Integer.parseInt / Long.parseLong / Double.parseDouble)
  JSON       ksqldb-serde/.../json/KsqlJsonDeserializer.java:149-300 + JsonSerdeUtils.java:95-136
             (Jackson tree: the field of the same name, else the upper-cased one; intValue() /
             asLong() / doubleValue() of numbers, the Java parsers of strings; booleans, objects
             and arrays are coercion errors for numbers).  The mapper enables
             USE_BIG_DECIMAL_FOR_FLOATS (KsqlJsonDeserializer.java:68-70): a token with a fraction or
             an exponent is a BigDecimal, whose intValue() / longValue() truncate toward zero and
             keep the low 32 / 64 bits of the integer part (no saturation, no rounding through a
             double); doubleValue() is the correctly rounded double.
Python's float() is correctly rounded like Double.parseDouble for decimal text.
"""
import decimal
import json
import math
import re
import struct


class JDec(str):
    """A JSON number token with a fraction or an exponent (Jackson: BigDecimal), kept as text."""


def bigdec_low_bits(tok, bits):
    """BigDecimal(tok).intValue() (bits 32) / longValue() (bits 64): integer part, low bits."""
    d = decimal.Decimal(tok)  # exact: the constructor does not round
    sign, digits, exp = d.as_tuple()
    if exp >= 64:  # 10^exp is a multiple of 2^64
        v = 0
    elif exp >= 0:
        v = int("".join(map(str, digits)) or "0") * 10 ** exp
    else:
        keep = len(digits) + exp
        v = int("".join(map(str, digits[:keep]))) if keep > 0 else 0
    return wrap(-v if sign else v, bits)

INT_RE = re.compile(r"^[+-]?[0-9]+$")
DBL_RE = re.compile(r"^[+-]?(NaN|Infinity|([0-9]+\.?[0-9]*|\.[0-9]+)([eE][+-]?[0-9]+)?[fFdD]?)$")


class Err(Exception):
    pass


def parse_int(s, bits):
    if not INT_RE.match(s):
        raise Err(s)
    v = int(s)
    if not -(1 << (bits - 1)) <= v < (1 << (bits - 1)):
        raise Err(s)
    return v


def parse_double(s):
    t = s.strip(" \t\n\r\x0b\x0c\x00\x01\x02\x03\x04\x05\x06\x07\x08\x0e\x0f\x10\x11\x12\x13\x14\x15\x16\x17"
                "\x18\x19\x1a\x1b\x1c\x1d\x1e\x1f")
    if not DBL_RE.match(t):
        raise Err(s)
    core = t.rstrip("fFdD") if t[-1] in "fFdD" and "Infinity" not in t else t
    if "NaN" in core:
        return float("nan")
    if "Infinity" in core:
        return float("-inf") if core.startswith("-") else float("inf")
    return float(core)


def java_d2i(d, bits):
    if math.isnan(d):
        return 0
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    if d >= hi:
        return hi
    if d <= lo:
        return lo
    return int(d)


def wrap(v, bits):
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def coerce_text(s, t):
    if t == "INT32":
        return parse_int(s, 32)
    if t == "INT64":
        return parse_int(s, 64)
    return parse_double(s)


def csv_first_record(text, delim):
    """Commons CSV DEFAULT lexer, first record: list of field strings (None never occurs)."""
    fields, i, n = [], 0, len(text)
    if n == 0:
        raise Err("no fields")
    while True:
        if i < n and text[i] == '"':
            j, buf = i + 1, []
            while True:
                if j >= n:
                    raise Err("eof in quotes")
                if text[j] == '"':
                    if j + 1 < n and text[j + 1] == '"':
                        buf.append('"')
                        j += 2
                        continue
                    break
                buf.append(text[j])
                j += 1
            j += 1
            if j < n and text[j] not in (delim, "\n", "\r"):
                raise Err("char after quote")
            fields.append(("".join(buf), True))
            i = j
        else:
            j = i
            while j < n and text[j] not in (delim, "\n", "\r"):
                j += 1
            fields.append((text[i:j], False))
            i = j
        if i < n and text[i] == delim:
            i += 1
            continue
        return fields


def decode_value(fmt, fields, raw, delim=","):
    """→ dict name → python value (None = NULL), or raises Err."""
    types = [t for _, t, _ in fields]
    if fmt == "KAFKA":
        (name, t, _), = fields
        if t == "INT32":
            if len(raw) != 4:
                raise Err("len")
            return {name: struct.unpack(">i", raw)[0]}
        if t == "INT64":
            if len(raw) != 8:
                raise Err("len")
            return {name: struct.unpack(">q", raw)[0]}
        if t == "DOUBLE":
            if len(raw) != 8:
                raise Err("len")
            return {name: struct.unpack(">d", raw)[0]}
        return {name: raw.decode("utf-8", "replace")}
    if fmt == "DELIMITED":
        recs = csv_first_record(raw.decode("utf-8", "replace"), delim)
        if len(recs) != len(fields):
            raise Err("arity")
        out = {}
        for (name, t, _), (v, quoted) in zip(fields, recs):
            if v == "":
                out[name] = None
            elif t == "STRING":
                out[name] = v
            else:
                out[name] = coerce_text(v, t)
        return out
    # JSON (Jackson tree; trailing content ignored; NaN / Infinity literals rejected)
    text = raw.decode("utf-8", "replace").lstrip(" \t\n\r")

    def bad_const(c):
        raise Err(c)
    pairs_seen = []

    def hook(pairs):
        pairs_seen.append(pairs)
        return pairs
    try:
        obj, _ = json.JSONDecoder(object_pairs_hook=hook, parse_constant=bad_const,
                                  parse_float=JDec).raw_decode(text)
    except ValueError as e:
        raise Err(str(e))
    if not isinstance(obj, list) or not pairs_seen or obj is not pairs_seen[-1]:
        raise Err("not an object")
    exact, upper = {}, {}
    for k, v in obj:
        exact[k] = v
        upper[k.upper()] = v
    out = {}
    for name, t, _ in fields:
        v = exact[name] if name in exact else upper.get(name)
        if v is None:
            out[name] = None
            continue
        if t == "STRING":
            out[name] = v
            continue
        if isinstance(v, bool) or isinstance(v, list):  # booleans, objects (pair lists), arrays
            raise Err("coercion")
        if isinstance(v, JDec):  # BigDecimal
            out[name] = bigdec_low_bits(v, 32) if t == "INT32" else (bigdec_low_bits(v, 64) if t == "INT64"
                                                                      else float(v))
        elif isinstance(v, str):
            out[name] = coerce_text(v, t)
        elif isinstance(v, int):
            out[name] = wrap(v, 32) if t == "INT32" else (wrap(v, 64) if t == "INT64" else float(v))
        else:
            raise Err("unexpected JSON value")
    return out


def decode_key(key_type, raw):
    if key_type == "INT64":
        if len(raw) != 8:
            raise Err("key len")
        return struct.unpack(">q", raw)[0]
    if key_type == "INT32":
        if len(raw) != 4:
            raise Err("key len")
        return struct.unpack(">i", raw)[0]
    return raw


def decode(fmt, fields, key_type, keys, values, delim=","):
    """Expected khip_serde_decode result: per record (key_valid, key, row_valid, {col: value})."""
    out = []
    errors = 0
    for k, v in zip(keys, values):
        try:
            key = None if k is None else decode_key(key_type, k)
            row = None if v is None else decode_value(fmt, fields, v, delim)
            out.append((k is not None, key, v is not None, row))
        except Err:
            errors += 1
            out.append((False, None, False, None))
    return out, errors
