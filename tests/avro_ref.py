"""AVRO values for the deserializer tests (test infrastructure): a Confluent-wire-format encoder
of Avro records and the CPU restatement of the decode the reference performs (the checker of
khip_serde_decode's AVRO path).

Reference path (ksqldb-serde): KsqlAvroSerdeFactory.createConnectDeserializer
(avro/KsqlAvroSerdeFactory.java:130-144) → Confluent's AvroConverter / KafkaAvroDeserializer →
connect/ConnectDataTranslator.toKsqlRow (:50-57) → toKsqlStruct (:290-318) / toKsqlValue
(:172-230) / validateSchema (:123-146).
  * wire format: magic byte 0, 4-byte big-endian schema id, then the Avro binary encoding of the
    writer schema's record (Avro 1.11 specification, "Binary Encoding": zig-zag varint int / long,
    at most 5 / 10 bytes; little-endian IEEE float / double; long length + bytes for string /
    bytes; a union is its branch index (an int) then the branch's value; one byte for boolean,
    true iff it is 1).  Bytes after the record are ignored.
  * a writer field lands in the ksql column of the same name, else of the upper-cased name; a
    writer type the column's type does not accept fails the record (BIGINT <- int / long,
    INT <- int, DOUBLE <- float / double, STRING <- any primitive but bytes); ksql columns with no
    writer field are NULL.
The writer schema is [(name, avro type, union)], union 0 = plain, 1 = ["null", T], 2 = [T, "null"].
ksqlDB's own AVRO schemas (what the QTT harness serializes test inputs with) make every column an
optional field: ["null", T] with the column's name.
"""
import struct

KSQL_TO_AVRO = {"INT32": "int", "INT64": "long", "DOUBLE": "double", "STRING": "string"}


class Err(Exception):
    pass


def ksql_writer_schema(fields):
    """The schema ksqlDB registers for a value schema [(name, ksql type, out)]: all optional."""
    return [(name, KSQL_TO_AVRO[t], 1) for name, t, _ in fields]


def _zz(v, bits):
    return ((v << 1) ^ (v >> (bits - 1))) & ((1 << bits) - 1)


def _varint(u):
    out = bytearray()
    while True:
        b = u & 0x7F
        u >>= 7
        if u:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def encode_value(atype, v):
    if atype == "boolean":
        return b"\x01" if v else b"\x00"
    if atype == "int":
        return _varint(_zz(int(v), 32))
    if atype == "long":
        return _varint(_zz(int(v), 64))
    if atype == "float":
        return struct.pack("<f", float(v))
    if atype == "double":
        return struct.pack("<d", float(v))
    if atype in ("string", "bytes"):
        b = v.encode() if isinstance(v, str) else bytes(v)
        return _varint(_zz(len(b), 64)) + b
    raise ValueError(atype)


def encode(schema, record, schema_id=1):
    """record: {name: python value or None}; Confluent wire format bytes."""
    out = bytearray(b"\x00" + struct.pack(">i", schema_id))
    for name, atype, union in schema:
        v = record.get(name)
        if union:
            null_branch = union - 1
            if v is None:
                out += _varint(_zz(null_branch, 32))
                continue
            out += _varint(_zz(1 - null_branch, 32))
        elif v is None:
            raise ValueError("null in a plain field " + name)
        out += encode_value(atype, v)
    return bytes(out)


def _read_varint(buf, j, maxb):
    v = 0
    for k in range(maxb):
        if j >= len(buf):
            raise Err("EOF")
        b = buf[j]
        j += 1
        v |= (b & 0x7F) << (7 * k)
        if not b & 0x80:
            return v, j
    raise Err("invalid varint")


def _unzz(u, bits):
    u &= (1 << bits) - 1
    v = (u >> 1) ^ -(u & 1)
    return v


ACCEPTS = {"INT64": ("int", "long"), "INT32": ("int",), "DOUBLE": ("float", "double"),
           "STRING": ("boolean", "int", "long", "float", "double", "string")}


def decode_value(fields, schema, raw, schema_id=-1):
    """The reference's row for one record value (raw bytes), as {column: value or None}; Err when
    the record fails to deserialize.  fields: the ksql value schema [(name, type, out)]."""
    if raw is None:
        return None
    names = [n for n, _, _ in fields]
    mapping = []
    for wn, at, un in schema:
        f = names.index(wn) if wn in names else (names.index(wn.upper()) if wn.upper() in names else -1)
        mapping.append(f)
        if f >= 0 and at not in ACCEPTS[fields[f][1]]:
            raise Err("type mismatch " + wn)
    if len(raw) < 5 or raw[0] != 0:
        raise Err("Unknown magic byte!")
    if schema_id >= 0 and struct.unpack(">i", raw[1:5])[0] != schema_id:
        raise Err("schema id")
    out = {n: None for n in names}
    j = 5
    for (wn, at, un), f in zip(schema, mapping):
        if un:
            u, j = _read_varint(raw, j, 5)
            idx = _unzz(u, 32)
            if idx not in (0, 1):
                raise Err("union index")
            if idx == un - 1:
                if f >= 0:
                    out[names[f]] = None
                continue
        if at == "boolean":
            if j >= len(raw):
                raise Err("EOF")
            v = raw[j] == 1
            j += 1
        elif at == "int":
            u, j = _read_varint(raw, j, 5)
            v = _unzz(u, 32)
        elif at == "long":
            u, j = _read_varint(raw, j, 10)
            v = _unzz(u, 64)
        elif at == "float":
            if len(raw) - j < 4:
                raise Err("EOF")
            v = struct.unpack("<f", raw[j:j + 4])[0]
            j += 4
        elif at == "double":
            if len(raw) - j < 8:
                raise Err("EOF")
            v = struct.unpack("<d", raw[j:j + 8])[0]
            j += 8
        else:
            u, j = _read_varint(raw, j, 10)
            ln = _unzz(u, 64)
            if ln < 0 or ln > len(raw) - j:
                raise Err("string length")
            v = bytes(raw[j:j + ln])
            j += ln
        if f < 0:
            continue
        t = fields[f][1]
        out[names[f]] = "s" if t == "STRING" else (float(v) if t == "DOUBLE" else int(v))
    return out


def decode(fields, schema, key_type, keys, values, schema_id=-1):
    """Expected khip_serde_decode result (serde_ref.decode's shape): per record (key_valid, key,
    row_valid, {col: value}), and the error count."""
    import serde_ref
    out, errors = [], 0
    for k, v in zip(keys, values):
        try:
            key = None if k is None else serde_ref.decode_key(key_type, k)
            row = decode_value(fields, schema, v, schema_id)
            out.append((k is not None, key, v is not None, row))
        except (Err, serde_ref.Err):
            errors += 1
            out.append((False, None, False, None))
    return out, errors
