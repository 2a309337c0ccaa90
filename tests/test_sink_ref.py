"""The sink serializers' CPU restatement (tests/sink_ref.py) pinned independently:
Double.toString digits against Python's shortest round-trip repr (which agrees with the JDK 19+
specification except where Java prefers a closer two-digit decimal for the smallest subnormals,
e.g. Double.MIN_VALUE = "4.9E-324"), the layout switches at 1e-3 and 1e7, and the key / value
formats on hand-written examples taken from the QTT expected records."""
import math
import random
import struct

import sink_ref


def test_schubfach_matches_shortest_repr():
    rng = random.Random(3)
    n = bad = 0
    for _ in range(60000):
        v = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0]
        if math.isnan(v) or abs(v) < 1e-320:
            continue
        n += 1
        bad += sink_ref.java_double_str(v) != sink_ref.python_java_str(v)
    for _ in range(60000):
        v = float("%de%d" % (rng.randint(1, 10 ** rng.randint(1, 17)), rng.randint(-300, 300)))
        n += 1
        bad += sink_ref.java_double_str(v) != sink_ref.python_java_str(v)
    assert n > 100000 and bad == 0


def test_java_layout_examples():
    cases = [(1.0, "1.0"), (-0.0, "-0.0"), (0.0, "0.0"), (100.0, "100.0")]
    cases += list({0.1: "0.1", 0.001: "0.001",
             9.999e-4: "9.999E-4", 1e7: "1.0E7", 9999999.0: "9999999.0", 1.5e-7: "1.5E-7",
             123456.789: "123456.789", 1.0 / 3: "0.3333333333333333", 2.0 ** 63: "9.223372036854776E18",
             5e-324: "4.9E-324", 1.7976931348623157e308: "1.7976931348623157E308",
             float("nan"): "NaN", float("inf"): "Infinity", float("-inf"): "-Infinity"}.items())
    for v, s in cases:
        assert sink_ref.java_double_str(v) == s, (v, sink_ref.java_double_str(v), s)


def test_formats():
    assert sink_ref.encode_key("KAFKA", [("K", "INT64")], [1]) == b"\0" * 7 + b"\1"
    assert sink_ref.encode_key("KAFKA", [("K", "INT32")], [-1]) == b"\xff" * 4
    assert sink_ref.encode_key("JSON", [("K", "INT32"), ("K2", "INT32")], [1, 2]) == b'{"K":1,"K2":2}'
    assert sink_ref.encode_key("JSON", [("K", "STRING")], ['a"b']) == b'"a\\"b"'
    assert sink_ref.encode_key("DELIMITED", [("A", "STRING"), ("B", "INT32")], ["x,y", 3]) == b'"x,y",3'
    assert sink_ref.window_suffix("TUMBLING", 5, 10) == struct.pack(">q", 5)
    assert sink_ref.window_suffix("SESSION", 5, 10) == struct.pack(">qq", 10, 5)
    assert sink_ref.encode_value("JSON", [("COUNT", "INT64"), ("A", "DOUBLE")], [3, None]) == b'{"COUNT":3,"A":null}'
    assert sink_ref.encode_value("JSON", [("A", "DOUBLE")], [float("nan")]) == b'{"A":"NaN"}'
    assert sink_ref.encode_value("DELIMITED", [("A", "INT64"), ("B", "DOUBLE")], [None, 2.5]) == b",2.5"
    assert sink_ref.encode_value("DELIMITED", [("A", "INT64")], [1], tombstone=True) is None
    # commons-csv 1.4 MINIMAL: first-field RFC 4180 TEXTDATA rule, leading <= '#', trailing <= ' '
    assert sink_ref.csv_field("STRING", "") == '""'
    assert sink_ref.csv_field("STRING", "#x") == '"#x"'
    assert sink_ref.csv_field("STRING", "x ") == '"x "'
    assert sink_ref.csv_field("STRING", 'a"b') == '"a""b"'
