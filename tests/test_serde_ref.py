"""The CPU deserializer restatement (tests/serde_ref.py) on known answers: Jackson's BigDecimal
intValue() / longValue() for JSON float tokens into INT / BIGINT columns
(KsqlJsonDeserializer.java:68-70, JsonSerdeUtils.java:95-121)."""
import serde_ref


def test_bigdecimal_low_bits():
    b = serde_ref.bigdec_low_bits
    assert b("3000000000.5", 32) == 3000000000 - (1 << 32)
    assert b("1e20", 64) == 10 ** 20 - 5 * (1 << 64)
    assert b("-1e20", 64) == -(10 ** 20 - 5 * (1 << 64))
    assert b("9007199254740993.7", 64) == 9007199254740993  # a double would give ...992
    assert b("1e400", 32) == 0 and b("1e400", 64) == 0  # 10^400 is a multiple of 2^64
    assert b("-2.9", 32) == -2 and b("12.5e-1", 64) == 1 and b("0.5e1", 64) == 5 and b("1e-5", 64) == 0


def test_json_decimal_tokens_decode():
    fields = [("A", "INT32", 0), ("B", "INT64", 1), ("C", "DOUBLE", 2)]
    out, err = serde_ref.decode("JSON", fields, "INT64", [b"\0" * 8],
                                [b'{"A": 3000000000.5, "B": 1e20, "C": 3000000000.5}'])
    assert err == 0
    row = out[0][3]
    assert row == {"A": -1294967296, "B": 7766279631452241920, "C": 3000000000.5}
