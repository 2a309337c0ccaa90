"""Host-side checks of the C-ABI library (no GPU needed): it loads, exports every
symbol include/ksqldb_hip.h declares, and rejects invalid plan-time descriptors
before touching the device (the reference raises KsqlException at plan time)."""
import ctypes as C
import os
import re

import pytest

from ksql_amd import abi

HEADER = os.path.join(abi.REPO, "include", "ksqldb_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(khip_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ["khip_agg_create", "khip_agg_push", "khip_agg_snapshot", "khip_agg_destroy", "khip_table_create",
              "khip_table_upsert", "khip_table_probe", "khip_table_destroy", "khip_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = abi.load_product()
    missing = [s for s in declared_symbols() if not hasattr(lib.dll, s)]
    assert missing == []


def test_version_and_target():
    lib = abi.load_product()
    assert lib.dll.khip_abi_version() == abi.ABI_VERSION == 8
    assert lib.dll.khip_build_target() == b"gfx950"


def test_library_is_gfx950_code_object():
    """Every offload bundle in the library targets gfx950 (one code object per HIP source),
    and no other GPU target (another gfx, or a CUDA sm_) is embedded."""
    data = open(abi.PRODUCT_LIB, "rb").read()
    targets = re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", data)
    assert len(targets) >= 4, targets  # agg, agg_part, join, shuffle
    assert set(targets) == {b"gfx950"}
    assert re.search(rb"nvptx|sm_[0-9]{2}\b", data) is None


@pytest.mark.parametrize("bad", [
    dict(window_kind=7),
    dict(window_kind="TUMBLING", size_ms=0),
    dict(window_kind="HOPPING", size_ms=1000, advance_ms=2000),
    dict(window_kind="NONE", col_types=["INT64"], aggs=[("SUM", 3)]),
    dict(window_kind="NONE", aggs=[(9, -1)]),
    dict(window_kind="NONE", key_type=5),
])
def test_invalid_descriptors_rejected_before_device(bad):
    lib = abi.load_product()
    desc = abi.make_agg_desc(**bad)
    h = C.c_void_p()
    st = lib.agg_create(C.byref(desc), C.byref(h))
    assert st == -1  # KHIP_E_INVALID
    assert lib.dll.khip_last_error()


def test_unsupported_fanout_rejected():
    lib = abi.load_product()
    desc = abi.make_agg_desc(window_kind="HOPPING", size_ms=3_600_000, advance_ms=1)
    h = C.c_void_p()
    assert lib.agg_create(C.byref(desc), C.byref(h)) == -4  # KHIP_E_UNSUPPORTED → CPU builder


def test_result_types():
    lib = abi.load_product()
    desc = abi.make_agg_desc(col_types=["INT32", "DOUBLE"],
                             aggs=[("COUNT_STAR", -1), ("SUM", 0), ("AVG", 0), ("MAX", 1), ("COUNT", 1)])
    out = []
    for i in range(5):
        t = C.c_int32()
        assert lib.agg_result_type(C.byref(desc), i, C.byref(t)) == 0
        out.append(t.value)
    assert out == [1, 0, 2, 2, 1]
    assert abi.result_types(desc) == out


def test_comm_argument_validation_cpu():
    """khip_comm_* reject bad arguments before touching a device or RCCL (no GPU needed)."""
    lib = abi.load_product()
    idb = (C.c_uint8 * abi.COMM_ID_BYTES)()
    h = C.c_void_p()
    assert lib.comm_init(0, 0, idb, 0, C.byref(h)) == -1      # no ranks
    assert lib.comm_init(2, 2, idb, 0, C.byref(h)) == -1      # rank outside the world
    assert lib.comm_init(2, -1, idb, 0, C.byref(h)) == -1
    assert lib.comm_init(2, 0, None, 0, C.byref(h)) == -1     # no unique id
    assert lib.comm_init(2, 0, idb, 0, None) == -1
    assert b"communicator" in lib.dll.khip_last_error()
    sc = (abi.i64 * 2)(1, 2)
    assert lib.comm_exchange_counts(None, sc, sc) == -1
    assert lib.comm_alltoall(None, None, sc, None, 0, sc, 3) == -1
    assert lib.comm_destroy(None) == 0


def test_sink_argument_validation_cpu():
    """khip_sink_create rejects descriptors the reference would not build (no GPU needed)."""
    lib = abi.load_product()
    with pytest.raises(abi.KsqlHipError):
        abi.SinkHandle(lib, "KAFKA", [("A", "INT32"), ("B", "INT32")], "JSON", [])  # KAFKA key: one column
    with pytest.raises(abi.KsqlHipError):
        abi.SinkHandle(lib, "JSON", [("A", "INT32")], "KAFKA", [("X", "INT64", 0), ("Y", "INT64", 1)])
    with pytest.raises(abi.KsqlHipError):
        abi.SinkHandle(lib, "AVRO", [("A", "INT32")], "JSON", [])
    with pytest.raises(abi.KsqlHipError):
        abi.SinkHandle(lib, "JSON", [("A", "INT32")], "JSON", [("WS", "DOUBLE", "WS")])  # WINDOWSTART is BIGINT
