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
    assert lib.dll.khip_abi_version() == abi.ABI_VERSION == 4
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
