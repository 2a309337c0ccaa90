"""ctypes mirror of include/ksqldb_hip.h.

The same structs drive two libraries with identical signatures:
  * ksql_amd/libksqldb_hip.so  — the product (HIP kernels, prefix ``khip_``);
  * oracle/liboracle.so        — the CPU restatement used only by tests/bench as
                                  the parity checker (prefix ``oracle_``).
Nothing here routes product calls to the oracle: ``load_product()`` fails loudly
if the HIP library is missing.
"""
import ctypes as C
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# KSQL_AMD_LIB_VARIANT=tune loads the tuning build (same HIP kernels, KHIP_* knobs read from the
# environment; ksql_amd/Makefile TUNING=1) for GPU parameter sweeps.  Both are the HIP library.
# (any other name V loads libksqldb_hip_V.so: a build kept for an A/B inside one GPU call).
_VARIANT = os.environ.get("KSQL_AMD_LIB_VARIANT", "")
PRODUCT_LIB = os.path.join(REPO, "ksql_amd", "libksqldb_hip_%s.so" % _VARIANT if _VARIANT else "libksqldb_hip.so")
ORACLE_LIB = os.path.join(REPO, "oracle", "liboracle.so")

ABI_VERSION = 8  # include/ksqldb_hip.h KHIP_ABI_VERSION the structs below mirror
KHIP_OK = 0
KHIP_E_BUFFER = -5

WINDOW = {"NONE": 0, "TUMBLING": 1, "HOPPING": 2, "SESSION": 3}
KEY = {"INT64": 0, "UTF8": 1}
TYPE = {"INT32": 0, "INT64": 1, "DOUBLE": 2}
AGG = {"COUNT_STAR": 0, "COUNT": 1, "SUM": 2, "MIN": 3, "MAX": 4, "AVG": 5}
OP = {"GT": 0, "GE": 1, "LT": 2, "LE": 3, "EQ": 4, "NE": 5}
JOIN = {"LEFT": 0, "INNER": 1}
MEM_HOST, MEM_DEVICE = 0, 1
FLAG_PROFILE = 1
FLAG_ENGINE_ATOMIC = 2
FLAG_PART_CLAIM = 4
FLAG_CHANGELOG = 8
FLAG_TABLE_SOURCE = 16
RETENTION_DEFAULT = -1
EMIT = {"CHANGES": 0, "FINAL": 1}
TIME = {"TASK": 0, "PARTITION": 1, "SUPPLIED": 2}  # ABI 5 stream-time domains
SHUFFLE_STREAM_TIME = 1  # ABI 7 khip_shuffle_desc.flags
NP_TYPE = {0: np.int32, 1: np.int64, 2: np.float64}

i32, i64, u8p = C.c_int32, C.c_int64, C.POINTER(C.c_uint8)


class Batch(C.Structure):
    _fields_ = [("n_rows", i64), ("mem", i32), ("n_cols", i32),
                ("key_i64", C.c_void_p), ("key_offsets", C.c_void_p), ("key_bytes", C.c_void_p),
                ("key_valid", C.c_void_p), ("row_valid", C.c_void_p), ("ts", C.c_void_p),
                ("col_data", C.POINTER(C.c_void_p)), ("col_valid", C.POINTER(C.c_void_p)),
                # ABI 5: stream-time domains
                ("partition", C.c_void_p), ("stream_time", C.c_void_p)]


class BatchStats(C.Structure):
    _fields_ = [("rows_in", i64), ("rows_accepted", i64), ("dropped_null_key", i64),
                ("dropped_null_row", i64), ("dropped_bad_ts", i64), ("windows_applied", i64),
                ("windows_late", i64), ("stream_time", i64)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class AggSpec(C.Structure):
    _fields_ = [("kind", i32), ("arg_col", i32)]


class Having(C.Structure):
    _fields_ = [("agg_index", i32), ("op", i32), ("i64", i64), ("f64", C.c_double)]


class AggDesc(C.Structure):
    _fields_ = [("window_kind", i32), ("key_type", i32), ("size_ms", i64), ("advance_ms", i64),
                ("grace_ms", i64), ("n_cols", i32), ("col_types", C.POINTER(i32)),
                ("n_aggs", i32), ("aggs", C.POINTER(AggSpec)), ("device", i32), ("flags", i32),
                ("capacity_hint", i64),
                # ABI 2
                ("retention_ms", i64), ("emit", i32), ("has_having", i32), ("having", Having),
                # ABI 5
                ("time_domain", i32), ("n_partitions", i32)]


class Snapshot(C.Structure):
    _fields_ = [("capacity", i64), ("n_rows", i64), ("key_bytes_capacity", i64),
                ("key_bytes_len", i64), ("key_i64", C.c_void_p), ("key_offsets", C.c_void_p),
                ("key_bytes", C.c_void_p), ("window_start", C.c_void_p), ("window_end", C.c_void_p),
                ("rowtime", C.c_void_p), ("agg_values", C.POINTER(C.c_void_p)),
                ("agg_null", C.POINTER(C.c_void_p))]


class Pull(C.Structure):
    _fields_ = [("n_keys", i64), ("keys", C.c_void_p), ("ws_lo", i64), ("ws_hi", i64),
                ("we_lo", i64), ("we_hi", i64), ("key_offsets", C.c_void_p), ("key_bytes", C.c_void_p)]


class TableDesc(C.Structure):
    _fields_ = [("key_type", i32), ("n_cols", i32), ("col_types", C.POINTER(i32)),
                ("device", i32), ("flags", i32), ("capacity_hint", i64)]


class Where(C.Structure):
    _fields_ = [("right_col", i32), ("op", i32), ("i64", i64), ("f64", C.c_double)]


class KernelTimes(C.Structure):
    _fields_ = [("stream_time_ms", C.c_double), ("dict_ms", C.c_double), ("partition_ms", C.c_double),
                ("apply_ms", C.c_double),
                ("finalize_ms", C.c_double), ("apply_launches", i64), ("records", i64),
                ("c1_pushes", i64), ("c1_declined", i64)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class TableSrc(C.Structure):
    """khip_table_src: the source table's PRIMARY KEY per batch row (table aggregation)."""
    _fields_ = [("key_type", i32), ("reserved", i32), ("key_i64", C.c_void_p), ("key_offsets", C.c_void_p),
                ("key_bytes", C.c_void_p), ("key_valid", C.c_void_p)]


class JoinDevOut(C.Structure):
    _fields_ = [("emit", C.c_void_p), ("matched", C.c_void_p), ("col_data", C.POINTER(C.c_void_p)),
                ("col_null", C.POINTER(C.c_void_p))]


class JoinOut(C.Structure):
    _fields_ = [("capacity", i64), ("n_rows", i64), ("stream_row", C.c_void_p),
                ("matched", C.c_void_p), ("col_data", C.POINTER(C.c_void_p)),
                ("col_null", C.POINTER(C.c_void_p))]


class ShuffleDesc(C.Structure):
    _fields_ = [("n_parts", i32), ("key_col", i32), ("n_cols", i32), ("col_types", C.POINTER(i32)),
                ("device", i32), ("flags", i32)]


class SerdeDesc(C.Structure):
    _fields_ = [("key_format", i32), ("key_type", i32), ("value_format", i32), ("n_fields", i32),
                ("field_types", C.POINTER(i32)), ("field_names", C.POINTER(C.c_char_p)),
                ("field_out", C.POINTER(i32)), ("delimiter", i32), ("device", i32),
                ("avro_schema_id", i32), ("avro_n_fields", i32), ("avro_field_names", C.POINTER(C.c_char_p)),
                ("avro_field_types", C.POINTER(i32)), ("avro_field_union", C.POINTER(i32))]


class RawBatch(C.Structure):
    _fields_ = [("n_rows", i64), ("mem", i32), ("ts", C.c_void_p), ("key_offsets", C.c_void_p),
                ("key_bytes", C.c_void_p), ("key_valid", C.c_void_p), ("value_offsets", C.c_void_p),
                ("value_bytes", C.c_void_p), ("value_valid", C.c_void_p)]


class SinkDesc(C.Structure):
    _fields_ = [("key_format", i32), ("n_key_cols", i32), ("key_types", C.POINTER(i32)),
                ("key_names", C.POINTER(C.c_char_p)), ("window_kind", i32), ("value_format", i32),
                ("n_value_cols", i32), ("value_types", C.POINTER(i32)), ("value_names", C.POINTER(C.c_char_p)),
                ("value_src", C.POINTER(i32)), ("delimiter", i32), ("device", i32)]


class KeyCol(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offsets", C.c_void_p), ("bytes", C.c_void_p), ("valid", C.c_void_p)]


class SinkRows(C.Structure):
    _fields_ = [("n_rows", i64), ("mem", i32), ("key_serialized", i32), ("key_i64", C.c_void_p),
                ("key_offsets", C.c_void_p), ("key_bytes", C.c_void_p), ("window_start", C.c_void_p),
                ("window_end", C.c_void_p), ("col_data", C.POINTER(C.c_void_p)), ("col_null", C.POINTER(C.c_void_p)),
                ("tombstone", C.c_void_p)]


class SinkOut(C.Structure):
    _fields_ = [("mem", i32), ("reserved", i32), ("key_capacity", i64), ("value_capacity", i64),
                ("key_offsets", C.c_void_p), ("key_bytes", C.c_void_p), ("value_offsets", C.c_void_p),
                ("value_bytes", C.c_void_p), ("value_null", C.c_void_p), ("key_len", i64), ("value_len", i64)]


FMT = {"NONE": 0, "KAFKA": 1, "DELIMITED": 2, "JSON": 3, "AVRO": 4}
SINK_SRC = {"WS": -2, "WE": -3}
AVRO_TYPE = {"boolean": 1, "int": 2, "long": 3, "float": 4, "double": 5, "string": 6, "bytes": 7}
TYPE_STRING = 3
COMM_ID_BYTES = 128

_P = C.c_void_p
SIGS = {
    "agg_create": ([C.POINTER(AggDesc), C.POINTER(_P)]),
    "agg_push": ([_P, C.POINTER(Batch), C.POINTER(BatchStats)]),
    "agg_push_table": ([_P, C.POINTER(Batch), C.POINTER(TableSrc), C.POINTER(BatchStats)]),
    "agg_snapshot_size": ([_P, C.POINTER(i64), C.POINTER(i64)]),
    "agg_snapshot": ([_P, C.POINTER(Having), C.POINTER(Snapshot)]),
    "agg_destroy": ([_P]),
    "agg_changes_size": ([_P, C.POINTER(i64), C.POINTER(i64)]),
    "agg_changes": ([_P, C.POINTER(Snapshot), _P]),
    "table_create": ([C.POINTER(TableDesc), C.POINTER(_P)]),
    "table_upsert": ([_P, C.POINTER(Batch)]),
    "table_size": ([_P, C.POINTER(i64)]),
    "table_probe": ([_P, C.POINTER(Batch), i32, C.POINTER(Where), C.POINTER(JoinOut)]),
    "table_destroy": ([_P]),
}
PRODUCT_ONLY = {
    "agg_result_type": ([C.POINTER(AggDesc), i32, C.POINTER(i32)]),
    "agg_count_rows": ([_P, C.POINTER(Having), C.POINTER(i64)]),
    "agg_get": ([_P, C.POINTER(Pull), C.POINTER(Having), C.POINTER(Snapshot)]),
    "agg_reset": ([_P]),
    "agg_sync": ([_P]),
    "agg_stream": ([_P, C.POINTER(_P)]),
    "agg_kernel_times": ([_P, C.POINTER(KernelTimes), i32]),
    "stream_time_scan": ([_P, C.POINTER(Batch), i64, _P, C.POINTER(i64)]),
    "table_probe_device": ([_P, C.POINTER(Batch), i32, C.POINTER(Where), C.POINTER(JoinDevOut), C.POINTER(i64)]),
    "table_sync": ([_P]),
    "shuffle_create": ([C.POINTER(ShuffleDesc), C.POINTER(_P)]),
    "shuffle_pack": ([_P, C.POINTER(Batch), _P, i64, C.POINTER(i64)]),
    "shuffle_unpack": ([_P, _P, i64, _P, _P, C.POINTER(_P), C.POINTER(_P)]),
    "shuffle_pack_v": ([_P, C.POINTER(Batch), _P, i64, C.POINTER(i64), C.POINTER(i64)]),
    "shuffle_unpack_stream_time": ([_P, _P, i64, _P]),
    "shuffle_stream_time_seed": ([_P, i64]),
    "agg_lost_windows": ([_P, _P, i64, _P, i64, _P]),
    "agg_supplied_close": ([_P, i64, i64, _P, i64]),
    "agg_push_shuffled": ([_P, _P, _P, i64, C.POINTER(BatchStats)]),
    "shuffle_sync": ([_P]),
    "shuffle_destroy": ([_P]),
    "comm_unique_id": ([C.POINTER(C.c_uint8)]),
    "comm_init": ([i32, i32, C.POINTER(C.c_uint8), i32, C.POINTER(_P)]),
    "comm_exchange_counts": ([_P, C.POINTER(i64), C.POINTER(i64)]),
    "comm_alltoall": ([_P, _P, C.POINTER(i64), _P, i64, C.POINTER(i64), i32]),
    "comm_alltoall_v": ([_P, _P, C.POINTER(i64), C.POINTER(i64), _P, i64, C.POINTER(i64), i32]),
    "comm_destroy": ([_P]),
    "serde_create": ([C.POINTER(SerdeDesc), C.POINTER(_P)]),
    "serde_decode": ([_P, C.POINTER(RawBatch), C.POINTER(Batch), C.POINTER(i64)]),
    "serde_destroy": ([_P]),
    "sink_create": ([C.POINTER(SinkDesc), C.POINTER(_P)]),
    "sink_key": ([_P, C.POINTER(Batch), C.POINTER(KeyCol), C.POINTER(Batch)]),
    "sink_encode": ([_P, C.POINTER(SinkRows), C.POINTER(SinkOut)]),
    "sink_sync": ([_P]),
    "sink_destroy": ([_P]),
}


class KsqlHipError(RuntimeError):
    pass


class Lib:
    """Binds one library (product or oracle) by prefix."""

    def __init__(self, path, prefix, product):
        if not os.path.exists(path):
            raise KsqlHipError("library not built: %s" % path)
        self.path = path
        self.dll = C.CDLL(path)
        self.prefix = prefix
        self.product = product
        sigs = dict(SIGS)
        if product:
            sigs.update(PRODUCT_ONLY)
        for name, args in sigs.items():
            fn = getattr(self.dll, prefix + name)
            fn.argtypes = args
            fn.restype = i32
            setattr(self, name, fn)
        if product:
            self.dll.khip_last_error.restype = C.c_char_p
            self.dll.khip_last_error.argtypes = []
            self.dll.khip_abi_version.restype = i32
            self.dll.khip_build_target.restype = C.c_char_p
            self.dll.khip_shuffle_row_words.restype = i32
            self.dll.khip_shuffle_row_words.argtypes = [_P]
            self.dll.khip_shuffle_pack_capacity.restype = i64
            self.dll.khip_shuffle_pack_capacity.argtypes = [_P, i64]
        else:
            self.dll.oracle_kafka_partition.argtypes = [_P, i64, i32, i32, _P]
            self.dll.oracle_kafka_partition.restype = None
            self.dll.oracle_murmur2.argtypes = [C.c_char_p, i32]
            self.dll.oracle_murmur2.restype = i32
            self.dll.oracle_agg_push_sharded.argtypes = [C.POINTER(_P), i32, C.POINTER(Batch), C.POINTER(BatchStats)]
            self.dll.oracle_agg_push_sharded.restype = i32
            self.dll.oracle_agg_snapshot_size_sharded.argtypes = [C.POINTER(_P), i32, C.POINTER(i64), C.POINTER(i64)]
            self.dll.oracle_agg_snapshot_size_sharded.restype = i32
            self.dll.oracle_agg_snapshot_sharded.argtypes = [C.POINTER(_P), i32, C.POINTER(Having), C.POINTER(Snapshot)]
            self.dll.oracle_agg_snapshot_sharded.restype = i32
            self.dll.oracle_agg_changes_size_sharded.argtypes = [C.POINTER(_P), i32, C.POINTER(i64), C.POINTER(i64)]
            self.dll.oracle_agg_changes_size_sharded.restype = i32
            self.dll.oracle_agg_changes_sharded.argtypes = [C.POINTER(_P), i32, C.POINTER(Snapshot), _P]
            self.dll.oracle_agg_changes_sharded.restype = i32

    def check(self, status, what):
        if status != KHIP_OK:
            msg = self.dll.khip_last_error().decode() if self.product else ""
            raise KsqlHipError("%s%s failed (%d): %s" % (self.prefix, what, status, msg))


_product = None
_oracle = None


def load_product():
    """The HIP library.  Raises if it was not built: there is no fallback."""
    global _product
    if _product is None:
        _product = Lib(PRODUCT_LIB, "khip_", True)
    return _product


def load_oracle():
    """CPU restatement — test infrastructure only."""
    global _oracle
    if _oracle is None:
        _oracle = Lib(ORACLE_LIB, "oracle_", False)
    return _oracle


# ------------------------------------------------------------------ helpers

def bitmap(valid):
    """bool array -> Arrow LSB bitmap (uint8), or None if all valid."""
    valid = np.asarray(valid, dtype=bool)
    if valid.all():
        return None
    return np.packbits(valid, bitorder="little")


def _ptr(a):
    return None if a is None else a.ctypes.data


class HostBatch:
    """Owns numpy arrays for one host batch and the ctypes struct pointing at them."""

    def __init__(self, ts, keys=None, key_valid=None, row_valid=None, cols=(), col_valid=(),
                 utf8_keys=None, key_offsets=None, key_bytes=None, partition=None, stream_time=None):
        """utf8_keys: a list of str/bytes (None → b""), or the columnar form key_offsets
        (int64, n+1) + key_bytes (uint8).  partition (int32) / stream_time (int64): the ABI 5
        stream-time domain columns (TIME["PARTITION"] / TIME["SUPPLIED"])."""
        self.ts = np.ascontiguousarray(ts, dtype=np.int64)
        n = len(self.ts)
        self.keys = None if keys is None else np.ascontiguousarray(keys, dtype=np.int64)
        self.key_offsets = None if key_offsets is None else np.ascontiguousarray(key_offsets, dtype=np.int64)
        self.key_bytes = None if key_bytes is None else np.ascontiguousarray(key_bytes, dtype=np.uint8)
        if utf8_keys is not None:
            enc = [b"" if k is None else (k.encode() if isinstance(k, str) else bytes(k)) for k in utf8_keys]
            self.key_offsets = np.zeros(n + 1, dtype=np.int64)
            self.key_offsets[1:] = np.cumsum([len(e) for e in enc])
            self.key_bytes = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8).copy()
        self.key_valid = None if key_valid is None else bitmap(key_valid)
        self.row_valid = None if row_valid is None else bitmap(row_valid)
        self.cols = [np.ascontiguousarray(c) for c in cols]
        self.col_valid = [None if v is None else bitmap(v) for v in col_valid] + \
            [None] * (len(self.cols) - len(col_valid))
        nc = len(self.cols)
        self._cd = (C.c_void_p * max(nc, 1))(*[_ptr(c) for c in self.cols])
        self._cv = (C.c_void_p * max(nc, 1))(*[_ptr(v) for v in self.col_valid])
        self.partition = None if partition is None else np.ascontiguousarray(partition, dtype=np.int32)
        self.stream_time = None if stream_time is None else np.ascontiguousarray(stream_time, dtype=np.int64)
        self.struct = Batch(n, MEM_HOST, nc, _ptr(self.keys), _ptr(self.key_offsets),
                            _ptr(self.key_bytes), _ptr(self.key_valid), _ptr(self.row_valid),
                            _ptr(self.ts), self._cd, self._cv, _ptr(self.partition), _ptr(self.stream_time))


def having_struct(having):
    """{"agg": i, "op": "GT", "value": v} → Having (integer constant for int values, both set)."""
    v = having["value"]
    return Having(having["agg"], OP[having["op"]], 0 if isinstance(v, float) else int(v), float(v))


def make_agg_desc(window_kind="NONE", key_type="INT64", size_ms=0, advance_ms=0, grace_ms=-1,
                  col_types=(), aggs=(), device=0, capacity_hint=0, flags=0, retention_ms=RETENTION_DEFAULT,
                  emit="CHANGES", having=None, time_domain="TASK", n_partitions=0):
    """having: the query's HAVING ({"agg", "op", "value"}), maintained by the library (ABI 2).
    time_domain / n_partitions: the stream-time domain (ABI 5; include/ksqldb_hip.h KHIP_TIME_*)."""
    ct = (i32 * max(len(col_types), 1))(*[TYPE[t] if isinstance(t, str) else t for t in col_types])
    sp = (AggSpec * max(len(aggs), 1))(*[AggSpec(AGG[k] if isinstance(k, str) else k, c) for k, c in aggs])
    d = AggDesc(WINDOW[window_kind] if isinstance(window_kind, str) else window_kind,
                KEY[key_type] if isinstance(key_type, str) else key_type,
                size_ms, advance_ms if advance_ms else size_ms, grace_ms, len(col_types), ct,
                len(aggs), sp, device, flags, capacity_hint, retention_ms,
                EMIT[emit] if isinstance(emit, str) else emit, 0 if having is None else 1,
                Having() if having is None else having_struct(having),
                TIME[time_domain] if isinstance(time_domain, str) else time_domain, n_partitions)
    d._keep = (ct, sp)
    return d


def result_types(desc):
    out = []
    for i in range(desc.n_aggs):
        k = desc.aggs[i].kind
        if k in (AGG["COUNT_STAR"], AGG["COUNT"]):
            out.append(TYPE["INT64"])
        elif k == AGG["AVG"]:
            out.append(TYPE["DOUBLE"])
        else:
            out.append(desc.col_types[desc.aggs[i].arg_col])
    return out


class DeviceBatch:
    """A khip_batch over device tensors (torch) — the caller keeps the tensors alive."""

    def __init__(self, ts, keys=None, key_valid=None, row_valid=None, cols=(), col_valid=(),
                 key_offsets=None, key_bytes=None, partition=None, stream_time=None):
        self._keep = [ts, keys, key_valid, row_valid, key_offsets, key_bytes, partition, stream_time] + \
            list(cols) + list(col_valid)
        p = lambda t: None if t is None else t.data_ptr()
        nc = len(cols)
        cv = list(col_valid) + [None] * (nc - len(col_valid))
        self._cd = (C.c_void_p * max(nc, 1))(*[p(c) for c in cols])
        self._cv = (C.c_void_p * max(nc, 1))(*[p(v) for v in cv])
        self.struct = Batch(int(ts.numel()), MEM_DEVICE, nc, p(keys), p(key_offsets), p(key_bytes),
                            p(key_valid), p(row_valid), p(ts), self._cd, self._cv, p(partition), p(stream_time))


def bitmap_torch(valid_bool):
    """bool tensor (n,) on device → packed LSB-first uint8 bitmap tensor."""
    import torch
    n = valid_bool.numel()
    pad = (-n) % 8
    v = valid_bool.to(torch.uint8)
    if pad:
        v = torch.cat([v, torch.zeros(pad, dtype=torch.uint8, device=v.device)])
    v = v.view(-1, 8)
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=v.device)
    return (v * w).sum(dim=1, dtype=torch.int32).to(torch.uint8)


class AggHandle:
    """A windowed/unwindowed aggregate task on one library (product or oracle)."""

    def __init__(self, lib, desc):
        self.lib = lib
        self.desc = desc
        self.h = C.c_void_p()
        lib.check(lib.agg_create(C.byref(desc), C.byref(self.h)), "agg_create")

    def push(self, batch, stats=True):
        st = BatchStats()
        self.lib.check(self.lib.agg_push(self.h, C.byref(batch.struct if hasattr(batch, "struct") else batch),
                                         C.byref(st) if stats else None), "agg_push")
        return st.as_dict() if stats else None

    def push_shuffled(self, shuffle, rows, n, stats=True):
        """khip_agg_push_shuffled (ABI 6): `n` rows a ShuffleHandle packed / received (a device tensor
        [>= n, row_words]) into this aggregation, without unpacking them to columns first."""
        st = BatchStats()
        self.lib.check(self.lib.agg_push_shuffled(self.h, shuffle.h, None if rows is None else rows.data_ptr(), n,
                                                  C.byref(st) if stats else None), "agg_push_shuffled")
        return st.as_dict() if stats else None

    def push_table(self, batch, src_keys=None, src_utf8_keys=None, src_key_valid=None, stats=True):
        """khip_agg_push_table (handle created with FLAG_TABLE_SOURCE): `batch` holds the rows'
        GROUP BY keys / tombstones / ts / argument columns, src_* the source PRIMARY KEY of each row
        (host memory, like `batch`)."""
        n = batch.struct.n_rows
        keep = []
        if src_utf8_keys is not None:
            enc = [b"" if k is None else (k.encode() if isinstance(k, str) else bytes(k)) for k in src_utf8_keys]
            off = np.zeros(n + 1, dtype=np.int64)
            off[1:] = np.cumsum([len(e) for e in enc])
            kb = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8).copy()
            keep += [off, kb]
            src = TableSrc(KEY["UTF8"], 0, None, off.ctypes.data, kb.ctypes.data, None)
            if src_key_valid is None:
                src_key_valid = [k is not None for k in src_utf8_keys]
        else:
            k = np.ascontiguousarray(src_keys, dtype=np.int64)
            keep.append(k)
            src = TableSrc(KEY["INT64"], 0, k.ctypes.data, None, None, None)
        bm = None if src_key_valid is None else bitmap(src_key_valid)
        if bm is not None:
            keep.append(bm)
            src.key_valid = bm.ctypes.data
        st = BatchStats()
        self.lib.check(self.lib.agg_push_table(self.h, C.byref(batch.struct), C.byref(src),
                                               C.byref(st) if stats else None), "agg_push_table")
        return st.as_dict() if stats else None

    def snapshot(self, having=None, raw_keys=False):
        """raw_keys: UTF8 keys as the columnar (key_offsets, key_bytes) arrays instead of a list of
        str (for tables of tens of millions of rows)."""
        return self._materialize(having, lambda hv, s: self.lib.agg_snapshot(self.h, hv, s), "agg_snapshot",
                                 raw_keys=raw_keys)

    def changes(self, raw_keys=False):
        """Rows the last push emitted downstream (khip_agg_changes): snapshot layout sorted by
        (key, ws), plus "tombstone" (bool per row: a HAVING delete)."""
        return self._changes(self.lib.agg_changes_size, lambda s, t: self.lib.agg_changes(self.h, s, t), raw_keys)

    def _changes(self, size_fn, call, raw_keys):
        n, kb = i64(), i64()
        self.lib.check(size_fn(self.h, C.byref(n), C.byref(kb)), "agg_changes_size")
        cap = max(n.value, 1)
        tomb = np.zeros(cap, np.uint8)
        out, st, _ = self._materialize_into(None, lambda hv, s: call(s, tomb.ctypes.data), cap, max(kb.value, 1),
                                            raw_keys)
        self.lib.check(st, "agg_changes")
        out["tombstone"] = tomb[:out["n"]].astype(bool)
        return out

    def get(self, keys=None, ws=(None, None), we=(None, None), having=None):
        """Pull query (khip_agg_get): rows of `keys` (None = every key) whose WINDOWSTART and
        WINDOWEND lie in the closed bounds (None = unbounded), sorted by (key, ws)."""
        lo, hi = -(1 << 63), (1 << 63) - 1
        koff = kbytes = None
        if keys is not None and self.desc.key_type == KEY["UTF8"]:
            enc = [k.encode("utf-8", "surrogateescape") if isinstance(k, str) else bytes(k) for k in keys]
            koff = np.zeros(len(enc) + 1, np.int64)
            koff[1:] = np.cumsum([len(e) for e in enc]) if enc else []
            kbytes = np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy()
            ka = np.zeros(len(enc), np.int64)
        else:
            ka = None if keys is None else np.ascontiguousarray(keys, np.int64)
        q = Pull(0 if ka is None else len(ka), None if ka is None or len(ka) == 0 else ka.ctypes.data,
                 lo if ws[0] is None else ws[0], hi if ws[1] is None else ws[1],
                 lo if we[0] is None else we[0], hi if we[1] is None else we[1],
                 None if koff is None else koff.ctypes.data, None if kbytes is None else kbytes.ctypes.data)
        if ka is not None and len(ka) == 0:
            return self._materialize(None, None, "agg_get", cap=1)
        # point lookups: start from a small output buffer, grow to the row count on KHIP_E_BUFFER
        return self._materialize(having, lambda hv, s: self.lib.agg_get(self.h, C.byref(q), hv, s), "agg_get",
                                 cap=4096 if self.desc.key_type == KEY["INT64"] else None)

    def _materialize(self, having, call, what, cap=None, raw_keys=False):
        if cap is None:
            n, kb = i64(), i64()
            self.lib.check(self.lib.agg_snapshot_size(self.h, C.byref(n), C.byref(kb)), "agg_snapshot_size")
            cap, kcap = max(n.value, 1), max(kb.value, 1)
        else:
            kcap = 1
        while True:
            out, st, n_needed = self._materialize_into(having, call, cap, kcap, raw_keys)
            if st == KHIP_E_BUFFER and n_needed > cap:
                cap = n_needed
                continue
            self.lib.check(st, what)
            return out

    def _materialize_into(self, having, call, cap, kcap, raw_keys=False):
        rt = result_types(self.desc)
        arrays = {
            "key": np.zeros(cap, np.int64), "key_offsets": np.zeros(cap + 1, np.int64),
            "key_bytes": np.zeros(kcap, np.uint8), "ws": np.zeros(cap, np.int64),
            "we": np.zeros(cap, np.int64), "rowtime": np.zeros(cap, np.int64),
            "values": [np.zeros(cap, NP_TYPE[t]) for t in rt],
            "nulls": [np.zeros(cap, np.uint8) for _ in rt],
        }
        av = (C.c_void_p * max(len(rt), 1))(*[a.ctypes.data for a in arrays["values"]])
        an = (C.c_void_p * max(len(rt), 1))(*[a.ctypes.data for a in arrays["nulls"]])
        s = Snapshot(cap, 0, kcap, 0, arrays["key"].ctypes.data, arrays["key_offsets"].ctypes.data,
                     arrays["key_bytes"].ctypes.data, arrays["ws"].ctypes.data, arrays["we"].ctypes.data,
                     arrays["rowtime"].ctypes.data, av, an)
        hv = None
        if having is not None:
            hv = Having(having["agg"], OP[having["op"]], int(having["value"]) if not isinstance(having["value"], float) else 0,
                        float(having["value"]))
        st = KHIP_OK if call is None else call(C.byref(hv) if hv else None, C.byref(s))
        if st != KHIP_OK:
            return None, st, s.n_rows
        m = s.n_rows
        out = {"n": m, "ws": arrays["ws"][:m], "we": arrays["we"][:m], "rowtime": arrays["rowtime"][:m],
               "values": [v[:m] for v in arrays["values"]], "nulls": [v[:m].astype(bool) for v in arrays["nulls"]]}
        if self.desc.key_type == KEY["UTF8"] and raw_keys:
            out["key_offsets"] = arrays["key_offsets"][: m + 1]
            out["key_bytes"] = arrays["key_bytes"][: int(arrays["key_offsets"][m]) if m else 0]
        elif self.desc.key_type == KEY["UTF8"]:
            offs = arrays["key_offsets"][: m + 1]
            kbts = arrays["key_bytes"].tobytes()
            out["key"] = [kbts[offs[i]:offs[i + 1]].decode("utf-8", "surrogateescape") for i in range(m)]
        else:
            out["key"] = arrays["key"][:m]
        return out, KHIP_OK, m

    def stream_time_scan(self, batch, seed=-1, out=None):
        """khip_stream_time_scan (ABI 5): the stream time observed at each row of `batch` starting
        from `seed`.  Host batch → (int64 array, max); device batch → `out` (an int64 device tensor
        of n_rows) is filled and (out, max) returned."""
        n = int(batch.struct.n_rows)
        mx = i64()
        if batch.struct.mem == MEM_HOST:
            res = np.zeros(max(n, 1), np.int64)
            self.lib.check(self.lib.stream_time_scan(self.h, C.byref(batch.struct), seed, res.ctypes.data, C.byref(mx)),
                           "stream_time_scan")
            return res[:n], mx.value
        self.lib.check(self.lib.stream_time_scan(self.h, C.byref(batch.struct), seed, out.data_ptr(), C.byref(mx)),
                       "stream_time_scan")
        return out, mx.value

    def lost_windows(self, batch, seed=-1):
        """khip_agg_lost_windows (ABI 8): [(lo, hi), ...] window-start ranges the batch's stream-time
        jumps (from `seed`) close after they expired."""
        cap = 64
        while True:
            buf = np.zeros(2 * cap, np.int64)
            n = i64()
            st = self.lib.agg_lost_windows(self.h, C.byref(batch.struct), int(seed), buf.ctypes.data, cap,
                                                    C.byref(n))
            if st == KHIP_E_BUFFER and n.value > cap:
                cap = int(n.value)
                continue
            self.lib.check(st, "agg_lost_windows")
            return [(int(buf[2 * k]), int(buf[2 * k + 1])) for k in range(n.value)]

    def supplied_close(self, st_before, st_after, ranges=()):
        """khip_agg_supplied_close (ABI 8): the GLOBAL stream time around the next push and the
        union of the ranks' lost ranges."""
        r = np.asarray([x for p in ranges for x in p], np.int64)
        self.lib.check(self.lib.agg_supplied_close(self.h, int(st_before), int(st_after),
                                                   r.ctypes.data if len(r) else None, len(r) // 2),
                       "agg_supplied_close")

    def kernel_times(self, reset=False):
        kt = KernelTimes()
        self.lib.check(self.lib.agg_kernel_times(self.h, C.byref(kt), 1 if reset else 0), "agg_kernel_times")
        return kt.as_dict()

    def reset(self):
        self.lib.check(self.lib.agg_reset(self.h), "agg_reset")

    def snapshot_size(self):
        """Rows of the materialized table (khip_agg_snapshot_size, no key-byte count: no device work)."""
        n = i64()
        self.lib.check(self.lib.agg_snapshot_size(self.h, C.byref(n), None), "agg_snapshot_size")
        return n.value

    def count_rows(self, having=None):
        n = i64()
        hv = None
        if having is not None:
            v = having["value"]
            hv = Having(having["agg"], OP[having["op"]], 0 if isinstance(v, float) else int(v), float(v))
        self.lib.check(self.lib.agg_count_rows(self.h, C.byref(hv) if hv else None, C.byref(n)), "agg_count_rows")
        return n.value

    def close(self):
        if self.h:
            self.lib.agg_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedOracleAgg(AggHandle):
    """The oracle's key-sharded P-thread restatement (oracle_agg_push_sharded): one task's
    windowed aggregate over P key-hash shards, one thread each — results identical to the
    sequential oracle.  Test infrastructure / CPU baseline only."""

    def __init__(self, orc, desc, shards):
        assert not orc.product
        self.lib = orc
        self.desc = desc
        self.P = int(shards)
        self._hs = (C.c_void_p * self.P)()
        for p in range(self.P):
            h = C.c_void_p()
            orc.check(orc.agg_create(C.byref(desc), C.byref(h)), "agg_create")
            self._hs[p] = h
        self.h = self._hs[0]
        d = orc.dll
        self._push = d.oracle_agg_push_sharded
        self._size = d.oracle_agg_snapshot_size_sharded
        self._snap = d.oracle_agg_snapshot_sharded

    def push(self, batch, stats=True):
        st = BatchStats()
        self.lib.check(self._push(self._hs, self.P, C.byref(batch.struct), C.byref(st) if stats else None),
                       "agg_push_sharded")
        return st.as_dict() if stats else None

    def snapshot(self, having=None, raw_keys=False):
        return self._materialize(having, lambda hv, s: self._snap(self._hs, self.P, hv, s), "agg_snapshot_sharded",
                                 raw_keys=raw_keys)

    def changes(self, raw_keys=False):
        d = self.lib.dll
        return self._changes(lambda h, n, kb: d.oracle_agg_changes_size_sharded(self._hs, self.P, n, kb),
                             lambda s, t: d.oracle_agg_changes_sharded(self._hs, self.P, s, t), raw_keys)

    def _materialize(self, having, call, what, cap=None, raw_keys=False):
        if cap is None:
            n, kb = i64(), i64()
            self.lib.check(self._size(self._hs, self.P, C.byref(n), C.byref(kb)), "agg_snapshot_size_sharded")
            cap, kcap = max(n.value, 1), max(kb.value, 1)
        else:
            kcap = 1
        out, st, _ = self._materialize_into(having, call, cap, kcap, raw_keys)
        self.lib.check(st, what)
        return out

    def close(self):
        if getattr(self, "_hs", None) is not None:
            for p in range(self.P):
                if self._hs[p]:
                    self.lib.agg_destroy(self._hs[p])
            self._hs = None
            self.h = C.c_void_p()


class TableHandle:
    def __init__(self, lib, col_types, device=0, capacity_hint=0, key_type="INT64"):
        self.lib = lib
        self.col_types = [TYPE[t] if isinstance(t, str) else t for t in col_types]
        ct = (i32 * max(len(col_types), 1))(*self.col_types)
        self._ct = ct
        self.desc = TableDesc(KEY[key_type], len(col_types), ct, device, 0, capacity_hint)
        self.h = C.c_void_p()
        lib.check(lib.table_create(C.byref(self.desc), C.byref(self.h)), "table_create")

    def upsert(self, batch):
        self.lib.check(self.lib.table_upsert(self.h, C.byref(batch.struct)), "table_upsert")

    def size(self):
        n = i64()
        self.lib.check(self.lib.table_size(self.h, C.byref(n)), "table_size")
        return n.value

    def probe(self, batch, join_type="LEFT", where=None, capacity=None):
        n = batch.struct.n_rows
        cap = max(n if capacity is None else capacity, 1)
        sr = np.zeros(cap, np.int64)
        mt = np.zeros(cap, np.uint8)
        cols = [np.zeros(cap, NP_TYPE[t]) for t in self.col_types]
        nulls = [np.zeros(cap, np.uint8) for _ in self.col_types]
        cd = (C.c_void_p * max(len(cols), 1))(*[c.ctypes.data for c in cols])
        cn = (C.c_void_p * max(len(cols), 1))(*[c.ctypes.data for c in nulls])
        out = JoinOut(cap, 0, sr.ctypes.data, mt.ctypes.data, cd, cn)
        wv = None
        if where is not None:
            wv = Where(where["col"], OP[where["op"]], int(where.get("i64", 0)), float(where.get("f64", 0.0)))
        self.lib.check(self.lib.table_probe(self.h, C.byref(batch.struct), JOIN[join_type],
                                            C.byref(wv) if wv else None, C.byref(out)), "table_probe")
        m = out.n_rows
        return {"n": m, "stream_row": sr[:m], "matched": mt[:m].astype(bool),
                "cols": [c[:m] for c in cols], "nulls": [x[:m].astype(bool) for x in nulls]}

    def probe_device(self, batch, join_type="LEFT", where=None, emit=None, matched=None, cols=None, nulls=None,
                     count=True):
        """khip_table_probe_device: row-aligned device outputs (torch tensors, caller-owned);
        returns the emitted-row count (synchronising) or None (count=False, asynchronous)."""
        p = lambda t: None if t is None else t.data_ptr()
        nc = len(self.col_types)
        cd = (C.c_void_p * max(nc, 1))(*[p(c) for c in (cols or [None] * nc)])
        cn = (C.c_void_p * max(nc, 1))(*[p(c) for c in (nulls or [None] * nc)])
        out = JoinDevOut(p(emit), p(matched), cd, cn)
        wv = None
        if where is not None:
            wv = Where(where["col"], OP[where["op"]], int(where.get("i64", 0)), float(where.get("f64", 0.0)))
        n = i64()
        self.lib.check(self.lib.table_probe_device(self.h, C.byref(batch.struct), JOIN[join_type],
                                                   C.byref(wv) if wv else None, C.byref(out),
                                                   C.byref(n) if count else None), "table_probe_device")
        return n.value if count else None

    def sync(self):
        self.lib.check(self.lib.table_sync(self.h), "table_sync")

    def close(self):
        if self.h:
            self.lib.table_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShuffleHandle:
    """Repartition of a device batch by a value column (khip_shuffle_*), the device side of
    the repartition topic StreamGroupByBuilderBase inserts for a non-key GROUP BY."""

    def __init__(self, lib, n_parts, key_col, col_types, device=0, stream_time=False):
        """stream_time: KHIP_SHUFFLE_STREAM_TIME (ABI 7), the rows carry the batch's stream_time
        column (the GLOBAL stream-time domain)."""
        self.lib = lib
        self.col_types = [TYPE[t] if isinstance(t, str) else t for t in col_types]
        self._ct = (i32 * len(self.col_types))(*self.col_types)
        self.stream_time = bool(stream_time)
        self.desc = ShuffleDesc(n_parts, key_col, len(self.col_types), self._ct, device,
                                SHUFFLE_STREAM_TIME if stream_time else 0)
        self.n_parts = n_parts
        self.device = device
        self.h = C.c_void_p()
        lib.check(lib.shuffle_create(C.byref(self.desc), C.byref(self.h)), "shuffle_create")
        self.row_words = lib.dll.khip_shuffle_row_words(self.h)

    def pack(self, batch, send=None):
        """Returns (send rows tensor [rows, row_words] uint64-as-int64, counts list)."""
        import torch
        counts = (i64 * self.n_parts)()
        cap = 0 if send is None else send.shape[0]
        st = self.lib.shuffle_pack(self.h, C.byref(batch.struct), None if send is None else send.data_ptr(),
                                   cap, counts)
        if st == KHIP_E_BUFFER:
            send = torch.empty((max(sum(counts), 1), self.row_words), dtype=torch.int64,
                               device=torch.device("cuda", self.device))
            st = self.lib.shuffle_pack(self.h, C.byref(batch.struct), send.data_ptr(), send.shape[0], counts)
        self.lib.check(st, "shuffle_pack")
        return send, list(counts)

    def pack_capacity(self, n_rows):
        """Rows khip_shuffle_pack_v's send buffer needs for a batch of n_rows."""
        return int(self.lib.dll.khip_shuffle_pack_capacity(self.h, n_rows))

    def pack_v(self, batch, send=None):
        """khip_shuffle_pack_v (ABI 7, one pass): returns (send, counts, offsets) — destination d's
        rows are send[offsets[d] : offsets[d] + counts[d]]."""
        import torch
        n = int(batch.struct.n_rows)
        need = max(self.pack_capacity(n), 1)
        if send is None or send.shape[0] < need:
            send = torch.empty((need, self.row_words), dtype=torch.int64, device=torch.device("cuda", self.device))
        counts = (i64 * self.n_parts)()
        offs = (i64 * self.n_parts)()
        self.lib.check(self.lib.shuffle_pack_v(self.h, C.byref(batch.struct), send.data_ptr(), send.shape[0],
                                               counts, offs), "shuffle_pack_v")
        return send, list(counts), list(offs)

    def stream_time_seed(self, seed):
        """khip_shuffle_stream_time_seed (ABI 8): the next packs write max(seed, stream_time[i])."""
        self.lib.check(self.lib.shuffle_stream_time_seed(self.h, int(seed)), "shuffle_stream_time_seed")

    def unpack_stream_time(self, rows, n):
        """The stream_time column of KHIP_SHUFFLE_STREAM_TIME rows (device int64 tensor)."""
        import torch
        st = torch.empty(max(n, 1), dtype=torch.int64, device=torch.device("cuda", self.device))
        self.lib.check(self.lib.shuffle_unpack_stream_time(self.h, None if rows is None else rows.data_ptr(), n,
                                                           st.data_ptr()), "shuffle_unpack_stream_time")
        return st[:n]

    def unpack(self, rows, n, key_as_col=False):
        """Packed rows → (key, ts, cols, col_valid bitmaps) device tensors.  key_as_col: the
        GROUP BY column is not written again (it IS the key: cols[key_col] is the key tensor,
        valid by construction — pack drops NULL keys — so its bitmap is None)."""
        import torch
        dev = torch.device("cuda", self.device)
        key = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        ts = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        tdt = {0: torch.int32, 1: torch.int64, 2: torch.float64}
        kc = self.desc.key_col if key_as_col and self.col_types[self.desc.key_col] == TYPE["INT64"] else -1
        cols = [key if c == kc else torch.empty(max(n, 1), dtype=tdt[t], device=dev)
                for c, t in enumerate(self.col_types)]
        valid = [None if c == kc else torch.empty(max((n + 7) // 8, 1), dtype=torch.uint8, device=dev)
                 for c in range(len(self.col_types))]
        cd = (C.c_void_p * len(cols))(*[None if c == kc else x.data_ptr() for c, x in enumerate(cols)])
        cv = (C.c_void_p * len(cols))(*[None if v is None else v.data_ptr() for v in valid])
        self.lib.check(self.lib.shuffle_unpack(self.h, None if rows is None else rows.data_ptr(), n,
                                               key.data_ptr(), ts.data_ptr(), cd, cv), "shuffle_unpack")
        return key[:n], ts[:n], [c[:n] for c in cols], [None if v is None else v[:(n + 7) // 8] for v in valid]

    def close(self):
        if self.h:
            self.lib.shuffle_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id(lib):
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    lib.check(lib.comm_unique_id(buf), "comm_unique_id")
    return bytes(buf)


class Comm:
    """RCCL communicator owned by the library (one rank per GPU)."""

    def __init__(self, lib, nranks, rank, uid, device):
        self.lib = lib
        self.nranks = nranks
        self.device = device
        self.h = C.c_void_p()
        idb = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        lib.check(lib.comm_init(nranks, rank, idb, device, C.byref(self.h)), "comm_init")

    def alltoall(self, send, send_counts, row_words, send_offsets=None):
        """Two collective steps: exchange counts, then the rows (send_offsets: peer p's rows start
        at row send_offsets[p], khip_shuffle_pack_v's layout; None: adjacent, by peer).  Returns
        (recv, recv_counts); recv holds the rows by source rank."""
        import torch
        sc = (i64 * self.nranks)(*send_counts)
        rc = (i64 * self.nranks)()
        self.lib.check(self.lib.comm_exchange_counts(self.h, sc, rc), "comm_exchange_counts")
        recv = torch.empty((max(sum(rc), 1), row_words), dtype=torch.int64, device=torch.device("cuda", self.device))
        sp = None if send is None else send.data_ptr()
        if send_offsets is None:
            self.lib.check(self.lib.comm_alltoall(self.h, sp, sc, recv.data_ptr(), recv.shape[0], rc, row_words),
                           "comm_alltoall")
        else:
            so = (i64 * self.nranks)(*send_offsets)
            self.lib.check(self.lib.comm_alltoall_v(self.h, sp, sc, so, recv.data_ptr(), recv.shape[0], rc, row_words),
                           "comm_alltoall_v")
        return recv, list(rc)

    def allgather_ranges(self, ranges):
        """Every rank's list of (lo, hi) int64 pairs, concatenated in rank order: the all-to-all
        with this rank's list sent to every peer from one region (send offsets all 0)."""
        import torch
        m = len(ranges)
        send = torch.tensor([list(r) for r in ranges] if m else [[0, 0]], dtype=torch.int64,
                            device=torch.device("cuda", self.device))
        recv, rc = self.alltoall(send, [m] * self.nranks, 2, send_offsets=[0] * self.nranks)
        return [tuple(r) for r in recv[:sum(rc)].cpu().tolist()]

    def allgather_i64(self, x):
        """One int64 from every rank (the count exchange with x sent to every peer)."""
        sc = (i64 * self.nranks)(*([int(x)] * self.nranks))
        rc = (i64 * self.nranks)()
        self.lib.check(self.lib.comm_exchange_counts(self.h, sc, rc), "comm_exchange_counts")
        return list(rc)

    def close(self):
        if self.h:
            self.lib.comm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SerdeHandle:
    """khip_serde_*: Kafka record bytes (KAFKA / DELIMITED / JSON / AVRO) → a device batch."""

    def __init__(self, lib, value_format, fields, key_type="INT64", key_format="KAFKA", delimiter=",",
                 device=0, avro_schema=None, avro_schema_id=-1):
        """fields: [(name, type, out_col or -1)], type in INT32 / INT64 / DOUBLE / STRING.
        avro_schema (AVRO): the writer record's fields [(name, avro type, union)], avro type in
        boolean / int / long / float / double / string / bytes, union 0 (plain), 1 (["null", T]) or
        2 ([T, "null"]); registered under avro_schema_id (-1: any id)."""
        self.lib = lib
        tmap = dict(TYPE, STRING=TYPE_STRING)
        self._ft = (i32 * len(fields))(*[tmap[t] for _, t, _ in fields])
        self._fn = (C.c_char_p * len(fields))(*[n.encode() for n, _, _ in fields])
        self._fo = (i32 * len(fields))(*[o for _, _, o in fields])
        self.n_out = max([o for _, _, o in fields] + [-1]) + 1
        aw = avro_schema or []
        self._an = (C.c_char_p * max(len(aw), 1))(*[n.encode() for n, _, _ in aw])
        self._at = (i32 * max(len(aw), 1))(*[AVRO_TYPE[t] for _, t, _ in aw])
        self._au = (i32 * max(len(aw), 1))(*[u for _, _, u in aw])
        self.desc = SerdeDesc(FMT[key_format], tmap[key_type], FMT[value_format], len(fields), self._ft, self._fn,
                              self._fo, ord(delimiter), device, avro_schema_id, len(aw), self._an, self._at,
                              self._au)
        self.h = C.c_void_p()
        lib.check(lib.serde_create(C.byref(self.desc), C.byref(self.h)), "serde_create")

    def decode(self, ts, keys, values):
        """ts: int64 array; keys / values: lists of bytes or None (host batch).  Returns (batch
        object usable by AggHandle.push / TableHandle.upsert, n_errors)."""
        n = len(ts)
        keep = {}

        def pack(items):
            offs = np.zeros(n + 1, np.int64)
            offs[1:] = np.cumsum([0 if x is None else len(x) for x in items])
            data = np.frombuffer(b"".join(b"" if x is None else x for x in items) + b"\0", np.uint8).copy()
            valid = bitmap([x is not None for x in items])
            return offs, data, valid
        ts = np.ascontiguousarray(ts, np.int64)
        koff, kbytes, kval = pack(keys) if keys is not None else (None, None, None)
        voff, vbytes, vval = pack(values)
        keep.update(ts=ts, koff=koff, kbytes=kbytes, kval=kval, voff=voff, vbytes=vbytes, vval=vval)
        raw = RawBatch(n, MEM_HOST, _ptr(ts), _ptr(koff), _ptr(kbytes), _ptr(kval), _ptr(voff), _ptr(vbytes),
                       _ptr(vval))
        out = Batch()
        nerr = i64()
        self.lib.check(self.lib.serde_decode(self.h, C.byref(raw), C.byref(out), C.byref(nerr)), "serde_decode")

        class _Decoded:
            pass
        d = _Decoded()
        d.struct = out
        d._keep = keep
        return d, nerr.value

    def decode_device(self, ts, key_offsets, key_bytes, value_offsets, value_bytes, key_valid=None,
                      value_valid=None):
        """Device raw batch (torch tensors, caller-owned and kept alive while the result is used)
        → (decoded batch, n_errors)."""
        p = lambda t: None if t is None else t.data_ptr()
        raw = RawBatch(int(ts.numel()), MEM_DEVICE, p(ts), p(key_offsets), p(key_bytes), p(key_valid),
                       p(value_offsets), p(value_bytes), p(value_valid))
        out = Batch()
        nerr = i64()
        self.lib.check(self.lib.serde_decode(self.h, C.byref(raw), C.byref(out), C.byref(nerr)), "serde_decode")

        class _Decoded:
            pass
        d = _Decoded()
        d.struct = out
        d._keep = (ts, key_offsets, key_bytes, value_offsets, value_bytes, key_valid, value_valid)
        return d, nerr.value

    def columns(self, decoded, out_types):
        """Copy a decoded batch's columns back to the host (for tests): dict of numpy arrays."""
        b = decoded.struct
        n = b.n_rows
        nb = (n + 7) // 8

        def dget(ptr, count, dtype):
            a = np.zeros(max(count, 1), dtype)
            if count and ptr:
                self.lib.check(_hip_copy(a, ptr, a.nbytes if count else 0), "copy")
            return a[:count]
        res = {"key_valid": np.unpackbits(dget(b.key_valid, nb, np.uint8), bitorder="little")[:n].astype(bool),
               "row_valid": np.unpackbits(dget(b.row_valid, nb, np.uint8), bitorder="little")[:n].astype(bool)}
        if b.key_i64:
            res["key"] = dget(b.key_i64, n, np.int64)
        cols, valid = [], []
        for c, t in enumerate(out_types):
            cols.append(dget(b.col_data[c], n, NP_TYPE[TYPE[t]] if t != "STRING" else np.int64))
            valid.append(np.unpackbits(dget(b.col_valid[c], nb, np.uint8), bitorder="little")[:n].astype(bool))
        res["cols"], res["valid"] = cols, valid
        return res

    def close(self):
        if self.h:
            self.lib.serde_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SinkHandle:
    """khip_sink_*: columnar rows → sink record bytes (windowed key, value or null), and GROUP BY
    columns → the serialized composite key."""

    def __init__(self, lib, key_format, key_cols, value_format, value_cols, window_kind="NONE", delimiter=",",
                 device=0):
        """key_cols: [(name, type)]; value_cols: [(name, type, src)] with src a rows column index or
        "WS" / "WE"; types INT32 / INT64 / DOUBLE / STRING (keys)."""
        self.lib = lib
        tmap = dict(TYPE, STRING=TYPE_STRING)
        nk, nv = len(key_cols), len(value_cols)
        self._kt = (i32 * max(nk, 1))(*[tmap[t] for _, t in key_cols])
        self._kn = (C.c_char_p * max(nk, 1))(*[n.encode() for n, _ in key_cols])
        self._vt = (i32 * max(nv, 1))(*[tmap[t] for _, t, _ in value_cols])
        self._vn = (C.c_char_p * max(nv, 1))(*[n.encode() for n, _, _ in value_cols])
        self._vs = (i32 * max(nv, 1))(*[SINK_SRC[s] if isinstance(s, str) else s for _, _, s in value_cols])
        self.key_cols, self.value_cols = key_cols, value_cols
        self.desc = SinkDesc(FMT[key_format], nk, self._kt, self._kn, WINDOW[window_kind], FMT[value_format], nv,
                             self._vt, self._vn, self._vs, ord(delimiter), device)
        self.h = C.c_void_p()
        lib.check(lib.sink_create(C.byref(self.desc), C.byref(self.h)), "sink_create")

    def key(self, batch, cols):
        """batch: a HostBatch (host columns) or any batch object with .struct; cols: per key column
        a numpy array (INT32 / INT64 / DOUBLE; or (array, bool validity)) or a list of str / bytes /
        None (STRING), host
        memory, or a dict {"data" | "offsets" + "bytes", "valid"} of device pointers for a device
        batch.  Returns a batch object whose key is the serialized key (UTF-8 key layout, usable by
        AggHandle.push on a UTF8 handle); NULL in any column = a null key."""
        keep = []
        kc = (KeyCol * len(cols))()
        for i, c in enumerate(cols):
            if isinstance(c, dict):
                kc[i] = KeyCol(c.get("data"), c.get("offsets"), c.get("bytes"), c.get("valid"))
                continue
            if isinstance(c, tuple):  # (numpy array, bool validity)
                a = np.ascontiguousarray(c[0])
                vb = bitmap(c[1])
                keep += [a, vb]
                kc[i].data, kc[i].valid = a.ctypes.data, _ptr(vb)
                continue
            if isinstance(c, np.ndarray):
                a = np.ascontiguousarray(c)
                keep.append(a)
                kc[i].data = a.ctypes.data
                continue
            enc = [None if x is None else (x.encode() if isinstance(x, str) else bytes(x)) for x in c]
            offs = np.zeros(len(enc) + 1, np.int64)
            offs[1:] = np.cumsum([0 if e is None else len(e) for e in enc]) if enc else []
            data = np.frombuffer(b"".join(e or b"" for e in enc) + b"\0", np.uint8).copy()
            vb = bitmap([e is not None for e in enc])
            keep += [offs, data, vb]
            kc[i].offsets, kc[i].bytes, kc[i].valid = offs.ctypes.data, data.ctypes.data, _ptr(vb)
        out = Batch()
        self.lib.check(self.lib.sink_key(self.h, C.byref(batch.struct), kc, C.byref(out)), "sink_key")

        class _Keyed:
            pass
        k = _Keyed()
        k.struct = out
        k._keep = (batch, kc, keep)
        return k

    def key_bytes(self, keyed):
        """Host copy of a keyed host batch's keys: list of bytes or None (null key)."""
        b = keyed.struct
        n = b.n_rows
        offs = np.ctypeslib.as_array(C.cast(b.key_offsets, C.POINTER(i64)), shape=(n + 1,))
        tot = int(offs[n]) if n else 0
        data = bytes(np.ctypeslib.as_array(C.cast(b.key_bytes, C.POINTER(C.c_uint8)), shape=(max(tot, 1),))[:tot])
        nb = (n + 7) // 8
        valid = np.unpackbits(np.ctypeslib.as_array(C.cast(b.key_valid, C.POINTER(C.c_uint8)), shape=(max(nb, 1),)),
                              bitorder="little")[:n].astype(bool)
        return [data[offs[i]:offs[i + 1]] if valid[i] else None for i in range(n)]

    def encode(self, snap, tombstone=None, key_serialized=False, device_out=False, align=0):
        """snap: a snapshot dict (AggHandle.snapshot() / changes() layout: key or key_bytes/key_offsets,
        ws, we, values, nulls); host rows.  Returns (keys, values): lists of bytes / None.
        device_out: into device buffers (the one-pass encoder), `align` bytes past 16-byte alignment."""
        n = int(snap["n"])
        keep = []

        def arr(a, dtype):
            a = np.ascontiguousarray(a, dtype)
            keep.append(a)
            return a.ctypes.data
        rows = SinkRows()
        rows.n_rows = n
        rows.mem = MEM_HOST
        rows.key_serialized = 1 if key_serialized else 0
        if snap.get("key_offsets") is None and len(snap.get("key", [])) and isinstance(snap["key"][0], (str, bytes)):
            enc = [k.encode("utf-8", "surrogateescape") if isinstance(k, str) else k for k in snap["key"]]
            snap = dict(snap, key_offsets=np.concatenate([[0], np.cumsum([len(e) for e in enc])]).astype(np.int64),
                        key_bytes=np.frombuffer(b"".join(enc) or b"\0", np.uint8)[:sum(len(e) for e in enc)])
        if snap.get("key_offsets") is not None:
            rows.key_offsets = arr(snap["key_offsets"], np.int64)
            rows.key_bytes = arr(np.concatenate([np.asarray(snap["key_bytes"], np.uint8), np.zeros(1, np.uint8)]), np.uint8)
        else:
            rows.key_i64 = arr(snap["key"], np.int64)
        rows.window_start = arr(snap["ws"], np.int64)
        rows.window_end = arr(snap["we"], np.int64)
        vals = snap.get("values", [])
        nulls = snap.get("nulls", [])
        cd = (C.c_void_p * max(len(vals), 1))()
        cn = (C.c_void_p * max(len(vals), 1))()
        for j, v in enumerate(vals):
            v = np.asarray(v)
            cd[j] = arr(v, v.dtype)
            cn[j] = arr(np.asarray(nulls[j], np.uint8), np.uint8) if j < len(nulls) and nulls[j] is not None else None
        rows.col_data = cd
        rows.col_null = cn
        if tombstone is not None:
            rows.tombstone = arr(np.asarray(tombstone, np.uint8), np.uint8)
        if device_out:
            return self._encode_device(rows, n, align)
        out = SinkOut()
        out.mem = MEM_HOST
        koff = np.zeros(n + 1, np.int64)
        voff = np.zeros(n + 1, np.int64)
        vnull = np.zeros(max(n, 1), np.uint8)
        out.key_offsets, out.value_offsets, out.value_null = koff.ctypes.data, voff.ctypes.data, vnull.ctypes.data
        st = self.lib.sink_encode(self.h, C.byref(rows), C.byref(out))
        if st == KHIP_E_BUFFER:
            kb = np.zeros(max(out.key_len, 1), np.uint8)
            vb = np.zeros(max(out.value_len, 1), np.uint8)
            out.key_capacity, out.value_capacity = out.key_len, out.value_len
            out.key_bytes, out.value_bytes = kb.ctypes.data, vb.ctypes.data
            st = self.lib.sink_encode(self.h, C.byref(rows), C.byref(out))
        else:
            kb = vb = np.zeros(1, np.uint8)
        self.lib.check(st, "sink_encode")
        kbs, vbs = kb.tobytes(), vb.tobytes()
        keys = [kbs[koff[i]:koff[i + 1]] for i in range(n)]
        values = [None if vnull[i] else vbs[voff[i]:voff[i + 1]] for i in range(n)]
        return keys, values

    def _encode_device(self, rows, n, align):
        """encode() into device outputs (tests): a first call with 1-byte capacities (KHIP_E_BUFFER
        unless everything fits), then buffers of the exact sizes starting `align` bytes into a
        0xAB-filled allocation with 16 guard bytes either side, which must come back untouched."""
        import torch
        dev = torch.device("cuda")
        koff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        voff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        vnull = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        out = SinkOut()
        out.mem = MEM_DEVICE
        out.key_offsets, out.value_offsets, out.value_null = koff.data_ptr(), voff.data_ptr(), vnull.data_ptr()
        small = torch.zeros(2, dtype=torch.uint8, device=dev)
        out.key_capacity = out.value_capacity = 1
        out.key_bytes = out.value_bytes = small.data_ptr()
        st = self.lib.sink_encode(self.h, C.byref(rows), C.byref(out))
        kl, vl = out.key_len, out.value_len
        if st == KHIP_E_BUFFER:
            assert kl > 1 or vl > 1, (kl, vl)
        else:
            self.lib.check(st, "sink_encode")
        g = 16 + align
        kbuf = torch.full((g + kl + 16,), 0xAB, dtype=torch.uint8, device=dev)
        vbuf = torch.full((g + vl + 16,), 0xAB, dtype=torch.uint8, device=dev)
        out.key_capacity, out.value_capacity = kl, vl
        out.key_bytes, out.value_bytes = kbuf.data_ptr() + g, vbuf.data_ptr() + g
        self.lib.check(self.lib.sink_encode(self.h, C.byref(rows), C.byref(out)), "sink_encode")
        assert (out.key_len, out.value_len) == (kl, vl)
        kb, vb = kbuf.cpu().numpy(), vbuf.cpu().numpy()
        for b, ln in ((kb, kl), (vb, vl)):
            assert (b[:g] == 0xAB).all() and (b[g + ln:] == 0xAB).all(), "write outside the output bytes"
        ko, vo, vn = koff.cpu().numpy(), voff.cpu().numpy(), vnull.cpu().numpy()
        assert ko[0] == 0 and vo[0] == 0 and ko[n] == kl and vo[n] == vl
        kbs, vbs = kb[g:g + kl].tobytes(), vb[g:g + vl].tobytes()
        keys = [kbs[ko[i]:ko[i + 1]] for i in range(n)]
        values = [None if vn[i] else vbs[vo[i]:vo[i + 1]] for i in range(n)]
        return keys, values

    def close(self):
        if self.h:
            self.lib.sink_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _hip_copy(dst, src_ptr, nbytes):
    """Device → host copy through torch's HIP runtime (tests only)."""
    import torch
    t = torch.from_numpy(dst.view(np.uint8).reshape(-1))
    if nbytes:
        # wrap the device pointer as a torch tensor via the CUDA array interface
        class _Dev:
            __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (int(src_ptr), False), "version": 2}
        t[:nbytes].copy_(torch.as_tensor(_Dev(), device="cuda"))
    return KHIP_OK

