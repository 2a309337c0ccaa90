"""Oracle-side restatement of the repartition contract (include/ksqldb_hip.h khip_shuffle_*):
routing by Kafka's default partitioner (oracle rule R8, murmur2 pinned by Kafka's published
vectors), the packed row layout, and its inverse.  Test infrastructure only."""
import numpy as np


def kafka_partition(orc, keys, width, n_parts):
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    out = np.zeros(len(keys), np.int32)
    orc.dll.oracle_kafka_partition(keys.ctypes.data, len(keys), width, n_parts, out.ctypes.data)
    return out


def _raw_i64(col):
    if col.dtype == np.float64:
        return col.view(np.int64)
    return col.astype(np.int64)


def expected_pack(orc, key_col, cols, col_valid, row_valid, ts, n_parts, stream_time=None):
    """khip_shuffle_pack restated: (rows int64 [m, 2+nc], counts per destination).  stream_time
    (KHIP_SHUFFLE_STREAM_TIME): one more word, before the validity word."""
    n = len(ts)
    width = 4 if cols[key_col].dtype == np.int32 else 8
    ok = row_valid & col_valid[key_col] & (ts >= 0)
    dest = kafka_partition(orc, cols[key_col], width, n_parts)
    nc = len(cols)
    st = 0 if stream_time is None else 1
    words = np.zeros((n, 2 + nc + st), np.int64)
    words[:, 0] = cols[key_col].astype(np.int64)
    words[:, 1] = ts
    vm = np.zeros(n, np.int64)
    w = 2
    for c in range(nc):
        vm |= (col_valid[c].astype(np.int64) << c)
        if c == key_col:
            continue
        words[:, w] = np.where(col_valid[c], _raw_i64(cols[c]), 0)
        w += 1
    if st:
        words[:, w] = stream_time
        w += 1
    words[:, w] = vm
    rows, counts = [], []
    for d in range(n_parts):
        sel = np.nonzero(ok & (dest == d))[0]  # arrival order
        rows.append(words[sel])
        counts.append(len(sel))
    return np.concatenate(rows), counts


def expected_unpack(rows, key_col, col_types):
    """khip_shuffle_unpack restated: packed rows → (key, ts, cols, col_valid bool arrays)."""
    nc = len(col_types)
    vm = rows[:, 2 + nc - 1] if nc else np.zeros(len(rows), np.int64)
    cols, valid = [], []
    w = 2
    for c, t in enumerate(col_types):
        valid.append(((vm >> c) & 1).astype(bool))
        if c == key_col:
            raw = rows[:, 0]
        else:
            raw = rows[:, w]
            w += 1
        cols.append(raw.astype(np.int32) if t == "INT32" else (raw.view(np.float64) if t == "DOUBLE" else raw.copy()))
    return rows[:, 0].copy(), rows[:, 1].copy(), cols, valid
