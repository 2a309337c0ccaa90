"""Helpers that replay the extracted QTT golden cases (tests/golden/qtt_*.json)
through either library (product or oracle) and compare the final table state the
way the reference's ExpectedRecordComparator does
(F/tools/ExpectedRecordComparator.java:133-152: integers exact, doubles |Δ| < 1e-6).
"""
import json
import math
import os

import numpy as np

from ksql_amd import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_cases(kind):
    with open(os.path.join(GOLDEN, "qtt_%s.json" % kind)) as f:
        return json.load(f)["cases"]


def case_desc(case, device=0, flags=0, changelog=True):
    d = case["desc"]
    return abi.make_agg_desc(d["window_kind"], d["key_type"], d["size_ms"], d["advance_ms"],
                             d["grace_ms"], d["col_types"],
                             [(a["kind"], a["arg_col"]) for a in d["aggs"]], device=device,
                             flags=flags | (abi.FLAG_CHANGELOG if changelog else 0),
                             retention_ms=d.get("retention_ms", -1),
                             emit=d.get("emit", "CHANGES"), having=d["having"])


def case_batch(case, lo=0, hi=None):
    d = case["desc"]
    rows = case["input"][lo:hi]
    ts = [r["ts"] for r in rows]
    key_valid = [r["key"] is not None for r in rows]
    row_valid = [r["row_valid"] for r in rows]
    cols, cvalid = [], []
    for ci, t in enumerate(d["col_types"]):
        vals = [r["cols"][ci] for r in rows]
        dt = abi.NP_TYPE[abi.TYPE[t]]
        cols.append(np.array([0 if v is None else v for v in vals], dtype=dt))
        cvalid.append([v is not None for v in vals])
    if d["key_type"] == "UTF8":
        return abi.HostBatch(ts, utf8_keys=[r["key"] for r in rows], key_valid=key_valid,
                             row_valid=row_valid, cols=cols, col_valid=cvalid)
    return abi.HostBatch(ts, keys=[0 if r["key"] is None else r["key"] for r in rows],
                         key_valid=key_valid, row_valid=row_valid, cols=cols, col_valid=cvalid)


def _rows_of(chg):
    """khip_agg_changes output → list of row dicts (emission order)."""
    out = []
    for i in range(chg["n"]):
        k = chg["key"][i]
        out.append({"key": k if isinstance(k, str) else int(k), "ws": int(chg["ws"][i]), "we": int(chg["we"][i]),
                    "rowtime": int(chg["rowtime"][i]), "tombstone": bool(chg["tombstone"][i]),
                    "values": [v[i].item() for v in chg["values"]], "nulls": [bool(x[i]) for x in chg["nulls"]]})
    return out


def run_agg_outputs(lib, case, split=None, device=0, flags=0):
    """The emitted changelog: pushes of `split` rows (None = one batch), the rows each push emits
    (khip_agg_changes), concatenated in emission order."""
    h = abi.AggHandle(lib, case_desc(case, device, flags))
    n = len(case["input"])
    step = n if not split else split
    rows = []
    for lo in range(0, max(n, 1), max(step, 1)):
        h.push(case_batch(case, lo, lo + step))
        rows += _rows_of(h.changes())
    h.close()
    return rows


def fold(rows):
    """Changelog → final table (last row per (key, window), tombstones delete), snapshot layout."""
    state = {}
    for r in rows:
        state[(r["key"], r["ws"])] = None if r["tombstone"] else r
    live = sorted((r for r in state.values() if r is not None),
                  key=lambda r: ((r["key"].encode() if isinstance(r["key"], str) else r["key"]), r["ws"]))
    na = len(live[0]["values"]) if live else 0
    return {"n": len(live), "key": [r["key"] for r in live], "ws": np.array([r["ws"] for r in live], np.int64),
            "we": np.array([r["we"] for r in live], np.int64), "rowtime": np.array([r["rowtime"] for r in live], np.int64),
            "values": [np.array([r["values"][a] for r in live]) for a in range(na)],
            "nulls": [np.array([r["nulls"][a] for r in live], bool) for a in range(na)]}


def run_agg_store(lib, case, split=None, device=0, flags=0):
    """The window store after every record (khip_agg_snapshot with the query's HAVING): what a
    pull query sees — retention applied, tombstoned rows absent."""
    h = abi.AggHandle(lib, case_desc(case, device, flags, changelog=False))
    n = len(case["input"])
    step = n if not split else split
    for lo in range(0, max(n, 1), max(step, 1)):
        h.push(case_batch(case, lo, lo + step))
    snap = h.snapshot(case["desc"]["having"])
    h.close()
    return snap


def run_agg_case(lib, case, split=None, device=0, flags=0):
    """The final table the query emitted (fold of its changelog; the reference's expected final
    state is the last output per (key, window)).  split: None = one batch; k = batches of k rows."""
    return fold(run_agg_outputs(lib, case, split, device, flags))


def run_tagg_case(lib, case, split=None, device=0):
    """Table aggregation (khip_agg_push_table): the source table's changelog in pushes of `split`
    rows, then the materialized table with the query's HAVING."""
    d = case["desc"]
    desc = abi.make_agg_desc(d["window_kind"], d["key_type"], 0, 0, -1, d["col_types"],
                             [(a["kind"], a["arg_col"]) for a in d["aggs"]], device=device,
                             flags=abi.FLAG_TABLE_SOURCE)
    h = abi.AggHandle(lib, desc)
    n = len(case["input"])
    step = n if not split else split
    for lo in range(0, max(n, 1), max(step, 1)):
        rows = case["input"][lo:lo + step]
        pk = [r["src_key"] for r in rows]
        if d["src_key_type"] == "UTF8":
            h.push_table(case_batch(case, lo, lo + step), src_utf8_keys=pk)
        else:
            h.push_table(case_batch(case, lo, lo + step), src_keys=[0 if k is None else k for k in pk],
                         src_key_valid=[k is not None for k in pk])
    snap = h.snapshot(d["having"])
    h.close()
    return snap


def compare_outputs(case, rows):
    """Emitted rows vs the QTT expected output sequence, in order (1-row pushes = the reference's
    cache-off, emit-every-record run).  Returns mismatch descriptions."""
    exp = case["outputs"]
    errs = []
    if len(rows) != len(exp):
        errs.append("output count %d != expected %d" % (len(rows), len(exp)))
    for i, (r, e) in enumerate(zip(rows, exp)):
        if r["key"] != e["key"] or r["ws"] != e["ws"] or r["we"] != e["we"]:
            errs.append("out %d (%r,%d,%d) != (%r,%d,%d)" % (i, r["key"], r["ws"], r["we"], e["key"], e["ws"], e["we"]))
            continue
        if r["tombstone"] != e["tombstone"]:
            errs.append("out %d tombstone %r != %r" % (i, r["tombstone"], e["tombstone"]))
            continue
        if e["rowtime"] is not None and r["rowtime"] != e["rowtime"]:
            errs.append("out %d timestamp %d != %d" % (i, r["rowtime"], e["rowtime"]))
        if e["tombstone"]:
            continue
        for a, (v, present) in enumerate(zip(e["values"], e["present"])):
            if not present:
                continue
            if v is None:
                if not r["nulls"][a]:
                    errs.append("out %d agg %d expected null" % (i, a))
            elif r["nulls"][a]:
                errs.append("out %d agg %d unexpected null" % (i, a))
            elif not _num_eq(r["values"][a], v):
                errs.append("out %d agg %d %r != %r" % (i, a, r["values"][a], v))
    return errs


def _num_eq(a, b):
    if isinstance(b, float) or isinstance(a, float):
        if math.isnan(b) and math.isnan(a):
            return True
        return abs(float(a) - float(b)) < 1e-6
    return int(a) == int(b)


def compare_agg(case, snap):
    """Return a list of mismatch descriptions (empty = parity)."""
    errs = []
    exp = case["expected"]
    if snap["n"] != len(exp):
        errs.append("row count %d != expected %d" % (snap["n"], len(exp)))
        return errs
    for i, e in enumerate(exp):
        k = snap["key"][i]
        if (k if isinstance(k, str) else int(k)) != e["key"]:
            errs.append("row %d key %r != %r" % (i, k, e["key"]))
            continue
        if int(snap["ws"][i]) != e["ws"] or int(snap["we"][i]) != e["we"]:
            errs.append("row %d window (%d,%d) != (%d,%d)" % (i, snap["ws"][i], snap["we"][i], e["ws"], e["we"]))
        if e["rowtime"] is not None and int(snap["rowtime"][i]) != e["rowtime"]:
            errs.append("row %d rowtime %d != %d" % (i, snap["rowtime"][i], e["rowtime"]))
        for a, (v, present) in enumerate(zip(e["values"], e["present"])):
            if not present:
                continue
            isnull = bool(snap["nulls"][a][i])
            if v is None:
                if not isnull:
                    errs.append("row %d agg %d expected null" % (i, a))
            elif isnull:
                errs.append("row %d agg %d unexpected null" % (i, a))
            elif not _num_eq(snap["values"][a][i].item(), v):
                errs.append("row %d agg %d %r != %r" % (i, a, snap["values"][a][i].item(), v))
    return errs


# ---------------------------------------------------------------- join cases

def _ctype(t):
    return {"INT32": "INT32", "INT64": "INT64", "DOUBLE": "DOUBLE", "STRING": "INT32"}[t]


def run_join_case(lib, case, device=0):
    """Replays the interleaved table/stream inputs: consecutive table records are one
    upsert batch, consecutive stream records one probe batch.  Returns the emitted
    rows as dicts in the output schema (strings decoded from dictionary codes)."""
    tcols = case["table_cols"]
    scols = case["stream_cols"]
    dictionary = {}
    rev = {}

    def code(s):
        if s not in dictionary:
            dictionary[s] = len(dictionary)
            rev[dictionary[s]] = s
        return dictionary[s]

    if case["where"] is not None and isinstance(case["where"]["value"], str):
        code(case["where"]["value"])
    utf8 = case.get("key_type", "INT64") == "UTF8"
    th = abi.TableHandle(lib, [_ctype(c["type"]) for c in tcols], device=device, key_type="UTF8" if utf8 else "INT64")
    where = None
    if case["where"] is not None:
        wc = [c["name"] for c in tcols].index(case["where"]["col"])
        wv = case["where"]["value"]
        where = {"col": wc, "op": case["where"]["op"], "i64": code(wv) if isinstance(wv, str) else int(wv),
                 "f64": float(code(wv) if isinstance(wv, str) else wv)}
    out_rows = []
    events = case["events"]
    i = 0
    while i < len(events):
        j = i
        side = events[i]["side"]
        while j < len(events) and events[j]["side"] == side:
            j += 1
        grp = events[i:j]
        ts = [e["ts"] for e in grp]
        kvalid = [e["key"] is not None for e in grp]
        if utf8:  # STRING keys: serialized UTF-8 bytes
            kargs = {"utf8_keys": [None if e["key"] is None else str(e["key"]) for e in grp]}
        else:
            kargs = {"keys": [0 if e["key"] is None else int(e["key"]) for e in grp]}
        rvalid = [e["value"] is not None for e in grp]
        if side == "T":
            cols, cval = [], []
            for c in tcols:
                vals = [None if e["value"] is None else e["value"].get(c["name"]) for e in grp]
                if c["type"] == "STRING":
                    arr = np.array([0 if v is None else code(v) for v in vals], np.int32)
                else:
                    arr = np.array([0 if v is None else v for v in vals], abi.NP_TYPE[abi.TYPE[c["type"]]])
                cols.append(arr)
                cval.append([v is not None for v in vals])
            th.upsert(abi.HostBatch(ts, key_valid=kvalid, row_valid=rvalid, cols=cols, col_valid=cval, **kargs))
        else:
            b = abi.HostBatch(ts, key_valid=kvalid, row_valid=rvalid, **kargs)
            res = th.probe(b, case["join_type"], where)
            for r in range(res["n"]):
                e = grp[int(res["stream_row"][r])]
                row = {}
                for s in case["select"]:
                    if s["side"] == "S":
                        if any(c["name"] == s["col"] for c in scols):
                            row[s["name"]] = e["value"].get(s["col"])
                        else:
                            row[s["name"]] = e["key"]  # the stream key column
                    else:
                        if s["col"] not in [c["name"] for c in tcols]:
                            row[s["name"]] = e["key"] if res["matched"][r] else None
                            continue
                        ci = [c["name"] for c in tcols].index(s["col"])
                        if res["nulls"][ci][r]:
                            row[s["name"]] = None
                        else:
                            v = res["cols"][ci][r].item()
                            row[s["name"]] = rev[v] if tcols[ci]["type"] == "STRING" else v
                out_rows.append({"key": e["key"], "ts": e["ts"], "value": row})
        i = j
    th.close()
    return out_rows


_DEFAULT = {"INT32": 0, "INT64": 0, "DOUBLE": 0.0, "STRING": ""}


def compare_join(case, rows):
    errs = []
    exp = case["expected"]
    if case.get("null_as_default"):  # PROTOBUF output: a NULL column is written as its default
        types = {c["name"]: c["type"] for c in case["stream_cols"] + case["table_cols"]}
        rows = [dict(r, value={k: (_DEFAULT.get(types.get(k)) if v is None and k in types else v)
                               for k, v in r["value"].items()}) for r in rows]
    if len(rows) != len(exp):
        return ["row count %d != expected %d" % (len(rows), len(exp))]
    for i, (r, e) in enumerate(zip(rows, exp)):
        if e["ts"] is not None and r["ts"] != e["ts"]:
            errs.append("row %d ts %r != %r" % (i, r["ts"], e["ts"]))
        for name, v in e["value"].items():
            got = r["value"].get(name, "<missing>")
            if got == "<missing>" and name not in r["value"]:
                # key column projected into the value (e.g. T_ID) is carried as the key
                continue
            if v is None or got is None:
                if v is not got:
                    errs.append("row %d col %s %r != %r" % (i, name, got, v))
            elif isinstance(v, (int, float)) and not isinstance(v, bool):
                if not _num_eq(got, v):
                    errs.append("row %d col %s %r != %r" % (i, name, got, v))
            elif got != v:
                errs.append("row %d col %s %r != %r" % (i, name, got, v))
    return errs
