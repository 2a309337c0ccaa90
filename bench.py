#!/usr/bin/env python3
"""Headline benchmark: windowed GROUP BY records/sec on MI355X (BASELINE.json metric).

Workload (N=1): BASELINE.json configs[1], "possible_fraud":
    CREATE TABLE possible_fraud AS SELECT card_number, COUNT(*) FROM ...
    WINDOW TUMBLING (SIZE 5 SECONDS) GROUP BY card_number HAVING COUNT(*) > 3;
  100M records, 10M distinct card numbers (BIGINT form), 10 s of event time with
  <= 500 ms disorder (ksql_amd/synth.py).  One step = a fresh query instance over the
  whole workload: reset the HBM table, push the 100M device-resident records through
  the C ABI (stream time, late drop, window assignment, (key, window) upsert), and
  materialize the HAVING result count on the device.  Inputs are generated in HBM
  before the timed region; the PCIe-inclusive rate is reported separately
  (DESIGN.md).

Multi-GPU (torchrun): weak scaling, one process per GPU.  Rank r owns the card numbers
k with k % N == r (key-hash sharding = Kafka partitioning) and processes its own 100M
records with its own stream time (one Kafka task per partition): no data-path
collective.  value = all records / max-over-ranks time.

Output: one JSON line (rank 0) with `roofline` for the hot path (the device time of every
kernel of one push, HIP events on the library's own stream; per-kernel breakdown with each
kernel's own streamed bytes) and `cpu_baseline` (the C oracle, a
single-threaded restatement of the reference semantics — the JVM reference cannot run
on this image — timed on a bounded prefix of the same workload).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
BYTES_PER_RECORD_C2 = 80  # W_in 16 + F(1) * 2 * S_slot(32)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--records", type=int, default=100_000_000)
    ap.add_argument("--keys", type=int, default=10_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--engine", choices=["part", "atomic"], default="part")
    ap.add_argument("--config", choices=["possible_fraud", "hopping_double", "clickstream_join", "repartition_sum"],
                    default="possible_fraud",
                    help="possible_fraud = BASELINE configs[1] (the headline); hopping_double = configs[2]; "
                         "clickstream_join = configs[3]; repartition_sum = configs[4]")
    ap.add_argument("--slice", type=int, default=1 << 27, help="hopping_double: records per micro-batch push")
    ap.add_argument("--users", type=int, default=100_000_000, help="clickstream_join: table rows")
    return ap.parse_args()


def cpu_baseline(n_total, keys, target_s):
    """Oracle (single-threaded C restatement) on a prefix of the same workload."""
    from ksql_amd import abi, synth
    orc = abi.load_oracle()

    def run(m):
        card, ts = synth.possible_fraud(0, m, n_total, keys=keys)
        b = abi.HostBatch(ts, keys=card)
        h = abi.AggHandle(orc, abi.make_agg_desc(window_kind="TUMBLING", size_ms=5000, key_type="INT64",
                                                 aggs=[("COUNT_STAR", -1)]))
        t0 = time.perf_counter()
        h.push(b, stats=False)
        dt = time.perf_counter() - t0
        h.close()
        return dt

    m = 1_000_000
    dt = run(m)
    m2 = int(min(max(m * target_s / max(dt, 1e-3), m), 60_000_000))
    if m2 > m:
        m, dt = m2, run(m2)
    return {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
            "sample": "first %d of the %d possible_fraud records (C oracle, 1 thread, %.1f s)" % (m, n_total, dt)}


def load_traffic(path, n, engine):
    """HBM bytes per push from the committed PMC summary (tools/pmc_traffic.py), if it was
    measured on this workload size and engine."""
    try:
        with open(path) as f:
            t = json.load(f)
        rec = t.get("possible_fraud", {}).get("push" if engine == "part" else "k_apply")
        if rec and rec.get("records") == n:
            return rec["hbm_bytes_per_launch"]
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from ksql_amd import abi, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    lib = abi.load_product()
    if args.config == "repartition_sum":
        return bench_repartition(args, lib, rank, world, local)
    if args.config == "hopping_double":
        return bench_hopping_double(args, lib, rank, world, local)
    if args.config == "clickstream_join":
        return bench_join(args, lib, rank, world, local)

    n = args.records
    card, ts = synth.possible_fraud(0, n, n, xp="torch", device="cuda", rank=rank, world=world, keys=args.keys)
    torch.cuda.synchronize()
    batch = abi.DeviceBatch(ts, keys=card)
    desc = abi.make_agg_desc(window_kind="TUMBLING", size_ms=5000, key_type="INT64", aggs=[("COUNT_STAR", -1)],
                             device=local, capacity_hint=int(min(3 * args.keys, 2 * n)),
                             flags=abi.FLAG_PROFILE | (abi.FLAG_ENGINE_ATOMIC if args.engine == "atomic" else 0))
    h = abi.AggHandle(lib, desc)
    having = {"agg": 0, "op": "GT", "value": 3}

    def step():
        h.reset()
        st = h.push(batch)
        rows = h.count_rows(having)
        return st, rows

    for _ in range(max(args.warmup, 1)):
        st, rows = step()
    assert st["rows_accepted"] == n and st["windows_applied"] == n, st
    h.kernel_times(reset=True)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st, rows = step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kt = h.kernel_times()
    groups = int(h.count_rows(None))

    # PCIe-inclusive rate (host-resident input, one step) for DESIGN.md — not `value`
    pcie = None
    if rank == 0 and n <= 100_000_000:
        hb = abi.HostBatch(ts.cpu().numpy(), keys=card.cpu().numpy())
        h.reset()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        h.push(hb)
        h.count_rows(having)
        pcie = n / (time.perf_counter() - t1)

    # pull-query latency on the materialized table (khip_agg_get), not `value`
    pull = None
    if rank == 0:
        qk = card[: 1 << 12].cpu().numpy()
        pull = {}
        for nk in (1, 100, 4096):
            h.get(qk[:nk])  # warm
            t1 = time.perf_counter()
            reps = 5
            for _ in range(reps):
                r = h.get(qk[:nk])
            pull["keys_%d_ms" % nk] = (time.perf_counter() - t1) * 1000.0 / reps
            pull["keys_%d_rows" % nk] = int(r["n"])

    if rank == 0:
        ms_step = elapsed * 1000.0 / args.steps
        value = world * n * args.steps / elapsed
        launches = max(kt["apply_launches"], 1)
        phase = {k: kt[k] / launches for k in ("stream_time_ms", "partition_ms", "apply_ms", "finalize_ms")}
        push_ms = sum(phase.values())  # device time of every kernel of one push (HIP events)
        achieved = BYTES_PER_RECORD_C2 * n / (push_ms / 1000.0) / 1e9
        traffic = load_traffic(args.traffic_json, n, args.engine)
        # each kernel's own algorithmic streams (bytes / record) for the breakdown
        own = ({"stream_time_ms": 16, "partition_ms": 32, "apply_ms": 16 + 32.0 * groups / n, "finalize_ms": 0}
               if args.engine == "part" else
               {"stream_time_ms": 8, "partition_ms": 0, "apply_ms": 80, "finalize_ms": 0})
        per_kernel = {k: {"ms": phase[k], "bytes_per_record": own[k],
                          "GB/s": own[k] * n / (phase[k] / 1000.0) / 1e9 if phase[k] > 0 else None}
                      for k in phase if phase[k] > 0}
        out = {
            "metric": "records/sec, windowed GROUP BY (COUNT(*) TUMBLING 5 s GROUP BY card_number HAVING > 3)",
            "value": value,
            "unit": "records/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (splitmix64, ksql_amd/synth.py), device-resident columnar batch",
            "config": {"workload": "possible_fraud", "records_per_gpu": n, "keys_per_gpu": args.keys,
                       "window": "TUMBLING 5s, grace default", "having": "COUNT(*) > 3",
                       "groups_per_gpu": groups, "having_rows_per_gpu": int(rows),
                       "parallelism": "key-hash shards x%d" % world},
            "roofline": {"bound": "hbm",
                         "kernel": ("khip_agg_push = k_part_hist + scans + k_part_scatter + k_part_agg + commit"
                                    if args.engine == "part" else "khip_agg_push (k_apply dominant)"),
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_record": BYTES_PER_RECORD_C2, "push_ms": push_ms,
                         "engine": args.engine, "per_kernel": per_kernel},
            "pcie_inclusive_records_per_s": pcie,
            "pull_query": pull,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(n, args.keys, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out))
    h.close()
    if world > 1:
        dist.destroy_process_group()


def stream_copy_gbs(nbytes=1 << 31):
    """Achievable HBM rate on this box: one device-to-device copy of `nbytes` (read + write
    bytes / time), the practical ceiling next to the 8 TB/s spec peak."""
    import torch
    a = torch.empty(nbytes // 8, dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    del a, b
    return 2.0 * nbytes / (ms / 1000.0) / 1e9


def barrier_sync(world):
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(elapsed, world):
    import torch
    import torch.distributed as dist
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def finish(world):
    import torch.distributed as dist
    if world > 1:
        dist.destroy_process_group()


BYTES_PER_RECORD_C3 = 24.125 + 6 * 2 * 56  # W_in + F x 2 x S_slot = 696.1


def bench_hopping_double(args, lib, rank, world, local):
    """C3: HOPPING (SIZE 1 MINUTE, ADVANCE BY 10 SECONDS, GRACE PERIOD 1 MINUTE) SUM/AVG/MIN/MAX
    of a DOUBLE with 1 % nulls, 1e9 records (1 h of event time) per GPU, key BIGINT in [0, 1e5).
    One step = a fresh query instance: reset, the 1e9 device-resident records pushed as
    event-time micro-batches of `--slice` records (closed windows leave the live table between
    pushes), and the materialized row count."""
    import torch
    from ksql_amd import abi, synth
    n = args.records if args.records != 100_000_000 else 1_000_000_000
    S = max(8, args.slice // 8 * 8)
    cfg = synth.CONFIGS["hopping_double"]
    key, ts, val, valid = synth.hopping_double(0, n, n, xp="torch", device="cuda", rank=rank, world=world)
    vb = abi.bitmap_torch(valid)
    del valid
    torch.cuda.synchronize()
    batches = [abi.DeviceBatch(ts[lo:min(lo + S, n)], keys=key[lo:min(lo + S, n)], cols=[val[lo:min(lo + S, n)]],
                               col_valid=[vb[lo // 8:(min(lo + S, n) + 7) // 8]]) for lo in range(0, n, S)]
    keys_here = cfg["keys"] // world
    span_push = cfg["span_ms"] * S / n
    live = int(keys_here * (span_push + cfg["size_ms"] + cfg["grace_ms"] + cfg["disorder_ms"]) / cfg["advance_ms"])
    desc = abi.make_agg_desc(window_kind="HOPPING", size_ms=cfg["size_ms"], advance_ms=cfg["advance_ms"],
                             grace_ms=cfg["grace_ms"], key_type="INT64", col_types=["DOUBLE"],
                             aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0)], device=local,
                             capacity_hint=live, flags=abi.FLAG_PROFILE)
    h = abi.AggHandle(lib, desc)

    def step():
        h.reset()
        tot = {"rows_accepted": 0, "windows_applied": 0, "windows_late": 0}
        for b in batches:
            st = h.push(b)
            for k in tot:
                tot[k] += st[k]
        return tot, h.count_rows(None)

    for _ in range(max(args.warmup, 1)):
        st, groups = step()
    h.kernel_times(reset=True)
    barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st, groups = step()
    barrier_sync(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    kt = h.kernel_times()
    if rank == 0:
        ms_step = elapsed * 1000.0 / args.steps
        phase = {k: kt[k] / args.steps for k in ("stream_time_ms", "partition_ms", "apply_ms", "finalize_ms")}
        push_ms = sum(phase.values())  # device time of every kernel of the step's pushes (HIP events)
        achieved = BYTES_PER_RECORD_C3 * n / (push_ms / 1000.0) / 1e9
        out = {
            "metric": "records/sec, windowed GROUP BY (SUM/AVG/MIN/MAX(value DOUBLE) HOPPING 60 s / 10 s GROUP BY key)",
            "value": world * n * args.steps / elapsed, "unit": "records/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (splitmix64, ksql_amd/synth.py hopping_double), device-resident columnar batch",
            "config": {"workload": "hopping_double", "records_per_gpu": n, "keys_per_gpu": keys_here,
                       "window": "HOPPING 60s/10s GRACE 60s (F=6)", "micro_batch": S, "pushes": len(batches),
                       "windows_applied": st["windows_applied"], "windows_late": st["windows_late"],
                       "groups_per_gpu": int(groups), "parallelism": "key-hash shards x%d" % world},
            "roofline": {"bound": "hbm", "kernel": "khip_agg_push (all kernels of every micro-batch push)",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None, "algorithmic_bytes_per_record": BYTES_PER_RECORD_C3, "push_ms": push_ms,
                         "phase_ms_per_step": phase, "stream_copy_GBps": stream_copy_gbs()},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_hopping(n, args.cpu_seconds)
        print(json.dumps(out))
    h.close()
    finish(world)


def cpu_baseline_hopping(n_total, target_s):
    from ksql_amd import abi, synth
    orc = abi.load_oracle()
    cfg = synth.CONFIGS["hopping_double"]

    def run(m):
        key, ts, val, valid = synth.hopping_double(0, m, n_total)
        b = abi.HostBatch(ts, keys=key, cols=[val], col_valid=[valid])
        h = abi.AggHandle(orc, abi.make_agg_desc(window_kind="HOPPING", size_ms=cfg["size_ms"],
                                                 advance_ms=cfg["advance_ms"], grace_ms=cfg["grace_ms"],
                                                 key_type="INT64", col_types=["DOUBLE"],
                                                 aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0)]))
        t0 = time.perf_counter()
        h.push(b, stats=False)
        dt = time.perf_counter() - t0
        h.close()
        return dt

    m = 500_000
    dt = run(m)
    m2 = int(min(max(m * target_s / max(dt, 1e-3), m), 40_000_000))
    if m2 > m:
        m, dt = m2, run(m2)
    return {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
            "sample": "first %d of the %d hopping_double records (C oracle, 1 thread, %.1f s)" % (m, n_total, dt)}


def cpu_baseline_join(users, target_s):
    """Oracle stream-table LEFT JOIN (oracle_table_probe, 1 thread).  Bounded sample: a users
    table of min(users, 1e7) rows built first (untimed), then clicks drawn over the same
    1.1x id span probed against it (timed), WHERE level = 'Platinum'."""
    from ksql_amd import abi, synth
    orc = abi.load_oracle()
    U = min(users, 10_000_000)
    uid, level = synth.users_table(0, U)
    t = abi.TableHandle(orc, ["INT32"], capacity_hint=U)
    t.upsert(abi.HostBatch(np.zeros(U, np.int64), keys=uid, cols=[level.astype(np.int32)]))
    where = {"col": 0, "op": "EQ", "i64": synth.LEVELS.index("Platinum")}

    def run(m):
        cu, cts = synth.clicks(0, m, U, seed_clicks=5)
        b = abi.HostBatch(cts, keys=cu)
        t0 = time.perf_counter()
        t.probe(b, "LEFT", where)
        return time.perf_counter() - t0

    m = 1_000_000
    dt = run(m)
    m2 = int(min(max(m * target_s / max(dt, 1e-3), m), 50_000_000))
    if m2 > m:
        m, dt = m2, run(m2)
    t.close()
    return {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
            "sample": "%d clicks probed against a %d-row users table (C oracle, 1 thread, %.1f s)" % (m, U, dt)}


def cpu_baseline_repartition(n_total, target_s):
    """Oracle C5 step on a prefix of rank 0's source partition (1 thread): Kafka partitioner of
    the new key (oracle_kafka_partition, 8 destinations) + SUM(amount) TUMBLING 1 MINUTE
    GROUP BY region_id (oracle_agg_push)."""
    from ksql_amd import abi, synth
    orc = abi.load_oracle()

    def run(m):
        _eid, ts, region, amount = synth.repartition_sum(0, m, n_total)
        region = np.ascontiguousarray(region, np.int64)
        dest = np.empty(m, np.int32)
        h = abi.AggHandle(orc, abi.make_agg_desc(window_kind="TUMBLING", size_ms=60_000, key_type="INT64",
                                                 col_types=["INT64"], aggs=[("SUM", 0)]))
        b = abi.HostBatch(ts, keys=region, cols=[amount])
        t0 = time.perf_counter()
        orc.dll.oracle_kafka_partition(region.ctypes.data, m, 8, 8, dest.ctypes.data)
        h.push(b, stats=False)
        dt = time.perf_counter() - t0
        h.close()
        return dt

    m = 1_000_000
    dt = run(m)
    m2 = int(min(max(m * target_s / max(dt, 1e-3), m), 60_000_000))
    if m2 > m:
        m, dt = m2, run(m2)
    return {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
            "sample": "first %d of rank 0's %d repartition_sum records: partitioner + aggregate "
                      "(C oracle, 1 thread, %.1f s)" % (m, n_total, dt)}


def random_gather_rows_per_s(table_bytes, rows=100_000_000):
    """Practical ceiling of a hash probe into a table far larger than the caches: torch's
    gather of `rows` uniformly random 32-byte rows from a `table_bytes` table (one random
    line per row, the access pattern of a probe), in rows/s."""
    import torch
    tab = torch.empty(max(table_bytes // 32, 1), 4, dtype=torch.int64, device="cuda")
    idx = torch.randint(0, tab.shape[0], (rows,), device="cuda")
    out = tab[idx]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        out = tab[idx]
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    del tab, idx, out
    return rows / (ms / 1000.0)


BYTES_PER_PROBE_C4 = 31  # W_in 16 + table slot 8 + 0.30 x output 24


def bench_join(args, lib, rank, world, local):
    """C4: clickstream LEFT JOIN users WHERE level = 'Platinum'.  The 1e8-row users table is
    replicated in every GPU's HBM (built once, timed separately); each GPU probes its own
    1e9 clicks (weak scaling, no exchange).  One step = khip_table_probe_device over all
    clicks: row-aligned emit/matched bitmaps + the right column, then the emitted count."""
    import torch
    from ksql_amd import abi, synth
    n = args.records if args.records != 100_000_000 else 1_000_000_000
    U = args.users
    uid, level = synth.users_table(0, U, xp="torch", device="cuda")
    level = level.to(torch.int32)
    t = abi.TableHandle(lib, ["INT32"], device=local, capacity_hint=U)
    tb = abi.DeviceBatch(torch.zeros(U, dtype=torch.int64, device="cuda"), keys=uid, cols=[level])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t.upsert(tb)
    t.sync()
    build_s = time.perf_counter() - t0
    # khip_table_create: cap = next_pow2(4/3 x hint) slots of 32 bytes (one INT32 column)
    table_bytes = (1 << max(10, ((U * 4 + 2) // 3 - 1).bit_length())) * 32
    del tb, uid, level
    cu, cts = synth.clicks(0, n, U, xp="torch", device="cuda", seed_clicks=5 + 1000 * rank)
    batch = abi.DeviceBatch(cts, keys=cu)
    nb = (n + 7) // 8 + 8
    emit = torch.empty(nb, dtype=torch.uint8, device="cuda")
    matched = torch.empty(nb, dtype=torch.uint8, device="cuda")
    col = torch.empty(n, dtype=torch.int32, device="cuda")
    null = torch.empty(nb, dtype=torch.uint8, device="cuda")
    where = {"col": 0, "op": "EQ", "i64": synth.LEVELS.index("Platinum")}
    torch.cuda.synchronize()

    def step():
        return t.probe_device(batch, "LEFT", where, emit, matched, [col], [null])

    for _ in range(max(args.warmup, 1)):
        rows = step()
    barrier_sync(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rows = step()
    barrier_sync(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    if rank == 0:
        ms_step = elapsed * 1000.0 / args.steps
        achieved = BYTES_PER_PROBE_C4 * n / (ms_step / 1000.0) / 1e9
        out = {
            "metric": "stream records/sec, stream-table LEFT JOIN (clickstream x users WHERE level = 'Platinum')",
            "value": world * n * args.steps / elapsed, "unit": "records/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (splitmix64, ksql_amd/synth.py users_table/clicks), device-resident columnar batch",
            "config": {"workload": "clickstream_join", "table_rows": U, "clicks_per_gpu": n,
                       "table_build_s": build_s, "table_build_rows_per_s": U / build_s,
                       "emitted_rows_per_gpu": int(rows), "parallelism": "replicated table x%d" % world},
            "roofline": {"bound": "hbm", "kernel": "k_probe (khip_table_probe_device)", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "algorithmic_bytes_per_record": BYTES_PER_PROBE_C4, "stream_copy_GBps": stream_copy_gbs(),
                         "table_bytes": table_bytes,
                         "random_gather_rows_per_s": random_gather_rows_per_s(table_bytes)},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_join(U, args.cpu_seconds)
        print(json.dumps(out))
    t.close()
    finish(world)


BYTES_PER_RECORD_C5 = 136  # read 24 + pack 24 + recv 24 + 2 x 32 (slot)


def bench_repartition(args, lib, rank, world, local):
    """C5: GROUP BY region_id (a value column) forces the repartition.  One step per rank:
    khip_shuffle_pack (Kafka partitioner) → RCCL count exchange + all-to-all over xGMI (N>1)
    → khip_shuffle_unpack → SUM(amount) TUMBLING 1 MINUTE push → row count.  Weak scaling:
    every rank owns one source partition of `records` records (1e9 node-wide at N=8 with the
    default 125M)."""
    import torch
    import torch.distributed as dist
    from ksql_amd import abi, synth
    from ksql_amd.repartition import Repartition

    n = args.records if args.records != 100_000_000 else 125_000_000
    eid, ts, region, amount = synth.repartition_sum(0, n, n, xp="torch", device="cuda", rank=rank, world=world)
    torch.cuda.synchronize()
    src = abi.DeviceBatch(ts, cols=[region, amount])
    comm = None
    if world > 1:
        obj = [abi.comm_unique_id(lib) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = abi.Comm(lib, world, rank, obj[0], local)
    rp = Repartition(lib, 0, ["INT64", "INT64"], rank=rank, world=world, comm=comm, device=local)
    desc = abi.make_agg_desc(window_kind="TUMBLING", size_ms=60_000, key_type="INT64", col_types=["INT64", "INT64"],
                             aggs=[("SUM", 1)], device=local, capacity_hint=60 * 1_000_000 // max(world, 1),
                             flags=abi.FLAG_PROFILE)
    h = abi.AggHandle(lib, desc)
    phases = {"pack": 0.0, "exchange_unpack": 0.0, "aggregate": 0.0}

    def step(timed=False):
        t0 = time.perf_counter()
        send, counts = rp.shuffle.pack(src)
        t1 = time.perf_counter()
        if world > 1:
            recv, rc = comm.alltoall(send, counts, rp.shuffle.row_words)
        else:
            recv, rc = send, counts
        m = int(sum(rc))
        key, kts, cols, valid = rp.shuffle.unpack(recv, m)
        t2 = time.perf_counter()
        h.reset()
        st = h.push(abi.DeviceBatch(kts, keys=key, cols=cols, col_valid=valid))
        rows = h.count_rows(None)
        t3 = time.perf_counter()
        if timed:
            phases["pack"] += t1 - t0
            phases["exchange_unpack"] += t2 - t1
            phases["aggregate"] += t3 - t2
        return st, rows, m

    for _ in range(max(args.warmup, 1)):
        st, rows, m = step()
    assert st["rows_accepted"] == m, st
    h.kernel_times(reset=True)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    recv_total = 0
    for _ in range(args.steps):
        st, rows, m = step(timed=True)
        recv_total += m
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kt = h.kernel_times()
    if rank == 0:
        ms_step = elapsed * 1000.0 / args.steps
        per = {k: v * 1000.0 / args.steps for k, v in phases.items()}
        achieved = BYTES_PER_RECORD_C5 * n / (ms_step / 1000.0) / 1e9
        launches = max(kt["apply_launches"], 1)
        push_ms = sum(kt[k] for k in ("stream_time_ms", "partition_ms", "apply_ms", "finalize_ms")) / launches
        out = {
            "metric": "records/sec, non-key GROUP BY with repartition (SUM(amount) TUMBLING 1 MINUTE GROUP BY region_id)",
            "value": world * n * args.steps / elapsed,
            "unit": "records/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (splitmix64, ksql_amd/synth.py repartition_sum), device-resident columnar batch",
            "config": {"workload": "repartition_sum", "records_per_gpu": n, "regions": 1_000_000,
                       "window": "TUMBLING 1 MINUTE", "parallelism": "repartition all-to-all x%d" % world,
                       "rows_received_rank0": m, "groups_rank0": int(rows)},
            "roofline": {"bound": "hbm", "kernel": "whole step: pack + all-to-all + unpack + khip_agg_push",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None, "algorithmic_bytes_per_record": BYTES_PER_RECORD_C5,
                         "phase_ms": per, "push_device_ms": push_ms},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_repartition(n, args.cpu_seconds)
        print(json.dumps(out))
    h.close()
    rp.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
