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
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(n, args.keys, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out))
    h.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
