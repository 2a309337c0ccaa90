#!/usr/bin/env python3
"""Headline benchmark: windowed GROUP BY records/sec on MI355X (BASELINE.json metric).

Workload (default, N=1): BASELINE.json configs[1], "possible_fraud":
    CREATE TABLE possible_fraud AS SELECT card_number, COUNT(*) FROM ...
    WINDOW TUMBLING (SIZE 5 SECONDS) GROUP BY card_number HAVING COUNT(*) > 3;
  100M records, 10M distinct card numbers (BIGINT form; --utf8: 16-byte VARCHAR card numbers
  through the device key dictionary), 10 s of event time with <= 500 ms disorder
  (ksql_amd/synth.py).  One step = a fresh query instance over the whole workload: reset the
  HBM table, push the 100M device-resident records through the C ABI (stream time, late drop,
  window assignment, (key, window) upsert), and count the HAVING rows on the device.  Inputs
  are generated in HBM before the timed region; the PCIe-inclusive rate is reported
  separately (never `value`).

Other legs (--config), one JSON line each, same contract:
  hourly_metrics   configs[0]: 1M page views, VARCHAR url keys, COUNT(*) TUMBLING 1 HOUR
  hopping_double   configs[2]: 1e9 records, HOPPING 60 s / 10 s SUM/AVG/MIN/MAX(DOUBLE)
  clickstream_join configs[3]: 1e8-row users table in HBM, 1e9 clicks, LEFT JOIN + WHERE
  repartition_sum  configs[4]: GROUP BY a value column → pack → RCCL all-to-all → aggregate
Legs for the rows SURVEY §8(f) ranks next (same contract, not BASELINE configs):
  serde_json       C2's records as Kafka bytes (KAFKA BIGINT key, JSON value) → device columns
  table_agg        CREATE TABLE .. AS SELECT region, COUNT(*), SUM(amount) FROM users GROUP BY region
                   over a 1e8-row source-table changelog (updates move users between regions)
  session          C2's records, COUNT(*) WINDOW SESSION (1 SECOND) GROUP BY card_number

Multi-GPU: `--gpus N` (N > 1) without torchrun's environment relaunches this script under
`torch.distributed.run` (one process per GPU, 127.0.0.1 rendezvous) before anything touches
the GPU.  Weak scaling: rank r owns the keys k with k % N == r (key-hash sharding = Kafka
partitioning) and processes its own records with its own stream time (one Kafka task per
partition): no data-path collective, except the repartition leg's all-to-all.  Every rank
runs barrier + synchronize around exactly --steps timed steps; value = all ranks' records /
max-over-ranks time.

Output: one JSON line (rank 0) with `roofline` and `cpu_baseline`:
  roofline.achieved / frac   algorithmic bytes per step ÷ the wall time of one
                             step (ms_per_step, barrier-to-barrier) — the conservative figure;
  roofline.push              the same bytes ÷ the device time of the push's kernels alone (HIP
                             events on the library's stream), with a per-kernel breakdown;
  roofline.traffic           HBM bytes per step from the committed rocprofv3 PMC summary
                             (profiles/traffic.json: read requests by size,
                             TCC_EA0_RDREQ_{32B,64B,128B} + WRITE_SIZE, tools/pmc_traffic.py)
                             when it was measured on this exact configuration;
  cpu_baseline               the oracle (oracle/oracle.c, a C restatement of the reference
                             semantics — the JVM reference cannot run on this image) timed on a
                             bounded sample of the same workload, single-threaded and with P
                             threads over P key-hash shards, with the host's CPU model.
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
CPU_LABEL = "CPU restatement of the reference semantics (oracle/oracle.c), not the JVM reference"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=["possible_fraud", "hourly_metrics", "hopping_double", "clickstream_join",
                                         "repartition_sum", "serde_json", "serde_avro", "sink_json", "table_agg",
                                         "session"],
                    default="possible_fraud",
                    help="possible_fraud = BASELINE configs[1] (the headline); hourly_metrics = configs[0]; "
                         "hopping_double = configs[2]; clickstream_join = configs[3]; repartition_sum = configs[4]")
    ap.add_argument("--records", type=int, default=None, help="records per GPU (default: the config's)")
    ap.add_argument("--keys", type=int, default=10_000_000, help="possible_fraud: card numbers per GPU")
    ap.add_argument("--utf8", action="store_true", help="possible_fraud: VARCHAR card numbers (16 bytes)")
    ap.add_argument("--card-format", choices=["digits", "alnum"], default="digits",
                    help="possible_fraud --utf8: 16 decimal digits (SURVEY §8(d); inline key ids), or the same "
                         "numbers with a letter first ('C' for the leading '4': every key through the dictionary)")
    ap.add_argument("--sparse-keys", action="store_true",
                    help="possible_fraud: card numbers spread over [0, 2^53) by a bijection of the dense ids "
                         "(the key range does not fit 32 bits)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="target CPU baseline sample time per run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--engine", choices=["part", "atomic"], default="part")
    ap.add_argument("--unpack", action="store_true",
                    help="repartition_sum: unpack the received rows to columns, then khip_agg_push")
    ap.add_argument("--slice", type=int, default=1 << 27, help="hopping_double: records per micro-batch push")
    ap.add_argument("--users", type=int, default=100_000_000, help="clickstream_join: table rows")
    ap.add_argument("--sparse-ids", action="store_true",
                    help="clickstream_join: user ids spread over 2^40 (a bijection of 1..U), so the dense "
                         "direct-map index is ineligible and the hash-probe kernel runs")
    ap.add_argument("--no-extras", action="store_true", help="skip the PCIe-inclusive and pull-query side numbers")
    ap.add_argument("--exchange", choices=["rccl", "gloo"], default="rccl",
                    help="repartition_sum at N > 1: RCCL all-to-all over xGMI (production), or the same two "
                         "collective steps over a gloo process group through host memory (rehearsal)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on cuda:0 (with --exchange gloo: an N-rank rehearsal on a 1-GPU box)")
    return ap.parse_args()


# ------------------------------------------------------------------ multi-GPU launch

def relaunch(args):
    """--gpus N without torchrun's environment: run this script under torch.distributed.run as
    a child (one rank per GPU) and exit with its code.  Nothing here has touched the GPU.  The
    rendezvous binds its own port (--standalone on 127.0.0.1): a port probed here and bound later
    by torchrun could be taken in between (EADDRINUSE on a busy box)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--standalone", "--local-addr", "127.0.0.1", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------ helpers

def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "model": model}


def cpu_threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def sized_run(run, m0, target_s, m_max):
    """run(m) -> seconds; grow the sample so it takes about target_s (bounded by m_max)."""
    dt = run(m0)
    m = int(min(max(m0 * target_s / max(dt, 1e-3), m0), m_max))
    if m > m0:
        dt = run(m)
        return m, dt
    return m0, dt


KS_THREADS = 4  # ksqlDB's default Kafka Streams threads per query (C/util/KsqlConstants.java:42)


def cpu_baseline_block(single, par, P, unit, sample, ks=None):
    """single / ks / par: (records, seconds) at 1, KS_THREADS and P threads.  P is this job's CPU
    share (16 on the GPU box, whose nproc counts the whole host)."""
    b = {"value": par[0] / par[1], "unit": unit, "cores": P, "kind": "port", "sample": sample % (par[0], P),
         "single_thread": {"value": single[0] / single[1], "cores": 1, "records": single[0],
                           "seconds": single[1]},
         "parallel_seconds": par[1], "cpu": cpu_info(), "label": CPU_LABEL}
    if ks is not None:
        b["ksql_default_threads"] = {"value": ks[0] / ks[1], "cores": KS_THREADS, "records": ks[0], "seconds": ks[1]}
    return b


def load_traffic(path, config, n, variant=""):
    """HBM bytes per step from the committed PMC summary (tools/pmc_traffic.py), if it was
    measured on this configuration and size with the size-classed read counters (method_version
    2; round-4 entries doubled FETCH_SIZE from a hand-kept kernel list and are not used)."""
    try:
        with open(path) as f:
            t = json.load(f)
        rec = t.get(config + variant)
        if rec and rec.get("records") == n and rec.get("method_version", 1) >= 2:
            return rec["hbm_bytes_per_step"]
    except (OSError, ValueError):
        pass
    return None


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
        dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def timed_loop(step, steps, world):
    barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        r = step()
    barrier_sync(world)
    return r, max_over_ranks(time.perf_counter() - t0, world)


def roofline(bytes_per_step, ms_step, push_ms=None, per_kernel=None, traffic=None, bytes_per_record=None,
             kernel="", extra=None):
    achieved = bytes_per_step / (ms_step / 1000.0) / 1e9
    r = {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "algorithmic_bytes_per_record": bytes_per_record,
         "basis": "algorithmic bytes per step / ms_per_step (wall, barrier to barrier)"}
    if push_ms:
        pa = bytes_per_step / (push_ms / 1000.0) / 1e9
        r["push"] = {"ms": push_ms, "achieved": pa, "frac": pa / HBM_PEAK_GBS,
                     "basis": "the same bytes / device time of the push kernels (HIP events, library stream)"}
        if per_kernel:
            r["push"]["per_kernel"] = per_kernel
    if traffic:
        r["traffic_over_algorithmic"] = traffic / bytes_per_step
    if extra:
        r.update(extra)
    return r


def line(metric, value, world, args, ms_step, dtype, data, config, roof, cpu, **kw):
    out = {"metric": metric, "value": value, "unit": "records/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": dtype, "data": data, "config": config, "roofline": roof,
           "cpu_baseline": cpu}
    out.update(kw)
    print(json.dumps(out), flush=True)


def push_phases(kt, launches):
    launches = max(launches, 1)
    return {k: kt[k] / launches for k in ("stream_time_ms", "dict_ms", "partition_ms", "apply_ms", "finalize_ms")}


# The library's phase events (khip_agg_kernel_times) bracket, on the COUNT(*) pipeline
# (ksql_amd/csrc/khip_agg_c1.hip, ev_record_part 0..3):
#   stream_time_ms  k_c1_scatter + the run scan + k_c1_bases   key 8 + ts 8 read, one record written
#   partition_ms    k_c1_check + k_c1_chunks + k_c1_refine     one record read, one record written
#   apply_ms        k_c1_merge (+ retries) + k_part_commit     one record read + the rows written
#   dict_ms         UTF-8 keys: k_key_inline (offsets 8 + key bytes 16 read, id 8 written; a lower
#                   bound on the dictionary path, whose slot reads are random)
# and on the general partitioned engine (khip_agg_part.hip): k_part_hist + scans (key + ts read),
# scatter + refine (key + ts read, a record written, read and written again), merge.
# A record is 8 bytes (12 when the key range does not fit 32 bits: --sparse-keys).  These are the
# bytes the phases move, so their sum is the pipeline's bytes per record — not SURVEY §8(d)'s
# hash-update model (80 B/record), which the sort-based engine does not perform.
def c2_phase_bytes(c1, wide, utf8, groups, n):
    rows = 32.0 * groups / n  # every group's 32-byte row written once (the table is reset each step)
    rec = 12 if wide else 8
    if c1:
        own = {"stream_time_ms": 16 + rec, "partition_ms": rec + rec, "apply_ms": rec + rows}
    else:
        own = {"stream_time_ms": 16, "partition_ms": 16 + rec + rec + rec, "apply_ms": rec + rows}
    own["dict_ms"] = 32 if utf8 else 0
    own["finalize_ms"] = 0
    return own


def value_phase_bytes(rows_in):
    """The value-record pipeline's phases (k_c1v_scatter | k_c1v_refine | k_c1v_merge), per record:
    the scatter reads key + ts + the argument + its validity bit (or one received 32-byte row,
    `khip_agg_push_shuffled`) and writes a 16-byte record; the refine reads and writes it; the merge
    reads it — plus the resident rows' read-modify-write, not counted here (a lower bound)."""
    return {"stream_time_ms": (32 if rows_in else 24.125) + 16, "partition_ms": 32, "apply_ms": 16,
            "dict_ms": 0, "finalize_ms": 0}


def per_phase_block(phase, own, n):
    """Per-phase device time and rate over the bytes the phase moves (c2_phase_bytes)."""
    return {k: {"ms": phase[k], "bytes_per_record": own[k],
                "GB/s": own[k] * n / (phase[k] / 1000.0) / 1e9} for k in phase if phase[k] > 0 and own.get(k)}


def stream_copy_gbs(nbytes=1 << 31):
    """Achievable HBM rate on this box: one device-to-device copy (read + write bytes / time)."""
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



# ------------------------------------------------------------------ §8(f) legs

def bench_serde_json(args, lib, rank, world, local):
    """§8(f)1: deserialization of C2's records as the consumer returns them — KAFKA BIGINT key
    (8 bytes big-endian card number) and a JSON value {"AMOUNT":<10 digits>} — into device
    columns (khip_serde_decode).  One step = decode the whole device-resident raw batch."""
    import torch
    from ksql_amd import abi, synth
    n = args.records or 100_000_000
    card, ts = synth.possible_fraud(0, n, n, xp="torch", device="cuda", rank=rank, world=world, keys=args.keys)
    kb = torch.stack([((card >> (8 * (7 - i))) & 0xFF).to(torch.uint8) for i in range(8)], dim=1).reshape(-1)
    koff = torch.arange(0, 8 * (n + 1), 8, dtype=torch.int64, device="cuda")
    amount = 1_000_000_000 + card % 999_999_937  # always 10 digits
    head, tail = b'{"AMOUNT":', b"}"
    w = len(head) + 10 + len(tail)
    vb = torch.empty((n, w), dtype=torch.uint8, device="cuda")
    vb[:, :len(head)] = torch.tensor(list(head), dtype=torch.uint8, device="cuda")
    rem = amount.clone()
    for i in range(9, -1, -1):
        vb[:, len(head) + i] = (rem % 10 + 48).to(torch.uint8)
        rem //= 10
    vb[:, -1] = ord("}")
    vb = vb.reshape(-1)
    voff = torch.arange(0, w * (n + 1), w, dtype=torch.int64, device="cuda")
    sd = abi.SerdeHandle(lib, "JSON", [("AMOUNT", "INT64", 0)], key_type="INT64", key_format="KAFKA", device=local)
    torch.cuda.synchronize()

    def step():
        d, nerr = sd.decode_device(ts, koff, kb, voff, vb)
        return nerr

    for _ in range(max(args.warmup, 1)):
        nerr = step()
    assert nerr == 0, nerr
    nerr, elapsed = timed_loop(step, args.steps, world)
    sd.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    bpr = 8 + w + 2 * 8 + 8 + 8  # key bytes + value bytes + 2 offsets read; key + value columns written
    roof = roofline(bpr * n, ms_step, None, None, load_traffic(args.traffic_json, "serde_json", n), bpr,
                    kernel="khip_serde_decode (k_serde_decode)")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        import json as _json
        m = 200_000
        keys = [int(x).to_bytes(8, "big") for x in card[:m].cpu().numpy()]
        vals = [bytes(v) for v in vb[: m * w].cpu().numpy().reshape(m, w)]
        t0 = time.perf_counter()
        out = [(int.from_bytes(k, "big", signed=True), _json.loads(v)["AMOUNT"]) for k, v in zip(keys, vals)]
        dt = time.perf_counter() - t0
        assert len(out) == m
        cpu = {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d of the records, CPython int.from_bytes + json.loads per record" % m,
               "cpu": cpu_info(), "label": "CPU restatement of the KAFKA / JSON deserializers, not the JVM reference"}
    line("records/sec, Kafka record bytes (KAFKA BIGINT key, JSON value) -> device columns",
         world * n * args.steps / elapsed, world, args, ms_step, "u8",
         "synthetic (C2's records serialized on the device), device-resident raw batch",
         {"workload": "serde_json", "records_per_gpu": n, "key": "KAFKA BIGINT", "value": "JSON {\"AMOUNT\": BIGINT}",
          "value_bytes": w, "errors": int(nerr), "parallelism": "records x%d" % world}, roof, cpu)


def bench_serde_avro(args, lib, rank, world, local):
    """§8(f)1: the same records in the reference's example-data format — KAFKA BIGINT key and an
    AVRO value in the Confluent wire format (magic byte 0, 4-byte schema id, the Avro binary record
    {AMOUNT: long} as a zig-zag varint) — into device columns (khip_serde_decode, KHIP_FMT_AVRO)."""
    import torch
    from ksql_amd import abi, synth
    n = args.records or 100_000_000
    card, ts = synth.possible_fraud(0, n, n, xp="torch", device="cuda", rank=rank, world=world, keys=args.keys)
    kb = torch.stack([((card >> (8 * (7 - i))) & 0xFF).to(torch.uint8) for i in range(8)], dim=1).reshape(-1)
    koff = torch.arange(0, 8 * (n + 1), 8, dtype=torch.int64, device="cuda")
    amount = 1_000_000_000 + card % 999_999_937  # zig-zag 2e9..4e9: always 5 varint bytes
    zz = amount * 2
    w = 5 + 5
    vb = torch.zeros((n, w), dtype=torch.uint8, device="cuda")
    vb[:, 4] = 1  # schema id 1, big-endian
    for i in range(5):
        vb[:, 5 + i] = (((zz >> (7 * i)) & 0x7F) | (0x80 if i < 4 else 0)).to(torch.uint8)
    vb = vb.reshape(-1)
    voff = torch.arange(0, w * (n + 1), w, dtype=torch.int64, device="cuda")
    sd = abi.SerdeHandle(lib, "AVRO", [("AMOUNT", "INT64", 0)], key_type="INT64", key_format="KAFKA", device=local,
                         avro_schema=[("AMOUNT", "long", 0)], avro_schema_id=1)
    torch.cuda.synchronize()

    def step():
        d, nerr = sd.decode_device(ts, koff, kb, voff, vb)
        return nerr

    for _ in range(max(args.warmup, 1)):
        nerr = step()
    assert nerr == 0, nerr
    nerr, elapsed = timed_loop(step, args.steps, world)
    sd.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    bpr = 8 + w + 2 * 8 + 8 + 8  # key bytes + value bytes + 2 offsets read; key + value columns written
    roof = roofline(bpr * n, ms_step, None, None, load_traffic(args.traffic_json, "serde_avro", n), bpr,
                    kernel="khip_serde_decode (k_serde_decode, AVRO)")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        m = 200_000
        keys = [int(x).to_bytes(8, "big") for x in card[:m].cpu().numpy()]
        vals = [bytes(v) for v in vb[: m * w].cpu().numpy().reshape(m, w)]

        def avro_long(b):  # the wire header, then BinaryDecoder.readLong
            assert b[0] == 0 and int.from_bytes(b[1:5], "big") == 1
            v, sh, j = 0, 0, 5
            while True:
                x = b[j]
                v |= (x & 0x7F) << sh
                j += 1
                sh += 7
                if not x & 0x80:
                    break
            return (v >> 1) ^ -(v & 1)
        t0 = time.perf_counter()
        out = [(int.from_bytes(k, "big", signed=True), avro_long(v)) for k, v in zip(keys, vals)]
        dt = time.perf_counter() - t0
        assert len(out) == m and out[0][1] == int(amount[0])
        cpu = {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d of the records, CPython per-record wire header + zig-zag varint" % m,
               "cpu": cpu_info(), "label": "CPU restatement of the KAFKA / AVRO deserializers, not the JVM reference"}
    line("records/sec, Kafka record bytes (KAFKA BIGINT key, AVRO value) -> device columns",
         world * n * args.steps / elapsed, world, args, ms_step, "u8",
         "synthetic (C2's records serialized on the device, Confluent wire format), device-resident raw batch",
         {"workload": "serde_avro", "records_per_gpu": n, "key": "KAFKA BIGINT", "value": "AVRO {AMOUNT: long}",
          "value_bytes": w, "errors": int(nerr), "parallelism": "records x%d" % world}, roof, cpu)


def bench_sink_json(args, lib, rank, world, local):
    """§8(f)2: C2's changelog as sink records — one row per (card number, 5 s window): a
    TimeWindowed KAFKA BIGINT key (8-byte key + 8-byte window start) and a JSON value
    {"KSQL_COL_0":<count>} (khip_sink_encode, device rows → device record bytes).  One step =
    encode --records rows (default 22M, C2's group count)."""
    import torch
    from ksql_amd import abi, synth
    n = args.records or 22_000_000
    be = synth.backend("torch")
    h0 = synth._stream(be, 8, 0, n, "cuda")
    key = (h0 % 10_000_000).to(torch.int64)
    ws = ((h0 >> 24) % 3).to(torch.int64) * 5000
    we = ws + 5000
    cnt = ((h0 >> 40) % 30 + 1).to(torch.int64)
    nul = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = abi.SinkHandle(lib, "KAFKA", [("CARD_NUMBER", "INT64")], "JSON", [("KSQL_COL_0", "INT64", 0)],
                       window_kind="TUMBLING", device=local)
    rows = abi.SinkRows()
    rows.n_rows, rows.mem, rows.key_serialized = n, abi.MEM_DEVICE, 0
    rows.key_i64, rows.window_start, rows.window_end = key.data_ptr(), ws.data_ptr(), we.data_ptr()
    cd = (abi.C.c_void_p * 1)(cnt.data_ptr())
    cn = (abi.C.c_void_p * 1)(nul.data_ptr())
    rows.col_data, rows.col_null = cd, cn
    kcap, vcap = 16 * n, 40 * n
    koff = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    voff = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    kbytes = torch.empty(kcap, dtype=torch.uint8, device="cuda")
    vbytes = torch.empty(vcap, dtype=torch.uint8, device="cuda")
    vnull = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = abi.SinkOut()
    out.mem, out.key_capacity, out.value_capacity = abi.MEM_DEVICE, kcap, vcap
    out.key_offsets, out.key_bytes = koff.data_ptr(), kbytes.data_ptr()
    out.value_offsets, out.value_bytes, out.value_null = voff.data_ptr(), vbytes.data_ptr(), vnull.data_ptr()
    torch.cuda.synchronize()

    def step():
        lib.check(lib.sink_encode(s.h, abi.C.byref(rows), abi.C.byref(out)), "sink_encode")
        return out.key_len, out.value_len

    for _ in range(max(args.warmup, 1)):
        kl, vl = step()
    assert kl == 16 * n, kl
    (kl, vl), elapsed = timed_loop(step, args.steps, world)
    s.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    # rows read (key, ws, we, count, null flag) + record bytes and offsets written
    bpr = 8 + 8 + 8 + 8 + 1 + 16 + vl / n + 2 * 8 + 1
    roof = roofline(bpr * n, ms_step, None, None, load_traffic(args.traffic_json, "sink_json", n), bpr,
                    kernel="khip_sink_encode (k_sink_measure + scans + k_sink_write)")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        # the CPU restatement of the serializers (tests/sink_ref.py) on a bounded sample
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import sink_ref
        m = min(n, 2_000_000)
        kk, ww, cc = (x[:m].cpu().numpy().tolist() for x in (key, ws, cnt))
        kc, vc = [("CARD_NUMBER", "INT64")], [("KSQL_COL_0", "INT64")]
        t0 = time.perf_counter()
        recs = [(sink_ref.encode_key("KAFKA", kc, [k]) + sink_ref.window_suffix("TUMBLING", w, w + 5000),
                 sink_ref.encode_value("JSON", vc, [c])) for k, w, c in zip(kk, ww, cc)]
        dt = time.perf_counter() - t0
        assert len(recs[0][0]) == 16
        cpu = {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "%d of the rows, tests/sink_ref.py per row (CPython)" % m, "cpu": cpu_info(),
               "label": "CPU restatement of the KAFKA key / JSON value serializers, not the JVM reference"}
    line("records/sec, changelog rows -> sink records (TimeWindowed KAFKA BIGINT key, JSON value)",
         world * n * args.steps / elapsed, world, args, ms_step, "u8",
         "synthetic C2-shaped changelog rows (splitmix64), device-resident columns",
         {"workload": "sink_json", "rows_per_gpu": n, "key": "KAFKA BIGINT + 8-byte window start",
          "value": "JSON {\"KSQL_COL_0\": BIGINT}", "value_bytes_per_row": vl / n,
          "parallelism": "rows x%d" % world}, roof, cpu)


def bench_table_agg(args, lib, rank, world, local):
    """§8(f)4: CREATE TABLE by_region AS SELECT region, COUNT(*), SUM(amount) FROM users GROUP BY
    region — a source table of 1e7 users whose changelog (1e8 rows, 5 % tombstones) moves users
    between 1e5 regions; pushed as micro-batches of --slice rows (khip_agg_push_table).  One step =
    a fresh query instance over the whole changelog."""
    import torch
    from ksql_amd import abi, synth
    n = args.records or 100_000_000
    users = 10_000_000 // world
    S = max(8, min(args.slice, 1 << 24) // 8 * 8)
    be = synth.backend("torch")
    h0 = synth._stream(be, 7, 0, n, "cuda")
    pk = (h0 % users).to(torch.int64)
    if args.sparse_ids:  # the same users under ids spread over 2^40 (synth.sparse_ids, as C4's)
        pk = synth.sparse_ids(pk)
    region = ((h0 >> 24) % 100_000).to(torch.int64)
    amount = ((h0 >> 40) % 2_000_001 - 1_000_000).to(torch.int64)
    live = (h0 >> 60) != 0  # 1 in 16 rows: a tombstone
    ts = torch.arange(n, dtype=torch.int64, device="cuda")
    rv = abi.bitmap_torch(live)
    batches = [(abi.DeviceBatch(ts[lo:min(lo + S, n)], keys=region[lo:min(lo + S, n)], row_valid=rv[lo // 8:],
                                cols=[amount[lo:min(lo + S, n)]]), pk[lo:min(lo + S, n)]) for lo in range(0, n, S)]
    desc = abi.make_agg_desc("NONE", "INT64", col_types=["INT64"], aggs=[("COUNT_STAR", -1), ("SUM", 0)],
                             device=local, capacity_hint=200_000, flags=abi.FLAG_TABLE_SOURCE)
    h = abi.AggHandle(lib, desc)
    torch.cuda.synchronize()

    def push_dev(b, k):
        src = abi.TableSrc(abi.KEY["INT64"], 0, k.data_ptr(), None, None, None)
        st = abi.BatchStats()
        lib.check(lib.agg_push_table(h.h, abi.C.byref(b.struct), abi.C.byref(src), abi.C.byref(st)), "agg_push_table")
        return st.rows_accepted

    def step():
        lib.check(lib.agg_reset(h.h), "agg_reset")
        return sum(push_dev(b, k) for b, k in batches)

    for _ in range(max(args.warmup, 1)):
        acc = step()
    acc, elapsed = timed_loop(step, args.steps, world)
    groups = h.count_rows(None)
    h.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    bpr = 32 + 2 * 32 + 2 * 2 * 32  # row in (pk, region, ts, amount) + 32-B source-row RMW + undo and apply group RMWs
    roof = roofline(bpr * n, ms_step, None, None, load_traffic(args.traffic_json, "table_agg" + ("_sparse_ids" if args.sparse_ids else ""), n), bpr,
                    kernel="khip_agg_push_table (k_tagg_keys + radix sort + k_tagg_apply + finalize)")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        orc = abi.load_oracle()
        m = 2_000_000
        hb = abi.HostBatch(ts[:m].cpu().numpy(), keys=region[:m].cpu().numpy(), row_valid=live[:m].cpu().numpy(),
                           cols=[amount[:m].cpu().numpy()])
        ho = abi.AggHandle(orc, abi.make_agg_desc("NONE", "INT64", col_types=["INT64"],
                                                  aggs=[("COUNT_STAR", -1), ("SUM", 0)], flags=abi.FLAG_TABLE_SOURCE))
        t0 = time.perf_counter()
        ho.push_table(hb, src_keys=pk[:m].cpu().numpy(), stats=False)
        dt = time.perf_counter() - t0
        ho.close()
        cpu = {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "first %d changelog rows, oracle_agg_push_table (R12)" % m, "cpu": cpu_info(),
               "label": CPU_LABEL}
    line("records/sec, table aggregation (source-table changelog rows, undo + apply)",
         world * n * args.steps / elapsed, world, args, ms_step, "int64",
         "synthetic (splitmix64), device-resident changelog",
         {"workload": "table_agg", "records_per_gpu": n, "source_keys": users, "regions": 100_000,
          "source_ids": "sparse over 2^40 (hash layout)" if args.sparse_ids else "dense 0..users (dense layout)",
          "micro_batch": S, "groups_per_gpu": int(groups), "rows_accepted": int(acc), "parallelism": "key-hash shards x%d" % world}, roof, cpu)


def bench_session(args, lib, rank, world, local):
    """§8(f)4: C2's records with SESSION windows: SELECT card_number, COUNT(*) ... WINDOW SESSION
    (1 SECOND) GROUP BY card_number (khip_agg session engine).  One step = a fresh query instance
    over the 100M device-resident records."""
    import torch
    from ksql_amd import abi, synth
    n = args.records or 100_000_000
    card, ts = synth.possible_fraud(0, n, n, xp="torch", device="cuda", rank=rank, world=world, keys=args.keys)
    batch = abi.DeviceBatch(ts, keys=card)
    kw = dict(window_kind="SESSION", size_ms=1000, key_type="INT64", aggs=[("COUNT_STAR", -1)])
    h = abi.AggHandle(lib, abi.make_agg_desc(**kw, device=local, capacity_hint=3 * args.keys))
    torch.cuda.synchronize()

    def step():
        h.reset()
        return h.push(batch)

    for _ in range(max(args.warmup, 1)):
        st = step()
    assert st["rows_accepted"] == n, st
    st, elapsed = timed_loop(step, args.steps, world)
    groups = h.count_rows(None)
    h.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    bpr = 16 + 2 * 32  # key + ts in, one session-row RMW
    roof = roofline(bpr * n, ms_step, None, None, load_traffic(args.traffic_json, "session", n), bpr,
                    kernel="khip_agg_push, SESSION engine (key-range sort + LDS per-key replay + store rebuild)")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        orc = abi.load_oracle()
        m = 4_000_000
        c2, t2 = synth.possible_fraud(0, m, n, keys=args.keys)
        ho = abi.AggHandle(orc, abi.make_agg_desc(**kw))
        t0 = time.perf_counter()
        ho.push(abi.HostBatch(t2, keys=c2), stats=False)
        dt = time.perf_counter() - t0
        ho.close()
        cpu = {"value": m / dt, "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "first %d of the records, oracle R11" % m, "cpu": cpu_info(), "label": CPU_LABEL}
    line("records/sec, SESSION-windowed GROUP BY (COUNT(*) WINDOW SESSION 1 SECOND GROUP BY card_number)",
         world * n * args.steps / elapsed, world, args, ms_step, "int64",
         "synthetic (splitmix64, ksql_amd/synth.py possible_fraud), device-resident columnar batch",
         {"workload": "session", "records_per_gpu": n, "keys_per_gpu": args.keys, "window": "SESSION 1 s",
          "sessions_per_gpu": int(groups), "windows_late": int(st["windows_late"]),
          "parallelism": "key-hash shards x%d" % world}, roof, cpu)

# ------------------------------------------------------------------ main

def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        return relaunch(args)
    import torch
    import torch.distributed as dist
    from ksql_amd import abi

    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.one_device:
        if args.exchange != "gloo":
            raise SystemExit("bench.py: --one-device needs --exchange gloo (RCCL refuses two ranks on one GPU)")
        local = 0
    torch.cuda.set_device(local)
    if world > 1 and args.exchange == "gloo":
        dist.init_process_group("gloo")
    elif world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    lib = abi.load_product()
    legs = {"possible_fraud": bench_possible_fraud, "hourly_metrics": bench_hourly_metrics,
            "hopping_double": bench_hopping_double, "clickstream_join": bench_join,
            "repartition_sum": bench_repartition, "serde_json": bench_serde_json, "serde_avro": bench_serde_avro,
            "sink_json": bench_sink_json, "table_agg": bench_table_agg,
            "session": bench_session}
    legs[args.config](args, lib, rank, world, local)
    if world > 1:
        dist.destroy_process_group()
    return 0


# ------------------------------------------------------------------ C2 possible_fraud

SPARSE_MULT = 0x5DEECE66D  # --sparse-keys: odd, so id -> id * SPARSE_MULT mod 2^64 is a bijection
BYTES_PER_RECORD_C2 = 80  # W_in 16 + F(1) x 2 x S_slot(32)
BYTES_PER_RECORD_C2_UTF8 = 16 + 8 + 8 + 64  # key bytes 16 + offset 8 + ts 8 + 2 x S_slot(32)


def bench_possible_fraud(args, lib, rank, world, local):
    import torch
    from ksql_amd import abi, synth
    n = args.records or 100_000_000
    card, ts = synth.possible_fraud(0, n, n, xp="torch", device="cuda", rank=rank, world=world, keys=args.keys)
    if args.sparse_keys:  # a bijection on [0, 2^53): odd multiplier mod 2^64, then the low 53 bits
        card = (card * SPARSE_MULT) & ((1 << 53) - 1)
    if args.utf8:
        offs, kbytes = synth.card_utf8(card, xp="torch")
        if args.card_format == "alnum":
            kbytes[offs[:-1]] = ord("C")
        batch = abi.DeviceBatch(ts, key_offsets=offs, key_bytes=kbytes)
    else:
        batch = abi.DeviceBatch(ts, keys=card)
    torch.cuda.synchronize()
    having = {"agg": 0, "op": "GT", "value": 3}  # the query's HAVING: part of the plan (TableFilter)
    desc = abi.make_agg_desc(window_kind="TUMBLING", size_ms=5000, key_type="UTF8" if args.utf8 else "INT64",
                             aggs=[("COUNT_STAR", -1)], device=local, capacity_hint=int(min(3 * args.keys, 2 * n)),
                             flags=abi.FLAG_PROFILE | (abi.FLAG_ENGINE_ATOMIC if args.engine == "atomic" else 0),
                             having=having)
    h = abi.AggHandle(lib, desc)

    def step():
        h.reset()
        st = h.push(batch)
        return st, h.count_rows(having)

    for _ in range(max(args.warmup, 1)):
        st, rows = step()
    assert st["rows_accepted"] == n and st["windows_applied"] == n, st
    h.kernel_times(reset=True)
    (st, rows), elapsed = timed_loop(step, args.steps, world)
    kt = h.kernel_times()
    groups = int(h.snapshot_size())  # host bookkeeping: no device work after the timed loop

    pcie = pull = None
    if rank == 0 and not args.no_extras and not args.utf8 and n <= 100_000_000:
        # PCIe-inclusive rate (host-resident input, one step) for DESIGN.md — never `value`
        hb = abi.HostBatch(ts.cpu().numpy(), keys=card.cpu().numpy())
        h.reset()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        h.push(hb)
        h.count_rows(having)
        pcie = n / (time.perf_counter() - t1)
        del hb
        # pull-query latency on the materialized table (khip_agg_get)
        qk = card[: 1 << 12].cpu().numpy()
        pull = {}
        for nk in (1, 100, 4096):
            h.get(qk[:nk])
            t1 = time.perf_counter()
            for _ in range(5):
                r = h.get(qk[:nk])
            pull["keys_%d_ms" % nk] = (time.perf_counter() - t1) * 1000.0 / 5
            pull["keys_%d_rows" % nk] = int(r["n"])
    h.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    phase = push_phases(kt, kt["apply_launches"])
    push_ms = sum(phase.values())
    bpr = BYTES_PER_RECORD_C2_UTF8 if args.utf8 else BYTES_PER_RECORD_C2
    c1 = kt.get("c1_pushes", 0) > 0
    own = c2_phase_bytes(c1, args.sparse_keys, args.utf8, groups, n)
    per_kernel = per_phase_block(phase, own, n)
    variant = ("_utf8" + ("_card_format_alnum" if args.card_format == "alnum" else "") if args.utf8 else
               ("_sparse_keys" if args.sparse_keys else ""))  # profile_leg.sh's leg names
    traffic = load_traffic(args.traffic_json, "possible_fraud" + ("_atomic" if args.engine == "atomic" else ""), n,
                           variant)
    # beside SURVEY's model: the I/O floor (the input read once, every group's row written once)
    floor = (16 + 16 + 8 if args.utf8 else 16) + 32.0 * groups / n
    pipe = sum(own.values())
    roof = roofline(bpr * n, ms_step, push_ms, per_kernel, traffic, bpr,
                    kernel=("khip_agg_push (COUNT(*) pipeline: k_c1_scatter (step runs) + run scan + k_c1_check + "
                            "k_c1_chunks + k_c1_refine + k_c1_merge + commit) + HAVING count") if c1 else
                           "khip_agg_push (k_part_hist + scans + k_part_scatter + k_part_refine + k_part_merge + "
                           "commit) + HAVING count",
                    extra={"floor_bytes_per_record": floor,
                           "floor_basis": "input once (key + ts%s) + each group's 32-B row written once" %
                                          (" + key bytes + offsets" if args.utf8 else ""),
                           "floor_frac": floor * n / (ms_step / 1000.0) / 1e9 / HBM_PEAK_GBS,
                           "pipeline_bytes_per_record": pipe,
                           "pipeline_basis": "sum of the per-phase bytes (push.per_kernel): what the passes move",
                           "pipeline_frac": pipe * n / (ms_step / 1000.0) / 1e9 / HBM_PEAK_GBS})
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_agg(
            lambda m: synth.possible_fraud(0, m, n, keys=args.keys), args.utf8,
            dict(window_kind="TUMBLING", size_ms=5000, aggs=[("COUNT_STAR", -1)]),
            args.cpu_seconds, 40_000_000, "first %%d of the %d possible_fraud records, %%d key-hash shards" % n)
    line("records/sec, windowed GROUP BY (COUNT(*) TUMBLING 5 s GROUP BY card_number HAVING > 3)",
         world * n * args.steps / elapsed, world, args, ms_step, "int64",
         "synthetic (splitmix64, ksql_amd/synth.py), device-resident columnar batch",
         {"workload": "possible_fraud", "key": ("VARCHAR(16) card_number" if args.utf8 else "BIGINT card_number") +
                                                 (" spread over 2^53" if args.sparse_keys else ""),
          "key_ids": (("inline (16 ASCII digits: exact 64-bit ids, no dictionary)" if args.card_format == "digits"
                       else "device dictionary (letter-led keys)") if args.utf8 else None),
          "records_per_gpu": n, "keys_per_gpu": args.keys, "window": "TUMBLING 5s, grace default",
          "having": "COUNT(*) > 3", "groups_per_gpu": groups, "having_rows_per_gpu": int(rows),
          "parallelism": "key-hash shards x%d" % world},
         roof, cpu, pcie_inclusive_records_per_s=pcie, pull_query=pull)


def cpu_baseline_agg(gen, utf8, kw, target_s, m_max, sample):
    """Oracle on a prefix of the workload: 1 thread (sequential oracle_agg_push) and P threads
    (oracle_agg_push_sharded over P key-hash shards).  Each run is a fresh task."""
    from ksql_amd import abi, synth
    orc = abi.load_oracle()
    P = cpu_threads()

    def batch(m):
        out = gen(m)
        key, ts = out[0], out[1]
        cols = list(out[2:3]) if len(out) > 2 else []
        cval = list(out[3:4]) if len(out) > 3 else []
        if utf8:
            offs, kb = synth.card_utf8(key)
            return abi.HostBatch(ts, key_offsets=offs, key_bytes=kb, cols=cols, col_valid=cval)
        return abi.HostBatch(ts, keys=key, cols=cols, col_valid=cval)

    def run(m, shards):
        b = batch(m)
        desc = abi.make_agg_desc(key_type="UTF8" if utf8 else "INT64", **kw)
        h = abi.AggHandle(orc, desc) if shards == 1 else abi.ShardedOracleAgg(orc, desc, shards)
        t0 = time.perf_counter()
        h.push(b, stats=False)
        dt = time.perf_counter() - t0
        h.close()
        return dt

    single = sized_run(lambda m: run(m, 1), 500_000, target_s, m_max)
    ks = sized_run(lambda m: run(m, KS_THREADS), 1_000_000, target_s, m_max)
    par = sized_run(lambda m: run(m, P), 1_000_000, target_s, m_max)
    return cpu_baseline_block(single, par, P, "records/s", sample, ks)


# ------------------------------------------------------------------ C1 hourly_metrics

def bench_hourly_metrics(args, lib, rank, world, local):
    """configs[0]: COUNT(*) TUMBLING 1 HOUR GROUP BY url over 1M page views (VARCHAR url keys through
    the device dictionary).  One step = reset + push + row count.  The reference's own
    CPU-runnable case; at 1M records one step is a handful of small launches."""
    import torch
    from ksql_amd import abi, synth
    n = args.records or synth.CONFIGS["hourly_metrics"]["n"]
    offs, kb, ts = synth.hourly_metrics_utf8(0, n, n)
    dev = lambda a: torch.from_numpy(a).to("cuda")
    batch = abi.DeviceBatch(dev(ts), key_offsets=dev(offs), key_bytes=dev(kb))
    torch.cuda.synchronize()
    kw = dict(window_kind="TUMBLING", size_ms=3_600_000, key_type="UTF8", aggs=[("COUNT_STAR", -1)])
    h = abi.AggHandle(lib, abi.make_agg_desc(**kw, device=local, capacity_hint=40_000, flags=abi.FLAG_PROFILE))

    def step():
        h.reset()
        st = h.push(batch)
        return st, h.count_rows(None)

    for _ in range(max(args.warmup, 1)):
        st, groups = step()
    assert st["rows_accepted"] == n, st
    h.kernel_times(reset=True)
    (st, groups), elapsed = timed_loop(step, args.steps, world)
    kt = h.kernel_times()
    h.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    bpr = float(kb.size) / n + 8 + 8 + 2 * 32  # key bytes + offset + ts + 2 x S_slot(32)
    phase = push_phases(kt, kt["apply_launches"])
    roof = roofline(bpr * n, ms_step, sum(phase.values()), None, load_traffic(args.traffic_json, "hourly_metrics", n),
                    bpr, kernel="khip_agg_push (UTF8 dictionary + partitioned aggregate) + row count",
                    extra={"note": "1M records: launch/latency-bound, not HBM-bound"})
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_hourly(n, args.cpu_seconds)
    line("records/sec, windowed GROUP BY (COUNT(*) TUMBLING 1 HOUR GROUP BY url)",
         world * n * args.steps / elapsed, world, args, ms_step, "int64",
         "synthetic (splitmix64, ksql_amd/synth.py hourly_metrics), device-resident columnar batch",
         {"workload": "hourly_metrics", "key": "VARCHAR url", "records_per_gpu": n, "urls": 10_000,
          "window": "TUMBLING 1 HOUR", "groups_per_gpu": int(groups), "parallelism": "key-hash shards x%d" % world},
         roof, cpu)


def cpu_baseline_hourly(n, target_s):
    from ksql_amd import abi, synth
    orc = abi.load_oracle()
    P = cpu_threads()
    kw = dict(window_kind="TUMBLING", size_ms=3_600_000, key_type="UTF8", aggs=[("COUNT_STAR", -1)])
    offs, kb, ts = synth.hourly_metrics_utf8(0, n, n)
    b = abi.HostBatch(ts, key_offsets=offs, key_bytes=kb)

    def run(shards, reps):
        t0 = time.perf_counter()
        for _ in range(reps):
            h = abi.AggHandle(orc, abi.make_agg_desc(**kw)) if shards == 1 else \
                abi.ShardedOracleAgg(orc, abi.make_agg_desc(**kw), shards)
            h.push(b, stats=False)
            h.close()
        return time.perf_counter() - t0

    out = []
    for shards in (1, P, KS_THREADS):
        dt = run(shards, 1)
        reps = max(1, int(target_s / max(dt, 1e-3)))
        out.append((n * reps, run(shards, reps)))
    return cpu_baseline_block(out[0], out[1], P, "records/s",
                              "%d records (the 1M-record hourly_metrics run, repeated), %d key-hash shards", out[2])


# ------------------------------------------------------------------ C3 hopping_double

BYTES_PER_RECORD_C3 = 24.125 + 6 * 2 * 56  # W_in + F x 2 x S_slot = 696.1


def bench_hopping_double(args, lib, rank, world, local):
    """configs[2]: HOPPING (SIZE 1 MINUTE, ADVANCE BY 10 SECONDS, GRACE PERIOD 1 MINUTE)
    SUM/AVG/MIN/MAX of a DOUBLE with 1 % nulls, 1e9 records (1 h of event time) per GPU, key
    BIGINT in [0, 1e5).  One step = a fresh query instance: reset, the device-resident records
    pushed as event-time micro-batches of --slice records (closed windows leave the live table
    between pushes), and the materialized row count."""
    import torch
    from ksql_amd import abi, synth
    n = args.records or 1_000_000_000
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
    kw = dict(window_kind="HOPPING", size_ms=cfg["size_ms"], advance_ms=cfg["advance_ms"], grace_ms=cfg["grace_ms"],
              key_type="INT64", col_types=["DOUBLE"], aggs=[("SUM", 0), ("AVG", 0), ("MIN", 0), ("MAX", 0)])
    h = abi.AggHandle(lib, abi.make_agg_desc(**kw, device=local, capacity_hint=live, flags=abi.FLAG_PROFILE))

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
    (st, groups), elapsed = timed_loop(step, args.steps, world)
    kt = h.kernel_times()
    h.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    phase = {k: kt[k] / args.steps for k in ("stream_time_ms", "partition_ms", "apply_ms", "finalize_ms")}
    # frac over the ALGORITHMIC FLOOR of the step: every input column read once (W_in = key 8 + ts 8
    # + value 8 + validity 1/8 = 24.125 B/record) plus, per push, one read-modify-write of the live
    # (key, window) rows (S_slot = key 8 + ws 8 + sum/count/min/max 32 + rowtime 8 = 56 B, read and
    # written: 112 B).  Live rows per push = the windows the push's span, size, grace and disorder
    # keep open per key, at most the step's groups.  The counter bytes the kernels move stay in
    # `traffic` (their rate over the wall time is `streamed_frac`: utilisation, not efficiency);
    # SURVEY §8(d)'s 696 B/record (one HBM slot read-modify-write per (record, window), which the
    # engine never does: windows fan out in LDS, panes fold them) gives `survey_equivalent_frac`.
    traffic = load_traffic(args.traffic_json, "hopping_double", n)
    floor_rec = 24.125
    live_rows = min(groups, live)
    floor_bytes = floor_rec * n + len(batches) * live_rows * 2 * 56.0
    moved_model = 16 + 24 + 32 + 32 + 32 + 32 + 2 * 64.0 * groups / n * len(batches)
    moved = traffic / n if traffic else moved_model
    roof = roofline(floor_bytes, ms_step, sum(phase.values()), None, traffic, floor_bytes / n,
                    kernel="khip_agg_push (all kernels of every micro-batch push) + row count",
                    extra={"basis": "algorithmic floor (input columns once + one read-modify-write of the live rows "
                                    "per push, %.3f B/record) / ms_per_step (wall, barrier to barrier)"
                                    % (floor_bytes / n),
                           "live_rows_per_push": live_rows, "pushes": len(batches),
                           "streamed_bytes_per_record": moved,
                           "streamed_basis": "PMC counter bytes, profiles/traffic.json" if traffic else
                                             "model of the passes: no counter record for this size",
                           "streamed_frac": moved * n / (ms_step / 1000.0) / 1e9 / HBM_PEAK_GBS,
                           "survey_algorithmic_bytes_per_record": BYTES_PER_RECORD_C3,
                           "survey_equivalent_frac": BYTES_PER_RECORD_C3 * n / (ms_step / 1000.0) / 1e9 / HBM_PEAK_GBS,
                           "phase_ms_per_step": phase,
                           "per_kernel": per_phase_block(phase, value_phase_bytes(False), n),
                           "stream_copy_GBps": stream_copy_gbs()})
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_agg(lambda m: synth.hopping_double(0, m, n), False,
                               {k: v for k, v in kw.items() if k != "key_type"},
                               args.cpu_seconds, 20_000_000,
                               "first %%d of the %d hopping_double records, %%d key-hash shards" % n)
    line("records/sec, windowed GROUP BY (SUM/AVG/MIN/MAX(value DOUBLE) HOPPING 60 s / 10 s GROUP BY key)",
         world * n * args.steps / elapsed, world, args, ms_step, "f64",
         "synthetic (splitmix64, ksql_amd/synth.py hopping_double), device-resident columnar batch",
         {"workload": "hopping_double", "records_per_gpu": n, "keys_per_gpu": keys_here,
          "window": "HOPPING 60s/10s GRACE 60s (F=6)", "micro_batch": S, "pushes": len(batches),
          "windows_applied": st["windows_applied"], "windows_late": st["windows_late"],
          "groups_per_gpu": int(groups), "parallelism": "key-hash shards x%d" % world,
          "double_tolerance": "SUM / AVG within 1e-12 x sum|x| of the oracle's sequential sum (DoubleSumKudaf.java:"
                              "26-31; the device adds in LDS-atomic order, panes first); for these non-negative "
                              "values that is the north star's relative 1e-12.  Signed values U[-1000,1000) in "
                              "C3's shape (tests/test_gpu_fullsize.py::test_c3_signed_cancellation, 124K groups): "
                              "plain relative error <= 6.9e-15 wherever sum|x| <= 50 |sum|; worst 1.75e-11 on 12 "
                              "groups (0.0097%) at condition numbers >= 1.7e4, where no reordered summation meets "
                              "a plain relative bound.  MIN / MAX, counts bit-exact"},
         roof, cpu)


# ------------------------------------------------------------------ C4 clickstream_join

BYTES_PER_PROBE_C4 = 31  # W_in 16 + table slot 8 + 0.30 x output 24


def random_gather_rows_per_s(table_bytes, rows=100_000_000):
    """Practical ceiling of a hash probe into a table far larger than the caches: torch's gather
    of `rows` uniformly random 32-byte rows from a `table_bytes` table, in rows/s."""
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


def bench_join(args, lib, rank, world, local):
    """configs[3]: clickstream LEFT JOIN users WHERE level = 'Platinum'.  The 1e8-row users table
    is replicated in every GPU's HBM (built once, timed separately); each GPU probes its own 1e9
    clicks (weak scaling, no exchange).  One step = khip_table_probe_device over all clicks:
    row-aligned emit/matched bitmaps + the right column, then the emitted count."""
    import torch
    from ksql_amd import abi, synth
    n = args.records or 1_000_000_000
    U = args.users
    uid, level = synth.users_table(0, U, xp="torch", device="cuda")
    if args.sparse_ids:
        uid = synth.sparse_ids(uid)
    level = level.to(torch.int32)
    t = abi.TableHandle(lib, ["INT32"], device=local, capacity_hint=U)
    tb = abi.DeviceBatch(torch.zeros(U, dtype=torch.int64, device="cuda"), keys=uid, cols=[level])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t.upsert(tb)
    t.sync()
    build_s = time.perf_counter() - t0
    del tb, uid, level
    cu, cts = synth.clicks(0, n, U, xp="torch", device="cuda", seed_clicks=5 + 1000 * rank)
    if args.sparse_ids:
        cu = synth.sparse_ids(cu)
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
    rows, elapsed = timed_loop(step, args.steps, world)
    # khip_table_create: cap = next_pow2(2 x hint) slots of 16 bytes (one INT column: the compact
    # layout, the value inside the meta word); a probe's first read is its 32-byte home pair
    info = {"table_bytes": (1 << max(10, (2 * U - 1).bit_length())) * 16, "slot_bytes": 16, "home_read_bytes": 32}
    t.close()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    roof = roofline(BYTES_PER_PROBE_C4 * n, ms_step, None, None, load_traffic(args.traffic_json, "clickstream_join" + ("_sparse_ids" if args.sparse_ids else ""), n),
                    BYTES_PER_PROBE_C4, kernel="khip_table_probe_device (probe kernels) + emitted count",
                    extra={"stream_copy_GBps": stream_copy_gbs(), "table": info,
                           "random_gather_rows_per_s": random_gather_rows_per_s(info["table_bytes"])})
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_join(U, args.cpu_seconds, args.sparse_ids)
    line("stream records/sec, stream-table LEFT JOIN (clickstream x users WHERE level = 'Platinum')",
         world * n * args.steps / elapsed, world, args, ms_step, "int64",
         "synthetic (splitmix64, ksql_amd/synth.py users_table/clicks), device-resident columnar batch",
         {"workload": "clickstream_join", "user_ids": "sparse over 2^40 (hash probe)" if args.sparse_ids else
          "1..U (dense direct-map index)", "table_rows": U, "clicks_per_gpu": n, "table_build_s": build_s,
          "table_build_rows_per_s": U / build_s, "emitted_rows_per_gpu": int(rows),
          "parallelism": "replicated table x%d" % world},
         roof, cpu)


def cpu_baseline_join(users, target_s, sparse=False):
    """Oracle stream-table LEFT JOIN WHERE level = 'Platinum': a users table of min(users, 1e7)
    rows built first (untimed), then clicks over the same 1.1x id span probed against it —
    1 thread, and P threads over P chunks of the stream (the table is read-only)."""
    from ksql_amd import abi, synth
    orc = abi.load_oracle()
    P = cpu_threads()
    U = min(users, 10_000_000)
    uid, level = synth.users_table(0, U)
    if sparse:
        uid = synth.sparse_ids(uid)
    t = abi.TableHandle(orc, ["INT32"], capacity_hint=U)
    t.upsert(abi.HostBatch(np.zeros(U, np.int64), keys=uid, cols=[level.astype(np.int32)]))
    where = {"col": 0, "op": "EQ", "i64": synth.LEVELS.index("Platinum")}

    def run(m, threads):
        cu, cts = synth.clicks(0, m, U, seed_clicks=5)
        if sparse:
            cu = synth.sparse_ids(cu)
        bounds = np.linspace(0, m, threads + 1).astype(np.int64)
        bs = [abi.HostBatch(cts[bounds[k]:bounds[k + 1]], keys=cu[bounds[k]:bounds[k + 1]]) for k in range(threads)]
        th = [threading.Thread(target=t.probe, args=(bs[k], "LEFT", where)) for k in range(threads)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        return time.perf_counter() - t0

    single = sized_run(lambda m: run(m, 1), 1_000_000, target_s, 50_000_000)
    ks = sized_run(lambda m: run(m, KS_THREADS), 2_000_000, target_s, 100_000_000)
    par = sized_run(lambda m: run(m, P), 2_000_000, target_s, 100_000_000)
    t.close()
    return cpu_baseline_block(single, par, P, "records/s",
                              "%%d clicks probed against a %d-row users table, %%d threads" % U, ks)


# ------------------------------------------------------------------ C5 repartition_sum

BYTES_PER_RECORD_C5 = 136  # read 24 + pack 24 + recv 24 + 2 x 32 (slot)


def bench_repartition(args, lib, rank, world, local):
    """configs[4]: GROUP BY region_id (a value column) forces the repartition.  One step per rank:
    khip_shuffle_pack (Kafka partitioner) → RCCL count exchange + all-to-all over xGMI (N > 1) →
    khip_agg_push_shuffled (the received rows read where they lie; --unpack: khip_shuffle_unpack +
    khip_agg_push) → SUM(amount) TUMBLING 1 MINUTE → row count.  Weak scaling: every
    rank owns one source partition of --records records (1e9 node-wide at N = 8 with 125M)."""
    import torch
    import torch.distributed as dist
    from ksql_amd import abi, synth
    from ksql_amd.repartition import Repartition

    n = args.records or 125_000_000
    eid, ts, region, amount = synth.repartition_sum(0, n, n, xp="torch", device="cuda", rank=rank, world=world)
    torch.cuda.synchronize()
    src = abi.DeviceBatch(ts, cols=[region, amount])
    from ksql_amd.repartition import GlooExchange
    comm = None
    if world > 1 and args.exchange == "gloo":
        comm = GlooExchange()
    elif world > 1:
        obj = [abi.comm_unique_id(lib) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = abi.Comm(lib, world, rank, obj[0], local)
    rp = Repartition(lib, 0, ["INT64", "INT64"], rank=rank, world=world, comm=comm, device=local)
    desc = abi.make_agg_desc(window_kind="TUMBLING", size_ms=60_000, key_type="INT64", col_types=["INT64", "INT64"],
                             aggs=[("SUM", 1)], device=local, capacity_hint=60 * 1_000_000 // max(world, 1),
                             flags=abi.FLAG_PROFILE)
    h = abi.AggHandle(lib, desc)
    phases = {"pack": 0.0, "exchange": 0.0, "aggregate": 0.0}
    state = {"timed": False, "m": 0}

    # one destination: sized for every source row (khip_shuffle_pack's one-pass compaction);
    # several: khip_shuffle_pack_v's regions (one pass, khip_shuffle_pack_capacity rows)
    send_buf = torch.empty((rp.shuffle.pack_capacity(n), rp.shuffle.row_words), dtype=torch.int64,
                           device=torch.device("cuda", local))

    def step():
        t0 = time.perf_counter()
        if world > 1:
            send, counts, offs = rp.shuffle.pack_v(src, send=send_buf)
        else:
            send, counts = rp.shuffle.pack(src, send=send_buf)
        t1 = time.perf_counter()
        if world > 1:
            recv, rc = comm.alltoall(send, counts, rp.shuffle.row_words, send_offsets=offs)
        else:
            recv, rc = send, counts
        m = int(sum(rc))
        t2 = time.perf_counter()
        h.reset()
        if args.unpack:  # the columnar route: khip_shuffle_unpack, then khip_agg_push
            key, kts, cols, valid = rp.shuffle.unpack(recv, m, key_as_col=True)  # region = the key
            st = h.push(abi.DeviceBatch(kts, keys=key, cols=cols, col_valid=valid))
        else:  # the received rows read where they lie (khip_agg_push_shuffled)
            st = h.push_shuffled(rp.shuffle, recv, m)
        rows = h.count_rows(None)
        t3 = time.perf_counter()
        if state["timed"]:
            phases["pack"] += t1 - t0
            phases["exchange"] += t2 - t1
            phases["aggregate"] += t3 - t2
        state["m"] = m
        return st, rows, m

    for _ in range(max(args.warmup, 1)):
        st, rows, m = step()
    assert st["rows_accepted"] == m, st
    h.kernel_times(reset=True)
    state["timed"] = True
    (st, rows, m), elapsed = timed_loop(step, args.steps, world)
    kt = h.kernel_times()
    h.close()
    rp.close()
    if comm is not None:
        getattr(comm, "close", lambda: None)()
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    per = {k: v * 1000.0 / args.steps for k, v in phases.items()}
    pph = push_phases(kt, kt["apply_launches"])
    push_ms = sum(pph.values())
    roof = roofline(BYTES_PER_RECORD_C5 * n, ms_step, None, None, load_traffic(args.traffic_json, "repartition_sum", n),
                    BYTES_PER_RECORD_C5, kernel="whole step: pack + all-to-all + khip_agg_push_shuffled (or unpack + khip_agg_push) + row count",
                    extra={"phase_ms": per, "push_device_ms": push_ms,
                           "push_per_kernel": per_phase_block(pph, value_phase_bytes(not args.unpack), m)})
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_repartition(n, args.cpu_seconds)
    line("records/sec, non-key GROUP BY with repartition (SUM(amount) TUMBLING 1 MINUTE GROUP BY region_id)",
         world * n * args.steps / elapsed, world, args, ms_step, "int64",
         "synthetic (splitmix64, ksql_amd/synth.py repartition_sum), device-resident columnar batch",
         {"workload": "repartition_sum", "records_per_gpu": n, "regions": 1_000_000, "window": "TUMBLING 1 MINUTE",
          "parallelism": "repartition all-to-all x%d" % world, "exchange": args.exchange if world > 1 else None,
          "rows_received_rank0": m, "groups_rank0": int(rows),
          "aggregate_input": "columns (khip_shuffle_unpack)" if args.unpack else "shuffled rows (khip_agg_push_shuffled)"},
         roof, cpu)


def cpu_baseline_repartition(n_total, target_s):
    """Oracle C5 step on a prefix of rank 0's source partition: Kafka partitioner of the new key
    (oracle_kafka_partition, 8 destinations) + SUM(amount) TUMBLING 1 MINUTE GROUP BY region_id —
    1 thread, and P threads (partitioner over P chunks, aggregate over P key-hash shards)."""
    from ksql_amd import abi, synth
    orc = abi.load_oracle()
    P = cpu_threads()
    kw = dict(window_kind="TUMBLING", size_ms=60_000, key_type="INT64", col_types=["INT64", "INT64"],
              aggs=[("SUM", 1)])

    def run(m, threads):
        _eid, ts, region, amount = synth.repartition_sum(0, m, n_total)
        region = np.ascontiguousarray(region, np.int64)
        dest = np.empty(m, np.int32)
        b = abi.HostBatch(ts, keys=region, cols=[region, amount])
        h = abi.AggHandle(orc, abi.make_agg_desc(**kw)) if threads == 1 else \
            abi.ShardedOracleAgg(orc, abi.make_agg_desc(**kw), threads)
        bounds = np.linspace(0, m, threads + 1).astype(np.int64)

        def part(k):
            lo, hi = int(bounds[k]), int(bounds[k + 1])
            orc.dll.oracle_kafka_partition(region.ctypes.data + 8 * lo, hi - lo, 8, 8, dest.ctypes.data + 4 * lo)

        t0 = time.perf_counter()
        th = [threading.Thread(target=part, args=(k,)) for k in range(threads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        h.push(b, stats=False)
        dt = time.perf_counter() - t0
        h.close()
        return dt

    single = sized_run(lambda m: run(m, 1), 1_000_000, target_s, 40_000_000)
    ks = sized_run(lambda m: run(m, KS_THREADS), 2_000_000, target_s, 80_000_000)
    par = sized_run(lambda m: run(m, P), 2_000_000, target_s, 80_000_000)
    return cpu_baseline_block(single, par, P, "records/s",
                              "first %%d of rank 0's %d repartition_sum records: partitioner + aggregate, %%d threads"
                              % n_total, ks)


if __name__ == "__main__":
    sys.exit(main())
