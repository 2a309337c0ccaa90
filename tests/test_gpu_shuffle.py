"""Parity of the repartition path (khip_shuffle_* + khip_comm_*, through the C ABI).

1. pack: the packed rows equal a numpy restatement built on the oracle's Kafka partitioner
   (rule R8, pinned by Kafka's murmur2 known answers): same rows, same destination, same
   order (stable per source), null value / null new key / negative ts dropped
   (S/GroupByParamsFactory.java:92-100), bit-exact words.
2. unpack(pack(x)) restores the columns of the surviving rows exactly.
3. Non-key GROUP BY end to end with N simulated source tasks on one GPU: each destination
   task's aggregate (product) equals the oracle run over the same re-keyed rows in the same
   order, and the union over tasks equals one task over every record (no late drops here).
4. RCCL on one rank: the library's communicator moves rows to itself unchanged.
"""
import numpy as np
import pytest
import torch

from ksql_amd import abi, synth
from pg_store import init_gloo, store_url
from ksql_amd.repartition import Repartition
from shuffle_ref import expected_pack, kafka_partition

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def _kafka_partition(orc, keys, width, n_parts):
    return kafka_partition(orc, keys, width, n_parts)


def _random_source(n, key_type, seed, null_frac=0.05):
    rng = np.random.default_rng(seed)
    if key_type == "INT32":
        key = rng.integers(-(1 << 31), 1 << 31, n, dtype=np.int64).astype(np.int32)
    else:
        key = rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64)
    v32 = rng.integers(-(1 << 31), 1 << 31, n, dtype=np.int64).astype(np.int32)
    vd = rng.standard_normal(n) * 1e6
    cols = [key, v32, vd]
    types = [key_type, "INT32", "DOUBLE"]
    col_valid = [rng.random(n) > null_frac for _ in cols]
    row_valid = rng.random(n) > null_frac
    ts = rng.integers(0, 1 << 40, n, dtype=np.int64)
    ts[rng.random(n) < 0.01] = -5
    return cols, types, col_valid, row_valid, ts


def _device_batch(cols, col_valid, row_valid, ts):
    dev = "cuda"
    tcols = [torch.from_numpy(c).to(dev) for c in cols]
    tval = [abi.bitmap_torch(torch.from_numpy(v).to(dev)) for v in col_valid]
    rv = abi.bitmap_torch(torch.from_numpy(row_valid).to(dev))
    tts = torch.from_numpy(ts).to(dev)
    return abi.DeviceBatch(tts, row_valid=rv, cols=tcols, col_valid=tval)


@pytest.mark.parametrize("key_type", ["INT64", "INT32"])
@pytest.mark.parametrize("n_parts", [1, 2, 3, 8, 64, 256])
def test_pack_matches_oracle_partitioner(prod, orc, key_type, n_parts):
    n = 70_001
    cols, types, cv, rv, ts = _random_source(n, key_type, seed=n_parts)
    sh = abi.ShuffleHandle(prod, n_parts, 0, types)
    send, counts = sh.pack(_device_batch(cols, cv, rv, ts))
    exp_rows, exp_counts = expected_pack(orc, 0, cols, cv, rv, ts, n_parts)
    assert counts == exp_counts
    got = send[: sum(counts)].cpu().numpy()
    assert got.shape == exp_rows.shape
    np.testing.assert_array_equal(got, exp_rows)
    sh.close()


@pytest.mark.parametrize("key_type", ["INT64", "INT32"])
@pytest.mark.parametrize("n", [1, 4095, 4097, 70_001, 1_000_003])
def test_pack_one_destination_one_pass(prod, orc, key_type, n):
    """One destination with a send buffer for every row: k_shuf_count1 + scan + k_shuf_write1 (no
    histogram pass, no look-back) — the same rows, in the same order, as the oracle."""
    import torch
    cols, types, cv, rv, ts = _random_source(n, key_type, seed=n)
    sh = abi.ShuffleHandle(prod, 1, 0, types)
    send = torch.empty((n, sh.row_words), dtype=torch.int64, device="cuda")
    out, counts = sh.pack(_device_batch(cols, cv, rv, ts), send=send)
    exp_rows, exp_counts = expected_pack(orc, 0, cols, cv, rv, ts, 1)
    assert counts == exp_counts
    np.testing.assert_array_equal(out[: counts[0]].cpu().numpy(), exp_rows)
    sh.close()


@pytest.mark.parametrize("key_col", [0, 1])
def test_unpack_round_trip(prod, orc, key_col):
    n = 50_000
    cols, types, cv, rv, ts = _random_source(n, "INT64", seed=7 + key_col)
    sh = abi.ShuffleHandle(prod, 4, key_col, types)
    send, counts = sh.pack(_device_batch(cols, cv, rv, ts))
    m = sum(counts)
    key, uts, ucols, uvalid = sh.unpack(send, m)
    ok = rv & cv[key_col] & (ts >= 0)
    dest = _kafka_partition(orc, cols[key_col], 4 if cols[key_col].dtype == np.int32 else 8, 4)
    order = np.concatenate([np.nonzero(ok & (dest == d))[0] for d in range(4)])
    np.testing.assert_array_equal(key.cpu().numpy(), cols[key_col][order].astype(np.int64))
    np.testing.assert_array_equal(uts.cpu().numpy(), ts[order])
    for c in range(len(cols)):
        valid = np.unpackbits(uvalid[c].cpu().numpy(), bitorder="little")[:m].astype(bool)
        np.testing.assert_array_equal(valid, cv[c][order])
        got = ucols[c].cpu().numpy()
        np.testing.assert_array_equal(got[valid].view(np.int64) if got.dtype == np.float64 else got[valid],
                                      cols[c][order][valid].view(np.int64) if got.dtype == np.float64
                                      else cols[c][order][valid])
    sh.close()


def test_pack_empty_and_all_dropped(prod):
    sh = abi.ShuffleHandle(prod, 3, 0, ["INT64", "INT64"])
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    send, counts = sh.pack(abi.DeviceBatch(e, cols=[e, e]))
    assert counts == [0, 0, 0]
    n = 1000
    ts = torch.arange(n, dtype=torch.int64, device="cuda")
    k = torch.arange(n, dtype=torch.int64, device="cuda")
    null = abi.bitmap_torch(torch.zeros(n, dtype=torch.bool, device="cuda"))
    send, counts = sh.pack(abi.DeviceBatch(ts, cols=[k, k], col_valid=[null, None]))
    assert counts == [0, 0, 0]
    key, uts, ucols, uvalid = sh.unpack(None, 0)
    assert key.numel() == 0
    sh.close()


def test_pack_large_property(prod, orc):
    """2^24 rows, 8 destinations: counts and per-row routing equal the oracle partitioner."""
    n = 1 << 24
    eid, ts, region, amount = synth.repartition_sum(0, n, n, xp="torch", device="cuda", rank=0, world=1)
    sh = abi.ShuffleHandle(prod, 8, 0, ["INT64", "INT64"])
    send, counts = sh.pack(abi.DeviceBatch(ts, cols=[region, amount]))
    assert sum(counts) == n
    dest = _kafka_partition(orc, region.cpu().numpy(), 8, 8)
    assert counts == np.bincount(dest, minlength=8).tolist()
    rows = send[:n].cpu().numpy()
    off = 0
    for d in range(8):
        seg = rows[off:off + counts[d]]
        assert (_kafka_partition(orc, seg[:, 0], 8, 8) == d).all()
        assert (np.diff(seg[:, 1]) > -1000).all()  # arrival order (ts nondecreasing up to disorder)
        off += counts[d]
    # multiset of (region, ts, amount) preserved: order-independent checksum of checksums
    def mix(a, b, c):
        with np.errstate(over="ignore"):
            z = a.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) ^ b.astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9) \
                ^ c.astype(np.uint64) * np.uint64(0x94D049BB133111EB)
            z ^= z >> np.uint64(29)
            return int(z.sum(dtype=np.uint64))
    assert mix(region.cpu().numpy(), ts.cpu().numpy(), amount.cpu().numpy()) == mix(rows[:, 0], rows[:, 1], rows[:, 2])
    sh.close()


WORLD = 3
N_SRC = 40_000


def _agg_desc(device=0):
    return abi.make_agg_desc(window_kind="TUMBLING", size_ms=60_000, key_type="INT64",
                             col_types=["INT64", "INT64"], aggs=[("SUM", 1), ("COUNT_STAR", -1)], device=device)


def _sorted_snap(s):
    o = np.lexsort((s["ws"], s["key"]))
    return {k: (s[k][o] if k in ("key", "ws", "we", "rowtime") else [v[o] for v in s[k]])
            for k in ("key", "ws", "we", "rowtime", "values", "nulls")}


def test_non_key_group_by_simulated_tasks(prod, orc):
    """C5 at small size: WORLD source tasks → pack → (all-to-all emulated on one GPU) →
    unpack → per-task SUM(amount) TUMBLING 1 MINUTE GROUP BY region_id."""
    srcs = [synth.repartition_sum(0, N_SRC, N_SRC, xp="torch", device="cuda", rank=r, world=WORLD, regions=500)
            for r in range(WORLD)]
    sends = []
    for eid, ts, region, amount in srcs:
        sh = abi.ShuffleHandle(prod, WORLD, 0, ["INT64", "INT64"])
        sends.append(sh.pack(abi.DeviceBatch(ts, cols=[region, amount])))
        sh.close()
    host = [tuple(t.cpu().numpy() for t in s) for s in srcs]
    union = []
    for d in range(WORLD):
        # what the all-to-all delivers to task d: source 0's rows for d, then source 1's, ...
        parts = []
        for s, (send, counts) in enumerate(sends):
            off = sum(counts[:d])
            parts.append(send[off:off + counts[d]])
        recv = torch.cat(parts)
        sh = abi.ShuffleHandle(prod, WORLD, 0, ["INT64", "INT64"])
        key, ts, cols, valid = sh.unpack(recv, recv.shape[0])
        h = abi.AggHandle(prod, _agg_desc())
        h.push(abi.DeviceBatch(ts, keys=key, cols=cols, col_valid=valid))
        got = _sorted_snap(h.snapshot())
        h.close()
        sh.close()
        # oracle over the same re-keyed rows in the same order
        rk, rts, ramt = [], [], []
        for eid, t, region, amount in host:
            sel = _kafka_partition(orc, region, 8, WORLD) == d
            rk.append(region[sel]), rts.append(t[sel]), ramt.append(amount[sel])
        rk, rts, ramt = np.concatenate(rk), np.concatenate(rts), np.concatenate(ramt)
        ho = abi.AggHandle(orc, _agg_desc())
        ho.push(abi.HostBatch(rts, keys=rk, cols=[rk, ramt]))
        exp = _sorted_snap(ho.snapshot())
        ho.close()
        for k in ("key", "ws", "we", "rowtime"):
            np.testing.assert_array_equal(got[k], exp[k])
        for a in range(2):
            np.testing.assert_array_equal(got["values"][a], exp["values"][a])
        union.append(exp)
    # union over tasks == one task over every record (grace default: nothing late)
    allk = np.concatenate([h_[2] for h_ in host])
    allt = np.concatenate([h_[1] for h_ in host])
    alla = np.concatenate([h_[3] for h_ in host])
    ho = abi.AggHandle(orc, _agg_desc())
    ho.push(abi.HostBatch(allt, keys=allk, cols=[allk, alla]))
    g = _sorted_snap(ho.snapshot())
    ho.close()
    uk = np.concatenate([u["key"] for u in union])
    uw = np.concatenate([u["ws"] for u in union])
    us = np.concatenate([u["values"][0] for u in union])
    o = np.lexsort((uw, uk))
    np.testing.assert_array_equal(uk[o], g["key"])
    np.testing.assert_array_equal(uw[o], g["ws"])
    np.testing.assert_array_equal(us[o], g["values"][0])


def test_rccl_single_rank_alltoall(prod):
    uid = abi.comm_unique_id(prod)
    comm = abi.Comm(prod, 1, 0, uid, 0)
    n = 12_345
    eid, ts, region, amount = synth.repartition_sum(0, n, n, xp="torch", device="cuda")
    rp = Repartition(prod, 0, ["INT64", "INT64"], rank=0, world=1)
    sh = rp.shuffle
    send, counts = sh.pack(abi.DeviceBatch(ts, cols=[region, amount]))
    recv, rc = comm.alltoall(send, counts, sh.row_words)
    assert rc == counts
    torch.testing.assert_close(recv[:n], send[:n], rtol=0, atol=0)
    out = rp(abi.DeviceBatch(ts, cols=[region, amount]))
    assert out.struct.n_rows == n
    comm.close()
    rp.close()


# ---- two source tasks in two processes (both on cuda:0), rows exchanged over gloo ----------
import os

import torch.multiprocessing as mp

MP_WORLD = 2
MP_N = 60_000


def _mp_worker(rank, port, q):
    import torch.distributed as dist
    from ksql_amd.repartition import GlooExchange
    init_gloo(port, rank, MP_WORLD)
    try:
        torch.cuda.init()
        prod = abi.load_product()
        eid, ts, region, amount = synth.repartition_sum(0, MP_N, MP_N, xp="torch", device="cuda", rank=rank,
                                                        world=MP_WORLD, regions=400)
        rp = Repartition(prod, 0, ["INT64", "INT64"], rank=rank, world=MP_WORLD, comm=GlooExchange())
        out = rp(abi.DeviceBatch(ts, cols=[region, amount]))
        h = abi.AggHandle(prod, _agg_desc())
        h.push(out)
        s = h.snapshot()
        h.close()
        res = {"src": tuple(t.cpu().numpy() for t in (region, ts, amount)), "counts": rp.last_counts,
               "snap": (s["key"], s["ws"], s["values"][0], s["values"][1], s["rowtime"])}
        rp.close()
        gathered = [None] * MP_WORLD
        dist.all_gather_object(gathered, res)
        if rank == 0:
            q.put(gathered)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_process_repartition_gloo(orc):
    """Product pack → exchange between two processes → product unpack → product aggregate, per
    task equal to the oracle over the rows Kafka's partitioner routes to it (source order)."""
    port = store_url()  # (a FileStore: pg_store.py)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_mp_worker, args=(r, port, q)) for r in range(MP_WORLD)]
    for p in procs:
        p.start()
    g = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for d in range(MP_WORLD):
        rk, rts, ramt = [], [], []
        for src in range(MP_WORLD):
            region, ts, amount = g[src]["src"]
            sel = _kafka_partition(orc, region, 8, MP_WORLD) == d
            rk.append(region[sel]), rts.append(ts[sel]), ramt.append(amount[sel])
        assert g[d]["counts"][1] == [g[src]["counts"][0][d] for src in range(MP_WORLD)]
        rk, rts, ramt = np.concatenate(rk), np.concatenate(rts), np.concatenate(ramt)
        ho = abi.AggHandle(orc, _agg_desc())
        ho.push(abi.HostBatch(rts, keys=rk, cols=[rk, ramt]))
        exp = ho.snapshot()
        ho.close()
        key, ws, sm, cn, rt = g[d]["snap"]
        np.testing.assert_array_equal(key, exp["key"])
        np.testing.assert_array_equal(ws, exp["ws"])
        np.testing.assert_array_equal(sm, exp["values"][0])
        np.testing.assert_array_equal(cn, exp["values"][1])
        np.testing.assert_array_equal(rt, exp["rowtime"])


def test_rccl_error_paths_single_rank(prod):
    """khip_comm_* argument validation and the capacity check that runs before any group opens
    (a capacity error there must not leave a half-open group: the next call still works)."""
    uid = abi.comm_unique_id(prod)
    c = abi.Comm(prod, 1, 0, uid, 0)
    sc = (abi.i64 * 1)(5)
    rc = (abi.i64 * 1)(5)
    recv = torch.empty((4, 3), dtype=torch.int64, device="cuda")
    send = torch.arange(15, dtype=torch.int64, device="cuda").reshape(5, 3)
    st = prod.comm_alltoall(c.h, send.data_ptr(), sc, recv.data_ptr(), 4, rc, 3)
    assert st == abi.KHIP_E_BUFFER, st
    assert prod.comm_alltoall(None, send.data_ptr(), sc, recv.data_ptr(), 4, rc, 3) == -1
    assert prod.comm_alltoall(c.h, send.data_ptr(), sc, recv.data_ptr(), 4, rc, 0) == -1
    assert prod.comm_exchange_counts(c.h, None, rc) == -1
    out, counts = c.alltoall(send, [5], 3)  # the communicator is still usable
    assert counts == [5] and torch.equal(out[:5], send)
    c.close()


def test_bench_repartition_two_ranks_one_gpu_gloo():
    """bench.py's own repartition step loop at N = 2 (both ranks on this GPU, the exchange over a
    gloo group): the multi-rank branches of the leg, the barrier and the max-over-ranks timing."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--config", "repartition_sum", "--gpus", "2",
                        "--exchange", "gloo", "--one-device", "--records", "2000000", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], cwd=repo, env=env, capture_output=True, text=True, timeout=220)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["exchange"] == "gloo"
    assert d["value"] > 0 and d["config"]["rows_received_rank0"] > 0
