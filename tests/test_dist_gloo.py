"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path.

bench.py shards the key space across ranks (rank r owns keys k with k % N == r, the
Kafka key-partitioning analogue) and runs one independent task per rank with its own
stream time; the final table is the disjoint union of the shards and the throughput is
all records / max-over-ranks time.  Here each rank runs the CPU oracle on its shard
(the GPU path is covered by the -m gpu parity tests), and rank 0 checks that the union
equals one task over all records (no late drops at this disorder),
and that the max-over-ranks reduction the bench uses is what it claims.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ksql_amd import abi, synth
from pg_store import init_gloo, store_url

WORLD = 2
N = 30_000
KEYS = 700


def _free_port():
    return store_url()  # the process group's FileStore (pg_store.py), not a TCP port


def _shard_snapshot(rank, world):
    card, ts = synth.possible_fraud(0, N, N, rank=rank, world=world, keys=KEYS)
    h = abi.AggHandle(abi.load_oracle(), abi.make_agg_desc(window_kind="TUMBLING", size_ms=5000,
                                                           key_type="INT64", aggs=[("COUNT_STAR", -1)]))
    h.push(abi.HostBatch(ts, keys=card))
    s = h.snapshot()
    h.close()
    return card, ts, s


def _worker(rank, port, q):
    init_gloo(port, rank, WORLD)
    try:
        card, ts, s = _shard_snapshot(rank, WORLD)
        shard = {"key": s["key"], "ws": s["ws"], "cnt": s["values"][0], "rt": s["rowtime"],
                 "card": card, "ts": ts}
        gathered = [None] * WORLD
        dist.all_gather_object(gathered, shard)
        # the bench's timing reduction: MAX over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((gathered, float(t.item())))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_key_sharded_union_equals_single_task():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    gathered, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(WORLD)
    # shards own disjoint keys
    k0, k1 = set(gathered[0]["key"].tolist()), set(gathered[1]["key"].tolist())
    assert not (k0 & k1)
    # union of shard tables == one task over every record (arrival order: shard 0 then 1)
    card = np.concatenate([g["card"] for g in gathered])
    ts = np.concatenate([g["ts"] for g in gathered])
    h = abi.AggHandle(abi.load_oracle(), abi.make_agg_desc(window_kind="TUMBLING", size_ms=5000,
                                                           key_type="INT64", aggs=[("COUNT_STAR", -1)]))
    h.push(abi.HostBatch(ts, keys=card))
    ref = h.snapshot()
    h.close()
    key = np.concatenate([g["key"] for g in gathered])
    ws = np.concatenate([g["ws"] for g in gathered])
    cnt = np.concatenate([g["cnt"] for g in gathered])
    rt = np.concatenate([g["rt"] for g in gathered])
    order = np.lexsort((ws, key))
    assert np.array_equal(key[order], ref["key"])
    assert np.array_equal(ws[order], ref["ws"])
    assert np.array_equal(cnt[order], ref["values"][0])
    assert np.array_equal(rt[order], ref["rowtime"])
    assert cnt.sum() == WORLD * N


# ------------------------------------------------------------------ repartition across ranks
# a non-key GROUP BY is one exchange step.  Each rank is one source task:
# pack (the contract restated on the oracle's Kafka partitioner, tests/shuffle_ref.py) →
# GlooExchange (the two collective steps abi.Comm runs over RCCL, here over gloo) → unpack →
# aggregate (oracle).  Rank 0 checks what each task received and the union of the tables.

SH_N = 20_000
SH_COLS = ["INT64", "INT64"]  # region_id (the new key), amount


def _shuffle_desc():
    return abi.make_agg_desc(window_kind="TUMBLING", size_ms=60_000, key_type="INT64", col_types=SH_COLS,
                             aggs=[("SUM", 1), ("COUNT_STAR", -1)])


def _shuffle_worker(rank, port, q):
    from shuffle_ref import expected_pack, expected_unpack
    from ksql_amd.repartition import GlooExchange
    init_gloo(port, rank, WORLD)
    try:
        orc = abi.load_oracle()
        eid, ts, region, amount = synth.repartition_sum(0, SH_N, SH_N, rank=rank, world=WORLD, regions=300)
        n = len(ts)
        ones = np.ones(n, bool)
        rows, counts = expected_pack(orc, 0, [region, amount], [ones, ones], ones, ts, WORLD)
        ex = GlooExchange()
        recv, rcounts = ex.alltoall(torch.from_numpy(rows), counts, rows.shape[1])
        recv = recv[:sum(rcounts)].numpy()
        key, rts, cols, valid = expected_unpack(recv, 0, SH_COLS)
        h = abi.AggHandle(orc, _shuffle_desc())
        h.push(abi.HostBatch(rts, keys=key, cols=cols, col_valid=valid))
        s = h.snapshot()
        h.close()
        out = {"src": (region, ts, amount), "recv": recv, "rcounts": rcounts,
               "snap": (s["key"], s["ws"], s["values"][0], s["values"][1], s["rowtime"])}
        gathered = [None] * WORLD
        dist.all_gather_object(gathered, out)
        if rank == 0:
            q.put(gathered)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_repartition_exchange_across_ranks():
    from shuffle_ref import expected_pack, kafka_partition
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shuffle_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    g = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    orc = abi.load_oracle()
    # task d receives source 0's rows for d, then source 1's, each in arrival order
    packs = []
    for s in range(WORLD):
        region, ts, amount = g[s]["src"]
        ones = np.ones(len(ts), bool)
        packs.append(expected_pack(orc, 0, [region, amount], [ones, ones], ones, ts, WORLD))
    for d in range(WORLD):
        exp = np.concatenate([rows[sum(c[:d]):sum(c[:d + 1])] for rows, c in packs])
        assert g[d]["rcounts"] == [c[d] for _, c in packs]
        np.testing.assert_array_equal(g[d]["recv"], exp)
        # every received key routes here
        assert (kafka_partition(orc, g[d]["recv"][:, 0], 8, WORLD) == d).all()
    # tasks own disjoint new keys; union of their tables == one task over every record
    keys = [set(g[d]["snap"][0].tolist()) for d in range(WORLD)]
    assert not (keys[0] & keys[1])
    allr = np.concatenate([g[s]["src"][0] for s in range(WORLD)])
    allt = np.concatenate([g[s]["src"][1] for s in range(WORLD)])
    alla = np.concatenate([g[s]["src"][2] for s in range(WORLD)])
    h = abi.AggHandle(orc, _shuffle_desc())
    h.push(abi.HostBatch(allt, keys=allr, cols=[allr, alla]))
    ref = h.snapshot()
    h.close()
    k, ws, sm, cn, rt = (np.concatenate([g[d]["snap"][i] for d in range(WORLD)]) for i in range(5))
    o = np.lexsort((ws, k))
    np.testing.assert_array_equal(k[o], ref["key"])
    np.testing.assert_array_equal(ws[o], ref["ws"])
    np.testing.assert_array_equal(sm[o], ref["values"][0])
    np.testing.assert_array_equal(cn[o], ref["values"][1])
    np.testing.assert_array_equal(rt[o], ref["rowtime"])
    assert cn.sum() == WORLD * SH_N


# ------------------------------------------------------------------ ABI 7 exchange shapes
# khip_shuffle_pack_v leaves each destination's rows in its own region of the send buffer (gaps
# between regions); the exchange sends region p to peer p (send_offsets), and the GLOBAL stream
# time needs one int64 from every rank (allgather_i64).

def _regions_worker(rank, port, q):
    from ksql_amd.repartition import GlooExchange
    init_gloo(port, rank, WORLD)
    try:
        ex = GlooExchange()
        rw = 3
        counts = [3 + rank, 5 - rank]
        offs = [2, 20]  # regions with gaps before, between and after them
        send = torch.full((30, rw), -1, dtype=torch.int64)
        for p in range(WORLD):
            for i in range(counts[p]):
                send[offs[p] + i] = torch.tensor([rank, p, i])
        recv, rc = ex.alltoall(send, counts, rw, send_offsets=offs)
        got = ex.allgather_i64(1000 + 7 * rank)
        out = {"recv": recv[:sum(rc)].numpy(), "rc": rc, "gathered": got}
        res = [None] * WORLD
        dist.all_gather_object(res, out)
        if rank == 0:
            q.put(res)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_exchange_regions_and_allgather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_regions_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for d in range(WORLD):
        exp = [[s, d, i] for s in range(WORLD) for i in range([3 + s, 5 - s][d])]
        assert res[d]["rc"] == [[3 + s, 5 - s][d] for s in range(WORLD)]
        np.testing.assert_array_equal(res[d]["recv"], np.array(exp, np.int64))
        assert res[d]["gathered"] == [1000 + 7 * r for r in range(WORLD)]
