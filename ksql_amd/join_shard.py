"""Sharded stream-table join with probe routing (the option beside replicating
the table on every GPU).

StreamTableJoinBuilder (ksqldb-streams/.../StreamTableJoinBuilder.java:77-86) joins a stream with a
table co-partitioned with it: both sides are keyed by the join key over the same partition count,
so a task holds the table rows of its partitions and sees exactly the stream records with those
keys.  Here there is one task per GPU: rank r owns the keys that Kafka's default partitioner
sends to partition r of `world`.  That partitioner is murmur2 of the KAFKA-format key bytes, the
repartition topic's own.

- Table changelog rows and stream rows reach their owner through the device shuffle
  (khip_shuffle_pack → exchange → khip_shuffle_unpack, ksql_amd/repartition.py).
- The owner upserts or probes its shard (khip_table_upsert / khip_table_probe_device).
- The join's output rows stay on the owner, as the reference's task writes its join output.

Tombstones travel as a flag column: the shuffle drops rows without a value, as a stream
repartition must.  Stream rows that the join drops anyway (null key or value, negative ts;
KStreamKTableJoin skips them) are dropped by the shuffle at the source.
"""
from . import abi
from .repartition import Repartition


class ShardedTable:
    """One rank's shard of a join table plus the two routes into it.

    `comm` is the exchange (abi.Comm over RCCL, or repartition.GlooExchange); world 1 needs none.
    """

    def __init__(self, lib, col_types, rank=0, world=1, comm=None, device=0, capacity_hint=0, key_type="INT64"):
        import torch
        self.torch = torch
        self.col_types = list(col_types)
        self.rank, self.world, self.device = rank, world, device
        shard_hint = capacity_hint // max(world, 1) + (capacity_hint > 0)
        self.table = abi.TableHandle(lib, self.col_types, device=device, capacity_hint=shard_hint, key_type=key_type)
        # table rows: [key, value columns..., tombstone flag]; stream rows: [key, passthrough columns...]
        self._up = Repartition(lib, 0, [key_type] + self.col_types + ["INT32"], rank, world, comm, device)
        self._stream_types = None
        self._pr = None
        self._lib, self._comm, self._key_type = lib, comm, key_type

    def _route_stream(self, stream_types):
        if self._pr is None or self._stream_types != stream_types:
            if self._pr is not None:
                self._pr.close()
            self._pr = Repartition(self._lib, 0, [self._key_type] + stream_types, self.rank, self.world, self._comm,
                                   self.device)
            self._stream_types = stream_types
        return self._pr

    def upsert(self, keys, ts, cols=(), col_valid=None, deleted=None, key_valid=None):
        """This rank's source changelog rows (device tensors): keys, ts, the value columns, their
        validity (bool tensors or None), `deleted` (bool: tombstone rows) → routed to the key
        owners, each owner upserting what it received in (source rank, arrival) order."""
        torch = self.torch
        n = ts.shape[0]
        flag = (deleted.to(torch.int32) if deleted is not None
                else torch.zeros(n, dtype=torch.int32, device=ts.device))
        cv = list(col_valid) if col_valid is not None else [None] * len(cols)
        bitmaps = [None if key_valid is None else abi.bitmap_torch(key_valid)]
        bitmaps += [None if v is None else abi.bitmap_torch(v) for v in cv] + [None]
        src = abi.DeviceBatch(ts, cols=[keys] + list(cols) + [flag], col_valid=bitmaps)
        recv, m = self._up.exchange(src)
        key, rts, rcols, rvalid = self._up.shuffle.unpack(recv, m)
        if m == 0:
            return 0
        live = abi.bitmap_torch(rcols[-1] == 0)
        batch = abi.DeviceBatch(rts, keys=key, cols=rcols[1:-1], col_valid=rvalid[1:-1], row_valid=live)
        batch._keep.append(recv)
        self.table.upsert(batch)
        return m

    def probe(self, keys, ts, join_type="LEFT", where=None, cols=(), stream_types=(), key_valid=None,
              row_valid=None):
        """This rank's stream rows (device tensors; `cols` are passthrough columns of
        `stream_types`) → routed to the key owners → probed against this rank's shard.  Returns
        the rows this rank received (key, ts, passthrough columns: the left side of the join
        output) and the probe's row-aligned outputs (emit / matched bitmaps, right columns and
        their null bitmaps) and the emitted count."""
        torch = self.torch
        rp = self._route_stream(list(stream_types))
        bitmaps = [None if key_valid is None else abi.bitmap_torch(key_valid)] + [None] * len(cols)
        src = abi.DeviceBatch(ts, cols=[keys] + list(cols), col_valid=bitmaps,
                              row_valid=None if row_valid is None else abi.bitmap_torch(row_valid))
        recv, m = rp.exchange(src)
        key, rts, rcols, _ = rp.shuffle.unpack(recv, m)
        dev = torch.device("cuda", self.device)
        nb = (m + 7) // 8
        tdt = {"INT32": torch.int32, "INT64": torch.int64, "DOUBLE": torch.float64}
        out = {"key": key, "ts": rts, "cols": rcols[1:], "n": m,
               "emit": torch.zeros(max(nb, 1), dtype=torch.uint8, device=dev),
               "matched": torch.zeros(max(nb, 1), dtype=torch.uint8, device=dev),
               "right": [torch.zeros(max(m, 1), dtype=tdt[t], device=dev) for t in self.col_types],
               "right_null": [torch.zeros(max(nb, 1), dtype=torch.uint8, device=dev) for _ in self.col_types]}
        if m == 0:
            out["emitted"] = 0
            return out
        batch = abi.DeviceBatch(rts, keys=key)
        batch._keep.append(recv)
        out["emitted"] = self.table.probe_device(batch, join_type, where, out["emit"], out["matched"], out["right"],
                                                 out["right_null"])
        return out

    def size(self):
        return self.table.size()

    def close(self):
        self.table.close()
        self._up.close()
        if self._pr is not None:
            self._pr.close()
