"""Host side of the repartition step for a non-key GROUP BY / PARTITION BY.

Mirrors what StreamGroupByBuilderBase.build does per task
(ksqldb-streams/.../StreamGroupByBuilderBase.java:101-103: filter(v != null).groupBy(mapper)
→ sink "<ctx>-repartition" → source, i.e. the shuffle of SURVEY.md §8(e)) with the device
pieces of libksqldb_hip.so:

    khip_shuffle_pack[_v]  re-key by the group-by column, route with Kafka's default
                           partitioner (murmur2 of the KAFKA-format key), stable per source;
                           one destination: a one-pass compaction; several: the one-pass
                           region pack (ABI 7), each destination's rows at its own offset
    khip_comm_*            RCCL count exchange + grouped send/recv all-to-all over xGMI
                           (skipped at one task: the destination is this task)
    khip_shuffle_unpack    back to a columnar device batch keyed by the new key

The result feeds khip_agg_push exactly like a batch read back from the repartition topic:
records from source rank 0 first, then rank 1, ..., each source's records in arrival order — or
goes straight into the aggregation with khip_agg_push_shuffled (Repartition.push_into: the rows
are read where they lie, no columnar copy).

GLOBAL stream time (`global_time=True`, ABI 7 KHIP_SHUFFLE_STREAM_TIME): the owner tasks late-drop
against the stream time ONE task over the whole stream would have observed — what the reference's
TopologyTestDriver does (one task per query, ksqldb-functional-tests/.../TestExecutorUtil.java:
123-126).  Each rank holds a contiguous chunk of the global arrival order; before routing, it scans
its chunk's per-row stream time (khip_stream_time_scan) seeded with max(the global stream time
before the batch, the chunk maxima of the ranks before it) — an all-gather of one int64 per rank —
and the rows travel with it; the owner's aggregation is KHIP_TIME_SUPPLIED.

The exchange is pluggable: `abi.Comm` (RCCL over xGMI, one process per GPU, the production
path) or `GlooExchange` (any torch.distributed process group, rows staged through host memory:
the CPU tests, and several ranks sharing one GPU, where RCCL refuses duplicate devices).
"""
from . import abi


class GlooExchange:
    """The same collective steps as abi.Comm (counts, then rows laid out by source rank; one
    int64 from every rank) over a torch.distributed group, through host memory."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.nranks = dist.get_world_size(group)

    def alltoall(self, send, send_counts, row_words, send_offsets=None):
        import torch
        dist = self.dist
        if len(send_counts) != self.nranks:
            raise ValueError("send_counts has %d entries, world is %d" % (len(send_counts), self.nranks))
        sc = torch.tensor(list(send_counts), dtype=torch.int64)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=self.group)
        rcounts = [int(x) for x in rc.tolist()]
        n_send = int(sc.sum())
        dev = send.device if send is not None else torch.device("cpu")
        if send is None or n_send == 0:
            hsend = torch.empty((0, row_words), dtype=torch.int64)
        elif send_offsets is None:
            hsend = send[:n_send].to("cpu").contiguous()
        else:  # khip_shuffle_pack_v's regions, peer by peer
            hsend = torch.cat([send[o:o + c].to("cpu") for o, c in zip(send_offsets, send_counts)]).contiguous()
        hrecv = torch.empty((sum(rcounts), row_words), dtype=torch.int64)
        dist.all_to_all_single(hrecv.view(-1), hsend.view(-1), [c * row_words for c in rcounts],
                               [int(c) * row_words for c in send_counts], group=self.group)
        if hrecv.shape[0] == 0:
            hrecv = torch.zeros((1, row_words), dtype=torch.int64)
        return hrecv.to(dev), rcounts

    def allgather_i64(self, x):
        import torch
        out = torch.zeros(self.nranks, dtype=torch.int64)
        self.dist.all_gather_into_tensor(out, torch.tensor([int(x)], dtype=torch.int64), group=self.group)
        return [int(v) for v in out.tolist()]

    def allgather_ranges(self, ranges):
        """Every rank's list of (lo, hi) pairs, concatenated in rank order."""
        out = [None] * self.nranks
        self.dist.all_gather_object(out, list(ranges), group=self.group)
        return [tuple(r) for rs in out for r in rs]


class _StreamTimeBatch:
    """The caller's device batch with a stream_time column attached (a copy of its struct)."""

    def __init__(self, batch, st):
        self.struct = abi.Batch.from_buffer_copy(batch.struct)
        self.struct.stream_time = st.data_ptr()
        self._keep = [batch, st]


class _RekeyedView:
    """The caller's batch as the GROUP BY sees it for the stream-time scan: the key validity is
    the GROUP BY column's (all valid when the batch has no bitmap for it)."""

    def __init__(self, batch, key_col):
        self.struct = abi.Batch.from_buffer_copy(batch.struct)
        cv = batch.struct.col_valid
        self.struct.key_valid = cv[key_col] if cv else None
        self._keep = batch


class Repartition:
    def __init__(self, lib, key_col, col_types, rank=0, world=1, comm=None, device=0, global_time=False):
        if world > 1 and comm is None:
            raise ValueError("world > 1 needs an exchange (abi.Comm over RCCL, or GlooExchange)")
        self.world = world
        self.rank = rank
        self.comm = comm
        self.global_time = bool(global_time)
        self.shuffle = abi.ShuffleHandle(lib, world, key_col, col_types, device, stream_time=global_time)
        self.last_counts = None
        self.gst = -1  # global_time: the stream time over every rank's rows so far
        self._send = None

    def stream_times(self, scan, batch):
        """global_time: the GLOBAL stream time observed at each row of this rank's chunk (device
        int64 tensor), as the pack will write it.  `scan` is any product AggHandle
        (khip_stream_time_scan only uses its scratch).

        Which rows raise it: those that reach the owner's aggregate — a non-null value
        (StreamGroupByBuilderBase.java:102 filters null values), a non-null GROUP BY column
        (GroupByParamsFactory.java:92-100: a null one excludes the row, so Kafka Streams' repartition
        never forwards it) and ts >= 0 — the pack's own row test.  The source key plays no part, so
        the scan sees the batch re-keyed by the GROUP BY column (its validity as the key bitmap).

        One pass per rank: the chunk is scanned unseeded; the seed (the global stream time before
        the batch and the chunk maxima of the ranks before this one) is applied by the pack as
        max(seed, st[i]) (khip_shuffle_stream_time_seed): a seeded prefix max is the unseeded one
        raised to the seed."""
        import torch
        n = int(batch.struct.n_rows)
        out = torch.empty(max(n, 1), dtype=torch.int64, device=torch.device("cuda", self.shuffle.device))
        _, mx = scan.stream_time_scan(_RekeyedView(batch, self.shuffle.desc.key_col), -1, out)
        maxima = self.comm.allgather_i64(mx) if self.world > 1 else [mx]
        seed = max([self.gst] + maxima[:self.rank])
        self.shuffle.stream_time_seed(seed)
        before = self.gst
        self.gst = max([self.gst] + maxima)
        self._ctx = (seed, before, self.gst)
        return out[:n]

    def final_context(self, agg, batch):
        """global_time + EMIT FINAL (ABI 8): the owner closes windows by the GLOBAL stream time, as
        one task over the whole stream (StreamAggregateBuilder.java:282-285).  After exchange():
        this rank's chunk's lost windows (khip_agg_lost_windows: closed after they expired, by the
        stream-time jumps of the chunk from its seed) are gathered from every rank, and the owner
        gets them with the global stream time before / after the batch (khip_agg_supplied_close).
        Collective: every rank calls it once per batch."""
        seed, before, after = self._ctx
        mine = agg.lost_windows(_RekeyedView(batch, self.shuffle.desc.key_col), seed)
        every = self.comm.allgather_ranges(mine) if self.world > 1 else mine
        agg.supplied_close(before, after, every)

    def exchange(self, batch, scan=None):
        """Device batch (source partition) → (this task's received rows [n, row_words], n).
        The rows are only valid until the next exchange: at one task they ARE the send buffer,
        which the next call reuses (copy them to keep them).  global_time needs `scan`."""
        import torch
        if self.global_time:
            if scan is None:
                raise ValueError("global_time: exchange needs a scan handle (an AggHandle)")
            batch = _StreamTimeBatch(batch, self.stream_times(scan, batch))
        n = max(int(batch.struct.n_rows), 1)
        if self.world == 1:
            # a send buffer for every row the batch holds, kept across calls: one pack launch
            # sequence per call (no count-only pass to size the buffer)
            if self._send is None or self._send.shape[0] < n:
                self._send = torch.empty((n, self.shuffle.row_words), dtype=torch.int64,
                                         device=torch.device("cuda", self.shuffle.device))
            send, counts = self.shuffle.pack(batch, send=self._send)
            recv, rcounts = send, counts
        else:
            self._send, counts, offs = self.shuffle.pack_v(batch, send=self._send)
            recv, rcounts = self.comm.alltoall(self._send, counts, self.shuffle.row_words, send_offsets=offs)
        self.last_counts = (counts, rcounts)
        return recv, int(sum(rcounts))

    def push_into(self, agg, batch):
        """The GROUP BY's aggregation reads this task's received rows where they lie
        (khip_agg_push_shuffled); returns its batch statistics.  global_time: `agg` is the
        KHIP_TIME_SUPPLIED owner task and also scans this rank's chunk."""
        recv, n = self.exchange(batch, scan=agg if self.global_time else None)
        if self.global_time and agg.desc.emit == abi.EMIT["FINAL"]:
            self.final_context(agg, batch)
        return agg.push_shuffled(self.shuffle, recv, n)

    def __call__(self, batch, scan=None):
        """Device batch (source partition) → (DeviceBatch of this task's rows, tensors)."""
        recv, n = self.exchange(batch, scan=scan)
        key, ts, cols, valid = self.shuffle.unpack(recv, n)
        st = self.shuffle.unpack_stream_time(recv, n) if self.global_time else None
        return abi.DeviceBatch(ts, keys=key, cols=cols, col_valid=valid, stream_time=st)

    def close(self):
        self.shuffle.close()
