"""Host side of the repartition step for a non-key GROUP BY / PARTITION BY.

Mirrors what StreamGroupByBuilderBase.build does per task
(ksqldb-streams/.../StreamGroupByBuilderBase.java:101-103: filter(v != null).groupBy(mapper)
→ sink "<ctx>-repartition" → source, i.e. the shuffle of SURVEY.md §8(e)) with the device
pieces of libksqldb_hip.so:

    khip_shuffle_pack      re-key by the group-by column, route with Kafka's default
                           partitioner (murmur2 of the KAFKA-format key), stable per source
    khip_comm_*            RCCL count exchange + grouped send/recv all-to-all over xGMI
                           (skipped at one task: the destination is this task)
    khip_shuffle_unpack    back to a columnar device batch keyed by the new key

The result feeds khip_agg_push exactly like a batch read back from the repartition topic:
records from source rank 0 first, then rank 1, ..., each source's records in arrival order — or
goes straight into the aggregation with khip_agg_push_shuffled (Repartition.push_into: the rows
are read where they lie, no columnar copy).

The exchange is pluggable: `abi.Comm` (RCCL over xGMI, one process per GPU, the production
path) or `GlooExchange` (any torch.distributed process group, rows staged through host memory:
the CPU tests, and several ranks sharing one GPU, where RCCL refuses duplicate devices).
"""
from . import abi


class GlooExchange:
    """The same two collective steps as abi.Comm.alltoall (counts, then rows laid out by source
    rank) over a torch.distributed group, through host memory."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.nranks = dist.get_world_size(group)

    def alltoall(self, send, send_counts, row_words):
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
        hsend = (send[:n_send].to("cpu") if send is not None and n_send
                 else torch.empty((0, row_words), dtype=torch.int64)).contiguous()
        hrecv = torch.empty((sum(rcounts), row_words), dtype=torch.int64)
        dist.all_to_all_single(hrecv.view(-1), hsend.view(-1), [c * row_words for c in rcounts],
                               [int(c) * row_words for c in send_counts], group=self.group)
        if hrecv.shape[0] == 0:
            hrecv = torch.zeros((1, row_words), dtype=torch.int64)
        return hrecv.to(dev), rcounts


class Repartition:
    def __init__(self, lib, key_col, col_types, rank=0, world=1, comm=None, device=0):
        if world > 1 and comm is None:
            raise ValueError("world > 1 needs an exchange (abi.Comm over RCCL, or GlooExchange)")
        self.world = world
        self.rank = rank
        self.comm = comm
        self.shuffle = abi.ShuffleHandle(lib, world, key_col, col_types, device)
        self.last_counts = None
        self._send = None

    def exchange(self, batch):
        """Device batch (source partition) → (this task's received rows [n, row_words], n)."""
        import torch
        n = max(int(batch.struct.n_rows), 1)
        # a send buffer for every row the batch holds, kept across calls: one pack launch
        # sequence per call (no count-only pass to size the buffer)
        if self._send is None or self._send.shape[0] < n:
            self._send = torch.empty((n, self.shuffle.row_words), dtype=torch.int64,
                                     device=torch.device("cuda", self.shuffle.device))
        send, counts = self.shuffle.pack(batch, send=self._send)
        if self.world == 1:
            recv, rcounts = send, counts
        else:
            recv, rcounts = self.comm.alltoall(send, counts, self.shuffle.row_words)
        self.last_counts = (counts, rcounts)
        return recv, int(sum(rcounts))

    def push_into(self, agg, batch):
        """The GROUP BY's aggregation reads this task's received rows where they lie
        (khip_agg_push_shuffled); returns its batch statistics."""
        recv, n = self.exchange(batch)
        return agg.push_shuffled(self.shuffle, recv, n)

    def __call__(self, batch):
        """Device batch (source partition) → (DeviceBatch of this task's rows, tensors)."""
        recv, n = self.exchange(batch)
        key, ts, cols, valid = self.shuffle.unpack(recv, n)
        out = abi.DeviceBatch(ts, keys=key, cols=cols, col_valid=valid)
        out._keep.append(recv)
        return out

    def close(self):
        self.shuffle.close()
