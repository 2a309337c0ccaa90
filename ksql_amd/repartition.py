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
records from source rank 0 first, then rank 1, ..., each source's records in arrival order.
"""
from . import abi


class Repartition:
    def __init__(self, lib, key_col, col_types, rank=0, world=1, comm=None, device=0):
        if world > 1 and comm is None:
            raise ValueError("world > 1 needs an RCCL communicator (abi.Comm)")
        self.world = world
        self.rank = rank
        self.comm = comm
        self.shuffle = abi.ShuffleHandle(lib, world, key_col, col_types, device)
        self.last_counts = None

    def __call__(self, batch):
        """Device batch (source partition) → (DeviceBatch of this task's rows, tensors)."""
        send, counts = self.shuffle.pack(batch)
        if self.world == 1:
            recv, rcounts = send, counts
        else:
            recv, rcounts = self.comm.alltoall(send, counts, self.shuffle.row_words)
        self.last_counts = (counts, rcounts)
        n = int(sum(rcounts))
        key, ts, cols, valid = self.shuffle.unpack(recv, n)
        out = abi.DeviceBatch(ts, keys=key, cols=cols, col_valid=valid)
        out._keep.append(recv)
        return out

    def close(self):
        self.shuffle.close()
