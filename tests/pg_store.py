"""Rendezvous for the multi-process tests: a FileStore in a fresh temporary directory instead of a
TCP port probed in the parent and bound later in a child (another process can take such a port in
between: EADDRINUSE on a busy box).  Gloo's own connections still use ports the OS assigns."""
import os
import tempfile


def store_url():
    """A file:// init_method for one process group (the file must not exist yet)."""
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="ksql_amd_pg_"), "store")


def init_gloo(url, rank, world):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=url, rank=rank, world_size=world)
