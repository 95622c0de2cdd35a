"""Process-group rendezvous for the multi-process tests without a free-port race.

The tests used to bind port 0, close the socket and hand the number to their workers as
MASTER_PORT; between the close and the workers' bind another process could take the port
(the cause of round 4's intermittent spawn failure, bench.spawn_ranks). Here the parent
binds a TCPStore on port 0 and KEEPS it (``HeldStore``) until its workers are done; the
workers join it as clients (``init_group``), so the port is never free in between."""
import datetime

import torch.distributed as dist


class HeldStore:
    """A TCPStore server on 127.0.0.1, port chosen by the OS and held while this object lives."""

    def __init__(self, world_size: int):
        self.store = dist.TCPStore("127.0.0.1", 0, world_size, True, timeout=datetime.timedelta(seconds=120),
                                   wait_for_workers=False)
        self.port = self.store.port


def init_group(backend: str, rank: int, world_size: int, port: int, **kw) -> None:
    """init_process_group over the parent's HeldStore at ``port`` (a client connection)."""
    store = dist.TCPStore("127.0.0.1", port, world_size, False, timeout=datetime.timedelta(seconds=120))
    dist.init_process_group(backend, store=store, rank=rank, world_size=world_size, **kw)


def init_world1(backend: str, **kw) -> None:
    """A one-rank group with its own store bound on port 0 (nothing to share)."""
    dist.init_process_group(backend, store=dist.TCPStore("127.0.0.1", 0, 1, True), rank=0, world_size=1, **kw)
