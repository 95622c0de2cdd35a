"""Opt-in placement of client-delta memory (include/fjalloc.h, DESIGN.md §3 "Caller-side
placement").

The pytree fold reads every client's leaves from every CU. Deltas that torch's caching
allocator spread over separately hipMalloc'd segments cost the fold compulsory address
translation (configs[1]: 94.6 us per k_ptrs launch against 87.6 us when the same bytes share
one allocation). ``delta_pool()`` is a ``torch.cuda.MemPool`` whose segments come from
libfjagg's allocator — slices of 1 GiB hipMalloc chunks, each segment staggered by a
multiple of 68 KiB so row starts do not alias modulo 2 MiB — so tensors allocated under it
share a few large mappings (configs[1]: 88.96 us, 0 translation misses)
while every (client, leaf) stays its own tensor::

    pool = fedjax_amd.memory.delta_pool()
    with torch.cuda.use_mem_pool(pool):
        deltas = [train_client(...) for ...]      # or copies of them
    fedjax_amd.tree_util.tree_mean(list(zip(deltas, weights)))

Nothing else changes: results are the same bits (the fold does not depend on placement).
The reference has no counterpart (its deltas are XLA buffers)."""

from __future__ import annotations

import contextlib
from typing import Dict, Optional

import numpy as np
import torch

from fedjax_amd import _lib

_POOLS: Dict[int, "torch.cuda.MemPool"] = {}
_ALLOCATOR = None


def _allocator():
    global _ALLOCATOR
    if _ALLOCATOR is None:
        _lib.load()  # the same libfjagg.so, already bound to torch's HIP runtime
        _ALLOCATOR = torch.cuda.memory.CUDAPluggableAllocator(_lib.LIB_PATH, "fjalloc_alloc", "fjalloc_free")
    return _ALLOCATOR


def delta_pool(device: Optional[torch.device] = None) -> "torch.cuda.MemPool":
    """The process's fjalloc-backed memory pool for ``device`` (default: the current one),
    created on first use. Allocate client deltas under ``torch.cuda.use_mem_pool(pool)``."""
    idx = torch.device(device).index if device is not None else None
    idx = torch.cuda.current_device() if idx is None else idx
    pool = _POOLS.get(idx)
    if pool is None:
        with torch.cuda.device(idx):
            pool = _POOLS[idx] = torch.cuda.MemPool(_allocator().allocator())
    return pool


@contextlib.contextmanager
def delta_allocation(device: Optional[torch.device] = None):
    """``with delta_allocation(): ...`` — torch allocations on ``device`` inside the block
    come from :func:`delta_pool`."""
    pool = delta_pool(device)
    with torch.cuda.use_mem_pool(pool):
        yield pool


# set_default: the process-wide switch for the deltas fedjax_amd itself produces
_DEFAULT = {"on": False}


def set_default(enabled: bool = True) -> None:
    """Process-wide switch: while on, the client deltas fedjax_amd itself
    produces are allocated from :func:`delta_pool` — device copies of host deltas
    (:func:`to_device`), client-delta slabs (:class:`~fedjax_amd.slab.ClientDeltaSlab`, the rows
    :class:`~fedjax_amd.ingest.DeltaIngestor` fills) and the materialised results of
    ``tree_weight`` — so callers get the pooled placement without changing their code.
    Results are the same bits either way; off by default (the pool keeps 1 GiB chunks)."""
    _DEFAULT["on"] = bool(enabled)


def default_enabled() -> bool:
    return _DEFAULT["on"]


def producing(device) -> "contextlib.AbstractContextManager":
    """The scope fedjax_amd allocates the client deltas it produces on ``device`` in:
    :func:`delta_allocation` under :func:`set_default`, else a no-op."""
    dev = torch.device(device) if device is not None else None
    if not _DEFAULT["on"] or dev is None or dev.type != "cuda":
        return contextlib.nullcontext()
    return delta_allocation(dev)


def to_device(tree, device: Optional[torch.device] = None):
    """A client's delta pytree (torch tensors or numpy arrays, any container this package
    flattens) copied to ``device`` leaf by leaf — each leaf its own tensor, as a client's
    training output is — from :func:`delta_pool` under :func:`set_default`. The copies are
    asynchronous on the current stream (pinned sources) like ``Tensor.to``."""
    from fedjax_amd import pytree

    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    leaves, td = pytree.flatten(tree)
    with producing(dev):
        out = [(torch.from_numpy(np.ascontiguousarray(x)) if isinstance(x, np.ndarray) else x).to(dev)
               for x in leaves]
    return pytree.unflatten(td, out)


def release(device: Optional[torch.device] = None) -> None:
    """Drop the process's delta pool for ``device``: once no tensor allocated from it is
    alive, torch frees its segments and fjalloc returns the emptied chunks to the runtime
    (a later :func:`delta_pool` starts a new pool). Call it outside ``delta_allocation``.
    It also empties torch's own cache (``torch.cuda.empty_cache``), which is what hands a
    released pool's segments back."""
    idx = torch.device(device).index if device is not None else None
    idx = torch.cuda.current_device() if idx is None else idx
    pool = _POOLS.pop(idx, None)
    if pool is not None:
        del pool
        torch.cuda.synchronize(idx)
        torch.cuda.empty_cache()


def stats(device: Optional[torch.device] = None) -> dict:
    """fjalloc's counters for ``device`` (include/fjalloc.h ``fjalloc_stats``): bytes in live
    segments, live segments, segments created, reused ranges, failed requests, granularity,
    first chunk's top and base address (``bump_offset``, ``base``), last failure, placement
    hints, chunks and the free bytes inside them."""
    idx = torch.device(device).index if device is not None else None
    idx = torch.cuda.current_device() if idx is None else idx
    out = np.zeros(13, dtype=np.int64)
    if _lib.load().fjalloc_stats(idx, out.ctypes.data) != 0:
        raise ValueError(f"fjalloc_stats: bad device {idx}")
    keys = ("mapped_bytes", "live_segments", "segments", "reused_ranges", "failures", "granularity",
            "bump_offset", "base", "last_failure", "at_hint", "off_hint", "chunks", "free_bytes")
    return dict(zip(keys, (int(v) for v in out)))


__all__ = ["delta_pool", "delta_allocation", "release", "stats", "set_default", "default_enabled", "producing",
           "to_device"]
