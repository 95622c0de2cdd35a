"""Client-sharded aggregation over the GPUs of one node.

The reference has no device-side reduction: its only multi-device mechanism,
``ForEachClientPmapBackend`` (fedjax/core/for_each_client.py:266-357), spreads
client *training* over ``jax.local_devices()`` and copies every client output
back to ``devices[0]`` (:351-353), where ``tree_mean`` runs on one device.

Here every rank (one process per GPU, ``torch.distributed`` over RCCL/xGMI)
owns a contiguous range of clients, folds them with the HIP kernel into a
float32 partial that is already multiplied by f32(1/W), and the partials are
summed by ``reduce`` (or ``all_reduce``) over xGMI — the only exchange step.
The parameter axis is cut into buckets so the reduce of bucket b overlaps the
fold of bucket b+1 (the collective runs on RCCL's own stream).

Two exchange engines share that contract:

* :class:`RcclCommunicator` + :func:`sharded_weighted_mean` with ``comm=`` — the
  native pipeline of ``include/fjcomm.h``: ONE library call folds the buckets on the
  caller's stream and reduces each on the communicator's high-priority stream, with
  device-scope events between them (no per-bucket system-scope cache write-back, no
  per-bucket Python);
* ``torch.distributed`` collectives (``comm=None``) — any backend (gloo on CPU tests).

Numerics: the result differs from the single-GPU exact fold only by the G-way
combine and the per-rank scaling; tests/test_distributed.py and the GPU tests
check it against the per-element bound in DESIGN.md §4.
"""

from __future__ import annotations

import ctypes
from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist

from fedjax_amd import _lib, kernels, pytree, tree_util

# bucket edges are multiples of this many elements (keeps 16-byte alignment)
BUCKET_ALIGN = 1024


def shard_range(num_clients: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous client range [k0, k1) of ``rank`` (sizes differ by at most 1)."""
    base, extra = divmod(num_clients, world_size)
    k0 = rank * base + min(rank, extra)
    return k0, k0 + base + (1 if rank < extra else 0)


def bucket_edges(P: int, buckets: Union[int, Sequence[float]]) -> List[Tuple[int, int]]:
    """Parameter buckets [p0, p1) covering [0, P); every p0 a multiple of BUCKET_ALIGN.

    ``buckets`` is a count (equal buckets) or a sequence of relative sizes, e.g.
    ``(4, 2, 1)``: a tapered schedule. Each reduce then overlaps the next, smaller
    fold, and only the small last bucket's reduce is left exposed at the end of the
    step. Interior edges are rounded to BUCKET_ALIGN; buckets that round away vanish.
    """
    if isinstance(buckets, (int, np.integer)):
        buckets = max(1, int(buckets))
        step = -(-P // buckets)
        step = max(BUCKET_ALIGN, -(-step // BUCKET_ALIGN) * BUCKET_ALIGN)
        return [(p0, min(P, p0 + step)) for p0 in range(0, P, step)]
    sizes = [float(s) for s in buckets]
    if not sizes or any(not s > 0 for s in sizes):
        raise ValueError(f"bucket sizes must be positive, got {tuple(buckets)}")
    if P <= 0:
        return []
    total, acc, edges = sum(sizes), 0.0, [0]
    for s in sizes[:-1]:
        acc += s
        e = int(round(P * acc / total / BUCKET_ALIGN)) * BUCKET_ALIGN
        if edges[-1] < e < P:
            edges.append(e)
    edges.append(P)
    return list(zip(edges[:-1], edges[1:]))


def bucket_name(buckets) -> str:
    """``4`` -> "4", ``(4, 2, 1)`` -> "4:2:1" (bench labels)."""
    if isinstance(buckets, (int, np.integer)):
        return str(int(buckets))
    return ":".join(f"{s:g}" for s in buckets)


def total_weight(local_weights: Sequence, group=None, device=None):
    """W over all ranks' clients when no rank knows every weight: the local sums
    (reference accumulation, Python float) are summed in float64 across ranks."""
    W = 0.0
    for w in local_weights:
        W += tree_util._host_weight(w)
    t = torch.tensor([float(W)], dtype=torch.float64, device=device)
    dist.all_reduce(t, group=group)
    return float(t.item())


def _default_partial(x: torch.Tensor, w: torch.Tensor, scale: float, out: torch.Tensor) -> None:
    nbytes = x.numel() * x.element_size()
    kernels.weighted_sum_dense(x, w, scale=scale, out=out,
                               nontemporal=nbytes >= tree_util.NONTEMPORAL_MIN_BYTES)


class RcclCommunicator:
    """An RCCL communicator over the ranks of ``group`` (one process per GPU), made by
    ``fjcomm_init`` on the current device; rank 0's ``ncclUniqueId`` is broadcast over
    ``group`` (a torch.distributed group of any backend). Collective: every rank of the
    group constructs it. ``close()`` (or garbage collection) destroys it."""

    def __init__(self, group=None, device: Optional[torch.device] = None):
        lib = _lib.load()
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        dev = device or torch.device("cuda", torch.cuda.current_device())
        uid = torch.zeros(_lib.COMM_ID_BYTES, dtype=torch.uint8)
        if self.rank == 0:
            buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
            _lib.check(lib.fjcomm_unique_id(buf), "fjcomm_unique_id")
            uid.copy_(torch.frombuffer(bytearray(buf), dtype=torch.uint8))
        backend = dist.get_backend(group)
        t = uid.to(dev) if backend == "nccl" else uid
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        ids = (ctypes.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(t.cpu().numpy().tobytes())
        handle = ctypes.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(lib.fjcomm_init(ctypes.byref(handle), ids, self.world_size, self.rank), "fjcomm_init")
        self.handle = handle
        self.device = dev

    def abort(self) -> None:
        """``fjcomm_abort``: end this communicator's outstanding collectives without waiting for
        the other ranks (after a collective missed its deadline). The communicator refuses every
        later step; every rank must stop using it (agree over another group first)."""
        if getattr(self, "handle", None) is not None and self.handle.value:
            _lib.check(_lib.load().fjcomm_abort(self.handle), "fjcomm_abort")
            self.aborted = True

    def close(self) -> None:
        if getattr(self, "handle", None) is not None and self.handle.value:
            _lib.load().fjcomm_destroy(self.handle)
            self.handle = None

    __del__ = close


def _native_sharded(comm: RcclCommunicator, x_local: torch.Tensor, w_local: torch.Tensor, scale: float,
                    out: torch.Tensor, root: int, buckets, nontemporal: Optional[bool],
                    fold_events=None) -> None:
    K, P = x_local.shape
    if x_local.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError("the native sharded fold takes float32 or bfloat16 deltas")
    if K and x_local.stride(1) != 1:
        raise ValueError("client rows need unit column stride")
    if out.dtype != torch.float32 or out.numel() != P or not out.is_contiguous():
        raise ValueError("out must be a contiguous float32 [P] tensor")
    if isinstance(w_local, np.ndarray):
        w_local = torch.from_numpy(w_local)
    if w_local.dtype != torch.float32 or w_local.numel() != K:
        raise ValueError("w_local must be float32 [K_g]")
    nbytes = K * P * x_local.element_size()
    nt = (nbytes >= tree_util.NONTEMPORAL_MIN_BYTES) if nontemporal is None else nontemporal
    spans = bucket_edges(P, buckets)
    if not spans:
        return
    if len(spans) > _lib.COMM_MAX_BUCKETS:
        raise ValueError(f"at most {_lib.COMM_MAX_BUCKETS} buckets")
    edges = np.array([p0 for p0, _ in spans] + [P], dtype=np.int64)
    ev = None
    if fold_events is not None:
        if len(fold_events) < 2 * len(spans):
            raise ValueError(f"fold_events needs 2 events per bucket ({2 * len(spans)})")
        ev = (ctypes.c_void_p * len(fold_events))(*[e.handle for e in fold_events])
    flags = _lib.NONTEMPORAL if nt else 0
    stream = torch.cuda.current_stream(out.device).cuda_stream
    if not w_local.is_cuda:  # host weights: in the bucket folds' kernel arguments when those launches allow it
        w_local = w_local.contiguous()
        rc = _lib.load().fjcomm_sharded_wsum_dense_edges(
            comm.handle, kernels.dtype_code(x_local.dtype), x_local.data_ptr() if K else None,
            x_local.stride(0) if K else P, K, P, w_local.data_ptr() if K else None, float(np.float32(scale)),
            out.data_ptr(), edges.ctypes.data, len(spans), int(root), flags | _lib.HOST_TABLES, stream, ev)
        if rc != kernels._EUNSUPPORTED:
            _lib.check(rc, "fjcomm_sharded_wsum_dense_edges")
            kernels.HOST_WEIGHT_PATHS["kernel_args"] += 1
            return
        w_local = _lib.upload(w_local, out.device)
        kernels.HOST_WEIGHT_PATHS["uploaded"] += 1
    _lib.call("fjcomm_sharded_wsum_dense_edges", comm.handle, kernels.dtype_code(x_local.dtype),
              x_local.data_ptr() if K else None, x_local.stride(0) if K else P, K, P,
              w_local.data_ptr() if K else None, float(np.float32(scale)), out.data_ptr(), edges.ctypes.data,
              len(spans), int(root), flags, stream, ev)


def sharded_weighted_mean(x_local: torch.Tensor, w_local: torch.Tensor, W_total, *, group=None,
                          dst: int = 0, all_ranks: bool = False,
                          buckets: Union[int, Sequence[float]] = 4,
                          out: Optional[torch.Tensor] = None,
                          partial_fn: Optional[Callable] = None,
                          comm: Optional[RcclCommunicator] = None,
                          nontemporal: Optional[bool] = None,
                          fold_events=None) -> torch.Tensor:
    """Weighted mean over all ranks' client rows.

    x_local: this rank's client deltas [K_g, P] (unit column stride, may be K_g = 0
    only if partial_fn handles it); w_local: their float32 weights [K_g], on the same
    device or on the host (a numpy array / CPU tensor: then carried in the folds' kernel
    arguments, FJAGG_HOST_TABLES, when the launches allow it — no upload in front of the
    step); W_total: sum of ALL clients' weights (reference semantics, host scalar).
    Returns the float32 mean [P] — valid on ``dst`` (every rank with ``all_ranks``).
    partial_fn(x, w, scale, out) computes ``out = fl(sum_k x_k w_k) * scale`` for one
    bucket; the default is the HIP kernel (tests inject the oracle to run on gloo).
    buckets: a count of equal buckets or relative sizes (:func:`bucket_edges`).
    comm: an :class:`RcclCommunicator` selects the native pipeline (``fjcomm.h``);
    fold_events then takes two :class:`fedjax_amd.kernels.Event` per bucket that
    bracket each bucket's fold on the current stream.
    """
    P = x_local.shape[1]
    scale = float(np.float32(tree_util._inverse(W_total)))
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=x_local.device)
    if comm is not None:
        if partial_fn is not None:
            raise ValueError("partial_fn and comm are exclusive (the native pipeline folds in the library)")
        root = -1 if all_ranks else (dist.get_group_rank(group, dst) if group is not None else dst)
        _native_sharded(comm, x_local, w_local, scale, out, root, buckets, nontemporal, fold_events)
        return out
    fn = partial_fn or _default_partial
    works = []
    for p0, p1 in bucket_edges(P, buckets):
        seg = out[p0:p1]
        fn(x_local[:, p0:p1], w_local, scale, seg)
        if all_ranks:
            works.append(dist.all_reduce(seg, op=dist.ReduceOp.SUM, group=group, async_op=True))
        else:
            works.append(dist.reduce(seg, dst=dst, op=dist.ReduceOp.SUM, group=group, async_op=True))
    for wk in works:
        wk.wait()
    return out


def sharded_tree_mean(local_pytrees_and_weights, *, W_total=None, group=None, dst: int = 0,
                      all_ranks: bool = False, template=None):
    """``tree_mean`` over the union of every rank's clients.

    Each rank folds its own (pytree, weight) pairs in one pytree-kernel launch
    (already scaled by f32(1/W)); the float32 partial leaves are packed into one
    buffer and summed across ranks. Returns the mean pytree (float32 leaves) on the
    global rank ``dst`` (on every rank with ``all_ranks``), ``None`` elsewhere.

    A rank may hold no clients (``shard_range`` gives some ranks none when K < world
    size): it contributes a zero partial, so every rank reaches the same collectives.
    One small all_gather of (local W, partial size) runs first; it gives every rank
    W (when ``W_total`` is None) and lets all ranks agree on the partial's size — or
    raise together when the ranks' trees disagree, or when one rank's own clients fail
    validation (that rank raises its own error, the others a ValueError naming it: no rank is left waiting in a collective). A rank that must return the mean
    but has no clients needs ``template`` (any pytree with the clients' structure and
    leaf shapes, e.g. the server params) for the structure of the result. Returns
    ``None`` on every rank when no rank has a client.
    """
    pairs = list(local_pytrees_and_weights)
    trees = [t for t, _ in pairs]
    nccl = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
    td, views, sizes, weights, W_local = None, None, None, [], 0.0
    # Local validation runs BEFORE the header exchange, but a failure does not raise here
    # alone (the other ranks would block in the all_gather): it is flagged in the header,
    # and every rank raises after the exchange.
    local_error = None
    try:
        weights = [tree_util._host_weight(w) for _, w in pairs]
        for w in weights:
            W_local += w  # tree_util.py:95 on this rank's share
        if trees:
            td, rows = tree_util._client_table(trees)
            row0 = rows[0]
            if any(x.dtype != torch.float32 for x in row0):
                raise TypeError("sharded_tree_mean needs float32 leaves")
            sizes = [x.numel() for x in row0]
            shapes = [x.shape for x in row0]
            dev = row0[0].device if row0 else dev
        elif template is not None:
            leaves, td = pytree.flatten(template)
            shapes = [tuple(tree_util._to_tensor(x).shape) for x in leaves]
            sizes = [int(np.prod(s, dtype=np.int64)) for s in shapes]
    except Exception as e:  # noqa: BLE001 - re-raised below, after the other ranks are told
        local_error, sizes, W_local = e, None, 0.0
    P = sum(sizes) if sizes is not None else -1
    hdr = torch.tensor([float(W_local), float(P), float(len(trees)), 1.0 if local_error else 0.0],
                       dtype=torch.float64, device=dev if nccl else None)
    world = dist.get_world_size(group)
    got = [torch.empty_like(hdr) for _ in range(world)]
    dist.all_gather(got, hdr, group=group)
    got = [t.cpu().numpy() for t in got]
    failed = [r for r, g in enumerate(got) if g[3] != 0]
    if local_error is not None:
        raise local_error
    if failed:
        raise ValueError(f"sharded_tree_mean: rank(s) {failed} rejected their local clients (see their error)")
    if W_total is None:
        W_total = 0.0
        for g in got:
            W_total += float(g[0])  # rank order: the same W on every rank
    if sum(int(g[2]) for g in got) == 0:
        return None  # no rank has a client (tree_util.py:96)
    Ps = {int(g[1]) for g in got} - {-1}
    if len(Ps) != 1:  # every rank sees the same header, so all of them raise here together
        raise ValueError(f"ranks disagree on the number of parameters: {sorted(Ps)}")
    flat = torch.zeros(Ps.pop(), dtype=torch.float32, device=dev)
    if trees:
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        views = [flat[o:o + n].view(sh) for o, n, sh in zip(offs[:-1], sizes, shapes)]
        tree_util._fold(rows, weights, scale=tree_util._inverse(W_total), out=views, accumulate=False,
                        validated=True)
    elif td is not None:
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        views = [flat[o:o + n].view(sh) for o, n, sh in zip(offs[:-1], sizes, shapes)]
    if all_ranks:
        dist.all_reduce(flat, group=group)
    else:
        dist.reduce(flat, dst=dst, group=group)  # dst is a global rank (torch.distributed)
    if all_ranks or dist.get_rank() == dst:
        if views is None:
            raise ValueError("this rank holds no clients and must return the mean: pass template= "
                             "(a pytree with the clients' structure) to shape the result")
        return pytree.unflatten(td, views)
    return None


# ------------------------------------------------------------- one process, several GPUs
class MultiDeviceCommunicator:
    """RCCL communicators over several GPUs of ONE process (``fjcomm_init_all`` =
    ``ncclCommInitAll``): the shape of FedJAX's server, one Python process over
    ``jax.local_devices()`` (fedjax/core/for_each_client.py:266-357). No launcher and no
    torch.distributed process group are involved. ``close()`` destroys the handles."""

    def __init__(self, devices: Sequence):
        lib = _lib.load()
        self.devices = [torch.device(d) if not isinstance(d, torch.device) else d for d in devices]
        idx = []
        for d in self.devices:
            if d.type != "cuda":
                raise ValueError(f"{d} is not a GPU")
            idx.append(d.index if d.index is not None else torch.cuda.current_device())
        n = len(idx)
        if not 1 <= n <= _lib.COMM_MAX_DEVICES:
            raise ValueError(f"need 1..{_lib.COMM_MAX_DEVICES} devices, got {n}")
        if len(set(idx)) != n:
            raise ValueError(f"devices must be distinct, got {idx}")
        self.indices = idx
        handles = (ctypes.c_void_p * n)()
        _lib.check(lib.fjcomm_init_all(handles, n, (ctypes.c_int * n)(*idx)), "fjcomm_init_all")
        self.handles = handles

    def __len__(self):
        return len(self.indices)

    def close(self) -> None:
        hs = getattr(self, "handles", None)
        if hs is not None:
            lib = _lib.load()
            for h in hs:
                if h:
                    lib.fjcomm_destroy(ctypes.c_void_p(h))
            self.handles = None

    __del__ = close


def multi_device_weighted_mean(xs: Sequence[torch.Tensor], ws: Sequence[torch.Tensor], W_total, *,
                               comm: MultiDeviceCommunicator, root: int = 0, all_devices: bool = False,
                               buckets: Union[int, Sequence[float]] = 1,
                               outs: Optional[Sequence[torch.Tensor]] = None,
                               nontemporal: Optional[bool] = None) -> List[torch.Tensor]:
    """Weighted mean over clients spread across the GPUs of this process.

    xs[d]: the client slab [K_d, P] (unit column stride, float32 or bfloat16) on
    ``comm.devices[d]``; ws[d]: its float32 weights [K_d] there, or every ws[d] on the
    host (carried in the folds' kernel arguments when they allow it); W_total: the sum of ALL
    clients' weights (tree_util.py:86,95, host value). Each device folds its clients into
    a float32 partial already scaled by f32(1/W); the partials are summed by one grouped
    RCCL reduce per bucket (all-reduce with ``all_devices``). Returns the per-device
    float32 [P] buffers: the mean is in ``outs[root]`` (in every one with
    ``all_devices``). Asynchronous on each device's current stream. Numerics as
    :func:`sharded_weighted_mean`; with one device, bitwise the exact fold.
    """
    n = len(comm)
    if len(xs) != n or len(ws) != n:
        raise ValueError(f"need one slab and one weight vector per device ({n})")
    ws = [torch.from_numpy(w) if isinstance(w, np.ndarray) else w for w in ws]
    host_w = all(not w.is_cuda for w in ws)  # host weights: kernel arguments of the folds (FJAGG_HOST_TABLES)
    P = xs[0].shape[1]
    dt = xs[0].dtype
    for d, (x, w, dev) in enumerate(zip(xs, ws, comm.devices)):
        if x.dim() != 2 or x.shape[1] != P or x.dtype != dt or dt not in (torch.float32, torch.bfloat16):
            raise ValueError(f"device {d}: slabs must be [K_d, {P}] of one float dtype")
        if x.shape[0] and x.stride(1) != 1:
            raise ValueError(f"device {d}: client rows need unit column stride")
        if x.device != dev or (w.device != dev and not host_w):
            raise ValueError(f"device {d}: slab and weights must be on {dev} (or every weight vector on the host)")
        if w.dtype != torch.float32 or w.numel() != x.shape[0]:
            raise ValueError(f"device {d}: weights must be float32 [K_d]")
    if outs is None:
        outs = [torch.empty(P, dtype=torch.float32, device=dev) for dev in comm.devices]
    for d, (o, dev) in enumerate(zip(outs, comm.devices)):
        if o.dtype != torch.float32 or o.numel() != P or not o.is_contiguous() or o.device != dev:
            raise ValueError(f"device {d}: out must be a contiguous float32 [P] tensor on {dev}")
    spans = bucket_edges(P, buckets)
    if not spans:
        return list(outs)
    if len(spans) > _lib.COMM_MAX_BUCKETS:
        raise ValueError(f"at most {_lib.COMM_MAX_BUCKETS} buckets")
    edges = np.array([p0 for p0, _ in spans] + [P], dtype=np.int64)
    nbytes = max(x.shape[0] for x in xs) * P * xs[0].element_size()
    nt = (nbytes >= tree_util.NONTEMPORAL_MIN_BYTES) if nontemporal is None else nontemporal
    scale = float(np.float32(tree_util._inverse(W_total)))
    vp = ctypes.c_void_p * n
    i64 = ctypes.c_int64 * n
    flags = _lib.NONTEMPORAL if nt else 0

    def issue(wv, fl):
        return _lib.load().fjcomm_multi_wsum_dense(
            comm.handles, n, kernels.dtype_code(dt), vp(*[x.data_ptr() if x.shape[0] else None for x in xs]),
            i64(*[x.stride(0) if x.shape[0] > 1 else P for x in xs]), i64(*[x.shape[0] for x in xs]), P,
            vp(*[w.data_ptr() if w.numel() else None for w in wv]), scale, vp(*[o.data_ptr() for o in outs]),
            edges.ctypes.data, len(spans), -1 if all_devices else int(root), fl,
            vp(*[torch.cuda.current_stream(dev).cuda_stream for dev in comm.devices]))

    if host_w:
        ws = [w.contiguous() for w in ws]
        rc = issue(ws, flags | _lib.HOST_TABLES)
        if rc != kernels._EUNSUPPORTED:
            _lib.check(rc, "fjcomm_multi_wsum_dense")
            kernels.HOST_WEIGHT_PATHS["kernel_args"] += 1
            return list(outs)
        ws = [_lib.upload(w, dev) for w, dev in zip(ws, comm.devices)]
        kernels.HOST_WEIGHT_PATHS["uploaded"] += 1
    _lib.check(issue(ws, flags), "fjcomm_multi_wsum_dense")
    return list(outs)
