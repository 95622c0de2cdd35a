"""Client-sharded aggregation with the HIP kernel on the GPU, world_size 2.

Both ranks share the box's single GPU, so the exchange uses gloo (RCCL refuses
two ranks on one device); the RCCL path itself runs in bench.py --gpus N.
"""

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import tree_util_ref as ref
from tests.rendezvous import HeldStore, init_group, init_world1  # noqa: F401

pytestmark = pytest.mark.gpu
K, P = 48, 70001
P2 = (1 << 20) + 3  # host-weight runs: buckets too wide for the narrow kernel (which takes device weights)


def _worker(rank, world, port, q):
    init_group("gloo", rank, world, port)
    try:
        import fedjax_amd
        from fedjax_amd import distributed as fd, kernels
        dev = torch.device("cuda:0")
        weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
        W = 0.0
        for w in weights:
            W += w
        k0, k1 = fd.shard_range(K, rank, world)
        x = torch.empty(k1 - k0, P, dtype=torch.float32, device=dev)
        kernels.fill_synth(x, seed=9, k0=k0)
        wl = torch.tensor(np.float32(weights[k0:k1]), device=dev)
        y = fd.sharded_weighted_mean(x, wl, W, buckets=3, all_ranks=True)
        trees = [({"a": x[i, :1000], "b": x[i, 1000:]}, weights[k0 + i]) for i in range(k1 - k0)]
        m = fd.sharded_tree_mean(trees, all_ranks=True)
        # K < world size: rank 1 holds no client and contributes zeros (template shapes the result)
        tmpl = {"a": torch.zeros(1000), "b": torch.zeros(P - 1000)}
        m1 = fd.sharded_tree_mean(trees[:1] if rank == 0 else [], all_ranks=True, template=tmpl)
        # dst is a global rank: only rank 1 (which holds the clients this time) gets the mean
        m2 = fd.sharded_tree_mean(trees if rank == 1 else [], dst=1)
        torch.cuda.synchronize()
        flat = lambda t: None if t is None else torch.cat([t["a"], t["b"]]).cpu().numpy()  # noqa: E731
        q.put((rank, y.cpu().numpy(), flat(m), (flat(m1), flat(m2), k0, k1)))
    finally:
        dist.destroy_process_group()


def test_sharded_mean_world2_on_gpu(cuda, coracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = HeldStore(2)
    port = store.port
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (y, m, extra) for r, y, m, extra in (q.get(timeout=300) for _ in procs)}
    res = {r: v[:2] for r, v in got.items()}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
    x = coracle.synth_f32(K, P, seed=9)
    r = ref.mean_scale(weights)
    want = coracle.wsum_f32(x, np.float32(weights), scale=r)
    bound = coracle.bound_f32(x, np.float32(weights), r, want) * (K + 4) / (K + 2)
    for rank in (0, 1):
        for y in res[rank]:
            assert np.all(np.abs(y.astype(np.float64) - want) <= bound)
    # one rank's partial + the other rank's zeros: bitwise the single-rank exact fold
    want1 = coracle.wsum_f32(x[:1], np.float32(weights[:1]), scale=ref.mean_scale(weights[:1]))
    for rank in (0, 1):
        assert np.array_equal(got[rank][2][0].view(np.uint32), want1.astype(np.float32).view(np.uint32))
    k0, k1 = got[1][2][2:]
    want2 = coracle.wsum_f32(np.ascontiguousarray(x[k0:k1]), np.float32(weights[k0:k1]),
                             scale=ref.mean_scale(weights[k0:k1]))
    assert got[0][2][1] is None
    assert np.array_equal(got[1][2][1].view(np.uint32), want2.astype(np.float32).view(np.uint32))


def _native_worker(port, q):
    """World-1 RCCL communicator: the native fold+reduce pipeline of include/fjcomm.h."""
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    init_world1("nccl", device_id=dev)
    try:
        from fedjax_amd import distributed as fd, kernels
        weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
        W = 0.0
        for w in weights:
            W += w
        comm = fd.RcclCommunicator(device=dev)
        x = torch.empty(K, P + 3, dtype=torch.float32, device=dev)[:, :P]  # ld > P
        kernels.fill_synth(x, seed=9)
        wl = torch.tensor(np.float32(weights), device=dev)
        res = {}
        for buckets, all_ranks in ((1, False), (3, False), (7, True), ((3, 1), False), ((4, 2, 1), True)):
            nb = len(fd.bucket_edges(P, buckets))
            evs = [kernels.Event() for _ in range(2 * nb)]
            y = fd.sharded_weighted_mean(x, wl, W, buckets=buckets, all_ranks=all_ranks, comm=comm,
                                         fold_events=evs)
            torch.cuda.synchronize()
            ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(0, 2 * nb, 2)]
            res[(buckets, all_ranks)] = (y.cpu().numpy(), ms)
        # host weights (FJAGG_HOST_TABLES): the bucket folds carry them in their kernel arguments
        x2 = torch.empty(K, P2 + 1, dtype=torch.float32, device=dev)[:, :P2]
        kernels.fill_synth(x2, seed=11)
        before = dict(kernels.HOST_WEIGHT_PATHS)
        for buckets, all_ranks in ((1, False), ((4, 2, 1), True)):
            y = fd.sharded_weighted_mean(x2, np.float32(weights), W, buckets=buckets, all_ranks=all_ranks, comm=comm)
            torch.cuda.synchronize()
            res[("host", buckets, all_ranks)] = (y.cpu().numpy(), [1.0])
        # narrow buckets refuse kernel-argument weights: uploaded instead, same bits
        y = fd.sharded_weighted_mean(x, np.float32(weights), W, buckets=3, comm=comm)
        torch.cuda.synchronize()
        res[("host-narrow", 3, False)] = (y.cpu().numpy(), [1.0])
        res["host_paths"] = {k: v - before[k] for k, v in kernels.HOST_WEIGHT_PATHS.items()}
        del x2
        xb = torch.empty(K, P, dtype=torch.bfloat16, device=dev)
        kernels.fill_synth(xb, seed=9)
        yb = fd.sharded_weighted_mean(xb, wl, W, buckets=2, comm=comm)
        y0 = fd.sharded_weighted_mean(x[:0], wl[:0], W, buckets=2, comm=comm,
                                      out=torch.full((P,), 7.0, device=dev))
        # explicit edges are validated: unaligned, non-increasing, not ending at P
        import ctypes
        from fedjax_amd import _lib
        errs = []
        for edges in ([0, 1000, P], [0, 2048, 2048, P], [0, 1024, P - 1]):
            e = np.array(edges, dtype=np.int64)
            rc = _lib.load().fjcomm_sharded_wsum_dense_edges(
                comm.handle, _lib.F32, x.data_ptr(), x.stride(0), K, P, wl.data_ptr(), 1.0, y0.data_ptr(),
                e.ctypes.data, len(edges) - 1, 0, 0, torch.cuda.current_stream().cuda_stream, None)
            errs.append((rc, _lib.load().fjagg_last_error().decode()))
        torch.cuda.synchronize()
        q.put((res, yb.cpu().numpy(), y0.cpu().numpy(), errs))
        comm.close()
    finally:
        dist.destroy_process_group()


def test_native_rccl_pipeline_world1(cuda, coracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_native_worker, args=(None, q))
    p.start()
    res, yb, y0, errs = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
    x = coracle.synth_f32(K, P, seed=9)
    r = ref.mean_scale(weights)
    want = coracle.wsum_f32(x, np.float32(weights), scale=r)
    assert res.pop("host_paths") == {"kernel_args": 2, "uploaded": 1}
    want2 = coracle.wsum_f32(coracle.synth_f32(K, P2, seed=11), np.float32(weights), scale=r)
    for key in [k for k in res if k[0] == "host"]:
        y, _ = res.pop(key)
        assert np.array_equal(y.view(np.uint32), want2.astype(np.float32).view(np.uint32)), key
    for key, (y, ms) in res.items():
        # one rank: the partial is the exact fold (per-element, so bucketing is invisible)
        assert np.array_equal(y.view(np.uint32), want.astype(np.float32).view(np.uint32)), key
        assert all(m > 0 for m in ms), key
    assert np.all(y0 == 0)  # a rank without clients contributes zeros
    assert all(rc != 0 and msg for rc, msg in errs), errs  # bad bucket edges are refused before any launch
    xb = (coracle.synth_bf16(K, P, seed=9).astype(np.uint32) << 16).view(np.float32)  # bf16 -> f32 exactly
    want_b = coracle.wsum_f32(np.ascontiguousarray(xb), np.float32(weights), scale=r)
    assert np.array_equal(yb.view(np.uint32), want_b.astype(np.float32).view(np.uint32))


def _multi_device_worker(q):
    """One process over its GPUs (here the box's one GPU): fjcomm_init_all +
    fjcomm_multi_wsum_dense, no launcher, no process group."""
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from fedjax_amd import distributed as fd, kernels
    weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
    W = 0.0
    for w in weights:
        W += w
    comm = fd.MultiDeviceCommunicator([dev])
    x = torch.empty(K, P + 5, dtype=torch.float32, device=dev)[:, :P]
    kernels.fill_synth(x, seed=9)
    wl = torch.tensor(np.float32(weights), device=dev)
    res = {}
    for buckets, alld in ((1, False), (3, False), ((4, 2, 1), True)):
        outs = fd.multi_device_weighted_mean([x], [wl], W, comm=comm, buckets=buckets, all_devices=alld)
        torch.cuda.synchronize()
        res[(fd.bucket_name(buckets), alld)] = outs[0].cpu().numpy()
    x2 = torch.empty(K, P2 + 1, dtype=torch.float32, device=dev)[:, :P2]
    kernels.fill_synth(x2, seed=11)
    before = dict(kernels.HOST_WEIGHT_PATHS)
    for buckets in (1, (4, 2, 1)):  # host weights: kernel arguments of every device's folds
        outs = fd.multi_device_weighted_mean([x2], [np.float32(weights)], W, comm=comm, buckets=buckets)
        torch.cuda.synchronize()
        res[("host", fd.bucket_name(buckets))] = outs[0].cpu().numpy()
    res["host_paths"] = {k: v - before[k] for k, v in kernels.HOST_WEIGHT_PATHS.items()}
    del x2
    z = fd.multi_device_weighted_mean([x[:0]], [wl[:0]], W, comm=comm)[0]  # a device without clients
    torch.cuda.synchronize()
    errs = []
    for bad in (lambda: fd.multi_device_weighted_mean([x, x], [wl, wl], W, comm=comm),
                lambda: fd.multi_device_weighted_mean([x], [wl[:3]], W, comm=comm),
                lambda: fd.MultiDeviceCommunicator([dev, dev])):
        try:
            bad()
            errs.append(None)
        except (ValueError, RuntimeError) as e:
            errs.append(type(e).__name__)
    comm.close()
    q.put((res, z.cpu().numpy(), errs))


def test_single_process_multi_device_ndev1(cuda, coracle):
    """the single-process entry point at ndev = 1 is bitwise the exact
    fold (a one-rank reduce is the identity) for equal and tapered buckets, reduce and
    all-reduce; a device without clients contributes zeros; bad inputs are refused."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_multi_device_worker, args=(q,))
    p.start()
    res, z, errs = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
    x = coracle.synth_f32(K, P, seed=9)
    want = coracle.wsum_f32(x, np.float32(weights), scale=ref.mean_scale(weights))
    assert res.pop("host_paths") == {"kernel_args": 2, "uploaded": 0}
    want2 = coracle.wsum_f32(coracle.synth_f32(K, P2, seed=11), np.float32(weights), scale=ref.mean_scale(weights))
    for key in [k for k in res if k[0] == "host"]:
        y = res.pop(key)
        assert np.array_equal(y.view(np.uint32), want2.astype(np.float32).view(np.uint32)), key
    for key, y in res.items():
        assert np.array_equal(y.view(np.uint32), want.astype(np.float32).view(np.uint32)), key
    assert np.all(z == 0)
    assert errs == ["ValueError", "ValueError", "ValueError"]


def _abort_worker(q):
    """A world-1 RCCL communicator with a sharded step enqueued behind 1.5 s of other work on the
    stream: fjcomm_abort with the step still queued returns (RCCL's teardown waits for the work
    already on the device: about the blocker's 1.5 s here), the stream drains, and the aborted
    communicator refuses the next step (include/fjcomm.h)."""
    import time
    init_world1("gloo")
    try:
        import bench
        from fedjax_amd import _lib, distributed as fd, kernels
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        comm = fd.RcclCommunicator(device=dev)
        x = torch.empty(K, P, dtype=torch.float32, device=dev)
        kernels.fill_synth(x, seed=9)
        wl = torch.tensor(np.float32(ref.fedavg_weights(K, seed=3)), device=dev)
        W = float(wl.double().sum())
        fd.sharded_weighted_mean(x, wl, W, buckets=2, comm=comm)  # a healthy step first
        stream = torch.cuda.current_stream(dev)
        torch.cuda.synchronize()
        _lib.check(_lib.load().fjcomm_test_block(1_500_000, stream.cuda_stream), "fjcomm_test_block")
        fd.sharded_weighted_mean(x, wl, W, buckets=2, comm=comm)  # queued behind the blocker
        queued = not stream.query()
        t0 = time.perf_counter()
        comm.abort()
        t_abort = time.perf_counter() - t0
        drained = bench.drain_stream(stream, 30.0)
        t_drain = time.perf_counter() - t0
        try:
            fd.sharded_weighted_mean(x, wl, W, buckets=2, comm=comm)
            refused = None
        except Exception as e:  # noqa: BLE001
            refused = str(e)
        comm.abort()  # (idempotent)
        comm.close()
        q.put({"queued": queued, "t_abort": t_abort, "drained": drained, "t_drain": t_drain, "refused": refused})
    finally:
        dist.destroy_process_group()


def test_fjcomm_abort_with_a_queued_step(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_abort_worker, args=(q,))
    p.start()
    got = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert got["queued"], got  # the step was still behind the blocker when abort was called
    assert got["t_abort"] < 30.0 and got["drained"] and got["t_drain"] < 30.0, got
    assert got["refused"] and "aborted" in got["refused"], got
