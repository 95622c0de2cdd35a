"""Client-sharded aggregation over world_size 2 with the gloo backend (CPU).

The per-rank fold is injected (``partial_fn``) with the oracle restatement so
the sharding, bucketing, W handling and reduce/all_reduce logic of
fedjax_amd.distributed run without a GPU; the GPU test runs the same function
with the HIP kernel.
"""
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import tree_util_ref as ref
from tests.rendezvous import HeldStore, init_group

K, P = 24, 5000


def _oracle_partial(x, w, scale, out):
    y = ref.wsum_dense(x.numpy(), w.numpy(), scale=np.float32(scale))
    out.copy_(torch.from_numpy(y))


def _worker(rank, world, port, all_ranks, buckets, q):
    init_group("gloo", rank, world, port)
    try:
        from fedjax_amd import distributed as fd
        weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
        W = 0.0
        for w in weights:
            W += w
        k0, k1 = fd.shard_range(K, rank, world)
        x = torch.from_numpy(ref.synth(k1 - k0, P, seed=9, k0=k0))
        wl = torch.tensor(np.float32(weights[k0:k1]))
        out = fd.sharded_weighted_mean(x, wl, W, buckets=buckets, all_ranks=all_ranks,
                                       partial_fn=_oracle_partial)
        W2 = fd.total_weight(weights[k0:k1])
        q.put((rank, out.numpy().copy(), W2))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("all_ranks,buckets", [(False, 3), (True, 3), (False, (4, 2, 1))])
def test_sharded_mean_world2_gloo(all_ranks, buckets, coracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = HeldStore(2)
    port = store.port
    procs = [ctx.Process(target=_worker, args=(r, 2, port, all_ranks, buckets, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (y, W2)) for r, y, W2 in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
    x = ref.synth(K, P, seed=9)
    r = ref.mean_scale(weights)
    want = ref.wsum_dense(x, np.float32(weights), scale=r)
    bound = coracle.bound_f32(x, np.float32(weights), r, want)
    G = 2
    # sequential-sum bound with G extra roundings
    bound = bound * (K + G + 2) / (K + 2)
    for rank in ([0, 1] if all_ranks else [0]):
        y = res[rank][0]
        assert np.all(np.abs(y.astype(np.float64) - want) <= bound), rank
        assert res[rank][1] == float(sum(weights))


def _worker_ragged(rank, world, port, q):
    init_group("gloo", rank, world, port)
    try:
        from fedjax_amd import distributed as fd
        Kr = 7
        weights = [0.5 + k for k in range(Kr)]
        k0, k1 = fd.shard_range(Kr, rank, world)
        x = torch.from_numpy(ref.synth(k1 - k0, 999, seed=4, k0=k0))
        wl = torch.tensor(np.float32(weights[k0:k1]))
        W = fd.total_weight(weights[k0:k1])
        out = fd.sharded_weighted_mean(x, wl, W, buckets=2, partial_fn=_oracle_partial)
        q.put((rank, k1 - k0, out.numpy().copy(), W))
    finally:
        dist.destroy_process_group()


def test_ragged_shards_world3_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = HeldStore(3)
    port = store.port
    procs = [ctx.Process(target=_worker_ragged, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = {r: (n, y, W) for r, n, y, W in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [res[r][0] for r in range(3)] == [3, 2, 2]
    weights = [0.5 + k for k in range(7)]
    assert all(res[r][2] == sum(weights) for r in range(3))
    x = ref.synth(7, 999, seed=4)
    want = ref.wsum_dense(x, np.float32(weights), scale=ref.mean_scale(weights))
    np.testing.assert_allclose(res[0][1], want, rtol=2e-6, atol=1e-9)


def _worker_empty(rank, world, port, q):
    init_group("gloo", rank, world, port)
    try:
        from fedjax_amd import distributed as fd
        tmpl = {"w": torch.zeros(3, 2), "b": torch.zeros(2)}
        # no rank holds a client: every rank returns None, nobody blocks in a collective
        a = fd.sharded_tree_mean([], template=tmpl if rank == 0 else None)
        b = fd.sharded_tree_mean(iter([]), all_ranks=True)
        q.put((rank, a is None and b is None))
    finally:
        dist.destroy_process_group()


def test_sharded_tree_mean_without_clients_world3_gloo():
    """ranks without clients must reach the same collectives (no hang)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = HeldStore(3)
    port = store.port
    procs = [ctx.Process(target=_worker_empty, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: True, 1: True, 2: True}


def _worker_bad(rank, world, port, q):
    init_group("gloo", rank, world, port)
    try:
        from fedjax_amd import distributed as fd
        tmpl = {"w": torch.zeros(3, 2), "b": torch.zeros(2)}
        # rank 1's own clients fail its local checks (here: no GPU for the fold's pointer
        # table); rank 0 has none. Both must raise — neither may wait in the all_gather.
        clients = [(tmpl, 1), ({"w": torch.zeros(3, 2), "c": torch.zeros(2)}, 2)] if rank == 1 else []
        try:
            fd.sharded_tree_mean(clients, template=tmpl)
            q.put((rank, "returned"))
        except Exception as e:  # noqa: BLE001
            q.put((rank, type(e).__name__ + ": " + str(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_tree_mean_local_failure_raises_on_every_rank_gloo():
    """a rank whose local validation fails flags it in the header exchange, so
    every rank raises (that rank its own error, the others a ValueError naming it)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = HeldStore(2)
    port = store.port
    procs = [ctx.Process(target=_worker_bad, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0].startswith("ValueError") and "rank(s) [1]" in res[0], res
    assert not res[1].startswith(("returned", "ValueError: sharded_tree_mean: rank")), res


@pytest.mark.parametrize("world", [1, 4, 8])
def test_sharded_mean_1_to_8_ranks_gloo(world, coracle):
    """The analogue of for_each_client_test.py:388-438 (the pmap backend on 1..8 simulated
    devices against the single-device result): 1, 4 and 8 gloo ranks on the CPU. One rank
    is bitwise the single fold; G ranks stay within the G-partial bound of DESIGN.md §4."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = HeldStore(world)
    port = store.port
    procs = [ctx.Process(target=_worker, args=(r, world, port, True, 2, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (y, W2)) for r, y, W2 in (q.get(timeout=180) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    weights = [int(v) for v in ref.fedavg_weights(K, seed=3)]
    x = ref.synth(K, P, seed=9)
    r = ref.mean_scale(weights)
    want = ref.wsum_dense(x, np.float32(weights), scale=r)
    if world == 1:
        assert np.array_equal(res[0][0].view(np.uint32), want.astype(np.float32).view(np.uint32))
    bound = coracle.bound_f32(x, np.float32(weights), r, want) * (K + world + 2) / (K + 2)
    for rank in range(world):  # all_ranks: every rank holds the mean, the same bits on each
        assert np.all(np.abs(res[rank][0].astype(np.float64) - want) <= bound), rank
        assert np.array_equal(res[rank][0], res[0][0])
        assert res[rank][1] == float(sum(weights))
