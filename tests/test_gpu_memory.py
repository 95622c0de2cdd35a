"""fedjax_amd.memory (include/fjalloc.h): client deltas allocated under the fjalloc-backed
pool fold to the same bits as default allocations, the pool's segments are slices of its
chunks (the caller-side placement of DESIGN.md §3), and a released pool gives its chunks back."""
import numpy as np
import pytest
import torch

from fedjax_amd import memory, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu


def test_delta_pool_allocations_fold_bitwise(cuda):
    g = torch.Generator().manual_seed(5)
    shapes = [(1001,), (64, 33), (9216, 16)]
    host = [[torch.rand(s, generator=g) - 0.5 for s in shapes] for _ in range(24)]
    weights = [int(w) for w in ref.fedavg_weights(24, seed=2)]
    with memory.delta_allocation(cuda):
        pooled = [[x.to(cuda) for x in c] for c in host]
    plain = [[x.to(cuda) for x in c] for c in host]
    st = memory.stats(cuda)
    assert st["live_segments"] >= 1 and st["failures"] == 0
    from fedjax_amd import _lib
    assert _lib.load().fjalloc_configure(1 << 30, 64 << 10, 2, 68 << 10) == -1  # layout fixed once allocating
    lo, hi = st["base"], st["base"] + st["bump_offset"]
    assert all(lo <= x.data_ptr() < hi for c in pooled for x in c)  # inside the first chunk
    assert not any(lo <= x.data_ptr() < hi for c in plain for x in c)
    a = tu.tree_mean(list(zip(pooled, weights)))
    b = tu.tree_mean(list(zip(plain, weights)))
    want = ref.tree_mean([([x.numpy() for x in c], w) for c, w in zip(host, weights)])
    for x, y, z in zip(a, b, want):
        assert np.array_equal(x.cpu().numpy().view(np.uint32), z.view(np.uint32))
        assert np.array_equal(y.cpu().numpy().view(np.uint32), z.view(np.uint32))
    del pooled
    torch.cuda.synchronize()


def test_released_pool_returns_its_chunks_and_a_new_pool_works(cuda):
    """Segments over one chunk (1 GiB) spill into a second; releasing the pool after its
    tensors are gone frees every segment and returns both chunks; a new pool then
    allocates and folds correctly."""
    memory.release(cuda)  # (whatever earlier tests left)
    free0 = torch.cuda.mem_get_info(cuda)[0]
    with memory.delta_allocation(cuda):
        big = [torch.full((100 << 20,), float(k + 1), device=cuda) for k in range(4)]  # 4 x 400 MiB
    st = memory.stats(cuda)
    assert st["live_segments"] >= 4 and st["failures"] == 0 and st["mapped_bytes"] >= 4 * (400 << 20)
    assert [float(x[-1]) for x in big] == [1.0, 2.0, 3.0, 4.0]
    del big
    memory.release(cuda)
    st = memory.stats(cuda)
    assert st["live_segments"] == 0 and st["mapped_bytes"] == 0, st
    assert torch.cuda.mem_get_info(cuda)[0] >= free0 - (64 << 20)  # the chunks went back
    host = [[torch.full((3000,), 0.5 * (k + 1))] for k in range(5)]
    with memory.delta_allocation(cuda):
        pooled = [[x.to(cuda) for x in c] for c in host]
    got = tu.tree_mean([(c, k + 1) for k, c in enumerate(pooled)])
    want = ref.tree_mean([([x.numpy() for x in c], k + 1) for k, c in enumerate(host)])
    assert np.array_equal(got[0].cpu().numpy().view(np.uint32), want[0].view(np.uint32))
    del pooled, got
    memory.release(cuda)


def test_freed_neighbours_coalesce_and_take_a_larger_segment(cuda):
    """ADVICE r4 (fjalloc mode 2): freed slices are merged with their free neighbours and
    reused best-fit, so a segment that fits only in freed space (a torch out-of-memory retry
    after freeing its cache) needs no new hipMalloc; the bump tail takes back a freed range at
    its end; an emptied chunk still goes back to the runtime."""
    from fedjax_amd import _lib
    lib = _lib.load()
    memory.release(cuda)
    dev = cuda.index if cuda.index is not None else 0
    MiB = 1 << 20
    st0 = memory.stats(cuda)
    a = lib.fjalloc_alloc(100 * MiB, dev, None)
    b = lib.fjalloc_alloc(200 * MiB, dev, None)
    c = lib.fjalloc_alloc(700 * MiB, dev, None)  # a 1 GiB chunk now has < 290 MiB of bump tail
    assert a and b and c
    st1 = memory.stats(cuda)
    assert st1["failures"] == st0["failures"]
    lib.fjalloc_free(a, 0, dev, None)
    lib.fjalloc_free(b, 0, dev, None)
    st2 = memory.stats(cuda)
    assert st2["free_bytes"] >= st1["free_bytes"] + 300 * MiB  # a and b (with b's stagger bytes)
    d = lib.fjalloc_alloc(290 * MiB, dev, None)  # only the merged a+b range holds it
    st3 = memory.stats(cuda)
    assert d and st3["chunks"] == st1["chunks"] and st3["reused_ranges"] == st2["reused_ranges"] + 1
    if st0["chunks"] == 0:  # a, b, c shared one fresh chunk: d starts where a's range did
        assert a - 31 * (68 << 10) <= d <= a
    lib.fjalloc_free(d, 0, dev, None)
    lib.fjalloc_free(c, 0, dev, None)
    st4 = memory.stats(cuda)
    assert st4["chunks"] == st0["chunks"] and st4["live_segments"] == st0["live_segments"]
    assert st4["failures"] == st0["failures"]


def test_set_default_pools_the_deltas_fedjax_amd_produces(cuda):
    """under memory.set_default(True) the deltas fedjax_amd produces — host
    deltas copied by memory.to_device, ClientDeltaSlab storage (DeltaIngestor's rows) and a
    materialised tree_weight — come from the delta pool's chunks; the fold gives the same bits;
    switched off, allocations are torch's own again."""
    import fedjax_amd
    memory.release(cuda)
    g = torch.Generator().manual_seed(8)
    host = [{"a": torch.rand(5000, generator=g) - 0.5, "b": [torch.rand(33, 3, generator=g) - 0.5]}
            for _ in range(6)]
    weights = [3, 1, 4, 1, 5, 9]

    def in_pool(ptr):  # inside the first chunk (these few KB all fit in it)
        st = memory.stats(cuda)
        return st["chunks"] > 0 and st["base"] <= ptr < st["base"] + (1 << 30)
    memory.set_default(True)
    try:
        pooled = [memory.to_device(t, cuda) for t in host]
        slab = fedjax_amd.ClientDeltaSlab(host[0], 4, device=cuda)
        wt = tu.tree_weight(pooled[0], 2).materialize()  # (a deferred WeightedTree, made concrete here)
    finally:
        memory.set_default(False)
    assert not memory.default_enabled()
    assert all(in_pool(x.data_ptr()) for c in pooled for x in [c["a"], c["b"][0]])
    assert in_pool(slab.storage.data_ptr())
    assert in_pool(wt["a"].data_ptr())
    plain = [memory.to_device(t, cuda) for t in host]
    assert not in_pool(plain[0]["a"].data_ptr())
    a = tu.tree_mean(list(zip(pooled, weights)))
    b = tu.tree_mean(list(zip(plain, weights)))
    want = ref.tree_mean([({"a": t["a"].numpy(), "b": [t["b"][0].numpy()]}, w) for t, w in zip(host, weights)])
    for x, y, z in zip([a["a"], a["b"][0]], [b["a"], b["b"][0]], [want["a"], want["b"][0]]):
        assert np.array_equal(x.cpu().numpy().view(np.uint32), z.view(np.uint32))
        assert torch.equal(x.view(torch.int32), y.view(torch.int32))
    del pooled, slab, wt, a
    torch.cuda.synchronize()
    memory.release(cuda)
