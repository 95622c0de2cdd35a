"""fedjax_amd.memory (include/fjalloc.h): client deltas allocated under the fjalloc-backed
pool fold to the same bits as default allocations, and the pool's segments come from one
reserved virtual range (the caller-side placement of DESIGN.md §3)."""
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
    lo, hi = st["base"], st["base"] + st["bump_offset"]
    assert all(lo <= x.data_ptr() < hi for c in pooled for x in c)  # inside the reserved range
    assert not any(lo <= x.data_ptr() < hi for c in plain for x in c)
    a = tu.tree_mean(list(zip(pooled, weights)))
    b = tu.tree_mean(list(zip(plain, weights)))
    want = ref.tree_mean([([x.numpy() for x in c], w) for c, w in zip(host, weights)])
    for x, y, z in zip(a, b, want):
        assert np.array_equal(x.cpu().numpy().view(np.uint32), z.view(np.uint32))
        assert np.array_equal(y.cpu().numpy().view(np.uint32), z.view(np.uint32))
    del pooled
    torch.cuda.synchronize()
