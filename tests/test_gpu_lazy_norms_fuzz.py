"""Random programs over standalone lazy norms (fjhost.cpp "standalone lazy norms"): norms and
squared norms taken in any order, views read early or late or dropped, tree_mean /
mean_aggregator().apply over random subsets (some with a delta listed twice), orders and
container kinds (list, tuple, generator), leaves replaced after a norm, pending limits and buffer boundaries crossed. Every
read value must be the bits of that delta's norm computed alone (the value does not depend on
when or how it is computed) and every mean the oracle's bits (oracle/tree_util_ref.py restates
tree_util.py:76-96)."""
import os

import numpy as np
import pytest
import torch

import fedjax_amd
from fedjax_amd import pytree, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu
H = tu._HOST
SHAPES = [{"a": (701,), "b": {"c": (33, 3)}}, {"w": (2053,), "b": (9,)}]


def tmap(fn, t):
    return {k: tmap(fn, v) for k, v in t.items()} if isinstance(t, dict) else fn(t)


def bits1(v):
    return int(v.detach().reshape(()).view(torch.int32).item())


def run_program(seed, cuda):
    rng = np.random.RandomState(seed)
    shapes = SHAPES[seed % len(SHAPES)]
    g = torch.Generator(device=cuda).manual_seed(seed)
    n = int(rng.randint(4, 24))
    deltas = [tmap(lambda s: (torch.rand(s, device=cuda, generator=g) - 0.5), shapes) for _ in range(n)]
    # each delta's norms computed alone (immediate reads): the bits every later view must show
    canon = []
    for d in deltas:
        a, b = tu.tree_l2_norm(d), tu.tree_l2_squared(d)
        canon.append((bits1(a), bits1(b)))
    if rng.rand() < 0.3:
        tu.set_lazy_norms(True, max_pending=int(rng.randint(1, 8)))
    views = []  # (delta index, which, view)
    for _ in range(int(rng.randint(5, 40))):
        op = rng.randint(6)
        if op <= 1:  # take a norm
            i, which = int(rng.randint(n)), int(rng.randint(2))
            views.append((i, which, (tu.tree_l2_norm if which else tu.tree_l2_squared)(deltas[i])))
        elif op == 2 and views:  # read one
            i, which, v = views[rng.randint(len(views))]
            assert bits1(v) == canon[i][1 - which], (seed, i, which)
        elif op == 3 and views:  # drop one
            views.pop(rng.randint(len(views)))
        elif op == 4:  # a mean over a random subset, order and container
            m = int(rng.randint(1, n + 1))
            # (sometimes with replacement: a client sampled twice lists its delta twice)
            idx = list(rng.randint(n, size=m)) if rng.rand() < 0.3 else list(rng.permutation(n)[:m])
            ws = [int(rng.randint(1, 9)) if rng.rand() < 0.7 else float(rng.rand() + 0.1) for _ in idx]
            pairs = [(deltas[i], w) for i, w in zip(idx, ws)]
            kind = rng.randint(4)
            if kind == 0:
                m = tu.tree_mean(pairs)
            elif kind == 1:
                m = tu.tree_mean(tuple(pairs))
            elif kind == 2:
                m = tu.tree_mean(p for p in pairs)
            else:
                m, _ = fedjax_amd.aggregators.mean_aggregator().apply(
                    [(str(i), d, w) for i, (d, w) in enumerate(pairs)], fedjax_amd.aggregators.mean_aggregator().init())
            want = ref.tree_mean([(tmap(lambda x: x.cpu().numpy(), d), w) for d, w in pairs])
            for a, b in zip(pytree.leaves_of(m), pytree.leaves_of(want)):
                assert np.array_equal(a.cpu().numpy().reshape(-1).view(np.uint32),
                                      np.asarray(b).reshape(-1).view(np.uint32)), seed
        elif op == 5:  # replace a leaf: views taken before keep the old value, new ones see the new
            i = int(rng.randint(n))
            d = deltas[i]
            key = sorted(d)[0]
            if isinstance(d[key], torch.Tensor):
                d[key] = d[key] * 2.0
                a, b = tu.tree_l2_norm(d), tu.tree_l2_squared(d)
                old = canon[i]
                canon[i] = (bits1(a), bits1(b))
                # pending views of the old contents: compute them now, against the old bits
                for j, which, v in views:
                    if j == i:
                        assert bits1(v) == old[1 - which], (seed, i)
                views = [(j, w_, v) for j, w_, v in views if j != i]
    for i, which, v in views:
        assert bits1(v) == canon[i][1 - which], (seed, i, which)
    x64 = [np.sqrt(sum(float((x.double() ** 2).sum()) for x in pytree.leaves_of(d))) for d in deltas]
    np.testing.assert_allclose([np.float32(np.array(c[0], np.int32).view(np.float32)) for c in canon], x64, rtol=2e-6)


# FJ_FUZZ_CASES / FJ_FUZZ_SEED0: a longer campaign over other seeds (the suite runs the defaults)
NCASES = int(os.environ.get("FJ_FUZZ_CASES", "200"))
SEED0 = int(os.environ.get("FJ_FUZZ_SEED0", "0"))
BLOCK = 50


@pytest.mark.parametrize("block", range((NCASES + BLOCK - 1) // BLOCK))
def test_lazy_norm_programs(block, cuda):
    tu.set_deferred_sums(True)
    try:
        for seed in range(SEED0 + block * BLOCK, SEED0 + min(NCASES, (block + 1) * BLOCK)):
            run_program(seed, cuda)
            tu.set_lazy_norms(True, max_pending=16383)
    finally:
        H.solo_resolve(None)
        tu.set_lazy_norms(True, max_pending=16383)
