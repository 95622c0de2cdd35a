"""Randomised running-sum programs through fedjax_amd.tree_util on the GPU against the oracle.

The library algorithms build their sums one client at a time (fedjax/algorithms/fed_avg.py:
132-146; hyp_cluster.py:284-304 keeps one sum per cluster and interleaves them). Each case
here draws a pytree structure (nested dict / list / tuple / None nodes, float32 leaves of
random shapes, empty ones included), 1-3 running sums, a client order, Python int or float
weights, and per client the calls a caller may make around its tree_add: tree_l2_norm /
tree_l2_squared of the delta, an unweighted tree_add, reading a sum or a norm mid-round. The deferred
chain's limits (max_clients, early-flush thresholds) are drawn too, so the chains split at
random places; each case also runs with deferral off. Every sum, mid-round read and final
tree_inverse_weight must be bitwise the oracle's op sequence (oracle/tree_util_ref.py,
tree_util.py:29-60); norms within rtol 2e-6 of the float64 norm (the reference's per-leaf
reduction order is XLA's)."""
import os

import numpy as np
import pytest
import torch

from fedjax_amd import pytree, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu

# FJ_FUZZ_CASES / FJ_FUZZ_SEED0: a longer campaign over other seeds (the suite runs the defaults)
NCASES = int(os.environ.get("FJ_FUZZ_CASES", "100"))
SEED0 = int(os.environ.get("FJ_FUZZ_SEED0", "1000"))


def _structure(rs, depth=0, budget=None):
    """A random pytree of leaf shapes (tuples) and None; budget[0] counts leaves left."""
    budget = [rs.randint(1, 13)] if budget is None else budget
    r = rs.rand()
    if depth >= 3 or budget[0] <= 1 or r < 0.35:
        if rs.rand() < 0.08:
            return None
        budget[0] -= 1
        nd = rs.randint(0, 4)
        dims = [int(rs.choice([0, 1, 3, 17, 64, 70])) if rs.rand() < 0.1 else int(rs.randint(1, 40))
                for _ in range(nd)]
        return ("leaf", tuple(dims))
    n = int(rs.randint(1, 4))
    kids = [_structure(rs, depth + 1, budget) for _ in range(n)]
    if r < 0.75:
        names = ["w", "b", "kernel", "scale", "z", "a"]
        keys = list(rs.choice(names, size=n, replace=False))
        return {str(k): v for k, v in zip(keys, kids)}  # insertion order as drawn
    return list(kids) if rs.rand() < 0.5 else tuple(kids)


def _build(spec, make):
    if isinstance(spec, dict):
        return {k: _build(v, make) for k, v in spec.items()}
    if isinstance(spec, list):
        return [_build(v, make) for v in spec]
    if isinstance(spec, tuple) and spec and spec[0] == "leaf":
        return make(spec[1])
    if isinstance(spec, tuple):
        return tuple(_build(v, make) for v in spec)
    return None


def _tmap(fn, t):
    """fn over the tensor leaves of t, keeping every node (dict insertion order included)."""
    if isinstance(t, dict):
        return {k: _tmap(fn, v) for k, v in t.items()}
    if isinstance(t, list):
        return [_tmap(fn, v) for v in t]
    if isinstance(t, tuple):
        return tuple(_tmap(fn, v) for v in t)
    return None if t is None else fn(t)


def _has_leaf(spec):
    if isinstance(spec, dict):
        return any(_has_leaf(v) for v in spec.values())
    if isinstance(spec, tuple) and spec and spec[0] == "leaf":
        return True
    if isinstance(spec, (list, tuple)):
        return any(_has_leaf(v) for v in spec)
    return False


def _bits_equal(got, want):
    g = [np.asarray(x.detach().cpu().numpy(), np.float32).reshape(-1) for x in pytree.leaves_of(got)]
    w = [np.asarray(x, np.float32).reshape(-1) for x in ref.flatten(want)[0]]
    assert len(g) == len(w)
    return all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(g, w))


def _norm64(tree_np):
    return float(np.sqrt(sum(float(np.dot(x.astype(np.float64).ravel(), x.astype(np.float64).ravel()))
                             for x in ref.flatten(tree_np)[0])))


@pytest.fixture(params=["deferred", "eager"])
def mode(request):
    tu.set_deferred_sums(request.param == "deferred")
    yield request.param
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)


@pytest.mark.parametrize("seed", range(NCASES))
def test_random_running_sum_program(cuda, mode, seed):
    rs = np.random.RandomState(SEED0 + seed)
    spec = _structure(rs)
    while not _has_leaf(spec):
        spec = _structure(rs)
    g = torch.Generator().manual_seed(seed)
    if mode == "deferred":
        tu.set_deferred_sums(True, max_clients=int(rs.choice([2, 3, 7, 4095])),
                             flush_bytes=int(rs.choice([1, 4096, 256 << 20])),
                             flush_clients=int(rs.choice([1, 2, 5, 64])))
    K, S = int(rs.randint(1, 41)) if rs.rand() < 0.9 else int(rs.randint(41, 300)), int(rs.randint(1, 4))
    hosts = [_build(spec, lambda s: ((torch.rand(s, generator=g) * 2 - 1) * 0.1)) for _ in range(K)]
    deltas = [_tmap(lambda x: x.to(cuda), h) for h in hosts]
    host_np = [_tmap(lambda x: x.numpy(), h) for h in hosts]
    params = _build(spec, lambda s: torch.zeros(s, device=cuda))
    sums = [tu.tree_zeros_like(params) for _ in range(S)]
    want = [ref.tree_zeros_like(_tmap(lambda x: x.cpu().numpy(), params)) for _ in range(S)]
    W = [0.0] * S
    used = [False] * S
    norms, want_norms = [], []
    for k in range(K):
        j = int(rs.randint(0, S))
        w = int(rs.randint(1, 501)) if rs.rand() < 0.7 else float(np.round(rs.uniform(0.05, 3.0), 3))
        if rs.rand() < 0.08:  # an unweighted add (tree_util.py:47-50)
            sums[j] = tu.tree_add(sums[j], deltas[k])
            want[j] = ref.tree_add(want[j], host_np[k])
            w_used = 1.0
        else:
            sums[j] = tu.tree_add(sums[j], tu.tree_weight(deltas[k], w))
            want[j] = ref.tree_add(want[j], ref.tree_weight(host_np[k], w))
            w_used = w
        W[j] += w_used
        used[j] = True
        u = rs.rand()
        if u < 0.3:
            norms.append(tu.tree_l2_norm(deltas[k]))
            want_norms.append(_norm64(host_np[k]))
        elif u < 0.4:
            norms.append(tu.tree_l2_squared(deltas[k]))
            want_norms.append(_norm64(host_np[k]) ** 2)
        if rs.rand() < 0.06:  # a caller reading the sum mid-round
            assert _bits_equal(sums[j], want[j]), (seed, k, "mid-round read")
        if norms and rs.rand() < 0.05:  # ... or one of the norms so far (folds the chain it waits on)
            i = int(rs.randint(0, len(norms)))
            np.testing.assert_allclose(float(norms[i]), want_norms[i], rtol=2e-6, atol=1e-30)
    for j in range(S):
        if not used[j]:
            continue
        got = tu.tree_inverse_weight(sums[j], W[j])
        assert _bits_equal(got, ref.tree_inverse_weight(want[j], W[j])), (seed, j)
    if norms:
        np.testing.assert_allclose([float(v) for v in norms], want_norms, rtol=2e-6, atol=1e-30)
