"""Per-call tree ops on the GPU (include/fjtree.h, fedjax_amd/csrc/fjtree.hip): the running
sum of fedjax/algorithms/fed_avg.py:132-146 called literally —

    s = tree_zeros_like(params)
    for each client: s = tree_add(s, tree_weight(delta, n)); tree_l2_norm(delta)
    mean = tree_inverse_weight(s, sum n)

— must be bitwise the reference's op sequence (numpy restatement: fl(s + fl(x * f32(n))),
then fl(s * f32(1/W))), with tree_weight deferred into the tree_add that consumes it and
the delta's l2 norm taken from that launch. Edge cases: unaligned views, empty leaves,
more leaves than one launch holds, non-float32 leaves, structure mismatch, a delta
modified between tree_weight and tree_add.
"""
import numpy as np
import pytest
import torch

import fedjax_amd
from fedjax_amd import pytree, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu


def pytest_generate_tests(metafunc):
    """Every test runs with deferred running sums (PendingSum, the default) and with one
    fused launch per tree_add (set_deferred_sums(False)); tests marked deferred_only test
    the deferred chain itself and run in that mode only."""
    if "sum_mode" in metafunc.fixturenames:
        only = metafunc.definition.get_closest_marker("deferred_only") is not None
        metafunc.parametrize("sum_mode", ["deferred"] if only else ["deferred", "eager"], indirect=True)


@pytest.fixture(autouse=True)
def sum_mode(request):
    mode = getattr(request, "param", "deferred")
    tu.set_deferred_sums(mode == "deferred")
    yield mode
    tu.set_deferred_sums(True)


EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def tmap(fn, t):
    return {k: tmap(fn, v) for k, v in t.items()} if isinstance(t, dict) else fn(t)


def rand_tree(shapes, g, scale=0.01):
    return tmap(lambda s: (torch.rand(s, generator=g) * 2 - 1) * scale, shapes)


def to_dev(t, dev):
    return tmap(lambda x: x.to(dev), t)


def to_np(t):
    return tmap(lambda x: x.detach().cpu().numpy(), t)


def leaves_np(t):
    return [x.detach().cpu().numpy().reshape(-1) for x in pytree.leaves_of(t)]


def literal_loop(tu_mod, params, deltas, weights, with_norm=True):
    """fedjax/algorithms/fed_avg.py:132-146 written against a tree_util module."""
    s = tu_mod.tree_zeros_like(params)
    n_sum = 0.
    norms = []
    for d, n in zip(deltas, weights):
        s = tu_mod.tree_add(s, tu_mod.tree_weight(d, n))
        n_sum += n
        if with_norm:
            norms.append(tu_mod.tree_l2_norm(d))
    return tu_mod.tree_inverse_weight(s, n_sum), norms


def test_literal_running_sum_bitwise_emnist(cuda, sum_mode):
    g = torch.Generator().manual_seed(3)
    K = 24
    deltas_h = [rand_tree(EMNIST, g) for _ in range(K)]
    weights = [int(v) for v in ref.fedavg_weights(K, seed=4)]
    weights[5] = 2.5  # a float weight in the middle (weak float)
    params = to_dev(tmap(lambda s: torch.zeros(s), EMNIST), cuda)
    deltas = [to_dev(d, cuda) for d in deltas_h]
    mean, norms = literal_loop(tu, params, deltas, weights)
    # the reference's op sequence in numpy (oracle/tree_util_ref.py restates tree_util.py:29-61)
    s = tmap(lambda s: np.zeros(s, np.float32), EMNIST)
    n_sum = 0.
    for d, n in zip(deltas_h, weights):
        s = ref.tree_add(s, ref.tree_weight(to_np(d), n))
        n_sum += n
    want = ref.tree_inverse_weight(s, n_sum)
    for got, w in zip(leaves_np(mean), [x.reshape(-1) for x in pytree.leaves_of(want)]):
        assert np.array_equal(bits(got), bits(w))
    # eager mode: the fused norms are the standalone fjtree norms' bits; deferred mode: the
    # fold's fused per-client norms (another fixed order). Both within f32 rounding of f64.
    for d, nrm in zip(deltas, norms):
        alone = tu._leaf_fold([d], [1], [None], norm_operand=0, no_out=True)[2]
        if sum_mode == "eager":
            assert torch.equal(nrm.view(torch.int32), alone.view(torch.int32))
        else:
            assert type(nrm) is tu._NormView
            np.testing.assert_allclose(float(nrm), float(alone), rtol=2e-6)
        x64 = np.concatenate([x.astype(np.float64) for x in leaves_np(d)])
        np.testing.assert_allclose(float(nrm), np.sqrt((x64 * x64).sum()), rtol=2e-6)


def test_weighted_tree_is_deferred_and_fused(cuda, monkeypatch, sum_mode):
    """tree_weight returns a WeightedTree that is never computed on its own. Eager mode:
    tree_add consumes it in ONE fjtree launch and tree_l2_norm of the same delta reuses
    that launch. Deferred mode: tree_add launches nothing (a PendingSum), the norm is one
    norm-only launch, and the sum is folded when read."""
    g = torch.Generator().manual_seed(5)
    d = to_dev(rand_tree({"a": (1000,), "b": (7, 3)}, g), cuda)
    s = to_dev(rand_tree({"a": (1000,), "b": (7, 3)}, g), cuda)
    wt = tu.tree_weight(d, 7)
    assert type(wt) is tu.WeightedTree and wt._value is None
    calls = []
    real = tu._leaf_fold
    monkeypatch.setattr(tu, "_leaf_fold", lambda *a, **k: calls.append(a) or real(*a, **k))
    out = tu.tree_add(s, wt)
    assert type(out) is (tu.PendingSum if sum_mode == "deferred" else dict)
    assert len(calls) == (0 if sum_mode == "deferred" else 1)
    nrm = tu.tree_l2_norm(d)
    # eager: one fused launch gave the sum and the norm; deferred: nothing launched yet
    assert len(calls) == (0 if sum_mode == "deferred" else 1) and wt._value is None
    want = {k: to_np(s)[k] + to_np(d)[k] * np.float32(7) for k in ("a", "b")}
    for k in ("a", "b"):
        assert np.array_equal(bits(out[k].cpu().numpy()), bits(want[k]))
    x64 = np.concatenate([to_np(d)[k].astype(np.float64).reshape(-1) for k in ("a", "b")])
    np.testing.assert_allclose(float(nrm), np.sqrt((x64 ** 2).sum()), rtol=2e-6)
    assert float(tu.tree_l2_squared(d)) == pytest.approx(float(nrm) ** 2, rel=1e-6)


def test_weighted_tree_materializes_on_use(cuda):
    g = torch.Generator().manual_seed(6)
    d = to_dev(rand_tree({"a": (33,), "b": {"c": (5, 5)}}, g), cuda)
    wt = tu.tree_weight(d, 3)
    want = {"a": to_np(d)["a"] * np.float32(3), "c": to_np(d)["b"]["c"] * np.float32(3)}
    assert np.array_equal(bits(wt["a"].cpu().numpy()), bits(want["a"]))  # indexing
    assert sorted(wt) == ["a", "b"] and len(wt) == 2 and "b" in wt and list(wt.keys()) == ["a", "b"]
    leaves = pytree.leaves_of(wt)  # pytree walks see the weighted tree
    assert np.array_equal(bits(leaves[1].cpu().numpy()), bits(want["c"]))
    # tree_mean / tree_sum / tree_inverse_weight over deferred trees
    m = tu.tree_mean([(tu.tree_weight(d, 2), 1), (tu.tree_weight(d, 4), 3)])
    wm = (to_np(d)["a"] * np.float32(2) * np.float32(1) + to_np(d)["a"] * np.float32(4) * np.float32(3)) \
        * np.float32(1 / 4)
    assert np.array_equal(bits(m["a"].cpu().numpy()), bits(wm))
    iw = tu.tree_inverse_weight(tu.tree_weight(d, 3), 3.0)
    assert np.array_equal(bits(iw["a"].cpu().numpy()), bits(want["a"] * np.float32(1 / 3.0)))
    # both operands deferred
    both = tu.tree_add(tu.tree_weight(d, 2), tu.tree_weight(d, 5))
    wb = to_np(d)["a"] * np.float32(2) + to_np(d)["a"] * np.float32(5)
    assert np.array_equal(bits(both["a"].cpu().numpy()), bits(wb))


def test_modified_delta_raises(cuda, sum_mode):
    d = {"a": torch.ones(100, device=cuda)}
    s = {"a": torch.zeros(100, device=cuda)}
    wt = tu.tree_weight(d, 2)
    d["a"].add_(1.0)  # in place, before the weighted value is used: the sum refuses
    with pytest.raises(RuntimeError, match="modified"):
        tu.tree_add(s, wt).materialize()  # (a deferred sum raises at its fold)
    wt = tu.tree_weight(d, 2)
    d["a"] = torch.zeros(100, device=cuda)  # leaf replaced
    if sum_mode == "deferred":  # the deferred sum holds the captured leaves: the value tree_weight saw
        got = tu.tree_add(s, wt)
        assert torch.equal(got["a"], torch.full((100,), 4.0, device=cuda))
    else:  # one launch per tree_add over the input as it is now: refused
        with pytest.raises(RuntimeError, match="modified"):
            tu.tree_add(s, wt)
    wt = tu.tree_weight(d, 2)
    d["a"] = torch.ones(100, device=cuda)  # replaced, then the weighted value itself is used: refused
    with pytest.raises(RuntimeError, match="changed structure|modified"):
        wt.materialize()
    # the fused-norm cache does not answer for a modified delta
    d = {"a": torch.ones(100, device=cuda)}
    tu.tree_add(s, tu.tree_weight(d, 2))
    d["a"].mul_(2.0)
    assert float(tu.tree_l2_norm(d)) == pytest.approx(20.0)


def test_fast_path_edges(cuda):
    # unaligned views (scalar loads), empty leaves, alias-free outputs
    base = torch.arange(1, 4001, dtype=torch.float32, device=cuda) / 1000
    d = {"u": base[1:3002], "e": base[:0], "v": base[3002:3999]}
    s = {"u": base[:3001].clone(), "e": base[:0].clone(), "v": base[3:1000].clone()}
    out = tu.tree_add(s, tu.tree_weight(d, 3))
    for k in ("u", "v"):
        want = s[k].cpu().numpy() + d[k].cpu().numpy() * np.float32(3)
        assert np.array_equal(bits(out[k].cpu().numpy()), bits(want))
    assert out["e"].numel() == 0
    x64 = np.concatenate([d[k].cpu().numpy().astype(np.float64) for k in ("e", "u", "v")])
    np.testing.assert_allclose(float(tu.tree_l2_norm(d)), np.sqrt((x64 ** 2).sum()), rtol=2e-6)
    assert float(tu.tree_l2_norm({"e": base[:0]})) == 0.0
    # more leaves than one fjtree launch holds: the pytree kernel path, same bits
    many = {f"l{i:03d}": torch.full((3,), float(i), device=cuda) for i in range(70)}
    got = tu.tree_add(many, tu.tree_weight(many, 2))
    assert all(torch.equal(got[k], many[k] * 3) for k in many)
    # bf16 leaves and int leaves: computed eagerly by the pytree kernel
    hb = {"a": torch.ones(10, dtype=torch.bfloat16, device=cuda)}
    assert type(tu.tree_weight(hb, 3)) is not tu.WeightedTree
    hi = {"a": torch.arange(10, dtype=torch.int32, device=cuda)}
    r = tu.tree_add(hi, tu.tree_weight(hi, 2))
    assert r["a"].dtype == torch.int32 and torch.equal(r["a"], hi["a"] * 3)
    # structure mismatch raises like jax.tree.map
    with pytest.raises(ValueError):
        tu.tree_add({"a": torch.ones(3, device=cuda)}, tu.tree_weight({"b": torch.ones(3, device=cuda)}, 2))
    with pytest.raises(ValueError):
        tu.tree_add({"a": torch.ones(3, device=cuda)}, tu.tree_weight({"a": torch.ones(4, device=cuda)}, 2))


@pytest.mark.parametrize("K", [128])
def test_literal_loop_configs1_bitwise_and_host_cost(K, cuda, sum_mode):
    """configs[1] shape (EMNIST-CNN, 1,206,590 params): the literal loop over K=128 clients
    is bitwise RunningMean / tree_mean and costs one launch per client (timed in
    tools/time_literal_loop.py)."""
    g = torch.Generator(device=cuda).manual_seed(8)
    deltas = [tmap(lambda s: (torch.rand(s, device=cuda, generator=g) - 0.5) * 0.02, EMNIST) for _ in range(K)]
    weights = [int(v) for v in ref.fedavg_weights(K, seed=9)]
    params = tmap(lambda s: torch.zeros(s, device=cuda), EMNIST)
    mean, norms = literal_loop(tu, params, deltas, weights)
    rm = fedjax_amd.aggregators.RunningMean(params, buffer_clients=16, device=cuda)
    for d, n in zip(deltas, weights):
        rm.add(d, n)
    want = rm.result()
    for a, b in zip(pytree.leaves_of(mean), pytree.leaves_of(want)):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    nn = tu.tree_l2_norms(deltas)
    np.testing.assert_allclose(torch.stack(norms).cpu().numpy(), nn.cpu().numpy(), rtol=2e-6)


@pytest.mark.deferred_only
def test_pending_sum_chain_semantics(cuda, sum_mode):
    """PendingSum keeps every intermediate sum valid (s1 stays s0 + x1 after s2 is built),
    folds in bounded chunks under the budget, applies tree_inverse_weight's scale in the
    same launch, and refuses a delta modified in place after its tree_weight."""
    g = torch.Generator().manual_seed(11)
    shapes = {"a": (1001,), "b": {"c": (6, 7)}}
    xs = [to_dev(rand_tree(shapes, g), cuda) for _ in range(9)]
    z = tu.tree_zeros_like(xs[0])
    s1 = tu.tree_add(z, tu.tree_weight(xs[0], 3))
    s2 = tu.tree_add(s1, tu.tree_weight(xs[1], 5))
    s3 = tu.tree_add(tu.tree_weight(xs[2], 0.5), s2)  # the sum on the right
    assert all(type(v) is tu.PendingSum for v in (s1, s2, s3))
    npz = [to_np(x) for x in xs]

    def want(ks, ws, inv=None):
        acc = tmap(lambda s: np.zeros(s, np.float32), shapes)
        for k, w in zip(ks, ws):
            acc = ref.tree_add(acc, ref.tree_weight(npz[k], w))
        return acc if inv is None else ref.tree_inverse_weight(acc, inv)

    def same(got, w):
        return all(np.array_equal(bits(a), bits(b.reshape(-1)))
                   for a, b in zip(leaves_np(got), pytree.leaves_of(w)))
    assert same(s3, want([0, 1, 2], [3, 5, 0.5]))
    assert same(s1, want([0], [3]))  # an older link, folded after a newer one
    assert same(tu.tree_inverse_weight(s2, 8.0), want([0, 1], [3, 5], 8.0))
    # a plain tree added to a pending sum (weight 1), then more clients after a fold
    s4 = tu.tree_add(s3, xs[3])
    s5 = tu.tree_add(s4, tu.tree_weight(xs[4], 2))
    assert same(s5, want([0, 1, 2, 3, 4], [3, 5, 0.5, 1, 2]))
    # budget: at most 3 pending clients per fold, same bits
    tu.set_deferred_sums(True, max_clients=3)
    try:
        s = z
        for k in range(9):
            s = tu.tree_add(s, tu.tree_weight(xs[k], k + 1))
        assert same(s, want(range(9), [k + 1 for k in range(9)]))
    finally:
        tu.set_deferred_sums(True, max_clients=4096)
    # a delta updated in place after it joined the chain: the fold refuses
    s = tu.tree_add(z, tu.tree_weight(xs[5], 2))
    xs[5]["a"].add_(1.0)
    with pytest.raises(RuntimeError, match="modified"):
        s.materialize()
    # the base of the chain: a leaf replaced after tree_add keeps the value the call saw
    # (the reference's semantics); a leaf updated in place makes the fold refuse
    base = tu.tree_zeros_like(xs[0])
    s = tu.tree_add(base, tu.tree_weight(xs[6], 2))
    base["a"] = torch.ones_like(base["a"])
    assert same(s, want([6], [2]))
    base = tu.tree_zeros_like(xs[0])
    s = tu.tree_add(tu.tree_add(base, tu.tree_weight(xs[6], 2)), tu.tree_weight(xs[7], 3))
    base["b"]["c"].add_(1.0)
    with pytest.raises(RuntimeError, match="running sum passed to tree_add was modified"):
        tu.tree_inverse_weight(s, 5.0)


@pytest.mark.deferred_only
def test_lazy_norms_of_a_deferred_sum(cuda, sum_mode):
    """tree_l2_norm of the delta just added to a deferred sum is a _NormView that the sum's
    fold fills: reading it first runs the fold (any torch function or method), reading it
    after tree_inverse_weight needs nothing more, and once filled the view no longer keeps
    the chain (or its deltas) alive."""
    import gc
    import weakref
    g = torch.Generator().manual_seed(12)
    shapes = {"a": (5000,), "b": {"c": (33, 3)}}
    xs = [to_dev(rand_tree(shapes, g), cuda) for _ in range(6)]

    def f64norm(t):
        x = np.concatenate([v.astype(np.float64) for v in leaves_np(t)])
        return np.sqrt((x * x).sum())
    # read before the sum is used: the read runs the fold
    s = tu.tree_zeros_like(xs[0])
    views = []
    for k, x in enumerate(xs):
        s = tu.tree_add(s, tu.tree_weight(x, k + 1))
        views.append((tu.tree_l2_norm(x), tu.tree_l2_squared(x)))
    assert all(type(v) is tu._NormView for pair in views for v in pair)
    assert s._value is None
    got = torch.stack([v for v, _ in views]).cpu().numpy()  # one flush covers the chain
    assert s._value is not None
    np.testing.assert_allclose(got, [f64norm(x) for x in xs], rtol=2e-6)
    np.testing.assert_allclose([float(q) for _, q in views], [f64norm(x) ** 2 for x in xs], rtol=4e-6)
    assert f"{views[0][0]:.4f}" == f"{float(views[0][0]):.4f}"
    # read after tree_inverse_weight: the fold that produced the mean filled them
    s = tu.tree_zeros_like(xs[0])
    norms = {}
    for k, x in enumerate(xs):
        s = tu.tree_add(s, tu.tree_weight(x, 2))
        norms[k] = {"delta_l2_norm": tu.tree_l2_norm(x)}
    link = weakref.ref(s)
    mean = tu.tree_inverse_weight(s, 12.0)
    del s
    gc.collect()
    assert link() is None  # the filled views hold no link (nor the deltas it captured)
    np.testing.assert_allclose([float(norms[k]["delta_l2_norm"]) for k in range(6)],
                               [f64norm(x) for x in xs], rtol=2e-6)
    want = tmap(lambda s: np.zeros(s, np.float32), shapes)
    for x in xs:
        want = ref.tree_add(want, ref.tree_weight(to_np(x), 2))
    want = ref.tree_inverse_weight(want, 12.0)
    for a, b in zip(leaves_np(mean), pytree.leaves_of(want)):
        assert np.array_equal(bits(a), bits(b.reshape(-1)))
    # a norm of a delta that is not the last one added is not the chain's: a standalone lazy norm
    s = tu.tree_add(tu.tree_zeros_like(xs[0]), tu.tree_weight(xs[0], 1))
    s = tu.tree_add(s, tu.tree_weight(xs[1], 1))
    v = tu.tree_l2_norm(xs[0])
    assert type(v._ticket) is tu._HOST.SoloNorm
    np.testing.assert_allclose(float(v), f64norm(xs[0]), rtol=2e-6)


@pytest.mark.deferred_only
def test_lazy_norm_pool_across_rounds(cuda, sum_mode):
    """The library loop's per-client tree_l2_norm takes pre-made views (fjhost's lazy-norm pool,
    built while each round's final fold runs) and recognises the captured dict tree by its dict
    version tags instead of re-walking it. Over rounds of growing size (more clients than the
    pool holds), with a mid-round read, every norm equals the float64 norm, every mean is the
    oracle's bits, and the pool is refilled to the round's size; a delta dict changed after its
    tree_weight gets the norm of its new contents, eagerly."""
    H = tu._HOST
    H.drop_pool()
    g = torch.Generator().manual_seed(41)
    shapes = {"a": (5000,), "b": {"c": (33, 3)}}
    xs = [to_dev(rand_tree(shapes, g), cuda) for _ in range(20)]

    def f64norm(t):
        x = np.concatenate([v.astype(np.float64) for v in leaves_np(t)])
        return np.sqrt((x * x).sum())
    kept = alias = None
    for rnd, K in enumerate((6, 9, 12, 12, 12, 12)):
        s, norms = tu.tree_zeros_like(xs[0]), []
        for k in range(K):
            s = tu.tree_add(s, tu.tree_weight(xs[rnd + k], k + 1))
            norms.append(tu.tree_l2_norm(xs[rnd + k]))
            if rnd == 2 and k == 3:
                np.testing.assert_allclose(float(norms[1]), f64norm(xs[rnd + 1]), rtol=2e-6)  # folds links 0..3
        assert all(type(v) is tu._NormView for v in norms)
        W = float(sum(range(1, K + 1)))
        mean = tu.tree_inverse_weight(s, W)
        assert H.pool_info()[0] == K  # the next round's views, made while this fold ran
        np.testing.assert_allclose([float(v) for v in norms], [f64norm(x) for x in xs[rnd:rnd + K]], rtol=2e-6)
        want = tmap(lambda s_: np.zeros(s_, np.float32), shapes)
        for k in range(K):
            want = ref.tree_add(want, ref.tree_weight(to_np(xs[rnd + k]), k + 1))
        want = ref.tree_inverse_weight(want, W)
        for a, b in zip(leaves_np(mean), pytree.leaves_of(want)):
            assert np.array_equal(bits(a), bits(b.reshape(-1)))
        if rnd == 0:
            kept = norms  # round 0's views stay referenced: their pool is never reused
        if rnd == 1:
            alias = norms[2].view(1)  # a plain tensor on round 1's norm buffer: that pool is never reused
        assert H.pool_info()[3] <= 4
    assert H.pool_info()[4] >= 1  # later rounds reused pools nobody held (rounds 2, 3, ...), never these
    np.testing.assert_allclose([float(v) for v in kept], [f64norm(x) for x in xs[:6]], rtol=2e-6)
    np.testing.assert_allclose(float(alias[0]), f64norm(xs[3]), rtol=2e-6)  # round 1, client 2
    t = {"a": xs[0]["a"].clone(), "b": {"c": xs[0]["b"]["c"].clone()}}
    s = tu.tree_add(tu.tree_zeros_like(t), tu.tree_weight(t, 1))
    t["b"] = {"c": xs[1]["b"]["c"]}  # a new inner dict: the root's version tag moved
    v = tu.tree_l2_norm(t)
    assert type(v._ticket) is H.SoloNorm  # not the chain's: a standalone lazy norm of the new contents
    np.testing.assert_allclose(float(v), f64norm({"a": xs[0]["a"], "b": {"c": xs[1]["b"]["c"]}}), rtol=2e-6)
    tu.tree_inverse_weight(s, 1.0)
    # the same dict with a leaf updated in place after tree_weight: the view is lazy, and the
    # chain's fold refuses the modified capture when the view is read (no stale value is filled)
    t = {"a": xs[0]["a"].clone(), "b": {"c": xs[0]["b"]["c"].clone()}}
    s = tu.tree_add(tu.tree_zeros_like(t), tu.tree_weight(t, 1))
    t["a"].add_(1.0)
    v = tu.tree_l2_norm(t)
    with pytest.raises(RuntimeError, match="modified"):
        float(v)
    H.drop_pool()


def test_library_loop_on_alternating_streams(cuda, sum_mode):
    """The library loop with its per-client norms (fed_avg.py:132-146), rounds alternating between
    the default stream and a side stream (the folds run on the current stream; a retired norm pool
    is reused only on the stream it was built on): after a synchronize every mean is the
    reference's bits and every norm the first round's bits (within 2e-6 of f64), including the
    views kept from earlier rounds."""
    g = torch.Generator().manual_seed(43)
    shapes = {"a": (5000,), "b": {"c": (33, 3)}}
    xs = [to_dev(rand_tree(shapes, g), cuda) for _ in range(8)]
    W = float(sum(range(1, 9)))
    want = ref.tree_zeros_like(to_np(xs[0]))
    for k, x in enumerate(xs):
        want = ref.tree_add(want, ref.tree_weight(to_np(x), k + 1))
    want = ref.tree_inverse_weight(want, W)
    f64 = [np.sqrt(sum((v.astype(np.float64) ** 2).sum() for v in leaves_np(x))) for x in xs]
    side = torch.cuda.Stream(cuda)
    first, kept = None, []
    for r in range(10):
        st = side if r % 2 else torch.cuda.current_stream(cuda)
        with torch.cuda.stream(st):
            s, norms = tu.tree_zeros_like(xs[0]), []
            for k, x in enumerate(xs):
                s = tu.tree_add(s, tu.tree_weight(x, k + 1))
                norms.append(tu.tree_l2_norm(x))
            mean = tu.tree_inverse_weight(s, W)
        st.synchronize()
        for a, b in zip(leaves_np(mean), pytree.leaves_of(want)):
            assert np.array_equal(bits(a), bits(b.reshape(-1))), r
        got = [bits(v.detach().cpu().numpy().reshape(-1)).copy() for v in norms]
        if first is None:
            first = got
            np.testing.assert_allclose([float(v) for v in norms], f64, rtol=2e-6)
        assert all(np.array_equal(a, b) for a, b in zip(got, first)), r
        if r % 3 == 0:
            kept.append(norms)
    torch.cuda.synchronize()
    for norms in kept:
        assert all(np.array_equal(bits(v.detach().cpu().numpy().reshape(-1)), b) for v, b in zip(norms, first))


def test_norm_combine_orders_give_the_same_bits(cuda):
    """The per-call fused norm with its workgroup partials handed off by the gfx950
    write-through + drain form (default) and by release/acquire atomics (FJTREE_ORDERED,
    tree_util.set_norm_combine('ordered')): the same bits, many workgroups, repeated."""
    g = torch.Generator().manual_seed(31)
    d = to_dev(rand_tree({"a": (3_000_001,), "b": (513, 7), "c": (64,)}, g), cuda)
    s = to_dev(rand_tree({"a": (3_000_001,), "b": (513, 7), "c": (64,)}, g), cuda)
    got = {}
    try:
        for mode in ("handoff", "ordered"):
            tu.set_norm_combine(mode)
            outs = []
            for _ in range(20):
                alone = tu._leaf_fold([d], [1], [None], norm_operand=0, no_out=True)[2]
                fused = tu._leaf_fold([s, d], [1, 5], [None, None], norm_operand=1)[2]
                outs.append((alone.view(torch.int32).item(), fused.view(torch.int32).item()))
            assert len(set(outs)) == 1, (mode, outs[:3])
            got[mode] = outs[0]
    finally:
        tu.set_norm_combine("handoff")
    assert got["handoff"] == got["ordered"]
    assert got["handoff"][0] == got["handoff"][1]  # fused and standalone norms of d: one order
    x64 = np.concatenate([x.astype(np.float64) for x in leaves_np(d)])
    np.testing.assert_allclose(np.int32(got["handoff"][0]).view(np.float32), np.sqrt((x64 * x64).sum()), rtol=2e-6)


def test_data_writes_bypass_the_deferred_guard_as_documented(cuda, sum_mode):
    """the deferred sum's staleness guard is torch's in-place version counter.
    A write through ``tensor.data`` does not bump it (its own counter), so — as
    set_deferred_sums / PendingSum document — a deferred fold reads the NEW values, while
    the eager path (set_deferred_sums(False)) has already summed the old ones, as the
    reference does. An ordinary in-place write is caught in deferred mode."""
    g = torch.Generator().manual_seed(41)
    h0, h1 = rand_tree({"a": (500,)}, g), rand_tree({"a": (500,)}, g)
    d = to_dev(h0, cuda)
    s = tu.tree_add(tu.tree_zeros_like(d), tu.tree_weight(d, 3))
    d["a"].data.copy_(h1["a"].to(cuda))  # bypasses d["a"]._version
    got = tu.tree_inverse_weight(s, 3.)["a"].cpu().numpy()
    old = ref.tree_inverse_weight(ref.tree_weight(to_np(h0), 3), 3.)["a"]
    new = ref.tree_inverse_weight(ref.tree_weight(to_np(h1), 3), 3.)["a"]
    want = new if sum_mode == "deferred" else old
    assert np.array_equal(bits(got), bits(want))
    # an in-place write the counter sees: deferred mode raises, eager mode kept the old value
    d2 = to_dev(h0, cuda)
    s2 = tu.tree_add(tu.tree_zeros_like(d2), tu.tree_weight(d2, 3))
    d2["a"].add_(1.0)
    if sum_mode == "deferred":
        with pytest.raises(RuntimeError, match="modified"):
            tu.tree_inverse_weight(s2, 3.)
    else:
        assert np.array_equal(bits(tu.tree_inverse_weight(s2, 3.)["a"].cpu().numpy()), bits(old))


def test_data_reassignment_is_refused_by_the_deferred_fold(cuda, sum_mode):
    """``x.data = other`` moves a captured leaf to another storage (its version counter
    need not change): the capture's data pointers (fjhost capture element 4) make the
    deferred fold raise instead of summing the other storage; eager mode has already summed
    the old value, as the reference does. The same for the running sum's base, and for a
    bf16 storage of the same element count (element-count check only)."""
    g = torch.Generator().manual_seed(43)
    h0, h1 = rand_tree({"a": (500,), "b": (7,)}, g), rand_tree({"a": (500,), "b": (7,)}, g)
    old = ref.tree_inverse_weight(ref.tree_weight(to_np(h0), 3), 3.)
    for replacement in (lambda: h1["a"].to(cuda), lambda: h1["a"].to(cuda).to(torch.bfloat16)):
        d = to_dev(h0, cuda)
        s = tu.tree_add(tu.tree_zeros_like(d), tu.tree_weight(d, 3))
        d["a"].data = replacement()
        if sum_mode == "deferred":
            with pytest.raises(RuntimeError, match="modified"):
                tu.tree_inverse_weight(s, 3.)
        else:
            got = tu.tree_inverse_weight(s, 3.)
            assert all(np.array_equal(bits(got[k].cpu().numpy()), bits(old[k])) for k in ("a", "b"))
    if sum_mode == "deferred":
        d = to_dev(h0, cuda)
        base = tu.tree_zeros_like(d)
        s = tu.tree_add(base, tu.tree_weight(d, 3))
        base["b"].data = torch.ones(7, device=cuda)
        with pytest.raises(RuntimeError, match="running sum passed to tree_add was modified"):
            tu.tree_inverse_weight(s, 3.)


@pytest.mark.deferred_only
def test_deferred_chain_budget_is_bounded_by_free_memory(cuda, sum_mode):
    """the automatic per-chain budget is min(4 GiB, free/8); a tiny explicit
    budget folds the older part of the chain early with the same bits."""
    b = tu._defer_budget(torch.device(cuda))
    free, _ = torch.cuda.mem_get_info()
    assert 64 << 20 <= b <= 4 << 30 and b <= max(64 << 20, free // 4)
    g = torch.Generator().manual_seed(42)
    hs = [rand_tree({"a": (4096,)}, g) for _ in range(9)]
    ds = [to_dev(h, cuda) for h in hs]
    try:
        tu.set_deferred_sums(True, budget_bytes=3 * 4096 * 4)  # at most 3 deltas per fold
        s = tu.tree_zeros_like(ds[0])
        for k, d in enumerate(ds):
            s = tu.tree_add(s, tu.tree_weight(d, k + 1))
        assert type(s) is tu.PendingSum and s._n <= 3
        got = tu.tree_inverse_weight(s, 45.)["a"].cpu().numpy()
    finally:
        tu.set_deferred_sums(True, budget_bytes=0)
    want = tmap(lambda x: np.zeros(x.shape, np.float32), to_np(hs[0]))
    for k, h in enumerate(hs):
        want = ref.tree_add(want, ref.tree_weight(to_np(h), k + 1))
    assert np.array_equal(bits(got), bits(ref.tree_inverse_weight(want, 45.)["a"]))


@pytest.mark.deferred_only
def test_early_flush_of_the_running_sum(cuda, sum_mode):
    """The deferred chain folds its pending part once it holds flush_bytes in flush_clients
    links (set_deferred_sums): the literal loop with the per-client norm of fed_avg.py:
    137-144 keeps the reference's bits for the mean, and each norm is the same value the
    one-launch chain gives."""
    g = torch.Generator().manual_seed(23)
    shapes = {"w": (3000,), "b": {"c": (17,)}}
    K = 23
    xs = [to_dev(rand_tree(shapes, g), cuda) for _ in range(K)]
    ws = [int(v) for v in np.random.RandomState(4).randint(1, 50, size=K)]

    def loop():
        s, norms, chains = tu.tree_zeros_like(xs[0]), [], set()
        for x, w in zip(xs, ws):
            s = tu.tree_add(s, tu.tree_weight(x, w))
            norms.append(tu.tree_l2_norm(x))
            chains.add(id(s._chain))
        # an early flush keeps the run's chain (its norm buffer serves the next links)
        assert len(chains) == 1
        mean = tu.tree_inverse_weight(s, float(sum(ws)))
        return leaves_np(mean), [float(n) for n in norms]

    base_mean, base_norms = loop()  # defaults: one fold (23 small clients < 1 GiB)
    acc = tmap(lambda s: np.zeros(s, np.float32), shapes)
    for x, w in zip(xs, ws):
        acc = ref.tree_add(acc, ref.tree_weight(to_np(x), w))
    want = [a.reshape(-1) for a in pytree.leaves_of(ref.tree_inverse_weight(acc, float(sum(ws))))]
    for a, b in zip(base_mean, want):
        assert np.array_equal(bits(a), bits(b))
    for fb, fc in [(1, 1), (12_100 * 3, 2), (40_000, 5)]:
        tu.set_deferred_sums(True, flush_bytes=fb, flush_clients=fc)
        try:
            mean, norms = loop()
        finally:
            tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)
        for a, b in zip(mean, want):
            assert np.array_equal(bits(a), bits(b)), (fb, fc)
        n64 = [float(np.sqrt(sum(float(np.dot(v.astype(np.float64), v.astype(np.float64)))
                                 for v in leaves_np(x)))) for x in xs]
        np.testing.assert_allclose(norms, n64, rtol=2e-6)


@pytest.mark.deferred_only
def test_native_chain_fold_equals_python_path(cuda, sum_mode, monkeypatch):
    """A deferred sum's fold through fjhost.fold_caps (one native call) against the Python
    path (_FOLD_CAPS off): the literal loop's mean and lazy norms bitwise, with early
    flushes (several folds per round), a nested / list / None structure, and the stale
    errors (base and client) raised the same way."""
    g = torch.Generator().manual_seed(21)
    shapes = {"z": [(70,), None, ((3,), (5, 2))], "a": {"q": (8,), "p": (1001,)}}

    def dev_tree(t):
        if isinstance(t, dict):
            return {k: dev_tree(v) for k, v in t.items()}
        if isinstance(t, list):
            return [dev_tree(v) for v in t]
        if isinstance(t, tuple) and t and not isinstance(t[0], int):
            return tuple(dev_tree(v) for v in t)
        if t is None:
            return None
        return (torch.rand(t, generator=g) - 0.5).to(cuda)

    K = 37
    deltas = [dev_tree(shapes) for _ in range(K)]
    weights = [1 + (k % 9) for k in range(K)]
    weights[4] = 0.75
    params = tu.tree_zeros_like(deltas[0])

    def run(native, flush):
        monkeypatch.setattr(tu, "_FOLD_CAPS", native)
        tu.set_deferred_sums(True, flush_bytes=flush, flush_clients=4)
        try:
            mean, norms = literal_loop(tu, params, deltas, weights)
            return [x.cpu() for x in pytree.leaves_of(mean)], torch.stack(norms).cpu(), ref.flatten(mean)[1]
        finally:
            tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)

    want, want_n, want_td = run(False, 1 << 30)
    for flush in (1 << 30, 20_000):  # one fold per round / a fold every ~5 clients
        got, got_n, got_td = run(True, flush)
        assert got_td == want_td
        for a, b in zip(got, want):
            assert torch.equal(a.view(torch.int32), b.view(torch.int32))
        assert torch.equal(got_n.view(torch.int32), want_n.view(torch.int32))
    monkeypatch.setattr(tu, "_FOLD_CAPS", True)
    s = tu.tree_add(tu.tree_zeros_like(deltas[0]), tu.tree_weight(deltas[1], 2))
    s = tu.tree_add(s, tu.tree_weight(deltas[2], 3))
    deltas[2]["a"]["q"].add_(1.0)
    with pytest.raises(RuntimeError, match="client 1 of a pending tree_add sum was modified"):
        s.materialize()
    base = tu.tree_zeros_like(deltas[0])
    s = tu.tree_add(base, tu.tree_weight(deltas[3], 2))
    base["a"]["p"].add_(1.0)
    with pytest.raises(RuntimeError, match="running sum passed to tree_add was modified"):
        tu.tree_inverse_weight(s, 2.0)


def test_tree_zeros_like_one_allocation_own_leaves(cuda, sum_mode):
    """tree_zeros_like of a float32 device pytree (fjhost.zeros_like): zeros of every leaf's
    shape, dict keys sorted as jax.tree.map builds them, one storage, 256-byte aligned
    disjoint slices, and each leaf its own tensor: an in-place write to one leaf bumps only
    its own version counter (views shared one counter)."""
    tree = {"z": torch.ones(5, 3, device=cuda), "a": [torch.ones(1001, device=cuda), None,
                                                       (torch.ones((), device=cuda),)]}
    z = tu.tree_zeros_like(tree)
    assert list(z) == ["a", "z"]
    leaves = pytree.leaves_of(z)
    src = pytree.leaves_of(tree)
    assert [x.shape for x in leaves] == [x.shape for x in src]
    assert all(x.dtype == torch.float32 and x.device == src[0].device and x.is_contiguous() for x in leaves)
    assert all(not x.any().item() for x in leaves)
    assert z["a"][1] is None and isinstance(z["a"][2], tuple)
    assert len({x.untyped_storage().data_ptr() for x in leaves}) == 1
    ptrs = sorted((x.data_ptr(), x.numel() * 4) for x in leaves)
    assert all(p % 256 == 0 for p, _ in ptrs)
    assert all(p0 + n0 <= p1 for (p0, n0), (p1, _) in zip(ptrs, ptrs[1:]))
    v = [x._version for x in leaves]
    leaves[0].add_(1.0)
    assert [x._version for x in leaves][1:] == v[1:] and leaves[0]._version > v[0]
    assert all(not x.any().item() for x in leaves[1:])
    # a running sum on that base is still guarded per leaf: modifying a sibling after
    # tree_add does not make the fold raise, modifying the base leaf in place does
    d = {"a": [torch.full((1001,), 2.0, device=cuda), None, (torch.full((), 2.0, device=cuda),)],
         "z": torch.full((5, 3), 2.0, device=cuda)}
    base = tu.tree_zeros_like(d)
    s = tu.tree_add(base, tu.tree_weight(d, 3))
    other = tu.tree_zeros_like(d)
    other["z"].add_(1.0)
    assert float(tu.tree_inverse_weight(s, 3.0)["z"][0, 0]) == 2.0
    if sum_mode == "deferred":  # (eager: tree_add has already read the base)
        base2 = tu.tree_zeros_like(d)
        s2 = tu.tree_add(base2, tu.tree_weight(d, 3))
        base2["z"].add_(1.0)
        with pytest.raises(RuntimeError, match="running sum passed to tree_add was modified"):
            tu.tree_inverse_weight(s2, 3.0)


_LOOP_SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
from fedjax_amd import kernels, tree_util as tu
dev = torch.device("cuda:0")
shapes = {{"a": (300,), "b": (64, 33), "c": (1000,)}}
deltas = []
for k in range(80):
    t = {{}}
    for i, (name, shp) in enumerate(shapes.items()):
        x = torch.empty(1, int(np.prod(shp)), device=dev)
        kernels.fill_synth(x, seed=i + 1, k0=k)
        t[name] = x.view(shp)
    deltas.append(t)
s, norms = tu.tree_zeros_like(deltas[0]), []
tu.set_deferred_sums(True, max_clients=4095, flush_bytes=1, flush_clients=32)
for k, d in enumerate(deltas):
    s = tu.tree_add(s, tu.tree_weight(d, k + 1))
    norms.append(tu.tree_l2_norm(d))
m = tu.tree_inverse_weight(s, float(sum(range(1, 81))))
print(np.array([float(n) for n in norms], dtype=np.float32).view(np.uint32).tolist())
print(torch.cat([m[k].reshape(-1) for k in sorted(m)]).view(torch.int32).sum().item())
"""


@pytest.mark.deferred_only
def test_library_loop_norms_with_and_without_the_combine_launch(cuda):
    """The library loop's lazy norms come from the chain folds' combine, in the fold's last
    workgroup by default; FJAGG_L2_COMBINE_LAUNCH=1 (read once per process by fjhost) keeps the
    separate combine launch. A child process with the switch and one without: the same norm bits
    and the same mean (early flushes every 32 clients, 80 clients)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = _LOOP_SCRIPT.format(root=root)
    outs = []
    for switch in ("0", "1"):
        env = dict(os.environ, FJAGG_L2_COMBINE_LAUNCH=switch)
        r = subprocess.run([sys.executable, "-c", script], env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout.strip().splitlines()[-2:])
    assert outs[0] == outs[1]


def test_lazy_sums_pickle_and_copy_as_pytrees(cuda, sum_mode):
    """tree_weight's result and a running sum mid-loop pickle, deepcopy and copy as the pytrees
    they stand for (plain dicts of tensors, the reference's values); the loop then goes on from
    the original and ends with the reference's bits."""
    import copy
    import pickle
    g = torch.Generator().manual_seed(47)
    shapes = {"a": (5000,), "b": {"c": (33, 3)}}
    xs = [to_dev(rand_tree(shapes, g), cuda) for _ in range(3)]
    wt = tu.tree_weight(xs[0], 3)
    s = tu.tree_zeros_like(xs[0])
    s = tu.tree_add(s, tu.tree_weight(xs[0], 1))
    s = tu.tree_add(s, tu.tree_weight(xs[1], 2))
    want_w = ref.tree_weight(to_np(xs[0]), 3)
    want_s = ref.tree_add(ref.tree_add(ref.tree_zeros_like(to_np(xs[0])), ref.tree_weight(to_np(xs[0]), 1)),
                          ref.tree_weight(to_np(xs[1]), 2))
    for obj, want in ((wt, want_w), (s, want_s)):
        for got in (pickle.loads(pickle.dumps(obj)), copy.deepcopy(obj), copy.copy(obj)):
            assert type(got) is dict
            for a, b in zip(leaves_np(got), pytree.leaves_of(want)):
                assert np.array_equal(bits(a), bits(b.reshape(-1)))
    s = tu.tree_add(s, tu.tree_weight(xs[2], 3))
    mean = tu.tree_inverse_weight(s, 6.0)
    want = ref.tree_inverse_weight(ref.tree_add(want_s, ref.tree_weight(to_np(xs[2]), 3)), 6.0)
    for a, b in zip(leaves_np(mean), pytree.leaves_of(want)):
        assert np.array_equal(bits(a), bits(b.reshape(-1)))
