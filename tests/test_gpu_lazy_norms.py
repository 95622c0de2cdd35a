"""Standalone lazy norms (fjhost.cpp "standalone lazy norms", tree_util.set_lazy_norms): the
round of examples/fed_avg.py:72-82 as written —

    for each client: deltas.append((delta, n)); diag[cid] = tree_l2_norm(delta)
    mean = tree_mean(deltas)

— reads every delta once: each norm is a lazy view that the tree_mean launch folding the same,
unmodified delta fills (fjagg_wsum_l2_ptrs_rows). The mean stays the oracle's bits; a norm's
value must not depend on when it is computed (in the mean's launch, read first, past the
pending budget, with other clients or alone): the same bits every way, within f32 rounding of
an f64 norm (XLA's own reduction order is not pinned, tree_util.py:105-114). A delta updated in
place after its norm makes the view raise; a replaced leaf keeps the captured value.
"""
import gc
import weakref

import numpy as np
import pytest
import torch

import fedjax_amd
from fedjax_amd import pytree, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu

EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
SMALL = {"a": (5003,), "b": {"c": (33, 3)}}
H = tu._HOST


@pytest.fixture(autouse=True)
def lazy_on():
    tu.set_deferred_sums(True)
    tu.set_lazy_norms(True, budget_bytes=0)
    yield
    H.solo_resolve(None)
    tu.set_lazy_norms(True, budget_bytes=0, max_pending=16383)


def tmap(fn, t):
    return {k: tmap(fn, v) for k, v in t.items()} if isinstance(t, dict) else fn(t)


def make_deltas(shapes, K, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    return [tmap(lambda s: (torch.rand(s, device=dev, generator=g) - 0.5) * 0.02, shapes) for _ in range(K)]


def bits(t):
    return t.detach().reshape(-1).view(torch.int32).cpu()


def f64norm(t):
    x = np.concatenate([v.detach().cpu().numpy().astype(np.float64).reshape(-1) for v in pytree.leaves_of(t)])
    return float(np.sqrt((x * x).sum()))


def example_round(deltas, weights, read_at=()):
    """examples/fed_avg.py:72-82 with the clients' updates already made."""
    client_diagnostics = {}
    client_delta_params_weights = []
    for cid, (delta_params, n) in enumerate(zip(deltas, weights)):
        client_delta_params_weights.append((delta_params, n))
        client_diagnostics[cid] = {"delta_l2_norm": tu.tree_l2_norm(delta_params)}
        if cid in read_at:
            float(client_diagnostics[cid]["delta_l2_norm"])  # a read before the mean
    mean = tu.tree_mean(client_delta_params_weights)
    return mean, [client_diagnostics[c]["delta_l2_norm"] for c in range(len(deltas))]


def want_mean(deltas, weights):
    return ref.tree_mean([(tmap(lambda x: x.cpu().numpy(), d), n) for d, n in zip(deltas, weights)])


def same_mean(got, want):
    return all(np.array_equal(a.cpu().numpy().reshape(-1).view(np.uint32), np.asarray(b).reshape(-1).view(np.uint32))
               for a, b in zip(pytree.leaves_of(got), pytree.leaves_of(want)))


@pytest.mark.parametrize("K", [10, 128])
def test_example_round_fuses_the_norms_into_the_mean(cuda, K):
    deltas = make_deltas(EMNIST, K, 1, cuda)
    weights = [int(v) for v in ref.fedavg_weights(K, seed=2)]
    before = H.solo_info()
    mean, norms = example_round(deltas, weights)
    info = H.solo_info()
    assert info["fused"] - before["fused"] == K  # every norm came from the mean's launches
    assert info["eager"] == before["eager"] and info["pending"] == 0
    assert all(type(v) is tu._NormView and v._ticket.node is None for v in norms)
    assert same_mean(mean, want_mean(deltas, weights))
    np.testing.assert_allclose([float(v) for v in norms], [f64norm(d) for d in deltas], rtol=2e-6)
    # each norm computed on its own (read before any mean): the same bits
    alone = []
    for d in deltas:
        v = tu.tree_l2_norm(d)
        assert type(v._ticket) is H.SoloNorm and v._ticket.node is not None
        alone.append(bits(v).clone())  # (the read computes it: one launch)
    assert H.solo_info()["eager"] - info["eager"] == K
    for v, a in zip(norms, alone):
        assert torch.equal(bits(v), a)
    # squared norms share the node of the norm taken just before
    d = deltas[0]
    n, q = tu.tree_l2_norm(d), tu.tree_l2_squared(d)
    assert n._ticket is q._ticket
    tu.tree_mean([(d, 1), (deltas[1], 2)])
    assert float(q) == pytest.approx(float(n) ** 2, rel=1e-6)


def test_read_before_mean_and_partial_rounds(cuda):
    """Reading some norms mid-loop computes just those; the rest fuse into the mean. Values
    equal the all-fused round's bits; the mean is unchanged."""
    K = 40
    deltas = make_deltas(SMALL, K, 3, cuda)
    weights = [k % 7 + 1 for k in range(K)]
    mean0, norms0 = example_round(deltas, weights)
    ref0 = [bits(v).clone() for v in norms0]
    before = H.solo_info()
    mean1, norms1 = example_round(deltas, weights, read_at=(0, 3, 17, 39))
    info = H.solo_info()
    assert info["eager"] - before["eager"] == 4 and info["fused"] - before["fused"] == K - 4
    assert all(torch.equal(bits(v), r) for v, r in zip(norms1, ref0))
    assert all(torch.equal(a, b) for a, b in zip(pytree.leaves_of(mean0), pytree.leaves_of(mean1)))
    # norms of a subset of the mean's clients: a run of matched clients, then plain folds
    norms2 = [tu.tree_l2_norm(d) for d in deltas[:5]]
    mean2 = tu.tree_mean(list(zip(deltas, weights)))
    assert all(v._ticket.node is None for v in norms2)
    assert all(torch.equal(bits(v), r) for v, r in zip(norms2, ref0[:5]))
    assert all(torch.equal(a, b) for a, b in zip(pytree.leaves_of(mean0), pytree.leaves_of(mean2)))


def test_modified_and_replaced_leaves(cuda):
    deltas = make_deltas(SMALL, 6, 4, cuda)
    want = [f64norm(d) for d in deltas]
    norms = [tu.tree_l2_norm(d) for d in deltas]
    deltas[2]["a"].mul_(2.0)  # in place after the norm: the value at the call is gone
    deltas[4]["b"] = {"c": torch.zeros(33, 3, device=cuda)}  # replaced: the captured leaves hold the value
    mean = tu.tree_mean([(d, 1) for d in deltas])  # (the mean folds the current values, as always)
    assert same_mean(mean, want_mean(deltas, [1] * 6))
    with pytest.raises(RuntimeError, match="modified"):
        float(norms[2])
    with pytest.raises(RuntimeError, match="modified"):
        torch.stack(norms)
    ok = [0, 1, 3, 4, 5]
    np.testing.assert_allclose([float(norms[k]) for k in ok], [want[k] for k in ok], rtol=2e-6)
    assert norms[4]._ticket.node is None


@pytest.mark.parametrize("form", ["iterator", "generator", "aggregator"])
def test_one_shot_iterables_fuse(cuda, form):
    K = 12
    deltas = make_deltas(SMALL, K, 5, cuda)
    weights = [k + 1 for k in range(K)]
    norms = [tu.tree_l2_norm(d) for d in deltas]
    before = H.solo_info()
    if form == "iterator":
        mean = tu.tree_mean(iter(list(zip(deltas, weights))))
    elif form == "generator":
        mean = tu.tree_mean((d, w) for d, w in zip(deltas, weights))
    else:
        agg = fedjax_amd.aggregators.mean_aggregator()
        state = agg.init()
        mean, _ = agg.apply(iter([(str(k), d, w) for k, (d, w) in enumerate(zip(deltas, weights))]), state)
    assert H.solo_info()["fused"] - before["fused"] == K
    assert same_mean(mean, want_mean(deltas, weights))
    np.testing.assert_allclose([float(v) for v in norms], [f64norm(d) for d in deltas], rtol=2e-6)


def test_dropped_views_release_the_deltas(cuda):
    d = make_deltas(SMALL, 1, 6, cuda)[0]
    leaf = weakref.ref(d["a"])
    v = tu.tree_l2_norm(d)
    node = weakref.ref(v._ticket)
    assert H.solo_info()["pending"] == 1
    del d
    gc.collect()
    assert leaf() is not None  # the pending view holds the captured leaves
    del v
    gc.collect()
    # (a pool view's node lets its capture go when the pool next looks: any mean, the budget, solo_info)
    assert H.solo_info()["pending"] == 0
    gc.collect()
    assert leaf() is None


def test_budget_computes_the_deltas_only_views_hold(cuda):
    """Past the byte budget the norms whose pytree nobody else holds are computed; the ones
    whose pytree the caller still holds wait for the mean. Same bits either way."""
    deltas = make_deltas(SMALL, 8, 7, cuda)
    ref_bits = [bits(tu.tree_l2_norm(d)).clone() for d in deltas]
    per = 4 * (5003 + 99)
    tu.set_lazy_norms(True, budget_bytes=3 * per)
    before = H.solo_info()
    held = [tu.tree_l2_norm(d) for d in deltas]  # the caller holds every delta: all wait
    assert H.solo_info()["pending"] == 8
    tu.tree_mean([(d, 1) for d in deltas])
    assert H.solo_info()["fused"] - before["fused"] == 8
    orphans = []
    src = make_deltas(SMALL, 8, 7, cuda)
    for k in range(8):  # copies of the same values; nobody else keeps these trees
        orphans.append(tu.tree_l2_norm(tmap(lambda x: x.clone(), src[k])))
    assert H.solo_info()["pending"] <= 4 and H.solo_info()["eager"] > before["eager"]
    for v, r in zip(held + orphans, ref_bits + ref_bits):
        assert torch.equal(bits(v), r)
    tu.set_lazy_norms(True, max_pending=3)
    vs = [tu.tree_l2_norm(d) for d in deltas]
    assert H.solo_info()["pending"] <= 3
    assert all(torch.equal(bits(v), r) for v, r in zip(vs, ref_bits))


def test_misaligned_delta_is_computed_alone(cuda):
    """A leaf off 16 bytes walks element units: its client's chunk folds plainly and every
    norm of it is computed by its own launch (its own plan); the aligned clients' norms keep
    the all-16-byte plan's bits."""
    deltas = make_deltas(SMALL, 5, 8, cuda)
    ref_bits = [bits(tu.tree_l2_norm(d)).clone() for d in deltas]
    base = torch.empty(5004, device=cuda)
    odd = {"a": base[1:], "b": {"c": deltas[2]["b"]["c"]}}
    odd["a"].copy_(deltas[2]["a"])
    trees = deltas[:2] + [odd] + deltas[3:]
    norms = [tu.tree_l2_norm(d) for d in trees]
    mean = tu.tree_mean([(d, 3) for d in trees])
    assert same_mean(mean, want_mean(trees, [3] * 5))
    for k in (0, 1, 3, 4):
        assert torch.equal(bits(norms[k]), ref_bits[k])
    assert float(norms[2]) == pytest.approx(f64norm(odd), rel=2e-6)


def test_buffer_boundary_splits_the_run(cuda):
    """Norms of one round that straddle two norm buffers fold in two runs, all fused. (Squared
    norms take fresh columns in call order; the norms' pre-made pool pairs come in runs of their
    own, tested above.)"""
    deltas = make_deltas(SMALL, 16, 9, cuda)
    col = H.solo_info()["column"] % 4096
    junk = [tu.tree_l2_squared({"a": torch.ones(4, device=cuda)}) for _ in range((4090 - col) % 4096)]
    del junk
    gc.collect()
    assert H.solo_info()["column"] == 4090
    before = H.solo_info()
    sq = [tu.tree_l2_squared(d) for d in deltas]
    mean = tu.tree_mean([(d, k + 1) for k, d in enumerate(deltas)])
    assert H.solo_info()["fused"] - before["fused"] == 16
    assert len({v._ticket._buf.data_ptr() for v in sq}) == 2  # the run crossed into a new buffer
    np.testing.assert_allclose([float(v) for v in sq], [f64norm(d) ** 2 for d in deltas], rtol=4e-6)
    assert same_mean(mean, want_mean(deltas, list(range(1, 17))))


def test_switch_off_is_eager(cuda):
    d = make_deltas(SMALL, 1, 10, cuda)[0]
    tu.set_lazy_norms(False)
    v = tu.tree_l2_norm(d)
    assert type(v) is not tu._NormView
    tu.set_lazy_norms(True)
    tu.set_deferred_sums(False)
    try:
        assert type(tu.tree_l2_norm(d)) is not tu._NormView
    finally:
        tu.set_deferred_sums(True)
    assert float(v) == pytest.approx(f64norm(d), rel=2e-6)


def test_pool_pairs_are_reused_once_dropped(cuda):
    """After a mean that fused lazy norms, the next round's (view, node) pairs are pre-made; a
    full buffer whose views the caller dropped is reused whole; values stay the fused bits."""
    deltas = make_deltas(SMALL, 64, 11, cuda)
    ref_bits = [bits(tu.tree_l2_norm(d)).clone() for d in deltas]
    example_round(deltas, list(range(1, 65)))  # asks for 64 norms: the pool is sized to that
    assert H.solo_info()["pool_ready"] >= 64
    kept = None
    for rnd in range(80):  # > 4096 columns: buffers fill, the dropped ones come back
        mean, norms = example_round(deltas, list(range(1, 65)))
        if rnd == 3:
            kept = norms  # held: that buffer is never reused
        if rnd % 20 == 0:
            assert all(torch.equal(bits(v), r) for v, r in zip(norms, ref_bits))
    info = H.solo_info()
    assert info["pool_reuses"] >= 1
    assert all(torch.equal(bits(v), r) for v, r in zip(kept, ref_bits))
    assert all(torch.equal(bits(v), r) for v, r in zip(norms, ref_bits))


def test_a_second_view_keeps_the_capture(cuda):
    """tree_l2_norm and tree_l2_squared of one delta share a node: dropping the first view while
    the second is held keeps the capture, and the second reads the right value."""
    d = make_deltas(SMALL, 1, 12, cuda)[0]
    want = f64norm(d)
    n = tu.tree_l2_norm(d)
    q = tu.tree_l2_squared(d)
    assert n._ticket is q._ticket
    del n
    gc.collect()
    H.solo_info()  # (the registry looks at the views)
    assert q._ticket.node is not None and H.solo_info()["pending"] == 1
    assert float(q) == pytest.approx(want ** 2, rel=4e-6)


def test_deltas_with_autograd_history(cuda):
    """Deltas computed from trained parameters outside torch.no_grad carry autograd history
    (requires_grad, a grad_fn), as `server_p - client_p` of nn.Parameters does. The example
    round (fed_avg.py:72-82), the library's running sum (algorithms/fed_avg.py:132-146) and the
    aggregator read their values: the oracle's mean bits and the f64 norms, as for plain deltas.
    Results carry no autograd history: the server never differentiates its aggregation."""
    K = 6
    base = make_deltas(SMALL, K, 7, cuda)
    deltas = [tmap(lambda x: x.clone().requires_grad_(True) * 1.0, d) for d in base]  # same values
    assert all(x.requires_grad and x.grad_fn is not None for d in deltas for x in pytree.leaves_of(d))
    weights = [3, 1, 4, 1, 5, 9]
    want = want_mean(base, weights)
    before = H.solo_info()["fused"]
    mean, norms = example_round(deltas, weights)
    assert H.solo_info()["fused"] - before == K
    assert same_mean(mean, want)  # (.numpy() would raise on a result that requires grad)
    np.testing.assert_allclose([float(v) for v in norms], [f64norm(d) for d in base], rtol=2e-6)
    s = tu.tree_zeros_like(deltas[0])
    for d, n in zip(deltas, weights):
        s = tu.tree_add(s, tu.tree_weight(d, n))
    got = tu.tree_inverse_weight(s, float(sum(weights)))
    s_ref = ref.tree_zeros_like(tmap(lambda x: x.cpu().numpy(), base[0]))
    for d, n in zip(base, weights):
        s_ref = ref.tree_add(s_ref, ref.tree_weight(tmap(lambda x: x.cpu().numpy(), d), n))
    assert same_mean(got, ref.tree_inverse_weight(s_ref, float(sum(weights))))
    agg = fedjax_amd.aggregators.mean_aggregator()
    m2, _ = agg.apply([(str(i), d, w) for i, (d, w) in enumerate(zip(deltas, weights))], agg.init())
    assert same_mean(m2, want)
    assert not any(x.requires_grad for t in (mean, got, m2) for x in pytree.leaves_of(t))


def test_a_delta_twice_in_one_mean_and_two_views_of_one_tree(cuda):
    """A client delta listed twice in one tree_mean (a client sampled twice), and a tree normed
    twice with another norm in between (two pending nodes of one tree): the mean is the oracle's
    bits and every view the bits of its delta's norm computed alone, whichever node the mean
    fills and whichever is computed on its own."""
    d = make_deltas(SMALL, 3, 11, cuda)
    alone = []
    for x in d:
        alone.append(bits(tu.tree_l2_norm(x)).clone())
        tu.tree_mean([(x, 1)])  # (computes it; the mean does not change the value)
    v0 = tu.tree_l2_norm(d[0])
    v1 = tu.tree_l2_norm(d[1])
    v0b = tu.tree_l2_norm(d[0])  # a second node of d[0] (v1's node sits in between)
    v2 = tu.tree_l2_norm(d[2])
    pairs = [(d[0], 2), (d[1], 3), (d[0], 5), (d[2], 7), (d[1], 1)]
    mean = tu.tree_mean(pairs)
    assert same_mean(mean, ref.tree_mean([(tmap(lambda x: x.cpu().numpy(), t), w) for t, w in pairs]))
    for v, i in ((v0, 0), (v1, 1), (v0b, 0), (v2, 2)):
        assert torch.equal(bits(v), alone[i]), i
    assert H.solo_info()["pending"] == 0


def test_many_rounds_hold_no_growing_state(cuda):
    """300 example rounds of 10 clients, each round's diagnostics dropped when the next one
    starts, as a training loop does: the registry keeps nothing pending, the norm buffers stay
    within their bound and the device memory in use returns to where it started."""
    deltas = make_deltas(SMALL, 10, 13, cuda)
    weights = list(range(1, 11))
    mean, norms = example_round(deltas, weights)  # (the first round builds the pool and its buffers)
    del mean, norms
    torch.cuda.synchronize()
    start = torch.cuda.memory_allocated(cuda)
    for _ in range(300):
        mean, norms = example_round(deltas, weights)
        float(norms[-1])
    del mean, norms
    torch.cuda.synchronize()
    info = H.solo_info()
    assert info["pending"] == 0 and info["registry"] <= 64
    assert info["buffers"] <= 6
    assert torch.cuda.memory_allocated(cuda) <= start + 2 * 2 * 4096 * 4  # (at most the next buffers' columns)


def test_rounds_on_alternating_streams(cuda):
    """Example rounds that alternate between the default stream and a side stream (the mean and
    its norms run on the current stream; a pooled buffer is reused only on the stream it was
    written on): after a synchronize every view holds the bits of its delta's norm alone and
    every mean the oracle's."""
    deltas = make_deltas(SMALL, 8, 17, cuda)
    weights = [2, 7, 1, 8, 2, 8, 1, 8]
    alone = [bits(tu.tree_l2_norm(d)).clone() for d in deltas]
    want = want_mean(deltas, weights)
    side = torch.cuda.Stream(cuda)
    kept = []
    for r in range(12):
        stream = side if r % 2 else torch.cuda.current_stream(cuda)
        with torch.cuda.stream(stream):
            mean, norms = example_round(deltas, weights)
        stream.synchronize()
        assert same_mean(mean, want), r
        for v, a in zip(norms, alone):
            assert torch.equal(bits(v), a), r
        if r % 3 == 0:
            kept.append(norms)  # (some rounds' views stay alive: their buffers cannot be reused)
    torch.cuda.synchronize()
    for norms in kept:
        for v, a in zip(norms, alone):
            assert torch.equal(bits(v), a)


@pytest.mark.parametrize("kind", ["example", "library"])
def test_norm_views_pickle_and_copy_as_values(cuda, kind):
    """Client diagnostics travel (pickle to a logging process, torch.save with a checkpoint,
    copy.deepcopy): a lazy norm view pickles and copies as its value, a plain 0-d float32
    tensor of its own, as the reference's jnp scalar does (computed first when still pending).
    Both the standalone norms of examples/fed_avg.py and the running sum's norms."""
    import copy
    import io
    import pickle
    xs = make_deltas(SMALL, 4, 19, cuda)
    if kind == "example":
        diag = {i: {"delta_l2_norm": tu.tree_l2_norm(x)} for i, x in enumerate(xs)}
        pending = copy.deepcopy(diag[3])  # (before any mean: computed on its own)
        tu.tree_mean([(x, 1) for x in xs])
    else:
        s, diag = tu.tree_zeros_like(xs[0]), {}
        for i, x in enumerate(xs):
            s = tu.tree_add(s, tu.tree_weight(x, i + 1))
            diag[i] = {"delta_l2_norm": tu.tree_l2_norm(x)}
        pending = copy.deepcopy(diag[3])  # (before the fold: the chain folds first)
        tu.tree_inverse_weight(s, 10.0)
    want = [bits(diag[i]["delta_l2_norm"]) for i in range(4)]
    buf = io.BytesIO()
    torch.save(diag, buf)
    for got in (pickle.loads(pickle.dumps(diag)), torch.load(io.BytesIO(buf.getvalue()), weights_only=True),
                copy.deepcopy(diag), {k: copy.copy(v["delta_l2_norm"]) for k, v in diag.items()}):
        for i in range(4):
            v = got[i]["delta_l2_norm"] if isinstance(got[i], dict) else got[i]
            assert type(v) is torch.Tensor and v.dim() == 0 and v.dtype == torch.float32
            assert v.untyped_storage().nbytes() == 4  # (its own value, not the norm buffer)
            assert torch.equal(bits(v), want[i])
    assert type(pending["delta_l2_norm"]) is torch.Tensor and torch.equal(bits(pending["delta_l2_norm"]), want[3])


def test_a_generator_that_raises_mid_mean(cuda):
    """tree_mean over a one-shot iterable that raises partway (a client's data failed to load):
    the caller gets the generator's exception; every norm view taken before still reads its
    delta's bits (the launched chunk's clients stay pending and are computed alone on read), and
    the next round fuses as usual."""
    deltas = make_deltas(EMNIST, 40, 23, cuda)
    alone = [bits(tu.tree_l2_norm(d)).clone() for d in deltas]
    views = [tu.tree_l2_norm(d) for d in deltas]

    def pairs():
        for i, d in enumerate(deltas):
            if i == 30:
                raise ValueError("client 30 failed")
            yield d, i + 1

    with pytest.raises(ValueError, match="client 30 failed"):
        tu.tree_mean(pairs())
    for v, a in zip(views, alone):
        assert torch.equal(bits(v), a)
    before = H.solo_info()["fused"]
    weights = list(range(1, 41))
    mean, norms = example_round(deltas, weights)
    assert H.solo_info()["fused"] - before == 40
    assert same_mean(mean, want_mean(deltas, weights))
    for v, a in zip(norms, alone):
        assert torch.equal(bits(v), a)
