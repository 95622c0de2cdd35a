"""Fused server step: ignore_grads_haiku and learning-rate schedules.

* ``ignore_grads_haiku`` (fedjax/core/optimizers.py:69-109) is pinned by the reference's own
  known-answer test, fedjax/core/optimizers_test.py:28-56: sgd(1.0) over grads of 0.5 with
  ('linear_1', 'w') and ('linear_2', 'b') frozen leaves linear_2/w at 1.5 and the frozen
  leaves at their values. Here the "grads" are the round's mean delta (the server step of
  fedjax/algorithms/fed_avg.py:150-154), on the pytree path and the slab path.
* A frozen leaf's optimizer state passes through untouched too (its leaf gets no
  workgroups); trainable leaves stay bitwise the numpy restatement of optax.
* A schedule (ScalarOrSchedule, optimizers.py:114) is evaluated at optax's pre-increment
  count (optax.scale_by_schedule); the steps are bitwise the restatement with that lr.
"""
import numpy as np
import numpy.testing as npt
import pytest
import torch

import fedjax_amd
from fedjax_amd import server
from oracle import tree_util_ref as ref
from tests.test_gpu_parity import _np_server_step, bits, host

pytestmark = pytest.mark.gpu


def haiku_params(dev):
    return {"linear_1": {"w": torch.tensor([1., 1., 1.], device=dev)},
            "linear_2": {"w": torch.tensor([2., 2., 2.], device=dev), "b": torch.tensor([3., 3., 3.], device=dev)}}


def test_ignore_grads_haiku_kat_pytree_path(cuda):
    """optimizers_test.py:28-56 through fused_tree_mean_update (one client, delta 0.5)."""
    params = haiku_params(cuda)
    grads = {m: {n: torch.full_like(x, 0.5) for n, x in sub.items()} for m, sub in params.items()}
    opt = server.ignore_grads_haiku(server.sgd(learning_rate=1.0), [("linear_1", "w"), ("linear_2", "b")])
    state = opt.init(params)
    mean_out = {m: {n: torch.empty_like(x) for n, x in sub.items()} for m, sub in params.items()}
    state = server.fused_tree_mean_update([(grads, 1)], opt, params, state, mean_out=mean_out)
    npt.assert_array_equal(host(params["linear_1"]["w"]), [1., 1., 1.])
    npt.assert_array_equal(host(params["linear_2"]["w"]), [1.5, 1.5, 1.5])
    npt.assert_array_equal(host(params["linear_2"]["b"]), [3., 3., 3.])
    for sub in mean_out.values():  # the mean of every leaf, frozen ones included
        for x in sub.values():
            npt.assert_array_equal(host(x), [0.5, 0.5, 0.5])
    assert state["count"] == 1


def test_ignore_grads_haiku_kat_slab_path(cuda):
    """The same KAT through fused_mean_update on a ClientDeltaSlab (frozen leaves are
    column ranges of the slab)."""
    template = {"linear_1": {"w": np.zeros(3, np.float32)},
                "linear_2": {"w": np.zeros(3, np.float32), "b": np.zeros(3, np.float32)}}
    slab = fedjax_amd.ClientDeltaSlab(template, 2, device=cuda)
    for k in range(2):
        slab.set_client(k, {m: {n: torch.full((3,), 0.5) for n in sub} for m, sub in template.items()})
    p = haiku_params(cuda)
    params = torch.cat([x.reshape(-1) for x in fedjax_amd.pytree.leaves_of(p)])  # flatten order
    opt = server.ignore_grads_haiku(server.sgd(learning_rate=1.0), [("linear_1", "w"), ("linear_2", "b")])
    mean_out = torch.empty(9, device=cuda)
    state = server.fused_mean_update(slab, [3, 5], opt, params, opt.init(params), mean_out=mean_out)
    got = slab.unflatten(params)
    npt.assert_array_equal(host(got["linear_1"]["w"]), [1., 1., 1.])
    npt.assert_array_equal(host(got["linear_2"]["w"]), [1.5, 1.5, 1.5])
    npt.assert_array_equal(host(got["linear_2"]["b"]), [3., 3., 3.])
    npt.assert_array_equal(host(mean_out), [0.5] * 9)
    assert state["count"] == 1


def test_ignore_grads_unknown_name_raises(cuda):
    params = haiku_params(cuda)
    opt = server.ignore_grads_haiku(server.sgd(1.0), [("linear_3", "w")])
    with pytest.raises(KeyError):
        server.fused_tree_mean_update([(params, 1)], opt, params, opt.init(params))


@pytest.mark.parametrize("make", [lambda: server.adam(0.01), lambda: server.sgd(0.1, momentum=0.9),
                                  lambda: server.yogi(0.02)])
def test_frozen_leaves_keep_params_and_state(make, cuda, coracle):
    """3 rounds of a stateful optimizer with a frozen leaf: trainable leaves bitwise the
    restated optax step, the frozen leaf's params and moments bitwise their initial values."""
    opt = server.ignore_grads_haiku(make(), [("enc", "b")])
    shapes = {"enc": {"b": (40,), "w": (8, 33)}, "head": {"w": (1000,)}}
    K = 9
    g = torch.Generator().manual_seed(3)
    params = {m: {n: (torch.rand(s, generator=g) - 0.5).to(cuda) for n, s in sub.items()}
              for m, sub in shapes.items()}
    state = opt.init(params)
    frozen0 = host(params["enc"]["b"]).copy()
    mom0 = {k: host(state[k]["enc"]["b"]).copy() for k in ("m", "v") if k in state}
    flat = lambda t: [x for sub in (t["enc"]["b"], t["enc"]["w"], t["head"]["w"]) for x in [sub]]
    p_np = [host(x).reshape(-1).copy() for x in flat(params)]
    m_np = [np.full(x.size, opt.init_m, np.float32) for x in p_np]
    v_np = [np.full(x.size, opt.init_v, np.float32) for x in p_np]
    for rnd in range(3):
        deltas = [{m: {n: ((torch.rand(s, generator=g) - 0.5) * 0.01).to(cuda) for n, s in sub.items()}
                   for m, sub in shapes.items()} for _ in range(K)]
        wi = [int(v) for v in ref.fedavg_weights(K, seed=40 + rnd)]
        state = server.fused_tree_mean_update(list(zip(deltas, wi)), opt, params, state)
        d = opt.descriptor(state["count"])
        for li in (1, 2):  # enc/w, head/w trainable (flatten order: enc/b, enc/w, head/w)
            xs = np.stack([host(flat(t)[li]).reshape(-1) for t in deltas])
            gm = ref.wsum_dense(xs, np.float32(wi), scale=ref.mean_scale(wi))
            p_np[li], m_np[li], v_np[li] = _np_server_step(opt, d, gm, p_np[li], m_np[li], v_np[li])
            assert np.array_equal(bits(host(flat(params)[li]).reshape(-1)), bits(p_np[li])), (rnd, li)
            if "m" in state:
                assert np.array_equal(bits(host(flat(state["m"])[li]).reshape(-1)), bits(m_np[li]))
            if "v" in state:
                assert np.array_equal(bits(host(flat(state["v"])[li]).reshape(-1)), bits(v_np[li]))
        assert np.array_equal(bits(host(params["enc"]["b"])), bits(frozen0))
        for k, v0 in mom0.items():
            assert np.array_equal(bits(host(state[k]["enc"]["b"])), bits(v0))
    assert state["count"] == 3


@pytest.mark.parametrize("make", [
    lambda: server.sgd(lambda c: 0.1 * 0.5 ** c),
    lambda: server.adam(lambda c: np.float32(1e-3) * np.float32(c + 1), b1=0.9, b2=0.99, eps=1e-4),
    lambda: server.sgd(lambda c: [0.3, 0.2, 0.05][min(c, 2)], momentum=0.9, nesterov=True)])
def test_learning_rate_schedule(make, cuda, coracle):
    """ScalarOrSchedule (optimizers.py:114): the schedule at optax's pre-increment count
    0, 1, 2 goes into each round's descriptor; the rounds are bitwise the restatement."""
    opt = make()
    K, P = 17, 4099
    template = {"a": np.zeros(3, np.float32), "b": np.zeros(P - 3, np.float32)}
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=cuda)
    params = torch.from_numpy(coracle.synth_f32(1, P, seed=81)[0].copy()).to(cuda)
    state = opt.init(params)
    p_np = host(params).copy()
    m_np = np.full(P, opt.init_m, np.float32)
    v_np = np.full(P, opt.init_v, np.float32)
    for rnd in range(3):
        slab.fill_synthetic(seed=82 + rnd)
        xh = coracle.synth_f32(K, P, seed=82 + rnd)
        wi = [int(x) for x in ref.fedavg_weights(K, seed=90 + rnd)]
        state = server.fused_mean_update(slab, wi, opt, params, state)
        d = opt.descriptor(state["count"])
        assert d.neg_lr == np.float32(-opt.learning_rate(rnd))  # evaluated at the pre-increment count
        gm = coracle.wsum_f32(xh, np.float32(wi), scale=ref.mean_scale(wi))
        p_np, m_np, v_np = _np_server_step(opt, d, gm, p_np, m_np, v_np)
        assert np.array_equal(bits(host(params)), bits(p_np)), rnd


@pytest.mark.parametrize("make", [lambda s: s.adam(1e-3), lambda s: s.sgd(0.1, momentum=0.9),
                                  lambda s: s.rmsprop(0.01, centered=True)])
def test_native_server_step_equals_python_path(make, cuda):
    """fused_tree_mean_update's one-call native path (fjhost.server_pairs) against the Python
    path (taken when ``nontemporal`` is given; the cache policy changes no bits): params,
    state and mean_out bitwise, with a leaf at a 4-byte offset (element units) and float
    weights among ints."""
    opt = make(server)
    g = torch.Generator(device="cuda").manual_seed(5)
    K = 9
    slab = torch.rand(K, 70_001 + 129, device="cuda", generator=g) - 0.5
    clients = [{"a": slab[k, 1:70_001].view(7, 10_000), "b": {"c": slab[k, 70_001:70_129]}} for k in range(K)]
    weights = [3, 1.5, 4, 1, 5, 9, 2, 6, 5]
    pairs = list(zip(clients, weights))
    p0 = {"a": torch.randn(7, 10_000, device="cuda", generator=g), "b": {"c": torch.randn(128, device="cuda",
                                                                                         generator=g)}}
    runs = []
    for nt in (None, False):
        params = {"a": p0["a"].clone(), "b": {"c": p0["b"]["c"].clone()}}
        st = opt.init(params)
        mo = {"a": torch.empty_like(p0["a"]), "b": {"c": torch.empty_like(p0["b"]["c"])}}
        for _ in range(3):
            st = server.fused_tree_mean_update(pairs, opt, params, st, mean_out=mo, nontemporal=nt)
        runs.append((params, st, mo))
    (pa, sa, ma), (pb, sb, mb) = runs
    assert sa["count"] == sb["count"] == 3
    leaves = lambda t: [host(x) for x in fedjax_amd.pytree.leaves_of(t)]
    for x, y in zip(leaves(pa) + leaves(ma), leaves(pb) + leaves(mb)):
        npt.assert_array_equal(bits(x), bits(y))
    for key in ("m", "v"):
        if key in sa:
            for x, y in zip(leaves(sa[key]), leaves(sb[key])):
                npt.assert_array_equal(bits(x), bits(y))
