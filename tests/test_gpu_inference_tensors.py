"""Tree ops on inference tensors (torch.inference_mode). Such tensors carry no in-place
version counter (``Tensor._version`` raises), so the deferred paths that hold a delta by
reference cannot guard it: tree_weight / tree_add of an inference pytree run eagerly (the
value is read at the call, as the reference reads it at tree_util.py:29-50), and
RunningMean snapshots inference leaves at add(). Results stay bitwise the reference's op
sequence (oracle/tree_util_ref.py restates fedjax/core/tree_util.py:29-96)."""
import numpy as np
import pytest
import torch

from fedjax_amd import pytree, tree_util as tu
from fedjax_amd.aggregators import RunningMean
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu

SHAPES = {"a": (1000,), "b": (7, 3), "c": {"w": (64, 33)}}


def tmap(fn, t):
    return {k: tmap(fn, v) for k, v in t.items()} if isinstance(t, dict) else fn(t)


def host_tree(g):
    return tmap(lambda s: ((torch.rand(s, generator=g) * 2 - 1) * 0.01).numpy(), SHAPES)


def bits_equal(got, want):
    gl = [x.detach().cpu().numpy().reshape(-1) for x in pytree.leaves_of(got)]
    wl = [np.asarray(x, np.float32).reshape(-1) for x in pytree.leaves_of(want)]
    return all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(gl, wl))


@pytest.fixture(params=["deferred", "eager"])
def sum_mode(request):
    tu.set_deferred_sums(request.param == "deferred")
    yield request.param
    tu.set_deferred_sums(True)


def test_running_sum_on_inference_tensors(cuda, sum_mode):
    g = torch.Generator().manual_seed(11)
    hosts = [host_tree(g) for _ in range(6)]
    weights = [3, 5, 2.5, 7, 1, 4]
    with torch.inference_mode():
        deltas = [tmap(lambda x: torch.from_numpy(x).to(cuda), h) for h in hosts]
        params = tmap(lambda s: torch.zeros(s, device=cuda), SHAPES)
        assert pytree.leaves_of(deltas[0])[0].is_inference()
        s = tu.tree_zeros_like(params)
        n_sum = 0.
        norms = []
        for d, n in zip(deltas, weights):
            s = tu.tree_add(s, tu.tree_weight(d, n))
            n_sum += n
            norms.append(float(tu.tree_l2_norm(d)))
        mean = tu.tree_inverse_weight(s, n_sum)
    want_s = tmap(lambda s_: np.zeros(s_, np.float32), SHAPES)
    for h, n in zip(hosts, weights):
        want_s = ref.tree_add(want_s, ref.tree_weight(h, n))
    assert bits_equal(mean, ref.tree_inverse_weight(want_s, n_sum))
    for h, nrm in zip(hosts, norms):
        x64 = np.concatenate([np.asarray(x, np.float64).reshape(-1) for x in pytree.leaves_of(h)])
        np.testing.assert_allclose(nrm, np.sqrt((x64 * x64).sum()), rtol=2e-6)


def test_inference_delta_modified_after_tree_weight_keeps_the_call_time_value(cuda, sum_mode):
    """The reference computes tree_weight at the call; an inference tensor cannot be guarded
    lazily, so the product must already be taken when the caller reuses the buffer."""
    g = torch.Generator().manual_seed(12)
    h0, h1 = host_tree(g), host_tree(g)
    with torch.inference_mode():
        buf = tmap(lambda x: torch.from_numpy(x).to(cuda), h0)
        s = tu.tree_zeros_like(buf)
        s = tu.tree_add(s, tu.tree_weight(buf, 3))
        for x, y in zip(pytree.leaves_of(buf), pytree.leaves_of(h1)):
            x.copy_(torch.from_numpy(y))  # reuse the buffer for the next client, in place
        s = tu.tree_add(s, tu.tree_weight(buf, 5))
        mean = tu.tree_inverse_weight(s, 8.)
    want = ref.tree_add(ref.tree_add(tmap(lambda s_: np.zeros(s_, np.float32), SHAPES), ref.tree_weight(h0, 3)),
                        ref.tree_weight(h1, 5))
    assert bits_equal(mean, ref.tree_inverse_weight(want, 8.))


def test_tree_mean_and_sum_on_inference_tensors(cuda):
    g = torch.Generator().manual_seed(13)
    hosts = [host_tree(g) for _ in range(5)]
    weights = [1, 2, 3, 4, 5]
    with torch.inference_mode():
        deltas = [tmap(lambda x: torch.from_numpy(x).to(cuda), h) for h in hosts]
        got = tu.tree_mean(list(zip(deltas, weights)))
        got_sum = tu.tree_sum(deltas)
    assert bits_equal(got, ref.tree_mean(list(zip(hosts, weights))))
    assert bits_equal(got_sum, ref.tree_sum(hosts))


@pytest.mark.parametrize("inside", [True, False])
def test_running_mean_snapshots_inference_leaves(cuda, inside):
    """RunningMean buffers deltas by reference and checks version counters at flush; an
    inference leaf has none, so it is cloned at add(). Reusing the buffer in place (inside
    inference mode, where that is allowed) must not change the sum."""
    g = torch.Generator().manual_seed(14)
    hosts = [host_tree(g) for _ in range(4)]
    weights = [2, 9, 4, 1]
    with torch.inference_mode():
        buf = tmap(lambda x: torch.from_numpy(x).to(cuda), hosts[0])
        tmpl = tmap(lambda s: torch.zeros(s, device=cuda), SHAPES)
    rm = RunningMean(tmpl)
    for h, w in zip(hosts, weights):
        with torch.inference_mode():
            for x, y in zip(pytree.leaves_of(buf), pytree.leaves_of(h)):
                x.copy_(torch.from_numpy(y))
        if inside:
            with torch.inference_mode():
                rm.add(buf, w)
        else:
            rm.add(buf, w)
    got = rm.result()
    want_s = tmap(lambda s_: np.zeros(s_, np.float32), SHAPES)
    for h, w in zip(hosts, weights):
        want_s = ref.tree_add(want_s, ref.tree_weight(h, w))
    assert bits_equal(got, ref.tree_inverse_weight(want_s, float(sum(weights))))
