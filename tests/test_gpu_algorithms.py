"""The running-sum callers other than FedAvg on the GPU: FedProx,
Mime, Mime Lite (plain and with client delta clipping), AgnosticFedAvg, APFL, the stateful
FedAvg example and HypCluster (one running sum per cluster) rounds
(tests/algorithms_restated.py) aggregated through ``fedjax_amd.tree_util``, with
deferred running sums on and off. Each round reproduces the reference's KAT values at
the reference's tolerance, and every aggregated value (mean delta, server params, Mime's
server gradient from tree_sum, AgnosticFedAvg's tree_sum'd domain statistics) is
bitwise the oracle's (oracle/tree_util_ref.py). Norms come from the GPU's reduction
and f32 sqrt, so they are held to the KAT's rtol 1e-7, not bitwise."""
import numpy as np
import pytest
import torch

from fedjax_amd import tree_util as tu
from oracle import tree_util_ref as ref
from tests import algorithms_restated as ar
from tests.test_algorithms_oracle import float32_weight_case

pytestmark = pytest.mark.gpu


def host(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class _Recorder:
    """fedjax_amd.tree_util with tree_add's result types recorded."""

    def __init__(self):
        self.add_types = []

    def __getattr__(self, name):
        return getattr(tu, name)

    def tree_add(self, a, b):
        out = tu.tree_add(a, b)
        self.add_types.append(type(out).__name__)
        return out


def _gpu_round(fn, cuda, rec):
    to_leaf = lambda a: torch.from_numpy(np.array(a, dtype=np.float32)).to(cuda)  # (keeps 0-d shapes)
    to_weight = lambda w: torch.tensor(w, device=cuda)  # a jnp scalar array on the device
    return fn(rec, to_leaf, host, to_weight)


def _same_bits(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.fixture(params=[True, False], ids=["deferred", "eager"])
def deferral(request):
    tu.set_deferred_sums(request.param)
    yield request.param
    tu.set_deferred_sums(True)


@pytest.mark.parametrize("name,fn,want", ar.KATS, ids=[k[0] for k in ar.KATS])
def test_algorithm_round_on_gpu(name, fn, want, cuda, deferral):
    rec = _Recorder()
    got = _gpu_round(fn, cuda, rec)
    ar.check_kat(name, got, want)
    exp = fn(ref, np.asarray, np.asarray, lambda w: w)
    for key, want_v in exp.items():
        if key in ("norms", "clipped_norms"):  # the GPU's reduction order and f32 sqrt
            for cid, v in want_v.items():
                np.testing.assert_allclose(got[key][cid], v, rtol=1e-7, err_msg=f"{name} {key} {cid!r}")
        elif key in ("betas", "cluster_ids", "num_steps"):  # client-side values
            assert got[key] == want_v or all(_same_bits(got[key][c], want_v[c]) for c in want_v), (name, key)
        elif isinstance(want_v, dict):
            for cid, v in want_v.items():
                assert _same_bits(got[key][cid], v), (name, key, cid, got[key][cid], v)
        elif isinstance(want_v, list):
            assert len(got[key]) == len(want_v), (name, key)
            for a, b in zip(got[key], want_v):
                assert (a is None and b is None) or _same_bits(a, b), (name, key, a, b)
        elif want_v is None:
            assert got[key] is None, (name, key)
        else:  # every aggregated value: bitwise the oracle's
            assert _same_bits(got[key], want_v), (name, key, got[key], want_v)
    # the running sum of Python-number weights is deferred exactly when deferral is on
    if fn is not ar.agnostic_fed_avg_round and fn is not ar.mime_round:
        assert ("PendingSum" in rec.add_types) == deferral, rec.add_types


def test_float32_array_weights_take_the_float32_W_branch(cuda, deferral):
    """agnostic_fed_avg.py:282-289's loop with float32 array weights: tree_weight by a
    strongly typed f32 scalar, W = 0. + w_0 + ... in float32, then tree_inverse_weight
    by that float32 W. Bitwise the oracle's float32-W result, which differs from the
    Python-float-W one on these inputs (test_algorithms_oracle.py)."""
    w, x = float32_weight_case()
    s = tu.tree_zeros_like({"p": torch.zeros(x.shape[1], device=cuda)})
    W = 0.0
    for k in range(len(w)):
        wk = torch.tensor(w[k], device=cuda)
        s = tu.tree_add(s, tu.tree_weight({"p": torch.from_numpy(x[k]).to(cuda)}, wk))
        W = W + wk
    assert isinstance(W, torch.Tensor) and W.dtype == torch.float32
    got = host(tu.tree_inverse_weight(s, W)["p"])
    s_ref = ref.tree_zeros_like({"p": x[0]})
    W_ref = 0.0
    for k in range(len(w)):
        s_ref = ref.tree_add(s_ref, ref.tree_weight({"p": x[k]}, w[k]))
        W_ref += w[k]
    want = ref.tree_inverse_weight(s_ref, W_ref)["p"]
    assert _same_bits(got, want)
