"""The running-sum callers other than FedAvg pinned on the CPU: the
restated rounds of FedProx, Mime, Mime Lite (with and without client delta clipping),
AgnosticFedAvg, APFL, the stateful FedAvg example and HypCluster
(tests/algorithms_restated.py), aggregated through the oracle
(oracle/tree_util_ref.py), reproduce every value the reference's own tests assert, at
their tolerance (npt.assert_allclose's default rtol 1e-7)."""
import numpy as np
import pytest

from oracle import tree_util_ref as ref
from tests import algorithms_restated as ar


def _oracle_round(fn, to_weight=lambda w: w):
    return fn(ref, np.asarray, np.asarray, to_weight)


@pytest.mark.parametrize("name,fn,want", ar.KATS, ids=[k[0] for k in ar.KATS])
def test_algorithm_round_kats_through_the_oracle(name, fn, want):
    ar.check_kat(name, _oracle_round(fn), want)


def test_agnostic_weights_are_float32_arrays():
    """agnostic_fed_avg.py:279-285: beta is a jnp float32 array, so weight_sum = 0. +
    beta_0 + beta_1 stays float32 and 1/W is a float32 division."""
    got = _oracle_round(ar.agnostic_fed_avg_round)
    betas = list(got["betas"].values())
    assert all(type(b) is np.float32 for b in betas)
    W = 0.0
    for b in betas:
        W += b
    assert type(W) is np.float32
    np.testing.assert_allclose([float(b) for b in betas], [0.6, 0.3], rtol=1e-7)  # agnostic_fed_avg_test.py:167,172


def test_float32_weight_sum_differs_from_float64_on_some_inputs():
    """The array-weight branch is observable: for these float32 weights the reference's
    float32 W (0. + w_0 + ... in f32) and a Python-float W give different means, so the
    GPU test of the same inputs (test_gpu_algorithms.py) pins which one is taken."""
    w, x = float32_weight_case()
    t32 = ref.tree_mean(({"p": x[k]}, w[k]) for k in range(len(w)))
    t64 = ref.tree_mean(({"p": x[k]}, float(w[k])) for k in range(len(w)))
    assert not np.array_equal(t32["p"].view(np.uint32), t64["p"].view(np.uint32))


def float32_weight_case():
    """Float32 weights whose f32 running sum differs from the f64 one, and deltas."""
    rs = np.random.RandomState(7)
    w = rs.uniform(0.05, 0.95, 37).astype(np.float32)
    x = rs.standard_normal((37, 513)).astype(np.float32)
    return w, x
