"""The oracle (oracle/) pinned against the reference's own known-answer tests.

Every value below is copied from a reference test file (cited per test); the
reference itself cannot run here (JAX absent).
"""

import numpy as np
import numpy.testing as npt
import pytest

from oracle import tree_util_ref as ref
from tests import fedavg_restated as fr


def test_mean_aggregator_kat():
    # fedjax/aggregators/aggregator_test.py:24-37
    delta_params_and_weights = [("a", {"w": np.array([1., 2., 3.])}, 2.),
                                ("b", {"w": np.array([2., 4., 6.])}, 4.),
                                ("c", {"w": np.array([1., 3., 5.])}, 2.)]
    agg = ref.mean_aggregator()
    mean, _ = agg.apply(delta_params_and_weights, agg.init())
    npt.assert_array_equal(mean["w"], [1.5, 3.25, 5.])


def test_tree_weight_kat():
    # fedjax/core/tree_util_test.py:27-35 (int leaves * 2.0 -> float)
    t = {"x": np.array([[[4, 5]], [[1, 1]]]), "y": np.array([[3], [1]])}
    w = ref.tree_weight(t, 2.0)
    npt.assert_array_equal(w["x"], [[[8.0, 10.0]], [[2.0, 2.0]]])
    npt.assert_array_equal(w["y"], [[6.0], [2.0]])
    assert w["x"].dtype == np.float32


def test_tree_sum_kat():
    # fedjax/core/tree_util_test.py:37-51 (ints stay ints)
    t1 = {"x": np.array([[[4, 5]], [[1, 1]]]), "y": np.array([[3], [1]])}
    t2 = {"x": np.array([[[2, 3]], [[4, 5]]]), "y": np.array([[6], [7]])}
    s = ref.tree_sum([t1, t2])
    npt.assert_array_equal(s["x"], [[[6, 8]], [[5, 6]]])
    npt.assert_array_equal(s["y"], [[9], [8]])
    assert s["x"].dtype == np.int32


def test_tree_mean_kat():
    # fedjax/core/tree_util_test.py:53-62
    trees = [(np.array(0), np.array(1)), (np.array(2), np.array(3)), (np.array(4), np.array(5))]
    m = ref.tree_mean(zip(trees, [6., 7., 8.]))
    npt.assert_array_almost_equal(m, (2.1904761904761907, 3.1904761904761907))
    # bit-level: f32(46) * f32(1/21), f32(67) * f32(1/21)
    r = np.float32(1.0 / 21.0)
    assert m[0] == np.float32(46) * r and m[1] == np.float32(67) * r


def test_tree_clip_kat():
    # fedjax/core/tree_util_test.py:64-73 (via l2 norm + weight)
    t = {"x": np.array([[[4, 5]], [[1, 1]]]), "y": np.array([[3], [1]])}
    norm = ref.tree_l2_norm(t)
    scale = min(np.float32(1), np.float32(3.640055) / norm)
    c = ref.tree_weight(t, np.float32(scale))
    npt.assert_array_almost_equal(c["x"], [[[2, 2.5]], [[0.5, 0.5]]])
    npt.assert_array_almost_equal(c["y"], [[1.5], [0.5]])


def test_empty_mean_is_none():
    assert ref.tree_mean([]) is None
    assert ref.tree_sum([]) is None


def test_zero_total_weight_gives_zeros():
    m = ref.tree_mean([({"w": np.array([1., -2.], np.float32)}, 0.0)])
    assert np.array_equal(m["w"], np.zeros(2, np.float32))


@pytest.mark.parametrize("name,round_fn,bs,epochs,want,want_norms", fr.KATS)
def test_fedavg_round_kats(name, round_fn, bs, epochs, want, want_norms):
    new, norms = round_fn(ref, lambda a: a, np.asarray, fr.SERVER_PARAMS, fr.CLIENTS, bs, epochs, 0)
    npt.assert_allclose(new["w"], want, err_msg=name)
    for cid, v in want_norms.items():
        npt.assert_allclose(norms[cid], v, rtol=1e-6, err_msg=name)


def test_c_oracle_matches_numpy_oracle(coracle):
    K, P = 37, 1031
    x = coracle.synth_f32(K, P, seed=3)
    assert np.array_equal(x.view(np.uint32), ref.synth(K, P, seed=3).view(np.uint32))
    w = ref.fedavg_weights(K).astype(np.float32)
    r = ref.mean_scale([int(v) for v in ref.fedavg_weights(K)])
    want = ref.wsum_dense(x, w, scale=r)
    got = coracle.wsum_f32(x, w, scale=r)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    for nthreads in (1, 3, 8):
        seq = coracle.refseq_f32(x, w, r, nthreads=nthreads)
        assert np.array_equal(seq.view(np.uint32), want.view(np.uint32))


def test_oracle_fold_equals_pytree_tree_mean():
    # the dense restatement and the pytree restatement are the same arithmetic
    K, P = 9, 257
    x = ref.synth(K, P, seed=11)
    wi = [int(v) for v in ref.fedavg_weights(K, seed=5)]
    m = ref.tree_mean(({"a": x[k, :100], "b": x[k, 100:]}, wi[k]) for k in range(K))
    d = ref.wsum_dense(x, np.float32(wi), scale=ref.mean_scale(wi))
    assert np.array_equal(np.concatenate([m["a"], m["b"]]).view(np.uint32), d.view(np.uint32))


def test_bf16_oracles_are_consistent(coracle):
    K, P = 16, 513
    xb = coracle.synth_bf16(K, P, seed=2)
    w = np.float64(ref.fedavg_weights(K))
    r = 1.0 / w.sum()
    exact = coracle.wsum_bf16_f64(xb, w, r)
    refsem = coracle.wsum_bf16_refsem(xb, w.astype(np.float32), np.float32(r))
    from tests.coracle import bf16_to_f32
    # reference bf16 semantics accumulate in bf16: far looser than one bf16 rounding
    err = np.abs(bf16_to_f32(refsem) - exact)
    assert np.all(err <= 2.0 ** -8 * (np.abs(exact) + 0.01) * K)
