"""Pins the compression / PRNG restatement (oracle/compression_ref.py,
oracle/jax_random_ref.py) to the reference's own tests and to published
known-answer vectors. Every expected value below is copied from:

* fedjax/aggregators/compression_test.py (line numbers per test)
* fedjax/aggregators/walsh_hadamard_test.py
* Random123 kat_vectors, threefry2x32_20 (also jax random_test.py testThreefry2x32)
* the JAX docs' ``random.split(random.PRNGKey(0))`` printout
"""

import numpy as np
import numpy.testing as npt
import pytest

from oracle import compression_ref as c
from oracle import jax_random_ref as jr

F32 = np.float32


def _clients():
    # compression_test.py:87-93 (and every quantizer test after it)
    return [("a", {"w": np.array([1., 2., 3.], F32)}, 2.),
            ("b", {"w": np.array([2., 4., 6.], F32)}, 4.),
            ("c", {"w": np.array([1., 3., 5.], F32)}, 2.)]


@pytest.mark.parametrize("key,ctr,expect", [
    ((0, 0), (0, 0), (0x6b200159, 0x99ba4efe)),
    ((0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff), (0x1cb996fc, 0xbb002be7)),
    ((0x13198a2e, 0x03707344), (0x243f6a88, 0x85a308d3), (0xc4923a9c, 0x483df7a0)),
])
def test_threefry_kat(key, ctr, expect):
    y0, y1 = jr.threefry2x32(key, [ctr[0]], [ctr[1]])
    assert (int(y0[0]), int(y1[0])) == expect


def test_split_prngkey0_published_value():
    npt.assert_array_equal(jr.split(jr.prng_key(0)), [[4146024105, 967050713], [2718843009, 1272950319]])


def test_prng_key_layout():
    npt.assert_array_equal(jr.prng_key(42), [0, 42])
    npt.assert_array_equal(jr.prng_key((7 << 32) | 5), [7, 5])


def test_odd_count_padding():
    # an odd count array is padded with a zero counter, then trimmed
    bits5 = jr.random_bits(jr.prng_key(3), 5)
    y0, y1 = jr.threefry2x32(jr.prng_key(3), [0, 1, 2], [3, 4, 0])
    npt.assert_array_equal(bits5, np.concatenate([y0, y1])[:5])


def test_uniform_range_and_rademacher():
    u = jr.uniform(jr.prng_key(1), (10000,))
    assert u.dtype == np.float32 and u.min() >= 0 and u.max() < 1
    r = jr.rademacher(jr.prng_key(1), (10000,))
    npt.assert_array_equal(r, np.where(u < 0.5, 1, -1))


def test_prng_sequence_reserves_one_key_at_a_time():
    seq = jr.PRNGSequence(jr.prng_key(9))
    k0 = next(seq)
    a, b = jr.split(jr.prng_key(9))
    npt.assert_array_equal(k0, b)
    npt.assert_array_equal(next(seq), jr.split(a)[1])


def test_binary_stochastic_quantize_identity():  # compression_test.py:30-35
    v = np.array([0., 2., 2.], F32)
    npt.assert_array_equal(c.binary_stochastic_quantize(v, jr.prng_key(42)), v)


def test_binary_stochastic_quantize_unbiasedness():  # :37-44
    v = np.array([0., 1., 2.], F32)
    rng, s = jr.prng_key(42), np.zeros(3, F32)
    for _ in range(500):
        rng, use = jr.split(rng)
        s += c.binary_stochastic_quantize(v, use)
    npt.assert_array_almost_equal(s / 500, v, decimal=2)


def test_uniform_stochastic_quantize_identity():  # :46-52
    v = np.array([0., 2., 2., 4.], F32)
    npt.assert_array_equal(c.uniform_stochastic_quantize(v, 3, jr.prng_key(42)), v)


def test_uniform_stochastic_quantize_all_equal():  # :54-58
    v = np.array([4., 4., 4., 4.], F32)
    npt.assert_array_equal(c.uniform_stochastic_quantize(v, 4, jr.prng_key(42)), v)


@pytest.mark.parametrize("v,dec", [([0., 1., 100.], 2), ([[0., 1., 100.], [0.3, 2.3, 45.]], 1)])
def test_uniform_stochastic_quantize_unbiasedness(v, dec):  # :60-76
    v = np.array(v, F32)
    rng, s = jr.prng_key(42), np.zeros_like(v)
    for _ in range(500):
        rng, use = jr.split(rng)
        s += c.uniform_stochastic_quantize(v, 125, use)
    npt.assert_array_almost_equal(s / 500, v, decimal=dec)


def test_arithmetic_encoding_num_bits():  # :78-81
    npt.assert_array_almost_equal(c.arithmetic_encoding_num_bits(np.array([1., 2., 3., 4., 5.], F32)),
                                  [89.82311], decimal=3)


def test_uniform_stochastic_quantizer():  # :83-99
    init, apply = c.uniform_stochastic_quantizer(3, jr.prng_key(0))
    p, st = apply(_clients(), init())
    assert st.num_bits == 68.75489
    npt.assert_array_equal(p["w"], [1.5, 3.25, 5.])


def test_uniform_stochastic_quantizer_arithmetic_coding():  # :101-117
    init, apply = c.uniform_stochastic_quantizer(3, jr.prng_key(0), "arithmetic")
    p, st = apply(_clients(), init())
    assert st.num_bits == 78.08298
    npt.assert_array_equal(p["w"], [1.5, 3.25, 5.])


@pytest.mark.parametrize("commute", [False, True])
def test_rotated_uniform_stochastic_quantizer(commute):  # :119-137
    init, apply = c.rotated_uniform_stochastic_quantizer(2, jr.prng_key(0), commute_inverse=commute)
    st, ps = init(), []
    for _ in range(2000):
        p, st = apply(_clients(), st)
        ps.append(p["w"])
    assert st.num_bits == 67 * 2000
    npt.assert_array_almost_equal(np.mean(ps, axis=0), [1.5, 3.25, 5.], decimal=1)


def test_structured_drive_pytree():  # :139-143
    y = c.drive_pytree({"w": np.array([1., -2., 3.], F32)})
    npt.assert_array_almost_equal(y["w"], [2.333333, -2.333333, 2.333333], decimal=4)


def test_structured_drive_quantizer():  # :145-165
    init, apply = c.structured_drive_quantizer(jr.prng_key(0))
    st, ps = init(), []
    for _ in range(100):
        p, st = apply(_clients(), st)
        ps.append(p["w"])
    assert st.num_bits == 67 * 100
    npt.assert_array_almost_equal(sum(ps) / 100, [1.458334, 1.458334, 6.125], decimal=4)


def test_terngrad_quantize_identity():  # :167-172
    v = np.array([0., 2., 2.], F32)
    npt.assert_array_equal(c.terngrad_quantize(v, jr.prng_key(42)), v)


def test_terngrad_quantize_clipping():  # :174-185
    v = np.zeros(100, F32)
    v[0], v[1] = 100, -100
    expect = v.copy()
    expect[0], expect[1] = 35.355339, -35.355339
    npt.assert_array_equal(c.terngrad_quantize(v, jr.prng_key(42)), expect)


def test_terngrad_quantizer():  # :187-203 — depends on every bit of the key schedule
    init, apply = c.terngrad_quantizer(jr.prng_key(0))
    p, st = apply(_clients(), init())
    assert st.num_bits == 68.75489
    npt.assert_array_almost_equal(p["w"], [0.51031, 2.551552, 3.572173], decimal=4)


def test_walsh_hadamard_transform_matches_dense():  # walsh_hadamard_test.py:27-44
    import scipy.linalg
    n = 2 ** 10
    H = scipy.linalg.hadamard(n).astype(np.float64)
    for seed in range(5):
        x = np.random.RandomState(seed).standard_normal(n).astype(F32)
        npt.assert_allclose(c.fwht(x), H @ x.astype(np.float64), rtol=1e-4, atol=1e-4)


def test_structured_rotation_roundtrip():  # walsh_hadamard_test.py:46-55
    x = np.random.RandomState(100).standard_normal((5, 10)).astype(F32)
    y, shape = c.structured_rotation(x, jr.prng_key(10))
    assert shape == x.shape and y.size == 64
    npt.assert_allclose(c.inverse_structured_rotation(y, jr.prng_key(10), shape), x, rtol=1e-4, atol=1e-4)


def test_structured_rotation_pytree_roundtrip():  # walsh_hadamard_test.py:57-66
    params = {"a": np.array([[1., 0., 0.], [1., 2., 3.]], F32), "b": np.array([[1., 0.], [1., 2.]], F32)}
    y, shapes = c.structured_rotation_pytree(params, jr.prng_key(10))
    z = c.inverse_structured_rotation_pytree(y, jr.prng_key(10), shapes)
    npt.assert_allclose(z["a"], params["a"], rtol=1e-4, atol=1e-4)
    npt.assert_allclose(z["b"], params["b"], rtol=1e-4, atol=1e-4)
