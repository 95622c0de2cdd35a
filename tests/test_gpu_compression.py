"""GPU parity of the compression aggregators (include/fjcomp.h) against the oracle
restatement (oracle/compression_ref.py, oracle/jax_random_ref.py), and the
reference's own compression / Walsh-Hadamard tests re-run on the GPU path.

Bar: random bits, signs, quantized values, transforms and folds are
bitwise equal to the restatement (same float32 op order); the rotated quantizer,
which inverts the rotation once on the mean, is compared bitwise with the
restatement in that order and within float32 reassociation error of the
reference order; the reference's tests hold at their own tolerances.
"""
import numpy as np
import numpy.testing as npt
import pytest
import torch

import fedjax_amd
from fedjax_amd import _compress as C
from fedjax_amd import random
from fedjax_amd.aggregators import compression as comp
from fedjax_amd.aggregators import walsh_hadamard as wh
from oracle import compression_ref as cref
from oracle import jax_random_ref as jr

pytestmark = pytest.mark.gpu
F32 = np.float32


def host(t):
    return t.detach().cpu().numpy()


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def same(a, b):
    npt.assert_array_equal(bits(a), bits(b))


def dev(x, cuda):
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def _clients(cuda):
    return [("a", {"w": dev(np.array([1., 2., 3.], F32), cuda)}, 2.),
            ("b", {"w": dev(np.array([2., 4., 6.], F32), cuda)}, 4.),
            ("c", {"w": dev(np.array([1., 3., 5.], F32), cuda)}, 2.)]


def _ref_clients():
    return [("a", {"w": np.array([1., 2., 3.], F32)}, 2.),
            ("b", {"w": np.array([2., 4., 6.], F32)}, 4.),
            ("c", {"w": np.array([1., 3., 5.], F32)}, 2.)]


SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 16)},
          "linear": {"b": (128,), "w": (1152, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def _tree(rs, scale=0.01, shapes=SHAPES):
    return {k: (_tree(rs, scale, v) if isinstance(v, dict) else (rs.standard_normal(v) * scale).astype(F32))
            for k, v in shapes.items()}


def _to_dev(t, cuda):
    return {k: (_to_dev(v, cuda) if isinstance(v, dict) else dev(v, cuda)) for k, v in t.items()}


def _leaves(t):
    return [x for k in sorted(t) for x in (_leaves(t[k]) if isinstance(t[k], dict) else [t[k]])]


def _fleet(cuda, K=7, seed=0):
    rs = np.random.RandomState(seed)
    trees = [_tree(rs) for _ in range(K)]
    w = [int(v) for v in rs.randint(1, 500, K)]
    return ([(f"c{k}", _to_dev(t, cuda), w[k]) for k, t in enumerate(trees)],
            [(f"c{k}", t, w[k]) for k, t in enumerate(trees)])


# ------------------------------------------------------------------ random draws
@pytest.mark.parametrize("n", [1, 2, 3, 7, 1000, (1 << 20) + 3])
@pytest.mark.parametrize("seed", [0, 42])
def test_random_bits_and_uniform(n, seed, cuda):
    key = random.PRNGKey(seed)
    npt.assert_array_equal(host(random.random_bits(key, n, cuda)).view(np.uint32), jr.random_bits(key, n))
    same(host(random.uniform(key, (n,), cuda)), jr.uniform(key, (n,)))


def test_rademacher(cuda):
    key = random.PRNGKey(3)
    npt.assert_array_equal(host(random.rademacher(key, (5, 7), cuda)), jr.rademacher(key, (5, 7)))


@pytest.mark.parametrize("d", [1, 2, 4, 32, 64, 128, 1024, 1 << 16, 1 << 21])
def test_sign_words(d, cuda):
    keys = jr.split(jr.prng_key(d), 3)
    words, woff = C.rademacher_words(keys, [d] * 3, cuda)
    w = host(words).view(np.uint32)
    g = np.arange(d)
    for j in range(3):
        got = (w[woff[j] + (g >> 5)] >> (g & 31)) & 1
        npt.assert_array_equal(got == 1, jr.rademacher(keys[j], (d,)) == -1)


@pytest.mark.parametrize("block_pairs", [256, 512, 2048, 8192])
def test_sign_words_every_workgroup_share(block_pairs, cuda):
    """k_rademacher's fast path (even d, the wave's run inside the job) and general path
    (odd d, runs that cross the job end, jobs shorter than a wave) at every workgroup share,
    jobs of mixed lengths in one launch."""
    ds = [1, 63, 64, 96, 1000, 4095, 4096, 8193, 65536, 100001, 1 << 18, (1 << 18) + 3]
    keys = jr.split(jr.prng_key(block_pairs), len(ds))
    words, woff = C.rademacher_words(keys, ds, cuda, block_pairs=block_pairs)
    w = host(words).view(np.uint32)
    for j, d in enumerate(ds):
        g = np.arange(d)
        got = (w[woff[j] + (g >> 5)] >> (g & 31)) & 1
        npt.assert_array_equal(got == 1, jr.rademacher(keys[j], (d,)) == -1, err_msg=f"job {j}, d={d}")


def test_sign_words_bad_share(cuda):
    from fedjax_amd._lib import FjaggError

    with pytest.raises(FjaggError, match="block_pairs"):
        C.rademacher_words(jr.split(jr.prng_key(0), 1), [64], cuda, block_pairs=300)


@pytest.mark.parametrize("sums", [False, True])
@pytest.mark.parametrize("nan", [False, True])
def test_rotate_tile_partials_equal_row_stats(nan, sums, cuda):
    """The ROTATE pass's per-tile min / max partials (fjcomp_stats_combine) give the same
    stats min / max and the same UNIFORM qparams bytes as a k_row_stats pass over the rotated
    rows (one- and two-pass lengths, NaN propagation)."""
    rs = np.random.RandomState(5)
    ns = [1, 5, 64, 300, 8192, 8193, 100000, 1 << 18]
    ds = [C.padded_size(n) for n in ns]
    srcs = [rs.standard_normal(n).astype(F32) for n in ns]
    if nan:
        srcs[3][7] = np.nan
        srcs[6][99] = np.nan
    xs = [dev(x, cuda) for x in srcs]
    keys = jr.split(jr.prng_key(11), len(ns))
    signs, woff = C.rademacher_words(keys, ds, cuda)
    ys = [torch.empty(d, dtype=torch.float32, device=cuda) for d in ds]
    last = np.array([C.wht_tiles(d.bit_length() - 1, C.wht_passes(d.bit_length() - 1) - 1) for d in ds])
    pre = np.concatenate([[0], np.cumsum(last)]).astype(np.int64)
    slot = int(fedjax_amd._lib.load().fjcomp_row_stats_workspace_bytes(1))
    part = torch.empty(int(pre[-1]) * slot, dtype=torch.uint8, device=cuda)
    yp = np.array([y.data_ptr() for y in ys], dtype=np.uint64)
    sp = np.uint64(signs.data_ptr()) + np.uint64(4) * woff[:-1].astype(np.uint64)
    keep = C.run_wht(C.wht_jobs([x.data_ptr() for x in xs], yp, yp, ds, kind=fedjax_amd._lib.WHT_ROTATE,
                                n_in=ns, signs=sp,
                                stats=np.uint64(part.data_ptr()) + np.uint64(slot) * pre[:-1].astype(np.uint64),
                                flags=C.WHT_F_SUMS if sums else 0),
                     cuda)
    st_a, qp_a, up = C.stats_from_partials(yp, ds, pre, part, fedjax_amd._lib.COMP_UNIFORM, cuda)
    st_b, qp_b = C.row_stats_table(yp, ds, fedjax_amd._lib.COMP_UNIFORM, cuda)
    torch.cuda.synchronize()
    del keep, up
    a, b = host(st_a).view(C.STATS), host(st_b).view(C.STATS)
    for f in ("min", "max", "absmax"):
        npt.assert_array_equal(a[f].view(np.uint64), b[f].view(np.uint64), err_msg=f)
    npt.assert_array_equal(host(qp_a), host(qp_b))
    for f in ("sumsq", "sumabs"):  # f64 sums in tile order vs chunk order: equal to ~1e-15
        if sums:
            npt.assert_allclose(a[f], b[f], rtol=1e-13, err_msg=f)
        else:
            assert not a[f].any()


# ------------------------------------------------------------------ Walsh-Hadamard
@pytest.mark.parametrize("m", [0, 1, 2, 5, 12, 13, 14, 17, 21, 26, 27])
def test_wht_bitwise(m, cuda):
    x = np.random.RandomState(m).standard_normal(1 << m).astype(F32)
    same(host(wh.walsh_hadamard_transform(dev(x, cuda))), cref.fwht(x))


def test_wht_against_dense_hadamard(cuda):  # walsh_hadamard_test.py:27-44
    n = 1 << 10
    H = wh.hadamard_matrix(n).double().numpy()
    for seed in range(5):
        x = np.random.RandomState(seed).standard_normal(n).astype(F32)
        for small_n in [2, 8, 128, 2048]:
            y = host(wh.walsh_hadamard_transform(dev(x, cuda), small_n))
            assert y.shape == x.shape and y.dtype == np.float32
            npt.assert_allclose(y, H @ x.astype(np.float64), rtol=1e-4, atol=1e-4)
    with pytest.raises(ValueError):
        wh.walsh_hadamard_transform(dev(x, cuda), 1)
    with pytest.raises(ValueError):
        wh.walsh_hadamard_transform(dev(np.ones(12, F32), cuda))


@pytest.mark.parametrize("shape", [(1,), (3,), (5, 10), (100,), (18432,), (9216, 128)])
def test_structured_rotation_bitwise(shape, cuda):
    x = np.random.RandomState(1).standard_normal(shape).astype(F32)
    key = jr.prng_key(10)
    y, s = wh.structured_rotation(dev(x, cuda), key)
    ey, es = cref.structured_rotation(x, key)
    same(host(y), ey)
    assert tuple(s.tolist()) == es == shape
    z = wh.inverse_structured_rotation(y, key, s)
    same(host(z), cref.inverse_structured_rotation(ey, key, es))
    npt.assert_allclose(host(z), x, rtol=1e-4, atol=1e-4)  # walsh_hadamard_test.py:46-55


@pytest.mark.parametrize("n,offset", [(100, 1), (18433, 1), (9216 * 128, 2), (9216 * 128 + 3, 0), (64, 3)])
def test_structured_rotation_unaligned_and_ragged(n, offset, cuda):
    """16-byte quads vs the scalar path: a source view off 16-byte alignment, lengths that
    end inside a quad (zero padding) and outputs truncated inside a quad."""
    x = np.random.RandomState(n).standard_normal(n + offset).astype(F32)
    key = jr.prng_key(n)
    t = dev(x, cuda)[offset:]
    y, s = wh.structured_rotation(t, key)
    ey, es = cref.structured_rotation(x[offset:], key)
    same(host(y), ey)
    z = wh.inverse_structured_rotation(y, key, s)
    same(host(z), cref.inverse_structured_rotation(ey, key, es))
    same(host(wh.walsh_hadamard_transform(y)), cref.fwht(ey))


def test_structured_rotation_pytree(cuda):  # walsh_hadamard_test.py:57-66
    params = {"a": np.array([[1.0, 0.0, 0.0], [1.0, 2.0, 3.0]], F32), "b": np.array([[1.0, 0.0], [1.0, 2.0]], F32)}
    key = random.PRNGKey(10)
    y, shapes = wh.structured_rotation_pytree(_to_dev(params, cuda), key)
    ey, _ = cref.structured_rotation_pytree(params, key)
    same(host(y["a"]), ey["a"])
    same(host(y["b"]), ey["b"])
    z = wh.inverse_structured_rotation_pytree(y, key, shapes)
    npt.assert_allclose(host(z["a"]), params["a"], rtol=1e-4, atol=1e-4)
    npt.assert_allclose(host(z["b"]), params["b"], rtol=1e-4, atol=1e-4)


# ------------------------------------------------------------------ single-leaf quantizers
@pytest.mark.parametrize("n", [1, 2, 5, 1000, 65537])
@pytest.mark.parametrize("levels", [2, 3, 16, 256])
def test_uniform_quantize_bitwise(n, levels, cuda):
    v = (np.random.RandomState(n).standard_normal(n) * 0.1).astype(F32)
    key = jr.prng_key(n + levels)
    same(host(comp.uniform_stochastic_quantize(dev(v, cuda), levels, key)),
         cref.uniform_stochastic_quantize(v, levels, key))


def test_uniform_quantize_explicit_range_and_edges(cuda):
    v = np.linspace(-1, 1, 999).astype(F32)
    key = jr.prng_key(1)
    same(host(comp.uniform_stochastic_quantize(dev(v, cuda), 5, key, -2.0, 2.0)),
         cref.uniform_stochastic_quantize(v, 5, key, -2.0, 2.0))
    same(host(comp.uniform_stochastic_quantize(dev(v, cuda), 5, key, v_min=-0.5)),
         cref.uniform_stochastic_quantize(v, 5, key, v_min=-0.5))
    for arr, lv in [([0., 2., 2., 4.], 3), ([4., 4., 4., 4.], 4), ([0., 1., np.nan], 3), ([1., np.inf, 2.], 3)]:
        a = np.array(arr, F32)
        got = host(comp.uniform_stochastic_quantize(dev(a, cuda), lv, jr.prng_key(42)))
        exp = cref.uniform_stochastic_quantize(a, lv, jr.prng_key(42))
        npt.assert_array_equal(np.isnan(got), np.isnan(exp))
        same(np.nan_to_num(got), np.nan_to_num(exp))


@pytest.mark.parametrize("n", [3, 1001, 40000])
def test_binary_and_terngrad_bitwise(n, cuda):
    v = (np.random.RandomState(n).standard_normal(n)).astype(F32)
    v[0] = 40.0  # a clipped entry for terngrad
    key = jr.prng_key(7)
    same(host(comp.binary_stochastic_quantize(dev(v, cuda), key)), cref.binary_stochastic_quantize(v, key))
    same(host(comp.binary_stochastic_quantize(dev(v, cuda), key, 0.0, 3.0)),
         cref.binary_stochastic_quantize(v, key, 0.0, 3.0))
    same(host(comp.terngrad_quantize(dev(v, cuda), key)), cref.terngrad_quantize(v, key))


def test_reference_single_leaf_cases(cuda):  # compression_test.py:30-76, 167-185
    k42 = jr.prng_key(42)
    npt.assert_array_equal(host(comp.binary_stochastic_quantize(dev(np.array([0., 2., 2.], F32), cuda), k42)),
                           [0., 2., 2.])
    npt.assert_array_equal(host(comp.uniform_stochastic_quantize(dev(np.array([0., 2., 2., 4.], F32), cuda), 3,
                                                                 k42)), [0., 2., 2., 4.])
    npt.assert_array_equal(host(comp.uniform_stochastic_quantize(dev(np.array([4.] * 4, F32), cuda), 4, k42)),
                           [4.] * 4)
    npt.assert_array_equal(host(comp.terngrad_quantize(dev(np.array([0., 2., 2.], F32), cuda), k42)), [0., 2., 2.])
    v = np.zeros(100, F32)
    v[0], v[1] = 100, -100
    e = v.copy()
    e[0], e[1] = 35.355339, -35.355339
    npt.assert_array_equal(host(comp.terngrad_quantize(dev(v, cuda), k42)), e)
    for arr, lv, dec in [([0., 1., 100.], 125, 2), ([[0., 1., 100.], [0.3, 2.3, 45.]], 125, 1)]:
        a = np.array(arr, F32)
        rng, s = jr.prng_key(42), np.zeros_like(a)
        for _ in range(500):
            rng, use = jr.split(rng)
            s += host(comp.uniform_stochastic_quantize(dev(a, cuda), lv, use))
        npt.assert_array_almost_equal(s / 500, a, decimal=dec)


def test_arithmetic_encoding_num_bits(cuda):  # compression_test.py:78-81
    v = np.array([1., 2., 3., 4., 5.], F32)
    got = comp.arithmetic_encoding_num_bits(dev(v, cuda))
    npt.assert_array_almost_equal(got, [89.82311], decimal=3)
    assert got == cref.arithmetic_encoding_num_bits(v)


def test_drive_pytree(cuda):  # compression_test.py:139-143
    y = comp.drive_pytree({"w": dev(np.array([1., -2., 3.], F32), cuda)})
    npt.assert_array_almost_equal(host(y["w"]), [2.333333, -2.333333, 2.333333], decimal=4)


def test_quantize_pytrees_bitwise(cuda):
    t = _tree(np.random.RandomState(3))
    key = jr.prng_key(9)
    got = comp.uniform_stochastic_quantize_pytree(_to_dev(t, cuda), 16, key)
    exp = cref.uniform_stochastic_quantize_pytree(t, 16, key)
    for a, b in zip(_leaves(got), _leaves(exp)):
        same(host(a), b)
    got = comp.terngrad_quantize_pytree(_to_dev(t, cuda), key)
    exp = cref.terngrad_quantize_pytree(t, key)
    for a, b in zip(_leaves(got), _leaves(exp)):
        same(host(a), b)


# ------------------------------------------------------------------ aggregators: reference tests
def test_uniform_stochastic_quantizer(cuda):  # compression_test.py:83-99
    q = comp.uniform_stochastic_quantizer(3, random.PRNGKey(0))
    p, st = q.apply(_clients(cuda), q.init())
    assert st.num_bits == 68.75489
    npt.assert_array_equal(host(p["w"]), [1.5, 3.25, 5.])


def test_uniform_stochastic_quantizer_arithmetic_coding(cuda):  # :101-117
    q = comp.uniform_stochastic_quantizer(3, random.PRNGKey(0), "arithmetic")
    p, st = q.apply(_clients(cuda), q.init())
    assert st.num_bits == 78.08298
    npt.assert_array_equal(host(p["w"]), [1.5, 3.25, 5.])


def test_rotated_uniform_stochastic_quantizer(cuda):  # :119-137
    q = comp.rotated_uniform_stochastic_quantizer(2, random.PRNGKey(0))
    st, ps = q.init(), []
    for _ in range(2000):
        p, st = q.apply(_clients(cuda), st)
        ps.append(host(p["w"]))
    assert st.num_bits == 67 * 2000
    npt.assert_array_almost_equal(np.mean(ps, axis=0), [1.5, 3.25, 5.], decimal=1)


def test_structured_drive_quantizer(cuda):  # :145-165
    q = comp.structured_drive_quantizer(random.PRNGKey(0))
    st, ps = q.init(), []
    for _ in range(100):
        p, st = q.apply(_clients(cuda), st)
        ps.append(host(p["w"]))
    assert st.num_bits == 67 * 100
    npt.assert_array_almost_equal(sum(ps) / 100, [1.458334, 1.458334, 6.125], decimal=4)


def test_terngrad_quantizer(cuda):  # :187-203
    q = comp.terngrad_quantizer(random.PRNGKey(0))
    p, st = q.apply(_clients(cuda), q.init())
    assert st.num_bits == 68.75489
    npt.assert_array_almost_equal(host(p["w"]), [0.51031, 2.551552, 3.572173], decimal=4)


# ------------------------------------------------------------------ aggregators: bitwise vs oracle
@pytest.mark.parametrize("levels,enc", [(4, None), (256, None), (16, "arithmetic")])
def test_uniform_quantizer_bitwise(levels, enc, cuda):
    clients, ref_clients = _fleet(cuda)
    q = comp.uniform_stochastic_quantizer(levels, random.PRNGKey(5), enc)
    init, apply = cref.uniform_stochastic_quantizer(levels, jr.prng_key(5), enc)
    st, rst = q.init(), init()
    for _ in range(2):
        p, st = q.apply(iter(clients), st)
        rp, rst = apply(ref_clients, rst)
        for a, b in zip(_leaves(p), _leaves(rp)):
            same(host(a), b)
        assert st.num_bits == rst.num_bits
        npt.assert_array_equal(st.rng, rst.rng)


SMALL = {"b": (17,), "w": (3001,)}


@pytest.mark.parametrize("K", [257, 300, 513])
@pytest.mark.parametrize("kind", ["uniform16", "arithmetic", "terngrad"])
def test_quantizers_many_clients_bitwise(K, kind, cuda):
    """More clients than k_quant_fold stages in LDS at once (256): the per-client constants
    are restaged per chunk and the delta look-ahead restarts at each chunk boundary."""
    rs = np.random.RandomState(K)
    trees = [_tree(rs, shapes=SMALL) for _ in range(K)]
    w = [int(v) for v in rs.randint(1, 500, K)]
    clients = [(f"c{k}", _to_dev(t, cuda), w[k]) for k, t in enumerate(trees)]
    ref_clients = [(f"c{k}", t, w[k]) for k, t in enumerate(trees)]
    if kind == "terngrad":
        q, (init, apply) = comp.terngrad_quantizer(random.PRNGKey(6)), cref.terngrad_quantizer(jr.prng_key(6))
    else:
        enc = "arithmetic" if kind == "arithmetic" else None
        q = comp.uniform_stochastic_quantizer(16, random.PRNGKey(6), enc)
        init, apply = cref.uniform_stochastic_quantizer(16, jr.prng_key(6), enc)
    p, st = q.apply(clients, q.init())
    rp, rst = apply(ref_clients, init())
    for a, b in zip(_leaves(p), _leaves(rp)):
        same(host(a), b)
    assert st.num_bits == rst.num_bits


def test_terngrad_quantizer_bitwise(cuda):
    clients, ref_clients = _fleet(cuda, seed=1)
    q = comp.terngrad_quantizer(random.PRNGKey(2))
    init, apply = cref.terngrad_quantizer(jr.prng_key(2))
    p, st = q.apply(clients, q.init())
    rp, rst = apply(ref_clients, init())
    for a, b in zip(_leaves(p), _leaves(rp)):
        same(host(a), b)
    assert st.num_bits == rst.num_bits


@pytest.mark.parametrize("ws", [None, 300_000])
def test_rotated_quantizer_bitwise(ws, cuda):
    clients, ref_clients = _fleet(cuda, K=5, seed=2)
    kw = {} if ws is None else {"workspace_bytes": ws}  # 300 kB: one client per batch
    q = comp.rotated_uniform_stochastic_quantizer(4, random.PRNGKey(8), **kw)
    p, st = q.apply(clients, q.init())
    init, apply = cref.rotated_uniform_stochastic_quantizer(4, jr.prng_key(8), commute_inverse=True)
    rp, rst = apply(ref_clients, init())
    for a, b in zip(_leaves(p), _leaves(rp)):
        same(host(a), b)
    assert st.num_bits == rst.num_bits
    # the reference order (invert per client, then average) differs by float32 reassociation only
    init, apply = cref.rotated_uniform_stochastic_quantizer(4, jr.prng_key(8))
    rp2, _ = apply(ref_clients, init())
    for a, b in zip(_leaves(p), _leaves(rp2)):
        npt.assert_allclose(host(a), b, rtol=0, atol=1e-5 * float(np.abs(b).max()) + 1e-30)


@pytest.mark.parametrize("ws", [None, 300_000])
def test_drive_quantizer_bitwise(ws, cuda):
    clients, ref_clients = _fleet(cuda, K=5, seed=3)
    kw = {} if ws is None else {"workspace_bytes": ws}
    q = comp.structured_drive_quantizer(random.PRNGKey(4), **kw)
    init, apply = cref.structured_drive_quantizer(jr.prng_key(4))
    st, rst = q.init(), init()
    for _ in range(2):
        p, st = q.apply(clients, st)
        rp, rst = apply(ref_clients, rst)
        for a, b in zip(_leaves(p), _leaves(rp)):
            same(host(a), b)
        assert st.num_bits == rst.num_bits


def test_empty_round_and_key_advance(cuda):
    q = comp.uniform_stochastic_quantizer(3, random.PRNGKey(0))
    p, st = q.apply([], q.init())
    assert p is None and st.num_bits == 0
    npt.assert_array_equal(st.rng, jr.split(jr.prng_key(0))[0])


def test_bf16_leaves_rejected(cuda):
    q = comp.uniform_stochastic_quantizer(3, random.PRNGKey(0))
    with pytest.raises(TypeError):
        q.apply([("a", {"w": torch.ones(4, dtype=torch.bfloat16, device=cuda)}, 1.)], q.init())


def test_mismatched_client_shapes_rejected(cuda):
    q = comp.terngrad_quantizer(random.PRNGKey(0))
    bad = [("a", {"w": torch.ones(4, device=cuda)}, 1.), ("b", {"w": torch.ones(3, device=cuda)}, 1.)]
    with pytest.raises(ValueError):
        q.apply(bad, q.init())
