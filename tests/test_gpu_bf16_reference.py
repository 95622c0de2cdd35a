"""bfloat16 leaves under the reference's arithmetic (``set_bf16_semantics("reference")``,
fjagg acc dtype FJAGG_BF16): with bf16 leaves and weakly typed weights, the reference's
jnp ops (fedjax/core/tree_util.py:32 ``l * weight``, :50 ``jnp.add``, :60 the inverse
weight) turn every weight and 1/W into bf16 and round every product and sum to bf16.

The checker is a numpy restatement of that sequence (``refsem`` below: each op in f32,
then rounded to bf16 — the f32 product of two bf16 values is exact, and f32 has the
2p + 2 bits that make the sum's double rounding innocuous), cross-checked against the C
oracle's ``oracle_wsum_bf16_refsem`` (oracle/fold_ref.c). JAX is absent here, so the
restatement is pinned by its definition, not by a JAX run ("parity unpinned" in the
sense of SURVEY §8c: no reference fixture holds bf16 outputs). Every comparison is
bitwise (NaN matches NaN).
"""
import numpy as np
import pytest
import torch

import fedjax_amd
from fedjax_amd import aggregators, kernels, pytree, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu


def rnd(a):
    """float32 -> nearest bfloat16 value (RNE), as float32; NaN stays NaN."""
    a = np.asarray(a, dtype=np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    r = (((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16).astype(np.uint32).view(np.float32)
    return np.where(np.isnan(a), np.float32(np.nan), r).astype(np.float32)


def bits(a):
    """bfloat16 bits of bf16-representable float32 values."""
    return (np.asarray(a, np.float32).view(np.uint32) >> 16).astype(np.uint16)


def refsem(xs, ws, scale=None, init=None):
    """The reference's bf16 fold: t_k = bf16(x_k * bf16(w_k)); s_0 = t_0 (or bf16(init +
    t_0)); s_k = bf16(s_{k-1} + t_k); y = bf16(s * bf16(f32(scale))). xs: K float32 arrays
    holding bf16 values."""
    s = None
    for x, w in zip(xs, ws):
        t = rnd(x * rnd(np.float32(w)))
        s = (t if init is None else rnd(init + t)) if s is None else rnd(s + t)
    if scale is not None:
        s = rnd(s * rnd(np.float32(scale)))
    return s


def same_bits(got_u16, want_f32):
    g = np.asarray(got_u16, np.uint16)
    w = bits(want_f32)
    nan = np.isnan((g.astype(np.uint32) << 16).view(np.float32)) & np.isnan(want_f32)
    return bool(np.all((g == w) | nan))


def host_u16(t):
    return t.detach().cpu().view(torch.int16).numpy().view(np.uint16)


def to_bf16_dev(a_f32, dev):
    return torch.from_numpy(bits(a_f32).view(np.int16)).view(torch.bfloat16).to(dev)


@pytest.fixture
def reference_mode():
    tu.set_bf16_semantics("reference")
    yield
    tu.set_bf16_semantics("f32")


def test_restatement_matches_the_c_oracle(coracle):
    K, P = 23, 777
    xb = coracle.synth_bf16(K, P, seed=31)
    xs = [(xb[k].astype(np.uint32) << 16).view(np.float32) for k in range(K)]
    w = np.float32(ref.fedavg_weights(K, seed=32))
    r = np.float32(1.0 / float(w.astype(np.float64).sum()))
    assert np.array_equal(coracle.wsum_bf16_refsem(xb, w, r), bits(refsem(xs, w, r)))


@pytest.mark.parametrize("K,P,offset", [(37, 1000, 0), (64, 300_000, 0), (40, 70_001, 1), (5, 5000, 0),
                                        (200, 20_000, 0), (130, 1_100_000, 0), (32, 2_100_000, 0),
                                        (8, 100_001, 1)])
def test_dense_reference_fold_bitwise(cuda, coracle, K, P, offset):
    """Every dense shape family: narrow LDS stripes, E=8/E=4/E=1 lanes, element units
    (odd offset), the tail, K < 16."""
    xb = coracle.synth_bf16(K, P + offset, seed=K)
    x = torch.from_numpy(xb.view(np.int16)).view(torch.bfloat16).to(cuda)[:, offset:]
    xs = [(xb[k, offset:].astype(np.uint32) << 16).view(np.float32) for k in range(K)]
    wi = ref.fedavg_weights(K, seed=K + 1)
    W = float(wi.astype(np.float64).sum())
    r = 1.0 / W
    wd = torch.tensor(np.float32(wi), device=cuda)
    y = kernels.weighted_sum_dense(x, wd, scale=float(np.float32(r)), reference_bf16=True)
    assert y.dtype == torch.bfloat16
    assert same_bits(host_u16(y), refsem(xs, wi, r))
    # the C oracle agrees on the same inputs (contiguous rows only)
    if offset == 0:
        assert np.array_equal(host_u16(y), coracle.wsum_bf16_refsem(xb, np.float32(wi), np.float32(r)))
    # accumulate mode: s = bf16(out + t_0), then the chain
    init = rnd(np.linspace(-1, 1, P).astype(np.float32))
    out = to_bf16_dev(init, cuda)
    kernels.weighted_sum_dense(x, wd, out=out, accumulate=True, reference_bf16=True)
    assert same_bits(host_u16(out), refsem(xs, wi, init=init))


def test_weights_round_to_bf16(cuda):
    """257 is not a bf16 value: the reference multiplies by bf16(257) = 256."""
    x = to_bf16_dev(np.array([1.0, 3.0, -0.5], np.float32), cuda).reshape(1, 3)
    w = torch.tensor([257.0], device=cuda)
    y = kernels.weighted_sum_dense(x, w, reference_bf16=True)
    assert np.array_equal(host_u16(y), bits(np.array([256.0, 768.0, -128.0], np.float32)))
    y32 = kernels.weighted_sum_dense(x, w)  # f32 semantics: 257 * 3 = 771 -> bf16 772
    assert np.array_equal(host_u16(y32), bits(rnd(np.array([257.0, 771.0, -128.5], np.float32))))


def test_split_mode_refused(cuda):
    x = torch.zeros(64, 4096, dtype=torch.bfloat16, device=cuda)
    with pytest.raises(fedjax_amd._lib.FjaggError):
        kernels.weighted_sum_dense(x, torch.ones(64, device=cuda), mode="split", reference_bf16=True)


def _trees(K, shapes, seed, dev, views=False):
    g = np.random.RandomState(seed)
    host = [[rnd((g.rand(*s).astype(np.float32) * 2 - 1) * 0.1) for s in shapes] for _ in range(K)]
    out = []
    for leaves in host:
        if views:  # one buffer, leaves at odd element offsets (2-byte aligned rows)
            buf = torch.empty(sum(int(np.prod(s)) for s in shapes) + 2 * len(shapes) + 1, dtype=torch.bfloat16,
                              device=dev)
            off, ls = 1, []
            for a in leaves:
                v = buf[off:off + a.size].view(a.shape)
                v.copy_(to_bf16_dev(a, dev).view(a.shape))
                ls.append(v)
                off += a.size + 2
        else:
            ls = [to_bf16_dev(a, dev).view(a.shape) for a in leaves]
        out.append({"a": ls[0], "b": {"c": ls[1], "d": ls[2]}})
    return out, host


@pytest.mark.parametrize("views", [False, True])
def test_pytree_surface_bitwise(cuda, reference_mode, views):
    """tree_mean (one launch; K >= 16 small trees take the LDS-staged stripes), tree_sum,
    mean_aggregator, the library loop of fed_avg.py:132-146 through the per-call ops, and
    RunningMean — all the reference's bf16 sequence."""
    shapes = [(1001,), (33, 7), (4096,)]
    for K in (3, 40):
        trees, host = _trees(K, shapes, seed=K, dev=cuda, views=views)
        ws = [int(v) for v in np.random.RandomState(K).randint(1, 501, size=K)]
        W = 0.0
        for w in ws:
            W += w
        want = [refsem([h[l] for h in host], ws, 1.0 / W) for l in range(3)]
        got = pytree.leaves_of(tu.tree_mean(list(zip(trees, ws))))
        assert all(g.dtype == torch.bfloat16 for g in got)
        assert all(same_bits(host_u16(g).reshape(-1), w.reshape(-1)) for g, w in zip(got, want))
        agg = aggregators.mean_aggregator()
        got, _ = agg.apply(((str(k), t, w) for k, (t, w) in enumerate(zip(trees, ws))), agg.init())
        assert all(same_bits(host_u16(g).reshape(-1), w.reshape(-1)) for g, w in zip(pytree.leaves_of(got), want))
        want_sum = [refsem([h[l] for h in host], [1] * K) for l in range(3)]
        got = pytree.leaves_of(tu.tree_sum(trees))
        assert all(same_bits(host_u16(g).reshape(-1), w.reshape(-1)) for g, w in zip(got, want_sum))
        # the library loop: zeros, tree_add(s, tree_weight(x, n)), tree_inverse_weight
        s = tu.tree_zeros_like(trees[0])
        for t, w in zip(trees, ws):
            s = tu.tree_add(s, tu.tree_weight(t, w))
        loop = pytree.leaves_of(tu.tree_inverse_weight(s, W))
        want_loop = [refsem([h[l] for h in host], ws, 1.0 / W, init=np.zeros(host[0][l].shape, np.float32))
                     for l in range(3)]
        assert all(same_bits(host_u16(g).reshape(-1), w.reshape(-1)) for g, w in zip(loop, want_loop))
        rm = aggregators.RunningMean(trees[0], buffer_clients=7)
        for t, w in zip(trees, ws):
            rm.add(t, w)
        got = pytree.leaves_of(rm.result())
        assert all(same_bits(host_u16(g).reshape(-1), w.reshape(-1)) for g, w in zip(got, want_loop))


def test_strong_weights_promote_to_f32_in_both_modes(cuda, reference_mode):
    """A numpy float32 weight is strongly typed: bf16 * f32 -> the f32 fold of the
    reference (tree_util.py:32 under jnp promotion), float32 output."""
    trees, host = _trees(6, [(100,), (5, 5), (17,)], seed=3, dev=cuda)
    ws = [np.float32(v) for v in np.random.RandomState(4).rand(6)]
    got = pytree.leaves_of(tu.tree_mean(list(zip(trees, ws))))
    np_trees = [{"a": h[0], "b": {"c": h[1], "d": h[2]}} for h in host]
    want = ref.flatten(ref.tree_mean(list(zip(np_trees, ws))))[0]
    assert all(g.dtype == torch.float32 for g in got)
    assert all(np.array_equal(g.cpu().numpy().view(np.uint32), w.view(np.uint32)) for g, w in zip(got, want))


def test_mean_with_norms_and_slab_in_reference_mode(cuda, reference_mode):
    trees, host = _trees(20, [(300,), (4, 4), (2000,)], seed=5, dev=cuda)
    ws = list(range(1, 21))
    W = float(sum(ws))
    mean, norms = tu.tree_mean_with_l2_norms(list(zip(trees, ws)))
    want = [refsem([h[l] for h in host], ws, 1.0 / W) for l in range(3)]
    assert all(same_bits(host_u16(g).reshape(-1), w.reshape(-1)) for g, w in zip(pytree.leaves_of(mean), want))
    n64 = np.array([np.sqrt(sum(float(np.dot(a.astype(np.float64).ravel(), a.astype(np.float64).ravel()))
                                for a in h)) for h in host])
    assert np.allclose(norms.cpu().numpy(), n64, rtol=2e-6)
    # the slab: one dense launch with the reference's arithmetic
    template = {"a": np.zeros(300, np.float32), "b": {"c": np.zeros((4, 4), np.float32), "d": np.zeros(2000, np.float32)}}
    slab = fedjax_amd.ClientDeltaSlab(template, 20, dtype=torch.bfloat16, device=cuda)
    for k, t in enumerate(trees):
        slab.set_client(k, t)
    m, n = slab.mean(ws, with_norms=True)
    assert all(same_bits(host_u16(g).reshape(-1), w.reshape(-1)) for g, w in zip(pytree.leaves_of(m), want))
    assert np.allclose(n.cpu().numpy(), n64, rtol=2e-6)


def test_default_mode_is_the_f32_fold(cuda):
    assert tu.bf16_semantics() == "f32"
    trees, host = _trees(9, [(500,), (3, 3), (64,)], seed=6, dev=cuda)
    ws = list(range(1, 10))
    got = pytree.leaves_of(tu.tree_mean(list(zip(trees, ws))))
    W = float(sum(ws))
    for l, g in enumerate(got):
        s = None
        for h, w in zip(host, ws):
            t = h[l] * np.float32(w)
            s = t if s is None else s + t
        assert same_bits(host_u16(g).reshape(-1), rnd(s * np.float32(1.0 / W)).reshape(-1))
