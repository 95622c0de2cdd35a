"""GPU parity: the HIP path (through the C ABI) against the oracle.

Bar: float32 / int32 exact mode bitwise equal to the reference
restatement; split mode and multi-rank within the sequential-summation bound
|y - y_ref| <= (K + G + 2) * 2^-24 * |r| * sum_k |fl(x_k w_k)| + 2^-24 |y_ref|;
bfloat16 within one bf16 rounding of the f64 oracle plus that bound.
"""
import numpy as np
import numpy.testing as npt
import pytest
import torch

import fedjax_amd
from fedjax_amd import _lib, kernels, tree_util as tu
from oracle import tree_util_ref as ref
from tests import fedavg_restated as fr
from tests import golden_cases as gc
from tests.coracle import bf16_to_f32

pytestmark = pytest.mark.gpu
U = 2.0 ** -24


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype.itemsize == 4 else np.uint16)


def host(t):
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


# ------------------------------------------------------------------ golden fixtures
@pytest.mark.parametrize("name", gc.NAMES)
def test_golden_fixture_on_gpu(name, cuda, coracle):
    c = gc.load(name)
    x, shapes = c["x"], c["shapes"]
    if name.startswith("bf16"):
        xt = torch.from_numpy(x.view(np.int16)).view(torch.bfloat16).to(cuda)
    else:
        xt = torch.from_numpy(x).to(cuda)
    trees = [gc.split_leaves(xt[k], shapes) for k in range(x.shape[0])]
    m = tu.tree_mean(zip(trees, c["weight_list"]))
    got = np.concatenate([host(v).ravel() for v in m])
    if name.startswith("bf16"):
        y = bf16_to_f32(got).astype(np.float64)
        y64 = c["y_f64"]
        w = np.float32(c["weight_list"])
        r = np.float32(1.0 / sum(c["weight_list"]))
        xf = bf16_to_f32(x)
        tsum = np.abs(xf.astype(np.float64) * w[:, None]).sum(0)
        tol = 2.0 ** -8 * np.abs(y64) + (x.shape[0] + 3) * U * r * tsum
        assert np.all(np.abs(y - y64) <= tol)
        # and far closer than the reference's own bf16 arithmetic
        err_ref = np.abs(bf16_to_f32(c["y_refsem"]) - y64).max()
        assert np.abs(y - y64).max() <= err_ref
    else:
        assert np.array_equal(bits(got), bits(c["y"])), name


# ------------------------------------------------------------- reference KATs on GPU
def test_mean_aggregator_kat(cuda):
    # fedjax/aggregators/aggregator_test.py:24-37
    d = [("a", {"w": torch.tensor([1., 2., 3.], device=cuda)}, 2.),
         ("b", {"w": torch.tensor([2., 4., 6.], device=cuda)}, 4.),
         ("c", {"w": torch.tensor([1., 3., 5.], device=cuda)}, 2.)]
    agg = fedjax_amd.aggregators.mean_aggregator()
    state = agg.init()
    mean, new_state = agg.apply(d, state)
    npt.assert_array_equal(host(mean["w"]), [1.5, 3.25, 5.])
    assert new_state is state


def test_aggregator_consumes_generator_once(cuda):
    gen = ((str(k), {"w": torch.full((5,), float(k), device=cuda)}, 1) for k in range(4))
    mean, _ = fedjax_amd.aggregators.mean_aggregator().apply(gen, None)
    npt.assert_array_equal(host(mean["w"]), np.full(5, 1.5, np.float32))


def test_tree_weight_sum_mean_kats(cuda):
    # fedjax/core/tree_util_test.py:27-62
    p1 = {"x": torch.tensor([[[4, 5]], [[1, 1]]], device=cuda), "y": torch.tensor([[3], [1]], device=cuda)}
    p2 = {"x": torch.tensor([[[2, 3]], [[4, 5]]], device=cuda), "y": torch.tensor([[6], [7]], device=cuda)}
    w = tu.tree_weight(p1, 2.0)
    npt.assert_array_equal(host(w["x"]), [[[8.0, 10.0]], [[2.0, 2.0]]])
    npt.assert_array_equal(host(w["y"]), [[6.0], [2.0]])
    assert w["x"].dtype == torch.float32
    before = [t.clone() for t in (p1["x"], p1["y"], p2["x"], p2["y"])]
    s = tu.tree_sum([p1, p2])
    npt.assert_array_equal(host(s["x"]), [[[6, 8]], [[5, 6]]])
    npt.assert_array_equal(host(s["y"]), [[9], [8]])
    assert s["x"].dtype == torch.int32
    for a, b in zip(before, (p1["x"], p1["y"], p2["x"], p2["y"])):
        assert torch.equal(a, b)  # inputs are never written (tree_util_test.py:50-51)
    trees = [(torch.tensor(0, device=cuda), torch.tensor(1, device=cuda)),
             (torch.tensor(2, device=cuda), torch.tensor(3, device=cuda)),
             (torch.tensor(4, device=cuda), torch.tensor(5, device=cuda))]
    m = tu.tree_mean(zip(trees, [6., 7., 8.]))
    npt.assert_array_almost_equal([host(v) for v in m], (2.1904761904761907, 3.1904761904761907))
    assert tu.tree_mean([]) is None and tu.tree_sum([]) is None
    assert tu.tree_size(p1) == 6


def test_tree_clip_and_norm_kats(cuda):
    # fedjax/core/tree_util_test.py:64-73
    p = {"x": torch.tensor([[[4., 5.]], [[1., 1.]]], device=cuda), "y": torch.tensor([[3.], [1.]], device=cuda)}
    npt.assert_allclose(host(tu.tree_l2_norm(p)), 7.28011, rtol=1e-6)
    npt.assert_allclose(host(tu.tree_l2_squared(p)), 53.0, rtol=1e-7)
    c = tu.tree_clip_by_global_norm(p, 3.640055)
    npt.assert_array_almost_equal(host(c["x"]), [[[2, 2.5]], [[0.5, 0.5]]])
    npt.assert_array_almost_equal(host(c["y"]), [[1.5], [0.5]])


@pytest.mark.parametrize("name,round_fn,bs,epochs,want,want_norms", fr.KATS)
def test_fedavg_round_kats_on_gpu(name, round_fn, bs, epochs, want, want_norms, cuda):
    new, norms = round_fn(tu, lambda a: torch.from_numpy(np.asarray(a)).to(cuda), host,
                          fr.SERVER_PARAMS, fr.CLIENTS, bs, epochs, 0)
    npt.assert_allclose(new["w"], want, err_msg=name)
    for cid, v in want_norms.items():
        npt.assert_allclose(norms[cid], v, rtol=1e-6, err_msg=name)


def test_host_resident_leaves_are_copied(cuda):
    trees = [({"w": np.full(3, float(k), np.float32)}, 1) for k in range(3)]
    m = tu.tree_mean(trees)
    assert m["w"].is_cuda
    npt.assert_array_equal(host(m["w"]), [1., 1., 1.])


def test_tree_add_zeros_inverse(cuda):
    a = {"p": torch.arange(10, dtype=torch.float32, device=cuda)}
    z = tu.tree_zeros_like(a)
    s = tu.tree_add(z, tu.tree_weight(a, 3))
    s = tu.tree_inverse_weight(s, 3.0)
    want = ref.tree_inverse_weight(ref.tree_add(np.zeros(10, np.float32), np.arange(10, dtype=np.float32) * 3), 3.0)
    assert np.array_equal(bits(host(s["p"])), bits(want))


def test_error_behaviour(cuda):
    with pytest.raises(ValueError):
        tu.tree_mean([({"a": torch.ones(3, device=cuda)}, 1), ({"b": torch.ones(3, device=cuda)}, 1)])
    with pytest.raises(ValueError):
        tu.tree_mean([({"a": torch.ones(3, device=cuda)}, 1), ({"a": torch.ones(4, device=cuda)}, 1)])
    with pytest.raises(TypeError):
        tu.tree_mean([({"a": torch.ones(3, dtype=torch.float16, device=cuda)}, 1)])
    with pytest.raises(ValueError):
        kernels.weighted_sum_dense(torch.ones(2, 8), torch.ones(2))


# ------------------------------------------------------------------- dense kernel
SHAPES = [(1, 1), (1, 5), (2, 4), (3, 7), (37, 10007), (130, 12291), (9, 2 ** 16 + 3), (1000, 333)]


@pytest.mark.parametrize("K,P", SHAPES)
def test_dense_all_variants_bitwise(K, P, cuda, coracle):
    x = torch.empty(K, P, dtype=torch.float32, device=cuda)
    kernels.fill_synth(x, seed=K * 7 + P)
    xh = coracle.synth_f32(K, P, seed=K * 7 + P)
    assert np.array_equal(bits(host(x)), bits(xh))
    wi = [int(v) for v in ref.fedavg_weights(K, seed=P)]
    r = ref.mean_scale(wi)
    want = coracle.wsum_f32(xh, np.float32(wi), scale=r)
    w = torch.tensor(np.float32(wi), device=cuda)
    for variant in list(range(18)) + [18]:  # 18: k_dense_narrow (LDS-staged, one element per lane)
        for nt, bal in ((False, True), (True, True), (True, False)):
            y = kernels.weighted_sum_dense(x, w, scale=float(r), variant=variant, nontemporal=nt, balanced=bal)
            assert np.array_equal(bits(host(y)), bits(want)), (variant, nt, bal)


@pytest.mark.parametrize("K,P,dt,offset", [(300, 65536 + 7, "f32", 1), (129, 200, "bf16", 0), (1024, 4096, "f32", 0),
                                           (2, 70, "i32", 3), (257, 33, "f32", 2)])
def test_narrow_fold_bitwise_every_dtype_and_alignment(K, P, dt, offset, cuda, coracle):
    """k_dense_narrow (variant 18): clients not a multiple of its 128-client tile, columns
    not a multiple of its 64-element stripe, rows at odd element offsets (any alignment),
    accumulate mode, bf16 in/out, wrapping int32 — bitwise the other variants' fold."""
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "i32": torch.int32}[dt]
    base = torch.empty(K, P + offset + 5, dtype=torch.float32, device=cuda)
    kernels.fill_synth(base, seed=K + P)
    if dt == "i32":
        x = (base * 1e6).to(torch.int32)[:, offset:offset + P]
        w = torch.tensor([int(v) for v in ref.fedavg_weights(K, seed=3)], dtype=torch.int32, device=cuda)
    else:
        x = base.to(tdt)[:, offset:offset + P]
        w = torch.tensor(np.float32(ref.fedavg_weights(K, seed=3)), device=cuda)
    scale = None if dt == "i32" else 0.125
    for acc in (False, True):
        outs = []
        for variant in (2, 18):
            o = torch.full((P,), 3, dtype=x.dtype, device=cuda) if acc else None
            outs.append(kernels.weighted_sum_dense(x, w, scale=scale, variant=variant, out=o, accumulate=acc))
        assert torch.equal(outs[0].view(torch.uint8), outs[1].view(torch.uint8)), (dt, acc)
    if dt == "f32" and offset == 1:  # and against the oracle
        want = coracle.wsum_f32(np.ascontiguousarray(host(x)), host(w), scale=np.float32(scale))
        y18 = kernels.weighted_sum_dense(x, w, scale=scale, variant=18)
        assert np.array_equal(bits(host(y18)), bits(want))


STRIPE_CASES = [  # (K, P, dtype): tiles of 192 / 384 / 768 clients, stripes of 64 / 32 / 16 columns
    (16384, 4096, "f32"), (4096, 16384, "f32"), (1000, 4101, "f32"), (193, 70, "f32"), (16, 33, "f32"),
    (769, 2048 + 8, "bf16"), (385, 300, "bf16"), (300, 1000, "i32"), (2000, 9000, "f32")]


@pytest.mark.parametrize("K,P,dt", STRIPE_CASES)
def test_stripe_fold_bitwise(K, P, dt, cuda, coracle):
    """k_dense_stripe (variants 19-22: auto, 64, 32, 16 columns; fjstripe.hip): tiles not
    full (K not a multiple of 192 / 384 / 768, K below one tile), stripes not full, rows
    padded to 16 bytes, accumulate mode, bf16 in / out, the bf16 reference fold, wrapping
    int32 and int32 -> f32 — bitwise the E1U8 fold (variant 2) and, for f32, the oracle."""
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "i32": torch.int32}[dt]
    es = torch.empty((), dtype=tdt).element_size()
    ld = (P + 16 // es - 1) // (16 // es) * (16 // es) + 16 // es  # a padded, 16-byte multiple row
    base = torch.empty(K, ld, dtype=torch.float32, device=cuda)
    kernels.fill_synth(base, seed=K + 3 * P)
    if dt == "i32":
        x = (base * 1e6).to(torch.int32)[:, :P]
        wsets = [torch.tensor([int(v) for v in ref.fedavg_weights(K, seed=5)], dtype=torch.int32, device=cuda),
                 torch.tensor(np.float32(ref.fedavg_weights(K, seed=6)), device=cuda)]
    else:
        x = base.to(tdt)[:, :P]
        wsets = [torch.tensor(np.float32(ref.fedavg_weights(K, seed=5)), device=cuda)]
    assert x.stride(0) * es % 16 == 0 and x.data_ptr() % 16 == 0
    for w in wsets:
        scale = None if w.dtype == torch.int32 else 0.125
        modes = [dict()]
        if dt == "bf16":
            modes += [dict(reference_bf16=True), dict(out_dtype=torch.float32)]
        if dt == "f32":
            modes += [dict(out_dtype=torch.bfloat16)]
        for kw in modes:
            for acc in (False, True):
                outs = []
                for variant in (2, 19, 20, 21, 22):
                    o = None
                    if acc:
                        probe = kernels.weighted_sum_dense(x[:1], w[:1], scale=scale, **kw)
                        o = torch.full((P,), 3, dtype=probe.dtype, device=cuda)
                    for nt in (False, True):
                        oo = None if o is None else o.clone()
                        outs.append((variant, nt, kernels.weighted_sum_dense(
                            x, w, scale=scale, variant=variant, out=oo, accumulate=acc, nontemporal=nt, **kw)))
                ref_out = outs[0][2].view(torch.uint8)
                for variant, nt, y in outs[1:]:
                    assert torch.equal(y.view(torch.uint8), ref_out), (dt, kw, acc, variant, nt, w.dtype)
    if dt == "f32":  # and against the oracle
        w = wsets[0]
        want = coracle.wsum_f32(np.ascontiguousarray(host(x)), host(w), scale=np.float32(0.125))
        y = kernels.weighted_sum_dense(x, w, scale=0.125, variant=19)
        assert np.array_equal(bits(host(y)), bits(want))


def test_stripe_fold_special_values(cuda, coracle):
    """-0 / NaN / Inf / subnormal deltas and weights through k_dense_stripe: the -0.0 start
    and padding of the stripe pipeline keep every bit of the reference sequence."""
    K, P = 800, 256
    x = torch.empty(K, P, dtype=torch.float32, device=cuda)
    kernels.fill_synth(x, seed=9)
    x[0, :8] = torch.tensor([-0.0, 0.0, float("nan"), float("inf"), -float("inf"), 1e-45, -1e-45, -0.0])
    x[:, 8] = -0.0  # a column that stays -0 throughout: s_0 = -0*w... = -0, sums of -0 stay -0
    x[5, 9] = float("nan")
    w = torch.tensor(np.float32(ref.fedavg_weights(K, seed=8)), device=cuda)
    w[3] = -0.0
    w[4] = 1e-40
    want = coracle.wsum_f32(np.ascontiguousarray(host(x)), host(w), scale=np.float32(0.5))
    for variant in (19, 20, 21, 22):
        y = kernels.weighted_sum_dense(x, w, scale=0.5, variant=variant)
        assert np.array_equal(bits(host(y)), bits(want)), variant


@pytest.mark.parametrize("variant", [0, 2, 5, 12, 16, 17])
def test_f32_in_bf16_out_units(variant, cuda, coracle):
    """(F32, F32, BF16): a float32 16-byte unit holds 4 elements, i.e. 8 bytes of bf16
    output. Round 2's store wrote 16 bytes per unit (4 of them the next unit's), so the
    bf16 cast of the configs[4] step raced; now bitwise the RNE rounding of the f32 fold,
    in plain and accumulate mode."""
    K, P = 9, 4 * 4099
    x = torch.empty(K, P, dtype=torch.float32, device=cuda)
    kernels.fill_synth(x, seed=77)
    xh = coracle.synth_f32(K, P, seed=77)
    w = np.float32(ref.fedavg_weights(K, seed=78))
    want = coracle.wsum_f32(xh, w, scale=np.float32(0.25))
    u = want.view(np.uint32).astype(np.uint64)
    want16 = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    y = kernels.weighted_sum_dense(x, torch.from_numpy(w).to(cuda), scale=0.25, out_dtype=torch.bfloat16,
                                   variant=variant)
    assert np.array_equal(host(y.view(torch.int16)).view(np.uint16), want16)
    init16 = (np.arange(P) % 7).astype(np.float32)
    o = torch.from_numpy(init16).to(cuda).to(torch.bfloat16)
    kernels.weighted_sum_dense(x, torch.from_numpy(w).to(cuda), out=o, accumulate=True, variant=variant)
    want_acc = coracle.wsum_f32(xh, w, init=init16)
    ua = want_acc.view(np.uint32).astype(np.uint64)
    assert np.array_equal(host(o.view(torch.int16)).view(np.uint16),
                          ((ua + 0x7FFF + ((ua >> 16) & 1)) >> 16).astype(np.uint16))


def test_dense_accumulate_and_strided_rows(cuda, coracle):
    K, P, ld = 17, 3001, 3072
    base = torch.empty(K, ld, dtype=torch.float32, device=cuda)
    kernels.fill_synth(base, seed=1)
    x = base[:, :P]
    xh = coracle.synth_f32(K, ld, seed=1)[:, :P]
    w = np.float32(ref.fedavg_weights(K, seed=2))
    init = coracle.synth_f32(1, P, seed=3)[0]
    out = torch.from_numpy(init.copy()).to(cuda)
    kernels.weighted_sum_dense(x, torch.from_numpy(w).to(cuda), out=out, accumulate=True)
    want = coracle.wsum_f32(xh, w, init=init)
    assert np.array_equal(bits(host(out)), bits(want))


def test_dense_unaligned_views_take_scalar_path(cuda, coracle):
    K, P = 5, 1001
    base = torch.empty(K, P + 1, dtype=torch.float32, device=cuda)
    kernels.fill_synth(base, seed=4)
    x = base[:, 1:]  # 4-byte offset: not 16-byte aligned
    xh = coracle.synth_f32(K, P + 1, seed=4)[:, 1:]
    w = np.float32([1, 2, 3, 4, 5])
    y = kernels.weighted_sum_dense(x, torch.from_numpy(w).to(cuda), scale=0.25)
    assert np.array_equal(bits(host(y)), bits(coracle.wsum_f32(xh, w, scale=np.float32(0.25))))


def test_int_fold_wraps_like_xla(cuda):
    x = torch.tensor([[2 ** 30, -(2 ** 30), 7, 1], [2 ** 30, -(2 ** 30), 9, 1]], dtype=torch.int32, device=cuda)
    w = torch.tensor([3, 2], dtype=torch.int32, device=cuda)
    y = kernels.weighted_sum_dense(x, w)
    assert y.dtype == torch.int32
    npt.assert_array_equal(host(y), np.array([2 ** 30, -(2 ** 30), 39, 5], np.int32))


def _bound(coracle, xh, w, r, want, G=1):
    K = xh.shape[0]
    return coracle.bound_f32(xh, w, r, want) * (K + G + 2) / (K + 2)


@pytest.mark.parametrize("K,P", [(1024, 16384), (512, 1000), (64, 4097)])
def test_split_mode_within_bound(K, P, cuda, coracle):
    x = torch.empty(K, P, dtype=torch.float32, device=cuda)
    kernels.fill_synth(x, seed=5)
    xh = coracle.synth_f32(K, P, seed=5)
    wi = [int(v) for v in ref.fedavg_weights(K)]
    r = ref.mean_scale(wi)
    w = np.float32(wi)
    want = coracle.wsum_f32(xh, w, scale=r)
    y = host(kernels.weighted_sum_dense(x, torch.from_numpy(w).to(cuda), scale=float(r), mode="split"))
    # at most 64 client ranges are combined (kSplitMax in fjagg.hip)
    assert np.all(np.abs(y.astype(np.float64) - want) <= _bound(coracle, xh, w, r, want, G=64))


def test_bf16_dense_vs_f64_oracle(cuda, coracle):
    K, P = 64, 20000
    x = torch.empty(K, P, dtype=torch.bfloat16, device=cuda)
    kernels.fill_synth(x, seed=6)
    xb = coracle.synth_bf16(K, P, seed=6)
    assert np.array_equal(host(x), xb)
    wi = ref.fedavg_weights(K)
    r = 1.0 / wi.sum()
    y64 = coracle.wsum_bf16_f64(xb, np.float64(wi), r)
    w = torch.tensor(np.float32(wi), device=cuda)
    yb = bf16_to_f32(host(kernels.weighted_sum_dense(x, w, scale=float(np.float32(r)))))
    yf = host(kernels.weighted_sum_dense(x, w, scale=float(np.float32(r)), out_dtype=torch.float32))
    tsum = np.abs(bf16_to_f32(xb).astype(np.float64) * np.float32(wi)[:, None]).sum(0)
    fbound = (K + 3) * U * r * tsum + U * np.abs(y64)
    assert np.all(np.abs(yf - y64) <= fbound)
    assert np.all(np.abs(yb - y64) <= 2.0 ** -8 * np.abs(y64) + fbound)


# ------------------------------------------------------------------- pytree kernel
def test_pytree_unaligned_and_mixed_leaves(cuda, coracle):
    K = 6
    P = 4 * 1000 + 11
    base = torch.empty(K, P, dtype=torch.float32, device=cuda)
    kernels.fill_synth(base, seed=8)
    xh = coracle.synth_f32(K, P, seed=8)
    cuts = [0, 1, 33, 1000, 3003, P]  # odd offsets: unaligned leaf views
    trees = [{f"l{i}": base[k, cuts[i]:cuts[i + 1]] for i in range(len(cuts) - 1)} for k in range(K)]
    wi = [3, 1, 4, 1, 5, 9]
    m = tu.tree_mean(zip(trees, wi))
    got = np.concatenate([host(m[f"l{i}"]) for i in range(len(cuts) - 1)])
    want = coracle.wsum_f32(xh, np.float32(wi), scale=ref.mean_scale(wi))
    assert np.array_equal(bits(got), bits(want))


EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_pytree_mixed_alignment_per_leaf_units(cuda, coracle, dtype):
    """Client pytrees that are views into one slab at EMNIST-CNN leaf offsets: linear_1/w
    sits 8 bytes off a 16-byte boundary (f32), so that leaf walks element units while
    the others keep 16-byte units (fjagg_ptrs_plan_leaves). Bitwise equal to the oracle
    and to the same leaves cloned into aligned allocations; with l2 norms and with the
    fused server step too."""
    template = pytree_map(lambda s: np.zeros(s, np.float32), EMNIST)
    K = 12
    slab = fedjax_amd.ClientDeltaSlab(template, K, dtype=dtype, device=cuda).fill_synthetic(seed=21)
    views = [slab.client(k) for k in range(K)]
    ptrs = [x.data_ptr() % 16 for x in fedjax_amd.pytree.leaves_of(views[1])]
    assert any(ptrs) and not all(ptrs)  # mixed alignment
    clones = [pytree_map(lambda v: v.clone(), t) for t in views]
    wi = [int(v) for v in ref.fedavg_weights(K, seed=22)]
    m_v, m_c = tu.tree_mean(zip(views, wi)), tu.tree_mean(zip(clones, wi))
    flat_v = torch.cat([v.reshape(-1) for v in fedjax_amd.pytree.leaves_of(m_v)])
    flat_c = torch.cat([v.reshape(-1) for v in fedjax_amd.pytree.leaves_of(m_c)])
    assert torch.equal(flat_v, flat_c)
    if dtype == torch.float32:
        xh = coracle.synth_f32(K, slab.num_params, seed=21)
        want = coracle.wsum_f32(xh, np.float32(wi), scale=ref.mean_scale(wi))
        assert np.array_equal(bits(host(flat_v)), bits(want))
        mv, nv = tu.tree_mean_with_l2_norms(zip(views, wi))
        mc, nc = tu.tree_mean_with_l2_norms(zip(clones, wi))
        assert torch.equal(torch.cat([v.reshape(-1) for v in fedjax_amd.pytree.leaves_of(mv)]), flat_c)
        npt.assert_allclose(host(nv), host(nc), rtol=2e-6)
        from fedjax_amd import server
        opt = server.adam(10 ** -2.5, b1=0.9, b2=0.999, eps=1e-4)
        outs = []
        for clients in (views, clones):
            params = pytree_map(lambda v: torch.zeros(v.shape, device=cuda), clients[0])
            st = server.fused_tree_mean_update(zip(clients, wi), opt, params, opt.init(params))
            outs.append(torch.cat([v.reshape(-1) for v in fedjax_amd.pytree.leaves_of(params)]))
        assert torch.equal(outs[0], outs[1])


def test_slab_mean_equals_tree_mean_equals_oracle(cuda, coracle):
    shapes = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "linear": {"b": (128,), "w": (100, 128)}}
    template = pytree_map(lambda s: np.zeros(s, np.float32), shapes)
    K = 20
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=cuda).fill_synthetic(seed=10)
    P = slab.num_params
    xh = coracle.synth_f32(K, P, seed=10)
    wi = [int(v) for v in ref.fedavg_weights(K, seed=11)]
    want = coracle.wsum_f32(xh, np.float32(wi), scale=ref.mean_scale(wi))
    m1 = slab.mean(wi)
    m2 = tu.tree_mean((slab.client(k), wi[k]) for k in range(K))
    for m in (m1, m2):
        flat = np.concatenate([host(v).ravel() for v in fedjax_amd.pytree.leaves_of(m)])
        assert np.array_equal(bits(flat), bits(want))
    norms = host(slab.l2_norms())
    npt.assert_allclose(norms, np.sqrt((xh.astype(np.float64) ** 2).sum(1)), rtol=2e-6)
    norms2 = host(tu.tree_l2_norms([slab.client(k) for k in range(K)]))
    npt.assert_allclose(norms2, norms, rtol=2e-6)


def pytree_map(fn, shapes):
    if isinstance(shapes, dict):
        return {k: pytree_map(fn, v) for k, v in shapes.items()}
    return fn(shapes)


# -------------------------------------------------------------- full-size properties
def synth_cols(K, cols, seed, amp=0.01):
    """oracle synth restricted to some columns (same hash)."""
    k = (np.arange(K, dtype=np.uint64) << np.uint64(32))[:, None]
    p = np.asarray(cols, np.uint64)[None, :]
    h = ref._mix64(np.uint64(seed) ^ ref._mix64(k | p))
    u = (h >> np.uint64(40)).astype(np.uint32).astype(np.float32) * np.float32(1 / 8388608) - np.float32(1)
    return np.float32(amp) * u


@pytest.mark.parametrize("weights", ["device", "kernel_args"])
@pytest.mark.parametrize("K,P", [(128, 1206590), (1024, 4 * 1024 * 1024), (40, 700001), (128, 524288)])
def test_full_size_configs(K, P, weights, cuda):
    """BASELINE configs 2 and 3 at full size: sampled columns bitwise vs the oracle,
    weight-scaling invariance (2w gives the identical bits) over every element.

    ``kernel_args``: host weights, which travel in the launch's kernel arguments
    (FJAGG_HOST_TABLES, the k_dense<..., WK=1024> instance bench.py times at configs[2]);
    the test asserts that the launch took that route rather than an upload."""
    x = torch.empty(K, P, dtype=torch.float32, device=cuda)
    kernels.fill_synth(x, seed=0)
    wi = [int(v) for v in ref.fedavg_weights(K)]
    r = ref.mean_scale(wi)
    if weights == "device":
        w = torch.tensor(np.float32(wi), device=cuda)
        y = kernels.weighted_sum_dense(x, w, scale=float(r), nontemporal=True)
    else:
        before = dict(kernels.HOST_WEIGHT_PATHS)
        y = kernels.weighted_sum_dense(x, np.float32(wi), scale=float(r), nontemporal=True)
        assert kernels.HOST_WEIGHT_PATHS["kernel_args"] == before["kernel_args"] + 1
        assert kernels.HOST_WEIGHT_PATHS["uploaded"] == before["uploaded"]
    rs = np.random.RandomState(0)
    cols = np.unique(np.concatenate([rs.randint(0, P, 2000), [0, 1, 2, 3, P - 4, P - 3, P - 2, P - 1]]))
    xs = synth_cols(K, cols, 0)
    want = ref.wsum_dense(xs, np.float32(wi), scale=r)
    assert np.array_equal(bits(host(y)[cols]), bits(want))
    wi2 = [2 * v for v in wi]
    y2 = kernels.weighted_sum_dense(x, torch.tensor(np.float32(wi2), device=cuda), scale=float(ref.mean_scale(wi2)))
    assert torch.equal(y.view(torch.int32), y2.view(torch.int32))
    del x
    torch.cuda.empty_cache()


# ------------------------------------------------------------ streaming running sum
@pytest.mark.parametrize("buffer_clients", [1, 5, 8, None])
def test_running_mean_equals_library_fedavg_loop(buffer_clients, cuda, coracle):
    """fedjax/algorithms/fed_avg.py:132-146 restated: s = 0; s = s + x_k*n_k; s * f32(1/W)."""
    K, P = 37, 3001
    xh = coracle.synth_f32(K, P, seed=21)
    wi = [int(v) for v in ref.fedavg_weights(K, seed=22)]
    cut = 1000
    template = {"a": np.zeros(cut, np.float32), "b": np.zeros(P - cut, np.float32)}
    rm = fedjax_amd.aggregators.RunningMean(template, buffer_clients=buffer_clients, device=cuda)
    for k in range(K):
        xk = torch.from_numpy(xh[k]).to(cuda)
        rm.add({"a": xk[:cut], "b": xk[cut:]}, wi[k])
    m = rm.result()
    got = np.concatenate([host(m["a"]), host(m["b"])])
    s = np.zeros(P, np.float32)
    for k in range(K):
        s = s + xh[k] * np.float32(wi[k])
    W = 0.0
    for w in wi:
        W += w
    want = s * np.float32(1.0 / W)
    assert np.array_equal(bits(got), bits(want))
    assert rm.num_clients == K and rm.total_weight == W


def test_running_mean_native_flush_host_deltas_and_errors(cuda):
    """RunningMean folds a buffer through the native table (fjhost.fold_table into the
    running sum, accumulate mode): bitwise equal to the Python fold; host (numpy)
    deltas take the flatten-and-copy path with the same bits; a delta whose structure
    differs from the template raises when the buffer is folded."""
    g = torch.Generator(device="cpu").manual_seed(5)
    K = 11
    trees = [{"a": torch.randn(1003, generator=g), "b": torch.randn(4, 6, generator=g)} for _ in range(K)]
    w = [int(v) for v in torch.randint(1, 500, (K,), generator=g)]
    dev_trees = [{k: v.to(cuda) for k, v in t.items()} for t in trees]
    host_trees = [{k: v.numpy() for k, v in t.items()} for t in trees]
    results = []
    for clients in (dev_trees, host_trees):
        rm = fedjax_amd.aggregators.RunningMean(dev_trees[0], buffer_clients=4, device=cuda)
        for c, wk in zip(clients, w):
            rm.add(c, wk)
        results.append(rm.result())
    s = [torch.zeros(1003, device=cuda), torch.zeros(4, 6, device=cuda)]
    for k0 in range(0, K, 4):  # the Python fold of the same buffers
        rows = [[t["a"], t["b"]] for t in dev_trees[k0:k0 + 4]]
        tu._fold(rows, w[k0:k0 + 4], out=s, accumulate=True)
    W = float(sum(w))
    want = tu.tree_inverse_weight({"a": s[0], "b": s[1]}, W)
    for r in results:
        for key in ("a", "b"):
            assert torch.equal(r[key].view(torch.int32), want[key].view(torch.int32))
    # the native table path is the one taken for device deltas
    _, rows = tu._client_table(dev_trees[:4])
    out = [torch.zeros(1003, device=cuda), torch.zeros(4, 6, device=cuda)]
    got = tu._native_fold(rows, tu._pack_weights(w[:4]), None, out, True)
    assert got is not None and got[0] is out[0] and got[1] is out[1]
    rm = fedjax_amd.aggregators.RunningMean(dev_trees[0], buffer_clients=2, device=cuda)
    rm.add(dev_trees[0], 1)
    with pytest.raises(ValueError):
        rm.add({"a": dev_trees[1]["a"]}, 1)


def test_running_mean_detects_in_place_reuse(cuda):
    """a torch loop that reuses one delta buffer for every client.
    The reference sums each delta at its tree_add; a buffered reference would sum the
    last value K times. RunningMean raises instead; copy_on_add gives the reference's
    sum (bitwise the eager loop)."""
    K = 5
    g = torch.Generator(device="cpu").manual_seed(9)
    vals = [torch.randn(2000, generator=g).to(cuda) for _ in range(K)]
    tmpl = {"d": torch.zeros(2000, device=cuda)}
    buf = torch.empty(2000, device=cuda)
    rm = fedjax_amd.aggregators.RunningMean(tmpl, buffer_clients=8, device=cuda)
    for k in range(K):
        buf.copy_(vals[k])  # in place: bumps the version counter
        rm.add({"d": buf}, k + 1)
    with pytest.raises(RuntimeError, match="modified in place"):
        rm.result()
    rc = fedjax_amd.aggregators.RunningMean(tmpl, buffer_clients=8, device=cuda, copy_on_add=True)
    for k in range(K):
        buf.copy_(vals[k])
        rc.add({"d": buf}, k + 1)
    s = torch.zeros(2000, device=cuda)
    for k in range(K):
        s = s + vals[k] * float(np.float32(k + 1))
    want = s * float(np.float32(1.0 / 15.0))
    assert torch.equal(rc.result()["d"].view(torch.int32), want.view(torch.int32))
    # untouched deltas (the common case) fold without a copy
    ru = fedjax_amd.aggregators.RunningMean(tmpl, buffer_clients=2, device=cuda)
    for k in range(K):
        ru.add({"d": vals[k]}, k + 1)
    assert torch.equal(ru.result()["d"].view(torch.int32), want.view(torch.int32))


def test_running_mean_carved_sum_and_version_growth(cuda):
    """The zero sum of an all-float32 template is one allocation carved into leaf views
    (0-d, odd and 64-multiple sizes here); the add()-time version rows grow past their
    first 64 (150 buffered clients). Bitwise the eager loop, sum() mid-stream included."""
    K = 150
    shapes = {"s": (), "a": (3,), "b": (5, 7), "c": (64,), "d": (129,)}
    g = torch.Generator(device="cpu").manual_seed(13)
    trees = [{k: torch.randn(s, generator=g).to(cuda) for k, s in shapes.items()} for _ in range(K)]
    w = [int(v) for v in torch.randint(1, 500, (K,), generator=g)]
    rm = fedjax_amd.aggregators.RunningMean(trees[0], buffer_clients=200, device=cuda)
    s = {k: torch.zeros(sh, device=cuda) for k, sh in shapes.items()}
    for k in range(K):
        rm.add(trees[k], w[k])
        s = {n: s[n] + trees[k][n] * float(np.float32(w[k])) for n in shapes}
        if k == 99:
            mid = rm.sum()
            for n in shapes:
                assert mid[n].shape == shapes[n] and mid[n].is_contiguous()
                assert mid[n].data_ptr() % 256 == 0
                assert torch.equal(mid[n].view(torch.int32), s[n].view(torch.int32))
    W = float(sum(w))
    got = rm.result()
    for n in shapes:
        want = s[n] * float(np.float32(1.0 / W))
        assert torch.equal(got[n].view(torch.int32), want.view(torch.int32))


# ------------------------------------------------------------ fused fold + l2 norms
@pytest.mark.parametrize("K,P,dt", [(1, 7, "f32"), (37, 10007, "f32"), (128, 1206590, "f32"),
                                    (300, 65536 + 5, "f32"), (64, 20000, "bf16"), (5, 3, "f32")])
def test_fused_l2_matches_fold_and_norms(K, P, dt, cuda, coracle):
    tdt = torch.float32 if dt == "f32" else torch.bfloat16
    vw = 4 if dt == "f32" else 8
    x = torch.empty(K, (P + vw - 1) // vw * vw, dtype=tdt, device=cuda)[:, :P]
    kernels.fill_synth(x, seed=31)
    wi = [int(v) for v in ref.fedavg_weights(K, seed=32)]
    r = float(ref.mean_scale(wi))
    w = torch.tensor(np.float32(wi), device=cuda)
    y0 = kernels.weighted_sum_dense(x, w, scale=r)
    for nt in (False, True):
        y1, l2 = kernels.weighted_sum_l2_dense(x, w, scale=r, nontemporal=nt)
        assert np.array_equal(bits(host(y1)), bits(host(y0)))
        xf = x.float().cpu().numpy().astype(np.float64)
        want = (xf ** 2).sum(1)
        npt.assert_allclose(host(l2), want, rtol=2e-6)
    y2, l2b = kernels.weighted_sum_l2_dense(x, w, scale=r)
    assert torch.equal(l2, l2b)  # deterministic


def test_fused_l2_unaligned_and_slab(cuda, coracle):
    K, P = 9, 1001
    base = torch.empty(K, P + 1, dtype=torch.float32, device=cuda)
    kernels.fill_synth(base, seed=33)
    x = base[:, 1:]
    w = torch.arange(1, K + 1, dtype=torch.float32, device=cuda)
    y, l2 = kernels.weighted_sum_l2_dense(x, w)
    xh = coracle.synth_f32(K, P + 1, seed=33)[:, 1:]
    assert np.array_equal(bits(host(y)), bits(coracle.wsum_f32(xh, np.arange(1, K + 1, dtype=np.float32))))
    npt.assert_allclose(host(l2), (xh.astype(np.float64) ** 2).sum(1), rtol=2e-6)
    template = {"a": np.zeros(100, np.float32), "b": np.zeros((7, 11), np.float32)}
    slab = fedjax_amd.ClientDeltaSlab(template, 12, device=cuda).fill_synthetic(seed=34)
    wi = list(range(1, 13))
    m0 = slab.mean(wi)
    m1, norms = slab.mean(wi, with_norms=True)
    for a, b in zip(fedjax_amd.pytree.leaves_of(m0), fedjax_amd.pytree.leaves_of(m1)):
        assert torch.equal(a, b)
    npt.assert_allclose(host(norms), host(slab.l2_norms()), rtol=2e-6)


# ----------------------------------------------------------------- more edge cases
def test_bf16_pytree_tree_mean_vs_f64(cuda, coracle):
    K, P = 12, 5003
    xb = coracle.synth_bf16(K, P, seed=51)
    xt = torch.from_numpy(xb.view(np.int16)).view(torch.bfloat16).to(cuda)
    cut = 2001
    trees = [{"a": xt[k, :cut], "b": xt[k, cut:].reshape(-1)} for k in range(K)]
    wi = [int(v) for v in ref.fedavg_weights(K, seed=52)]
    m = tu.tree_mean(zip(trees, wi))
    assert m["a"].dtype == torch.bfloat16
    got = bf16_to_f32(np.concatenate([host(m["a"]), host(m["b"])])).astype(np.float64)
    r = 1.0 / sum(wi)
    y64 = coracle.wsum_bf16_f64(xb, np.float64(wi), r)
    tsum = np.abs(bf16_to_f32(xb).astype(np.float64) * np.float32(wi)[:, None]).sum(0)
    assert np.all(np.abs(got - y64) <= 2.0 ** -8 * np.abs(y64) + (K + 3) * U * r * tsum)


def test_split_mode_bf16_and_accumulate(cuda, coracle):
    K, P = 640, 3000
    x = torch.empty(K, P + 8 - P % 8, dtype=torch.bfloat16, device=cuda)[:, :P]
    kernels.fill_synth(x, seed=53)
    xb = coracle.synth_bf16(K, P, seed=53)
    w = np.float32(ref.fedavg_weights(K, seed=54))
    wd = torch.from_numpy(w).to(cuda)
    y = host(kernels.weighted_sum_dense(x, wd, out_dtype=torch.float32, mode="split"))
    y64 = coracle.wsum_bf16_f64(xb, np.float64(w), 1.0)
    tsum = np.abs(bf16_to_f32(xb).astype(np.float64) * w[:, None]).sum(0)
    assert np.all(np.abs(y - y64) <= (K + 66) * U * tsum + U * np.abs(y64))
    init = np.linspace(-1, 1, P).astype(np.float32)
    out = torch.from_numpy(init.copy()).to(cuda)
    kernels.weighted_sum_dense(x, wd, out=out, accumulate=True, mode="split")
    y2 = host(out).astype(np.float64)
    assert np.all(np.abs(y2 - (y64 + init)) <= (K + 67) * U * (tsum + np.abs(init)) + U * np.abs(y64 + init))


def test_rows_over_one_gib_are_chunked(cuda):
    K, P = 2, 300_000_000  # 1.2 GB rows: two column launches of <= 1 GiB each
    x = torch.empty(K, P, dtype=torch.float32, device=cuda)
    kernels.fill_synth(x, seed=55)
    wi = [3, 5]
    y = kernels.weighted_sum_dense(x, torch.tensor(np.float32(wi), device=cuda), scale=float(ref.mean_scale(wi)))
    cols = np.array([0, 1, 268435455, 268435456, 268435457, P - 1])
    xs = synth_cols(K, cols, 55)
    want = ref.wsum_dense(xs, np.float32(wi), scale=ref.mean_scale(wi))
    assert np.array_equal(bits(host(y)[cols]), bits(want))
    del x, y
    torch.cuda.empty_cache()


def test_int_dense_fold_with_scale_and_float_weights(cuda):
    xi = (np.arange(40, dtype=np.int32).reshape(4, 10) - 20) * 1000
    x = torch.from_numpy(xi).to(cuda)
    wi = np.array([3, 1, 4, 1], np.int32)
    y = kernels.weighted_sum_dense(x, torch.from_numpy(wi).to(cuda), scale=0.125)
    s = (xi * wi[:, None]).sum(0).astype(np.int32)
    assert y.dtype == torch.float32 and np.array_equal(host(y), s.astype(np.float32) * np.float32(0.125))
    wf = np.float32([0.5, 1.5, 2.0, 0.25])
    yf = kernels.weighted_sum_dense(x, torch.from_numpy(wf).to(cuda))
    want = ref.wsum_dense(xi.astype(np.float32), wf)
    assert np.array_equal(bits(host(yf)), bits(want))


def test_empty_and_scalar_leaves(cuda):
    trees = [({"e": torch.zeros(0, device=cuda), "s": torch.tensor(float(k), device=cuda),
               "v": torch.full((3,), float(k), device=cuda)}, k + 1) for k in range(3)]
    m = tu.tree_mean(trees)
    assert m["e"].shape == (0,) and m["s"].shape == ()
    want = (0 * 1 + 1 * 2 + 2 * 3) / 6
    npt.assert_allclose(host(m["s"]), want, rtol=1e-7)
    npt.assert_allclose(host(m["v"]), [want] * 3, rtol=1e-7)


def test_leaf_over_one_gib_through_the_pytree_kernel(cuda):
    """a leaf of 300 M float32 (1.2 GB) per client folds through tree_mean (the
    pytree kernel rebases every row at its workgroup's first element, so lane offsets stay
    32-bit), bitwise vs the oracle at columns on both sides of the 1 GiB and 2 GiB marks;
    with fused l2 norms too. A plan beyond 40-bit unit offsets is refused."""
    K, P = 2, 300_000_000
    x = torch.empty(K, P + 5, dtype=torch.float32, device=cuda)
    kernels.fill_synth(x[:, :P], seed=57)
    trees = [{"big": x[k, :P].clone(), "small": x[k, P:P + 5].clone()} for k in range(K)]
    del x
    wi = [3, 5]
    m = tu.tree_mean(zip(trees, wi))
    cols = np.array([0, 1, 2, 3, 268435455, 268435456, 268435457, 536870911 // 2, P - 2, P - 1])
    want = ref.wsum_dense(synth_cols(K, cols, 57), np.float32(wi), scale=ref.mean_scale(wi))
    assert np.array_equal(bits(host(m["big"])[cols]), bits(want))
    m2, norms = tu.tree_mean_with_l2_norms(zip(trees, wi))
    assert torch.equal(m2["big"].view(torch.int32), m["big"].view(torch.int32))
    for k in range(K):
        npt.assert_allclose(float(norms[k]), float(torch.linalg.vector_norm(
            torch.cat([trees[k]["big"], trees[k]["small"]]).double())), rtol=2e-6)
    del trees, m, m2
    torch.cuda.empty_cache()
    with pytest.raises(_lib.FjaggError):
        kernels.ptrs_plan(_lib.F32, [1 << 41], False)


# ------------------------------------------------------- fused server optimizer step
def _np_server_step(opt, d, g, p, m, v):
    """numpy restatement of optax's op order (sgd / trace / scale_by_adam, then
    scale_by_learning_rate and apply_updates) with the descriptor's f32 constants."""
    f = np.float32

    def rsqrt(x):  # jax.lax.rsqrt restated: 1 / sqrt in f64, rounded once
        with np.errstate(divide="ignore", invalid="ignore"):
            return (1.0 / np.sqrt(x.astype(np.float64))).astype(f)

    if opt.kind == 1:
        u = g
    elif opt.kind == 2:
        m = g + f(d.decay) * m
        u = g + f(d.decay) * m if opt.nesterov else m
    elif opt.kind == 3:
        m = f(d.one_minus_b1) * g + f(d.b1) * m
        v = f(d.one_minus_b2) * (g * g) + f(d.b2) * v
        u = (m / f(d.bc1)) / (np.sqrt(v / f(d.bc2) + f(d.eps_root)) + f(d.eps))
    elif opt.kind == 4:  # optax.scale_by_rss
        v = g * g + v
        u = np.where(v > 0, rsqrt(v + f(d.eps)), f(0)) * g
    elif opt.kind == 5:  # optax.rmsprop: scale_by_rms | scale_by_stddev, scale_by_learning_rate, [trace]
        v = f(d.one_minus_b2) * (g * g) + f(d.b2) * v
        den = v
        if opt.centered:  # scale_by_stddev: mu = (1 - decay) g + decay mu; rsqrt(nu - mu^2 + eps)
            m = f(d.one_minus_b2) * g + f(d.b2) * m
            den = v - m * m
        u = g * rsqrt(den + f(d.eps))
        if opt.momentum is not None:  # the trace of the lr-scaled update
            s_ = f(d.neg_lr) * u
            m = s_ + f(d.decay) * m
            return p + (s_ + f(d.decay) * m if opt.nesterov else m), m, v
    else:  # optax.scale_by_yogi
        m = f(d.one_minus_b1) * g + f(d.b1) * m
        v = v - (f(d.one_minus_b2) * np.sign(v - g * g)).astype(f) * (g * g)
        u = m / (np.sqrt(v + f(d.eps_root)) + f(d.eps))
    return p + f(d.neg_lr) * u, m, v


OPTIMIZERS = [lambda s: s.sgd(0.5), lambda s: s.sgd(0.1, momentum=0.9),
              lambda s: s.sgd(0.1, momentum=0.9, nesterov=True),
              lambda s: s.adam(10 ** -2.5, b1=0.9, b2=0.999, eps=1e-4),
              lambda s: s.adagrad(0.1), lambda s: s.adagrad(0.3, initial_accumulator_value=0.0, eps=1e-7),
              lambda s: s.rmsprop(0.01), lambda s: s.rmsprop(0.01, decay=0.8, initial_scale=1.0, momentum=0.5),
              lambda s: s.rmsprop(0.01, momentum=0.9, nesterov=True),
              lambda s: s.rmsprop(0.01, centered=True), lambda s: s.rmsprop(0.02, decay=0.7, centered=True, initial_scale=1.0),
              lambda s: s.yogi(0.01), lambda s: s.yogi(0.05, b1=0.5, b2=0.99, eps=1e-4)]


@pytest.mark.parametrize("make", OPTIMIZERS)
def test_fused_server_update_matches_restated_optax(make, cuda, coracle):
    from fedjax_amd import server
    opt = make(server)
    K, P = 33, 10007
    template = {"a": np.zeros(7, np.float32), "b": np.zeros(P - 7, np.float32)}
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=cuda)
    params = torch.from_numpy(coracle.synth_f32(1, P, seed=61)[0].copy()).to(cuda)
    state = opt.init(params)
    p_np = host(params).copy()
    m_np = np.full(P, opt.init_m, np.float32)
    v_np = np.full(P, opt.init_v, np.float32)
    for rnd in range(3):
        slab.fill_synthetic(seed=62 + rnd)
        xh = coracle.synth_f32(K, P, seed=62 + rnd)
        wi = [int(x) for x in ref.fedavg_weights(K, seed=70 + rnd)]
        mean_out = torch.empty(P, device=cuda)
        state = server.fused_mean_update(slab, wi, opt, params, state, mean_out=mean_out)
        g = coracle.wsum_f32(xh, np.float32(wi), scale=ref.mean_scale(wi))
        assert np.array_equal(bits(host(mean_out)), bits(g))
        d = opt.descriptor(state["count"])
        p_np, m_np, v_np = _np_server_step(opt, d, g, p_np, m_np, v_np)
        assert np.array_equal(bits(host(params)), bits(p_np)), rnd
        if "m" in state:
            assert np.array_equal(bits(host(state["m"])), bits(m_np))
        if "v" in state:
            assert np.array_equal(bits(host(state["v"])), bits(v_np))
    assert state["count"] == 3


def test_fused_server_update_reproduces_fedavg_example_kat(cuda):
    # examples/fed_avg_test.py:52-56: server sgd(lr=1.0) after tree_mean of two clients
    from fedjax_amd import server
    deltas = [fr.client_update(fr.SERVER_PARAMS, x, 2, 2, 0)["w"] for _, x in fr.CLIENTS]
    slab = fedjax_amd.ClientDeltaSlab({"w": np.zeros(3, np.float32)}, 2, device=cuda)
    for k, d in enumerate(deltas):
        slab.set_client(k, {"w": torch.from_numpy(d)})
    params = torch.from_numpy(fr.SERVER_PARAMS["w"].copy()).to(cuda)
    opt = server.sgd(1.0)
    server.fused_mean_update(slab, [len(x) for _, x in fr.CLIENTS], opt, params, opt.init(params))
    npt.assert_allclose(host(params), [0., 1.4425802, 2.8851604])


def test_emnist_fed_avg_rounds_example(cuda):
    import importlib.util, os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples",
                        "emnist_fed_avg_rounds.py")
    spec = importlib.util.spec_from_file_location("emnist_rounds", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    hist = mod.run(rounds=3, verbose=False)
    assert all(h["same_mean"] and h["same_params"] and h["norm_rel_diff"] < 2e-6 for h in hist), hist
    assert all(h["same_mean_library_loop"] and h["norm_rel_diff_library_loop"] < 2e-6 for h in hist), hist


# ------------------------------------------------- fused l2 norms on the pytree path
EMNIST_SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
                 "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def _separate_clients(K, shapes, seed, dtype, device, offset=0):
    """K pytrees of separately allocated leaves (offset > 0: leaves start off 16-byte alignment)."""
    flat_shapes = [s for _, d in sorted(shapes.items()) for _, s in sorted(d.items())]
    P = sum(int(np.prod(s)) for s in flat_shapes)
    base = torch.empty(K, P + offset, dtype=dtype, device=device)
    kernels.fill_synth(base, seed=seed)
    clients = []
    for k in range(K):
        o, leaves = offset, []
        for s in flat_shapes:
            n = int(np.prod(s))
            leaves.append(base[k, o:o + n].clone().view(s) if offset == 0 else base[k, o:o + n].view(s))
            o += n
        it = iter(leaves)
        clients.append({m: {n: next(it) for n in sorted(d)} for m, d in sorted(shapes.items())})
    return clients


@pytest.mark.parametrize("K,dt,offset", [(10, torch.float32, 0), (128, torch.float32, 0), (33, torch.float32, 1),
                                         (16, torch.bfloat16, 0), (1, torch.float32, 0)])
def test_tree_mean_with_l2_norms(K, dt, offset, cuda):
    clients = _separate_clients(K, EMNIST_SHAPES, 71, dt, cuda, offset)
    wi = [int(v) for v in ref.fedavg_weights(K, seed=72)]
    pairs = list(zip(clients, wi))
    m0 = tu.tree_mean(pairs)
    m1, norms = tu.tree_mean_with_l2_norms(iter(pairs))  # generators are consumed once
    for a, b in zip(fedjax_amd.pytree.leaves_of(m0), fedjax_amd.pytree.leaves_of(m1)):
        assert torch.equal(a, b)  # the fold is bitwise tree_mean's
    want = np.array([sum(float((x.double() ** 2).sum()) for x in fedjax_amd.pytree.leaves_of(c)) for c in clients])
    npt.assert_allclose(host(norms), np.sqrt(want), rtol=2e-6)
    _, norms2 = tu.tree_mean_with_l2_norms(pairs)
    assert torch.equal(norms, norms2)  # deterministic
    npt.assert_allclose(host(norms), host(tu.tree_l2_norms(clients)), rtol=2e-6)


def test_tree_mean_with_l2_norms_edges(cuda):
    assert tu.tree_mean_with_l2_norms([]) == (None, None)
    a = torch.arange(5, dtype=torch.float32, device=cuda)
    m, n = tu.tree_mean_with_l2_norms([({"x": a}, 1), ({"x": 2 * a}, 3)])
    npt.assert_allclose(host(n), [np.sqrt(30.0), np.sqrt(120.0)], rtol=1e-6)
    npt.assert_array_equal(host(m["x"]), host(tu.tree_mean([({"x": a}, 1), ({"x": 2 * a}, 3)])["x"]))
    # int and mixed-dtype leaves: the mean and the norms in two passes
    mi, ni = tu.tree_mean_with_l2_norms([({"x": torch.full((3,), 2, dtype=torch.int32, device=cuda)}, 1)])
    assert mi["x"].dtype == torch.float32 and host(ni).tolist() == [np.float32(np.sqrt(12.0))]
    mm, nm = tu.tree_mean_with_l2_norms([({"x": a, "y": a.bfloat16()}, 1)])
    npt.assert_allclose(host(nm), [np.sqrt(60.0)], rtol=1e-6)


@pytest.mark.parametrize("make", OPTIMIZERS)
@pytest.mark.parametrize("offset", [0, 1])
def test_fused_tree_server_update_matches_restated_optax(make, offset, cuda, coracle):
    """Pytree path (fjagg_server_update_ptrs): tree_mean of separate client pytrees + the
    server step, bitwise against tree_mean followed by the numpy optax restatement."""
    from fedjax_amd import server
    opt = make(server)
    K, sizes = 33, {"a": 8, "b": 10000, "c": (3, 5)}  # offset 0: every leaf 16-byte aligned, c has a tail
    n = {k: int(np.prod(v)) for k, v in sizes.items()}
    P = sum(n.values())

    def tree_of(vec):
        out, o = {}, 0
        for k in sorted(sizes):
            out[k] = vec[o:o + n[k]].reshape(sizes[k] if isinstance(sizes[k], tuple) else (n[k],))
            o += n[k]
        return out

    base = torch.from_numpy(coracle.synth_f32(1, P + offset, seed=61)[0].copy()).to(cuda)
    params = tree_of(base[offset:].clone())
    state = opt.init(params)
    p_np = {k: host(v).copy() for k, v in params.items()}
    m_np = {k: np.full_like(v, opt.init_m) for k, v in p_np.items()}
    v_np = {k: np.full_like(v, opt.init_v) for k, v in p_np.items()}
    for rnd in range(3):
        ld = (P + offset + 3) // 4 * 4
        x = torch.zeros(K, ld, device=cuda)
        x[:, :P + offset] = torch.from_numpy(coracle.synth_f32(K, P + offset, seed=62 + rnd)).to(cuda)
        clients = [tree_of(x[k, offset:]) for k in range(K)]  # views: offset 1 = unaligned path
        wi = [int(w) for w in ref.fedavg_weights(K, seed=70 + rnd)]
        g = tu.tree_mean(list(zip(clients, wi)))
        mean_out = {k: torch.empty_like(v) for k, v in params.items()}
        state = server.fused_tree_mean_update(zip(clients, wi), opt, params, state, mean_out=mean_out)
        d = opt.descriptor(state["count"])
        for k in sorted(sizes):
            assert np.array_equal(bits(host(mean_out[k])), bits(host(g[k]))), (rnd, k)
            p_np[k], m_np[k], v_np[k] = _np_server_step(opt, d, host(g[k]), p_np[k], m_np[k], v_np[k])
            assert np.array_equal(bits(host(params[k])), bits(p_np[k])), (rnd, k)
            if "m" in state:
                assert np.array_equal(bits(host(state["m"][k])), bits(m_np[k]))
            if "v" in state:
                assert np.array_equal(bits(host(state["v"][k])), bits(v_np[k]))
    assert state["count"] == 3
    with pytest.raises(ValueError):
        server.fused_tree_mean_update(zip(clients, wi), opt, {"a": params["a"]}, state)


# ---------------------------------------------------- native host helper (_fjhost)
def test_native_table_path_is_taken_and_bitwise_equal_to_python_path(cuda, coracle, monkeypatch):
    """Device-resident clients go through fjhost.gather_rows (a _Table) and give the same
    bits as the Python per-leaf path (forced by declining the native walk)."""
    rng = np.random.RandomState(5)
    shapes = {"conv": {"b": (32,), "w": (3, 3, 1, 32)}, "dense": [(9216, 16), (62,)], "none": None}
    K = 37

    def make():
        return {"conv": {k: torch.from_numpy(rng.uniform(-1, 1, s).astype(np.float32)).to(cuda)
                         for k, s in shapes["conv"].items()},
                "dense": [torch.from_numpy(rng.uniform(-1, 1, s).astype(np.float32)).to(cuda)
                          for s in shapes["dense"]], "none": None}

    trees = [make() for _ in range(K)]
    weights = [int(w) for w in rng.randint(1, 500, K)]
    _, rows = tu._client_table(trees)
    assert isinstance(rows, tu._Table)
    fast = tu.tree_mean(zip(trees, weights))
    fast_l2, norms = tu.tree_mean_with_l2_norms(zip(trees, weights))
    monkeypatch.setattr(tu.pytree, "native_spec", lambda td: None)
    assert isinstance(tu._client_table(trees)[1], list)
    slow = tu.tree_mean(zip(trees, weights))
    for a, b, c in zip(tu.pytree.leaves_of(fast), tu.pytree.leaves_of(slow), tu.pytree.leaves_of(fast_l2)):
        assert np.array_equal(bits(host(a)), bits(host(b))) and np.array_equal(bits(host(a)), bits(host(c)))
    want = ref.tree_mean([(tu.pytree.leaves_of(jax_free(t)), w) for t, w in zip(trees, weights)])
    for a, b in zip(tu.pytree.leaves_of(fast), want):
        assert np.array_equal(bits(host(a)), bits(b))


def jax_free(tree):
    """Host numpy copy of a device pytree (the oracle's input)."""
    return tu.pytree.unflatten(tu.pytree.flatten(tree)[1], [host(x) for x in tu.pytree.leaves_of(tree)])


def test_native_table_declines_mixed_clients(cuda):
    """A client whose leaf is on the host, of another dtype, or non-contiguous goes through
    the Python path (copied / canonicalised / rejected exactly as before)."""
    base = [{"a": torch.full((4, 4), float(k), device=cuda), "b": torch.ones(3, device=cuda)} for k in range(4)]
    mixed = [dict(t) for t in base]
    mixed[2]["a"] = mixed[2]["a"].cpu()               # host leaf: copied
    mixed[3]["a"] = mixed[3]["a"].t().contiguous().t()  # non-contiguous view: made contiguous
    assert isinstance(tu._client_table(mixed)[1], list)
    got = tu.tree_mean(zip(mixed, [1, 2, 3, 4]))
    want = tu.tree_mean(zip(base, [1, 2, 3, 4]))
    assert torch.equal(got["a"], want["a"]) and torch.equal(got["b"], want["b"])
    bad = [dict(t) for t in base]
    bad[1]["b"] = torch.ones(4, device=cuda)
    with pytest.raises(ValueError):
        tu.tree_mean(zip(bad, [1, 1, 1, 1]))
    bad[1]["b"] = torch.ones(3, dtype=torch.bfloat16, device=cuda)
    with pytest.raises(TypeError):
        tu.tree_mean(zip(bad, [1, 1, 1, 1]))


def test_native_fold_table_is_used_and_declines(cuda):
    """fjhost.fold_table (the native rest of tree_mean) launches for float32 tables, with
    misaligned leaves on element units, and gives the Python path's bits; bf16 leaves
    decline it."""
    g = torch.Generator(device="cpu").manual_seed(3)
    trees = [{"a": torch.randn(1000, generator=g).to(cuda), "b": torch.randn(7, generator=g).to(cuda)}
             for _ in range(5)]
    w = [1, 2, 3, 4, 5]
    _, rows = tu._client_table(trees)
    assert isinstance(rows, tu._Table)
    packed = tu._pack_weights(w)
    fast = tu._native_fold(rows, packed, tu._inverse(15.0))
    assert fast is not None
    slow = tu._fold([[t["a"], t["b"]] for t in trees], w, scale=tu._inverse(15.0), validated=True)
    for a, b in zip(fast, slow):
        assert a.shape == b.shape and a.dtype == b.dtype == torch.float32
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    t16 = [{"a": t["a"].bfloat16()} for t in trees]
    assert tu._native_fold(tu._client_table(t16)[1], packed, tu._inverse(15.0)) is None
    base = torch.randn(5, 1001, generator=g).to(cuda)
    odd = [{"a": base[k, 1:]} for k in range(5)]  # 4-byte offset: not 16-byte aligned
    rows_odd = tu._client_table(odd)[1]
    assert isinstance(rows_odd, tu._Table)
    fast_odd = tu._native_fold(rows_odd, packed, tu._inverse(15.0))  # per-leaf element units
    assert fast_odd is not None
    slow_odd = tu._fold([[t["a"]] for t in odd], w, scale=tu._inverse(15.0), validated=True)
    assert torch.equal(fast_odd[0].view(torch.int32), slow_odd[0].view(torch.int32))
    m = tu.tree_mean(zip(odd, w))
    assert torch.equal(m["a"], tu.tree_mean(zip([{"a": base[k, 1:].clone()} for k in range(5)], w))["a"])


@pytest.mark.parametrize("K", [4, 65, 100, 128, 129])
def test_last_workgroup_combine_matches_two_launches(K, cuda):
    """FJAGG_ZEROED_WS (include/fjagg.h): the fold's last workgroup adds the norm partials
    (K <= 128, partial rows padded to 4 floats; above, the flag only moves the partials past
    the counter). The
    norms are bitwise those of the two-launch path (k_l2_combine), the means bitwise the plain
    fold's, the counter is left zero — over calls that alternate two input sets (a stale partial
    of the previous call would show as that call's norms), with the image in device memory and
    in the kernel arguments, through fjagg_wsum_l2_ptrs and fjagg_wsum_l2_ptrs_rows."""
    import ctypes
    lib = _lib.load()
    shapes = [(32,), (3, 3, 1, 32), (64,), (3, 3, 32, 64), (128,), (9216, 128), (62,), (128, 62)]
    L = len(shapes)
    n = np.array([int(np.prod(s)) for s in shapes], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum((n + 3) // 4 * 4)])  # every leaf 16-byte aligned
    sets = []
    for seed in (5, 6):
        x = torch.empty(K, int(offs[-1]), device=cuda)
        kernels.fill_synth(x, seed=seed)
        sets.append([[x[k, offs[l]:offs[l] + n[l]] for l in range(L)] for k in range(K)])
    outs = [torch.empty(int(v), device=cuda) for v in n]
    nb = lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, None, 0)
    assert nb > 64  # many workgroups: the last-arrival order matters
    blocks = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, blocks.ctypes.data, nb)
    wh = np.float32(np.random.RandomState(K).randint(1, 50, size=K))
    need = lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, nb)
    ws0, ws1 = torch.zeros(need, dtype=torch.uint8, device=cuda), torch.empty(need, dtype=torch.uint8, device=cuda)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    sc = ctypes.c_float(0.25)
    karg_ok = lib.fjagg_karg_image_words(K, L, nb) <= 3584  # FJAGG_KARG_MAX_WORDS
    for call in range(6):
        leaves = sets[call % 2]
        karg = karg_ok and call >= 2
        img = np.concatenate([np.array([[t.data_ptr() for t in r] for r in leaves], dtype=np.int64).ravel(),
                              np.array([o.data_ptr() for o in outs], dtype=np.int64), n, blocks])
        if karg:
            img_p, w_p, flags = img.ctypes.data, wh.ctypes.data, _lib.SCALE | _lib.HOST_TABLES
        else:
            img_d, w_d = torch.from_numpy(img).to(cuda), torch.from_numpy(wh).to(cuda)
            img_p, w_p, flags = img_d.data_ptr(), w_d.data_ptr(), _lib.SCALE
        _lib.check(lib.fjagg_wsum_ptrs(_lib.F32, _lib.F32, _lib.F32, img_p, L, K, nb, w_p, sc, flags, s), "wsum")
        mean0 = torch.cat([o.clone() for o in outs])
        two, last = torch.empty(K, device=cuda), torch.empty(K, device=cuda)
        _lib.check(lib.fjagg_wsum_l2_ptrs(_lib.F32, _lib.F32, _lib.F32, img_p, L, K, nb, w_p, sc, two.data_ptr(),
                                          flags, ws1.data_ptr(), need, s), "two launches")
        _lib.check(lib.fjagg_wsum_l2_ptrs(_lib.F32, _lib.F32, _lib.F32, img_p, L, K, nb, w_p, sc, last.data_ptr(),
                                          flags | _lib.ZEROED_WS, ws0.data_ptr(), need, s), "last workgroup")
        rows = torch.full((2, K), -7.0, device=cuda)
        _lib.check(lib.fjagg_wsum_l2_ptrs_rows(_lib.F32, _lib.F32, _lib.F32, img_p, L, K, nb, w_p, sc,
                                               rows.data_ptr(), rows.data_ptr() + 4 * K, 1, flags | _lib.ZEROED_WS,
                                               ws0.data_ptr(), need, s), "rows, last workgroup")
        torch.cuda.synchronize()
        assert torch.equal(torch.cat(outs).view(torch.int32), mean0.view(torch.int32))
        assert torch.equal(last.view(torch.int32), two.view(torch.int32)), f"call {call}"
        assert torch.equal(rows[0, :K - 1].view(torch.int32), two[1:].view(torch.int32))
        assert bool((rows[:, K - 1] == -7.0).all())
        assert int(ws0[:16].count_nonzero()) == 0
        want = np.array([sum(float((t.double() ** 2).sum()) for t in r) for r in leaves])
        npt.assert_allclose(last.double().cpu().numpy(), want, rtol=2e-6)


@pytest.mark.parametrize("K,P", [(64, 1206590), (128, 1206590), (97, 1206590), (8, 1 << 25)])
def test_dense_last_workgroup_combine(K, P, cuda):
    """kernels.weighted_sum_l2_dense without a workspace uses the stream's zeroed-counter one
    (the last workgroup combines; a grid of more workgroups than CUs falls back to the combine
    launch with the flag's layout); with a caller's workspace, two launches: bitwise the same
    norms and mean, alternating two slabs."""
    xs = []
    for seed in (1, 2):
        x = torch.empty(K, (P + 3) // 4 * 4, device=cuda)[:, :P]
        kernels.fill_synth(x, seed=seed)
        xs.append(x)
    w = torch.arange(1, K + 1, dtype=torch.float32, device=cuda)
    ws = torch.empty(int(_lib.load().fjagg_wsum_l2_workspace_bytes(K, P)), dtype=torch.uint8, device=cuda)
    for call in range(4):
        x = xs[call % 2]
        o1, n1 = kernels.weighted_sum_l2_dense(x, w, scale=0.5)
        o2, n2 = kernels.weighted_sum_l2_dense(x, w, scale=0.5, workspace=ws)
        torch.cuda.synchronize()
        assert torch.equal(o1.view(torch.int32), o2.view(torch.int32))
        assert torch.equal(n1.view(torch.int32), n2.view(torch.int32)), f"call {call}"
        npt.assert_allclose(n1[:8].double().cpu().numpy(), (x[:8].double() ** 2).sum(1).cpu().numpy(), rtol=2e-6)


@pytest.mark.parametrize("zeroed", [False, True])
def test_fused_norms_propagate_nan_and_inf(zeroed, cuda):
    """tree_l2_norm semantics (tree_util.py:105-114: sqrt of a sum of squares) at the edges: a NaN
    anywhere in a client gives that client a NaN norm, an inf (or a square past f32) an inf one,
    the other clients' norms are untouched and finite; the mean is the plain fold's, bitwise. Both
    combine placements (second launch; last workgroup)."""
    import ctypes
    lib = _lib.load()
    shapes = [(37,), (4096,), (61, 13)]
    K, L = 9, len(shapes)
    g = torch.Generator().manual_seed(21)
    leaves = [[(torch.rand(s, generator=g) - 0.5).to(cuda) for s in shapes] for _ in range(K)]
    leaves[3][1][1000] = float("nan")
    leaves[5][2][7, 3] = float("inf")
    leaves[6][0][0] = 3.0e20  # its square overflows f32
    n = np.array([int(np.prod(sh)) for sh in shapes], dtype=np.int64)
    outs = [torch.empty(int(v), device=cuda) for v in n]
    nb = lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, None, 0)
    blocks = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, blocks.ctypes.data, nb)
    img = torch.from_numpy(np.concatenate([np.array([[x.data_ptr() for x in r] for r in leaves],
                                                    dtype=np.int64).ravel(),
                                           np.array([o.data_ptr() for o in outs], dtype=np.int64), n,
                                           blocks])).to(cuda)
    w = torch.arange(1, K + 1, dtype=torch.float32, device=cuda)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.fjagg_wsum_ptrs(_lib.F32, _lib.F32, _lib.F32, img.data_ptr(), L, K, nb, w.data_ptr(),
                                   ctypes.c_float(0.5), _lib.SCALE, s), "plain")
    mean0 = torch.cat([o.clone() for o in outs])
    need = lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, nb)
    ws = torch.zeros(need, dtype=torch.uint8, device=cuda)
    l2 = torch.empty(K, device=cuda)
    _lib.check(lib.fjagg_wsum_l2_ptrs(_lib.F32, _lib.F32, _lib.F32, img.data_ptr(), L, K, nb, w.data_ptr(),
                                      ctypes.c_float(0.5), l2.data_ptr(),
                                      _lib.SCALE | (_lib.ZEROED_WS if zeroed else 0), ws.data_ptr(), need, s), "l2")
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs).view(torch.int32), mean0.view(torch.int32))
    got = l2.cpu().numpy()
    assert np.isnan(got[3]) and np.isinf(got[5]) and got[5] > 0 and np.isinf(got[6]) and got[6] > 0
    want = np.array([sum(float((x.double() ** 2).sum()) for x in r) for r in leaves])
    ok = [k for k in range(K) if k not in (3, 5, 6)]
    npt.assert_allclose(got[ok].astype(np.float64), want[ok], rtol=2e-6)


@pytest.mark.parametrize("start", [5, 1000])
def test_nonzero_completion_counter_is_flagged(start, cuda):
    """FJAGG_ZEROED_WS with a counter that was NOT zero at the call (a caller that did not zero
    it, include/fjagg.h): the call sets the workspace's error word (bytes 4..7), so the invalid
    norms are detectable; zeroing both words restores the bitwise norms."""
    import ctypes
    lib = _lib.load()
    shapes = [(37,), (40960,), (61, 13)]
    K, L = 12, len(shapes)
    g = torch.Generator().manual_seed(23)
    leaves = [[(torch.rand(sh, generator=g) - 0.5).to(cuda) for sh in shapes] for _ in range(K)]
    n = np.array([int(np.prod(sh)) for sh in shapes], dtype=np.int64)
    outs = [torch.empty(int(v), device=cuda) for v in n]
    nb = lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, None, 0)
    blocks = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, blocks.ctypes.data, nb)
    img = torch.from_numpy(np.concatenate([np.array([[x.data_ptr() for x in r] for r in leaves],
                                                    dtype=np.int64).ravel(),
                                           np.array([o.data_ptr() for o in outs], dtype=np.int64), n,
                                           blocks])).to(cuda)
    w = torch.arange(1, K + 1, dtype=torch.float32, device=cuda)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    need = lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, nb)
    ws = torch.zeros(need, dtype=torch.uint8, device=cuda)
    l2, l2ok = torch.empty(K, device=cuda), torch.empty(K, device=cuda)

    def call(out):
        _lib.check(lib.fjagg_wsum_l2_ptrs(_lib.F32, _lib.F32, _lib.F32, img.data_ptr(), L, K, nb, w.data_ptr(),
                                          ctypes.c_float(0.5), out.data_ptr(), _lib.SCALE | _lib.ZEROED_WS,
                                          ws.data_ptr(), need, st), "l2")
        torch.cuda.synchronize()
        return ws[:8].view(torch.int32).cpu().tolist()
    assert call(l2ok) == [0, 0]  # a zeroed counter: left zero, no error
    ws[:4].view(torch.int32).fill_(start)
    hdr = call(l2)
    assert hdr[1] == 1, hdr  # flagged
    ws[:8].zero_()
    assert call(l2) == [0, 0]
    assert torch.equal(l2.view(torch.int32), l2ok.view(torch.int32))


def test_combine_launch_switch(cuda, monkeypatch):
    """FJAGG_L2_COMBINE_LAUNCH=1 (kernels._L2_COMBINE_LAUNCH) keeps the separate combine launch
    for weighted_sum_l2_dense's own workspace: the same bits as the in-launch combine."""
    K, P = 64, 300007
    x = torch.empty(K, (P + 3) // 4 * 4, device=cuda)[:, :P]
    kernels.fill_synth(x, seed=4)
    w = torch.arange(1, K + 1, dtype=torch.float32, device=cuda)
    o1, n1 = kernels.weighted_sum_l2_dense(x, w, scale=0.25)
    monkeypatch.setattr(kernels, "_L2_COMBINE_LAUNCH", True)
    o2, n2 = kernels.weighted_sum_l2_dense(x, w, scale=0.25)
    torch.cuda.synchronize()
    assert torch.equal(o1.view(torch.int32), o2.view(torch.int32))
    assert torch.equal(n1.view(torch.int32), n2.view(torch.int32))


def test_last_workgroup_combine_many_leaves(cuda):
    """A plan of more workgroups than CUs (one or more per leaf: 300 leaves) keeps the
    FJAGG_ZEROED_WS layout but combines in a second launch: norms bitwise the plain two-launch
    call's, the counter untouched."""
    import ctypes
    lib = _lib.load()
    K, L = 12, 300
    g = torch.Generator().manual_seed(11)
    leaves = [[(torch.rand(40 + 8 * l, generator=g) - 0.5).to(cuda) for l in range(L)] for _ in range(K)]
    n = np.array([40 + 8 * l for l in range(L)], dtype=np.int64)
    outs = [torch.empty(int(v), device=cuda) for v in n]
    nb = lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, None, 0)
    assert nb >= L
    blocks = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, blocks.ctypes.data, nb)
    img = torch.from_numpy(np.concatenate([np.array([[x.data_ptr() for x in r] for r in leaves],
                                                    dtype=np.int64).ravel(),
                                           np.array([o.data_ptr() for o in outs], dtype=np.int64), n,
                                           blocks])).to(cuda)
    w = torch.arange(1, K + 1, dtype=torch.float32, device=cuda)
    need = lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, nb)
    ws0, ws1 = torch.zeros(need, dtype=torch.uint8, device=cuda), torch.empty(need, dtype=torch.uint8, device=cuda)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a, b = torch.empty(K, device=cuda), torch.empty(K, device=cuda)
    _lib.check(lib.fjagg_wsum_l2_ptrs(_lib.F32, _lib.F32, _lib.F32, img.data_ptr(), L, K, nb, w.data_ptr(),
                                      ctypes.c_float(1.0), a.data_ptr(), 0, ws1.data_ptr(), need, s), "two launches")
    _lib.check(lib.fjagg_wsum_l2_ptrs(_lib.F32, _lib.F32, _lib.F32, img.data_ptr(), L, K, nb, w.data_ptr(),
                                      ctypes.c_float(1.0), b.data_ptr(), _lib.ZEROED_WS, ws0.data_ptr(), need, s),
               "flag, many workgroups")
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    assert int(ws0[:16].count_nonzero()) == 0
    want = np.array([sum(float((x.double() ** 2).sum()) for x in r) for r in leaves])
    npt.assert_allclose(b.double().cpu().numpy(), want, rtol=2e-6)


@pytest.mark.parametrize("karg", [False, True])
def test_wsum_l2_ptrs_rows_writes_the_norm_rows(karg, cuda):
    """fjagg_wsum_l2_ptrs_rows (the deferred running sum's lazy-norm rows, include/fjagg.h):
    the mean is bitwise fjagg_wsum_ptrs'; operand k >= first gets fjagg_wsum_l2_ptrs' squared
    norm (bitwise) in sq[k - first] and its correctly rounded sqrt in nrm[k - first]; nothing
    below `first`, nor past the K - first written entries, is touched (first = K: nothing). With
    the plan image in device memory and in the kernel arguments (FJAGG_HOST_TABLES), the combine
    in a second launch and in the last workgroup (FJAGG_ZEROED_WS)."""
    import ctypes
    lib = _lib.load()
    shapes = [(37,), (3, 3, 4), (1000,), (61, 13)]
    K, L = 7, len(shapes)
    g = torch.Generator().manual_seed(3)
    leaves = [[(torch.rand(s, generator=g) - 0.5).to(cuda) for s in shapes] for _ in range(K)]
    n = np.array([int(np.prod(s)) for s in shapes], dtype=np.int64)
    outs = [torch.empty(int(v), device=cuda) for v in n]
    nb = lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, None, 0)
    blocks = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, n.ctypes.data, None, L, blocks.ctypes.data, nb)
    img = np.concatenate([np.array([[x.data_ptr() for x in r] for r in leaves], dtype=np.int64).ravel(),
                          np.array([o.data_ptr() for o in outs], dtype=np.int64), n, blocks])
    wh = np.float32([3, 1, 4, 1, 5, 9, 2])
    flags = _lib.SCALE | (_lib.HOST_TABLES if karg else 0)
    if karg:
        img_p, w_p = img.ctypes.data, wh.ctypes.data
    else:
        img_d, w_d = torch.from_numpy(img).to(cuda), torch.from_numpy(wh).to(cuda)
        img_p, w_p = img_d.data_ptr(), w_d.data_ptr()
    ws = torch.empty(max(4, lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, nb)), dtype=torch.uint8, device=cuda)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.fjagg_wsum_ptrs(_lib.F32, _lib.F32, _lib.F32, img_p, L, K, nb, w_p, ctypes.c_float(0.04), flags, s),
               "wsum")
    mean0 = torch.cat([o.clone() for o in outs])
    l2 = torch.empty(K, device=cuda)
    _lib.check(lib.fjagg_wsum_l2_ptrs(_lib.F32, _lib.F32, _lib.F32, img_p, L, K, nb, w_p, ctypes.c_float(0.04),
                                      l2.data_ptr(), flags, ws.data_ptr(), ws.numel(), s), "l2")
    wz = torch.zeros_like(ws)  # FJAGG_ZEROED_WS: the last workgroup writes the rows
    for first, zeroed in ((0, False), (1, False), (3, False), (0, True), (1, True), (K, True), (K, False)):
        rows = torch.full((2, K + 2), -7.0, device=cuda)
        wsp, fl = (wz.data_ptr(), flags | _lib.ZEROED_WS) if zeroed else (ws.data_ptr(), flags)
        _lib.check(lib.fjagg_wsum_l2_ptrs_rows(_lib.F32, _lib.F32, _lib.F32, img_p, L, K, nb, w_p,
                                               ctypes.c_float(0.04), rows.data_ptr(), rows.data_ptr() + 4 * (K + 2),
                                               first, fl, wsp, ws.numel(), s), "rows")
        torch.cuda.synchronize()
        assert torch.equal(torch.cat(outs).view(torch.int32), mean0.view(torch.int32))
        m = K - first
        assert torch.equal(rows[0, :m].view(torch.int32), l2[first:].view(torch.int32))
        want_sqrt = np.sqrt(l2[first:].cpu().numpy())  # IEEE binary32 sqrt, correctly rounded
        assert np.array_equal(rows[1, :m].cpu().numpy().view(np.uint32), want_sqrt.view(np.uint32))
        assert bool((rows[:, m:] == -7.0).all())
        assert int(wz[:16].count_nonzero()) == 0
    want = np.array([sum(float((x.double() ** 2).sum()) for x in r) for r in leaves])
    npt.assert_allclose(l2.double().cpu().numpy(), want, rtol=2e-6)
    bad = lib.fjagg_wsum_l2_ptrs_rows(_lib.F32, _lib.F32, _lib.F32, img_p, L, K, nb, w_p, ctypes.c_float(1.0),
                                      None, None, 0, flags, ws.data_ptr(), ws.numel(), s)
    assert bad == -1 and b"null pointer" in lib.fjagg_last_error()  # FJAGG_EINVAL


def test_native_fold_table_fused_l2(cuda):
    """fjhost.fold_table with l2sq launches fjagg_wsum_l2_ptrs: the mean and norms are
    bitwise those of the Python fused path, for aligned and misaligned leaves."""
    g = torch.Generator(device="cpu").manual_seed(9)
    base = torch.randn(7, 3001, generator=g).to(cuda)
    for off in (0, 1):
        trees = [{"a": base[k, off:off + 1000], "b": base[k, off + 1000:off + 3000]} for k in range(7)]
        w = [3, 1, 4, 1, 5, 9, 2]
        _, rows = tu._client_table(trees)
        assert isinstance(rows, tu._Table)
        q_fast = torch.empty(7, device=cuda)
        fast = tu._native_fold(rows, tu._pack_weights(w), tu._inverse(25.0), None, False, q_fast)
        assert fast is not None
        q_slow = torch.empty(7, device=cuda)
        slow = tu._fold([[t["a"], t["b"]] for t in trees], w, scale=tu._inverse(25.0), validated=True, l2sq=q_slow)
        for a, b in zip(fast, slow):
            assert torch.equal(a.view(torch.int32), b.view(torch.int32))
        assert torch.equal(q_fast.view(torch.int32), q_slow.view(torch.int32))
        m, n = tu.tree_mean_with_l2_norms(zip(trees, w))
        assert torch.equal(m["a"], fast[0])
        # the norms: correctly rounded square roots (IEEE binary32, numpy's) of the same squares
        assert np.array_equal(n.cpu().numpy().view(np.uint32), np.sqrt(q_fast.cpu().numpy()).view(np.uint32))


def test_tree_mean_streams_one_shot_iterables(cuda, monkeypatch):
    """a generator is consumed in chunks under STREAM_BUDGET_BYTES (accumulate
    mode, scale fused into the last chunk) — bitwise the one-launch fold of the same list,
    for host (numpy) and device deltas, chunk boundaries landing anywhere (incl. exactly
    at the end), and only one chunk of host deltas is ever copied to the GPU."""
    K = 23
    g = np.random.RandomState(3)
    host_trees = [{"a": g.uniform(-1, 1, 1001).astype(np.float32), "b": g.uniform(-1, 1, (3, 4)).astype(np.float32)}
                  for _ in range(K)]
    wi = [int(v) for v in ref.fedavg_weights(K, seed=5)]
    wi[4] = 0.25
    want = tu.tree_mean(list(zip([{k: torch.from_numpy(v).to(cuda) for k, v in t.items()} for t in host_trees], wi)))
    per = 4 * (1001 + 12)
    for B in (1, 5, 23, 24, 100):
        monkeypatch.setattr(tu, "STREAM_BUDGET_BYTES", B * per)
        for trees in (host_trees, [{k: torch.from_numpy(v).to(cuda) for k, v in t.items()} for t in host_trees]):
            got = tu.tree_mean((t, w) for t, w in zip(trees, wi))
            for k in ("a", "b"):
                assert torch.equal(got[k].view(torch.int32), want[k].view(torch.int32)), (B, k)
    # the aggregator's lazy map goes through the same path
    monkeypatch.setattr(tu, "STREAM_BUDGET_BYTES", 4 * per)
    agg = fedjax_amd.aggregators.mean_aggregator()
    got, _ = agg.apply(((f"c{i}", t, w) for i, (t, w) in enumerate(zip(host_trees, wi))), agg.init())
    assert torch.equal(got["a"].view(torch.int32), want["a"].view(torch.int32))
    with pytest.raises(ValueError):
        tu.tree_mean(iter([({"a": np.zeros(3, np.float32)}, 1)] * 5 + [({"b": np.zeros(3, np.float32)}, 1)]))
    assert tu.tree_mean(iter([])) is None


def test_l2_of_int_and_mixed_leaves_and_many_clients(cuda):
    """tree_l2_squared / tree_l2_norm accept int32 and mixed-dtype pytrees like
    the reference's sum(jnp.vdot(x, x)) (int32 squares wrap), and tree_mean_with_l2_norms
    takes K > 4096 clients (two passes instead of the fused one)."""
    t = {"i": torch.tensor([3, 4], dtype=torch.int32, device=cuda), "f": torch.tensor([1.5], device=cuda)}
    sq = tu.tree_l2_squared(t)
    assert sq.dtype == torch.float32 and float(sq) == 27.25
    npt.assert_allclose(float(tu.tree_l2_norm(t)), np.sqrt(27.25), rtol=1e-7)
    ti = {"i": torch.tensor([46341, 1], dtype=torch.int32, device=cuda)}  # 46341^2 > 2^31: wraps
    want = np.int32(np.int64(46341) ** 2 + 1 - 2 ** 32)
    got = tu.tree_l2_squared(ti)
    assert got.dtype == torch.int32 and int(got) == int(want)
    K = 4100
    trees = [{"w": torch.full((3,), float(k % 7), device=cuda)} for k in range(K)]
    m, norms = tu.tree_mean_with_l2_norms(zip(trees, [1] * K))
    assert norms.shape == (K,)
    npt.assert_allclose(host(norms)[:8], [np.sqrt(3) * (k % 7) for k in range(8)], rtol=1e-6)
    assert torch.equal(m["w"], tu.tree_mean(list(zip(trees, [1] * K)))["w"])


@pytest.mark.parametrize("K,sizes,dt", [
    (4096, [32, 288, 64, 18432, 128, 20000, 62, 7936 - 2], "f32"),  # a small CNN, many clients
    (300, [5, 64, 1000, 3], "f32"), (1000, [4099, 17], "bf16"), (777, [100, 2000], "i32"),
    (16, [64 * 300], "f32")])
def test_ptrs_stripe_plan_bitwise(K, sizes, dt, cuda, coracle):
    """k_ptrs_stripe (FJAGG_NARROW | FJAGG_VARIANT(20 / 21 / 22)): C-element stripes of every
    leaf (leaves not multiples of C, shorter than C, tiles not full), client rows from the
    K x L pointer table staged in LDS by the fold wave, accumulate mode — bitwise the
    k_ptrs_narrow plan (variant 0) and, for f32, the oracle."""
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "i32": torch.int32}[dt]
    in_c = kernels.dtype_code(tdt)
    g = torch.Generator().manual_seed(K + len(sizes))
    leaves = []
    for k in range(K):
        row = []
        for n in sizes:
            x = (torch.rand(n, generator=g) * 2 - 1) * 0.01
            row.append((x * 1e6).to(torch.int32).to(cuda) if dt == "i32" else x.to(tdt).to(cuda))
        leaves.append(row)
    L = len(sizes)
    leaf_n = np.array(sizes, dtype=np.int64)
    in_ptrs = np.array([[t.data_ptr() for t in r] for r in leaves], dtype=np.int64)
    assert not (in_ptrs & 15).any()
    if dt == "i32":
        acc_c, out_dt = _lib.I32, torch.int32
        w = torch.tensor([int(v) for v in ref.fedavg_weights(K, seed=9)], dtype=torch.int32, device=cuda)
        scale = None
    else:
        acc_c, out_dt = _lib.F32, tdt
        w = torch.tensor(np.float32(ref.fedavg_weights(K, seed=9)), device=cuda)
        scale = 0.125
    res = {}
    for acc in (False, True):
        for v in (0, 20, 21, 22):
            outs = [torch.full((n,), 3, dtype=out_dt, device=cuda) for n in sizes]
            out_ptrs = np.array([o.data_ptr() for o in outs], dtype=np.int64)
            blocks = kernels.ptrs_plan(in_c, leaf_n, False, narrow=True, stripe_variant=v)
            image = np.concatenate([in_ptrs.ravel(), out_ptrs, leaf_n, blocks])
            img = torch.from_numpy(image).to(cuda)
            kernels.weighted_sum_ptrs(in_c, acc_c, kernels.dtype_code(out_dt), img, L, K, len(blocks) // 2, w, scale,
                                      accumulate=acc, narrow=True, stripe_variant=v)
            torch.cuda.synchronize()
            res[(acc, v)] = [o.view(torch.uint8).cpu().numpy() for o in outs]
        for v in (20, 21, 22):
            for a, b in zip(res[(acc, 0)], res[(acc, v)]):
                assert np.array_equal(a, b), (acc, v)
    if dt == "f32":
        for l, n in enumerate(sizes):
            xs = np.stack([leaves[k][l].cpu().numpy() for k in range(K)])
            want = coracle.wsum_f32(xs, host(w), scale=np.float32(0.125))
            assert np.array_equal(res[(False, 20)][l].view(np.uint32), bits(want)), l
