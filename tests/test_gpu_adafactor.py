"""fedjax.optimizers.adafactor (fedjax/core/optimizers.py:284-348 = optax.adafactor) as the
server step: the GPU chain of include/fjopt.h against the numpy restatement
oracle/optax_ref.py (parity unpinned against optax, which is absent: see its header).

Elementwise ops are the same float32 ops in the same order on both sides; the means are
float64 sums in different fixed orders, rounded once, so results agree to a few float32
ulps (rtol below), not bitwise. Shapes cover every factoring case of
optax's _factored_dims: d0 before / after d1, extra leading / middle / trailing axes,
equal dimensions (numpy's argsort tie order), small and 1-D leaves (unfactored)."""
import numpy as np
import pytest
import torch

from fedjax_amd import server, tree_util as tu
from oracle import optax_ref as ref

pytestmark = pytest.mark.gpu
RTOL, ATOL = 2e-5, 1e-9

SHAPES = {
    "a_dense": (300, 200),        # d0 = 0 (lo), d1 = 1
    "b_dense_t": (130, 257),      # d0 = 1 (hi)
    "c_3d": (4, 129, 160),        # A = 4
    "d_conv": (3, 3, 128, 256),   # d1 = 2, d0 = 3, A = 9
    "e_mid": (160, 2, 140),       # B = 2 between the factored axes
    "f_square": (128, 128),       # argsort tie
    "g_bias": (200,),             # 1-D: unfactored
    "h_small": (64, 32),          # second dim < 128: unfactored
    "i_scalar": (),               # 0-d
}

CONFIGS = {
    "defaults": dict(learning_rate=0.05),
    "momentum_wd_mask": dict(learning_rate=0.05, momentum=0.9, weight_decay_rate=0.01,
                             weight_decay_mask={k: k < "e" for k in SHAPES}),
    "no_clip_no_scale": dict(learning_rate=0.1, clipping_threshold=None, multiply_by_parameter_scale=False),
    "schedule_offset": dict(learning_rate=lambda c: 0.1 / (1 + c), decay_offset=1, decay_rate=0.7,
                            clipping_threshold=1.5, min_dim_size_to_factor=100),
    "unfactored": dict(learning_rate=0.05, factored=False, eps=1e-20),
    "no_lr": dict(learning_rate=None, clipping_threshold=0.5),
}


def _host(tree):
    return {k: v.detach().cpu().numpy() for k, v in tree.items()}


def _draw(seed, shapes=SHAPES, scale=1.0):
    rs = np.random.RandomState(seed)
    return {k: (rs.standard_normal(s) * scale).astype(np.float32) for k, s in shapes.items()}


def _dev(tree):
    return {k: torch.from_numpy(np.array(v, dtype=np.float32, copy=True)).cuda() for k, v in tree.items()}


def _compare(got, want, what):
    for k in want:
        np.testing.assert_allclose(got[k], want[k], rtol=RTOL, atol=ATOL, err_msg=f"{what}[{k}]")


@pytest.mark.parametrize("name", list(CONFIGS))
def test_adafactor_matches_restated_optax(name, cuda):
    cfg = CONFIGS[name]
    opt = server.adafactor(**cfg)
    p_host = _draw(0)
    params = _dev(p_host)
    state = opt.init(params)
    ref_state = ref.init(p_host, factored=opt.factored, min_dim_size_to_factor=opt.min_dim_size_to_factor,
                         momentum=opt.momentum)
    for k in SHAPES:  # optax's state shapes
        for what in ("v_row", "v_col", "v"):
            assert tuple(state[what][k].shape) == ref_state[what][k].shape, (k, what)
    kw = {k: v for k, v in cfg.items()}
    c0 = 3 if opt.decay_offset else 0  # decay_offset: fine-tuning that starts at a later step
    state["count"] = ref_state["count"] = c0
    for step in range(4):
        g_host = _draw(100 + step, scale=0.01 * (step + 1))
        state, params = opt.apply(_dev(g_host), state, params)
        ref_state, p_host = ref.apply(g_host, ref_state, p_host, **kw)
        torch.cuda.synchronize()
        assert state["count"] == ref_state["count"] == c0 + step + 1
        _compare(_host(params), p_host, f"step {step} params")
        for what in ("v_row", "v_col", "v") + (("m",) if opt.momentum is not None else ()):
            _compare(_host(state[what]), ref_state[what], f"step {step} {what}")


def test_adafactor_first_step_closed_form(cuda):
    """Count 0: decay_rate_t = 0, so v = g*g + eps and, unfactored, u = g / sqrt(g*g + eps);
    with clipping off, no param scale and lr 1 the params move by exactly -u."""
    opt = server.adafactor(1.0, clipping_threshold=None, multiply_by_parameter_scale=False, factored=False)
    g = np.array([0.5, -2.0, 3e-3, 0.0, 7.0], np.float32)
    p = np.ones(5, np.float32)
    params = {"w": torch.from_numpy(p.copy()).cuda()}
    state = opt.init(params)
    state, params = opt.apply({"w": torch.from_numpy(g).cuda()}, state, params)
    gs = (g * g + np.float32(1e-30)).astype(np.float32)
    u = (g * (1.0 / np.sqrt(gs.astype(np.float64))).astype(np.float32)).astype(np.float32)
    np.testing.assert_array_equal(params["w"].cpu().numpy(), p - u)
    np.testing.assert_array_equal(state["v"]["w"].cpu().numpy(), gs)


def test_fused_tree_mean_update_is_mean_then_apply(cuda):
    """fused_tree_mean_update with adafactor = tree_mean, then apply: the same kernels, bitwise."""
    opt = server.adafactor(0.05, momentum=0.5)
    K = 7
    clients = [_dev(_draw(10 + k, scale=0.01)) for k in range(K)]
    weights = [3, 1, 4, 1, 5, 9, 2]
    pa, pb = _dev(_draw(1)), _dev(_draw(1))
    sa, sb = opt.init(pa), opt.init(pb)
    mean_out = {k: torch.empty_like(v) for k, v in pa.items()}
    for _ in range(2):
        sa = server.fused_tree_mean_update(list(zip(clients, weights)), opt, pa, sa, mean_out=mean_out)
        mean = tu.tree_mean(list(zip(clients, weights)))
        sb, pb = opt.apply(mean, sb, pb)
    for k in SHAPES:
        np.testing.assert_array_equal(pa[k].cpu().numpy(), pb[k].cpu().numpy())
        np.testing.assert_array_equal(mean_out[k].cpu().numpy(), mean[k].cpu().numpy())
    assert sa["count"] == sb["count"] == 2


def test_slab_path_equals_pytree_path(cuda):
    from fedjax_amd.slab import ClientDeltaSlab
    shapes = {k: SHAPES[k] for k in ("a_dense", "d_conv", "g_bias", "h_small")}
    opt = server.adafactor(0.05, weight_decay_rate=1e-3)
    template = _dev(_draw(0, shapes))
    K = 5
    slab = ClientDeltaSlab(template, K)
    host = [_draw(20 + k, shapes, scale=0.01) for k in range(K)]
    for k in range(K):
        for name, leaf in slab.client(k).items():
            leaf.copy_(torch.from_numpy(host[k][name]))
    weights = [1.0, 2.0, 3.0, 4.0, 5.0]
    flat = torch.empty(slab.num_params, dtype=torch.float32, device="cuda")
    for name, leaf in slab.unflatten(flat).items():
        leaf.copy_(template[name])
    st_flat = opt.init(slab.unflatten(flat))
    st_flat = server.fused_mean_update(slab, weights, opt, flat, st_flat)
    tree_p = {k: v.clone() for k, v in template.items()}
    st_tree = opt.init(tree_p)
    st_tree = server.fused_tree_mean_update(list(zip([_dev(h) for h in host], weights)), opt, tree_p, st_tree)
    for name, leaf in slab.unflatten(flat).items():
        np.testing.assert_array_equal(leaf.cpu().numpy(), tree_p[name].cpu().numpy())
    assert st_flat["count"] == st_tree["count"] == 1


def test_ignore_grads_haiku_adafactor(cuda):
    params = {"linear": {"w": torch.randn(256, 130, device="cuda"), "b": torch.randn(130, device="cuda")},
              "norm": {"scale": torch.ones(130, device="cuda")}}
    opt = server.ignore_grads_haiku(server.adafactor(0.1), [("norm", "scale"), ("linear", "b")])
    before = {m: {n: t.clone() for n, t in d.items()} for m, d in params.items()}
    state = opt.init(params)
    grads = {m: {n: torch.randn_like(t) for n, t in d.items()} for m, d in params.items()}
    state, params = opt.apply(grads, state, params)
    assert torch.equal(params["norm"]["scale"], before["norm"]["scale"])
    assert torch.equal(params["linear"]["b"], before["linear"]["b"])
    assert not torch.equal(params["linear"]["w"], before["linear"]["w"])
    assert float(state["v"]["norm"]["scale"].abs().sum()) == 0.0  # frozen state untouched


def test_adafactor_rejects_bad_state(cuda):
    opt = server.adafactor(0.1)
    params = {"w": torch.randn(256, 200, device="cuda")}
    state = opt.init(params)
    state["v_row"] = {"w": torch.zeros(199, device="cuda")}
    with pytest.raises(ValueError, match="factored shapes"):
        opt.apply({"w": torch.randn(256, 200, device="cuda")}, state, params)
    with pytest.raises(ValueError, match="grads"):
        opt.apply({"w": torch.randn(256, 200, device="cuda", dtype=torch.float64)}, opt.init(params), params)
