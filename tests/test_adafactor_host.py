"""Host side of the adafactor server step (no GPU): optax's factoring rule, the state
shapes of init, the C plan's validation (include/fjopt.h), and the numpy restatement's
closed-form first step (oracle/optax_ref.py, test infrastructure)."""
import ctypes

import numpy as np
import pytest
import torch

from fedjax_amd import _lib, server
from oracle import optax_ref as ref

SHAPES = [(), (7,), (64, 32), (128, 128), (300, 200), (130, 257), (3, 3, 128, 256), (160, 2, 140), (127, 4096),
          (128, 127), (5, 129, 1, 130)]


@pytest.mark.parametrize("factored", [True, False])
@pytest.mark.parametrize("min_dim", [1, 64, 128, 200])
def test_factored_dims_agree_with_the_restatement(factored, min_dim):
    for s in SHAPES:
        assert server._factored_dims(s, factored, min_dim) == ref.factored_dims(s, factored, min_dim), s


def test_init_has_optax_state_shapes():
    params = {f"p{i}": torch.zeros(s) for i, s in enumerate(SHAPES)}
    opt = server.adafactor(0.1, momentum=0.9)
    st = opt.init(params)
    want = ref.init({k: v.numpy() for k, v in params.items()}, momentum=0.9)
    assert st["count"] == 0
    for what in ("v_row", "v_col", "v", "m"):
        for k in params:
            assert tuple(st[what][k].shape) == want[what][k].shape, (what, k)


def test_hparams_follow_optax_constants():
    opt = server.adafactor(lambda c: 0.5 / (c + 1), decay_rate=0.8, decay_offset=2, momentum=0.9,
                           weight_decay_rate=0.1)
    h = opt.hparams(5)
    d = np.float32(1) - np.power(np.float32(4), np.float32(-0.8))
    assert np.float32(h.decay_rate_t) == d and np.float32(h.one_minus_decay) == np.float32(1) - d
    assert np.float32(h.lr) == np.float32(0.5 / 6)
    assert np.float32(h.one_minus_mom) == np.float32(1.0 - 0.9)  # weak-typed Python 1 - decay
    assert (h.clip, h.param_scale, h.momentum, h.weight_decay, h.has_lr) == (1, 1, 1, 1, 1)
    assert server.adafactor(None).hparams(0).has_lr == 0


def _leaf(n, dims, factored=0, d0lo=0):
    r = _lib.AfLeaf()
    r.g, r.p, r.n = 1 << 20, 2 << 20, n
    r.v_row, r.v_col, r.v = 3 << 20, 4 << 20, 5 << 20
    r.dims[:] = dims
    r.factored, r.d0_is_lo = factored, d0lo
    return r


def test_plan_validates_and_sizes():
    lib = _lib.load()
    hp = server.adafactor(0.1, momentum=0.5).hparams(0)
    ws = ctypes.c_int64()
    recs = (_lib.AfLeaf * 2)(_leaf(60000, (1, 300, 1, 200, 1), 1, 1), _leaf(200, (1, 200, 1, 1, 1)))
    assert lib.fjopt_adafactor_plan(recs, 2, ctypes.byref(hp), None, 0, ctypes.byref(ws)) < 0  # momentum, no m
    assert b"momentum" in lib.fjagg_last_error()
    hp = server.adafactor(0.1).hparams(0)
    words = lib.fjopt_adafactor_plan(recs, 2, ctypes.byref(hp), None, 0, ctypes.byref(ws))
    assert words > 0 and ws.value > 0
    table = np.zeros(words, np.int64)
    assert lib.fjopt_adafactor_plan(recs, 2, ctypes.byref(hp), table.ctypes.data, words, ctypes.byref(ws)) == words
    assert table[21] == 2  # leaves
    assert lib.fjopt_adafactor_plan(recs, 2, ctypes.byref(hp), table.ctypes.data, words - 1, ctypes.byref(ws)) < 0
    bad = (_lib.AfLeaf * 1)(_leaf(100, (1, 300, 1, 200, 1), 1, 1))
    assert lib.fjopt_adafactor_plan(bad, 1, ctypes.byref(hp), None, 0, ctypes.byref(ws)) < 0
    assert b"multiply" in lib.fjagg_last_error()


def test_restatement_first_step_closed_form():
    """Count 0: decay_rate_t = 0, v = g*g + eps; unfactored u = g / sqrt(v); factored u =
    g * (v_row / mean(v_row)) ** -0.5 * v_col ** -0.5 with v_row, v_col the means of g*g+eps."""
    rs = np.random.RandomState(0)
    g = {"b": rs.standard_normal(5).astype(np.float32), "w": rs.standard_normal((256, 130)).astype(np.float32)}
    p = {k: np.zeros_like(v) for k, v in g.items()}
    kw = dict(learning_rate=1.0, clipping_threshold=None, multiply_by_parameter_scale=False)
    st, out = ref.apply(g, ref.init(p), p, **kw)
    gs = g["b"] * g["b"] + np.float32(1e-30)
    np.testing.assert_array_equal(st["v"]["b"], gs)
    np.testing.assert_allclose(out["b"], -g["b"] / np.sqrt(gs), rtol=1e-6)
    gw = g["w"].astype(np.float64) ** 2 + 1e-30
    vr, vc = gw.mean(axis=0), gw.mean(axis=1)  # d0 = 0 (256 rows), d1 = 1
    np.testing.assert_allclose(st["v_row"]["w"], vr, rtol=1e-6)
    np.testing.assert_allclose(st["v_col"]["w"], vc, rtol=1e-6)
    u = g["w"] * (vr / vr.mean())[None, :] ** -0.5 * vc[:, None] ** -0.5
    np.testing.assert_allclose(out["w"], -u, rtol=1e-5)
