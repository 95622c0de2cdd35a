"""Test infrastructure only (the product never imports this): a numpy restatement of
fedjax.optimizers.adafactor (fedjax/core/optimizers.py:284-348), which wraps
optax.adafactor with create_optimizer_from_optax (optimizers.py:57-66).

PARITY UNPINNED: optax is a third-party dependency of the reference (setup.py:42, no
version pin) that is absent from this image and from /root/reference, and no reference
test covers adafactor. The chain below restates optax's published algorithm
(optax/_src/alias.py ``adafactor``, optax/_src/factorized.py ``scale_by_factored_rms``):

    scale_by_factored_rms(factored, decay_rate, decay_offset, min_dim_size_to_factor, eps)
    clip_by_block_rms(clipping_threshold)            if clipping_threshold is not None
    scale_by_learning_rate(learning_rate, flip_sign=False)   if learning_rate is not None
    scale_by_param_block_rms()                       if multiply_by_parameter_scale
    ema(momentum, debias=False)                      if momentum is not None
    add_decayed_weights(weight_decay_rate, mask)     if weight_decay_rate is not None
    scale(-1);  apply_updates: p + u

Elementwise ops are float32 numpy ops in optax's order (numpy does not contract into FMA);
``x ** -0.5``, divisions and sqrt are correctly rounded (computed in float64, rounded
once). Means (jnp.mean) are float64 sums of the float32 terms, divided by the count and
rounded once — the GPU kernels (fedjax_amd/csrc/fjopt.hip) do the same in another fixed
order, so the two agree to a few float32 ulps, not bitwise.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

f32 = np.float32


def factored_dims(shape, factored: bool, min_dim_size_to_factor: int):
    """optax factorized._factored_dims: (d1, d0) = (second largest, largest) axis, or None."""
    if not factored or len(shape) < 2:
        return None
    sorted_dims = np.argsort(shape)
    if shape[sorted_dims[-2]] < min_dim_size_to_factor:
        return None
    return int(sorted_dims[-2]), int(sorted_dims[-1])


def decay_rate_pow(i: int, exponent: float) -> np.float32:
    """optax factorized._decay_rate_pow: 1 - (i + 1) ** -exponent in float32."""
    t = f32(i + 1)
    return f32(1) - np.power(t, f32(-exponent))


def _mean(x, axis=None, keepdims=False) -> np.ndarray:
    n = x.size if axis is None else x.shape[axis]
    s = np.sum(x.astype(np.float64), axis=axis, keepdims=keepdims)
    return np.asarray(s / n).astype(np.float32)


def _rsqrt(x) -> np.ndarray:
    return (1.0 / np.sqrt(np.asarray(x, np.float64))).astype(np.float32)


def _sqrt(x) -> np.ndarray:
    return np.sqrt(np.asarray(x, np.float64)).astype(np.float32)


def _div(a, b) -> np.ndarray:
    return (np.asarray(a, np.float64) / np.asarray(b, np.float64)).astype(np.float32)


def init(params: dict, *, factored=True, min_dim_size_to_factor=128, momentum=None) -> dict:
    """optax state for a flat dict of float32 leaves: count, v_row / v_col / v per leaf
    (the shapes of scale_by_factored_rms's init) and the ema when momentum is on."""
    st = {"count": 0, "v_row": {}, "v_col": {}, "v": {}}
    for k, p in params.items():
        fd = factored_dims(p.shape, factored, min_dim_size_to_factor)
        if fd is not None:
            d1, d0 = fd
            st["v_row"][k] = np.zeros(np.delete(p.shape, d0), f32)
            st["v_col"][k] = np.zeros(np.delete(p.shape, d1), f32)
            st["v"][k] = np.zeros((1,), f32)
        else:
            st["v_row"][k] = np.zeros((1,), f32)
            st["v_col"][k] = np.zeros((1,), f32)
            st["v"][k] = np.zeros(p.shape, f32)
    if momentum is not None:
        st["m"] = {k: np.zeros(p.shape, f32) for k, p in params.items()}
    return st


def apply(grads: dict, state: dict, params: dict, *, learning_rate=None, min_dim_size_to_factor=128,
          decay_rate=0.8, decay_offset=0, multiply_by_parameter_scale=True,
          clipping_threshold: Optional[float] = 1.0, momentum: Optional[float] = None,
          weight_decay_rate: Optional[float] = None, eps=1e-30, factored=True, weight_decay_mask=None):
    """One optimizer.apply(grads, state, params) -> (state, params), new arrays."""
    count = state["count"]
    d = decay_rate_pow(count - decay_offset, decay_rate)
    omd = f32(1) - d
    new = {"count": count + 1, "v_row": {}, "v_col": {}, "v": {}}
    out = {}
    if momentum is not None:
        new["m"] = {}
    for k in params:
        g, p = grads[k].astype(f32), params[k].astype(f32)
        gs = g * g + f32(eps)
        fd = factored_dims(p.shape, factored, min_dim_size_to_factor)
        if fd is not None:
            d1, d0 = fd
            vr = d * state["v_row"][k] + omd * _mean(gs, axis=d0)
            vc = d * state["v_col"][k] + omd * _mean(gs, axis=d1)
            rd1 = d1 - 1 if d1 > d0 else d1
            rcm = _mean(vr, axis=rd1, keepdims=True)
            rf = _rsqrt(_div(vr, rcm))
            cf = _rsqrt(vc)
            u = g * np.expand_dims(rf, d0) * np.expand_dims(cf, d1)
            new["v_row"][k], new["v_col"][k], new["v"][k] = vr, vc, state["v"][k]
        else:
            v = d * state["v"][k] + omd * gs
            u = g * _rsqrt(v)
            new["v_row"][k], new["v_col"][k], new["v"][k] = state["v_row"][k], state["v_col"][k], v
        if clipping_threshold is not None:
            denom = np.maximum(f32(1), _div(_sqrt(_mean(u * u)), f32(clipping_threshold)))
            u = _div(u, denom)
        if learning_rate is not None:
            lr = learning_rate(count) if callable(learning_rate) else learning_rate
            u = u * f32(lr)
        if multiply_by_parameter_scale:
            u = u * np.maximum(_sqrt(_mean(p * p)), f32(1e-3))
        if momentum is not None:
            u = f32(1.0 - momentum) * u + f32(momentum) * state["m"][k]
            new["m"][k] = u
        if weight_decay_rate is not None and (weight_decay_mask is None or weight_decay_mask[k]):
            u = u + f32(weight_decay_rate) * p
        out[k] = p + (-u)
    return new, out
