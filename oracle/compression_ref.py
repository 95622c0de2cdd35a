"""TEST INFRASTRUCTURE ONLY — numpy restatement of FedJAX's compression
aggregators (the callers that feed ``tree_mean``).

Only ``tests/`` may import this module, and only as the checker.

Restates, op for op in float32:

* ``binary_stochastic_quantize``        fedjax/aggregators/compression.py:43-63
* ``uniform_stochastic_quantize``       compression.py:66-97
* ``uniform_stochastic_quantize_pytree`` compression.py:100-118 (per-leaf keys = split(rng, L))
* ``arithmetic_encoding_num_bits``      compression.py:125-149
* ``uniform_stochastic_quantizer``      compression.py:152-221
* ``rotated_uniform_stochastic_quantizer`` compression.py:224-266
* ``drive_pytree``                      compression.py:269-277
* ``structured_drive_quantizer``        compression.py:280-320
* ``terngrad_quantize(_pytree)``        compression.py:323-353
* ``terngrad_quantizer``                compression.py:356-400
* ``walsh_hadamard_transform``, ``structured_rotation``, ``inverse_structured_rotation``
  and the pytree forms                  fedjax/aggregators/walsh_hadamard.py:25-194

Where the reference's float results depend on XLA:CPU's evaluation order, this
restatement fixes one order and the product kernels follow the same one:

* Walsh-Hadamard: radix-2 butterflies ``(a + b, a - b)`` over bit 0, 1, …, m-1 in
  float32. The reference runs ``jnp.einsum`` against 2^7-point Hadamard blocks at
  ``precision='highest'``; the two agree to float32 reassociation error
  (the reference's own tests use rtol = atol = 1e-4, walsh_hadamard_test.py:44,57).
* Reductions (``jnp.std``, the DRIVE sums) are evaluated in float64 and rounded
  once to float32, which is at least as accurate as XLA's float32 reduction.
* ``v_min + q * (v_max - v_min)`` is a separate multiply and add (no FMA).
* ``jnp.log2`` (arithmetic-coding bit count) is ``log(x) / log(2)`` in float32 via
  numpy's ``logf``; XLA's own ``log`` may differ by an ulp.
Bitwise parity with XLA is therefore unpinned for these pieces; the end-to-end
pins are the reference's tests (tests/test_compression_oracle.py).
"""

from __future__ import annotations

import math
from typing import Any, Iterable, List, Tuple

import numpy as np

from oracle import jax_random_ref as jr
from oracle import tree_util_ref as tu

F32 = np.float32
_FMAX = np.finfo(np.float32).max


def nan_to_num(x):
    x = np.asarray(x, np.float32)
    return np.nan_to_num(x, nan=0.0, posinf=_FMAX, neginf=-_FMAX).astype(np.float32)


def xla_sign(x):
    """lax.sign: -1 / +1, and the argument itself for ±0 and NaN."""
    x = np.asarray(x, np.float32)
    return np.where(x > 0, F32(1), np.where(x < 0, F32(-1), x)).astype(np.float32)


def _minimum(a, b):
    return np.minimum(a, b).astype(np.float32)  # NaN-propagating, like lax.min


def _maximum(a, b):
    return np.maximum(a, b).astype(np.float32)


# ---------------------------------------------------------------------------
# quantizers (compression.py:43-97, 323-336)
# ---------------------------------------------------------------------------

def binary_stochastic_quantize(v, key, v_min=None, v_max=None, rand=None):
    v = np.asarray(v, np.float32)
    v_min = F32(np.min(v)) if v_min is None else F32(v_min)
    v_max = F32(np.max(v)) if v_max is None else F32(v_max)
    with np.errstate(all="ignore"):
        a = nan_to_num((v - v_min) / (v_max - v_min))
    a = _maximum(F32(0), _minimum(a, F32(1)))
    if rand is None:
        rand = jr.uniform(key, v.shape)
    return np.where(rand > a, v_min, v_max).astype(np.float32)


def uniform_stochastic_quantize(v, num_levels: int, key, v_min=None, v_max=None, rand=None):
    v = np.asarray(v, np.float32)
    v_min = F32(np.min(v)) if v_min is None else F32(v_min)
    v_max = F32(np.max(v)) if v_max is None else F32(v_max)
    lm1 = F32(num_levels - 1)
    with np.errstate(all="ignore"):
        a = nan_to_num((v - v_min) / (v_max - v_min))
        a = _maximum(F32(0), _minimum(a, F32(1)))
        v_ceil = (np.ceil(a * lm1) / lm1).astype(np.float32)
        v_floor = (np.floor(a * lm1) / lm1).astype(np.float32)
        if rand is None:
            rand = jr.uniform(key, v.shape)
        threshold = nan_to_num((a - v_floor) / (v_ceil - v_floor))
        q = np.where(rand > threshold, v_floor, v_ceil).astype(np.float32)
        return (v_min + (q * (v_max - v_min)).astype(np.float32)).astype(np.float32)


def std_f32(v) -> np.float32:
    v = np.asarray(v, np.float64).ravel()
    if v.size == 0:
        return F32(np.nan)
    s1, s2 = v.sum(), (v * v).sum()
    mean = s1 / v.size
    var = max(s2 / v.size - mean * mean, 0.0)
    return F32(math.sqrt(var)) if np.isfinite(var) else F32(np.nan)


def terngrad_quantize(v, key, rand=None):
    v = np.asarray(v, np.float32)
    sigma = std_f32(v)
    thr = F32(F32(2.5) * sigma)
    vc = np.where(np.abs(v) > thr, (thr * xla_sign(v)).astype(np.float32), v).astype(np.float32)
    av = np.abs(vc)
    vmax = F32(np.max(av))
    return (binary_stochastic_quantize(av, key, 0.0, vmax, rand=rand) * xla_sign(vc)).astype(np.float32)


def _map_leaves(fn, tree, key):
    leaves, td = tu.flatten(tree)
    keys = jr.split(key, len(leaves))
    return tu.unflatten(td, [fn(np.asarray(l, np.float32), k) for l, k in zip(leaves, keys)])


def uniform_stochastic_quantize_pytree(params, num_levels: int, key):
    return _map_leaves(lambda l, k: uniform_stochastic_quantize(l, num_levels, k), params, key)


def terngrad_quantize_pytree(params, key):
    return _map_leaves(terngrad_quantize, params, key)


# ---------------------------------------------------------------------------
# arithmetic-coding bit count (compression.py:125-149)
# ---------------------------------------------------------------------------

def _log2_f32(x):
    x = np.asarray(x, np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        return (np.log(x) / np.log(F32(2))).astype(np.float32)


def arithmetic_bits_from_counts(counts, d: int) -> np.float32:
    """Bits for a vector of d values whose distinct-value histogram is ``counts``."""
    hist = np.asarray(counts, np.int64)
    k = hist.size
    p = (hist.astype(np.float32) / F32(hist.sum())).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        ent = F32(-np.sum((p * _log2_f32(p)).astype(np.float32), dtype=np.float32))
        e = F32(np.exp(F32(1)))
        hist_bits = F32(F32(k) * _log2_f32(F32(F32(e * F32(d + k)) / F32(k))))
    return F32(F32(F32(hist_bits + F32(F32(d) * ent)) + F32(64)) + F32(2))


def arithmetic_encoding_num_bits(v) -> np.float32:
    v = nan_to_num(v).ravel()
    _, counts = np.unique(v, return_counts=True)
    return arithmetic_bits_from_counts(counts, v.size)


# ---------------------------------------------------------------------------
# Walsh-Hadamard (walsh_hadamard.py)
# ---------------------------------------------------------------------------

def fwht(x) -> np.ndarray:
    """Unnormalised Sylvester-order WHT, float32 butterflies over bits 0..m-1."""
    y = np.asarray(x, np.float32).ravel().copy()
    d = y.size
    assert d & (d - 1) == 0, d
    s = 1
    while s < d:
        v = y.reshape(-1, 2, s)
        a, b = v[:, 0, :].copy(), v[:, 1, :].copy()
        v[:, 0, :] = a + b
        v[:, 1, :] = a - b
        s *= 2
    return y


def padded_size(n: int) -> int:
    return 2 ** math.ceil(math.log2(n)) if n > 0 else 1


def structured_rotation(x, key):
    x = np.asarray(x, np.float32)
    flat = x.ravel()
    d = padded_size(flat.size)
    w = np.concatenate([flat, np.zeros(d - flat.size, np.float32)])
    rad = jr.rademacher(key, (d,)).astype(np.float32)
    return (fwht(w * rad) / np.sqrt(F32(d))).astype(np.float32), tuple(x.shape)


def inverse_structured_rotation(x, key, shape):
    x = np.asarray(x, np.float32)
    rad = jr.rademacher(key, x.shape).astype(np.float32)
    w = ((fwht(x) * rad) / np.sqrt(F32(x.size))).astype(np.float32)
    n = int(np.prod(shape)) if len(shape) else 1
    return w[:n].reshape(shape)


def structured_rotation_pytree(params, key):
    leaves, td = tu.flatten(params)
    keys = jr.split(key, len(leaves))
    out = [structured_rotation(l, k) for l, k in zip(leaves, keys)]
    return tu.unflatten(td, [o[0] for o in out]), [o[1] for o in out]


def inverse_structured_rotation_pytree(params, key, shapes):
    leaves, td = tu.flatten(params)
    keys = jr.split(key, len(leaves))
    return tu.unflatten(td, [inverse_structured_rotation(l, k, s) for l, k, s in zip(leaves, keys, shapes)])


def drive(leaf):
    y = np.asarray(leaf, np.float32)
    y64 = y.astype(np.float64)
    a = F32((y64 * y64).sum())
    b = F32(np.abs(y64).sum())
    with np.errstate(all="ignore"):
        return ((a * xla_sign(y)).astype(np.float32) / b).astype(np.float32)


def drive_pytree(params):
    leaves, td = tu.flatten(params)
    return tu.unflatten(td, [drive(l) for l in leaves])


# ---------------------------------------------------------------------------
# aggregators
# ---------------------------------------------------------------------------

class CompressionState:
    def __init__(self, num_bits, rng):
        self.num_bits, self.rng = num_bits, np.asarray(rng, np.uint32)


def _tree_size(tree) -> int:
    return sum(int(np.asarray(l).size) for l in tu.flatten(tree)[0])


def _num_leaves(tree) -> int:
    return len(tu.flatten(tree)[0])


def _bits_per_param(per_param_bits: float, agg) -> np.float32:
    """``per_param * tree_size(agg) + 32 * 2 * num_leaves`` with tree_size an int32."""
    return F32(F32(F32(per_param_bits) * F32(_tree_size(agg))) + F32(32 * 2 * _num_leaves(agg)))


def _accumulate_bits(state_bits, new_bits) -> np.float32:
    return F32(state_bits + new_bits)


def uniform_stochastic_quantizer(num_levels: int, rng, encode_algorithm=None):
    def init():
        return CompressionState(0.0, rng)

    def apply(clients, state):
        rng2, use_rng = jr.split(state.rng)
        seq = jr.PRNGSequence(use_rng)
        qs, total_bits = [], []
        for (_, params, w) in clients:
            q = uniform_stochastic_quantize_pytree(params, num_levels, next(seq))
            if encode_algorithm == "arithmetic":
                bits = 0
                for leaf in tu.flatten(q)[0]:
                    bits = bits + arithmetic_encoding_num_bits(leaf)
                total_bits.append(F32(bits))
            qs.append((q, w))
        agg = tu.tree_mean(qs)
        if encode_algorithm == "arithmetic":
            # compression.py:211: sum(total_bits) / len(total_bits) -- Python's sequential sum of
            # float32 scalars (np.sum would add pairwise and differ from K = 9 clients on)
            total = 0
            for b in total_bits:
                total = total + b
            new_bits = F32(F32(total) / F32(len(total_bits))) if total_bits else 0.0
        else:
            new_bits = _bits_per_param(math.log2(num_levels), agg)
        return agg, CompressionState(_accumulate_bits(state.num_bits, new_bits), rng2)

    return init, apply


def rotated_uniform_stochastic_quantizer(num_levels: int, rng, *, commute_inverse: bool = False):
    """``commute_inverse`` averages in the rotated domain and inverts once (the
    product's operation order); False is the reference order (invert per client)."""

    def init():
        return CompressionState(0.0, rng)

    def apply(clients, state):
        rng2, rot_rng = jr.split(state.rng)
        rng2, use_rng = jr.split(rng2)
        seq = jr.PRNGSequence(use_rng)
        qs, shapes = [], None
        for (_, params, w) in clients:
            rot, shapes = structured_rotation_pytree(params, rot_rng)
            q = uniform_stochastic_quantize_pytree(rot, num_levels, next(seq))
            qs.append((q if commute_inverse else inverse_structured_rotation_pytree(q, rot_rng, shapes), w))
        agg = tu.tree_mean(qs)
        if commute_inverse and agg is not None:
            agg = inverse_structured_rotation_pytree(agg, rot_rng, shapes)
        return agg, CompressionState(_accumulate_bits(state.num_bits, _bits_per_param(math.log2(num_levels), agg)),
                                     rng2)

    return init, apply


def structured_drive_quantizer(rng):
    def init():
        return CompressionState(0.0, rng)

    def apply(clients, state):
        rng2, rot_rng = jr.split(state.rng)
        seq = jr.PRNGSequence(rot_rng)
        qs = []
        for (_, params, w) in clients:
            crng = next(seq)
            rot, shapes = structured_rotation_pytree(params, crng)
            qs.append((inverse_structured_rotation_pytree(drive_pytree(rot), crng, shapes), w))
        agg = tu.tree_mean(qs)
        new_bits = F32(_tree_size(agg) + 32 * 2 * _num_leaves(agg))
        return agg, CompressionState(_accumulate_bits(state.num_bits, new_bits), rng2)

    return init, apply


def terngrad_quantizer(rng):
    def init():
        return CompressionState(0.0, rng)

    def apply(clients, state):
        rng2, use_rng = jr.split(state.rng)
        seq = jr.PRNGSequence(use_rng)
        qs = [(terngrad_quantize_pytree(params, next(seq)), w) for (_, params, w) in clients]
        agg = tu.tree_mean(qs)
        return agg, CompressionState(_accumulate_bits(state.num_bits, _bits_per_param(math.log2(3), agg)), rng2)

    return init, apply
