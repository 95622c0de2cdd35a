"""Compression aggregators on the GPU (``fedjax/aggregators/compression.py``).

Same names, arguments, state and randomness as the reference: a round seeded with
``fedjax_amd.random.PRNGKey(s)`` (bit-identical to ``jax.random.PRNGKey(s)``) draws
exactly the reference's jax.random stream, client keys come from a
haiku.PRNGSequence-equivalent, per-leaf keys from ``split(client_key, num_leaves)``.

Where the reference runs, per client and per leaf, a jitted quantizer and then
tree_mean's fold, a round here is a few kernel launches over every client and leaf
at once (fedjax_amd/_compress.py, include/fjcomp.h):

* uniform / terngrad: one statistics pass, then ONE kernel that draws the uniform
  bits, quantizes and folds the clients in order (the quantized deltas never reach
  HBM); the fold is tree_mean's (``fl(q * w_k)`` summed in client order, then
  ``* f32(1/W)``), bitwise;
* rotated uniform: the rotation key is shared by all clients (compression.py:241),
  so the mean is taken in the rotated domain and inverted once;
* DRIVE: per-client rotation, per-client scale, inverse rotation, dense fold.

``num_bits`` follows the reference's float32 arithmetic (``tree_size`` is an int32
there), so ``num_bits`` compares equal to the reference's values.

Leaves must be float32 (int32 leaves are converted exactly below 2^24; bfloat16
raises TypeError). Numerics: DESIGN.md §4.
"""

from __future__ import annotations

import itertools
import math
from typing import Any, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from fedjax_amd import _compress as C
from fedjax_amd import _lib, dataclasses, pytree, random, tree_util
from fedjax_amd.aggregators import aggregator

PyTree = Any
F32 = np.float32


@dataclasses.dataclass
class CompressionState:
    """compression.py:32-40: bits transmitted so far and the aggregator's key."""
    num_bits: Any
    rng: Any


# ----------------------------------------------------------------------------- helpers
def _f32_leaf(x, device) -> torch.Tensor:
    t = tree_util._device_leaf(x, device)
    if t.dtype == torch.float32:
        return t
    if t.dtype == torch.bfloat16:
        raise TypeError("bfloat16 leaves are not supported by the compression kernels (float32 only)")
    return t.to(torch.float32)


def _rows(trees: Sequence[PyTree]):
    """Client leaves as float32 device tensors; _client_rows has already checked every
    client against client 0's structure, shapes and dtypes (the kernels size every row
    from client 0), so only client 0's dtypes need looking at."""
    td, rows = tree_util._client_table(trees)
    if rows[0] and not all(x.dtype == torch.float32 for x in rows[0]):
        td, rows = tree_util._client_rows(trees)
        device = rows[0][0].device
        rows = [[_f32_leaf(x, device) for x in r] for r in rows]
    return td, rows


def _weights(weights: Sequence[Any]) -> Tuple[np.ndarray, Optional[float]]:
    """f32(w_k) and tree_mean's f32(1/W) (tree_util.py:85-96)."""
    sum_weight = 0.0
    hw = []
    for w in weights:
        w = tree_util._host_weight(w)
        tree_util._weight_kind(w)
        hw.append(w)
        sum_weight += w
    return np.array([np.float32(w) for w in hw], dtype=np.float32), float(np.float32(tree_util._inverse(sum_weight)))


def _single(v, method: int, rng, *, num_levels: int = 2, v_min=None, v_max=None) -> torch.Tensor:
    """One leaf quantized with one key (K = 1, weight 1, no scale: q * 1 is exact)."""
    device = tree_util._find_device([v])
    t = _f32_leaf(v, device)
    out = torch.empty(t.shape, dtype=torch.float32, device=device)
    if t.numel() == 0:
        raise ValueError("cannot quantize an empty array (the reference fails on amin of an empty array)")
    keys = np.asarray(rng, np.uint32).reshape(1, 1, 2)
    qp = None
    if v_min is not None or v_max is not None:
        if v_min is None or v_max is None:
            stats, _ = C.row_stats([(t.data_ptr(), t.numel())], method, device, want_qparams=False)
            s = np.frombuffer(stats.cpu().numpy().tobytes(), dtype=C.STATS)[0]
            v_min = s["min"] if v_min is None else v_min
            v_max = s["max"] if v_max is None else v_max
        host = C.qparams_host(v_min, v_max)
        qp = torch.from_numpy(host.view(np.uint8).copy()).to(device)
    C.quantized_mean(method, [[t]], keys, np.ones(1, np.float32), None, [out], num_levels=num_levels, qparams=qp)
    return out


# ----------------------------------------------------------------------------- quantizers
def binary_stochastic_quantize(v, rng, v_min: Optional[float] = None, v_max: Optional[float] = None) -> torch.Tensor:
    """compression.py:43-63."""
    return _single(v, _lib.COMP_BINARY, rng, v_min=v_min, v_max=v_max)


def uniform_stochastic_quantize(v, num_levels: int, rng, v_min: Optional[float] = None,
                                v_max: Optional[float] = None) -> torch.Tensor:
    """compression.py:66-97."""
    return _single(v, _lib.COMP_UNIFORM, rng, num_levels=int(num_levels), v_min=v_min, v_max=v_max)


def terngrad_quantize(v, rng) -> torch.Tensor:
    """compression.py:323-336."""
    return _single(v, _lib.COMP_TERNGRAD, rng)


def _quantize_pytree(params: PyTree, rng, method: int, num_levels: int = 2) -> PyTree:
    td, rows = _rows([params])
    if not rows[0]:
        return params
    L = len(rows[0])
    keys = random.split(rng, L).reshape(1, L, 2)
    outs = [torch.empty(x.shape, dtype=torch.float32, device=x.device) for x in rows[0]]
    C.quantized_mean(method, rows, keys, np.ones(1, np.float32), None, outs, num_levels=num_levels)
    return pytree.unflatten(td, outs)


def uniform_stochastic_quantize_pytree(params: PyTree, num_levels: int, rng) -> PyTree:
    """compression.py:100-118 (leaf keys = split(rng, num_leaves))."""
    return _quantize_pytree(params, rng, _lib.COMP_UNIFORM, int(num_levels))


def terngrad_quantize_pytree(params: PyTree, rng) -> PyTree:
    """compression.py:339-353."""
    return _quantize_pytree(params, rng, _lib.COMP_TERNGRAD)


def num_leaves(pytree_: PyTree) -> int:
    """compression.py:121-122."""
    return len(pytree.leaves_of(pytree_))


def arithmetic_encoding_num_bits(v) -> np.float32:
    """compression.py:143-149: bits to store v with arithmetic coding."""
    device = tree_util._find_device([v])
    t = _f32_leaf(v, device).reshape(-1)
    t = torch.nan_to_num(t, nan=0.0, posinf=float(np.finfo(np.float32).max), neginf=-float(np.finfo(np.float32).max))
    _, counts = torch.unique(t, sorted=True, return_counts=True)
    return C.arithmetic_bits_from_counts(counts.cpu().numpy(), t.numel())


def drive_pytree(params: PyTree) -> PyTree:
    """compression.py:269-277: every leaf becomes sum(y^2) * sign(y) / sum(|y|)."""
    leaves, td = pytree.flatten(params)
    if not leaves:
        return params
    device = tree_util._find_device(leaves)
    ts = [_f32_leaf(x, device) for x in leaves]
    stats, _ = C.row_stats([(t.data_ptr(), t.numel()) for t in ts], 0, device, want_qparams=False)
    s = np.frombuffer(stats.cpu().numpy().tobytes(), dtype=C.STATS)
    out = []
    for t, st in zip(ts, s):
        a, b = float(np.float32(st["sumsq"])), float(np.float32(st["sumabs"]))
        sign = torch.where(t > 0, 1.0, torch.where(t < 0, -1.0, t))
        out.append((a * sign) / b)
    return pytree.unflatten(td, out)


# ----------------------------------------------------------------------------- bits
def _bits_per_param(per_param: float, P: int, L: int) -> np.float32:
    """``per_param * tree_size + 32 * 2 * num_leaves`` with tree_size an int32 array."""
    return F32(F32(F32(per_param) * F32(P)) + F32(32 * 2 * L))


def _consume(clients: Iterable) -> Tuple[list, list]:
    trees, weights = [], []
    for _, params, weight in clients:  # client ids are ignored (aggregator.py:69)
        trees.append(params)
        weights.append(weight)
    return trees, weights


def _mean_round(trees, weights, client_keys, method, num_levels=2, hist=False):
    """tree_mean over the quantized client deltas, one fused launch."""
    td, rows = _rows(trees)
    if not rows[0]:
        return pytree.unflatten(td, []), td, rows, None
    K, L = len(rows), len(rows[0])
    leaf_keys = random.split_many(client_keys, L)
    w, scale = _weights(weights)
    outs = [torch.empty(x.shape, dtype=torch.float32, device=x.device) for x in rows[0]]
    h, qp = C.quantized_mean(method, rows, leaf_keys, w, scale, outs, num_levels=num_levels, hist=hist)
    bits = C.arithmetic_bits(h, qp, K, [x.numel() for x in rows[0]], num_levels) if hist else None
    return pytree.unflatten(td, outs), td, rows, bits


# ----------------------------------------------------------------------------- aggregators
def uniform_stochastic_quantizer(num_levels: int, rng, encode_algorithm: Optional[str] = None) -> aggregator.Aggregator:
    """compression.py:152-221."""

    def init():
        return CompressionState(0.0, np.asarray(rng, np.uint32))

    def apply(clients_params_and_weights, aggregator_state):
        if encode_algorithm is not None:
            assert encode_algorithm == "arithmetic"
        new_rng, use_rng = random.split(aggregator_state.rng)
        trees, weights = _consume(clients_params_and_weights)
        client_keys = random.PRNGSequence(use_rng).take(len(trees))
        arith = encode_algorithm == "arithmetic"
        if not trees:
            agg, P, L, bits = None, 0, 0, []
        else:
            agg, _, rows, bits = _mean_round(trees, weights, client_keys, _lib.COMP_UNIFORM, int(num_levels), arith)
            P, L = sum(x.numel() for x in rows[0]), len(rows[0])
        if arith:
            new_bits = F32(F32(sum(bits)) / F32(len(bits))) if bits else 0.0
        else:
            new_bits = _bits_per_param(math.log2(num_levels), P, L)
        return agg, CompressionState(F32(aggregator_state.num_bits + new_bits), new_rng)

    return aggregator.Aggregator(init, apply)


def rotated_uniform_stochastic_quantizer(num_levels: int, rng, *,
                                         workspace_bytes: int = C.DEFAULT_WORKSPACE_BYTES) -> aggregator.Aggregator:
    """compression.py:224-266. ``workspace_bytes`` bounds the rotated-delta batch
    kept in HBM (a build-side knob; the reference holds one client at a time)."""

    def init():
        return CompressionState(0.0, np.asarray(rng, np.uint32))

    def apply(clients_params_and_weights, aggregator_state):
        new_rng, rotation_rng = random.split(aggregator_state.rng)
        new_rng, use_rng = random.split(new_rng)
        trees, weights = _consume(clients_params_and_weights)
        client_keys = random.PRNGSequence(use_rng).take(len(trees))
        agg, P, L = None, 0, 0
        if trees:
            td, rows = _rows(trees)
            L = len(rows[0])
            if L:
                P = sum(x.numel() for x in rows[0])
                w, scale = _weights(weights)
                outs = [torch.empty(x.shape, dtype=torch.float32, device=x.device) for x in rows[0]]
                C.rotated_quantized_mean(rows, random.split(rotation_rng, L), random.split_many(client_keys, L),
                                         w, scale, outs, num_levels=int(num_levels), workspace_bytes=workspace_bytes)
                agg = pytree.unflatten(td, outs)
            else:
                agg = pytree.unflatten(td, [])
        new_bits = _bits_per_param(math.log2(num_levels), P, L)
        return agg, CompressionState(F32(aggregator_state.num_bits + new_bits), new_rng)

    return aggregator.Aggregator(init, apply)


def structured_drive_quantizer(rng, *, workspace_bytes: int = C.DEFAULT_WORKSPACE_BYTES) -> aggregator.Aggregator:
    """compression.py:280-320."""

    def init():
        return CompressionState(0.0, np.asarray(rng, np.uint32))

    def apply(clients_params_and_weights, aggregator_state):
        new_rng, rotation_rng = random.split(aggregator_state.rng)
        trees, weights = _consume(clients_params_and_weights)
        client_keys = random.PRNGSequence(rotation_rng).take(len(trees))
        agg, P, L = None, 0, 0
        if trees:
            td, rows = _rows(trees)
            L = len(rows[0])
            if L:
                P = sum(x.numel() for x in rows[0])
                w, scale = _weights(weights)
                flat = torch.empty(P, dtype=torch.float32, device=rows[0][0].device)
                C.drive_mean(rows, random.split_many(client_keys, L), w, scale, flat,
                             workspace_bytes=workspace_bytes)
                outs, o = [], 0
                for x in rows[0]:
                    outs.append(flat[o:o + x.numel()].view(x.shape))
                    o += x.numel()
                agg = pytree.unflatten(td, outs)
            else:
                agg = pytree.unflatten(td, [])
        new_bits = F32(P + 32 * 2 * L)  # int32 tree_size + int, then float32 accumulation
        return agg, CompressionState(F32(aggregator_state.num_bits + new_bits), new_rng)

    return aggregator.Aggregator(init, apply)


def terngrad_quantizer(rng) -> aggregator.Aggregator:
    """compression.py:356-400."""

    def init():
        return CompressionState(0.0, np.asarray(rng, np.uint32))

    def apply(clients_params_and_weights, aggregator_state):
        new_rng, use_rng = random.split(aggregator_state.rng)
        trees, weights = _consume(clients_params_and_weights)
        client_keys = random.PRNGSequence(use_rng).take(len(trees))
        agg, P, L = None, 0, 0
        if trees:
            agg, _, rows, _ = _mean_round(trees, weights, client_keys, _lib.COMP_TERNGRAD)
            P, L = sum(x.numel() for x in rows[0]), len(rows[0])
        new_bits = _bits_per_param(math.log2(3), P, L)
        return agg, CompressionState(F32(aggregator_state.num_bits + new_bits), new_rng)

    return aggregator.Aggregator(init, apply)


__all__ = ["CompressionState", "arithmetic_encoding_num_bits", "binary_stochastic_quantize", "drive_pytree",
           "num_leaves", "rotated_uniform_stochastic_quantizer", "structured_drive_quantizer", "terngrad_quantize",
           "terngrad_quantize_pytree", "terngrad_quantizer", "uniform_stochastic_quantize",
           "uniform_stochastic_quantize_pytree", "uniform_stochastic_quantizer"]
