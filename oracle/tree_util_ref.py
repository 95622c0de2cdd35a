"""TEST INFRASTRUCTURE ONLY — numpy restatement of FedJAX's aggregation semantics.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker. The product package
``fedjax_amd`` never imports it (tests/test_boundary.py asserts that).

Restates google/fedjax 0.0.17 ``fedjax/core/tree_util.py`` op for op:

* ``tree_weight``            tree_util.py:29-32   ``l * weight`` under ``jax.jit``
* ``tree_inverse_weight``    tree_util.py:35-38   ``1/W if W > 0 else 0`` on the host
* ``tree_zeros_like``        tree_util.py:41-44
* ``tree_add``               tree_util.py:47-50   ``jnp.add`` leafwise
* ``tree_sum``               tree_util.py:64-73   copy of tree 0, then donated adds
* ``tree_mean``              tree_util.py:76-96   weighted fold, W summed in Python
* ``tree_size``              tree_util.py:99-102
* ``tree_l2_squared/norm``   tree_util.py:105-114
* ``tree_clip_by_global_norm`` tree_util.py:117-133
* ``mean_aggregator``        fedjax/aggregators/aggregator.py:61-75

and the JAX dtype rules those lines run under (x64 disabled, the jax default):
Python ints/floats are *weakly typed* (they take the leaf's dtype), int64/float64
arrays canonicalise to int32/float32, int32 * weak float promotes to float32.
numpy >= 2 (NEP 50) gives Python scalars the same weak behaviour, which is what
makes ``sum_weight = 0.; sum_weight += w`` below follow the reference for both
Python-number and float32-array weights.

JAX itself is not installed here, so parity is pinned by the
reference's own known-answer tests (tests/test_oracle.py) and, for large shapes,
by the bit-level spec these functions restate.
"""

from __future__ import annotations

import collections
import numbers
from typing import Any, Iterable, List, Tuple

import numpy as np

# ----------------------------------------------------------------------------
# Minimal pytree flatten (jax.tree_util order: dict keys sorted, sequences and
# namedtuples positional, None is an empty subtree).
# ----------------------------------------------------------------------------


def _is_namedtuple(x):
    return isinstance(x, tuple) and hasattr(x, "_fields")


def flatten(tree) -> Tuple[List[Any], Any]:
    if tree is None:
        return [], ("none",)
    if isinstance(tree, dict):
        keys = sorted(tree)
        leaves, defs = [], []
        for k in keys:
            l, d = flatten(tree[k])
            leaves += l
            defs.append(d)
        return leaves, ("dict", tuple(keys), tuple(defs))
    if _is_namedtuple(tree):
        leaves, defs = [], []
        for v in tree:
            l, d = flatten(v)
            leaves += l
            defs.append(d)
        return leaves, ("namedtuple", type(tree), tuple(defs))
    if isinstance(tree, (list, tuple)):
        leaves, defs = [], []
        for v in tree:
            l, d = flatten(v)
            leaves += l
            defs.append(d)
        return leaves, (type(tree).__name__, tuple(defs))
    return [tree], ("leaf",)


def unflatten(treedef, leaves):
    it = iter(leaves)

    def build(d):
        kind = d[0]
        if kind == "none":
            return None
        if kind == "leaf":
            return next(it)
        if kind == "dict":
            return {k: build(sd) for k, sd in zip(d[1], d[2])}
        if kind == "namedtuple":
            return d[1](*[build(sd) for sd in d[2]])
        vals = [build(sd) for sd in d[1]]
        return vals if kind == "list" else tuple(vals)

    return build(treedef)


def tree_map(fn, *trees):
    leaves0, td = flatten(trees[0])
    others = []
    for t in trees[1:]:
        l, d = flatten(t)
        if d != td:
            raise ValueError("pytree structure mismatch")
        others.append(l)
    return unflatten(td, [fn(*xs) for xs in zip(leaves0, *others)])


# ----------------------------------------------------------------------------
# JAX dtype semantics (x64 disabled)
# ----------------------------------------------------------------------------


def canonical_leaf(x) -> np.ndarray:
    """jnp.asarray(x) with x64 disabled: int64->int32, float64->float32."""
    a = np.asarray(x)
    if a.dtype == np.bool_:
        return a
    if np.issubdtype(a.dtype, np.integer):
        return a.astype(np.int32)
    if np.issubdtype(a.dtype, np.floating):
        return a.astype(np.float32) if a.dtype != np.float16 else a
    return a


def _is_weak(w) -> bool:
    return isinstance(w, (bool, numbers.Integral, numbers.Real)) and not isinstance(w, np.generic)


def _mul_weak(leaf: np.ndarray, w) -> np.ndarray:
    """``l * weight`` as traced by jax.jit (tree_util.py:32)."""
    leaf = canonical_leaf(leaf)
    if _is_weak(w):
        if isinstance(w, numbers.Integral) and np.issubdtype(leaf.dtype, np.integer):
            return leaf * np.int32(w)  # int32 * weak int -> int32 (wraps)
        if np.issubdtype(leaf.dtype, np.integer):
            return leaf.astype(np.float32) * np.float32(w)  # int * weak float -> f32
        return leaf * leaf.dtype.type(w)  # float leaf: weight takes the leaf dtype
    wa = canonical_leaf(w)  # strongly typed scalar/array weight
    dt = jax_promote(leaf.dtype, wa.dtype)
    return np.multiply(leaf.astype(dt), wa.astype(dt))


def jax_promote(a: np.dtype, b: np.dtype) -> np.dtype:
    """jnp.promote_types for the int32/float32/float16 subset (x64 disabled):
    int op float -> the float type; float op float -> the wider; int op int -> int32."""
    a, b = np.dtype(a), np.dtype(b)
    af, bf = np.issubdtype(a, np.floating), np.issubdtype(b, np.floating)
    if af and bf:
        return a if a.itemsize >= b.itemsize else b
    if af:
        return a
    if bf:
        return b
    return np.dtype(np.int32)


def tree_weight(pytree, weight):
    """tree_util.py:29-32."""
    return tree_map(lambda l: _mul_weak(l, weight), pytree)


def tree_inverse_weight(pytree, weight):
    """tree_util.py:35-38 (and the donated form :58-61)."""
    inverse_weight = (1.0 / weight) if weight > 0.0 else 0.0
    return tree_weight(pytree, inverse_weight)


def tree_zeros_like(pytree):
    """tree_util.py:41-44."""
    return tree_map(lambda l: np.zeros_like(canonical_leaf(l)), pytree)


def tree_add(left, right):
    """tree_util.py:47-50 (jnp.add, dtype promotion of the two leaves)."""
    def add(a, b):
        a, b = canonical_leaf(a), canonical_leaf(b)
        dt = jax_promote(a.dtype, b.dtype)
        return np.add(a.astype(dt), b.astype(dt))

    return tree_map(add, left, right)


def tree_sum(pytrees: Iterable):
    """tree_util.py:64-73: copy of the first tree, then in-place adds."""
    s = None
    for t in pytrees:
        s = tree_map(lambda l: canonical_leaf(l).copy(), t) if s is None else tree_add(s, t)
    return s


def tree_mean(pytrees_and_weights: Iterable[Tuple[Any, Any]]):
    """tree_util.py:76-96, op for op."""
    sum_weighted_pytree = None
    sum_weight = 0.0
    for pytree, weight in pytrees_and_weights:
        weighted_pytree = tree_weight(pytree, weight)
        if sum_weighted_pytree is None:
            sum_weighted_pytree = weighted_pytree
        else:
            sum_weighted_pytree = tree_add(sum_weighted_pytree, weighted_pytree)
        sum_weight += weight
    if sum_weighted_pytree is None:
        return None
    return tree_inverse_weight(sum_weighted_pytree, sum_weight)


def tree_size(pytree) -> int:
    """tree_util.py:99-102."""
    return int(sum(np.asarray(l).size for l in flatten(pytree)[0]))


def tree_l2_squared(pytree) -> np.float32:
    """tree_util.py:105-108 (sum of per-leaf vdot; f32). XLA's reduction order is
    unspecified, so this is a float64 sum rounded to f32 — a tolerance oracle."""
    tot = 0.0
    for l in flatten(pytree)[0]:
        a = canonical_leaf(l).astype(np.float64).ravel()
        tot += float(np.dot(a, a))
    return np.float32(tot)


def tree_l2_norm(pytree) -> np.float32:
    """tree_util.py:111-114."""
    return np.float32(np.sqrt(np.float32(tree_l2_squared(pytree))))


def tree_clip_by_global_norm(pytree, max_norm):
    """tree_util.py:117-133 under jax.jit: max_norm is a weakly typed f32 argument,
    ``scale = min(1, max_norm / norm)`` in float32, then ``scale * t`` per leaf."""
    norm = tree_l2_norm(pytree)
    with np.errstate(divide="ignore", invalid="ignore"):
        scale = np.minimum(np.float32(1), np.float32(max_norm) / norm)
    return tree_map(lambda l: (np.float32(scale) * canonical_leaf(l)).astype(np.float32), pytree)


# ----------------------------------------------------------------------------
# Aggregator (fedjax/aggregators/aggregator.py:26-75)
# ----------------------------------------------------------------------------

Aggregator = collections.namedtuple("Aggregator", ["init", "apply"])


def mean_aggregator():
    def init():
        return ()

    def apply(clients_params_and_weights, state):
        return tree_mean((p, w) for _, p, w in clients_params_and_weights), state

    return Aggregator(init, apply)


# ----------------------------------------------------------------------------
# Synthetic inputs, identical to fjagg_fill_synth / oracle_fill_synth_*.
# ----------------------------------------------------------------------------

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth(K: int, P: int, seed: int = 0, amp: float = 0.01, k0: int = 0) -> np.ndarray:
    """x[k, p] = amp * u(seed, k0+k, p) as float32 [K, P]."""
    k = (np.arange(k0, k0 + K, dtype=np.uint64) << np.uint64(32))[:, None]
    p = np.arange(P, dtype=np.uint64)[None, :] & np.uint64(0xFFFFFFFF)
    h = _mix64(np.uint64(seed) ^ _mix64(k | p))
    u = (h >> np.uint64(40)).astype(np.uint32).astype(np.float32) * np.float32(1.0 / 8388608.0) - np.float32(1.0)
    return np.float32(amp) * u


def fedavg_weights(K: int, seed: int = 1) -> np.ndarray:
    """Integer client weights in [1, 500] (len(client_dataset), examples/fed_avg.py:76)."""
    return np.random.RandomState(seed).randint(1, 501, size=K).astype(np.int64)


def wsum_dense(x: np.ndarray, w, scale=None, init=None) -> np.ndarray:
    """Dense [K, P] float32 restatement of the fold (same bits as tree_mean)."""
    w32 = np.asarray(w, dtype=np.float32)
    s = x[0] * w32[0]
    if init is not None:
        s = init + s
    for k in range(1, x.shape[0]):
        s = s + x[k] * w32[k]
    return s if scale is None else s * np.float32(scale)


def mean_scale(weights) -> np.float32:
    """f32(1/W), W summed as the reference does (Python float for Python numbers)."""
    W = 0.0
    for w in weights:
        W += w
    return np.float32((1.0 / W) if W > 0.0 else 0.0)
