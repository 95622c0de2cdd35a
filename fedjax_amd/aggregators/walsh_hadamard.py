"""Walsh-Hadamard transform and structured rotations on the GPU
(``fedjax/aggregators/walsh_hadamard.py``).

``walsh_hadamard_transform`` is the LDS-tiled radix-2 transform of
``fjcomp_wht`` (13 butterfly bits per pass, bit order 0, 1, ..., m-1); the reference
runs ``jnp.einsum`` against 2^7-point Hadamard blocks. Both compute the Sylvester-
order transform; they differ only by float32 reassociation (the reference's tests
allow rtol = atol = 1e-4, walsh_hadamard_test.py:44). ``small_n`` and ``precision``
tune the reference's einsum and are accepted for API compatibility.

The rotations fuse the zero padding, the Rademacher signs (``jax.random.rademacher``
bits, bit-packed once per key) and the ``/ sqrt(d)`` into the transform's first and
last passes.
"""

from __future__ import annotations

from typing import Any, Sequence, Tuple

import numpy as np
import scipy.linalg
import torch

from fedjax_amd import _compress as C
from fedjax_amd import _lib, pytree, random, tree_util

PyTree = Any


def _vector(x) -> torch.Tensor:
    t = tree_util._device_leaf(x, tree_util._find_device([x]))
    if t.dtype != torch.float32:
        if t.dtype == torch.bfloat16:
            raise TypeError("bfloat16 leaves are not supported by the compression kernels (float32 only)")
        t = t.to(torch.float32)
    return t


def walsh_hadamard_transform(x, small_n: int = 2 ** 7, precision: Any = "highest") -> torch.Tensor:
    """Unnormalised Walsh-Hadamard transform of a vector whose length is a power of 2
    (walsh_hadamard.py:25-98)."""
    if small_n <= 1:
        raise ValueError(f"small_n must be > 1, got {small_n}")
    t = _vector(x)
    if t.dim() != 1:
        raise ValueError("walsh_hadamard_transform takes a vector")
    d = t.numel()
    out = torch.empty_like(t)
    job = C.wht_job(t.data_ptr(), out.data_ptr(), out.data_ptr(), d, kind=_lib.WHT_PLAIN)
    C.run_wht(job, t.device)
    return out


def hadamard_matrix(n: int, dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """The n x n Sylvester Hadamard matrix (walsh_hadamard.py:101-114), on the host."""
    return torch.from_numpy(scipy.linalg.hadamard(n)).to(dtype)


def _shape_of(shape) -> Tuple[int, ...]:
    if isinstance(shape, torch.Tensor):
        shape = shape.tolist()
    return tuple(int(s) for s in np.asarray(shape).reshape(-1))


def _rotate(leaves: Sequence[torch.Tensor], keys: np.ndarray) -> list:
    dev = leaves[0].device
    ns = [x.numel() for x in leaves]
    ds = [C.padded_size(n) for n in ns]
    signs, woff = C.rademacher_words(keys, ds, dev)
    outs = [torch.empty(d, dtype=torch.float32, device=dev) for d in ds]
    jobs = np.concatenate([
        C.wht_job(x.data_ptr(), o.data_ptr(), o.data_ptr(), d, kind=_lib.WHT_ROTATE, n_in=n,
                  signs=signs.data_ptr() + 4 * int(woff[i]))
        for i, (x, o, n, d) in enumerate(zip(leaves, outs, ns, ds))])
    C.run_wht(jobs, dev)
    return outs


def _unrotate(rotated: Sequence[torch.Tensor], keys: np.ndarray, shapes: Sequence[Tuple[int, ...]]) -> list:
    dev = rotated[0].device
    ds = [x.numel() for x in rotated]
    signs, woff = C.rademacher_words(keys, ds, dev)
    outs, jobs = [], []
    for i, (x, d, shp) in enumerate(zip(rotated, ds, shapes)):
        n = int(np.prod(shp)) if len(shp) else 1
        if n > d:
            raise ValueError(f"original shape {shp} is larger than the rotated vector ({d})")
        o = torch.empty(shp, dtype=torch.float32, device=dev)
        mid = torch.empty(d, dtype=torch.float32, device=dev) if C.wht_passes(C.log2_exact(d)) > 1 else o
        jobs.append(C.wht_job(x.data_ptr(), mid.data_ptr(), o.data_ptr(), d, kind=_lib.WHT_UNROTATE, n_out=n,
                              signs=signs.data_ptr() + 4 * int(woff[i])))
        outs.append((o, mid))
    C.run_wht(np.concatenate(jobs), dev)
    return [o for o, _ in outs]


def structured_rotation(x, rng) -> Tuple[torch.Tensor, torch.Tensor]:
    """``H D pad(x) / sqrt(d)`` and the original shape (walsh_hadamard.py:127-148)."""
    t = _vector(x)
    return _rotate([t.reshape(-1)], np.asarray(rng, np.uint32).reshape(1, 2))[0], \
        torch.tensor(tuple(t.shape), dtype=torch.int32)


def inverse_structured_rotation(x, rng, original_shape) -> torch.Tensor:
    """``(H x * D) / sqrt(d)`` truncated to ``original_shape`` (walsh_hadamard.py:151-176)."""
    t = _vector(x)
    return _unrotate([t.reshape(-1)], np.asarray(rng, np.uint32).reshape(1, 2), [_shape_of(original_shape)])[0]


def structured_rotation_pytree(params: PyTree, rng) -> Tuple[PyTree, PyTree]:
    """Rotates every leaf with keys ``split(rng, num_leaves)`` (walsh_hadamard.py:179-203)."""
    leaves, td = pytree.flatten(params)
    if not leaves:
        return params, params
    ts = [_vector(x) for x in leaves]
    keys = random.split(rng, len(ts))
    rot = _rotate([t.reshape(-1) for t in ts], keys)
    shapes = [torch.tensor(tuple(t.shape), dtype=torch.int32) for t in ts]
    return pytree.unflatten(td, rot), pytree.unflatten(td, shapes)


def inverse_structured_rotation_pytree(params: PyTree, rng, shapes: PyTree) -> PyTree:
    """Inverse of :func:`structured_rotation_pytree` (walsh_hadamard.py:206-226)."""
    leaves, td = pytree.flatten(params)
    if not leaves:
        return params
    shape_leaves = pytree.flatten_as(td, shapes)
    keys = random.split(rng, len(leaves))
    return pytree.unflatten(td, _unrotate([_vector(x).reshape(-1) for x in leaves], keys,
                                          [_shape_of(s) for s in shape_leaves]))


__all__ = ["hadamard_matrix", "inverse_structured_rotation", "inverse_structured_rotation_pytree",
           "structured_rotation", "structured_rotation_pytree", "walsh_hadamard_transform"]
