"""JAX-compatible PRNG keys and draws for the compression aggregators.

FedJAX's compression aggregators draw from ``jax.random`` (threefry2x32, with
``jax_threefry_partitionable`` off as in ``compression_test.py:22``) and iterate
client keys with ``haiku.PRNGSequence`` (``compression.py:195-197``). Keys here are
plain ``numpy.uint32[2]`` arrays with the same bits as a raw ``jax.random.PRNGKey``
(``np.asarray(jax_key)`` converts one), so a round seeded here draws exactly what the
reference would draw:

* key algebra (``PRNGKey``, ``split``, ``PRNGSequence``) runs on the host in the C++
  of ``libfjagg.so`` (``fjcomp_random_split`` / ``fjcomp_prng_sequence``): a few
  threefry blocks per client, sequential by nature;
* the per-element draws (``random_bits``, ``uniform``, ``rademacher``) are HIP
  kernels writing device tensors (``fjcomp_random_bits`` / ``fjcomp_uniform``).
"""

from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple, Union

import numpy as np
import torch

from fedjax_amd import _lib

Key = np.ndarray  # uint32[2]
Shape = Union[int, Sequence[int]]


def _key(key) -> np.ndarray:
    k = np.ascontiguousarray(np.asarray(key, dtype=np.uint32).reshape(-1))
    if k.shape != (2,):
        raise ValueError(f"a PRNG key is two uint32 words, got shape {np.shape(key)}")
    return k


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def PRNGKey(seed: int) -> np.ndarray:  # noqa: N802 (jax.random.PRNGKey)
    """``jax.random.PRNGKey(seed)``: ``[seed >> 32, seed & 0xffffffff]`` (uint32)."""
    seed = int(seed)
    return np.array([(seed >> 32) & 0xFFFFFFFF, seed & 0xFFFFFFFF], dtype=np.uint32)


def split(key, num: int = 2) -> np.ndarray:
    """``jax.random.split(key, num)`` -> uint32 [num, 2]."""
    return split_many(_key(key)[None], num)[0]


def split_many(keys, num: int) -> np.ndarray:
    """Split each of ``keys`` [n, 2] into ``num`` keys -> uint32 [n, num, 2]."""
    keys = np.ascontiguousarray(np.asarray(keys, dtype=np.uint32).reshape(-1, 2))
    out = np.empty((keys.shape[0], int(num), 2), dtype=np.uint32)
    _lib.call("fjcomp_random_split", _ptr(keys), keys.shape[0], int(num), _ptr(out))
    return out


class PRNGSequence:
    """``haiku.PRNGSequence`` over a key: each ``next`` reserves one subkey
    (``key, sub = split(key)``). ``take(n)`` draws n subkeys in one host call."""

    def __init__(self, key_or_seed):
        if isinstance(key_or_seed, (int, np.integer)):
            key_or_seed = PRNGKey(int(key_or_seed))
        self._key = _key(key_or_seed).copy()

    def __iter__(self):
        return self

    def __next__(self) -> np.ndarray:
        return self.take(1)[0]

    def take(self, n: int) -> np.ndarray:
        out = np.empty((int(n), 2), dtype=np.uint32)
        _lib.call("fjcomp_prng_sequence", _ptr(self._key), int(n), _ptr(out))
        return out

    @property
    def internal_state(self) -> np.ndarray:
        return self._key.copy()


def _size(shape: Shape) -> Tuple[Tuple[int, ...], int]:
    shape = (int(shape),) if isinstance(shape, (int, np.integer)) else tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    if n >= 1 << 32:
        raise ValueError("draws of 2^32 or more elements use a different counter layout in jax; not supported")
    return shape, n


def _device(device) -> torch.device:
    if device is None:
        if not torch.cuda.is_available():
            raise _lib.FjaggError("fedjax_amd draws on a ROCm GPU; torch.cuda.is_available() is False")
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


def random_bits(key, shape: Shape = (), device=None) -> torch.Tensor:
    """``jax.random.bits(key, shape, uint32)``, as an int32 tensor holding the bits."""
    k = _key(key)
    shape, n = _size(shape)
    dev = _device(device)
    out = torch.empty(shape, dtype=torch.int32, device=dev)
    _lib.call("fjcomp_random_bits", int(k[0]), int(k[1]), n, out.data_ptr(),
              torch.cuda.current_stream(dev).cuda_stream)
    return out


def uniform(key, shape: Shape = (), device=None) -> torch.Tensor:
    """``jax.random.uniform(key, shape)`` (float32 in [0, 1))."""
    k = _key(key)
    shape, n = _size(shape)
    dev = _device(device)
    out = torch.empty(shape, dtype=torch.float32, device=dev)
    _lib.call("fjcomp_uniform", int(k[0]), int(k[1]), n, out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    return out


def rademacher(key, shape: Shape = (), device=None) -> torch.Tensor:
    """``jax.random.rademacher(key, shape)``: int32 +-1 (+1 where uniform < 0.5)."""
    u = uniform(key, shape, device)
    return torch.where(u < 0.5, 1, -1).to(torch.int32)


__all__ = ["PRNGKey", "PRNGSequence", "rademacher", "random_bits", "split", "split_many", "uniform"]
