"""TEST INFRASTRUCTURE ONLY — numpy restatement of the JAX / Haiku PRNG that
FedJAX's compression aggregators draw from.

Only ``tests/`` may import this module, and only as the checker; the product's
key schedule is the C++ host code in ``fedjax_amd/csrc/fjcomp.hip`` and its
device bits come from the HIP kernels there.

The randomness in ``fedjax/aggregators/compression.py`` and
``fedjax/aggregators/walsh_hadamard.py`` comes from third-party code that is
absent here: ``jax.random`` (jax >= 0.4.x, unpinned by
``setup.py:38-47``; the tests run it with ``jax_threefry_partitionable`` off,
``compression_test.py:22``) and ``haiku.PRNGSequence`` (dm-haiku, unpinned). Their
published algorithms are restated:

* ``threefry2x32``   Threefry-2x32, 20 rounds (Salmon et al., SC'11; Random123),
                     with JAX's counter layout: the count array is padded to even
                     length and split into halves (x0 = first half, x1 = second)
* ``prng_key``       ``jax.random.PRNGKey(seed)`` = ``[seed >> 32, seed & 0xffffffff]``
* ``split``          ``threefry_2x32(key, iota(2 * num)).reshape(num, 2)``
* ``random_bits``    ``threefry_2x32(key, iota(n))`` (32-bit draws)
* ``uniform``        ``bitcast((bits >> 9) | 0x3f800000) - 1`` (f32, [0, 1))
* ``rademacher``     ``2 * (uniform < 0.5) - 1``
* ``PRNGSequence``   Haiku: ``next()`` reserves one key at a time,
                     ``key, sub = split(key, 2)``

Pinned by the Random123 known-answer vectors for threefry2x32_20 and the JAX
docs' ``split(PRNGKey(0))`` value (tests/test_compression_oracle.py), and
end-to-end by the reference's RNG-dependent compression tests
(``compression_test.py:185-205`` terngrad, ``:155-175`` DRIVE).
"""

from __future__ import annotations

import collections

import numpy as np

_U32 = np.uint32
_ROT = ((13, 15, 26, 6), (17, 29, 16, 24))


def _rotl(x, r):
    return (x << _U32(r)) | (x >> _U32(32 - r))


def threefry2x32(key, x0, x1):
    """Threefry-2x32-20 of counter pairs (x0[i], x1[i]) under key (k0, k1)."""
    k0, k1 = _U32(key[0]), _U32(key[1])
    ks = (k0, k1, k0 ^ k1 ^ _U32(0x1BD11BDA))
    x0 = np.asarray(x0, np.uint32).copy()
    x1 = np.asarray(x1, np.uint32).copy()
    with np.errstate(over="ignore"):
        x0 += ks[0]
        x1 += ks[1]
        for g in range(5):
            for r in _ROT[g % 2]:
                x0 += x1
                x1 = _rotl(x1, r)
                x1 ^= x0
            x0 += ks[(g + 1) % 3]
            x1 += ks[(g + 2) % 3] + _U32(g + 1)
    return x0, x1


def threefry_2x32_counts(key, count):
    """jax._src.prng.threefry_2x32 over a flat uint32 count array."""
    count = np.asarray(count, np.uint32).ravel()
    n = count.size
    if n % 2:
        count = np.concatenate([count, np.zeros(1, np.uint32)])
    h = count.size // 2
    y0, y1 = threefry2x32(key, count[:h], count[h:])
    return np.concatenate([y0, y1])[:n]


def prng_key(seed: int) -> np.ndarray:
    seed = int(seed)
    return np.array([(seed >> 32) & 0xFFFFFFFF, seed & 0xFFFFFFFF], np.uint32)


def split(key, num: int = 2) -> np.ndarray:
    return threefry_2x32_counts(key, np.arange(2 * num, dtype=np.uint32)).reshape(num, 2)


def random_bits(key, n: int) -> np.ndarray:
    return threefry_2x32_counts(key, np.arange(n, dtype=np.uint32))


def uniform(key, shape) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    bits = random_bits(key, n)
    f = ((bits >> _U32(9)) | _U32(0x3F800000)).view(np.float32) - np.float32(1.0)
    return np.maximum(np.float32(0.0), f).reshape(shape)


def rademacher(key, shape) -> np.ndarray:
    """int32 ±1 (jax.random.rademacher, default dtype int)."""
    return (2 * (uniform(key, shape) < np.float32(0.5)).astype(np.int32) - 1).astype(np.int32)


class PRNGSequence:
    """haiku.PRNGSequence over a key: ``next`` reserves one subkey at a time."""

    def __init__(self, key):
        self._key = np.asarray(key, np.uint32)
        self._subkeys = collections.deque()

    def reserve(self, num: int) -> None:
        if num > 0:
            keys = split(self._key, num + 1)
            self._key = keys[0]
            self._subkeys.extend(keys[1:])

    def __iter__(self):
        return self

    def __next__(self):
        if not self._subkeys:
            self.reserve(1)
        return self._subkeys.popleft()
