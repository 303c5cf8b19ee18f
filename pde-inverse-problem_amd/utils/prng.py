"""Explicit PRNG keys with jax.random's calling conventions (host side).

The reference threads `jax.random` keys through every call (main.py:43-44, trainer.py:80-83,
consistency.py:36-39). JAX is absent, and its threefry bit-stream is not reproducible here
(SURVEY.md §0.1), so keys are (seed, counter) pairs over Philox4x32-10 — the same generator the
device kernels use. `split` derives child seeds on the host by one Philox block each; the
device streams then use the child seed as the Philox key (include/pdeinv.h).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import numpy as np

_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = (int(x) & _MASK for x in ctr)
    k0, k1 = (int(x) & _MASK for x in key)
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & _MASK, p1 & _MASK, ((p0 >> 32) ^ c3 ^ k1) & _MASK, p0 & _MASK
        k0 = (k0 + _W0) & _MASK
        k1 = (k1 + _W1) & _MASK
    return c0, c1, c2, c3


@dataclass(frozen=True)
class Key:
    seed: int

    def __int__(self):
        return self.seed


def PRNGKey(seed: int) -> Key:  # noqa: N802 - jax.random name
    s = int(seed) & 0xFFFFFFFFFFFFFFFF
    o = philox4x32_10((0, 0, 0, 0xA0000000), (s & _MASK, s >> 32))
    return Key(o[0] | (o[1] << 32))


def split(key: Key, num: int = 2) -> List[Key]:
    s = key.seed
    out = []
    for i in range(num):
        o = philox4x32_10((i, 0, 0, 0xC0000000), (s & _MASK, s >> 32))
        out.append(Key(o[0] | (o[1] << 32)))
    return out


def fold_in(key: Key, data: int) -> Key:
    s = key.seed
    o = philox4x32_10((int(data) & _MASK, (int(data) >> 32) & _MASK, 0, 0xB0000000), (s & _MASK, s >> 32))
    return Key(o[0] | (o[1] << 32))


def numpy_rng(key: Key) -> np.random.Generator:
    """Host generator for small index draws (offline subsample permutation, time shifts)."""
    return np.random.Generator(np.random.Philox(key=key.seed))


def uniform(key: Key, shape=(), minval=0.0, maxval=1.0):
    return numpy_rng(key).uniform(minval, maxval, size=shape)


def randint(key: Key, shape, minval, maxval):
    return numpy_rng(key).integers(minval, maxval, size=shape)


def permutation(key: Key, n: int):
    return numpy_rng(key).permutation(n)


def normal(key: Key, shape):
    return numpy_rng(key).standard_normal(shape)
