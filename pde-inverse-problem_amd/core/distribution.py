"""Distributions of the hot path (core/distribution.py of the reference).

`Gaussian.sample` is the initial-ensemble / exact-sample generator (distribution.py:52-65):
z = C^{1/2} xi + mu, with C^{1/2} = U diag(sqrt S) U^T from the SVD of C, computed once on the
host in fp64 and sampled on the GPU by pdeinv_gaussian_sample (Philox normals in registers).
score / logdensity follow distribution.py:67-81.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from utils import native
from utils.prng import Key


class Distribution:
    def sample(self, batch_size: int, key: Key):
        raise NotImplementedError

    def score(self, x):
        raise NotImplementedError

    def logdensity(self, x):
        raise NotImplementedError

    def density(self, x):
        return torch.exp(self.logdensity(x))


class Gaussian(Distribution):
    def __init__(self, mu, cov, device: Optional[str] = None):
        mu = np.asarray(mu, dtype=np.float64)
        cov = np.asarray(cov, dtype=np.float64)
        if not (mu.ndim == 1 and cov.ndim == 2 and cov.shape[0] == cov.shape[1] == mu.shape[0]):
            raise ValueError("Gaussian needs mu [d] and cov [d, d]")  # distribution.py:54
        self.dim = mu.shape[0]
        self.mu_host, self.cov_host = mu, cov
        U, S, _ = np.linalg.svd(cov)
        self.cov_half_host = U @ np.diag(np.sqrt(S)) @ U.T
        self.inv_cov_host = np.linalg.inv(cov)
        self.log_det = float(np.log(np.linalg.det(cov * 2 * math.pi)))
        self._device = device
        self._dev_cache = None

    def _dev(self):
        if self._dev_cache is None:
            dev = self._device or "cuda"
            f = lambda a: torch.as_tensor(a, dtype=torch.float32, device=dev).contiguous()
            self._dev_cache = (f(self.mu_host), f(self.cov_half_host), f(self.inv_cov_host))
        return self._dev_cache

    @property
    def mu(self):
        return self._dev()[0]

    @property
    def cov_half(self):
        return self._dev()[1]

    def sample(self, batch_size: int, key: Key, row_offset: int = 0, counter_offset: int = 0):
        """[batch_size, d] on the GPU (distribution.py:64-65)."""
        mu, ch, _ = self._dev()
        return native.gaussian_sample(int(batch_size), mu, ch, seed=key.seed,
                                      counter_offset=counter_offset, row_offset=row_offset)

    def score(self, x: torch.Tensor):
        mu, _, inv = self._dev()
        return (mu - x) @ inv.T

    def logdensity(self, x: torch.Tensor):
        mu, _, inv = self._dev()
        off = x - mu
        quad = torch.sum(off * (off @ inv.T), dim=-1)
        return -0.5 * (self.log_det + quad)


class Uniform(Distribution):
    """distribution.py:162-186 (the time sampler)."""

    def __init__(self, mins, maxs):
        mins = np.asarray(mins, dtype=np.float64)
        maxs = np.asarray(maxs, dtype=np.float64)
        if mins.ndim != maxs.ndim:
            raise ValueError("mins and maxs should be arrays of the same size")
        if mins.ndim == 1 and len(mins) != len(maxs):
            raise ValueError("mins and maxs should be of the same dimension")
        if mins.ndim > 1:
            raise ValueError("mins and maxs should be either 0D or 1D arrays")
        self.dim = mins.shape[0] if mins.ndim == 1 else 0
        self.mins, self.maxs = mins, maxs

    def sample(self, batch_size: int, key: Key):
        from utils import prng
        shape = [batch_size, self.dim] if self.dim else [batch_size]
        return prng.uniform(key, shape, self.mins, self.maxs)
