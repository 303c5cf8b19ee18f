"""Potentials (core/potential.py of the reference).

Each potential knows how to describe itself to the native simulator (`native_desc`), which is
how `underdamped_langevin_dynamics_scan` receives "potential_grad" without a Python callback
inside the kernel. value / gradient over batches run on the GPU.
"""
from __future__ import annotations

import numpy as np
import torch

from utils import native


class Potential:
    def gradient(self, x):
        raise NotImplementedError

    def native_desc(self) -> dict:
        raise NotImplementedError


class QuadraticPotential(Potential):
    """grad U(x) = A (x - mu); the reference's QuadraticPotential uses A = cov^-1
    (potential.py:11-24); KOU's V_true uses A = tilde_F, mu = 0 (…_OU.py:130-138)."""

    def __init__(self, mu=None, cov=None, A=None):
        if A is None:
            cov = np.asarray(cov, dtype=np.float64)
            if cov.ndim != 2 or cov.shape[0] != cov.shape[1]:
                raise ValueError("cov must be square")
            A = np.linalg.inv(cov)
        self.A = np.asarray(A, dtype=np.float64)
        self.dim = self.A.shape[0]
        self.mu = None if mu is None else np.asarray(mu, dtype=np.float64)

    def value(self, x: torch.Tensor):
        A = torch.as_tensor(self.A, dtype=x.dtype, device=x.device)
        y = x if self.mu is None else x - torch.as_tensor(self.mu, dtype=x.dtype, device=x.device)
        return 0.5 * torch.sum(y * (y @ A.T), -1)

    def gradient(self, x: torch.Tensor):
        A = torch.as_tensor(self.A, dtype=x.dtype, device=x.device)
        y = x if self.mu is None else x - torch.as_tensor(self.mu, dtype=x.dtype, device=x.device)
        return y @ A.T

    def native_desc(self) -> dict:
        has_c = self.mu is not None and np.any(self.mu != 0)
        params = self.A.ravel() if not has_c else np.concatenate([self.A.ravel(), self.mu])
        return dict(kind=native.POT_QUADRATIC, params=params, has_center=bool(has_c))


class VoidPotential(Potential):
    def gradient(self, x):
        return torch.zeros_like(x)

    def native_desc(self) -> dict:
        return dict(kind=native.POT_NONE)


class GMMPotential(Potential):
    """V(x) = -logsumexp_k(-|x - mu_k|^2 / (2 sigma^2)) (potential.py:32-61)."""

    def __init__(self, mus, sigma=1.0):
        self.mus = np.asarray(mus, dtype=np.float64)
        self.sigma = float(np.asarray(sigma))
        self.n_centers, self.dim = self.mus.shape

    def value(self, x: torch.Tensor):
        single = x.dim() == 1
        v, _ = native.gmm_potential(x.reshape(-1, self.dim).contiguous(), self.mus, self.sigma, True, False)
        return v[0] if single else v

    def gradient(self, x: torch.Tensor):
        single = x.dim() == 1
        _, g = native.gmm_potential(x.reshape(-1, self.dim).contiguous(), self.mus, self.sigma, False, True)
        return g[0] if single else g

    def native_desc(self) -> dict:
        return dict(kind=native.POT_GMM, params=self.mus.ravel(), n_centers=self.n_centers, sigma=self.sigma)


class MeanFieldQuadraticPotential(Potential):
    """McKean–Vlasov interaction Phi*(y) = 0.5 y^T A y: the drift on particle i is
    mean_j grad Phi*(x_i - x_j) = A (x_i - xbar) (kinetic_mckean_vlasov.py:20-23, README.md:55-80)."""

    def __init__(self, A):
        self.A = np.asarray(A, dtype=np.float64)
        self.dim = self.A.shape[0]

    def native_desc(self) -> dict:
        return dict(kind=native.POT_MEANFIELD_QUADRATIC, params=self.A.ravel())


def resolve(potential_grad) -> Potential:
    """Accept a Potential or its bound `.gradient` (what the reference passes, …_GMM.py:120)."""
    if isinstance(potential_grad, Potential):
        return potential_grad
    owner = getattr(potential_grad, "__self__", None)
    if isinstance(owner, Potential):
        return owner
    raise NotImplementedError(
        "potential_grad must be a core.potential.Potential (or its .gradient): arbitrary Python "
        "callables cannot run inside the HIP simulator and there is no CPU fallback")
