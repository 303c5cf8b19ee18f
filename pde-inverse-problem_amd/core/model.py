"""Hypothesis models (core/model.py and the problems' create_parametric_model of the reference).

A model is a small object with `init(key, x) -> params` and `apply(params, x)` like a flax
module, where params is the same nested dict the reference's flax modules produce
({"params": {"tilde_F": {"kernel", "bias"}}} etc.) holding torch device tensors.
`residual_kind` tells the consistency method which fused native residual evaluates it.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from utils import prng


def _truncated_normal(rng: np.random.Generator, shape, std):
    # flax/jax variance_scaling "truncated_normal": N(0,1) truncated to [-2, 2], rescaled so the
    # variance is std^2 (0.87962566 = std of the truncated unit normal)
    out = rng.standard_normal(int(np.prod(shape)))
    bad = np.abs(out) > 2
    while bad.any():
        out[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(out) > 2
    return (out * std / 0.87962566103423978).reshape(shape)


def _dense_params(rng, fan_in, fan_out, scale, device):
    k = _truncated_normal(rng, (fan_in, fan_out), np.sqrt(scale / fan_in))
    return {"kernel": torch.as_tensor(k, dtype=torch.float32, device=device),
            "bias": torch.zeros(fan_out, dtype=torch.float32, device=device)}


class QuadraticModel:
    """V_theta(y) = sum(y * Dense_d(y)) — KOU V_parametric (…_OU.py:209-220) and KMV
    Phi_parametric (kinetic_mckean_vlasov_example_quadratic.py:205-216). lecun_normal kernel."""

    residual_kind = "quadratic"

    def __init__(self, dim: int, name: str = "tilde_F"):
        self.dim = int(dim)
        self.name = name

    def init(self, key: prng.Key, x=None, device="cuda"):
        rng = prng.numpy_rng(key)
        return {"params": {self.name: _dense_params(rng, self.dim, self.dim, 1.0, device)}}

    def apply(self, params, y: torch.Tensor):
        p = params["params"][self.name]
        v = torch.sum(y * (y @ p["kernel"] + p["bias"]), dim=-1)
        return v[None]

    def flat(self, params) -> torch.Tensor:
        p = params["params"][self.name]
        return torch.cat([p["kernel"].reshape(-1), p["bias"].reshape(-1)]).contiguous()

    def unflat(self, flat: torch.Tensor):
        d = self.dim
        return {"params": {self.name: {"kernel": flat[: d * d].view(d, d), "bias": flat[d * d:]}}}


class GMMModel:
    """V_theta = GMM with learnable means, uniform weights, sigma = 1 (…_GMM.py:214-234)."""

    residual_kind = "gmm"

    def __init__(self, dim: int, n_Gaussians: int, sigma: float = 1.0):
        self.dim = int(dim)
        self.n_Gaussians = int(n_Gaussians)
        self.sigma = float(sigma)

    def init(self, key: prng.Key, x=None, device="cuda"):
        mus = prng.normal(key, (self.n_Gaussians, self.dim))
        return {"params": {"mus": torch.as_tensor(mus, dtype=torch.float32, device=device)}}

    def apply(self, params, y: torch.Tensor):
        mus = params["params"]["mus"]
        d2 = torch.sum((y[..., None, :] - mus) ** 2, dim=-1)
        return -torch.logsumexp(-d2 / (2 * self.sigma ** 2), dim=-1)[None]

    def flat(self, params) -> torch.Tensor:
        return params["params"]["mus"].reshape(-1).contiguous()

    def unflat(self, flat):
        return {"params": {"mus": flat.view(self.n_Gaussians, self.dim)}}


class V_hypothesis:  # noqa: N801 - reference name
    """Non-parametric model (core/model.py:32-62): Dense(h) x L with tanh, Dense(40), sum y^2.
    kaiming_normal kernels, zero biases. (The reference's `self.F = nn.Dense(4)` is never called
    and owns no parameters.)"""

    residual_kind = "mlp"

    def __init__(self, output_dim: int, hidden_dims: Sequence[int], out_features: int = 40):
        self.output_dim = output_dim
        self.hidden_dims = list(hidden_dims)
        self.out_features = out_features

    def init(self, key: prng.Key, x, device="cuda"):
        rng = prng.numpy_rng(key)
        dims = [int(np.shape(x)[-1])] + self.hidden_dims + [self.out_features]
        return {"params": {f"layers_{i}": _dense_params(rng, dims[i], dims[i + 1], 2.0, device)
                           for i in range(len(dims) - 1)}}

    def dims(self, d: int):
        return [d] + self.hidden_dims + [self.out_features]

    def flat(self, params) -> torch.Tensor:
        p = params["params"]
        return torch.cat([t for i in range(len(p)) for t in (p[f"layers_{i}"]["kernel"].reshape(-1),
                                                              p[f"layers_{i}"]["bias"])]).contiguous()

    def unflat(self, flat: torch.Tensor, d: int):
        dims = self.dims(d)
        out, o = {}, 0
        for i in range(len(dims) - 1):
            k = flat[o:o + dims[i] * dims[i + 1]].view(dims[i], dims[i + 1]); o += dims[i] * dims[i + 1]
            b = flat[o:o + dims[i + 1]]; o += dims[i + 1]
            out[f"layers_{i}"] = {"kernel": k, "bias": b}
        return {"params": out}

    def apply(self, params, y: torch.Tensor):
        h = y
        n = len(params["params"])
        for i in range(n):
            p = params["params"][f"layers_{i}"]
            h = h @ p["kernel"] + p["bias"]
            if i < n - 1:
                h = torch.tanh(h)
        return torch.sum(h * h, dim=-1)[None]


def get_model(cfg, DEBUG=False, pde_instance=None):  # noqa: N803 - reference signature
    """core/model.py:109-131."""
    if cfg.estimation_mode == "parametric":
        print("----Using parametric model----")
        return pde_instance.create_parametric_model()
    if cfg.estimation_mode == "non-parametric":
        print("----Using non-parametric model----")
        if cfg.neural_network.n_resblocks > 0:
            raise NotImplementedError
        if DEBUG:
            return QuadraticModel(pde_instance.dim, name="F")
        return V_hypothesis(output_dim=1, hidden_dims=[cfg.neural_network.hidden_dim] * cfg.neural_network.layers)
    raise NotImplementedError


def tree_leaves(params):
    if isinstance(params, dict):
        out = []
        for k in sorted(params):
            out.extend(tree_leaves(params[k]))
        return out
    return [params]


def tree_map(fn, *trees):
    t0 = trees[0]
    if isinstance(t0, dict):
        return {k: tree_map(fn, *[t[k] for t in trees]) for k in t0}
    return fn(*trees)


def compute_pytree_norm(tree) -> torch.Tensor:
    """utils/common_utils.py:74-76."""
    return torch.sqrt(sum(torch.sum(g.double() * g.double()) for g in tree_leaves(tree))).float()
