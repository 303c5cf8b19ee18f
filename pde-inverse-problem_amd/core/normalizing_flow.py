"""Time-conditioned RealNVP (core/normalizing_flow.py of the reference, :8-229).

Same constructor arguments and call convention as the reference's flax modules:
`MNF(dim, couple_mul, mask_type, soft_init, ignore_time, activation_layer, embed_time_dim)` and
`RealNVP(mnf, log_prob_0)`; `init(key, t, x) -> params`, `apply(params, t, x) -> log p_t(x)` for a
single (t, x) or batched rows (the reference vmaps the same call). The evaluation is the HIP
kernel `pdeinv_realnvp_logdensity` (one thread per sample, VALU); params are a flat fp32 device
vector in the layout documented in include/pdeinv.h. `log_prob_0` must be a `core.distribution.Gaussian`
(the reference passes `distribution_initial_x.logdensity`, log_density_estimation.py:22).
"""
from __future__ import annotations

import numpy as np
import torch

from utils import native
from utils import prng


def make_masks(dim: int, couple_mul: int, mask_type: str) -> np.ndarray:
    """MNF.setup (:174-199): 'loop' (one coordinate per layer) or 'random' (RandomState(888))."""
    if mask_type == "loop":
        masks = np.ones((dim * couple_mul, dim))
        for i in range(dim * couple_mul):
            masks[i, i % dim] = 0
        return masks
    if mask_type != "random":
        raise ValueError(f"unknown mask_type {mask_type}")
    rng = np.random.RandomState(seed=888)
    prev = np.zeros(dim, dtype=int)
    out = []
    for _ in range(couple_mul):
        while True:
            m = rng.binomial(1, p=0.5, size=[dim])
            if not (m.sum() in [0, dim] or (m == prev).all()):
                prev = m
                break
        out.append(m)
    return np.asarray(out, dtype=np.float64)


class MNF:
    """Masked normalizing flow (:166-220)."""

    def __init__(self, dim: int, couple_mul: int, mask_type: str, soft_init: float, ignore_time: bool,
                 activation_layer: str, embed_time_dim: int):
        self.dim = int(dim)
        self.couple_mul = int(couple_mul)
        self.mask_type = mask_type
        self.soft_init = float(soft_init)
        self.ignore_time = bool(ignore_time)
        self.activation_layer = activation_layer
        self.embed_time_dim = int(embed_time_dim)
        self.masks = make_masks(self.dim, self.couple_mul, mask_type)

    @property
    def n_layers(self) -> int:
        return self.masks.shape[0]

    def in_dim(self) -> int:
        return self.dim if self.ignore_time else self.dim + (self.embed_time_dim if self.embed_time_dim > 0 else 1)

    def param_count(self) -> int:
        E = 0 if self.ignore_time else self.embed_time_dim
        i = self.in_dim()
        mlp = i * 8 + 8 + 8 * 16 + 16 + 16 * 16 + 16 + 16 * self.dim + self.dim
        return (2 * (E * E + E) if E > 0 else 0) + self.n_layers * (self.dim + 2 * mlp)

    def init(self, key: prng.Key, t=None, x=None, device="cuda"):
        """flax defaults: lecun_normal kernels (truncated normal), zero biases, zero scaling factors."""
        rng = prng.numpy_rng(key)
        parts = []

        def dense(i, o):
            k = rng.standard_normal(i * o)
            bad = np.abs(k) > 2
            while bad.any():
                k[bad] = rng.standard_normal(int(bad.sum()))
                bad = np.abs(k) > 2
            parts.extend([k / 0.87962566103423978 * np.sqrt(1.0 / i), np.zeros(o)])

        E = 0 if self.ignore_time else self.embed_time_dim
        if E > 0:
            dense(E, E)
            dense(E, E)
        i = self.in_dim()
        for _ in range(self.n_layers):
            parts.append(np.zeros(self.dim))
            for _ in range(2):
                dense(i, 8)
                dense(8, 16)
                dense(16, 16)
                dense(16, self.dim)
        flat = np.concatenate(parts)
        assert flat.size == self.param_count()
        return {"params": torch.as_tensor(flat, dtype=torch.float32, device=device)}


class RealNVP:
    """log p_t(x) = log p0(T_t^{-1}(x)) + sum ldj (:223-229)."""

    def __init__(self, mnf: MNF, log_prob_0):
        self.mnf = mnf
        self.log_prob_0 = log_prob_0
        g = log_prob_0.__self__ if hasattr(log_prob_0, "__self__") else log_prob_0
        if not all(hasattr(g, a) for a in ("mu_host", "inv_cov_host", "log_det")):
            raise NotImplementedError("RealNVP: log_prob_0 must be a core.distribution.Gaussian (or its .logdensity)")
        if g.mu_host.shape[0] != mnf.dim:
            raise ValueError("RealNVP: the base density's dimension differs from the flow's")
        self._desc, self._keep = native.realnvp_desc(
            mnf.dim, mnf.masks, mnf.embed_time_dim, mnf.ignore_time, mnf.soft_init, mnf.activation_layer,
            g.mu_host, g.inv_cov_host, float(g.log_det))

    def init(self, key: prng.Key, t=None, x=None, device="cuda"):
        return self.mnf.init(key, t, x, device=device)

    def apply(self, params, t, x):
        flat = params["params"] if isinstance(params, dict) else params
        x = torch.as_tensor(x, dtype=torch.float32, device=flat.device)
        single = x.dim() == 1
        rows = x.reshape(1, -1) if single else x
        tt = torch.as_tensor(t, dtype=torch.float32, device=flat.device).reshape(-1)
        out = native.realnvp_logdensity(self._desc, flat, tt, rows)
        return out[0] if single else out

    def value_and_grad(self, params, t, x):
        """(loss, grad) with loss = -mean_i log p_{t_i}(x_i) and grad flat like params
        (log_density_estimation.py:47-58), on the HIP kernel. celu / elu flows only."""
        flat = params["params"] if isinstance(params, dict) else params
        x = torch.as_tensor(x, dtype=torch.float32, device=flat.device)
        tt = torch.as_tensor(t, dtype=torch.float32, device=flat.device).reshape(-1)
        return native.realnvp_value_and_grad(self._desc, flat, tt, x.reshape(-1, self.mnf.dim) if x.dim() == 1 else x)

    __call__ = apply
