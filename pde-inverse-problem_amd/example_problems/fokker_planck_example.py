"""Overdamped Fokker–Planck / OU problem (example_problems/fokker_planck_example.py).

dX = -F X dt + sqrt(L) dW with F = G G^T SPD, L = 2 I (the Laplacian coefficient 1), X(0) ~
N(m0 = 1, P0 = 5 I) (:20-46). In the eigenbasis F = U diag(s) U^T the law stays Gaussian with the
closed form of OU_process (:48-55):
    U^T m(t) = e^{-ts} o U^T m0,   U^T P(t) U = e B0 e + B / (s_i + s_j) o (1 - e_i e_j),
    e = diag(e^{-ts}), B0 = U^T P0 U, B = U^T L U.
This is the reference's DEFAULT pde_instance (configurations/config.yaml:2). Its exact sampler
draws one random time per sample (sample_ground_truth :88-96, vmapped over split keys); here the
whole batch — times, moments, Cholesky factors and samples — is one HIP launch
(pdeinv_fp_exact_sample). G comes from numpy's PCG64 seeded 2217, the same recipe as the kinetic
problems (JAX's PRNGKey(2217) threefry stream is unavailable).
"""
from __future__ import annotations

from typing import Tuple, Union

import numpy as np
import torch

from api import ProblemInstance
from core.distribution import Gaussian
from core.potential import QuadraticPotential
from example_problems.kinetic_fokker_planck_example_OU import problem_matrix
from utils import prng
from utils.prng import Key


def initialize_configuration(domain_dim: int):
    """:20-46 (F_scale 1, L_scale 2, m_0_scale 1, P_0_scale 5)."""
    m_0 = np.ones(domain_dim) * 1.0
    P_0 = np.eye(domain_dim) * 5.0
    F = problem_matrix(domain_dim) * 1.0
    L = np.eye(domain_dim) * 2.0
    U, s, _ = np.linalg.svd(F)
    return {"F": F, "L": L, "U": U, "ss": s + s[:, None], "B": U.T @ L @ U, "B_0": U.T @ P_0 @ U, "s": s,
            "m_0": m_0, "P_0": P_0}


def OU_process(t, configuration):  # noqa: N802 - reference name
    """:48-55, vectorised over t (scalar or [n])."""
    t = np.asarray(t, dtype=np.float64)
    c = configuration
    e = np.exp(-t[..., None] * c["s"])                      # [..., d]
    m = (e * (c["U"].T @ c["m_0"])) @ c["U"].T
    ee = e[..., :, None] * e[..., None, :]
    B_S = c["B"] / c["ss"]
    P_eig = ee * c["B_0"] + B_S - ee * B_S
    P = c["U"] @ P_eig @ c["U"].T
    return m, P


def get_distribution(t, configuration):
    mean, cov = OU_process(t, configuration)
    return Gaussian(mean, cov)


class FokkerPlanck(ProblemInstance):
    def __init__(self, cfg, rng: Key):
        super().__init__(cfg, rng)
        self.initial_configuration = initialize_configuration(self.dim)
        self.get_distribution = lambda t: get_distribution(t, self.initial_configuration)
        self.distribution_initial = self.get_distribution(0.0)
        self.distribution_terminal = self.get_distribution(self.total_evolving_time)
        self.potential = QuadraticPotential(A=self.initial_configuration["F"])
        c = self.initial_configuration
        self._eig = {"U": c["U"], "s": c["s"], "Um0": c["U"].T @ c["m_0"], "B0": c["B_0"], "B": c["B"]}
        self._row = 0

    def V_true_fn(self, x: torch.Tensor):  # noqa: N802
        """x^T F x / 2 (:75-83)."""
        if x.dim() not in (1, 2):
            raise ValueError("x should be either 1D (unbatched) or 2D (batched) array.")
        return self.potential.value(x)

    def sample_ground_truth(self, rng: Key, batch_size: Union[int, Tuple[int, int]], return_time: bool = False):
        """:85-96 — every sample its own time t ~ distribution_time = U(1e-4, T) (api.py:34-36)."""
        if not isinstance(batch_size, int):
            raise NotImplementedError("Fokker-Planck samples one random time per sample (random_time mode only)")
        from utils import native
        lo, hi = float(self.distribution_time.mins), float(self.distribution_time.maxs)
        return native.fp_exact_sample(int(batch_size), self._eig, seed=rng.seed, t_range=(lo, hi),
                                      return_t=return_time)

    def create_parametric_model(self):
        # the reference's FP create_model_fn calls get_model without the instance, so its
        # parametric mode cannot run (fokker_planck.py:88-90 -> core/model.py:110-113)
        raise NotImplementedError("Fokker-Planck has no parametric model in the reference "
                                  "(use estimation_mode=non-parametric)")
