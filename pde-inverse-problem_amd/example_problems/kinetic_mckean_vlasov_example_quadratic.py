"""Kinetic McKean–Vlasov with a quadratic interaction (kinetic_mckean_vlasov_example_quadratic.py).

Like the reference, the class inherits the kinetic OU problem: with a quadratic interaction
Phi*(y) = 0.5 y^T tilde_F y and a centred ensemble, grad Phi* * rho_t (x) = tilde_F (x - xbar) is
the OU drift (README.md:55-80), so the exact sampler and the moment ODE are shared. Added here:
  * the score / log-density time derivatives of the X-marginal N(m1(s), P11(s)) used by the
    residual (:18-191): per time stamp the host forms, in fp64 from the closed-form moments, the
    quadratic-form coefficients; the per-particle evaluation runs in the pdeinv_kmv_weights kernel;
  * sample_scheme=SDE: the interacting-particle system itself, simulated with one all-reduced
    mean-field per update (utils/mean_field.py) — BASELINE.json config 4.
"""
from __future__ import annotations

import numpy as np
import torch

from core.model import QuadraticModel
from core.potential import MeanFieldQuadraticPotential
from example_problems.kinetic_fokker_planck_example_OU import KineticFokkerPlanck
from utils import native, prng
from utils.prng import Key


def _mean_cov_stamps(s, configuration):
    """(m(s_k), P(s_k)) at every stamp: the closed form of OU_process (…_OU.py:73-93) with the
    matrix exponentials of all stamps taken in one batched call."""
    from scipy.linalg import expm

    s = np.atleast_1d(np.asarray(s, dtype=np.float64))
    F, L, m0, P0 = (configuration[k] for k in ("F", "L", "m_0", "P_0"))
    n = F.shape[0]
    blk = np.zeros((2 * n, 2 * n))
    blk[:n, :n] = -F
    blk[:n, n:] = L
    blk[n:, n:] = F.T
    E = expm(F[None] * s[:, None, None])
    V = expm(blk[None] * s[:, None, None])
    P = E @ P0 @ E.transpose(0, 2, 1) + V[:, n:, n:].transpose(0, 2, 1) @ V[:, :n, n:]
    return E @ m0, 0.5 * (P + P.transpose(0, 2, 1))


def dlogrho_coefficients(s_values, configuration, dim: int) -> np.ndarray:
    """Coefficient rows [m1, a1, beta1, Gamma1, a2, beta2, Gamma2] (include/pdeinv.h) such that
    ds log rho = a1 + beta1.r + r^T Gamma1 r and ds2 log rho = a2 + beta2.r + r^T Gamma2 r, r = m1 - x,
    restating partial_s_log_density_fn (:51-69) and partial_s2_log_density_fn (:120-177), batched
    over the time stamps."""
    F, L = configuration["F"], configuration["L"]
    d = dim
    mean, cov = _mean_cov_stamps(s_values, configuration)
    K = mean.shape[0]
    m1, P11 = mean[:, :d], cov[:, :d, :d]
    Pinv = np.linalg.inv(P11)
    dm = mean @ F.T
    d2m = dm @ F.T
    dP = F @ cov + cov @ F.T + L
    d2P = F @ dP + dP @ F.T
    dm1, d2m1, dP11, d2P11 = dm[:, :d], d2m[:, :d], dP[:, :d, :d], d2P[:, :d, :d]
    PdP = Pinv @ dP11
    dPinv = -PdP @ Pinv
    d2Pinv = -Pinv @ d2P11 @ Pinv + 2 * PdP @ PdP @ Pinv
    tr = lambda X: np.einsum("kii->k", X)
    a1 = -0.5 * tr(dP11 @ Pinv)
    beta1 = -np.einsum("kij,kj->ki", Pinv, dm1)
    G1 = -0.5 * dPinv
    a2 = -np.einsum("ki,kij,kj->k", dm1, Pinv, dm1) + 0.5 * tr(PdP @ PdP) - 0.5 * tr(Pinv @ d2P11)
    beta2 = -np.einsum("kij,kj->ki", Pinv, d2m1) - np.einsum("kij,kj->ki", dPinv + dPinv.transpose(0, 2, 1), dm1)
    G2 = -0.5 * d2Pinv
    return np.concatenate([m1, a1[:, None], beta1, G1.reshape(K, -1), a2[:, None], beta2, G2.reshape(K, -1)], axis=1)


class KineticMcKeanVlasov(KineticFokkerPlanck):
    def __init__(self, cfg, rng: Key):
        super().__init__(cfg, rng)
        self.interaction = MeanFieldQuadraticPotential(self.initial_configuration["tilde_F"])

    def coefficients(self, s_values, device="cuda") -> torch.Tensor:
        c = dlogrho_coefficients(s_values, self.initial_configuration, self.dim)
        return torch.as_tensor(c, dtype=torch.float32, device=device).contiguous()

    def _ds(self, s, x: torch.Tensor):
        s_arr = np.atleast_1d(np.asarray(s, dtype=np.float64))
        x2 = x.reshape(-1, self.dim).contiguous()
        coef = self.coefficients(s_arr, x.device)
        _, ds = native.kmv_weights(self.dim, self.initial_configuration["gamma_friction"], coef, x2, len(s_arr),
                                   x2.shape[0], 0, self.dim, want_ds=True)
        return ds  # [n_s, n_x, 2]

    def _shape(self, s, x, v):
        s_scalar = np.ndim(s) == 0
        if x.dim() not in (1, 2) or np.ndim(s) > 1:
            raise ValueError("Shapes of s and x are not supported.")
        if x.dim() == 1:
            return v[0, 0] if s_scalar else v[:, 0]
        return v[0] if s_scalar else v.transpose(0, 1)  # [n_x] or [n_x, n_s] (vmap order of :74-83)

    def partial_s_log_density_fn(self, s, x: torch.Tensor):
        return self._shape(s, x, self._ds(s, x)[..., 0])

    def partial_s2_log_density_fn(self, s, x: torch.Tensor):
        return self._shape(s, x, self._ds(s, x)[..., 1])

    def Phi_true_fn(self, x: torch.Tensor):  # noqa: N802
        if x.dim() not in (1, 2):
            raise ValueError("x should be either 1D (unbatched) or 2D (batched) array.")
        F = torch.as_tensor(self.initial_configuration["tilde_F"], dtype=x.dtype, device=x.device)
        return 0.5 * torch.sum(x * (x @ F.T), -1)

    def simulate_interacting(self, rng: Key, batch_size: int, n_steps: int = None, particle_offset: int = 0,
                             stamp_sums: bool = False):
        """The McKean–Vlasov particle system (sample_scheme SDE): traj [n, N, 2d], shared tau [n].
        stamp_sums=True: no trajectory; instead the quadratic-Phi KMV residual's per-stamp sums formed inside the
        simulator ("kmv_mom" / "kmv_wst", pdeinv_sde_simulate_mf_kmv) and the shared stamps "tau_0T" [n] (fp64 of
        the simulator's fp32 stamps, computed on the host from the same Philox draw)."""
        from utils.mean_field import simulate_mean_field, stamp_times
        n_steps = n_steps or self.n_steps
        k_init, k_sde = prng.split(rng)
        z0 = self.distribution_initial.sample(batch_size, k_init, row_offset=particle_offset)
        dt = self.total_evolving_time / n_steps
        gamma = self.initial_configuration["gamma_friction"]
        ctr = self._next_counter(n_steps)
        if not stamp_sums:
            r = simulate_mean_field(z0, n_steps, dt, k_sde, self.interaction, gamma, particle_offset=particle_offset,
                                    counter_offset=ctr)
            return z0, r
        tau = stamp_times(k_sde.seed, ctr, n_steps, dt).astype(np.float64)
        r = simulate_mean_field(z0, n_steps, dt, k_sde, self.interaction, gamma, particle_offset=particle_offset,
                                counter_offset=ctr, traj=False, tau=False,
                                kmv_coef=self.coefficients(tau, z0.device), kmv_gamma=gamma)
        r["tau_0T"] = tau
        return z0, r

    def create_parametric_model(self):
        return QuadraticModel(self.dim, name="tilde_F")
