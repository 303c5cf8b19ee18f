"""Kinetic Ornstein–Uhlenbeck problem (example_problems/kinetic_fokker_planck_example_OU.py).

F = [[0, I], [-tilde_F, -gamma I]], L = diag(0, 2I) (…_OU.py:15-70). The moments
m' = F m, P' = F P + P F^T + L that the reference integrates with odeint (:73-106) are
evaluated in closed form (matrix exponential + Van Loan), on the host in fp64: they are
O(d^3) per time stamp, not per particle. All per-particle work (exact Gaussian samples, the
SDE simulator, residuals) runs on the GPU.

Beyond the reference (whose KOU data are always exact Gaussians, sample_scheme "exact"),
`pde_instance.sample_scheme=SDE` drives the same problem through the Euler–Maruyama
simulator with grad U = tilde_F x — the workload of BASELINE.json configs 1 and 2.
"""
from __future__ import annotations

import math
import warnings
from typing import Tuple, Union

import numpy as np
import torch
from scipy.linalg import expm

from api import ProblemInstance
from core.distribution import Gaussian
from core.model import QuadraticModel
from core.potential import QuadraticPotential
from utils import prng
from utils.prng import Key


def problem_matrix(domain_dim: int, seed: int = 2217) -> np.ndarray:
    """tilde_F = G G^T, G ~ N(0,1)^{d x (d+1)} (…_OU.py:16-19). JAX's PRNGKey(2217) threefry
    stream is unavailable, so G comes from numpy's PCG64 seeded 2217."""
    G = np.random.default_rng(seed).standard_normal((domain_dim, domain_dim + 1))
    return G @ G.T


def initialize_configuration(domain_dim: int, gamma_friction: float = 1.0, P_x_0_scale: float = 1.0,
                             P_v_0_scale: float = 1.0, tilde_L_scale: float = 2.0):
    tilde_F = problem_matrix(domain_dim)
    d = domain_dim
    I, Z = np.eye(d), np.zeros((d, d))
    m_x_0 = np.zeros(d)
    m_v_0 = np.zeros(d)
    P_x_0 = I * P_x_0_scale
    P_v_0 = I * P_v_0_scale
    return {
        "gamma_friction": gamma_friction,
        "tilde_F": tilde_F,
        "F": np.block([[Z, I], [-tilde_F, -gamma_friction * I]]),
        "L": np.block([[Z, Z], [Z, tilde_L_scale * I]]),
        "m_0": np.concatenate([m_x_0, m_v_0]),
        "P_0": np.block([[P_x_0, Z], [Z, P_v_0]]),
        "m_x_0": m_x_0,
        "P_x_0": P_x_0,
    }


def OU_process(t_space, configuration):  # noqa: N802 - reference name
    """Closed-form solution of the moment ODE (…_OU.py:73-93). Returns (m, P) at t_space[-1] if
    len(t_space) == 2, else at t_space[1:] (the reference's odeint output convention)."""
    t_space = np.atleast_1d(np.asarray(t_space, dtype=np.float64))
    assert t_space.size >= 2
    F, L, m0, P0 = (configuration[k] for k in ("F", "L", "m_0", "P_0"))
    n = F.shape[0]
    blk = np.zeros((2 * n, 2 * n))
    blk[:n, :n] = -F
    blk[:n, n:] = L
    blk[n:, n:] = F.T
    ms, Ps = [], []
    for t in t_space[1:]:
        E = expm(F * t)
        V = expm(blk * t)
        P = E @ P0 @ E.T + V[n:, n:].T @ V[:n, n:]
        ms.append(E @ m0)
        Ps.append(0.5 * (P + P.T))
    if t_space.size == 2:
        return ms[-1], Ps[-1]
    return np.stack(ms), np.stack(Ps)


def van_loan_powers(configuration, tmax: float, K: int = 18):
    """B^0..B^K of the Van Loan block B = [[-F, L], [0, F^T]] and the squarings s with |B|_1 tmax / 2^s <= 1 — the
    per-problem constants of the scaled Taylor exponential (host ou_moments_batched, device pdeinv_ou_exact_sample)."""
    F, L = configuration["F"], configuration["L"]
    n = F.shape[0]
    B = np.zeros((2 * n, 2 * n))
    B[:n, :n] = -F
    B[:n, n:] = L
    B[n:, n:] = F.T
    nrm = np.abs(B).sum(axis=0).max() * float(tmax)
    s = max(0, int(np.ceil(np.log2(nrm)))) if nrm > 1.0 else 0
    pw = np.empty((K + 1, 2 * n, 2 * n))
    pw[0] = np.eye(2 * n)
    for k in range(1, K + 1):
        pw[k] = pw[k - 1] @ B
    return pw, s


def ou_moments_batched(ts, configuration):
    """(m(t_g), P(t_g)) for a batch of times in one vectorised pass — the same Van Loan block
    exponential as OU_process, exp(B t) with B = [[-F, L], [0, F^T]], evaluated for every t_g at
    once: the powers B^k (k <= 18) are shared by the batch, so exp(B t_g / 2^s) is one contraction
    of the Taylor coefficients (t_g / 2^s)^k / k! with them, followed by s batched squarings
    (s makes |B| t_max / 2^s <= 1, truncation < 1e-16). Replaces one odeint / expm per random time
    of the reference's exact sampler (…_OU.py:140-156)."""
    ts = np.atleast_1d(np.asarray(ts, dtype=np.float64))
    m0, P0 = configuration["m_0"], configuration["P_0"]
    n = m0.shape[0]
    tmax = float(np.max(np.abs(ts))) if ts.size else 0.0
    pw, s = van_loan_powers(configuration, tmax)
    K = pw.shape[0] - 1
    tau = ts / (2.0 ** s)
    coef = np.ones((ts.size, K + 1))
    for k in range(1, K + 1):
        coef[:, k] = coef[:, k - 1] * tau / k  # tau^k / k!
    X = (coef @ pw.reshape(K + 1, -1)).reshape(-1, 2 * n, 2 * n)
    for _ in range(s):
        X = X @ X
    E = np.transpose(X[:, n:, n:], (0, 2, 1))  # e^{F t}
    P = E @ P0 @ np.transpose(E, (0, 2, 1)) + np.transpose(X[:, n:, n:], (0, 2, 1)) @ X[:, :n, n:]
    return E @ m0, 0.5 * (P + np.transpose(P, (0, 2, 1)))


def sym_sqrt_batched(C):
    """U diag(sqrt S) U^T per matrix — Gaussian.__init__'s SVD square root (distribution.py:59-61)."""
    U, S, _ = np.linalg.svd(C)
    return (U * np.sqrt(S)[:, None, :]) @ np.transpose(U, (0, 2, 1))


def cov_factor_batched(C):
    """A factor R with R R^T = C per matrix: Cholesky (30x cheaper than the SVD square root, the same
    Gaussian law — the reference's sample stream is not reproducible anyway), SVD root if a
    covariance is numerically singular."""
    try:
        return np.linalg.cholesky(C)
    except np.linalg.LinAlgError:
        return sym_sqrt_batched(C)


def get_mean_cov(t, configuration):
    """…_OU.py:96-106."""
    t = np.asarray(t, dtype=np.float64)
    if t.size == 1:
        return OU_process(np.array([0.0, float(t)]), configuration)
    assert t.ndim == 1
    warnings.warn("The user is responsible for ensuring t[0] == 0")
    return OU_process(t, configuration)


class KineticFokkerPlanck(ProblemInstance):
    def __init__(self, cfg, rng: Key):
        super().__init__(cfg, rng)
        self.initial_configuration = initialize_configuration(self.dim)
        self.get_mean_cov = lambda t: get_mean_cov(t, self.initial_configuration)
        ic = self.initial_configuration
        self.distribution_initial = Gaussian(ic["m_0"], ic["P_0"])
        self.distribution_initial_x = Gaussian(ic["m_x_0"], ic["P_x_0"])
        self.distribution_terminal = Gaussian(*self.get_mean_cov(self.total_evolving_time))
        self.potential = QuadraticPotential(A=ic["tilde_F"])
        pi = cfg.pde_instance
        self.sample_scheme = pi.get("sample_scheme", "exact") or "exact"
        self.n_steps = int(pi.get("n_steps", 100) or 100)
        if pi.get("sample_mode", "online") == "offline":
            raise NotImplementedError  # …_OU.py:126-127
        self._counter = 0

    def V_true_fn(self, x: torch.Tensor):  # noqa: N802
        if x.dim() not in (1, 2):
            raise ValueError("x should be either 1D (unbatched) or 2D (batched) array.")
        return self.potential.value(x)

    def exact_sampler(self):
        """The device exact sampler over distribution_time's range (built once per problem)."""
        if getattr(self, "_exact_sampler", None) is None:
            from utils import native
            ic = self.initial_configuration
            t_min, t_max = float(self.distribution_time.mins), float(self.distribution_time.maxs)
            pw, s = van_loan_powers(ic, t_max)
            self._exact_sampler = native.OuExactSampler(pw, s, ic["m_0"], ic["P_0"], t_min, t_max)
        return self._exact_sampler

    def _next_counter(self, n_steps: int) -> int:
        c = self._counter
        self._counter = (self._counter + n_steps + 1) & 0xFFFFFFFF
        return c

    def simulate(self, rng: Key, batch_size: int, n_steps: int = None, *, particle_offset: int = 0,
                 traj: bool = True, moments: bool = False):
        """EM ensemble from distribution_initial (sample_scheme SDE)."""
        from utils.sampling_utils import simulate
        n_steps = n_steps or self.n_steps
        k_init, k_sde = prng.split(rng)
        z0 = self.distribution_initial.sample(batch_size, k_init, row_offset=particle_offset)
        dt = self.total_evolving_time / n_steps
        return z0, simulate(z0, n_steps, dt, k_sde, self.potential, self.initial_configuration["gamma_friction"],
                            particle_offset=particle_offset, counter_offset=self._next_counter(n_steps),
                            traj=traj, tau=traj, moments=moments)

    def sample_ground_truth(self, rng: Key, batch_size: Union[int, Tuple[int, int]]):
        if self.sample_scheme == "SDE":
            # (initial, terminal, 0T) from one EM ensemble, like the GMM problem (…_GMM.py:104-142)
            z0, r = self.simulate(rng, int(batch_size))
            return z0, r["last"], r["traj"].reshape(-1, 2 * self.dim)
        if isinstance(batch_size, int):  # …_OU.py:141-156: 100 samples per random time
            sample_per_time = 100
            assert batch_size >= sample_per_time * 2
            n_random_time = batch_size // sample_per_time
            _, k_x = prng.split(rng)
            # one launch, no host work: the random times, their moments (Van Loan exponential), the Cholesky
            # factors and the rows, one workgroup per time (pdeinv_ou_exact_sample)
            return self.exact_sampler().sample(n_random_time, sample_per_time, seed=k_x.seed)
        k_shift, k = prng.split(rng)
        n_time_stamps, sample_per_time = batch_size
        assert n_time_stamps == 1  # …_OU.py:176 (the reference's grid mode is single-stamp)
        T = self.total_evolving_time
        shift = prng.uniform(k_shift, (n_time_stamps + 1,)) * (T / n_time_stamps)
        stamps = np.linspace(0, T, n_time_stamps + 1) + shift
        stamps = np.concatenate([[0.0], stamps[:-1]])
        means, covs = self.get_mean_cov(stamps)
        means = np.asarray(means).reshape(n_time_stamps, -1)
        covs = np.asarray(covs).reshape(n_time_stamps, 2 * self.dim, 2 * self.dim)
        keys = prng.split(k, n_time_stamps)
        samples = torch.stack([Gaussian(means[i], covs[i]).sample(sample_per_time, keys[i])
                               for i in range(n_time_stamps)], 1)
        return samples.reshape(-1, 2 * self.dim)

    def get_time_sample_ground_truth(self, rng: Key, batch_size):
        if isinstance(batch_size, int):
            raise NotImplementedError  # …_OU.py:193-194
        k_shift, _ = prng.split(rng)
        n_time_stamps = batch_size[0]
        T = self.total_evolving_time
        shift = prng.uniform(k_shift, (n_time_stamps + 1,)) * (T / n_time_stamps)
        return (np.linspace(0, T, n_time_stamps + 1) + shift)[:-1]

    def create_parametric_model(self):
        return QuadraticModel(self.dim, name="tilde_F")
