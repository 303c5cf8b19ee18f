"""Kinetic Fokker–Planck with a GMM potential (example_problems/kinetic_fokker_planck_example_GMM.py).

U(x) = -logsumexp_k(-|x - mu_k|^2/2), gamma = 0.5, x0 ~ N(0, 4I), v0 ~ N(0, 0.1I)
(…_GMM.py:16-63). Ground truth only by simulation: online (sample_ground_truth, :104-142) or
an offline dataset generated once (:158-204), both through the HIP simulator.

Reference quirk fixed here: the reference's online path unpacks two values from the
three-valued simulator (:115, :133) and raises ValueError on its first iteration
(SURVEY.md §0.1); this implementation returns what that code evidently intends.
"""
from __future__ import annotations

import numpy as np
import torch

from api import ProblemInstance
from core.distribution import Gaussian
from core.model import GMMModel
from core.potential import GMMPotential
from utils import prng
from utils.prng import Key
from utils.sampling_utils import simulate


def gmm_means(domain_dim: int, n_Gaussian: int, rng: Key, lo: float = -4.0, hi: float = 4.0):  # noqa: N803
    """mu_k ~ U[-4, 4]^d, one key per component (…_GMM.py:21-23, 52-59)."""
    return np.stack([prng.uniform(k, (domain_dim,), lo, hi) for k in prng.split(rng, n_Gaussian)])


def initialize_configuration(domain_dim: int, rng: Key, n_Gaussian: int = 3):  # noqa: N803
    d = domain_dim
    I, Z = np.eye(d), np.zeros((d, d))
    P_x_0 = I * 4.0
    P_v_0 = I * 0.1
    return {
        "n_Gaussian": n_Gaussian,  # 3 in the reference (:19); a config key here (BASELINE config 3: 8)
        "gamma_friction": 0.5,
        "m_0": np.zeros(2 * d),
        "P_0": np.block([[P_x_0, Z], [Z, P_v_0]]),
        "m_x_0": np.zeros(d),
        "P_x_0": P_x_0,
        "GMM": {"mus": gmm_means(d, n_Gaussian, rng)},
    }


class KineticFokkerPlanck(ProblemInstance):
    def __init__(self, cfg, rng: Key):
        super().__init__(cfg, rng)
        rng_config, rng_dataset = prng.split(rng)
        pi = cfg.pde_instance
        self.initial_configuration = initialize_configuration(self.dim, rng_config,
                                                              int(pi.get("n_Gaussian", 3) or 3))
        self.potential = GMMPotential(self.initial_configuration["GMM"]["mus"], 1.0)
        self.sample_scheme = "SDE"
        self.sample_mode = pi.sample_mode
        ic = self.initial_configuration
        self.distribution_initial = Gaussian(ic["m_0"], ic["P_0"])
        self.distribution_initial_x = Gaussian(ic["m_x_0"], ic["P_x_0"])
        self._counter = 0
        if self.sample_mode == "offline":
            self.dataset = self.generate_ground_truth_dataset(rng_dataset)

    def V_true_fn(self, x: torch.Tensor):  # noqa: N802
        if x.dim() not in (1, 2):
            raise ValueError("x should be either 1D (unbatched) or 2D (batched) array.")
        return self.potential.value(x)

    def _next_counter(self, n_steps):
        c = self._counter
        self._counter = (self._counter + n_steps + 1) & 0xFFFFFFFF
        return c

    def _run(self, key: Key, n: int, n_steps: int, traj: bool):
        k0, k1 = prng.split(key)
        z0 = self.distribution_initial.sample(n, k0)
        dt = self.total_evolving_time / n_steps
        r = simulate(z0, n_steps, dt, k1, self.potential, self.initial_configuration["gamma_friction"],
                     counter_offset=self._next_counter(n_steps), traj=traj, tau=traj)
        return r

    def sample_ground_truth(self, rng: Key, batch_size: int):
        """(initial [30B], terminal [30B], 0T [B*n]) — …_GMM.py:104-142."""
        rng, rng2, _, rng_init2, _ = prng.split(rng, 5)
        multiple_init = multiple_terminal = 30
        n_steps = int(self.cfg.pde_instance.n_steps)
        r = self._run(rng, batch_size, n_steps, traj=True)
        # flattened 0T samples (:124); sample order is irrelevant to the residual's means, so the
        # time-major buffer is flattened as is (no transpose copy)
        sample_0T = r["traj"].reshape(-1, 2 * self.dim)
        sample_initial = self.distribution_initial.sample(batch_size * multiple_init, rng_init2)
        sample_final = self._run(rng2, batch_size * multiple_terminal, n_steps, traj=False)["last"]
        return sample_initial, sample_final, sample_0T

    def generate_ground_truth_dataset(self, rng: Key):
        """…_GMM.py:158-204. "0T" is kept time-major [n, N, 2d] in "0T_tm" (the layout the
        simulator writes and the gather kernel reads); "0T" is the reference's [N, n, 2d] view."""
        rng_initial, rng_terminal, rng_0T = prng.split(rng, 3)
        pi = self.cfg.pde_instance
        dataset = {"initial": self.distribution_initial.sample(int(pi.sample_initial_size), rng_initial)}
        dataset["terminal"] = self._run(rng_terminal, int(pi.sample_terminal_size), int(pi.n_steps_terminal),
                                        traj=False)["last"]
        r = self._run(rng_0T, int(pi.sample_0T_size), int(pi.n_steps_0T), traj=True)
        dataset["0T_tm"] = r["traj"]
        dataset["0T"] = r["traj"].permute(1, 0, 2)
        dataset["tau_0T"] = r["tau"].permute(1, 0)
        return dataset

    def create_parametric_model(self):
        return GMMModel(self.dim, self.initial_configuration["n_Gaussian"])
