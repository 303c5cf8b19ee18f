"""Plugin API (api.py of the reference): ProblemInstance and Method.

Same names, fields and call signatures as the reference (api.py:15-103) so that problems and
methods written against it plug in unchanged; arrays are torch device tensors instead of
jax arrays and RNG keys are utils.prng.Key.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, Tuple, Union

import numpy as np

from core.distribution import Distribution, Uniform
from utils.prng import Key


class ProblemInstance:
    distribution_initial: Distribution
    distribution_initial_x: Distribution
    distribution_terminal: Distribution
    distribution_time: Distribution
    total_evolving_time: float = 1.0
    diffusion_coefficient: float = 0.0
    instance_name: str
    dim: int

    def __init__(self, cfg, rng: Key):
        self.cfg = cfg
        self.instance_name = f"{cfg.pde_instance.domain_dim}D-{cfg.pde_instance.name}"
        self.dim = int(cfg.pde_instance.domain_dim)
        # stored, never used by the reference either (the noise amplitude is hard-coded sqrt(2),
        # sampling_utils.py:14)
        self.diffusion_coefficient = float(cfg.pde_instance.diffusion_coefficient)
        self.total_evolving_time = float(cfg.pde_instance.total_evolving_time)
        # starting from 1e-4 to avoid numerical issue (api.py:34-36)
        self.distribution_time = Uniform(np.asarray(1e-4), np.asarray(self.total_evolving_time))
        self.sample_scheme = "exact"  # "exact" or "SDE"
        self.sample_mode = "online"  # "online" or "offline"

    def sample_ground_truth(self, rng: Key, batch_size: Union[int, Tuple[int, int]]):
        pass

    def get_time_sample_ground_truth(self, rng: Key, batch_size: Union[int, Tuple[int, int]]):
        pass

    def generate_ground_truth_dataset(self, rng: Key):
        pass

    def create_parametric_model(self):
        pass


@dataclass
class Method:
    pde_instance: ProblemInstance
    cfg: Any
    rng: Key

    def value_and_grad_fn(self, forward_fn, params, rng) -> Dict[str, Any]:
        raise NotImplementedError

    def test_fn(self, forward_fn, params, rng):
        pass

    def plot_fn(self, forward_fn, params, rng):
        return  # the reference returns before plotting (api.py:81-82)

    def create_model_fn(self):
        raise NotImplementedError
