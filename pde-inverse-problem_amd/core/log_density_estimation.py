"""Log-density estimation driver (core/log_density_estimation.py of the reference).

`create_normalizing_flow_fn` builds the same model as the reference (:103-114): MNF(dim,
embed_time_dim=10, couple_mul=4, mask_type='loop', activation 'celu', soft_init=1,
ignore_time=False) inside RealNVP with the problem's initial x-marginal as base density. Its
evaluation (the per-particle log-density of SURVEY.md §8(a) a12) runs on the HIP kernel.
The reference never calls `estimate_log_density` (main.py:50 is commented out); its training
loop needs the flow's parameter gradient, which has no native kernel yet, so it raises.
"""
from __future__ import annotations

from core.normalizing_flow import MNF, RealNVP


def create_normalizing_flow_fn(log_prob_0, dim):
    param_dict = {
        "dim": dim,
        "embed_time_dim": 10,
        "couple_mul": 4,
        "mask_type": "loop",
        "activation_layer": "celu",
        "soft_init": 1.0,
        "ignore_time": False,
    }
    return RealNVP(MNF(**param_dict), log_prob_0)


def estimate_log_density(cfg, pde_instance, rng):
    raise NotImplementedError("RealNVP training (log_density_estimation.py:13-101) needs the flow's parameter "
                              "gradient kernel; only the log-density evaluation is native (create_normalizing_flow_fn)")
