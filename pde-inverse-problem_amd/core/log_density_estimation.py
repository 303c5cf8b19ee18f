"""Log-density estimation driver (core/log_density_estimation.py of the reference).

`create_normalizing_flow_fn` builds the same model as the reference (:103-114): MNF(dim,
embed_time_dim=10, couple_mul=4, mask_type='loop', activation 'celu', soft_init=1,
ignore_time=False) inside RealNVP with the problem's initial x-marginal as base density.
`estimate_log_density` is the reference's maximum-likelihood training loop (:13-100): every epoch
takes one in five time stamps from a random phase and a random fifth of the offline trajectories
(the native gather kernel over the time-major dataset), evaluates loss = -mean log p and its
parameter gradient on the HIP kernel `pdeinv_realnvp_value_and_grad` (replacing
jax.value_and_grad) and takes an Adam step (b1 = 0.9, eps = 1e-4) on the fused native update,
with the reference's constant / cosine / constant learning-rate schedule (:116-145). Epoch losses
stay on the device and are fetched once per print interval. The closing density plot
(plot_trajectory_of_distributions, matplotlib + wandb) is out of scope.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from core.normalizing_flow import MNF, RealNVP
from utils import native, prng


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


def create_custom_schedule(lr, T0, T1):
    """optax.join_schedules([constant(lr), warmup_cosine_decay(lr, lr, 0, T1 - T0, lr * 1e-2),
    constant(lr * 1e-2)], [T0, T1]) (:116-145)."""
    def schedule(step):
        if step < T0:
            return lr
        if step < T1:
            s = min(step - T0, T1 - T0) / (T1 - T0)
            alpha = 1e-2
            return lr * ((1 - alpha) * 0.5 * (1 + math.cos(math.pi * s)) + alpha)
        return lr * 1e-2
    return schedule


def estimate_log_density(cfg, pde_instance, rng, num_epochs: int = 20000, frequency: int = 100, verbose=True):
    """Train the flow on pde_instance.dataset (offline "0T" trajectories and their tau) and return
    log_density_fn(t, x) (:13-100). Returns (log_density_fn, history of mean losses per interval)."""
    rngs = dict(zip(["model_init", "train"], prng.split(rng, 2)))
    dim = int(cfg.pde_instance.domain_dim)
    model = create_normalizing_flow_fn(pde_instance.distribution_initial_x.logdensity, dim)
    dataset = pde_instance.dataset
    traj_tm = dataset["0T_tm"]                       # [n_time, n_traj, 2d] (time-major)
    dev = traj_tm.device
    params = model.init(rngs["model_init"], 0.0, np.zeros(dim), device=dev)
    flat = params["params"]
    tau_tm = dataset["tau_0T"].permute(1, 0).contiguous().unsqueeze(-1)  # [n_time, n_traj, 1]
    n_time, n_traj = traj_tm.shape[0], traj_tm.shape[1]
    schedule = create_custom_schedule(1e-3, 5000, 15000)
    mu, nu = torch.zeros_like(flat), torch.zeros_like(flat)
    interval_time, interval_sample = 5, 5
    time_base = np.arange(n_time // interval_time) * interval_time
    rng_epoch = prng.split(rngs["train"], num_epochs)
    acc = torch.zeros((), device=dev, dtype=torch.float32)
    history = []
    for epoch in range(num_epochs):
        rng_time, rng_sample = prng.split(rng_epoch[epoch])
        time_index = time_base + int(prng.randint(rng_time, (), 0, interval_time))
        sample_index = prng.permutation(rng_sample, n_traj)[: n_traj // interval_sample]
        si = torch.as_tensor(sample_index, device=dev)
        ti = torch.as_tensor(time_index, device=dev)
        rows = native.gather_subsample(traj_tm, si, ti)        # [n_sel * n_t, 2d]
        times = native.gather_subsample(tau_tm, si, ti)[:, 0]  # the matching tau
        loss, grad = native.realnvp_value_and_grad(model._desc, flat, times, rows[:, :dim])
        native.adam_update(flat, grad, mu, nu, lr=schedule(epoch), b1=0.9, b2=0.999, eps=1e-4, weight_decay=0.0,
                           count=epoch + 1)
        acc += loss
        if (epoch + 1) % frequency == 0:
            mean = float(acc) / frequency
            history.append(mean)
            acc.zero_()
            if verbose:
                print(f"Epoch {epoch + 1}, Loss: {mean}")

    def log_density_fn(t, x):
        return model.apply(params, t, x)

    log_density_fn.history = history
    log_density_fn.params = params
    return log_density_fn
