"""Overdamped FP PDE-consistency residual (methods/consistency_instances/fokker_planck.py).

loss = E_0T|grad V_theta|^2 - 2 E_0T[lap V_theta] + E_0T|grad V*|^2
     + (2 E_T[V_theta] - 2 E_0[V_theta]) / T                                               (:48-55)
loss ground truth = E_0T |grad V* - grad V_theta|^2                                        (:57-58)
with V* = x^T F x / 2. The reference takes lap V as trace(jacfwd(grad V)) under vmap and
differentiates with jax.value_and_grad. Here the Laplacian is d Taylor-mode second derivatives
along the unit directions, evaluated by the same fused MLP residual kernels as the kinetic case
(rows [x | e_k], pdeinv_fp_rows) with the boundary sets weighting V itself; the kernels return
d loss / d theta directly.

test_fn (:66-85): relative L2 error of grad V on fresh initial / terminal samples — the ratio
sqrt(loss-ground-truth / nabla-true) of the same residual evaluated on those samples.
"""
from __future__ import annotations

import functools
import math

import numpy as np
import torch

from core.model import get_model
from methods.consistency_instances.kinetic_fokker_planck import grad_norm64, resolve_model, set_dp_grad_norm
from utils import distributed as dist
from utils import native, prng


def value_and_grad_fn(forward_fn, params, data, rng, pde_instance):
    model = resolve_model(forward_fn)
    if model.residual_kind != "mlp":
        raise NotImplementedError("the overdamped Fokker-Planck residual is defined for V_hypothesis (the "
                                  "reference builds no parametric FP model)")
    d = pde_instance.dim
    F = pde_instance.initial_configuration["F"]
    T = float(pde_instance.total_evolving_time)
    acc, grad = native.residual_fp_mlp(model.dims(d), model.flat(params), data["initial"], data["terminal"],
                                       data["0T"], tilde_F=F, total_time=T, world_scale=1.0 / dist.world_size())
    W = dist.world_size()
    if W > 1:  # the pmap mean (trainer.py:52); per-set boundary means are not pre-scaled
        both = dist.allreduce_sum(torch.cat([acc, grad.double(), grad_norm64(grad, W)]))
        acc, grad, gn = both[: acc.numel()], both[acc.numel():-1].float(), both[-1:] / W
        acc[native.GMM_NACC - 2:native.GMM_NACC] /= W
    out = native.kfp_terms_finalize(acc, grad, 0.0)
    if W > 1:
        set_dp_grad_norm(out, gn)  # the mean over ranks of per-rank norms (trainer.py:44-53)
    return {"loss": out[native.KFP_SLOTS.index("loss")], "grad": model.unflat(grad, d),
            "grad_norm": out[native.KFP_SLOTS.index("grad_norm")],
            "loss ground truth": out[native.KFP_SLOTS.index("loss ground truth")]}


def test_fn(forward_fn, pde_instance, rng):
    """:66-85 — relative L2 error of grad V at 10 000 initial and terminal samples. forward_fn is
    partial(net.apply, params), as ConsistencyBased.test_fn builds it (consistency.py:27-33)."""
    if not isinstance(forward_fn, functools.partial) or not forward_fn.args:
        raise ValueError("test_fn expects partial(forward_fn, params)")
    return relative_gradient_errors(resolve_model(forward_fn.func), forward_fn.args[0], pde_instance, rng)


def relative_gradient_errors(model, params, pde_instance, rng, n: int = 10000):
    d = pde_instance.dim
    F = pde_instance.initial_configuration["F"]
    rng_initial, rng_terminal = prng.split(rng, 2)
    out = {}
    for name, dist_, key in (("initial", pde_instance.distribution_initial, rng_initial),
                             ("terminal", pde_instance.distribution_terminal, rng_terminal)):
        x = dist_.sample(n, key)
        empty = torch.empty((0, d), device=x.device)
        acc, _ = native.residual_fp_mlp(model.dims(d), model.flat(params), empty, empty, x, tilde_F=F,
                                        total_time=float(pde_instance.total_evolving_time))
        a = acc.cpu().numpy()
        out[f"relative error of gradient estimation {name}"] = math.sqrt(
            a[native.GMM_ACC_SLOTS.index("loss_gt")] / a[native.GMM_ACC_SLOTS.index("nabla_true")])
    return out


def create_model_fn(pde_instance):
    """fokker_planck.py:88-97: params = net.init(PRNGKey(11), distribution_initial.sample(1, PRNGKey(1))[0])."""
    cfg = pde_instance.cfg
    if cfg.estimation_mode != "non-parametric":
        raise NotImplementedError("Fokker-Planck: the reference's create_model_fn passes no problem instance to "
                                  "get_model, so only estimation_mode=non-parametric can run")
    net = get_model(cfg, DEBUG=False, pde_instance=pde_instance)
    params = net.init(prng.PRNGKey(11), np.zeros(pde_instance.dim))
    return net, params
