"""KMV PDE-consistency residual (methods/consistency_instances/kinetic_mckean_vlasov.py).

loss = mean_i |mean_j grad Phi_theta(x_i - x_j)|^2 - 2 mean_i mean_j v_i^T Hess Phi_theta v_i
     + 2 mean_i [mean_j Phi_theta(x_i - x_j)] (ds2 log rho + (ds log rho)^2 + gamma ds log rho)
     + mean_i |mean_j grad Phi*(x_i - x_j)|^2                                   (:74-97, pairs per time)
For a general Phi_theta (the non-parametric V_hypothesis of get_model) the pairs are evaluated
as they are in the reference — every (i, j) of each time stamp's particles — in two passes over
pair rows on the MLP path (pdeinv_residual_kmv_mlp: gbar_i = mean_j grad Phi, then the per-pair
adjoint). For the quadratic Phi_theta every pairwise mean is a function of the time stamp's moments, so
the [m, n, n_time, d] pair tensor of :20-23 is replaced by per-time-stamp sums — [count, sum z, sum z z^T] and,
with the per-particle ds/ds2 log rho (the score/log-density evaluation) as weight c, [sum c, sum c x, sum c x x^T] —
  formed inside the McKean-Vlasov simulator from its own rows (pdeinv_sde_simulate_mf_kmv, data["kmv_sums"]), or
  by one read of given rows (pdeinv_kmv_moments_weights; d > 8: pdeinv_moments_batched + pdeinv_kmv_weights);
  final   pdeinv_residual_kmv    — loss, loss ground truth, d loss / d(K, b).
Multi-GPU: with a shared clock (the simulated interacting system, sample_scheme SDE) the
per-time-stamp sums are all-reduced before the finalize (the exact global loss); with
per-rank random time stamps (exact sampler) each rank finalizes and the outputs are averaged,
which is the reference's pmap mean (trainer.py:52).
"""
from __future__ import annotations

import numpy as np
import torch

from core.model import get_model
from methods.consistency_instances.kinetic_fokker_planck import _result, grad_norm64, resolve_model, set_dp_grad_norm
from utils import distributed as dist
from utils import native, prng


def layout(data: dict, d: int):
    """(z, n_sets, n_rows, set_stride, ld) for either the time-major simulator output or the
    reference's flattened [(i, t), 2d] sample order (x_0T.reshape(-1, n_time, d), :14-19)."""
    tau = np.atleast_1d(np.asarray(data["tau_0T"], dtype=np.float64))
    if "0T_tm" in data:
        z = data["0T_tm"]
        n_sets, n_rows = z.shape[0], z.shape[1]
        return z, n_sets, n_rows, n_rows * 2 * d, 2 * d, tau
    z = data["0T"].contiguous()
    n_sets = len(tau)
    n_rows = z.shape[0] // n_sets
    return z, n_sets, n_rows, 2 * d, n_sets * 2 * d, tau


def value_and_grad_fn(forward_fn, params, data, rng, pde_instance):
    model = resolve_model(forward_fn)
    if model.residual_kind == "mlp":
        return _value_and_grad_mlp(model, params, data, pde_instance)
    if model.residual_kind != "quadratic":
        raise NotImplementedError(f"no native KMV residual for model kind '{model.residual_kind}'")
    d = pde_instance.dim
    gamma = float(pde_instance.initial_configuration["gamma_friction"])
    if "kmv_sums" in data:  # formed inside the McKean-Vlasov simulator (pdeinv_sde_simulate_mf_kmv)
        mom, wst = data["kmv_sums"]
    else:
        z, n_sets, n_rows, set_stride, ld, tau = layout(data, d)
        coef = pde_instance.coefficients(tau, z.device)
        if d <= 8:  # one read of the rows for both sets of sums (pdeinv_kmv_moments_weights)
            mom, wst = native.kmv_moments_weights(d, gamma, coef, z, n_sets, n_rows, set_stride, ld)
        else:
            mom = native.moments_batched(z, n_sets, n_rows, 2 * d, set_stride, ld)
            wst, _ = native.kmv_weights(d, gamma, coef, z, n_sets, n_rows, set_stride, ld)
    theta = model.flat(params)
    F = pde_instance.initial_configuration["tilde_F"]
    if data.get("shared_time", False):
        W = dist.world_size()
        parts = [mom.reshape(-1), wst.reshape(-1)]
        if W > 1:  # this rank's own gradient norm (the pmap mean of per-device norms, trainer.py:44-53)
            parts.append(grad_norm64(native.residual_kmv(mom, wst, theta, F, gamma)[1]))
        both = dist.allreduce_sum(torch.cat(parts))
        nm = mom.numel()
        mom = both[:nm].view_as(mom)
        wst = both[nm:nm + wst.numel()].view_as(wst)
        out, grad = native.residual_kmv(mom, wst, theta, F, gamma)
        if W > 1:
            set_dp_grad_norm(out, both[-1:] / W)
    else:
        out, grad = native.residual_kmv(mom, wst, theta, F, gamma)
        if dist.world_size() > 1:
            both = dist.allreduce_mean(torch.cat([out, grad]))
            out, grad = both[: out.numel()], both[out.numel():]
    return _result(out, model.unflat(grad))


def _value_and_grad_mlp(model, params, data, pde_instance):
    """General Phi_theta = V_hypothesis: pairs within this rank's particles (the reference forms them
    within each device's batch, trainer.py:44-53), outputs averaged over ranks."""
    d = pde_instance.dim
    gamma = float(pde_instance.initial_configuration["gamma_friction"])
    z, n_sets, n_rows, set_stride, ld, tau = layout(data, d)
    coef = pde_instance.coefficients(tau, z.device)
    _, ds = native.kmv_weights(d, gamma, coef, z, n_sets, n_rows, set_stride, ld, want_ds=True)
    flat = model.flat(params)
    acc, grad = native.residual_kmv_mlp(model.dims(d), flat, z, n_sets, n_rows, set_stride, ld, ds,
                                        pde_instance.initial_configuration["tilde_F"], gamma)
    out = native.kfp_terms_finalize(acc, grad, 1.0)
    if dist.world_size() > 1:
        both = dist.allreduce_mean(torch.cat([out, grad]))
        out, grad = both[: out.numel()], both[out.numel():]  # incl. grad_norm: the pmap mean, trainer.py:52
    return _result(out, model.unflat(grad, d))


def test_fn(forward_fn, pde_instance, rng):
    return {}  # kinetic_mckean_vlasov.py:123-144 returns {}


def create_model_fn(pde_instance):
    net = get_model(pde_instance.cfg, DEBUG=False, pde_instance=pde_instance)
    params = net.init(prng.PRNGKey(11), np.zeros(pde_instance.dim))
    return net, params
