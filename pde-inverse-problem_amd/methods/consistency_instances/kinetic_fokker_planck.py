"""KFP PDE-consistency residual (methods/consistency_instances/kinetic_fokker_planck.py).

loss = E_0T|grad V_theta|^2 - 2 E_0T[v^T Hess V_theta v] + 2 gamma E_0T[grad V_theta . v]
     + E_0T|grad V*|^2 + (2/T)(E_term - E_init)[grad V_theta . v]                     (:33-50)
loss ground truth = E_0T |grad V* - grad V_theta|^2                                      (:52-58)

The reference differentiates this with jax.value_and_grad over vmapped autodiff. Here each
model kind has a fused native residual that returns the loss terms AND d loss / d theta:
  * quadratic V_theta = x.(xK + b): all terms are moments of z (moments kernel, or fused into
    the simulator) + an O(d^3) finalize kernel;
  * GMM V_theta: one fused per-sample kernel with the analytic softmax adjoint.
Multi-GPU: the fp64 pre-finalize sums are all-reduced (RCCL) — the pmap mean of trainer.py:52.
"""
from __future__ import annotations

import numpy as np
import torch
from scipy.linalg import solve_sylvester

from core.model import get_model
from utils import distributed as dist
from utils import native, prng


def resolve_model(forward_fn):
    """The reference passes `net.apply`; accept that bound method or the model itself."""
    owner = getattr(forward_fn, "__self__", None)
    model = owner if owner is not None and hasattr(owner, "residual_kind") else forward_fn
    if not hasattr(model, "residual_kind"):
        raise NotImplementedError("forward_fn must be a pdeinv model (or its .apply): the residual is a "
                                  "fused native kernel per model family, there is no autodiff fallback")
    return model


def grad_norm64(grad: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """[1] fp64: scale * ||grad|| (compute_pytree_norm of one rank's gradient)."""
    return (torch.linalg.vector_norm(grad.double()) * scale).reshape(1)


def set_dp_grad_norm(out: torch.Tensor, gn: torch.Tensor) -> torch.Tensor:
    """Data-parallel grad_norm as the reference reports it: under pmap every device returns the norm of
    ITS OWN gradient and trainer.py:44-53 averages all outputs over devices, so grad_norm is the mean
    over ranks of per-rank norms (not the norm of the mean gradient). gn: that mean, all-reduced."""
    out[native.KFP_SLOTS.index("grad_norm")] = gn.to(out.dtype)
    return out


def _result(out: torch.Tensor, grad_tree) -> dict:
    return {"loss": out[native.KFP_SLOTS.index("loss")], "grad": grad_tree,
            "grad_norm": out[native.KFP_SLOTS.index("grad_norm")],
            "loss ground truth": out[native.KFP_SLOTS.index("loss ground truth")]}


def kfp_moments(data: dict) -> torch.Tensor:
    """[3, L] fp64 sums for (initial, 0T, terminal); fused-simulator moments are used as is."""
    if data.get("moments") is not None:
        return data["moments"]
    return torch.stack([native.moments(data["initial"]), native.moments(data["0T"]),
                        native.moments(data["terminal"])])


def value_and_grad_fn(forward_fn, params, data, rng, pde_instance):
    model = resolve_model(forward_fn)
    ic = pde_instance.initial_configuration
    gamma = float(ic["gamma_friction"])
    T = float(pde_instance.total_evolving_time)
    if model.residual_kind == "quadratic":
        if "tilde_F" not in ic:
            raise NotImplementedError("quadratic model needs a quadratic true potential (tilde_F)")
        theta = model.flat(params)
        mom = kfp_moments(data).contiguous()
        W = dist.world_size()
        if W > 1:  # this rank's own gradient norm rides on the moment all-reduce
            _, g_loc = native.residual_kfp_quadratic(mom, theta, ic["tilde_F"], gamma, T)
            both = dist.allreduce_sum(torch.cat([mom.reshape(-1), grad_norm64(g_loc)]))
            mom, gn = both[:-1].view_as(mom), both[-1:] / W
        else:
            mom = dist.allreduce_sum(mom)
        out, grad = native.residual_kfp_quadratic(mom, theta, ic["tilde_F"], gamma, T)
        if W > 1:
            set_dp_grad_norm(out, gn)
        return _result(out, model.unflat(grad))
    if model.residual_kind == "gmm":
        mus_true = pde_instance.potential.mus
        n_i, n_t, n_0 = data["initial"].shape[0], data["terminal"].shape[0], data["0T"].shape[0]
        desc = native.kfp_gmm_desc(model.dim, model.n_Gaussians, mus_true, gamma, T, n_i, n_t, n_0,
                                   sigma=model.sigma, sigma_true=pde_instance.potential.sigma,
                                   world_scale=1.0 / dist.world_size())
        acc = native.residual_kfp_gmm(desc, data["initial"], data["terminal"], data["0T"], params["params"]["mus"])
        W = dist.world_size()
        if W > 1:
            # this rank's own finalize (its sums un-scaled, a world_scale = 1 descriptor) for its grad norm
            loc = acc * W  # c-weighted sums (loss slots and the mu adjoint) carry world_scale = 1/W ...
            loc[native.GMM_NACC - 2:native.GMM_NACC] = acc[native.GMM_NACC - 2:native.GMM_NACC]  # ... the per-set means do not
            desc1 = native.kfp_gmm_desc(model.dim, model.n_Gaussians, mus_true, gamma, T, n_i, n_t, n_0,
                                        sigma=model.sigma, sigma_true=pde_instance.potential.sigma, world_scale=1.0)
            _, g_loc = native.residual_kfp_gmm_finalize(desc1, loc)
            both = dist.allreduce_sum(torch.cat([acc, grad_norm64(g_loc)]))
            acc, gn = both[:-1], both[-1:] / W
            acc[native.GMM_NACC - 2:native.GMM_NACC] /= W  # the per-set means of the boundary terms are not pre-scaled
        else:
            acc = dist.allreduce_sum(acc)
        out, grad = native.residual_kfp_gmm_finalize(desc, acc)
        if W > 1:
            set_dp_grad_norm(out, gn)
        return _result(out, {"params": {"mus": grad}})
    if model.residual_kind == "mlp":
        d = pde_instance.dim
        if "tilde_F" in ic:
            true_kind, true_params, sigma_true = native.POT_QUADRATIC, ic["tilde_F"], 1.0
        else:
            true_kind, true_params, sigma_true = native.POT_GMM, pde_instance.potential.mus, pde_instance.potential.sigma
        acc, grad = native.residual_kfp_mlp(model.dims(d), model.flat(params), data["initial"], data["terminal"],
                                            data["0T"], true_kind=true_kind, true_params=true_params, gamma=gamma,
                                            total_time=T, sigma_true=sigma_true, world_scale=1.0 / dist.world_size())
        W = dist.world_size()
        if W > 1:  # grad is pre-scaled by 1/W: this rank's own gradient is W * grad
            both = dist.allreduce_sum(torch.cat([acc, grad.double(), grad_norm64(grad, W)]))
            acc, grad, gn = both[: acc.numel()], both[acc.numel():-1].float(), both[-1:] / W
            acc[native.GMM_NACC - 2:native.GMM_NACC] /= W
        out = native.kfp_terms_finalize(acc, grad, gamma)
        if W > 1:
            set_dp_grad_norm(out, gn)
        return _result(out, model.unflat(grad, d))
    raise NotImplementedError(f"no native KFP residual for model kind '{model.residual_kind}'")


def recover_quadratic_drift(moments3, gamma: float, T: float, d: int):
    """Exact minimiser (S = K + K^T, b) of the quadratic-model loss given the three moment sets:
    d loss/db = 0 gives b = -S E[x] + c, and d loss/dS = 0 the Lyapunov equation S C + C S = R with
    C = Cov_0T(x). What Adam on this convex quadratic converges to (main.py:11-29)."""
    mom = np.asarray(moments3.detach().cpu() if torch.is_tensor(moments3) else moments3, dtype=np.float64)
    m = 2 * d

    def unpack(v):
        n = v[0]
        mean = v[1:1 + m] / n
        M = np.zeros((m, m))
        M[np.triu_indices(m)] = v[1 + m:]
        M = M + M.T - np.diag(np.diag(M))
        return mean, M / n

    ei, Mi = unpack(mom[0])
    e0, M0 = unpack(mom[1])
    et, Mt = unpack(mom[2])
    ex, ev = e0[:d], e0[d:]
    Mxx, Mxv, Mvv = M0[:d, :d], M0[:d, d:], M0[d:, d:]
    c = -gamma * ev - (et[d:] - ei[d:]) / T
    C = Mxx - np.outer(ex, ex)
    R = (2 * Mvv - gamma * (Mxv.T + Mxv) + ((Mi[:d, d:].T + Mi[:d, d:]) - (Mt[:d, d:].T + Mt[:d, d:])) / T
         - (np.outer(c, ex) + np.outer(ex, c)))
    S = solve_sylvester(C, C, R)
    S = 0.5 * (S + S.T)
    return S, -S @ ex + c


def recover_drift_richardson(z0, F, gamma: float, T: float, n: int, seed: int, passes: int, counter_offset: int = 0,
                             particle_offset: int = 0, base=None, base_passes: int = 0):
    """Recovered drift of the kinetic OU problem (BASELINE metric, third part): S = K + K^T, the exact
    minimiser of the quadratic-model loss (recover_quadratic_drift — what Adam converges to on this convex
    loss, main.py:11-29 / kinetic_fokker_planck_example_OU.py:209-220), from the moments of `passes`
    Philox ensembles simulated at n, 2n and 4n EM steps (moments only, fused into the simulator).
    Semi-implicit EM is weak order 1 with a smooth expansion in dt, so two Richardson levels
    (8 S(4n) - 6 S(2n) + S(n)) / 3 cancel the dt and dt^2 bias; one level 2 S(2n) - S(n) is returned too.
    `base` (+ `base_passes`): moment sums already accumulated at n (bench.py's timed steps). Moments are
    all-reduced over ranks, so every rank returns the same S. Returns a dict with S_rich, S_rich1, S_n
    and the next free counter."""
    d = F.shape[0]
    pot = dict(kind=native.POT_QUADRATIC, params=F)
    ctr = int(counter_offset)
    S = {}
    for mult in (1, 2, 4):
        nn = mult * n
        mom = base.clone() if (mult == 1 and base is not None) else None
        todo = passes - (base_passes if mult == 1 and base is not None else 0)
        for _ in range(max(0, todo)):
            r = native.sde_simulate(z0, nn, T / nn, gamma, pot, seed=seed, counter_offset=ctr,
                                    particle_offset=particle_offset, traj=False, tau=False, last=False, moments=True)
            ctr = (ctr + nn + 1) & 0xFFFFFFFF
            m = dist.allreduce_sum(r["moments"])
            mom = m.clone() if mom is None else mom.add_(m)
        S[mult], _ = recover_quadratic_drift(mom, gamma, T, d)
    return {"S_rich": (8 * S[4] - 6 * S[2] + S[1]) / 3, "S_rich1": 2 * S[2] - S[1], "S_n": S[1], "counter": ctr}


def test_fn(forward_fn, pde_instance, rng):
    return {}  # kinetic_fokker_planck.py:72-92 returns {}


def create_model_fn(pde_instance):
    """kinetic_fokker_planck.py:96-104: params = net.init(PRNGKey(11), x)."""
    net = get_model(pde_instance.cfg, DEBUG=False, pde_instance=pde_instance)
    params = net.init(prng.PRNGKey(11), np.zeros(pde_instance.dim))
    return net, params
