"""McKean–Vlasov particle system drivers.

The interaction drift on particle i is mean_j grad Phi*(x_i - x_j) = A (x_i - xbar) for the
quadratic Phi* (kinetic_mckean_vlasov.py:20-23; README.md:55-80), so every update needs xbar, the
mean of the whole ensemble (all ranks) before it. Two drivers, the same system:

* exchange="fused" (default): averaged over the particles the drift vanishes, so the mean obeys
  vbar' = (1 - gamma h) vbar + sqrt(h) ns xibar_s, xbar' = xbar + h vbar' exactly, with xibar_s the
  mean of update s's noise — a function of particle ids and the RNG stream only. One native pass
  (pdeinv_mf_sums) sums z0 and every update's noise, ONE all-reduce makes them global, a one-block
  kernel unrolls the mean path, and the simulator then runs all n+1 updates of each particle in
  registers (one collective per simulate instead of one per update).
* exchange="per_update": n+1 pdeinv_mf_step launches, each followed by one all-reduce of
  [count, sum x] (d+1 doubles) — xbar from the fp32 states themselves. Kept as the cross-check of the
  closed form (tests/test_gpu_meanfield.py) and as the driver for interactions without a closed-form
  mean.

The reference never simulates this system (it samples the equivalent OU law exactly); with a centred
ensemble the two laws coincide (tests check it).
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import numpy as np
import torch

from utils import distributed as dist
from utils import native
from utils.prng import Key


def stamp_times(seed: int, counter_offset: int, n_steps: int, dt: float, random_shift: bool = True) -> np.ndarray:
    """The shared-clock time stamps tau_k = tau0 + k dt (fp32, bit-identical to the simulator's
    tau rows) computed on the host: tau0 = u dt with u from Philox4x32-10 at counter
    (UINT64_MAX, counter_offset, 0x80000000) (include/pdeinv.h stream layout). Lets callers build
    the per-stamp coefficient rows without waiting for the device."""
    from utils.prng import philox4x32_10
    dt32 = np.float32(dt)
    if random_shift:
        c0 = philox4x32_10((0xFFFFFFFF, 0xFFFFFFFF, counter_offset, 0x80000000), (seed, seed >> 32))[0]
        tau0 = np.float32(np.float32(c0 >> 8) * np.float32(2.0 ** -24)) * dt32
    else:
        tau0 = np.float32(0.0)
    k = np.arange(n_steps, dtype=np.float32)
    return (np.float32(tau0) + (k * dt32).astype(np.float32)).astype(np.float32)


def simulate_mean_field(q0_p0: torch.Tensor, n_steps: int, dt: float, key: Key, potential, gamma: float, *,
                        particle_offset: int = 0, counter_offset: int = 0, noise_scale: float = math.sqrt(2.0),
                        random_shift: bool = True, noise: Optional[torch.Tensor] = None, traj: bool = True,
                        tau: bool = True, exchange: str = "fused", out: Optional[dict] = None,
                        kmv_coef: Optional[torch.Tensor] = None, kmv_gamma: float = 1.0) -> dict:
    """Returns {"last" [N, 2d], "xsum" [n+2, 1+d] fp64 ([count, sum x] before each update and after the
    last, global over ranks), "traj" [n, N, 2d] time-major, "tau" [n, N]}. `out` may hold preallocated
    "traj" / "tau" / "last" buffers (fused path).

    exchange="per_update": xsum holds the MEASURED sums, recomputed from the fp32 states after every
    update (one all-reduce each). exchange="fused" (default): xsum = count * the closed-form fp64 mean
    path of DESIGN.md §4.3 (also returned as "xbar"), the model quantity the drift uses — equal to the
    measured ensemble mean in exact arithmetic and to fp32 rounding in practice (tested to 1e-6), but not
    a measurement; take moments of "traj" / "last" for the measured means.

    kmv_coef [n, 3d + 2 + 2d^2] (fused path, Philox noise): the simulator also forms the quadratic-Phi KMV residual's
    per-stamp sums of its own trajectory rows (pdeinv_sde_simulate_mf_kmv) — returned as "kmv_mom" / "kmv_wst"
    (rank-local), with traj=False the trajectory is never written at all."""
    N, m = q0_p0.shape
    d = m // 2
    dev = q0_p0.device
    desc, keep = native.mf_desc(N, d, n_steps, dt, gamma, potential.A, seed=key.seed, counter_offset=counter_offset,
                                particle_offset=particle_offset, noise_scale=noise_scale,
                                random_shift=random_shift, noise=noise)
    z0 = q0_p0.contiguous()
    if exchange == "fused":
        res = {} if out is None else out
        if traj and "traj" not in res:
            res["traj"] = torch.empty((n_steps, N, m), device=dev, dtype=torch.float32)
        if tau and "tau" not in res:
            res["tau"] = torch.empty((n_steps, N), device=dev, dtype=torch.float32)
        if "last" not in res:
            res["last"] = torch.empty((N, m), device=dev, dtype=torch.float32)
        sums = dist.allreduce_sum(native.mf_sums(desc, z0))  # the one collective of the simulate
        xbar, xs = native.mf_mean_path(desc, sums)
        desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
        if kmv_coef is not None:
            res["kmv_mom"], res["kmv_wst"] = native.sde_simulate_mf_kmv(
                desc, z0, res.get("traj") if traj else None, res.get("tau") if tau else None, res["last"],
                kmv_gamma, kmv_coef)
        else:
            native.sde_simulate_desc(desc, z0, res.get("traj") if traj else None, res.get("tau") if tau else None,
                                     res["last"])
        del keep
        res["xsum"] = xs
        res["xbar"] = xbar
        return res
    if exchange != "per_update":
        raise ValueError(f"exchange must be 'fused' or 'per_update', got {exchange!r}")
    states = torch.empty((n_steps if traj else 2, N, m), device=dev, dtype=torch.float32)
    taus = torch.empty((n_steps, N), device=dev, dtype=torch.float32) if tau else None
    last = torch.empty((N, m), device=dev, dtype=torch.float32)
    xs = torch.empty((n_steps + 2, 1 + d), device=dev, dtype=torch.float64)  # [count, sum x] per update
    xs[0] = native.moments(z0)[: 1 + d]
    dist.allreduce_sum(xs[0])
    ws = native.mf_workspace(desc, dev)
    for s in range(n_steps + 1):
        zin = z0 if s == 0 else states[(s - 1) if traj else (s - 1) % 2]
        zout = last if s == n_steps else states[s if traj else s % 2]
        native.mf_step(desc, s, zin, zout, taus[s] if (tau and s < n_steps) else None, xs[s], ws, xs[s + 1])
        dist.allreduce_sum(xs[s + 1])
    del keep
    out = {"last": last, "xsum": xs[: n_steps + 2]}
    if traj:
        out["traj"] = states
    if tau:
        out["tau"] = taus
    return out
