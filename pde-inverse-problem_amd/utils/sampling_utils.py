"""The particle simulator (utils/sampling_utils.py of the reference), on the GPU.

`underdamped_langevin_dynamics_scan(q0_p0, n_steps, dt, key, potential_grad, gamma_friction)`
keeps the reference's signature and returns `(last [N,2d], traj [N,n,2d], tau [N,n])`
(sampling_utils.py:25-52). The trajectory is produced time-major ([n, N, 2d], coalesced
stores) and returned as the `permute(1, 0, 2)` view in the reference's particle-major shape;
`traj_time_major` / `simulate` expose the underlying buffer for consumers that stream it.

`key` is a utils.prng.Key (the Philox key of the whole ensemble; particle i uses the global id
particle_offset + i as its counter, so results do not depend on how particles are sharded).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from core.potential import MeanFieldQuadraticPotential, resolve
from utils import native
from utils.prng import Key

SQRT2 = math.sqrt(2.0)


def simulate(q0_p0: torch.Tensor, n_steps: int, dt: float, key: Key, potential_grad, gamma_friction: float,
             *, particle_offset: int = 0, counter_offset: int = 0, noise_scale: float = SQRT2,
             random_shift: bool = True, noise: Optional[torch.Tensor] = None,
             shift_u: Optional[torch.Tensor] = None, traj: bool = True, tau: bool = True,
             last: bool = True, moments: bool = False, out: Optional[dict] = None) -> dict:
    """Time-major simulator call. Returns dict(traj [n,N,2d], tau [n,N], last [N,2d], moments [3,L])."""
    pot = resolve(potential_grad)
    if isinstance(pot, MeanFieldQuadraticPotential):
        from utils.mean_field import simulate_mean_field
        return simulate_mean_field(q0_p0, n_steps, dt, key, pot, gamma_friction, particle_offset=particle_offset,
                                   counter_offset=counter_offset, noise_scale=noise_scale,
                                   random_shift=random_shift, noise=noise, traj=traj, tau=tau)
    return native.sde_simulate(q0_p0, n_steps, dt, gamma_friction, pot.native_desc(), seed=key.seed,
                               counter_offset=counter_offset, particle_offset=particle_offset,
                               noise_scale=noise_scale, random_shift=random_shift, noise=noise,
                               shift_u=shift_u, traj=traj, tau=tau, last=last, moments=moments, out=out)


def underdamped_langevin_dynamics_scan(q0_p0, n_steps, dt, key, potential_grad, gamma_friction, **kw):
    """sampling_utils.py:25-52: returns (last [N,2d], traj [N,n,2d], tau [N,n])."""
    r = simulate(q0_p0, int(n_steps), float(dt), key, potential_grad, float(gamma_friction), **kw)
    return r["last"], r["traj"].permute(1, 0, 2), r["tau"].permute(1, 0)
