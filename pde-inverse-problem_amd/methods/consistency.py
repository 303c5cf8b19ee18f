"""ConsistencyBased method (methods/consistency.py of the reference).

Dispatches on cfg.pde_instance.name to the per-instance residual modules (:10-14) and assembles
the training data (:52-122): exact samples, the online SDE simulator, or the offline dataset
subsampled by the native gather kernel (every 5th time stamp from a random phase, a random
fifth of the trajectories).

Deviations (documented in DESIGN.md):
  * tau_0T is only computed for instances that consume it (McKean–Vlasov); the reference always
    calls get_time_sample_ground_truth, which raises NotImplementedError for KOU in its default
    random_time mode;
  * for a quadratic model on an SDE-sampled problem the simulator accumulates the residual's
    moment sets in the same kernel (data["moments"]; McKean–Vlasov: the per-stamp sums, data["kmv_sums"]),
    so the trajectory is never re-read.
"""
from __future__ import annotations

import functools

import numpy as np
import torch

import methods.consistency_instances.fokker_planck as fokker_planck
import methods.consistency_instances.kinetic_fokker_planck as kinetic_fokker_planck
import methods.consistency_instances.kinetic_mckean_vlasov as kinetic_mckean_vlasov
from api import Method
from utils import distributed as dist
from utils import native, prng

# McKean–Vlasov with a quadratic model: trajectories of at least this many bytes (n_steps x batch x 2d x 4) are not
# written; the simulator forms the KMV per-stamp sums from its own rows instead (0: always — C4 step 5.9 -> 5.7 ms,
# DESIGN.md §4.3 r06). A large value restores trajectory + KMV pass (tests compare the two routes).
STAMP_SUMS_MIN_BYTES = 0

INSTANCES = {
    "Fokker-Planck": fokker_planck,
    "Kinetic-Fokker-Planck": kinetic_fokker_planck,
    "Kinetic-McKean-Vlasov": kinetic_mckean_vlasov,
}


class ConsistencyBased(Method):
    def create_model_fn(self):
        if self.cfg.pde_instance.name in INSTANCES:
            net, params = INSTANCES[self.cfg.pde_instance.name].create_model_fn(self.pde_instance)
            self._model = net
            return net, params
        raise NotImplementedError

    def test_fn(self, forward_fn, params, rng):
        forward_fn = functools.partial(forward_fn, params)  # consistency.py:27
        if self.cfg.pde_instance.name in INSTANCES:
            return INSTANCES[self.cfg.pde_instance.name].test_fn(forward_fn=forward_fn, pde_instance=self.pde_instance,
                                                                rng=rng)
        raise NotImplementedError

    def value_and_grad_fn(self, forward_fn, params, rng):
        rng_sample, rng_vg = prng.split(rng, 2)
        data = self.sample_data(rng_sample, forward_fn=forward_fn)
        if self.cfg.pde_instance.name in INSTANCES:
            return INSTANCES[self.cfg.pde_instance.name].value_and_grad_fn(
                forward_fn=forward_fn, params=params, data=data, rng=rng_vg, pde_instance=self.pde_instance)
        raise NotImplementedError

    # ------------------------------------------------------------------------------------
    def sample_data(self, rng, forward_fn=None):
        pi = self.pde_instance
        tr = self.cfg.solver.train
        needs_tau = self.cfg.pde_instance.name == "Kinetic-McKean-Vlasov"
        if pi.sample_mode == "online":
            rng_initial, rng_terminal, rng_0T = prng.split(rng, 3)
            # every rank draws its own full batch, as every pmap device does (trainer.py:47-52):
            # either from a rank-folded key or, where the sampler takes global particle ids,
            # from the shared key at offset rank * batch (interacting systems need the shared key)
            rank = dist.rank()
            fold = (lambda k: prng.fold_in(k, rank)) if dist.world_size() > 1 else (lambda k: k)
            if pi.sample_scheme == "exact":
                rng_initial, rng_terminal, rng_0T = fold(rng_initial), fold(rng_terminal), fold(rng_0T)
                spec = {"random_time": int(tr.batch_size_0T),
                        "grid_time": (int(tr.n_time_stamps), int(tr.sample_per_time))}[tr.sample_mode]
                data = {
                    "initial": pi.distribution_initial.sample(int(tr.batch_size_init), rng_initial),
                    "terminal": pi.distribution_terminal.sample(int(tr.batch_size_terminal), rng_terminal),
                    "0T": pi.sample_ground_truth(rng_0T, spec),
                }
                if needs_tau:
                    data["tau_0T"] = pi.get_time_sample_ground_truth(rng_0T, spec)
            elif pi.sample_scheme == "SDE" and hasattr(pi, "simulate_interacting"):
                # McKean–Vlasov: the interacting system on a shared clock (one tau per time stamp). For a quadratic
                # model the residual needs only per-stamp sums, which the simulator forms from its own rows
                # (data["kmv_sums"], even dim <= 8: no trajectory written or re-read; STAMP_SUMS_MIN_BYTES).
                B = int(tr.sample_per_time)
                model = getattr(forward_fn, "__self__", forward_fn)
                traj_bytes = int(pi.n_steps) * B * 2 * pi.dim * 4
                if (getattr(model, "residual_kind", None) == "quadratic" and pi.dim % 2 == 0 and pi.dim <= 8
                        and traj_bytes >= STAMP_SUMS_MIN_BYTES):
                    _, r = pi.simulate_interacting(rng_0T, B, particle_offset=rank * B, stamp_sums=True)
                    data = {"kmv_sums": (r["kmv_mom"], r["kmv_wst"]), "tau_0T": r["tau_0T"], "shared_time": True}
                else:
                    _, r = pi.simulate_interacting(rng_0T, B, particle_offset=rank * B)
                    data = {"0T_tm": r["traj"], "tau_0T": r["tau"][:, 0].double().cpu().numpy(),
                            "shared_time": True}
            elif pi.sample_scheme == "SDE":
                model = getattr(forward_fn, "__self__", forward_fn)
                fused = getattr(model, "residual_kind", None) == "quadratic" and hasattr(pi, "simulate")
                if fused:
                    B = int(tr.batch_size_0T)
                    _, r = pi.simulate(rng_0T, B, particle_offset=rank * B, traj=False, moments=True)
                    data = {"moments": r["moments"]}
                else:
                    data = {}
                    data["initial"], data["terminal"], data["0T"] = pi.sample_ground_truth(fold(rng_0T),
                                                                                          int(tr.batch_size_0T))
            else:
                raise ValueError("unknown sampling scheme")
        elif pi.sample_mode == "offline":
            data = {"initial": pi.dataset["initial"], "terminal": pi.dataset["terminal"]}
            rng_time, rng_sample = prng.split(rng)
            traj_tm = pi.dataset["0T_tm"]  # [n_time, n_traj, 2d]
            n_time, n_traj = traj_tm.shape[0], traj_tm.shape[1]
            interval_time = 5
            time_index = np.arange(n_time // interval_time) * interval_time + int(prng.randint(rng_time, (), 0, interval_time))
            interval_sample = 5
            sample_index = prng.permutation(rng_sample, n_traj)[: n_traj // interval_sample]
            dev = traj_tm.device
            data["0T"] = native.gather_subsample(traj_tm, torch.as_tensor(sample_index, device=dev),
                                                 torch.as_tensor(time_index, device=dev))
            if needs_tau:
                data["tau_0T"] = pi.dataset["tau_0T"]
        else:
            raise ValueError("unknown sampling mode")
        return data
