#!/usr/bin/env python3
"""Headline benchmark: particle-steps/s of the hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): kinetic OU, d = 4, 2^21 particles per GPU,
n = 100 Euler–Maruyama steps, T = 2, gamma = 1, Gaussian-init ensemble N(0, I_8), parametric
drift recovery. One timed step = one pass of the hot path over one batch:
  1. the HIP simulator (all n+1 updates; trajectory [n,N,8], tau [n,N] and last [N,8] written to
     HBM — the reference's output contract, sampling_utils.py:52) with the KFP moment sets
     accumulated in the same kernel,
  2. [N > 1 GPUs] one RCCL all-reduce of the fp64 moment sums (the pmap mean, trainer.py:52),
  3. the KFP residual value_and_grad for the current parameters (finalize kernel).
value = particle-updates per second over all ranks = N_total * (n + 1) / step time (weak scaling).

After the timed region (untimed): the drift tilde_F is recovered as the exact minimiser of the
residual from the moments of all timed steps, with Richardson extrapolation over n = 100 / 200
to cancel the O(dt) Euler–Maruyama bias, and the CPU baseline — the NumPy
restatement of sampling_utils.py in oracle/ — is timed on a bounded sample on rank 0.

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from utils import distributed as dist  # noqa: E402
from utils import native  # noqa: E402

METRIC = "particle-steps/sec + achieved HBM GB/s; recovered-drift L2 error"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--particles", type=int, default=1 << 21, help="particles per GPU")
    p.add_argument("--n-steps", type=int, default=100)
    p.add_argument("--dim", type=int, default=4)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-recovery", action="store_true")
    p.add_argument("--cpu-particles", type=int, default=1 << 20)
    return p.parse_args()


def algorithmic_bytes(N, n, d):
    """z0 read 8d + n (traj 8d + tau 4) + last 8d bytes per particle."""
    return N * (8 * d + n * (8 * d + 4) + 8 * d)


def cpu_baseline(F, d, n, T, gamma, N):
    """NumPy restatement of sampling_utils.py:6-52 (+ the moment pass), single thread."""
    from oracle import numpy_ref as nr
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(1)
    except Exception:  # pragma: no cover
        limiter = None
    rng = np.random.default_rng(0)
    dt = np.float32(T / n)
    F32 = F.astype(np.float32)
    z0 = rng.standard_normal((N, 2 * d), dtype=np.float32)
    t0 = time.perf_counter()
    q, p = z0[:, :d].copy(), z0[:, d:].copy()
    tau0 = rng.random(N, dtype=np.float32) * dt
    acc = np.zeros((2 * d, 2 * d))
    for s in range(n + 1):
        h = tau0[:, None] if s == 0 else ((dt - tau0)[:, None] if s == n else dt)
        xi = rng.standard_normal((N, d), dtype=np.float32)
        q, p = nr.update_step(q, p, h, nr.grad_quadratic(F32), np.float32(gamma), xi, np.float32(math.sqrt(2)))
        if s < n:
            z = np.concatenate([q, p], 1)
            acc += z.T.astype(np.float64) @ z.astype(np.float64)
    el = time.perf_counter() - t0
    if limiter is not None:
        limiter.unregister()
    return N * (n + 1) / el, el


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def main():
    a = parse()
    dist.init_from_env("nccl")
    rank, world = dist.rank(), dist.world_size()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    native.lib()

    from example_problems.kinetic_fokker_planck_example_OU import problem_matrix
    from methods.consistency_instances.kinetic_fokker_planck import recover_quadratic_drift

    d, n, N, T, gamma = a.dim, a.n_steps, a.particles, 2.0, 1.0
    dt = T / n
    F = problem_matrix(d)
    pot = dict(kind=native.POT_QUADRATIC, params=F)
    seed = 0x5EED_0001
    poff = rank * N  # global particle ids: rank-count invariant streams
    z0 = native.gaussian_sample(N, torch.zeros(2 * d, device=dev), torch.eye(2 * d, device=dev),
                                seed=seed ^ 0xA5A5, row_offset=poff)
    theta = torch.zeros(d * d + d, device=dev)
    bufs = {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
            "last": torch.empty((N, 2 * d), device=dev),
            "moments": torch.empty((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)}
    mom_total = torch.zeros((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)
    counter = [0]

    def step(n_steps=n, out=bufs, record=None):
        if record is not None:
            record[0].record()
        r = native.sde_simulate(z0, n_steps, T / n_steps, gamma, pot, seed=seed, counter_offset=counter[0],
                                particle_offset=poff, moments=True, out=out)
        if record is not None:
            record[1].record()
        counter[0] = (counter[0] + n_steps + 1) & 0xFFFFFFFF
        mom = dist.allreduce_sum(r["moments"])
        res = native.residual_kfp_quadratic(mom, theta, F, gamma, T)
        return mom, res

    for _ in range(a.warmup):
        mom, _ = step()
        mom_total += mom
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        mom, res = step(record=evs[k])
        mom_total += mom
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    el = dist.allreduce_max_scalar(el, device=dev)
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    kern_ms = dist.allreduce_max_scalar(kern_ms, device=dev)
    ms_per_step = el * 1e3 / a.steps
    total_updates = world * N * (n + 1)
    value = total_updates / (ms_per_step / 1e3)
    bytes_launch = algorithmic_bytes(N, n, d)
    achieved = bytes_launch / (kern_ms / 1e3) / 1e9

    out = {
        "metric": METRIC, "value": value, "unit": "particle-steps/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic: Philox N(0, I) initial ensembles, fresh noise per step",
        "config": {"workload": "C2 kinetic OU d=4: EM simulate (traj+tau+last, fused moments) + KFP residual "
                               "value_and_grad, per GPU 2^21 particles x 101 updates",
                   "dim": d, "n_steps": n, "particles_per_gpu": N, "total_time": T, "gamma": gamma,
                   "parallelism": f"dp{world}"},
        "hbm_GBps": achieved,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                     "kernel": "sde_simulate_kernel<4,QUADRATIC,MOM> (+ its slab reduce)",
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": bytes_launch},
    }
    traffic_file = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(traffic_file) and (d, n, N) == (4, 100, 1 << 21):
        try:
            with open(traffic_file) as f:
                out["roofline"]["traffic"] = json.load(f).get("sde_simulate_C2_bytes_per_launch")
        except Exception:
            pass

    if not a.no_recovery:
        S100, _ = recover_quadratic_drift(mom_total, gamma, T, d)
        mom2 = torch.zeros_like(mom_total)
        for _ in range(a.steps + a.warmup):  # n = 200: moments only (no trajectory needed)
            r2 = native.sde_simulate(z0, 2 * n, T / (2 * n), gamma, pot, seed=seed, counter_offset=counter[0],
                                     particle_offset=poff, traj=False, tau=False, last=False, moments=True)
            counter[0] = (counter[0] + 2 * n + 1) & 0xFFFFFFFF
            mom2 += dist.allreduce_sum(r2["moments"])
        S200, _ = recover_quadratic_drift(mom2, gamma, T, d)
        S_rich = 2 * S200 - S100
        out["drift_err"] = float(np.abs(S_rich - F).max())
        out["drift_err_l2"] = float(np.linalg.norm(S_rich - F) / np.linalg.norm(F))
        out["drift_err_em_n100"] = float(np.abs(S100 - F).max())
        out["drift_recovery"] = ("max |S - tilde_F|, S = K + K^T the exact residual minimiser, Richardson "
                                 f"2*S(n=200) - S(n=100) over {(a.steps + a.warmup) * world * N} trajectories each")
        out["loss"] = float(res[0][0].item())

    if rank == 0 and not a.no_cpu_baseline:
        ups, secs = cpu_baseline(F, d, n, T, gamma, a.cpu_particles)
        out["cpu_baseline"] = {"value": ups, "unit": "particle-steps/s", "cores": 1, "kind": "port",
                               "sample": f"NumPy restatement of sampling_utils.py (oracle/numpy_ref.py update_step) "
                                         f"+ moment pass, fp32, d={d}, {a.cpu_particles} particles x {n + 1} updates, "
                                         f"{secs:.1f} s; host {cpu_model()}, os.cpu_count()={os.cpu_count()}"}
        out["gpu_over_cpu"] = value / ups
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_distributed():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
