"""A/B timing of simulator variants in ONE process (interleaved rounds, cdna guide §5.4 rule 24)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))
import numpy as np, torch
from utils import native

d, n, N = int(os.environ.get("D", 4)), 100, 1 << 21
F = np.random.default_rng(2217).standard_normal((d, d + 1)); F = F @ F.T
pot = dict(kind=native.POT_QUADRATIC, params=F)
z0 = native.gaussian_sample(N, torch.zeros(2 * d, device="cuda"), torch.eye(2 * d, device="cuda"), seed=1)
bufs = {"traj": torch.empty((n, N, 2 * d), device="cuda"), "tau": torch.empty((n, N), device="cuda"),
        "last": torch.empty((N, 2 * d), device="cuda"),
        "moments": torch.empty((3, native.moment_len(2 * d)), device="cuda", dtype=torch.float64)}
variants = []
for mode in (0, 1, 2):
    for mom in (True, False):
        variants.append((f"store{mode}_mom{int(mom)}", mode, mom, True))
variants.append(("notraj_mom1", 2, True, False))
variants.append(("notraj_mom0", 2, False, False))
times = {v[0]: [] for v in variants}
for rnd in range(6):
    for name, mode, mom, traj in variants:
        os.environ["PDEINV_STORE_MODE"] = str(mode)
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        native.sde_simulate(z0, n, 0.02, 1.0, pot, seed=7, moments=mom, traj=traj, tau=traj, out=bufs)
        s.record()
        for _ in range(3):
            native.sde_simulate(z0, n, 0.02, 1.0, pot, seed=7, moments=mom, traj=traj, tau=traj, out=bufs)
        e.record(); torch.cuda.synchronize()
        if rnd: times[name].append(s.elapsed_time(e) / 3)
B = N * (8 * d + n * (8 * d + 4) + 8 * d)
for k, v in times.items():
    ms = float(np.median(v))
    print(f"{k:14s} {ms:7.3f} ms  {B / ms / 1e6:8.1f} GB/s(alg)  {N * (n + 1) / ms / 1e9:7.2f} Gupd/s")
