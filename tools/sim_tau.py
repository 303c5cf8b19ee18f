import os, sys
ROOT = "/root/repo" if not os.environ.get("GRAFT_REPO_ROOT") else os.environ["GRAFT_REPO_ROOT"]
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))
import torch
from example_problems.kinetic_fokker_planck_example_OU import problem_matrix
from utils import native
d, N, n = 4, 1 << 21, 100
dev = torch.device("cuda")
pot = dict(kind=native.POT_QUADRATIC, params=problem_matrix(d))
z0 = torch.randn(N, 2 * d, device=dev)
bufs = {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
        "last": torch.empty((N, 2 * d), device=dev),
        "moments": torch.empty((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)}
def bench(fn, reps=30):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps
for r in range(2):
    out = []
    for mom in (True, False):
        for tau in (True, False):
            ms = bench(lambda: native.sde_simulate(z0, n, 0.02, 1.0, pot, seed=1, out=bufs, traj=True, tau=tau, moments=mom))
            byt = N * (8 * d + n * (8 * d + (4 if tau else 0)) + 8 * d)
            out.append(f"mom={int(mom)} tau={int(tau)} {ms:.4f} ms {byt / ms / 1e6:.0f} GB/s")
    fill = bench(lambda: bufs["traj"].fill_(1.0))
    out.append(f"fill traj {fill:.4f} ms {bufs['traj'].numel()*4/fill/1e6:.0f} GB/s")
    print(" | ".join(out), flush=True)
