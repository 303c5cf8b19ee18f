"""Does the C2 simulator launch time depend on WHERE its output buffers live? Allocates several
buffer sets in one process and times the same launch on each, round-robin, printing the buffers'
virtual addresses (mod 2 MiB / 64 MiB) next to the times. Usage: python tools/sim_alloc.py [SETS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))
import torch  # noqa: E402

from example_problems.kinetic_fokker_planck_example_OU import problem_matrix  # noqa: E402
from utils import native  # noqa: E402

n_sets = int(sys.argv[1]) if len(sys.argv) > 1 else 4
d, N, n = 4, 1 << 21, 100
dev = torch.device("cuda")
pot = dict(kind=native.POT_QUADRATIC, params=problem_matrix(d))
z0 = torch.randn(N, 2 * d, device=dev)
byt = N * (8 * d + n * (8 * d + 4) + 8 * d)
mode = os.environ.get("SIM_ALLOC_MODE", "separate")


def alloc():
    if mode == "one":  # traj, tau, last carved from one allocation (traj first)
        m = 2 * d
        flat = torch.empty(n * N * m + n * N + N * m, device=dev)
        return {"traj": flat[: n * N * m].view(n, N, m), "tau": flat[n * N * m: n * N * m + n * N].view(n, N),
                "last": flat[n * N * m + n * N:].view(N, m),
                "moments": torch.empty((3, native.moment_len(m)), device=dev, dtype=torch.float64)}
    return {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
            "last": torch.empty((N, 2 * d), device=dev),
            "moments": torch.empty((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)}


sets = [alloc() for _ in range(n_sets)]


def block(b, reps=20, mom=True):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        native.sde_simulate(z0, n, 0.02, 1.0, pot, seed=1, out=b, moments=mom)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for b in sets:  # warm every set once
    block(b, 3)
variants = os.environ.get("SIM_ALLOC_VARIANTS", "")  # e.g. "PDEINV_SIM_REMAP=0,PDEINV_SIM_REMAP=1"
variants = [v.split("=") for v in variants.split(",")] if variants else [None]
for rnd in range(3):
    for k, b in enumerate(sets):
        for var in variants:
            if var:
                os.environ[var[0]] = var[1]
            t = block(b)
            tr, ta = b["traj"].data_ptr(), b["tau"].data_ptr()
            tag = "=".join(var) if var else ""
            print(f"round {rnd} set {k} {tag}: {t:.4f} ms ({byt / t / 1e6:.0f} GB/s)  traj {tr:#x} "
                  f"(mod2M {tr % (1 << 21):#x}, mod64M {tr % (1 << 26):#x})  tau {ta:#x} (mod2M {ta % (1 << 21):#x})",
                  flush=True)
