"""Time the C2 simulator launch (d=4 KOU, 2^21 particles, n=100) with and without fused moments;
one line per call. Used with PDEINV_SIM_LDS_PAD (occupancy study) and PDEINV_LIBRARY (A/B builds)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))
import torch  # noqa: E402

from example_problems.kinetic_fokker_planck_example_OU import problem_matrix  # noqa: E402
from utils import native  # noqa: E402

d, N, n = 4, 1 << 21, 100
if len(sys.argv) > 1:
    N = int(sys.argv[1])
dev = torch.device("cuda")
pot = dict(kind=native.POT_QUADRATIC, params=problem_matrix(d))
z0 = torch.randn(N, 2 * d, device=dev)
bufs = {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
        "last": torch.empty((N, 2 * d), device=dev),
        "moments": torch.empty((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)}
byt = N * (8 * d + n * (8 * d + 4) + 8 * d)


def bench(fn, reps=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


out = []
for mom in (True, False):
    ms = bench(lambda: native.sde_simulate(z0, n, 0.02, 1.0, pot, seed=1, out=bufs, traj=True, tau=True, moments=mom))
    out.append(f"mom={int(mom)} {ms:.4f} ms {byt / ms / 1e6:.0f} GB/s")
print(f"pad={os.environ.get('PDEINV_SIM_LDS_PAD', '0')} N={N} " + " | ".join(out), flush=True)
