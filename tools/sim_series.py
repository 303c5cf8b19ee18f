"""Time series of the C2 simulator launch on one box: blocks of back-to-back launches (fused
moments on / off) and a torch fill of the trajectory buffer, for ~SECONDS seconds, one line per
block. Shows whether the launch time drifts within a process (clock ramp, page-table warm-up) or
is fixed per box. Usage: python tools/sim_series.py [SECONDS] [fresh]  ('fresh' reallocates the
trajectory buffer for every block)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))
import torch  # noqa: E402

from example_problems.kinetic_fokker_planck_example_OU import problem_matrix  # noqa: E402
from utils import native  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
fresh = len(sys.argv) > 2 and sys.argv[2] == "fresh"
d, N, n = 4, 1 << 21, 100
dev = torch.device("cuda")
pot = dict(kind=native.POT_QUADRATIC, params=problem_matrix(d))
z0 = torch.randn(N, 2 * d, device=dev)


def alloc():
    return {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
            "last": torch.empty((N, 2 * d), device=dev),
            "moments": torch.empty((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)}


bufs = alloc()
byt = N * (8 * d + n * (8 * d + 4) + 8 * d)


def block(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


t0 = time.perf_counter()
k = 0
while time.perf_counter() - t0 < secs:
    if fresh:
        del bufs
        torch.cuda.empty_cache()
        bufs = alloc()
    a = block(lambda: native.sde_simulate(z0, n, 0.02, 1.0, pot, seed=1, out=bufs, moments=True))
    b = block(lambda: native.sde_simulate(z0, n, 0.02, 1.0, pot, seed=1, out=bufs, moments=False))
    c = block(lambda: bufs["traj"].fill_(1.0))
    fill_gbps = bufs["traj"].numel() * 4 / c / 1e6
    print(f"t={time.perf_counter() - t0:6.2f}s blk={k} mom {a:.4f} ms ({byt / a / 1e6:.0f} GB/s) | "
          f"nomom {b:.4f} ms ({byt / b / 1e6:.0f} GB/s) | fill {fill_gbps:.0f} GB/s", flush=True)
    k += 1
