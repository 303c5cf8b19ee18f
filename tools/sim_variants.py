"""Time simulator variants on one box (d=4 KOU, 2^21 particles, n=100): with / without the fused
moments and the tau rows, plus a plain streaming-store kernel of the same byte count (torch fill)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))
import torch  # noqa: E402

from example_problems.kinetic_fokker_planck_example_OU import problem_matrix  # noqa: E402
from utils import native  # noqa: E402

d, N, n = 4, 1 << 21, 100
dev = torch.device("cuda")
F = problem_matrix(d)
pot = dict(kind=native.POT_QUADRATIC, params=F)
z0 = torch.randn(N, 2 * d, device=dev)
traj = torch.empty((n, N, 2 * d), device=dev)
tau = torch.empty((n, N), device=dev)
last = torch.empty((N, 2 * d), device=dev)
mom = torch.empty((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)


def bench(fn, reps=20):
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


byt = N * (8 * d + n * (8 * d + 4) + 8 * d)
byt_notau = N * (8 * d + n * 8 * d + 8 * d)
for name, flags, nb in [("traj+tau+last+moments", dict(traj=True, tau=True, moments=True), byt),
                        ("traj+tau+last", dict(traj=True, tau=True, moments=False), byt),
                        ("traj+last (no tau)", dict(traj=True, tau=False, moments=False), byt_notau),
                        ("last+moments only", dict(traj=False, tau=False, moments=True), N * 16 * d)]:
    bufs = {"traj": traj, "tau": tau, "last": last, "moments": mom}
    ms = bench(lambda: native.sde_simulate(z0, n, 0.02, 1.0, pot, seed=1, out=bufs, **flags))
    print(f"{name:28s} {ms:7.3f} ms  {nb / ms / 1e6:8.1f} GB/s")
big = torch.empty(byt // 4, device=dev)
ms = bench(lambda: big.fill_(1.0))
print(f"{'torch fill (same bytes)':28s} {ms:7.3f} ms  {byt / ms / 1e6:8.1f} GB/s")
src = torch.empty(byt // 8, device=dev)
dst = torch.empty(byt // 8, device=dev)
ms = bench(lambda: dst.copy_(src))
print(f"{'torch copy (R+W same bytes)':28s} {ms:7.3f} ms  {byt / ms / 1e6:8.1f} GB/s")

# C3-shaped GMM simulator (d = 4, K = 8, 2^22 particles) and the d = 8 GMM of C5
from example_problems.kinetic_fokker_planck_example_GMM import gmm_means  # noqa: E402
from utils import prng  # noqa: E402

for dg, Ng in [(4, 1 << 22), (8, 1 << 22)]:
    mus = gmm_means(dg, 8, prng.PRNGKey(2))
    potg = dict(kind=native.POT_GMM, params=mus, n_centers=8, sigma=1.0)
    zg = torch.randn(Ng, 2 * dg, device=dev)
    bufs = {"traj": torch.empty((n, Ng, 2 * dg), device=dev), "tau": torch.empty((n, Ng), device=dev),
            "last": torch.empty((Ng, 2 * dg), device=dev)}
    nbg = Ng * (8 * dg + n * (8 * dg + 4) + 8 * dg)
    ms = bench(lambda: native.sde_simulate(zg, n, 0.02, 0.5, potg, seed=1, out=bufs))
    print(f"{'GMM d=%d K=8 2^22' % dg:28s} {ms:7.3f} ms  {nbg / ms / 1e6:8.1f} GB/s")
    del bufs, zg
    torch.cuda.empty_cache()
