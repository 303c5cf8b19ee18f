"""CPU baseline for bench.py — the NumPy restatement of the simulator (TEST/BENCH INFRASTRUCTURE).

Only bench.py's cpu_baseline leg uses this module; the product package never does. The loop is
the reference's kinetic Langevin scan (utils/sampling_utils.py:6-52: tau0 shift, n-1 dt steps,
final dt - tau0 step, sqrt(2) noise) vectorised over particles with a Python loop over steps,
in fp32, plus the moment pass the KFP residual consumes (kinetic_fokker_planck.py:33-58) —
the same work as one bench step of config C2, on a bounded sample of particles.

Two forms: one process in-process (NumPy elementwise is single-threaded), and
P processes, each a fresh interpreter on its own particle shard, started together; the
multi-process rate is all shards' particle-updates over (last end - first start).

CLI (one shard): python -m oracle.cpu_baseline --dim 4 --particles N --steps n --F f00,f01,... --start T0
prints JSON {"t0": ..., "t1": ...} (wall clock) after waiting until T0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def simulate(F, d, n, T, gamma, N, seed=0):
    """One C2 step on N particles; returns elapsed seconds of the loop."""
    from oracle import numpy_ref as nr

    rng = np.random.default_rng(seed)
    dt = np.float32(T / n)
    F32 = np.asarray(F, dtype=np.float32)
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
    return time.perf_counter() - t0


def _limit_threads():
    try:
        from threadpoolctl import threadpool_limits
        return threadpool_limits(1)
    except Exception:  # pragma: no cover
        return None


def single(F, d, n, T, gamma, N):
    """particle-updates/s of one process (BLAS pinned to one thread)."""
    lim = _limit_threads()
    try:
        el = simulate(F, d, n, T, gamma, N)
    finally:
        if lim is not None:
            lim.unregister()
    return N * (n + 1) / el, el


def multi(F, d, n, T, gamma, N_per, P, timeout=300):
    """P shard processes started together; returns (particle-updates/s, wall seconds)."""
    F_arg = ",".join(repr(float(v)) for v in np.asarray(F, dtype=np.float64).ravel())
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    start = time.time() + 4.0 + 0.05 * P  # every shard imports NumPy before the common start
    procs = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_baseline", "--dim", str(d), "--particles", str(N_per),
                               "--steps", str(n), "--F", F_arg, "--total-time", str(T), "--gamma", str(gamma), "--seed", str(k),
                               "--start", repr(start)], cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True)
             for k in range(P)]
    spans = []
    for pr in procs:
        out, _ = pr.communicate(timeout=timeout)
        if pr.returncode != 0:
            raise RuntimeError(f"cpu_baseline shard failed with {pr.returncode}")
        spans.append(json.loads(out.strip().splitlines()[-1]))
    wall = max(s["t1"] for s in spans) - min(s["t0"] for s in spans)
    return P * N_per * (n + 1) / wall, wall


def _main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=4)
    ap.add_argument("--particles", type=int, required=True)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--F", required=True, help="tilde_F, d*d comma-separated (row-major)")
    ap.add_argument("--total-time", type=float, default=2.0)
    ap.add_argument("--gamma", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--start", type=float, default=0.0)
    a = ap.parse_args()
    F = np.array([float(v) for v in a.F.split(",")]).reshape(a.dim, a.dim)
    lim = _limit_threads()
    while time.time() < a.start:
        time.sleep(0.001)
    el = simulate(F, a.dim, a.steps, a.total_time, a.gamma, a.particles, seed=a.seed)
    t1 = time.time()
    t0 = t1 - el  # the timed loop only (the initial ensemble draw excluded, as in single())
    if lim is not None:
        lim.unregister()
    print(json.dumps({"t0": t0, "t1": t1}), flush=True)


if __name__ == "__main__":
    _main()
