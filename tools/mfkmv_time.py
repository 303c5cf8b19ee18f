"""Time the C4 McKean-Vlasov simulate variants alone (2^21 particles, d = 8, n = 100) with HIP events: the fused
simulate + KMV stamp sums + next noise sums (pdeinv_sde_simulate_mf_kmv) against the simulate + next sums
(pdeinv_sde_simulate_mf_next) followed by the KMV pass over the written trajectory. Libraries: the in-tree one and
every path given on the command line (each loaded in its own subprocess, alternating rounds).
Usage: python tools/mfkmv_time.py [lib.so ...]"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def child(reps=20):
    sys.path.insert(0, os.path.join(HERE, "..", "pde-inverse-problem_amd"))
    import ctypes
    import numpy as np
    import torch
    from utils import native
    from example_problems.kinetic_fokker_planck_example_OU import initialize_configuration
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    d, n, N = 8, 100, 1 << 21
    ic = initialize_configuration(d)
    A, gamma = ic["tilde_F"], ic["gamma_friction"]
    coef = torch.from_numpy(dlogrho_coefficients(np.linspace(0.02, 2.0, n), ic, d).astype(np.float32)).cuda()
    z0 = native.gaussian_sample(N, torch.zeros(2 * d, device="cuda"), torch.eye(2 * d, device="cuda"), seed=7)
    desc, keep = native.mf_desc(N, d, n, 2.0 / n, gamma, A, seed=99, counter_offset=0)
    nxt, keep2 = native.mf_desc(N, d, n, 2.0 / n, gamma, A, seed=99, counter_offset=n + 1)
    xbar, _ = native.mf_mean_path(desc, native.mf_sums(desc, z0), xsum=False)
    desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
    traj, tau, last = (torch.empty((n, N, 2 * d), device="cuda"), torch.empty((n, N), device="cuda"),
                       torch.empty((N, 2 * d), device="cuda"))
    runs = {
        "fused_sim_kmv": lambda: native.sde_simulate_mf_kmv(desc, z0, traj, tau, last, gamma, coef, nxt, z0),
        "fused_no_traj": lambda: native.sde_simulate_mf_kmv(desc, z0, None, None, last, gamma, coef, nxt, z0),
        "sim_next_no_traj": lambda: native.sde_simulate_mf_next(desc, z0, None, None, last, nxt, z0),
        "sim_next": lambda: native.sde_simulate_mf_next(desc, z0, traj, tau, last, nxt, z0),
        "kmv_pass": lambda: native.kmv_moments_weights(d, gamma, coef, traj, n, N, N * 2 * d, 2 * d),
    }
    only = os.environ.get("MFKMV_ONLY")
    if only:  # e.g. under rocprofv3 --pmc: just these runs, fewer reps
        runs = {k: v for k, v in runs.items() if k in only.split(",")}
        reps = 3
    out = {}
    for name, fn in runs.items():
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name] = float(np.median(ts))
    print(json.dumps(out))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        return
    libs = [None] + sys.argv[1:]
    for rnd in range(2):
        for lib in libs:
            env = dict(os.environ)
            if lib:
                env["PDEINV_LIBRARY"] = lib
            r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                               timeout=300)
            tag = os.path.basename(lib) if lib else "base"
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-800:]
            print(f"round {rnd} {tag}: {line}", flush=True)


if __name__ == "__main__":
    main()
