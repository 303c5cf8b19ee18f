#!/usr/bin/env python3
"""End-to-end trainer throughput: iterations/s of JaxTrainer.fit — data
sampling + residual value_and_grad + the fused Adam step — on the reference's own workload
recipes (scripts/*.sh and the solver defaults), one GPU. Prints one JSON line per workload.

    python tools/train_bench.py [--iters 200] [--warmup 20] [--only NAME]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))

import torch  # noqa: E402

WORKLOADS = {
    # scripts/run_OU.sh — the reference's default pde_instance (overdamped FP), MLP 32 x 2, T = 5
    "FP-exact-MLP32x2": ["estimation_mode=non-parametric", "neural_network.hidden_dim=32", "neural_network.layers=2",
                         "train.optimizer.learning_rate.initial=1e-2", "pde_instance.total_evolving_time=5",
                         "train.optimizer.learning_rate.scheduling=cosine"],
    # solver defaults (ConsistencyBased.yaml): random_time exact samples, 50 000 per set
    "KOU-exact-parametric": ["pde_instance=kinetic_fokker_planck", "pde_instance.domain_dim=4",
                             "estimation_mode=parametric"],
    # the KOU problem through the simulator (BASELINE configs 1-2 shape; moments fused in the kernel)
    "KOU-SDE-parametric-2M": ["pde_instance=kinetic_fokker_planck", "pde_instance.domain_dim=4",
                              "+pde_instance.sample_scheme=SDE", "solver.train.batch_size_0T=2097152",
                              "estimation_mode=parametric"],
    # scripts/parametric/KFP/run_KGMM_offline_parametric.sh
    "KGMM-offline-parametric": ["pde_instance=kinetic_fokker_planck", "pde_instance.domain_dim=4",
                                "pde_instance.potential=GMM", "pde_instance.sample_mode=offline",
                                "pde_instance.total_evolving_time=10", "estimation_mode=parametric", "seed=2"],
    # scripts/non-parametric/run_KGMM.sh (MLP 32 x 2)
    "KGMM-offline-MLP32x2": ["pde_instance=kinetic_fokker_planck", "pde_instance.domain_dim=4",
                             "pde_instance.potential=GMM", "pde_instance.sample_mode=offline",
                             "neural_network.hidden_dim=32", "neural_network.layers=2",
                             "pde_instance.total_evolving_time=4", "estimation_mode=non-parametric", "seed=2"],
    # scripts/parametric/KMV/run_quadratic_online.sh
    "KMV-online-parametric": ["pde_instance=kinetic_mckean_vlasov", "pde_instance.domain_dim=2",
                              "pde_instance.potential=Quadratic", "pde_instance.sample_mode=online",
                              "pde_instance.total_evolving_time=1", "seed=2", "estimation_mode=parametric",
                              "solver.train.sample_mode=grid_time", "solver.train.sample_per_time=5000",
                              "solver.train.n_time_stamps=1", "solver.train.batch_size_init=0",
                              "solver.train.batch_size_terminal=0"],
    # the same recipe with the reference's default non-parametric interaction net (MLP.yaml: 20 x 8):
    # 25 M pairs per iteration on the MFMA pair tiles
    "KMV-online-MLP20x8": ["pde_instance=kinetic_mckean_vlasov", "pde_instance.domain_dim=2",
                           "pde_instance.potential=Quadratic", "pde_instance.sample_mode=online",
                           "pde_instance.total_evolving_time=1", "seed=2", "estimation_mode=non-parametric",
                           "solver.train.sample_mode=grid_time", "solver.train.sample_per_time=5000",
                           "solver.train.n_time_stamps=1", "solver.train.batch_size_init=0",
                           "solver.train.batch_size_terminal=0"],
}
ITERS = {"KMV-online-MLP20x8": 40}  # per-workload cap (~45 ms per iteration)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--out", default=None, help="also append each JSON line to this file")
    a = ap.parse_args()
    import main as entry
    from utils import config as config_lib

    torch.cuda.set_device(0)
    for name, ov in WORKLOADS.items():
        if a.only and a.only != name:
            continue
        overrides = [o for o in ov if not o.startswith("+")] + [o[1:] for o in ov if o.startswith("+")]
        cfg = config_lib.compose("config", overrides + [f"test.frequency={a.iters + a.warmup + 10}"])
        t_build = time.perf_counter()
        iters = min(a.iters, ITERS.get(name, a.iters))
        trainer, _ = entry.run(cfg, log_path=None, number_of_iterations=min(a.warmup, iters))  # builds + warms up
        torch.cuda.synchronize()
        build_s = time.perf_counter() - t_build
        t0 = time.perf_counter()
        trainer.fit(iters)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        last = trainer.history[-1]
        line = json.dumps({"workload": name, "overrides": ov, "iters": iters, "iters_per_s": iters / el,
                           "ms_per_iter": el * 1e3 / iters, "setup_and_warmup_s": build_s,
                           "loss": last.get("loss"), "loss ground truth": last.get("loss ground truth")})
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")


if __name__ == "__main__":
    main()
