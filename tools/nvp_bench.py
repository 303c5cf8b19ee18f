#!/usr/bin/env python3
"""RealNVP maximum-likelihood step throughput (log_density_estimation.py:13-100).

One step = pdeinv_realnvp_value_and_grad over the reference's per-epoch batch (4 000 trajectories
x 80 time stamps = 320 000 (t, x) samples of the offline dataset; synthetic rows here) with the
reference's flow (create_normalizing_flow_fn: 4d coupling layers, celu, time embedding 10) +
the fused Adam update. Algorithmic FLOPs per sample = 2 x MACs of: the likelihood pass (2 nets per
layer), the backward's recomputed forward, its input-gradient and its weight-gradient products
(4 x 2 nets per layer). Prints one JSON line per dim.

    python tools/nvp_bench.py [--steps 50] [--dims 2,4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dims", default="2,4")
    ap.add_argument("--samples", type=int, default=4000 * 80)
    a = ap.parse_args()
    from core.distribution import Gaussian
    from core.log_density_estimation import create_normalizing_flow_fn
    from utils import native, prng
    dev = "cuda"
    for dim in (int(v) for v in a.dims.split(",")):
        flow = create_normalizing_flow_fn(Gaussian(np.zeros(dim), 4 * np.eye(dim)).logdensity, dim)
        params = flow.init(prng.PRNGKey(0), 0.0, np.zeros(dim))
        flat = params["params"]
        mu, nu = torch.zeros_like(flat), torch.zeros_like(flat)
        g = torch.Generator(device=dev).manual_seed(1)
        n = a.samples
        x = torch.randn((n, 2 * dim), device=dev, generator=g) * 2   # rows of the [., 2d] dataset
        t = torch.rand(n, device=dev, generator=g) * 10
        n_in = dim + 10
        macs_mlp = n_in * 8 + 8 * 16 + 16 * 16 + 16 * dim
        flop_per_sample = 2 * flow.mnf.n_layers * 2 * macs_mlp * 4
        for step in range(a.warmup + a.steps):
            if step == a.warmup:
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            loss, grad = flow.value_and_grad(flat, t, x[:, :dim])
            native.adam_update(flat, grad, mu, nu, lr=1e-3, b1=0.9, b2=0.999, eps=1e-4, weight_decay=0.0,
                               count=step + 1)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        tf = flop_per_sample * n / (ms * 1e-3) / 1e12
        print(json.dumps({"workload": f"RealNVP MLE step d={dim} ({flow.mnf.n_layers} coupling layers, E=10, celu)",
                          "samples": n, "params": flat.numel(), "ms_per_step": ms, "samples_per_s": n / (ms * 1e-3),
                          "flop_per_sample": flop_per_sample, "TFLOPs": tf, "valu_frac": tf / FP32_VALU_PEAK_TFLOPS,
                          "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
