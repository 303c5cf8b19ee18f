#!/usr/bin/env python3
"""Headline benchmark: particle-steps/s of the hot path on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1], "C2"): kinetic OU, d = 4, 2^21 particles per GPU,
n = 100 Euler–Maruyama steps, T = 2, gamma = 1, Gaussian-init ensemble N(0, I_8), parametric
drift recovery. One timed step = one pass of the hot path over one batch:
  1. the HIP simulator (all n+1 updates; trajectory [n,N,8], tau [n,N] and last [N,8] written to
     HBM — the reference's output contract, sampling_utils.py:52) with the KFP moment sets
     accumulated in the same kernel,
  2. [N > 1 GPUs] one RCCL all-reduce of the fp64 moment sums (the pmap mean, trainer.py:52),
  3. the KFP residual value_and_grad for the current parameters (finalize kernel).
value = particle-updates per second over all ranks = N_total * (n + 1) / step time (weak scaling; --scaling strong
fixes N_total instead and splits it over the ranks).

Other workloads (--config): C3 = kinetic FP with a GMM potential (d = 4, K = 8, 2^22 particles,
simulate + fused GMM residual over init/0T/terminal); C4 = kinetic McKean–Vlasov (d = 8, 2^21
particles per GPU, one all-reduced mean field per update, + the KMV residual).

After the timed region (untimed, C2): the drift tilde_F is recovered as the exact minimiser of the
residual from the moments of all timed steps, with Richardson extrapolation over n = 100 / 200
to cancel the O(dt) Euler–Maruyama bias; the CPU baseline — the NumPy
restatement of sampling_utils.py in oracle/ — is timed on a bounded sample on rank 0.

Launch: python bench.py [--gpus N --steps K --warmup W]. For N > 1 either under torch.distributed.run
(WORLD_SIZE must equal N, else the run exits non-zero) or plain, in which case bench.py starts the
N-rank torch.distributed.run itself as a child process before touching the GPU. The line carries
`ranks_seen` (the process group's size) and `backend`.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pde-inverse-problem_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from utils import distributed as dist  # noqa: E402
from utils import native  # noqa: E402

METRIC = "particle-steps/sec + achieved HBM GB/s; recovered-drift L2 error"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 (vector v_fma_f32 and MFMA alike)


def gmm_sim_flops(d, K):
    """Algorithmic fp32 FLOP of one particle-update of the GMM-potential simulator (FMA = 2):
    logits x.mu_k + c_k (2K(d+1)), softmax shift / sum / normalise (3K), mixture mean (2Kd),
    grad U = (x - mbar)/s^2 (2d), semi-implicit EM update of v and x (8d). Transcendentals
    (K exp2, Box-Muller) and the Philox integer work are not counted."""
    return 2 * K * (d + 1) + 3 * K + 2 * K * d + 2 * d + 8 * d


def gmm_residual_flops(d, K):
    """Algorithmic fp32 FLOP of one sample of the KFP-GMM residual value_and_grad (common.h
    gmm_residual_sample): softmax + mixture mean as above (2K(d+1) + 3K + 2Kd), e and g (2d), the dots
    e.e, e.v, v.v (6d), p_k = mu_k.v and em_k = e.mu_k (4Kd), pbar / sum w p^2 (4K), T terms (10),
    F_k (6K), Fbar (2K), cw / ce / cv (7K), sum cw (K), the mu-adjoint sum cw x + ce e + cv v (6Kd)."""
    return 2 * K * (d + 1) + 3 * K + 2 * K * d + 2 * d + 6 * d + 4 * K * d + 4 * K + 10 + 6 * K + 2 * K + 7 * K + K \
        + 6 * K * d


def mf_sim_flops(d):
    """Algorithmic fp32 FLOP of one particle-update of the McKean-Vlasov simulator (FMA = 2): y = x - xbar_s (d),
    A y (2d^2), the EM update of v and x (8d). Box-Muller and the Philox integer work are not counted."""
    return d + 2 * d * d + 8 * d


def kmv_stamp_flops(d):
    """Algorithmic fp32 FLOP of one particle-stamp of the quadratic-Phi KMV sums (kmv_moments_weights order): sum z
    (2d), sum z z^T over the upper triangle (2 per entry, m = 2d), r = m1 - x (d), the two quadratic forms of the
    weight over the symmetric pairs (4 per pair and per b_i: 4 (d(d+1)/2 + d)), w = q1 + q0^2 + gamma q0 (4),
    sum w (1), sum w x (2d), sum w x x^T (d products + 2 per upper entry)."""
    m, nt = 2 * d, d * (d + 1) // 2
    return 2 * d + m * (m + 1) + d + 4 * (nt + d) + 4 + 1 + 2 * d + d + 2 * nt


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="C2", choices=["C2", "C3", "C4", "C5"])
    p.add_argument("--particles", type=int, default=0, help="particles per GPU (0 = the config's)")
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                   help="weak: a fixed particle count per GPU (the headline); strong: a fixed job total "
                        "(--particles-total) split over the ranks (SURVEY.md §8(d) asks it for C4)")
    p.add_argument("--particles-total", type=int, default=0,
                   help="strong scaling: the job's particles (0 = 8 x the per-GPU count, the 8-GPU configuration)")
    p.add_argument("--n-steps", type=int, default=100)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-recovery", action="store_true")
    p.add_argument("--recovery-passes", type=int, default=128,
                   help="ensembles per discretisation for the (untimed) drift recovery")
    p.add_argument("--cpu-particles", type=int, default=1 << 20)
    p.add_argument("--chunk-rows", type=int, default=1 << 22,
                   help="C5: MLP-residual rows per chunk, capped at the call's rows; at most 2^30 / width (32-bit byte "
                        "offsets). r02: 2^19 / 2^20 / 2^21: 114.5 / 113.7 / 113.4 ms; r04: 2^21 / 2^22: 99.8 / 98.5-99.0 ms "
                        "residual (profiles/r04_c5_chunk_ab.txt); 28 / 56 GB workspace")
    p.add_argument("--c4-pipeline", action="store_true",
                   help="C4 at world 1: two streams, simulate k+1 concurrent with the KMV residual of step k on a "
                        "double-buffered trajectory (measured 6.85 vs 6.25 ms/step serial: the step is HBM-bound, "
                        "so overlap buys nothing and the fused next-simulate sums are lost); default serial")
    p.add_argument("--c4-separate-sums", action="store_true",
                   help="C4: the next simulate's mean-path sums as their own launch (pdeinv_mf_sums) instead of "
                        "inside the KMV pass (pdeinv_kmv_moments_weights_mf_sums), for A/B")
    p.add_argument("--c4-schedule", default="simkmv", choices=["fused", "concurrent", "sim", "simkmv"],
                   help="C4 steady state: 'simkmv' (default, the product path of methods/consistency.py) = the "
                        "simulator forms the KMV per-stamp sums from its staged rows and draws the next simulate's "
                        "noise sums (pdeinv_sde_simulate_mf_kmv): no trajectory written or read; 'sim' = the "
                        "simulator writes the trajectory and draws the next sums (pdeinv_sde_simulate_mf_next), then "
                        "one KMV pass reads it; 'fused' = the next sums inside the KMV pass; 'concurrent' = on a "
                        "side stream (DESIGN.md §4.3)")
    p.add_argument("--cpu-procs", type=int, default=0,
                   help="CPU-baseline shard processes (0 = the per-GPU host share, os.cpu_count() // 8)")
    return p.parse_args()


def sim_bytes(N, n, d):
    """z0 read 8d + n (traj 8d + tau 4) + last 8d bytes per particle."""
    return N * (8 * d + n * (8 * d + 4) + 8 * d)


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


RAMP_S = 0.3


KERN_STATS = {}  # per-launch spread of the dominant kernel over the timed steps (filled by timed())


def run_ramp(ramp, dev, seconds=RAMP_S, sync=None):
    """Repeat ramp() in rounds of 8 for about `seconds` of wall clock. Every rank runs the SAME number of
    rounds: the step a config ramps with may hold collectives (C3 / C4 / C5: the residual's all-reduce), and
    a rank that stopped one round earlier than its peer on its own clock would leave that peer's collective
    unmatched (a hang seen in the world-2 GPU tests). So after each round the ranks agree on whether any of
    them still wants to ramp. Returns the number of rounds."""
    sync = sync or torch.cuda.synchronize
    t_end = time.perf_counter() + seconds
    rounds = 0
    while True:
        for _ in range(8):
            ramp()
        sync()
        rounds += 1
        if dist.allreduce_max_scalar(1.0 if time.perf_counter() < t_end else 0.0, device=dev) == 0.0:
            return rounds


def timed(step, K, W, dev, ramp=None):
    """Clock ramp, W untimed warmup steps, then K steps between barrier+synchronize; max over ranks.
    step(record) records record[0]/record[1] around the dominant kernel's launch.
    The ramp (untimed setup, like allocating the buffers) repeats the step's work for RAMP_S seconds
    first: an MI355X raises its clocks over the first ~0.1-0.3 s of sustained load (one box measured a
    20-step run 8 % below its 200-step rate without it; on another the ramp changed nothing).
    ramp() (default: step(None)) must not feed any result of the run.
    Returns (ms per step, mean dominant-launch ms); the launch spread (min over ranks of the per-rank min,
    max over ranks of the median and of the max) goes to KERN_STATS for roofline.kernel_ms_*."""
    run_ramp(ramp or (lambda: step(None)), dev)
    for _ in range(W):
        step(None)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        step(evs[k])
    torch.cuda.synchronize()
    dist.barrier()
    el = dist.allreduce_max_scalar(time.perf_counter() - t0, device=dev)
    per = np.array([s.elapsed_time(e) for s, e in evs])
    kern_ms = dist.allreduce_max_scalar(float(per.mean()), device=dev)
    KERN_STATS.clear()
    KERN_STATS.update(kernel_ms_min=-dist.allreduce_max_scalar(-float(per.min()), device=dev),
                      kernel_ms_median=dist.allreduce_max_scalar(float(np.median(per)), device=dev),
                      kernel_ms_max=dist.allreduce_max_scalar(float(per.max()), device=dev),
                      kernel_launches_timed=int(K))
    return el * 1e3 / K, kern_ms


def write_ceiling(buf, reps=5):
    """This box's plain streaming-write rate: torch fill_ of an HBM buffer of the trajectory's size,
    timed with events after the timed region (context for roofline.frac: HBM write bandwidth
    differs by several tens of percent between MI355X boxes of the pool, MI355X_MICROARCH.md)."""
    buf.fill_(0.0)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        buf.fill_(1.0)
    e.record()
    torch.cuda.synchronize()
    return buf.numel() * buf.element_size() / (s.elapsed_time(e) / reps / 1e3) / 1e9


def traffic_from_profiles(key):
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(key)
    except Exception:
        return None


def particle_share(a, rank, world, per_gpu_default):
    """(N, first global id, job total) of this rank. Weak scaling: N = --particles or the config's per-GPU count
    on every rank, ids [rank N, rank N + N). Strong scaling: the job total (--particles-total, default 8 x the
    per-GPU count — the 8-GPU weak configuration, C4's 2^24 of SURVEY.md §8(d)) in contiguous shares. The
    Philox streams follow the global ids, so a particle's numbers do not depend on the rank count."""
    if a.scaling == "strong":
        total = a.particles_total or 8 * (a.particles or per_gpu_default)
        poff, N = dist.shard(total, rank, world)
        return N, poff, total
    N = a.particles or per_gpu_default
    return N, rank * N, world * N


def base_record(a, world, value, ms, config, kern_ms, bytes_launch, kernel, traffic=None, flops_launch=None):
    """roofline: HBM-bound launches (the simulators) report algorithmic bytes / launch time against the
    HBM peak; a VALU-bound launch (flops_launch given: C3's simulator with the fused GMM residual) reports
    its algorithmic fp32 FLOP / launch time against the fp32 vector peak, the HBM figure kept beside it."""
    achieved = bytes_launch / (kern_ms / 1e3) / 1e9
    if flops_launch is not None:
        tf = flops_launch / (kern_ms / 1e3) / 1e12
        roof = {"bound": "valu", "achieved": tf, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": tf / FP32_PEAK_TFLOPS, "traffic": traffic, "kernel": kernel, "kernel_ms": kern_ms,
                "algorithmic_flops_per_launch": flops_launch, "algorithmic_bytes_per_launch": bytes_launch,
                "hbm": {"achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS}}
    else:
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "kernel": kernel,
                "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": bytes_launch}
    return {
        "metric": METRIC, "value": value, "unit": "particle-steps/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": a.scaling,
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: Philox Gaussian-init ensembles, fresh noise per step",
        "config": config, "hbm_GBps": achieved, "roofline": roof,
    }


# ------------------------------------------------------------------------------------------
def run_c2(a, rank, world, dev):
    from example_problems.kinetic_fokker_planck_example_OU import problem_matrix
    from methods.consistency_instances.kinetic_fokker_planck import recover_drift_richardson

    d, n, T, gamma = 4, a.n_steps, 2.0, 1.0
    N, poff, total = particle_share(a, rank, world, 1 << 21)
    F = problem_matrix(d)
    pot = dict(kind=native.POT_QUADRATIC, params=F)
    seed = 0x5EED_0001
    z0 = native.gaussian_sample(N, torch.zeros(2 * d, device=dev), torch.eye(2 * d, device=dev),
                                seed=seed ^ 0xA5A5, row_offset=poff)
    theta = torch.zeros(d * d + d, device=dev)
    bufs = {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
            "last": torch.empty((N, 2 * d), device=dev),
            "moments": torch.empty((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)}
    mom_total = torch.zeros((3, native.moment_len(2 * d)), device=dev, dtype=torch.float64)
    counter = [0]
    last_res = [None]

    def step(record):
        if record is not None:
            record[0].record()
        r = native.sde_simulate(z0, n, T / n, gamma, pot, seed=seed, counter_offset=counter[0],
                                particle_offset=poff, moments=True, out=bufs)
        if record is not None:
            record[1].record()
        counter[0] = (counter[0] + n + 1) & 0xFFFFFFFF
        mom = dist.allreduce_sum(r["moments"])
        last_res[0] = native.residual_kfp_quadratic(mom, theta, F, gamma, T)
        mom_total.add_(mom)

    def ramp():  # the same launch, results discarded (mom_total feeds the drift recovery)
        native.sde_simulate(z0, n, T / n, gamma, pot, seed=seed, counter_offset=counter[0], particle_offset=poff,
                            moments=True, out=bufs)

    ms, kern_ms = timed(step, a.steps, a.warmup, dev, ramp=ramp)
    value = total * (n + 1) / (ms / 1e3)
    cfg = {"workload": "C2 kinetic OU d=4: EM simulate (traj+tau+last, fused moments) + KFP residual "
                       "value_and_grad", "dim": d, "n_steps": n, "particles_per_gpu": N, "particles_total": total, "total_time": T,
           "gamma": gamma, "parallelism": f"dp{world}"}
    out = base_record(a, world, value, ms, cfg, kern_ms, sim_bytes(N, n, d),
                      "sde_simulate_kernel<4,QUADRATIC,moments,staged> (+ its slab reduce)",
                      traffic_from_profiles("sde_simulate_C2_bytes_per_launch") if (N, n) == (1 << 21, 100) else None)
    out["loss"] = float(last_res[0][0][0].item())
    ceil = dist.allreduce_max_scalar(-write_ceiling(bufs["traj"]), device=dev) * -1.0  # min over ranks
    out["roofline"]["box_write_ceiling_GBps"] = ceil
    out["roofline"]["frac_of_box_write_ceiling"] = out["roofline"]["achieved"] / ceil
    if not a.no_recovery:
        # untimed; a fixed Monte-Carlo budget (independent of --steps) of fresh moments-only passes,
        # on top of the timed steps' moments, at n = 100 and n = 200
        passes = max(a.recovery_passes, a.steps + a.warmup)
        rec = recover_drift_richardson(z0, F, gamma, T, n, seed, passes, counter_offset=counter[0],
                                       particle_offset=poff, base=mom_total, base_passes=a.steps + a.warmup)
        counter[0] = rec["counter"]
        S_rich = rec["S_rich"]
        out["drift_err"] = float(np.abs(S_rich - F).max())
        out["drift_err_l2"] = float(np.linalg.norm(S_rich - F) / np.linalg.norm(F))
        out["drift_err_richardson1"] = float(np.abs(rec["S_rich1"] - F).max())
        out["drift_err_em_n100"] = float(np.abs(rec["S_n"] - F).max())
        out["drift_recovery"] = ("max |S - tilde_F|, S = K + K^T the exact residual minimiser from the EM moments, "
                                 "Richardson (8 S(n=400) - 6 S(n=200) + S(n=100)) / 3, "
                                 f"{passes * total} trajectories per level")
    if rank == 0 and world == 1 and not a.no_cpu_baseline:  # the CPU baseline: rank 0 at N = 1 only
        from oracle import cpu_baseline as cb
        from example_problems.kinetic_fokker_planck_example_OU import problem_matrix as pm
        ups1, secs1 = cb.single(F, d, n, T, gamma, a.cpu_particles)
        # the per-GPU share of the host: an 8-GPU node's cores / 8 (P = cores)
        P = a.cpu_procs or max(1, (os.cpu_count() or 8) // 8)
        P = max(1, min(P, os.cpu_count() or 1))
        n_per = max(1, a.cpu_particles // 4)
        upsP, secsP = cb.multi(F, d, n, T, gamma, n_per, P)
        # C1 (BASELINE configs[0], scripts/run_KOU.sh): KOU d = 2, 4 096 particles, 100 steps, in full
        ups_c1, secs_c1 = cb.single(pm(2), 2, n, T, gamma, 4096)
        what = (f"NumPy restatement of sampling_utils.py (oracle/cpu_baseline.py: update_step + moment pass), fp32, "
                f"d={d}, {n + 1} updates")
        host = f"host {cpu_model()}, os.cpu_count()={os.cpu_count()}"
        out["cpu_baseline"] = {"value": upsP, "unit": "particle-steps/s", "cores": P, "kind": "port",
                               "sample": f"{what}; {P} processes (os.cpu_count() // 8, the per-GPU host share) x "
                                         f"{n_per} particles started together, {secsP:.1f} s wall; {host}"}
        out["cpu_baseline_1core"] = {"value": ups1, "unit": "particle-steps/s", "cores": 1, "kind": "port",
                                     "sample": f"{what}; one process, {a.cpu_particles} particles, {secs1:.1f} s"}
        out["cpu_baseline_c1"] = {"value": ups_c1, "unit": "particle-steps/s", "cores": 1, "kind": "port",
                                  "sample": f"C1 in full: KOU d=2, 4096 particles x {n + 1} updates (+ moment pass), "
                                            f"one process, {secs_c1 * 1e3:.1f} ms"}
        out["gpu_over_cpu"] = value / upsP
    return out


def c3_valu_issue(kern_ms, N, n):
    """The C3 launch is VALU-issue-bound, and its FMA-only frac leaves out the transcendentals, Philox's
    v_mad_u64_u32 and the packed moves. profiles/c3_valu_issue.json (tools/c3_valu_model.py) prices the step loop's
    VALU opcodes with their measured issue cost (tools/valu_rate.hip, shader cycles) and checks the total against
    the SQ pass of the same launch (SQ_ACTIVE_INST_VALU). Here: the model's issue cycles over this run's launch
    time at the nominal 2.4 GHz (the clock the FMA peak is quoted at: a lower bound, the chip runs slower under
    this load), beside the committed busy shares at the profiled launch's own clock (GRBM_GUI_ACTIVE / 8)."""
    try:
        with open(os.path.join(ROOT, "profiles", "c3_valu_issue.json")) as f:
            m = json.load(f)
    except Exception:
        return None
    wave_updates = N / 64 * (n + 1)
    cyc = m["model_issue_cycles_per_update_asymptotic"]
    return {"issue_cycles_per_wave_update_model": cyc,
            "issue_cycles_per_wave_update_launch_profiled": m["launch_cycles_per_update"],
            "issue_frac_nominal_clock": cyc * wave_updates / (1024 * 2.4e9 * kern_ms / 1e3),
            "issue_frac_model_profiled": m["model_valu_busy_asymptotic"],
            "issue_frac_model_profiled_at_3_waves_per_simd": m["model_valu_busy"],
            "sq_active_inst_valu_share_profiled": m["sq_active_inst_valu_share"],
            "profiled_clock_ghz": m.get("profiled_clock_ghz"), "source": "profiles/c3_valu_issue.json"}


def run_c3(a, rank, world, dev):
    """KFP-GMM d=4, K=8 (BASELINE configs[2]), the reference's online iteration: simulate (traj, tau, last
    written) with the KFP-GMM residual value_and_grad over init = z0, 0T = every trajectory row,
    terminal = last fused into the same launch (pdeinv_sde_simulate_kfp_gmm), all-reduce, finalize."""
    from example_problems.kinetic_fokker_planck_example_GMM import gmm_means
    from utils import prng

    d, K, n, T, gamma = 4, 8, a.n_steps, 2.0, 0.5
    N, poff, total = particle_share(a, rank, world, 1 << 22)
    mus = gmm_means(d, K, prng.PRNGKey(2))
    pot = dict(kind=native.POT_GMM, params=mus, n_centers=K, sigma=1.0)
    seed = 0x5EED_0003
    ch = torch.diag(torch.tensor([2.0] * d + [math.sqrt(0.1)] * d, device=dev))  # x0~N(0,4I), v0~N(0,0.1I)
    z0 = native.gaussian_sample(N, torch.zeros(2 * d, device=dev), ch, seed=seed ^ 0xA5A5, row_offset=poff)
    mus_model = torch.as_tensor(np.random.default_rng(0).standard_normal((K, d)), dtype=torch.float32, device=dev)
    bufs = {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
            "last": torch.empty((N, 2 * d), device=dev)}
    Ng = total
    desc = native.kfp_gmm_desc(d, K, mus, gamma, T, Ng, Ng, Ng * n)
    counter = [0]
    last_out = [None]

    def step(record):
        if record is not None:
            record[0].record()
        r = native.sde_simulate_kfp_gmm(z0, n, T / n, gamma, pot, desc, mus_model, seed=seed,
                                        counter_offset=counter[0], particle_offset=poff, out=bufs)
        if record is not None:
            record[1].record()
        counter[0] = (counter[0] + n + 1) & 0xFFFFFFFF
        acc = dist.allreduce_sum(r["acc"])
        last_out[0] = native.residual_kfp_gmm_finalize(desc, acc)

    ms, kern_ms = timed(step, a.steps, a.warmup, dev)
    value = total * (n + 1) / (ms / 1e3)
    cfg = {"workload": "C3 kinetic FP, GMM potential K=8, d=4: EM simulate (traj+tau+last) with the GMM-model KFP "
                       "residual value_and_grad over init/0T/terminal fused into the same launch",
           "dim": d, "n_centers": K, "n_steps": n, "particles_per_gpu": N, "particles_total": total, "total_time": T, "gamma": gamma,
           "parallelism": f"dp{world}"}
    # VALU-bound: every particle-update runs the GMM simulator step and one residual sample (its 0T row;
    # z0 / last add one sample per particle each)
    flops = N * ((n + 1) * gmm_sim_flops(d, K) + (n + 2) * gmm_residual_flops(d, K))
    out = base_record(a, world, value, ms, cfg, kern_ms, sim_bytes(N, n, d),
                      "sde_simulate_kernel<4,GMM,staged,KM=8,fused KFP-GMM residual> (+ its slab reduce)",
                      traffic_from_profiles("sde_simulate_C3_bytes_per_launch") if (N, n) == (1 << 22, 100) else None,
                      flops_launch=flops)
    out["loss"] = float(last_out[0][0][0].item())
    if (N, n) == (1 << 22, 100):
        out["roofline"]["valu_issue"] = c3_valu_issue(kern_ms, N, n)

    # untimed context: the same simulator without the residual, and the standalone residual kernel
    # (the offline-dataset path) over the same trajectory, each timed with events on its stream
    def ev_time(fn, reps=5):
        fn()
        s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s_.record()
        for _ in range(reps):
            fn()
        e_.record()
        torch.cuda.synchronize()
        return s_.elapsed_time(e_) / reps

    sim_ms = ev_time(lambda: native.sde_simulate(z0, n, T / n, gamma, pot, seed=seed, counter_offset=counter[0],
                                                 particle_offset=poff, out=bufs))
    res_ms = ev_time(lambda: native.residual_kfp_gmm(desc, z0, bufs["last"], bufs["traj"].view(-1, 2 * d), mus_model))
    res_bytes = N * (n + 2) * 8 * d
    out["simulate_only_ms"] = sim_ms
    out["fused_over_simulate_only"] = kern_ms / sim_ms
    out["standalone_residual"] = {"kernel": "kfp_gmm_kernel<4,8> + slab reduce (offline path)", "ms": res_ms,
                                  "algorithmic_bytes": res_bytes, "GBps": res_bytes / (res_ms / 1e3) / 1e9}
    return out


def run_c4(a, rank, world, dev):
    """Kinetic McKean-Vlasov d=8 (BASELINE configs[3]): the fused driver (utils/mean_field.py) — noise/z0
    sums, ONE all-reduce per simulate, the closed-form mean path, all n+1 updates in registers — then the
    KMV residual from one fused read of the trajectory (per-stamp moments + d_s log rho weights)."""
    import ctypes
    from example_problems.kinetic_fokker_planck_example_OU import initialize_configuration
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    from utils.mean_field import stamp_times
    from utils import prng

    d, n, T = 8, a.n_steps, 2.0
    N, poff, total = particle_share(a, rank, world, 1 << 21)
    ic = initialize_configuration(d)
    gamma = ic["gamma_friction"]
    A = ic["tilde_F"]
    z0 = native.gaussian_sample(N, torch.zeros(2 * d, device=dev), torch.eye(2 * d, device=dev), seed=7,
                                row_offset=poff)
    theta = torch.zeros(d * d + d, device=dev)
    key = prng.Key(0x5EED_0004)
    counter = [0]
    bufs = {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
            "last": torch.empty((N, 2 * d), device=dev)}

    def host_coef(ctr):
        # the shared-clock stamps are known from (seed, counter) without touching the device, so the
        # per-stamp coefficient rows of the NEXT step are built on the host while the GPU runs this one
        tau = stamp_times(key.seed, ctr, n, T / n).astype(np.float64)
        return torch.from_numpy(dlogrho_coefficients(tau, ic, d).astype(np.float32)).pin_memory()

    coef_next = [host_coef(counter[0])]
    side = torch.cuda.Stream(device=dev)
    ev = {"sums": [], "res": []}
    sums_next = [None]  # rank-local mean-path sums of the next simulate, from the previous step's KMV pass

    def step(record):
        coef = coef_next[0].to(dev, non_blocking=True)
        desc, keep = native.mf_desc(N, d, n, T / n, gamma, A, seed=key.seed, counter_offset=counter[0],
                                    particle_offset=poff)
        e0 = torch.cuda.Event(enable_timing=True) if record is not None else None
        if e0 is not None:
            e0.record()
        local = sums_next[0] if sums_next[0] is not None else native.mf_sums(desc, z0)
        sums = dist.allreduce_sum(local)  # the one collective of the simulate
        xbar, _ = native.mf_mean_path(desc, sums, xsum=False)
        desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
        if record is not None:
            record[0].record()
        sim_sums = a.c4_schedule in ("sim", "simkmv") and not a.c4_separate_sums
        kmv_in_sim = a.c4_schedule == "simkmv" and not a.c4_separate_sums
        if kmv_in_sim:  # the simulator also forms the KMV per-stamp sums and draws the next simulate's noise sums
            desc_n, keep_n = native.mf_desc(N, d, n, T / n, gamma, A, seed=key.seed,
                                            counter_offset=(counter[0] + n + 1) & 0xFFFFFFFF, particle_offset=poff)
            # as the product path (methods/consistency.py): the residual needs only these sums, no trajectory
            mom, wst, sums_next[0] = native.sde_simulate_mf_kmv(desc, z0, None, None, bufs["last"],
                                                                gamma, coef, desc_n, z0)
            del keep_n
        elif sim_sums:  # the simulator also draws the NEXT simulate's mean-path noise sums (same z0 ensemble)
            desc_n, keep_n = native.mf_desc(N, d, n, T / n, gamma, A, seed=key.seed,
                                            counter_offset=(counter[0] + n + 1) & 0xFFFFFFFF, particle_offset=poff)
            sums_next[0] = native.sde_simulate_mf_next(desc, z0, bufs["traj"], bufs["tau"], bufs["last"], desc_n, z0)
            del keep_n
        else:
            native.sde_simulate_desc(desc, z0, bufs["traj"], bufs["tau"], bufs["last"])
        if record is not None:
            record[1].record()
        del keep
        counter[0] = (counter[0] + n + 1) & 0xFFFFFFFF
        if kmv_in_sim:
            pass
        elif sim_sums:
            mom, wst = native.kmv_moments_weights(d, gamma, coef, bufs["traj"], n, N, N * 2 * d, 2 * d)
        elif a.c4_schedule == "concurrent" and not a.c4_separate_sums:
            # the next simulate's sums depend only on (seed, counter, ids, z0): they run on the side stream
            # beside the read-bound KMV pass of this step; the next step's all-reduce waits for them
            desc_n, keep_n = native.mf_desc(N, d, n, T / n, gamma, A, seed=key.seed, counter_offset=counter[0],
                                            particle_offset=poff)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                sn = native.mf_sums(desc_n, z0)
            del keep_n
            mom, wst = native.kmv_moments_weights(d, gamma, coef, bufs["traj"], n, N, N * 2 * d, 2 * d)
            torch.cuda.current_stream().wait_stream(side)
            sn.record_stream(torch.cuda.current_stream())
            sums_next[0] = sn
        elif a.c4_separate_sums:
            mom, wst = native.kmv_moments_weights(d, gamma, coef, bufs["traj"], n, N, N * 2 * d, 2 * d)
        else:  # steady state: the KMV pass also sums the next simulate's mean-path noise (same z0 ensemble)
            desc_n, keep_n = native.mf_desc(N, d, n, T / n, gamma, A, seed=key.seed, counter_offset=counter[0],
                                            particle_offset=poff)
            mom, wst, sums_next[0] = native.kmv_moments_weights_mf_sums(d, gamma, coef, bufs["traj"], n, N,
                                                                        N * 2 * d, 2 * d, desc_n, z0)
            del keep_n
        if record is not None:
            e3 = torch.cuda.Event(enable_timing=True)
            e3.record()
            ev["sums"].append((e0, record[0]))
            ev["res"].append((record[1], e3))
        both = dist.allreduce_sum(torch.cat([mom.reshape(-1), wst.reshape(-1)]))
        native.residual_kmv(both[: mom.numel()].view_as(mom), both[mom.numel():].view_as(wst), theta, A, gamma)
        coef_next[0] = host_coef(counter[0])

    # Two-stream pipeline (world 1, --c4-pipeline; slower, kept for A/B): the simulate of step k+1 depends on z0 and the noise stream only — not on
    # step k's residual or parameters — so it runs on stream S while step k's KMV pass + residual run on
    # stream R over the other half of a double-buffered trajectory: store-bound simulator, VALU-bound noise
    # sums and read-bound KMV pass overlap. (Not at world > 1: two RCCL collectives in flight on two streams
    # could meet in different orders on different GPUs.)
    pipeline = a.c4_pipeline and world == 1
    if pipeline:
        S, Rs = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
        bsets = [bufs, {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
                        "last": torch.empty((N, 2 * d), device=dev)}]
        sim_done = [torch.cuda.Event(), torch.cuda.Event()]
        pass_done = [None, None]
        kstep = [0]

        def step(record):  # noqa: F811 - the pipelined step
            k = kstep[0] % 2
            kstep[0] += 1
            b = bsets[k]
            with torch.cuda.stream(S):
                if pass_done[k] is not None:
                    S.wait_event(pass_done[k])  # step k-2's pass has finished reading this buffer
                desc, keep = native.mf_desc(N, d, n, T / n, gamma, A, seed=key.seed, counter_offset=counter[0],
                                            particle_offset=poff)
                e0 = torch.cuda.Event(enable_timing=True) if record is not None else None
                if e0 is not None:
                    e0.record()
                sums = dist.allreduce_sum(native.mf_sums(desc, z0))
                xbar, _ = native.mf_mean_path(desc, sums, xsum=False)
                desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
                if record is not None:
                    record[0].record()
                native.sde_simulate_desc(desc, z0, b["traj"], b["tau"], b["last"])
                if record is not None:
                    record[1].record()
                sim_done[k].record()
                del keep
            counter[0] = (counter[0] + n + 1) & 0xFFFFFFFF
            with torch.cuda.stream(Rs):
                Rs.wait_event(sim_done[k])
                coef = coef_next[0].to(dev, non_blocking=True)
                e2 = torch.cuda.Event(enable_timing=True) if record is not None else None
                if e2 is not None:
                    e2.record()
                mom, wst = native.kmv_moments_weights(d, gamma, coef, b["traj"], n, N, N * 2 * d, 2 * d)
                if record is not None:
                    e3 = torch.cuda.Event(enable_timing=True)
                    e3.record()
                    ev["sums"].append((e0, record[0]))
                    ev["res"].append((e2, e3))
                both = dist.allreduce_sum(torch.cat([mom.reshape(-1), wst.reshape(-1)]))
                native.residual_kmv(both[: mom.numel()].view_as(mom), both[mom.numel():].view_as(wst), theta, A,
                                    gamma)
                ev_done = torch.cuda.Event()
                ev_done.record()
                pass_done[k] = ev_done
            coef_next[0] = host_coef(counter[0])

    ms, kern_ms = timed(step, a.steps, a.warmup, dev)
    value = total * (n + 1) / (ms / 1e3)
    cfg = {"workload": "C4 kinetic McKean-Vlasov quadratic interaction d=8: interacting-particle EM (closed-form "
                       "mean path from one all-reduced noise/z0 sum per simulate, all updates in registers) + KMV "
                       "residual value_and_grad (one fused read of the trajectory)",
           "dim": d, "n_steps": n, "particles_per_gpu": N, "particles_total": total, "total_time": T, "gamma": gamma,
           "parallelism": f"dp{world}"}
    kmv_in_sim = a.c4_schedule == "simkmv" and not a.c4_separate_sums and not pipeline
    if kmv_in_sim:  # no trajectory: the launch is bound by its fp32 issue (VALU and the f32 MFMA share the SIMD)
        cfg["workload"] = cfg["workload"].replace("KMV residual value_and_grad (one fused read of the trajectory)",
                                                  "KMV residual value_and_grad from per-stamp sums the simulator "
                                                  "forms (no trajectory written or read)")
        out = base_record(a, world, value, ms, cfg, kern_ms, N * (8 * d + 8 * d),
                          "sde_mf_kmv_kernel<8,4,next sums> (all 101 updates + the KMV per-stamp sums of 100 stamps "
                          "+ the next simulate's 101 x 8 normals per particle) + slab reduce + mf_sums tail",
                          None, flops_launch=N * ((n + 1) * mf_sim_flops(d) + n * kmv_stamp_flops(d)))
    else:
        out = base_record(a, world, value, ms, cfg, kern_ms, sim_bytes(N, n, d),
                          "sde_simulate_kernel<8,MEANFIELD_QUADRATIC,staged> (all 101 updates)",
                          traffic_from_profiles("sde_simulate_C4_bytes_per_launch") if (N, n) == (1 << 21, 100)
                          else None)
    sums_ms = float(np.mean([s.elapsed_time(e) for s, e in ev["sums"]]))
    res_ms = float(np.mean([s.elapsed_time(e) for s, e in ev["res"]]))
    res_bytes = N * n * 8 * d
    out["c4_schedule"] = ("two-stream pipeline: simulate k+1 (+ its mean-path sums) on one stream concurrent with "
                          "the KMV pass + residual of step k on another, double-buffered trajectory" if pipeline else
                          "serial" + (", separate mean-path sums" if a.c4_separate_sums else
                                      (", mean-path sums of the next simulate on a side stream concurrent with the "
                                       "KMV pass" if a.c4_schedule == "concurrent" else
                                       (", the KMV per-stamp sums and the next simulate's mean-path noise sums "
                                        "formed inside the simulator (no trajectory)" if kmv_in_sim else
                                        ", mean-path noise sums of the next simulate drawn inside the simulator"
                                        if a.c4_schedule == "sim" else
                                        ", mean-path sums of the next simulate inside the KMV pass"))))
    if a.c4_separate_sums or pipeline:
        out["mean_path"] = {"kernel": "mf_sums_kernel<8> + slab reduce (+ all-reduce) + mf_path_kernel",
                            "ms": sums_ms, "normals_per_s": N * (n + 1) * d / (sums_ms / 1e3)}
        out["residual"] = {"kernel": "kmv_moments_weights_kernel<8> + slab reduce + split", "ms": res_ms,
                           "algorithmic_bytes": res_bytes, "GBps": res_bytes / (res_ms / 1e3) / 1e9}
    elif kmv_in_sim:
        out["mean_path"] = {"kernel": "all-reduce of the sums the previous simulate drew + mf_path_kernel", "ms": sums_ms}
        out["residual"] = {"kernel": "all-reduce of the per-stamp sums + kmv_terms / kmv_combine", "ms": res_ms}
    elif a.c4_schedule == "sim":
        out["mean_path"] = {"kernel": "all-reduce of the sums the previous simulate drew + mf_path_kernel", "ms": sums_ms}
        out["roofline"]["kernel"] = ("sde_simulate_kernel<8,MEANFIELD_QUADRATIC,staged,next sums> (all 101 updates + the "
                                     "next simulate's 101 x 8 normals per particle)")
        out["residual"] = {"kernel": "kmv_moments_weights_kernel<8> + slab reduce + split", "ms": res_ms,
                           "algorithmic_bytes": res_bytes, "GBps": res_bytes / (res_ms / 1e3) / 1e9}
    elif a.c4_schedule == "concurrent":
        out["mean_path"] = {"kernel": "all-reduce of the sums the previous step's side stream produced + mf_path_kernel",
                            "ms": sums_ms}
        out["residual"] = {"kernel": "kmv_moments_weights_kernel<8> + slab reduce + split (main stream) concurrent with "
                                     "the next simulate's mf_sums_kernel<8> (side stream)", "ms": res_ms,
                           "algorithmic_bytes": res_bytes, "GBps": res_bytes / (res_ms / 1e3) / 1e9,
                           "next_normals_per_s": N * (n + 1) * d / (res_ms / 1e3)}
    else:
        out["mean_path"] = {"kernel": "all-reduce of the sums the previous KMV pass produced + mf_path_kernel",
                            "ms": sums_ms}
        out["residual"] = {"kernel": "kmv_moments_weights_kernel<8, MF> (+ the next simulate's mean-path noise sums "
                                     "of updates 0..n-1) + mf_sums tail (update n, z0) + slab reduces + split",
                           "ms": res_ms, "algorithmic_bytes": res_bytes, "GBps": res_bytes / (res_ms / 1e3) / 1e9,
                           "next_normals_per_s": N * (n + 1) * d / (res_ms / 1e3)}
    return out


def run_c5(a, rank, world, dev):
    """KFP-GMM d=8, K=8 simulate (traj written) + the non-parametric MLP residual (W=256, L=2,
    out 40) on one uniformly drawn step per particle."""
    from example_problems.kinetic_fokker_planck_example_GMM import gmm_means
    from core.model import V_hypothesis
    from utils import prng

    d, K, n, T, gamma, W, L = 8, 8, a.n_steps, 2.0, 0.5, 256, 2
    N, poff, total = particle_share(a, rank, world, 1 << 22)
    nb = N // 16  # boundary batches (initial / terminal)
    mus = gmm_means(d, K, prng.PRNGKey(5))
    pot = dict(kind=native.POT_GMM, params=mus, n_centers=K, sigma=1.0)
    seed = 0x5EED_0005
    ch = torch.diag(torch.tensor([2.0] * d + [math.sqrt(0.1)] * d, device=dev))
    z0 = native.gaussian_sample(N, torch.zeros(2 * d, device=dev), ch, seed=seed ^ 0xA5A5, row_offset=poff)
    net = V_hypothesis(output_dim=1, hidden_dims=[W] * L)
    params = net.init(prng.PRNGKey(11), np.zeros(d), device=dev)
    flat = net.flat(params)
    dims = net.dims(d)
    P_mac = sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))
    bufs = {"traj": torch.empty((n, N, 2 * d), device=dev), "tau": torch.empty((n, N), device=dev),
            "last": torch.empty((N, 2 * d), device=dev)}
    counter = [0]
    sim_ev = []

    def step(record):
        e0 = torch.cuda.Event(enable_timing=True) if record is not None else None
        if e0 is not None:
            e0.record()
        r = native.sde_simulate(z0, n, T / n, gamma, pot, seed=seed, counter_offset=counter[0],
                                particle_offset=poff, out=bufs)
        counter[0] = (counter[0] + n + 1) & 0xFFFFFFFF
        z0T = native.gather_random_step(r["traj"], seed=seed, ctr=counter[0])
        if record is not None:
            record[0].record()
            sim_ev.append((e0, record[0]))
        acc, grad = native.residual_kfp_mlp(dims, flat, z0[:nb], r["last"][:nb], z0T, true_kind=native.POT_GMM,
                                            true_params=mus, gamma=gamma, total_time=T, world_scale=1.0 / world,
                                            chunk_rows=min(a.chunk_rows, (N + 2 * nb + 63) // 64 * 64))
        if record is not None:
            record[1].record()
        both = dist.allreduce_sum(torch.cat([acc, grad.double()]))
        native.kfp_terms_finalize(both[: acc.numel()], both[acc.numel():].float(), gamma)

    ms, kern_ms = timed(step, a.steps, a.warmup, dev)
    rows = N + 2 * nb
    # 24P per 0T row (value, ∂v, ∂v² Taylor streams, the ∇x reverse and the θ reverse), 12P per
    # initial / terminal row — the reference evaluates only ∇V·v there (kinetic_fokker_planck.py:34-39)
    flops = 24.0 * P_mac * N + 12.0 * P_mac * 2 * nb
    value = total * (n + 1) / (ms / 1e3)
    sim_ms = float(np.mean([s.elapsed_time(e) for s, e in sim_ev]))
    cfg = {"workload": "C5 KFP-GMM d=8 K=8: EM simulate (traj+tau+last) + non-parametric MLP residual "
                       "value_and_grad (W=256, L=2, out 40) on one random step per particle + N/16 boundary rows",
           "dim": d, "n_centers": K, "n_steps": n, "particles_per_gpu": N, "particles_total": total, "mlp": dims, "residual_rows": rows,
           "parallelism": f"dp{world}"}
    achieved = flops / (kern_ms / 1e3) / 1e12
    out = {
        "metric": METRIC, "value": value, "unit": "particle-steps/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic: Philox Gaussian-init ensembles, fresh noise per step", "config": cfg,
        "residual_samples_per_s": world * rows / (kern_ms / 1e3),
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": 157.3, "unit": "TFLOP/s", "frac": achieved / 157.3,
                     "traffic": traffic_from_profiles("mlp_residual_C5_bytes_per_launch") if N == 1 << 22 else None,
                     "kernel": ("MLP residual, fused fp32-MFMA path (hand-written GEMMs with fused prologues/epilogues)"
                                if native.mlp_fused_supported(dims) else
                                "MLP residual, library path (rocBLAS sgemm + element-wise kernels)"),
                     "kernel_ms": kern_ms, "algorithmic_flops_per_launch": flops},
        "simulate_ms": sim_ms, "simulate_GBps": sim_bytes(N, n, d) / (sim_ms / 1e3) / 1e9,
    }
    return out


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a) -> int:
    """`--gpus N` (N > 1) without a torch.distributed.run rendezvous: start one as a CHILD process
    (python -m torch.distributed.run --nproc-per-node N bench.py <same args>), before this process
    touches the GPU, and hand back its exit code. The ranks inherit stdout, so rank 0's JSON line is
    this command's line. The reference gets its device count from pmap over all local devices
    (core/trainer.py:44-53); here one process per GPU is started explicitly."""
    port = os.environ.get("MASTER_PORT") or str(free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"bench.py: launching {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main():
    a = parse()
    if os.environ.get("PDEINV_BENCH_WATCHDOG"):  # tests: a stuck rank dumps its Python stacks and exits
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["PDEINV_BENCH_WATCHDOG"]), exit=True)
    if a.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {a.gpus})")
    env_ws = os.environ.get("WORLD_SIZE")
    if env_ws is None and a.gpus > 1:
        sys.exit(launch_ranks(a))
    if env_ws is not None and int(env_ws) != a.gpus:
        sys.exit(f"bench.py: launched with WORLD_SIZE={env_ws} but --gpus {a.gpus}; refusing to report a line "
                 f"whose n_gpus would not match the ranks that ran")
    backend = os.environ.get("PDEINV_DIST_BACKEND", "nccl")
    if backend == "nccl" and a.gpus > max(1, torch.cuda.device_count()):
        sys.exit(f"bench.py: --gpus {a.gpus} but {torch.cuda.device_count()} visible GPUs (RCCL needs one GPU per "
                 f"rank; PDEINV_DIST_BACKEND=gloo shares a GPU for tests)")
    dist.init_from_env("nccl")
    rank, world = dist.rank(), dist.world_size()
    ranks_seen = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    if ranks_seen != a.gpus:
        sys.exit(f"bench.py: {ranks_seen} ranks joined but --gpus {a.gpus}")
    local = dist.local_device()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    native.lib()
    out = {"C2": run_c2, "C3": run_c3, "C4": run_c4, "C5": run_c5}[a.config](a, rank, world, dev)
    out["roofline"].update(KERN_STATS)
    out["ranks_seen"] = ranks_seen
    out["backend"] = torch.distributed.get_backend() if torch.distributed.is_initialized() else "none (one process)"
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_distributed():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
