"""Multi-rank paths on the one GPU of a test box: several ranks launched by
torch.distributed.run share cuda:0 with the gloo backend (PDEINV_DIST_BACKEND=gloo; RCCL needs one
GPU per rank, the call sites are the same).

* McKean–Vlasov simulator (d = 8, the C4 dimension), both drivers: the fused one (one all-reduce per
  simulate of [count, sum z0, the noise sums of every update]) and the per-update exchange (one
  all-reduce of [count, sum x] per update). The Philox counter is the global particle id and the mean
  field is the all-reduced ensemble mean, so the 2- and 3-rank trajectories must equal the 1-rank
  trajectory of the whole ensemble (up to the fp64 summation order of the partial sums: 2e-5 after 31
  updates).
* bench.py --gpus 2 (the driver's scaling launch): one JSON line, n_gpus = 2, value = both ranks'
  particle-updates / the max-over-ranks step time — for the headline C2 and for C4 / C5.
* The data-parallel KFP residual reports what the reference's pmap branch reports (trainer.py:44-53:
  every output averaged over devices): loss and grad the means of the per-shard values, and grad_norm
  the MEAN OF PER-SHARD NORMS (not the norm of the mean gradient).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(nproc, args, port, timeout=180, rccl=False):
    env = dict(os.environ)
    if rccl:  # one rank on the one GPU, over RCCL, with the distributed path forced at world size 1
        env.pop("PDEINV_DIST_BACKEND", None)
        env.update(PDEINV_DIST_FORCE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    else:
        env["PDEINV_DIST_BACKEND"] = "gloo"
    env.setdefault("PDEINV_BENCH_WATCHDOG", str(max(30, timeout - 30)))  # bench.py: stuck ranks dump stacks
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}"] + args
    return subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)


def _gather(out_dir, world):
    parts = [dict(np.load(os.path.join(out_dir, f"rank{r}.npz"))) for r in range(world)]
    traj = np.concatenate([p["traj"] for p in parts], axis=1)
    last = np.concatenate([p["last"] for p in parts], axis=0)
    return traj, last, parts[0]["xsum"]


@pytest.mark.parametrize("exchange,port0", [("fused", 29611), ("per_update", 29621)])
def test_mean_field_simulator_is_rank_count_invariant(native, tmp_path, exchange, port0):
    ref_dir = tmp_path / "w1"
    ref_dir.mkdir()
    worker = [os.path.join(ROOT, "tests", "mp_gpu_worker.py"), "mean_field"]
    r = subprocess.run([sys.executable] + worker + [str(ref_dir), exchange],
                       cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    t1, l1, x1 = _gather(ref_dir, 1)
    for world, port in ((2, port0), (3, port0 + 1)):
        d = tmp_path / f"w{world}"
        d.mkdir()
        r = _launch(world, worker + [str(d), exchange], port)
        assert r.returncode == 0, r.stderr[-3000:]
        tw, lw, xw = _gather(d, world)
        scale = 1 + np.abs(t1).max()
        assert np.max(np.abs(tw - t1)) < 2e-5 * scale, (world, np.max(np.abs(tw - t1)))
        assert np.max(np.abs(lw - l1)) < 2e-5 * scale
        assert np.allclose(xw, x1, rtol=1e-6, atol=1e-6 * np.abs(x1).max())


def test_bench_two_ranks(native):
    r = _launch(2, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                    "--particles", "65536", "--no-cpu-baseline", "--no-recovery"], 29613)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["particles_per_gpu"] == 65536
    assert abs(out["value"] * out["ms_per_step"] / 1e3 - 2 * 65536 * 101) < 1e-6 * out["value"]


def test_bench_plain_gpus2_launches_two_ranks(native):
    """A plain `python bench.py --gpus 2` (no torch.distributed.run around it, as the driver may issue it)
    starts the 2-rank rendezvous itself (a child process, before any GPU call) and the line reports the
    ranks that really ran (gloo override: both ranks share the test box's one GPU)."""
    env = dict(os.environ, PDEINV_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--particles", "65536", "--no-cpu-baseline", "--no-recovery"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == out["ranks_seen"] == 2 and out["backend"] == "gloo", out
    assert abs(out["value"] * out["ms_per_step"] / 1e3 - 2 * 65536 * 101) < 1e-6 * out["value"]
    ks = out["roofline"]
    assert ks["kernel_ms_min"] <= ks["kernel_ms_median"] <= ks["kernel_ms_max"]


def test_bench_mismatched_launch_fails(native):
    """torch.distributed.run with 2 ranks but --gpus 1: bench.py refuses to print a line (non-zero exit)."""
    r = _launch(2, [os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
                    "--particles", "65536", "--no-cpu-baseline", "--no-recovery"], 29619, timeout=120)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")], r.stdout[-2000:]


@pytest.mark.parametrize("config,port,n", [("C4", 29615, 65536), ("C5", 29617, 65536)])
def test_bench_two_ranks_c4_c5(native, config, port, n):
    """The driver's 8-GPU scaling launch runs every config through the same code: world-2 bench.py
    --config C4 (closed-form McKean-Vlasov: the mean-path and KMV all-reduces) and C5 (MLP residual +
    its gradient all-reduce) print one line with both ranks' particle-updates."""
    r = _launch(2, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", config, "--steps", "2", "--warmup", "1",
                    "--particles", str(n), "--no-cpu-baseline", "--no-recovery"], port, timeout=150)  # ~10 s when healthy: a stuck rendezvous fails fast
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["particles_per_gpu"] == n
    assert abs(out["value"] * out["ms_per_step"] / 1e3 - 2 * n * 101) < 1e-6 * out["value"]


def test_bench_strong_scaling_c4_two_ranks(native):
    """bench.py --scaling strong (strong scaling for C4): a fixed job total — odd here, so the
    two contiguous shares differ by one particle — split over the ranks; value = total x (n + 1) / step time."""
    total = 100_003
    r = _launch(2, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C4", "--scaling", "strong",
                    "--particles-total", str(total), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                    "--no-recovery"], 29625, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["scaling"] == "strong" and out["n_gpus"] == 2 and out["config"]["particles_total"] == total
    assert out["config"]["particles_per_gpu"] == total // 2 + 1  # rank 0's share
    assert abs(out["value"] * out["ms_per_step"] / 1e3 - total * 101) < 1e-6 * out["value"]


def test_kmv_stamp_sums_route_is_rank_count_invariant(native, tmp_path):
    """The McKean-Vlasov SDE product route (the simulator's own KMV stamp sums, no trajectory) over 2 ranks equals
    the 1-rank run of the whole ensemble: the same stamps, the last states after concatenation to 2e-5 (ids are
    rank-invariant; the mean field's fp64 partial sums add in another order), loss / ground truth / gradient from
    the all-reduced stamp sums to the fp32 partial-sum order (1e-5 relative)."""
    worker = [os.path.join(ROOT, "tests", "mp_gpu_worker.py"), "kmv_stamp_sums"]
    ref = tmp_path / "w1"
    ref.mkdir()
    r = subprocess.run([sys.executable] + worker + [str(ref)], cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    a = dict(np.load(ref / "rank0.npz"))
    w2 = tmp_path / "w2"
    w2.mkdir()
    r = _launch(2, worker + [str(w2)], 29661)
    assert r.returncode == 0, r.stderr[-3000:]
    parts = [dict(np.load(w2 / f"rank{k}.npz")) for k in range(2)]
    assert all(int(p["world"]) == 2 for p in parts)
    assert np.array_equal(parts[0]["tau"], a["tau"])
    assert np.allclose(np.concatenate([p["last"] for p in parts]), a["last"], rtol=0, atol=2e-5)
    for p in parts:
        for k in ("loss", "loss_gt"):
            assert abs(float(p[k]) - float(a[k])) < 1e-5 * (1 + abs(float(a[k]))), (k, p[k], a[k])
        assert np.abs(p["grad"] - a["grad"]).max() < 1e-5 * (1 + np.abs(a["grad"]).max())


def test_dp_residual_matches_pmap_mean_of_shards(native, tmp_path):
    """2 ranks (gloo) vs the two shards evaluated one at a time: loss and grad = the shard means,
    grad_norm = the mean of the shard gradients' norms (trainer.py:44-53), for the quadratic, GMM and
    MLP models of the KFP residual; and the shared-clock KMV residual (pooled moments). Tolerance 1e-5
    relative (fp32 terms, fp64 all-reduce)."""
    worker = [os.path.join(ROOT, "tests", "mp_gpu_worker.py"), "dp_residual"]
    ref_dir, d2 = tmp_path / "shards", tmp_path / "w2"
    ref_dir.mkdir()
    d2.mkdir()
    r = subprocess.run([sys.executable] + worker + [str(ref_dir), "2"], cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _launch(2, worker + [str(d2), "0"], 29641, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    ref = dict(np.load(os.path.join(ref_dir, "rank0.npz")))
    got = [dict(np.load(os.path.join(d2, f"rank{k}.npz"))) for k in range(2)]
    kinds = ("Quadratic_mlp", "Quadratic_quadratic", "GMM_mlp", "GMM_gmm")
    for kind in kinds:
        loss = np.mean([ref[f"{kind}_{r}_loss"] for r in range(2)])
        grad = np.mean([ref[f"{kind}_{r}_grad"] for r in range(2)], axis=0)
        gnorm = np.mean([np.linalg.norm(ref[f"{kind}_{r}_grad"]) for r in range(2)])
        assert abs(gnorm - np.linalg.norm(grad)) > 1e-4 * gnorm, kind  # the two definitions differ here
        for k in range(2):  # both ranks return the same (all-reduced) values, each rank's own shard key
            g = got[k]
            assert abs(g[f"{kind}_{k}_loss"] - loss) < 1e-5 * (1 + abs(loss)), (kind, g[f"{kind}_{k}_loss"], loss)
            assert abs(g[f"{kind}_{k}_grad_norm"] - gnorm) < 1e-5 * (1 + gnorm), (kind, g[f"{kind}_{k}_grad_norm"], gnorm)
            assert np.abs(g[f"{kind}_{k}_grad"] - grad).max() < 1e-5 * (1 + np.abs(grad).max()), kind
    # KMV with a shared clock: loss / grad = the residual of the union of both ranks' particles (pooled
    # per-stamp moments: the moments enter the KMV loss nonlinearly, so this is NOT the mean of the shard
    # losses), grad_norm = the mean of the per-rank norms on rank-local moments (trainer.py:44-53)
    kind = "KMV_quadratic"
    loss, grad = ref[f"{kind}_all_loss"], ref[f"{kind}_all_grad"]
    gnorm = np.mean([np.linalg.norm(ref[f"{kind}_{r}_grad"]) for r in range(2)])
    assert abs(loss - np.mean([ref[f"{kind}_{r}_loss"] for r in range(2)])) > 1e-5 * (1 + abs(loss))  # pooled != mean
    for k in range(2):
        g = got[k]
        assert abs(g[f"{kind}_{k}_loss"] - loss) < 1e-5 * (1 + abs(loss)), (g[f"{kind}_{k}_loss"], loss)
        assert abs(g[f"{kind}_{k}_grad_norm"] - gnorm) < 1e-5 * (1 + gnorm), (g[f"{kind}_{k}_grad_norm"], gnorm)
        assert np.abs(g[f"{kind}_{k}_grad"] - grad).max() < 1e-5 * (1 + np.abs(grad).max())


@pytest.mark.parametrize("exchange,port", [("fused", 29631), ("per_update", 29632)])
def test_mean_field_over_rccl_world1(native, tmp_path, exchange, port):
    """The RCCL data path executes: one rank under torch.distributed.run with the nccl backend and the
    distributed path forced (PDEINV_DIST_FORCE=1), so every all-reduce call site of the McKean–Vlasov
    drivers runs through RCCL; the result equals the plain single-process run (a one-rank all-reduce
    is the identity, so bit-for-bit up to nothing)."""
    worker = [os.path.join(ROOT, "tests", "mp_gpu_worker.py"), "mean_field"]
    ref_dir, d = tmp_path / "plain", tmp_path / "rccl"
    ref_dir.mkdir()
    d.mkdir()
    r = subprocess.run([sys.executable] + worker + [str(ref_dir), exchange],
                       cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _launch(1, worker + [str(d), exchange], port, rccl=True)
    assert r.returncode == 0, r.stderr[-3000:]
    assert str(np.load(os.path.join(d, "rank0.npz"))["backend"]) == "nccl"
    t1, l1, x1 = _gather(ref_dir, 1)
    tr, lr, xr = _gather(d, 1)
    assert np.array_equal(tr, t1) and np.array_equal(lr, l1) and np.array_equal(xr, x1)


def test_bench_over_rccl_world1(native):
    """bench.py's headline step with its residual all-reduce carried by RCCL (one rank, forced path)."""
    r = _launch(1, [os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
                    "--particles", "65536", "--no-cpu-baseline", "--no-recovery"], 29633, rccl=True)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["value"] > 0 and np.isfinite(out["loss"])
