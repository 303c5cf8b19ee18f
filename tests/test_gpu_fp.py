"""GPU parity tests of the overdamped Fokker–Planck path (the reference's default pde_instance):
the exact per-sample-time sampler and the Laplacian residual with its parameter gradient, through
the C ABI, against the fp64 restatement in oracle/numpy_ref.py.

Tolerances: sampler moments within 5 sigma of the Monte-Carlo estimate (+ fp32 rounding);
residual loss / loss ground truth 1e-3 relative, gradient 2e-3 of its largest entry (fp32
accumulation over rows, as for the kinetic MLP residual)."""
import numpy as np
import pytest
import torch

from oracle import numpy_ref as nr
from utils import prng

pytestmark = pytest.mark.gpu
DEV = "cuda"
LIB, FUSED = 1, 2


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


def _eig(cfg):
    return {"U": cfg["U"], "s": cfg["s"], "Um0": cfg["U"].T @ cfg["m_0"], "B0": cfg["B_0"], "B": cfg["B"]}


@pytest.mark.parametrize("d,t", [(4, 0.0), (4, 0.37), (2, 2.0), (8, 1.1)])
def test_fp_exact_sample_fixed_time_moments(native, d, t):
    cfg = nr.fp_configuration(nr.problem_constants(d))
    n = 1 << 18
    x, ts = native.fp_exact_sample(n, _eig(cfg), seed=5, t_range=t, return_t=True)
    x = x.double().cpu().numpy()
    assert np.all(ts.cpu().numpy() == np.float32(t))
    m, P = nr.fp_mean_cov(t, cfg)
    sd_m = np.sqrt(np.diag(P) / n)
    assert np.all(np.abs(x.mean(0) - m) < 5 * sd_m + 1e-5 * (1 + np.abs(m)))
    C = np.cov(x.T)
    sd_C = np.sqrt((np.diag(P)[:, None] * np.diag(P)[None, :] + P ** 2) / n)
    assert np.all(np.abs(C - P) < 5 * sd_C + 1e-5 * (1 + np.abs(P).max()))


def test_fp_exact_sample_time_stream(native):
    """t_r = t_lo + u_r (t_hi - t_lo), u_r from Philox ctr {row, counter_offset, 0x10000000}."""
    cfg = nr.fp_configuration(nr.problem_constants(3))
    seed, ctr, off = 0x1234_5678_9ABC, 7, 100
    _, ts = native.fp_exact_sample(300, _eig(cfg), seed=seed, t_range=(1e-4, 2.0), counter_offset=ctr,
                                   row_offset=off, return_t=True)
    ts = ts.cpu().numpy()
    for r in (0, 1, 77, 299):
        g = off + r
        u = prng.philox4x32_10((g & 0xFFFFFFFF, g >> 32, ctr, 0x10000000), (seed & 0xFFFFFFFF, seed >> 32))[0]
        want = np.float32(np.float32((u >> 8) * 2.0 ** -24) * np.float32(2.0 - np.float32(1e-4)) + np.float32(1e-4))
        assert abs(ts[r] - want) <= 2 * np.spacing(want)
    assert ts.min() >= np.float32(1e-4) and ts.max() <= 2.0


@pytest.mark.parametrize("dims,impl,chunk", [([3, 20, 20, 40], LIB, 1 << 18), ([4, 32, 32, 40], FUSED, 700),
                                             ([2, 64, 64, 64, 5], FUSED, 1 << 18), ([4, 32, 32, 40], LIB, 500)])
def test_fp_residual_vs_restatement(native, dims, impl, chunk):
    rng = np.random.default_rng(dims[1] + len(dims))
    d = dims[0]
    flat = np.concatenate([np.concatenate([rng.standard_normal((dims[i], dims[i + 1])).ravel() * np.sqrt(1.0 / dims[i]),
                                           0.1 * rng.standard_normal(dims[i + 1])]) for i in range(len(dims) - 1)])
    P = nr.mlp_unflat(flat, dims)
    F = nr.problem_constants(d)
    xi, xt, x0 = (rng.standard_normal((m, d)).astype(np.float32) for m in (500, 300, 900))
    acc, grad = native.residual_fp_mlp(dims, _t(flat), _t(xi), _t(xt), _t(x0), tilde_F=F, total_time=2.0,
                                       chunk_rows=chunk, impl=impl)
    out = native.kfp_terms_finalize(acc, grad, 0.0).cpu().numpy()
    loss, loss_gt, parts = nr.fp_mlp_loss(P, xi, xt, x0, F, 2.0)
    g_ref = nr.mlp_flat(nr.fp_mlp_grad_analytic(P, xi, xt, x0, 2.0))
    assert abs(out[0] - loss) < 1e-3 * (1 + abs(loss)), (out[0], loss)
    assert abs(out[1] - loss_gt) < 1e-3 * (1 + abs(loss_gt))
    a = acc.cpu().numpy()
    assert abs(a[6] - parts["initial"]) < 1e-3 * (1 + abs(parts["initial"]))
    assert abs(a[7] - parts["terminal"]) < 1e-3 * (1 + abs(parts["terminal"]))
    assert abs(d * a[3] - parts["laplacian"]) < 1e-3 * (1 + abs(parts["laplacian"]))
    g = grad.cpu().numpy()
    assert np.max(np.abs(g - g_ref)) < 2e-3 * (1 + np.abs(g_ref).max()), np.max(np.abs(g - g_ref))


def test_fp_default_config_trains(native):
    """The reference's default config (pde_instance=fokker_planck, MLP) through main.run: loss and the
    relative gradient error of test_fn fall over a short run."""
    import main as entry
    from utils import config as config_lib
    cfg = config_lib.compose("config", ["estimation_mode=non-parametric", "neural_network.hidden_dim=32",
                                        "neural_network.layers=2", "train.optimizer.learning_rate.initial=1e-2",
                                        "solver.train.batch_size_0T=20000", "solver.train.batch_size_init=5000",
                                        "solver.train.batch_size_terminal=5000", "test.frequency=50"])
    trainer, _ = entry.run(cfg, log_path=None, number_of_iterations=150)
    h = trainer.history
    first = next(r for r in h if "relative error of gradient estimation initial" in r)
    last = [r for r in h if "relative error of gradient estimation initial" in r][-1]
    assert last["loss ground truth"] < 0.5 * h[0]["loss ground truth"]
    assert last["relative error of gradient estimation terminal"] < first["relative error of gradient estimation terminal"]
    assert np.isfinite(last["loss"])
