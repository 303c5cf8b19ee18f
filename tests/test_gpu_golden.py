"""GPU kernels against the committed golden fixtures (tests/golden, made by oracle/make_golden.py).
Tolerances: trajectories 1e-5 of the state scale after 100 steps (GMM 5e-5: softmax via v_exp_f32);
tau bit-exact; residuals 1e-4 relative; gradients vs central differences 1e-3."""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device="cuda")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "sde_*.npz"))), ids=os.path.basename)
def test_sde_kernel_vs_golden(native, path):
    g = np.load(path)
    kind = str(g["kind"])
    P = g["params"]
    pot = (dict(kind=native.POT_QUADRATIC, params=P) if kind == "quadratic"
           else dict(kind=native.POT_GMM, params=P, n_centers=P.shape[0], sigma=1.0))
    n = g["xi"].shape[0] - 1
    r = native.sde_simulate(_t(g["z0"]), n, float(g["dt"]), float(g["gamma"]), pot, seed=0, noise=_t(g["xi"]),
                            shift_u=_t(g["u"]))
    tol = 1e-5 if kind == "quadratic" else 5e-5
    scale = np.abs(g["traj"]).max() + 1
    assert np.max(np.abs(r["traj"].cpu().numpy()[g["keep"]] - g["traj"])) / scale < tol
    assert np.max(np.abs(r["last"].cpu().numpy() - g["last"])) / scale < tol
    assert np.array_equal(r["tau"].cpu().numpy(), g["tau"])


def test_kfp_quadratic_kernel_vs_golden(native):
    g = np.load(os.path.join(GOLD, "kfp_quadratic.npz"))
    mom = torch.stack([native.moments(_t(g[k])) for k in ("zi", "z0", "zt")])
    out, grad = native.residual_kfp_quadratic(mom, _t(np.concatenate([g["K"].ravel(), g["b"]])), g["F"], 1.0, 2.0)
    out = out.cpu().numpy()
    assert abs(out[0] - g["loss"]) < 1e-4 * (1 + abs(g["loss"]))
    assert abs(out[1] - g["loss_gt"]) < 1e-4 * (1 + abs(g["loss_gt"]))
    assert np.allclose(grad.cpu().numpy(), g["grad"], rtol=1e-3, atol=1e-3)


def test_kfp_gmm_kernel_vs_golden(native):
    g = np.load(os.path.join(GOLD, "kfp_gmm.npz"))
    K, d = g["mus"].shape
    dk = native.kfp_gmm_desc(d, K, g["mus_true"], 0.5, 2.0, len(g["zi"]), len(g["zt"]), len(g["z0"]))
    acc = native.residual_kfp_gmm(dk, _t(g["zi"]), _t(g["zt"]), _t(g["z0"]), _t(g["mus"]))
    out, grad = native.residual_kfp_gmm_finalize(dk, acc)
    out = out.cpu().numpy()
    assert abs(out[0] - g["loss"]) < 1e-4 * (1 + abs(g["loss"]))
    assert abs(out[4] - g["hessian"]) < 1e-4 * (1 + abs(g["hessian"]))
    assert np.allclose(grad.cpu().numpy(), g["grad"], rtol=1e-3, atol=1e-4)


def test_kmv_kernels_vs_golden(native):
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    from oracle import numpy_ref as nr
    g = np.load(os.path.join(GOLD, "kmv_pairwise.npz"))
    x, v, tau = g["x"], g["v"], g["tau"]
    n, n_t, d = x.shape
    z = _t(np.concatenate([x, v], -1).reshape(-1, 2 * d))
    cfg = nr.ou_configuration(g["F"])
    mom = native.moments_batched(z, n_t, n, 2 * d, 2 * d, n_t * 2 * d)
    coef = _t(dlogrho_coefficients(tau, cfg, d))
    wst, _ = native.kmv_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d)
    out, grad = native.residual_kmv(mom, wst, _t(np.concatenate([g["K"].ravel(), g["b"]])), g["F"], 1.0)
    out = out.cpu().numpy()
    assert abs(out[0] - g["loss"]) < 1e-4 * (1 + abs(g["loss"]))
    assert abs(out[1] - g["loss_gt"]) < 1e-4 * (1 + abs(g["loss_gt"]))
    assert np.allclose(grad.cpu().numpy(), g["grad"], rtol=1e-3, atol=1e-3)


def test_dlogrho_kernel_vs_golden(native):
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    from oracle import numpy_ref as nr
    g = np.load(os.path.join(GOLD, "dlogrho_d10.npz"))
    d = g["x"].shape[1]
    coef = _t(dlogrho_coefficients([float(g["s"])], nr.ou_configuration(g["F"]), d))
    _, ds = native.kmv_weights(d, 1.0, coef, _t(g["x"]), 1, len(g["x"]), 0, d, want_ds=True)
    ds = ds[0].double().cpu().numpy()
    assert np.max(np.abs(ds[:, 0] - g["ds"]) / (1 + np.abs(g["ds"]))) < 1e-4
    assert np.max(np.abs(ds[:, 1] - g["ds2"]) / (1 + np.abs(g["ds2"]))) < 1e-3
