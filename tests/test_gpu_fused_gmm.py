"""The GMM simulator with the KFP-GMM residual fused in (pdeinv_sde_simulate_kfp_gmm; BASELINE config
C3's online iteration: …_GMM.py:104-142 simulate, kinetic_fokker_planck.py:11-69 over init = z0,
0T = every trajectory row, terminal = last).

Checked against (a) the same simulator's trajectory fed to the standalone residual kernel (fp32
reassociation only: loss 1e-5 relative, gradient 1e-4 of its scale) and (b) the fp64 restatement of the
loss and of its analytic adjoint (oracle/numpy_ref.py kfp_gmm_loss / kfp_gmm_grad_analytic, the latter
FD-checked in tests/test_oracle.py) on the explicit-noise trajectory of the C oracle (loss 1e-4 relative,
gradient 1e-3 of its scale)."""
import numpy as np
import pytest
import torch

from oracle import numpy_ref as nr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


@pytest.mark.parametrize("d,K,Km,N,n", [(4, 8, 8, 3001, 50), (2, 3, 5, 1000, 30), (8, 8, 8, 700, 20),
                                        (4, 3, 3, 4096, 100)])
def test_fused_gmm_residual_equals_simulate_then_residual(native, d, K, Km, N, n):
    rng = np.random.default_rng(d * 100 + K)
    mus_true = nr.gmm_centres(d, K)
    pot = dict(kind=native.POT_GMM, params=mus_true, n_centers=K, sigma=1.0)
    z0 = _t(np.concatenate([2 * rng.standard_normal((N, d)), 0.3 * rng.standard_normal((N, d))], 1))
    mus = _t(rng.standard_normal((Km, d)))
    gamma, T = 0.5, 2.0
    desc = native.kfp_gmm_desc(d, Km, mus_true, gamma, T, N, N, N * n)
    kw = dict(seed=0x5EED_0003, counter_offset=11)
    f = native.sde_simulate_kfp_gmm(z0, n, T / n, gamma, pot, desc, mus, **kw)
    s = native.sde_simulate(z0, n, T / n, gamma, pot, **kw)
    assert torch.equal(f["traj"], s["traj"]) and torch.equal(f["last"], s["last"]) and torch.equal(f["tau"], s["tau"])
    acc = native.residual_kfp_gmm(desc, z0, s["last"], s["traj"].view(-1, 2 * d), mus)
    a, b = f["acc"].cpu().numpy(), acc.cpu().numpy()
    assert np.allclose(a[:8], b[:8], rtol=1e-5, atol=1e-6 * np.abs(b[:8]).max()), (a[:8], b[:8])
    assert np.max(np.abs(a[8:] - b[8:])) < 1e-4 * np.abs(b[8:]).max()
    out_f, g_f = native.residual_kfp_gmm_finalize(desc, f["acc"])
    out_s, g_s = native.residual_kfp_gmm_finalize(desc, acc)
    assert np.allclose(out_f.cpu().numpy(), out_s.cpu().numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("d,K,Km", [(4, 8, 8), (3, 2, 4)])
def test_fused_gmm_residual_vs_restatement(native, oracle_lib, d, K, Km):
    N, n, gamma, T = 800, 40, 0.5, 2.0
    rng = np.random.default_rng(K + Km)
    mus_true = nr.gmm_centres(d, K)
    z0 = np.concatenate([2 * rng.standard_normal((N, d)), 0.3 * rng.standard_normal((N, d))], 1).astype(np.float32)
    xi = rng.standard_normal((n + 1, N, d)).astype(np.float32)
    u = rng.random(N).astype(np.float32)
    mus = rng.standard_normal((Km, d))
    pot = dict(kind=native.POT_GMM, params=mus_true, n_centers=K, sigma=1.0)
    desc = native.kfp_gmm_desc(d, Km, mus_true, gamma, T, N, N, N * n)
    f = native.sde_simulate_kfp_gmm(_t(z0), n, T / n, gamma, pot, desc, _t(mus), seed=0, noise=_t(xi), shift_u=_t(u))
    o = oracle_lib.sde_simulate(z0, n, T / n, gamma, "gmm", mus_true.astype(np.float32), n_centers=K, sigma=1.0,
                                noise=xi, shift_u=u)
    z0T = o["traj"].reshape(-1, 2 * d)
    loss, loss_gt, parts = nr.kfp_gmm_loss(mus, z0, o["last"], z0T, mus_true, gamma, T)
    G = nr.kfp_gmm_grad_analytic(mus, z0, o["last"], z0T, mus_true, gamma, T)
    out, grad = native.residual_kfp_gmm_finalize(desc, f["acc"])
    out = out.cpu().numpy()
    assert abs(out[0] - loss) < 1e-4 * (1 + abs(loss)), (out[0], loss)
    assert abs(out[1] - loss_gt) < 1e-4 * (1 + abs(loss_gt))
    assert abs(out[4] - parts["hessian"]) < 1e-4 * (1 + abs(parts["hessian"]))
    assert np.max(np.abs(grad.cpu().numpy() - G)) < 1e-3 * (1 + np.abs(G).max())


def test_fused_gmm_residual_rejects_a_different_true_potential(native):
    d, K = 4, 3
    pot = dict(kind=native.POT_GMM, params=nr.gmm_centres(d, K), n_centers=K, sigma=1.0)
    other = nr.gmm_centres(d, K) + 0.5
    desc = native.kfp_gmm_desc(d, K, other, 0.5, 2.0, 10, 10, 100)
    with pytest.raises(ValueError):
        native.sde_simulate_kfp_gmm(_t(np.zeros((10, 8))), 10, 0.2, 0.5, pot, desc, _t(np.zeros((K, d))), seed=1)
