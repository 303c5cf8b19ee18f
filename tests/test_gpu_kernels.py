"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Tolerances (fp32 path vs fp32/fp64 restatement):
  * Philox bits, tau, gathers: bit-exact;
  * normals: |GPU - oracle| <= 2e-6 * (1 + |z|) (hardware v_log/v_sin vs libm, both fp32-rounded);
  * explicit-noise trajectories after 100 steps: rtol = atol = 1e-5 vs the fp64 restatement
    scaled by the state magnitude;
  * Philox-mode trajectories vs the C oracle: 1e-4 abs (normals differ in the last ulps);
  * moments / residuals: 1e-5 relative (fp32 accumulation, fp64 across blocks).
"""
import math

import numpy as np
import pytest
import torch

from oracle import numpy_ref as nr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=DEV)


def test_runtime_shared_with_torch(native):
    v = native.lib().pdeinv_runtime_version()
    assert v > 0


@pytest.mark.parametrize("cz,cw", [(0, 0), (5, 3), (0xFFFFFFFF, 0x80000000)])
def test_philox_bits_exact(native, oracle_lib, cz, cw):
    seed = 0x0123456789ABCDEF
    n = 4099
    g = native.philox_fill(seed, cz, cw, n).cpu().numpy().view(np.uint32)
    o = oracle_lib.philox_fill(seed, cz, cw, n)
    assert np.array_equal(g, o)


def test_philox_kat_through_gpu(native):
    g = native.philox_fill(0, 0, 0, 1).cpu().numpy().view(np.uint32)[0]
    assert [hex(x) for x in g] == ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]


@pytest.mark.parametrize("d", [1, 2, 3, 4, 8])
def test_sde_explicit_noise_vs_restatement(native, d):
    rng = np.random.default_rng(d)
    N, n, T = 333, 100, 2.0
    dt = T / n
    F = nr.problem_constants(d)
    z0 = rng.standard_normal((N, 2 * d)).astype(np.float32)
    xi = rng.standard_normal((n + 1, N, d)).astype(np.float32)
    u = rng.random(N).astype(np.float32)
    res = native.sde_simulate(_t(z0), n, dt, 1.0, dict(kind=native.POT_QUADRATIC, params=F), seed=1,
                              noise=_t(xi), shift_u=_t(u))
    torch.cuda.synchronize()
    last, traj, tau = nr.sde_scan(z0, n, dt, 1.0, nr.grad_quadratic(F), xi, u)
    scale = np.abs(traj).max(axis=(0, 2), keepdims=True) + 1.0
    assert np.max(np.abs(res["traj"].cpu().numpy() - traj) / scale) < 1e-5
    assert np.max(np.abs(res["last"].cpu().numpy() - last) / (np.abs(last).max(1, keepdims=True) + 1)) < 1e-5
    # tau = tau0 + s*dt with two fp32 roundings: bit-exact against the fp32 restatement
    _, _, tau32 = nr.sde_scan(z0, n, dt, 1.0, nr.grad_quadratic(F), xi, u, dtype=np.float32)
    assert np.array_equal(res["tau"].cpu().numpy(), tau32)


@pytest.mark.parametrize("d,K", [(2, 3), (4, 3), (4, 8), (8, 8)])
def test_sde_gmm_explicit_noise(native, d, K):
    rng = np.random.default_rng(10 + d + K)
    N, n, T = 257, 100, 2.0
    dt = T / n
    mus = nr.gmm_centres(d, K)
    z0 = np.concatenate([2 * rng.standard_normal((N, d)), 0.3 * rng.standard_normal((N, d))], 1).astype(np.float32)
    xi = rng.standard_normal((n + 1, N, d)).astype(np.float32)
    u = rng.random(N).astype(np.float32)
    res = native.sde_simulate(_t(z0), n, dt, 0.5, dict(kind=native.POT_GMM, params=mus, n_centers=K, sigma=1.0),
                              seed=1, noise=_t(xi), shift_u=_t(u))
    last, traj, _ = nr.sde_scan(z0, n, dt, 0.5, nr.grad_gmm(mus), xi, u)
    scale = np.abs(traj).max(axis=(0, 2), keepdims=True) + 1.0
    assert np.max(np.abs(res["traj"].cpu().numpy() - traj) / scale) < 1e-4


@pytest.mark.parametrize("d", [2, 4, 8])
def test_sde_philox_vs_c_oracle(native, oracle_lib, d):
    rng = np.random.default_rng(100 + d)
    N, n, T = 1000, 100, 2.0
    dt = T / n
    F = nr.problem_constants(d)
    z0 = rng.standard_normal((N, 2 * d)).astype(np.float32)
    seed, off, poff = 0xDEADBEEF12345, 77, 5_000_000_000
    res = native.sde_simulate(_t(z0), n, dt, 1.0, dict(kind=native.POT_QUADRATIC, params=F), seed=seed,
                              counter_offset=off, particle_offset=poff)
    o = oracle_lib.sde_simulate(z0, n, dt, 1.0, "quadratic", F, seed=seed, counter_offset=off,
                                particle_offset=poff)
    assert np.array_equal(res["tau"].cpu().numpy(), o["tau"])  # same shift stream, same fp32 ops
    assert np.max(np.abs(res["traj"].cpu().numpy() - o["traj"])) < 2e-4
    assert np.max(np.abs(res["last"].cpu().numpy() - o["last"])) < 2e-4


@pytest.mark.parametrize("poff", [(1 << 32) - 128, (1 << 32) - 100, (1 << 33) + 3, 0])
@pytest.mark.parametrize("kind", ["quadratic", "gmm"])
def test_sde_philox_id_high_word(native, oracle_lib, poff, kind):
    """Particle ids across a multiple of 2^32: the uniform-high-word kernel (64-aligned offsets or
    no crossing) and the general one (unaligned + crossing) draw the oracle's stream."""
    d, N, n = 4, 700, 20
    rng = np.random.default_rng(7)
    z0 = rng.standard_normal((N, 2 * d)).astype(np.float32)
    if kind == "quadratic":
        params, pot = nr.problem_constants(d), dict(kind=native.POT_QUADRATIC)
        pot["params"] = params
        ok = {}
    else:
        params = rng.uniform(-2, 2, (3, d)).astype(np.float32)
        pot = dict(kind=native.POT_GMM, params=params, n_centers=3, sigma=1.0)
        ok = dict(n_centers=3, sigma=1.0)
    res = native.sde_simulate(_t(z0), n, 0.02, 0.5, pot, seed=99, counter_offset=5, particle_offset=poff)
    o = oracle_lib.sde_simulate(z0, n, 0.02, 0.5, kind, params, seed=99, counter_offset=5, particle_offset=poff,
                                **ok)
    assert np.array_equal(res["tau"].cpu().numpy(), o["tau"])
    scale = np.abs(o["traj"]).max(axis=(0, 2), keepdims=True) + 1.0
    assert np.max(np.abs(res["traj"].cpu().numpy() - o["traj"]) / scale) < 1e-4
    assert np.max(np.abs(res["last"].cpu().numpy() - o["last"]) / scale[0]) < 1e-4


def test_sde_moments_match_discrete_chain(native):
    """Philox-mode law == exact law of the chain, 5 sigma_MC."""
    d, N, n, T = 4, 1 << 18, 100, 2.0
    dt = T / n
    F = nr.problem_constants(d)
    z0 = native.gaussian_sample(N, _t(np.zeros(2 * d)), _t(np.eye(2 * d)), seed=3)
    res = native.sde_simulate(z0, n, dt, 1.0, dict(kind=native.POT_QUADRATIC, params=F), seed=11,
                              traj=True, tau=False, last=True)
    mt, st, ml, sl = nr.em_chain_moments(F, 1.0, dt, n, np.zeros(2 * d), np.eye(2 * d))
    for s in (0, 1, 50, n - 1):
        z = res["traj"][s].double()
        emp = (z.T @ z / N).cpu().numpy()
        P = st[s]
        sig = np.sqrt((np.outer(np.diag(P), np.diag(P)) + P ** 2) / N)
        assert np.max(np.abs(emp - P) / sig) < 5.5, s
        assert np.max(np.abs(z.mean(0).cpu().numpy() - mt[s]) / np.sqrt(np.diag(P) / N)) < 5.5
    zl = res["last"].double()
    emp = (zl.T @ zl / N).cpu().numpy()
    sig = np.sqrt((np.outer(np.diag(sl), np.diag(sl)) + sl ** 2) / N)
    assert np.max(np.abs(emp - sl) / sig) < 5.5


@pytest.mark.parametrize("d", [1, 2, 4, 8])
def test_fused_moments_equal_recomputed(native, d):
    rng = np.random.default_rng(d)
    N, n = 5003, 37
    F = nr.problem_constants(d)
    z0 = _t(rng.standard_normal((N, 2 * d)))
    res = native.sde_simulate(z0, n, 0.02, 1.0, dict(kind=native.POT_QUADRATIC, params=F), seed=9,
                              moments=True)
    mom = res["moments"].cpu().numpy()
    ref = [nr.moments(z0.cpu().numpy()), nr.moments(res["traj"].cpu().numpy()),
           nr.moments(res["last"].cpu().numpy())]
    for k in range(3):
        assert np.allclose(mom[k], ref[k], rtol=2e-5, atol=1e-3 * max(1.0, ref[k][0] ** 0.5)), k


@pytest.mark.parametrize("d,N", [(4, 5003), (4, 64 * 40), (2, 777), (8, 130)])
def test_fused_moments_without_trajectory(native, d, N):
    """Moments with no trajectory output equal those of the same simulate with the trajectory written (same
    seed; the store path and the moment path are independent): full and partial waves."""
    rng = np.random.default_rng(d + N)
    F = nr.problem_constants(d)
    z0 = _t(rng.standard_normal((N, 2 * d)))
    pot = dict(kind=native.POT_QUADRATIC, params=F)
    a = native.sde_simulate(z0, 29, 0.02, 1.0, pot, seed=4, moments=True)
    b = native.sde_simulate(z0, 29, 0.02, 1.0, pot, seed=4, moments=True, traj=False, tau=False, last=False)
    assert torch.equal(a["moments"], b["moments"])
    ref = nr.moments(a["traj"].cpu().numpy())
    assert np.allclose(b["moments"][1].cpu().numpy(), ref, rtol=2e-5, atol=1e-3 * max(1.0, ref[0] ** 0.5))


@pytest.mark.parametrize("m", [2, 8, 16, 5])
def test_moments_kernel_strided(native, m):
    rng = np.random.default_rng(m)
    big = _t(rng.standard_normal((70001, m + 3)))
    view = big[:, :m]
    got = native.moments(view).cpu().numpy()
    ref = nr.moments(view.cpu().numpy())
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-2)


def test_moments_empty(native):
    got = native.moments(torch.empty((0, 8), device=DEV)).cpu().numpy()
    assert np.all(got == 0)


def test_residual_quadratic_vs_samples(native):
    d, gamma, T = 4, 1.0, 2.0
    rng = np.random.default_rng(0)
    F = nr.problem_constants(d)
    K = rng.standard_normal((d, d)).astype(np.float32)
    b = rng.standard_normal(d).astype(np.float32)
    zi, zt, z0 = (rng.standard_normal((n, 2 * d)).astype(np.float32) for n in (3000, 2000, 50000))
    mom = torch.stack([native.moments(_t(z)) for z in (zi, z0, zt)])
    theta = _t(np.concatenate([K.ravel(), b]))
    out, grad = native.residual_kfp_quadratic(mom, theta, F, gamma, T)
    out = out.cpu().numpy(); grad = grad.cpu().numpy()
    loss, loss_gt, parts = nr.kfp_quadratic_samples(K, b, zi, zt, z0, F, gamma, T)
    assert abs(out[0] - loss) < 1e-4 * (1 + abs(loss))
    assert abs(out[1] - loss_gt) < 1e-4 * (1 + abs(loss_gt))
    # gradient vs central finite differences of the per-sample restatement
    def f(theta64):
        return nr.kfp_quadratic_samples(theta64[:d * d].reshape(d, d), theta64[d * d:], zi, zt, z0, F, gamma, T)[0]
    g_fd = nr.fd_grad(f, np.concatenate([K.ravel(), b]).astype(np.float64), eps=1e-4)
    assert np.allclose(grad, g_fd, rtol=1e-4, atol=1e-3)
    assert abs(out[2] - np.linalg.norm(g_fd)) < 1e-3 * (1 + np.linalg.norm(g_fd))


@pytest.mark.parametrize("d,K,KT", [(2, 3, 3), (4, 8, 8), (4, 3, 8), (8, 8, 3)])
def test_residual_gmm_vs_restatement(native, d, K, KT):
    rng = np.random.default_rng(d * 10 + K)
    gamma, T = 0.5, 2.0
    mus_true = nr.gmm_centres(d, KT)
    mus = rng.standard_normal((K, d))
    zi = np.concatenate([2 * rng.standard_normal((1500, d)), 0.3 * rng.standard_normal((1500, d))], 1)
    zt = rng.standard_normal((1200, 2 * d)) * 1.5
    z0 = rng.standard_normal((20000, 2 * d)) * 1.5
    zi, zt, z0 = (a.astype(np.float32) for a in (zi, zt, z0))
    dk = native.kfp_gmm_desc(d, K, mus_true, gamma, T, len(zi), len(zt), len(z0))
    acc = native.residual_kfp_gmm(dk, _t(zi), _t(zt), _t(z0), _t(mus))
    out, grad = native.residual_kfp_gmm_finalize(dk, acc)
    out = out.cpu().numpy(); grad = grad.cpu().numpy()
    loss, loss_gt, parts = nr.kfp_gmm_loss(mus, zi, zt, z0, mus_true, gamma, T)
    assert abs(out[0] - loss) < 2e-4 * (1 + abs(loss))
    assert abs(out[1] - loss_gt) < 2e-4 * (1 + abs(loss_gt))
    assert abs(out[4] - parts["hessian"]) < 2e-4 * (1 + abs(parts["hessian"]))
    g_fd = nr.fd_grad(lambda th: nr.kfp_gmm_loss(th, zi, zt, z0, mus_true, gamma, T)[0], mus, eps=1e-5)
    assert np.allclose(grad, g_fd, rtol=2e-3, atol=2e-4), np.abs(grad - g_fd).max()


def test_gmm_potential(native, oracle_lib):
    rng = np.random.default_rng(5)
    d, K = 4, 8
    mus = nr.gmm_centres(d, K)
    x = (3 * rng.standard_normal((1000, d))).astype(np.float32)
    v, g = native.gmm_potential(_t(x), mus)
    vr, gr = nr.gmm_value_grad(x.astype(np.float64), mus)
    assert np.allclose(v.cpu().numpy(), vr, rtol=1e-5, atol=1e-5)
    assert np.allclose(g.cpu().numpy(), gr, rtol=1e-5, atol=1e-5)
    # far from every centre: the max-shift keeps the softmax finite
    far = _t(np.full((4, d), 40.0))
    v2, g2 = native.gmm_potential(far, mus)
    assert torch.isfinite(v2).all() and torch.isfinite(g2).all()


@pytest.mark.parametrize("m", [8, 16, 5])
def test_gaussian_sample_vs_oracle(native, oracle_lib, m):
    rng = np.random.default_rng(m)
    A = rng.standard_normal((m, m))
    cov = A @ A.T + np.eye(m)
    U, S, _ = np.linalg.svd(cov)
    ch = (U @ np.diag(np.sqrt(S)) @ U.T).astype(np.float32)
    mean = rng.standard_normal(m).astype(np.float32)
    g = native.gaussian_sample(4096, _t(mean), _t(ch), seed=42, counter_offset=3, row_offset=1000).cpu().numpy()
    o = oracle_lib.gaussian_sample(4096, mean, ch, 42, 3, 1000)
    assert np.max(np.abs(g - o)) < 2e-5 * (1 + np.abs(o).max())


def test_gaussian_sample_grouped_is_the_row_stream(native):
    """Grouped launch == per-group plain launches at the same global rows (bit-exact), and the
    KOU random-time sampler built on it reproduces each group's Gaussian."""
    rng = np.random.default_rng(7)
    G, R, m = 5, 300, 8
    means = rng.standard_normal((G, m)).astype(np.float32)
    chs = np.stack([np.linalg.cholesky(a @ a.T + np.eye(m)) for a in rng.standard_normal((G, m, m))]).astype(np.float32)
    out = native.gaussian_sample_grouped(R, _t(means), _t(chs), seed=9, counter_offset=2, row_offset=64).cpu().numpy()
    for g in range(G):
        ref = native.gaussian_sample(R, _t(means[g]), _t(chs[g]), seed=9, counter_offset=2,
                                     row_offset=64 + g * R).cpu().numpy()
        assert np.array_equal(out[g * R:(g + 1) * R], ref)
    with pytest.raises(ValueError):
        native.gaussian_sample_grouped(R, _t(means), _t(chs[:-1]), seed=9)


def test_kou_exact_random_time_sampler(native):
    """sample_ground_truth(rng, int) (…_OU.py:141-156): groups of 100 rows, each N(m(t_g), P(t_g))."""
    import registry
    from utils import config as config_lib, prng
    cfg = config_lib.compose("config", ["pde_instance=kinetic_fokker_planck", "pde_instance.domain_dim=2"])
    pi = registry.get_pde_instance(cfg)(cfg=cfg, rng=prng.PRNGKey(0))
    z = pi.sample_ground_truth(prng.PRNGKey(3), 20000).cpu().numpy()
    assert z.shape == (20000, 4) and np.isfinite(z).all()
    # pooled second moment = mean over groups of P(t_g) + m m^T; t_g ~ U(1e-4, T): compare with the
    # time-averaged continuous OU covariance (5 sigma of the 20000-sample estimate)
    cfg_o = nr.ou_configuration(pi.initial_configuration["tilde_F"])
    ts = np.linspace(1e-4, 2.0, 401)
    Pbar = np.mean([nr.ou_mean_cov(t, cfg_o)[1] for t in ts], 0)
    emp = z.T @ z / z.shape[0]
    sd = np.sqrt((np.diag(Pbar)[:, None] * np.diag(Pbar)[None, :] + Pbar ** 2) / (z.shape[0] / 100))
    assert np.all(np.abs(emp - Pbar) < 5 * sd + 1e-3)


@pytest.mark.parametrize("d", [1, 2, 4, 8, 9, 10, 12, 15, 16])
def test_ou_exact_sampler_device_moments(native, d):
    """pdeinv_ou_exact_sample (the device-resident exact KOU sampler): the drawn times lie in [t_min, t_max); the
    per-group mean and Cholesky factor equal the host closed form (ou_moments_batched, fp64 Van Loan) to fp32
    rounding — R R^T = P(t_g) to 1e-6 of the covariance scale; the rows equal pdeinv_gaussian_sample_grouped with
    those means / factors bit for bit; given times reproduce the drawn ones."""
    from example_problems.kinetic_fokker_planck_example_OU import (initialize_configuration, ou_moments_batched,
                                                                   van_loan_powers)
    ic = initialize_configuration(d)
    T, G, R = 2.0, 37, 100
    pw, s = van_loan_powers(ic, T)
    smp = native.OuExactSampler(pw, s, ic["m_0"], ic["P_0"], 1e-4, T)
    rows, t, means, fac = smp.sample(G, R, seed=123, ctr_t=5, ctr_z=9, want_moments=True)
    t64 = t.double().cpu().numpy()
    assert np.all(t64 >= 1e-4) and np.all(t64 < T) and len(np.unique(t64)) == G
    m_ref, P_ref = ou_moments_batched(t64, ic)
    scale = np.abs(P_ref).max()
    assert np.allclose(means.double().cpu().numpy(), m_ref, atol=1e-6 * scale)
    L = fac.double().cpu().numpy()
    assert np.all(np.triu(L, 1) == 0)
    assert np.max(np.abs(L @ np.transpose(L, (0, 2, 1)) - P_ref)) < 1e-6 * scale
    assert np.max(np.abs(L - np.linalg.cholesky(P_ref))) < 1e-5 * np.sqrt(scale)
    ref = native.gaussian_sample_grouped(R, means, fac, seed=123, counter_offset=9)
    assert torch.equal(rows, ref)
    assert torch.equal(smp.sample(G, R, seed=123, ctr_z=9, t=t), rows)


def test_gather_subsample_exact(native):
    rng = np.random.default_rng(1)
    n, N, m = 40, 300, 8
    traj = _t(rng.standard_normal((n, N, m)))
    ti = torch.as_tensor(rng.permutation(N)[:60], device=DEV)
    si = torch.as_tensor(np.arange(n // 5) * 5 + 2, device=DEV)
    out = native.gather_subsample(traj, ti, si).cpu().numpy()
    ref = traj.permute(1, 0, 2).cpu().numpy()[ti.cpu().numpy()][:, si.cpu().numpy(), :].reshape(-1, m)
    assert np.array_equal(out, ref)


def test_sde_edge_cases(native):
    F = nr.problem_constants(2)
    pot = dict(kind=native.POT_QUADRATIC, params=F)
    res = native.sde_simulate(torch.empty((0, 4), device=DEV), 10, 0.1, 1.0, pot, seed=1, moments=True)
    assert res["traj"].shape == (10, 0, 4) and torch.all(res["moments"] == 0)
    one = native.sde_simulate(_t(np.ones((1, 4))), 1, 0.1, 1.0, pot, seed=1)
    assert one["traj"].shape == (1, 1, 4) and torch.isfinite(one["last"]).all()
    with pytest.raises(NotImplementedError):
        native.sde_simulate(_t(np.ones((3, 22))), 5, 0.1, 1.0,
                            dict(kind=native.POT_QUADRATIC, params=np.eye(11)), seed=1)
    with pytest.raises(ValueError):
        native.sde_simulate(_t(np.ones((3, 4))), 0, 0.1, 1.0, pot, seed=1)


LIB, FUSED = 1, 2  # native.MLP_IMPL_LIBRARY / MLP_IMPL_FUSED


@pytest.mark.parametrize("dims,true_kind,chunk,impl", [
    ([2, 16, 16, 5], "gmm", 1000, LIB), ([4, 32, 32, 40], "quad", 1 << 18, LIB),
    ([8, 64, 64, 64, 40], "gmm", 777, LIB), ([8, 256, 256, 40], "gmm", 1 << 18, LIB),
    ([2, 128, 128, 5], "gmm", 1000, FUSED), ([4, 128, 128, 40], "quad", 1 << 18, FUSED),
    ([8, 256, 256, 40], "gmm", 777, FUSED), ([16, 128, 128, 128, 64], "quad", 1500, FUSED),
    ([8, 512, 512, 512, 40], "gmm", 3000, FUSED), ([4, 32, 32, 40], "gmm", 1000, FUSED),
    ([8, 64, 64, 64, 40], "quad", 777, FUSED), ([2, 32, 32, 32, 5], "quad", 1 << 18, FUSED),
    # out_features filling / partly filling the 16-wide output tiles (rgemm16: 48 = 3 full tiles, 44 a partial third)
    ([4, 128, 128, 48], "quad", 1500, FUSED), ([8, 256, 256, 44], "gmm", 1000, FUSED),
    # the reference's default net (MLP.yaml: width 20 x 8 layers), zero-padded onto the 32-wide MFMA kernels
    ([2] + [20] * 8 + [40], "gmm", 1000, FUSED), ([4] + [20] * 8 + [40], "quad", 1 << 18, 0),
    ([8, 100, 100, 40], "gmm", 1500, FUSED),
    # one hidden layer (the output layer straight off the layer-1 prologue modes), out_features > 64 (E_OUT
    # partials per 64-column block), dims other than 2 / 4 / 8 / 16 (rows and the true potential zero-padded)
    ([4, 64, 40], "quad", 1000, FUSED), ([8, 256, 40], "gmm", 777, FUSED), ([2, 20, 40], "gmm", 1 << 18, FUSED),
    ([4, 64, 64, 80], "quad", 1000, FUSED), ([8, 128, 128, 200], "gmm", 1500, FUSED),
    ([3, 32, 32, 40], "gmm", 1000, FUSED), ([10, 64, 64, 40], "quad", 1000, FUSED), ([1, 32, 32, 5], "quad", 777, FUSED),
    ([5, 20, 40], "gmm", 1000, 0), ([6, 48, 48, 48, 70], "quad", 1 << 18, 0),
    # width 1024 (and 1000, zero-padded to it) on the hand-written kernels: AUTO never reaches rocBLAS
    ([4, 1024, 1024, 40], "quad", 1500, 0), ([3, 1000, 40], "gmm", 1 << 18, 0)])
def test_residual_mlp_vs_restatement(native, dims, true_kind, chunk, impl):
    """V_hypothesis residual (value + d loss/d theta) vs the fp64 restatement whose adjoint is
    FD-checked in tests/test_oracle.py, on both implementations (rocBLAS library path and the
    fused MFMA path). Multi-chunk paths exercised (chunk < rows); L = 3 covers the middle layers.
    impl = 0 (AUTO) on out-of-envelope shapes must take the hand-written path: its result equals
    impl = FUSED bit for bit (the fused path is deterministic), no rocBLAS."""
    rng = np.random.default_rng(len(dims) + dims[1])
    d = dims[0]
    flat = np.concatenate([np.concatenate([rng.standard_normal((dims[i], dims[i + 1])).ravel() * np.sqrt(1.0 / dims[i]),
                                           0.1 * rng.standard_normal(dims[i + 1])]) for i in range(len(dims) - 1)])
    P = nr.mlp_unflat(flat, dims)
    zi, zt, z0 = (rng.standard_normal((m, 2 * d)).astype(np.float32) for m in (900, 700, 2500))
    if true_kind == "gmm":
        mus = nr.gmm_centres(d, 3)
        kind, tp, gt = native.POT_GMM, mus, nr.grad_gmm(mus)
    else:
        F = nr.problem_constants(d)
        kind, tp, gt = native.POT_QUADRATIC, F, nr.grad_quadratic(F)
    acc, grad = native.residual_kfp_mlp(dims, _t(flat), _t(zi), _t(zt), _t(z0), true_kind=kind, true_params=tp,
                                        gamma=0.5, total_time=2.0, chunk_rows=chunk, impl=impl)
    assert impl != FUSED or native.mlp_fused_supported(dims) or dims[1] not in (32, 64, 128, 256, 512) \
        or dims[0] not in (2, 4, 8, 16)
    if impl == 0:
        acc_f, grad_f = native.residual_kfp_mlp(dims, _t(flat), _t(zi), _t(zt), _t(z0), true_kind=kind, true_params=tp,
                                                gamma=0.5, total_time=2.0, chunk_rows=chunk, impl=FUSED)
        assert torch.equal(acc, acc_f) and torch.equal(grad, grad_f)
    out = native.kfp_terms_finalize(acc, grad, 0.5).cpu().numpy()
    loss, loss_gt, parts = nr.kfp_mlp_loss(P, zi, zt, z0, gt, 0.5, 2.0)
    g_ref = nr.mlp_flat(nr.kfp_mlp_grad_analytic(P, zi, zt, z0, 0.5, 2.0))
    assert abs(out[0] - loss) < 1e-3 * (1 + abs(loss)), (out[0], loss)
    assert abs(out[1] - loss_gt) < 1e-3 * (1 + abs(loss_gt))
    assert abs(out[4] - parts["hessian"]) < 1e-3 * (1 + abs(parts["hessian"]))
    g = grad.cpu().numpy()
    assert np.max(np.abs(g - g_ref)) < 2e-3 * (1 + np.abs(g_ref).max()), np.max(np.abs(g - g_ref))
    assert abs(out[2] - np.linalg.norm(g_ref)) < 2e-3 * (1 + np.linalg.norm(g_ref))


def test_auto_never_reaches_rocblas(native):
    """impl = AUTO never resolves to rocBLAS: AUTO KFP MLP residuals across the hand-written envelope (padded dims /
    widths, width 1024, depth 3, out 56) leave pdeinv_rocblas_calls unchanged, one shape past the envelope
    ([4, 2048, 2048, 40]) raises NotImplementedError, and the explicit impl = LIBRARY call does count."""
    pc = lambda dims: int(native.lib().pdeinv_mlp_param_count(dims[0], len(dims) - 2, dims[1], dims[-1]))
    rng = np.random.default_rng(5)
    before = native.rocblas_calls()
    for dims in ([4, 256, 256, 40], [3, 20, 20, 40], [4, 1024, 1024, 40], [12, 100, 60], [4, 64, 64, 64, 56]):
        d = dims[0]
        flat = _t(rng.standard_normal(pc(dims)) * 0.05)
        z = [_t(rng.standard_normal((m, 2 * d))) for m in (300, 200, 700)]
        native.residual_kfp_mlp(dims, flat, z[0], z[1], z[2], true_kind=native.POT_QUADRATIC,
                                true_params=np.eye(d, dtype=np.float32), gamma=0.5, total_time=2.0, chunk_rows=256)
    wide = [4, 2048, 2048, 40]
    with pytest.raises(NotImplementedError):
        native.residual_kfp_mlp(wide, torch.zeros(pc(wide), device=DEV), *[torch.zeros((64, 8), device=DEV)] * 3,
                                true_kind=native.POT_QUADRATIC, true_params=np.eye(4, dtype=np.float32), gamma=0.5,
                                total_time=2.0, chunk_rows=64)
    torch.cuda.synchronize()
    assert native.rocblas_calls() == before
    dims = [4, 64, 64, 40]
    z = [_t(rng.standard_normal((m, 8))) for m in (300, 200, 700)]
    native.residual_kfp_mlp(dims, _t(rng.standard_normal(pc(dims)) * 0.05), z[0], z[1], z[2],
                            true_kind=native.POT_QUADRATIC, true_params=np.eye(4, dtype=np.float32), gamma=0.5,
                            total_time=2.0, impl=native.MLP_IMPL_LIBRARY)
    assert native.rocblas_calls() == before + 1


def test_residual_mlp_fused_chunk_at_offset_limit(native):
    """The C5 default chunk: 2^22 rows x width 256 = 2^30 floats per plane, the largest chunk whose byte offsets
    (32-bit, from a uniform plane base) do not wrap. One 2^22-row 0T chunk equals two 2^21-row chunks to fp32
    reassociation; a chunk past 2^30 / W rows is rejected (the old 2^31 bound let byte offsets wrap)."""
    dims = [8, 256, 256, 40]
    rng = np.random.default_rng(22)
    flat = np.concatenate([np.concatenate([rng.standard_normal((dims[i], dims[i + 1])).ravel() * np.sqrt(1.0 / dims[i]),
                                           0.1 * rng.standard_normal(dims[i + 1])]) for i in range(len(dims) - 1)])
    n0t = 1 << 22
    z0 = torch.randn((n0t, 16), device=DEV)
    zi, zt = torch.randn((1000, 16), device=DEV), torch.randn((1000, 16), device=DEV)
    mus = nr.gmm_centres(8, 3)
    kw = dict(true_kind=native.POT_GMM, true_params=mus, gamma=0.5, total_time=2.0, impl=FUSED)
    acc_a, grad_a = native.residual_kfp_mlp(dims, _t(flat), zi, zt, z0, chunk_rows=1 << 22, **kw)
    acc_b, grad_b = native.residual_kfp_mlp(dims, _t(flat), zi, zt, z0, chunk_rows=1 << 21, **kw)
    a, b = acc_a.cpu().numpy(), acc_b.cpu().numpy()
    assert np.allclose(a, b, rtol=1e-4, atol=1e-4 * np.abs(b).max())
    ga, gb = grad_a.cpu().numpy(), grad_b.cpu().numpy()
    assert np.max(np.abs(ga - gb)) < 1e-4 * (1 + np.abs(gb).max())
    assert np.abs(gb).max() > 0
    with pytest.raises(ValueError, match="2\\^30"):
        native.residual_kfp_mlp(dims, _t(flat), zi, zt, z0[:1024], chunk_rows=(1 << 22) + 64, **kw)


@pytest.mark.parametrize("dims", [[8, 256, 256, 40], [4, 64, 40], [2, 32, 32, 32, 40], [4, 128, 128, 128, 40],
                                  [16, 128, 128, 24], [8, 128, 128, 64], [4, 256, 256, 56]])
def test_residual_mlp_boundary_sets_span_chunks(native, dims):
    """The initial / terminal sets take the first-order chain (no g, no forward adjoint: c_nabla = c_hess = 0 there,
    kinetic_fokker_planck.py:34-39) — here with boundary sets larger than the 0T set, split over several chunks
    (5000 rows at chunk 2048), L = 1 / 2 / 3: loss and gradient equal the fp64 restatement and the rocBLAS library
    path (which runs the full chain). Widths 128 / 256 run the two-stream kernels (mlp_fused.hip run_chunk_fo2:
    [h, z'] forward, [zbar, z'bar] back, the seeds in the output epilogue, 2-pair weight gradients), including a
    middle layer (L = 3) and out_features 24 / 40 (the 16-wide output tiles of rgemm16) and 56 / 64 (past 48 columns:
    the 64-column rgemm E_OUT_SEEDS1 epilogue); the narrower nets the zeroed-plane first-order path."""
    rng = np.random.default_rng(sum(dims))
    d = dims[0]
    flat = np.concatenate([np.concatenate([rng.standard_normal((dims[i], dims[i + 1])).ravel() * np.sqrt(1.0 / dims[i]),
                                           0.1 * rng.standard_normal(dims[i + 1])]) for i in range(len(dims) - 1)])
    P = nr.mlp_unflat(flat, dims)
    zi, zt, z0 = (rng.standard_normal((m, 2 * d)).astype(np.float32) for m in (5000, 4500, 1500))
    F = nr.problem_constants(d)
    kw = dict(true_kind=native.POT_QUADRATIC, true_params=F, gamma=0.5, total_time=2.0, chunk_rows=2048)
    acc, grad = native.residual_kfp_mlp(dims, _t(flat), _t(zi), _t(zt), _t(z0), impl=FUSED, **kw)
    acc_l, grad_l = native.residual_kfp_mlp(dims, _t(flat), _t(zi), _t(zt), _t(z0), impl=LIB, **kw)
    out = native.kfp_terms_finalize(acc, grad, 0.5).cpu().numpy()
    loss, loss_gt, _ = nr.kfp_mlp_loss(P, zi, zt, z0, nr.grad_quadratic(F), 0.5, 2.0)
    g_ref = nr.mlp_flat(nr.kfp_mlp_grad_analytic(P, zi, zt, z0, 0.5, 2.0))
    assert abs(out[0] - loss) < 1e-3 * (1 + abs(loss)), (out[0], loss)
    assert abs(out[1] - loss_gt) < 1e-3 * (1 + abs(loss_gt))
    g = grad.cpu().numpy()
    assert np.max(np.abs(g - g_ref)) < 2e-3 * (1 + np.abs(g_ref).max()), np.max(np.abs(g - g_ref))
    a, al = acc.cpu().numpy(), acc_l.cpu().numpy()
    assert np.allclose(a, al, rtol=2e-4, atol=1e-5 * np.abs(al).max())
    assert np.max(np.abs(g - grad_l.cpu().numpy())) < 2e-4 * (1 + np.abs(g_ref).max())


def test_residual_mlp_fused_matches_library(native):
    """The two implementations agree to fp32 reassociation level on the C5 shape, and the fused
    path is deterministic run to run (fixed-order slab sums, no atomics)."""
    dims = [8, 256, 256, 40]
    rng = np.random.default_rng(11)
    flat = np.concatenate([np.concatenate([rng.standard_normal((dims[i], dims[i + 1])).ravel() * np.sqrt(2.0 / dims[i]),
                                           np.zeros(dims[i + 1])]) for i in range(len(dims) - 1)])
    zi, zt, z0 = (_t(rng.standard_normal((m, 16)) * 2) for m in (3000, 3000, 40000))
    mus = nr.gmm_centres(8, 8)
    kw = dict(true_kind=native.POT_GMM, true_params=mus, gamma=0.5, total_time=2.0, chunk_rows=16384)
    a_l, g_l = native.residual_kfp_mlp(dims, _t(flat), zi, zt, z0, impl=LIB, **kw)
    a_f, g_f = native.residual_kfp_mlp(dims, _t(flat), zi, zt, z0, impl=FUSED, **kw)
    a_f2, g_f2 = native.residual_kfp_mlp(dims, _t(flat), zi, zt, z0, impl=FUSED, **kw)
    assert torch.equal(a_f, a_f2) and torch.equal(g_f, g_f2)
    a_l, a_f = a_l.cpu().numpy(), a_f.cpu().numpy()
    assert np.allclose(a_f, a_l, rtol=2e-4, atol=1e-5 * np.abs(a_l).max()), (a_f, a_l)
    g_l, g_f = g_l.cpu().numpy(), g_f.cpu().numpy()
    assert np.max(np.abs(g_f - g_l)) < 2e-4 * np.abs(g_l).max(), np.max(np.abs(g_f - g_l))


def test_residual_mlp_library_two_threads_two_streams(native):
    """ABI thread contract (include/pdeinv.h): two host threads call the rocBLAS
    library path concurrently on two streams (ctypes releases the GIL during the call). Each must get
    exactly the single-threaded result — a rocBLAS handle shared between threads would let one
    thread's set_stream retarget the other's GEMMs."""
    import threading
    dims = [4, 32, 32, 40]
    rng = np.random.default_rng(21)
    flat = np.concatenate([np.concatenate([rng.standard_normal((dims[i], dims[i + 1])).ravel() * np.sqrt(1.0 / dims[i]),
                                           0.1 * rng.standard_normal(dims[i + 1])]) for i in range(len(dims) - 1)])
    F = nr.problem_constants(4)
    sets = [tuple(_t(rng.standard_normal((m, 8))) for m in (1000, 1000, 60000)) for _ in range(2)]
    kw = dict(true_kind=native.POT_QUADRATIC, true_params=F, gamma=0.5, total_time=2.0, chunk_rows=4096, impl=LIB)
    ref = [native.residual_kfp_mlp(dims, _t(flat), *s, **kw) for s in sets]
    torch.cuda.synchronize()
    got, errs = [[None] * 4 for _ in range(2)], []

    def work(t):
        try:
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                for rep in range(4):
                    a, g = native.residual_kfp_mlp(dims, _t(flat), *sets[t], **kw)
                    got[t][rep] = (a, g)
            st.synchronize()
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errs, errs
    for t in range(2):  # 1e-6: run-to-run reassociation at most (a stream mix-up reads garbage)
        for a, g in got[t]:
            assert torch.allclose(a, ref[t][0], rtol=1e-6, atol=1e-9 * ref[t][0].abs().max().item())
            assert torch.allclose(g, ref[t][1], rtol=1e-6, atol=1e-6 * ref[t][1].abs().max().item())


@pytest.mark.parametrize("m", [8, 16, 6])  # 16-byte quads (m % 4 == 0) and the scalar kernel (m = 6)
def test_gather_random_step(native, m):
    rng = np.random.default_rng(3)
    n, N = 37, 5000
    traj = _t(rng.standard_normal((n, N, m)))
    out, t = native.gather_random_step(traj, seed=5, ctr=2, return_t=True)
    t = t.cpu().numpy()
    assert t.min() >= 0 and t.max() < n and len(np.unique(t)) == n
    ref = traj.cpu().numpy()[t, np.arange(N)]
    assert np.array_equal(out.cpu().numpy(), ref)
    # uniform over steps (chi-square, 36 dof)
    cnt = np.bincount(t, minlength=n)
    chi2 = np.sum((cnt - N / n) ** 2 / (N / n))
    assert chi2 < 80


def test_adam_update_matches_optax_formula(native):
    """pdeinv_adam_update == optax.chain(add_decayed_weights(wd), adam(lr, b1, b2, eps)) + apply_updates
    (core/trainer.py:85-86, main.py:11-29), evaluated in fp64 on the host, over several steps."""
    rng = np.random.default_rng(4)
    n, lr, b1, b2, eps, wd = 78376, 1e-3, 0.9, 0.999, 1e-4, 1e-2
    p = rng.standard_normal(n)
    mu, nu = np.zeros(n), np.zeros(n)
    dp, dmu, dnu = _t(p), _t(mu), _t(nu)
    for t in range(1, 5):
        g = rng.standard_normal(n)
        native.adam_update(dp, _t(g), dmu, dnu, lr=lr, b1=b1, b2=b2, eps=eps, weight_decay=wd, count=t)
        g = g + wd * p
        mu = b1 * mu + (1 - b1) * g
        nu = b2 * nu + (1 - b2) * g * g
        p = p - lr * (mu / (1 - b1 ** t)) / (np.sqrt(nu / (1 - b2 ** t)) + eps)
    assert np.allclose(dp.cpu().numpy(), p, rtol=0, atol=2e-6)
    assert np.allclose(dmu.cpu().numpy(), mu, rtol=1e-5, atol=1e-6)
    assert np.allclose(dnu.cpu().numpy(), nu, rtol=1e-5, atol=1e-7)
    with pytest.raises(ValueError):
        native.adam_update(dp, _t(np.zeros(3)), dmu, dnu, lr=lr, b1=b1, b2=b2, eps=eps, weight_decay=wd, count=1)


@pytest.mark.parametrize("dim,mask_type,E,soft_init,ignore_time,act", [
    (2, "loop", 10, 1.0, False, "celu"), (4, "random", 0, 0.0, False, "tanh"), (8, "loop", 10, 1.0, False, "silu"),
    (3, "random", 6, 1.0, True, "softplus"), (1, "loop", 4, 0.0, False, "gelu")])
def test_realnvp_logdensity_vs_restatement(native, dim, mask_type, E, soft_init, ignore_time, act):
    """pdeinv_realnvp_logdensity (normalizing_flow.py:115-229) vs the fp64 restatement that
    tests/test_oracle.py pins by invertibility and normalisation; fp32 tolerance."""
    from core.distribution import Gaussian
    from core.normalizing_flow import MNF, RealNVP
    couple = 4 if mask_type == "loop" else 3
    mnf = MNF(dim, couple, mask_type, soft_init, ignore_time, act, E)
    rng = np.random.default_rng(dim)
    mean = rng.standard_normal(dim) * 0.3
    Lc = rng.standard_normal((dim, dim)) * 0.3
    cov = Lc @ Lc.T + np.eye(dim)
    flow = RealNVP(mnf, Gaussian(mean, cov).logdensity)
    flat = nr.nvp_init(dim, mnf.n_layers, E, ignore_time, seed=dim + 1, scale=1.3, perturb=True)
    assert flat.size == mnf.param_count() == native.realnvp_param_count(flow._desc)
    x = rng.standard_normal((5000, dim)) * 1.5
    t = rng.uniform(0, 2, 5000)
    got = flow.apply({"params": _t(flat)}, _t(t), _t(x)).cpu().numpy()
    ref = nr.realnvp_logdensity(flat, t, x, dim=dim, masks=mnf.masks, base_mean=mean, base_cov=cov, E=E,
                                ignore_time=ignore_time, soft_init=soft_init, act=act)
    assert np.max(np.abs(got - ref)) < 2e-4 * (1 + np.abs(ref).max()), np.max(np.abs(got - ref))
    one = flow.apply({"params": _t(flat)}, float(t[0]), _t(x[0])).item()   # unbatched call
    assert abs(one - ref[0]) < 2e-4 * (1 + abs(ref[0]))
    # the reference's model (log_density_estimation.py:103-114) at its fresh init
    from core.log_density_estimation import create_normalizing_flow_fn
    from utils import prng
    f2 = create_normalizing_flow_fn(Gaussian(np.zeros(2), np.eye(2)).logdensity, 2)
    p2 = f2.init(prng.PRNGKey(0), 0.0, np.zeros(2))
    assert torch.isfinite(f2.apply(p2, _t(t[:10]), _t(x[:10, :2] if dim >= 2 else np.zeros((10, 2))))).all()


@pytest.mark.parametrize("dim,mask_type,E,soft_init,ignore_time,n", [
    (2, "loop", 10, 1.0, False, 3000), (1, "loop", 4, 0.0, False, 700), (3, "random", 0, 1.0, False, 1000),
    (4, "loop", 10, 1.0, False, 2561), (5, "random", 6, 0.0, False, 900), (8, "loop", 16, 1.0, True, 513)])
def test_realnvp_value_and_grad_vs_autograd(native, dim, mask_type, E, soft_init, ignore_time, n):
    """pdeinv_realnvp_value_and_grad (log_density_estimation.py:47-58: loss = -mean log p and its
    gradient, which the reference takes with jax.value_and_grad) vs the fp64 torch-autograd
    restatement (oracle/numpy_ref.py, FD-checked in tests/test_oracle.py). fp32 kernel: loss within
    2e-5 relative, gradient within 1e-4 of its norm (and 5e-4 of its max entry) elementwise."""
    from core.distribution import Gaussian
    from core.normalizing_flow import MNF, RealNVP
    couple = 2 if mask_type == "loop" else 3
    mnf = MNF(dim, couple, mask_type, soft_init, ignore_time, "celu", E)
    rng = np.random.default_rng(10 + dim)
    mean = rng.standard_normal(dim) * 0.3
    Lc = rng.standard_normal((dim, dim)) * 0.3
    cov = Lc @ Lc.T + np.eye(dim)
    flow = RealNVP(mnf, Gaussian(mean, cov).logdensity)
    flat = nr.nvp_init(dim, mnf.n_layers, E, ignore_time, seed=dim + 3, scale=1.2, perturb=True)
    x = rng.standard_normal((n, dim)) * 1.5
    t = rng.uniform(0, 2, n)
    loss, grad = flow.value_and_grad({"params": _t(flat)}, _t(t), _t(x))
    ref_loss, ref_grad = nr.realnvp_nll_value_and_grad(flat, t, x, dim=dim, masks=mnf.masks, base_mean=mean,
                                                       base_cov=cov, E=E, ignore_time=ignore_time,
                                                       soft_init=soft_init, act="celu")
    g = grad.cpu().numpy().astype(np.float64)
    assert abs(loss.item() - ref_loss) < 2e-5 * (1 + abs(ref_loss)), (loss.item(), ref_loss)
    err = np.abs(g - ref_grad)
    assert np.linalg.norm(g - ref_grad) < 1e-4 * np.linalg.norm(ref_grad) + 1e-6, np.linalg.norm(g - ref_grad)
    assert err.max() < 5e-4 * (1 + np.abs(ref_grad).max()), err.max()
    # deterministic: fixed-order reductions, no float atomics
    loss2, grad2 = flow.value_and_grad({"params": _t(flat)}, _t(t), _t(x))
    assert loss2.item() == loss.item() and torch.equal(grad, grad2)


def test_realnvp_value_and_grad_chunks_and_errors(native):
    """One launch covers kNvpMaxRows = 8192 slab rows of kNvSPB = 128 samples (realnvp.hip); past that
    the epoch is split into launches whose slabs are reduced into one fp64 accumulator (first / last
    flags of nvp_grad_reduce_kernel, the slab reused across launches, tile offsets). n is sized past
    two launches: the mean gradient over n rows must equal the row-count-weighted mean of the gradients
    over two disjoint parts (linearity, size-independent), with the split inside the second launch.
    Also: a broadcast t, the unsupported-activation and empty-batch errors."""
    from core.distribution import Gaussian
    from core.normalizing_flow import MNF, RealNVP
    dim, E = 2, 10
    mnf = MNF(dim, 4, "loop", 1.0, False, "celu", E)
    flow = RealNVP(mnf, Gaussian(np.zeros(dim), np.eye(dim)).logdensity)
    flat = _t(nr.nvp_init(dim, mnf.n_layers, E, False, seed=5, scale=1.2, perturb=True))
    per_launch = 8192 * 128  # kNvpMaxRows * kNvSPB
    n = 2 * per_launch + 777  # three launches, the last one partial
    gen = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn((n, dim), device=DEV, generator=gen) * 1.5
    t = torch.rand(n, device=DEV, generator=gen) * 2
    loss, grad = flow.value_and_grad(flat, t, x)
    n1 = per_launch + 300_001  # part 1 spans two launches, part 2 ends in a partial one
    l1, g1 = flow.value_and_grad(flat, t[:n1], x[:n1])
    l2, g2 = flow.value_and_grad(flat, t[n1:], x[n1:])
    mix = (n1 * g1.double() + (n - n1) * g2.double()) / n
    assert torch.linalg.norm(grad.double() - mix) < 1e-5 * torch.linalg.norm(mix)
    assert abs(loss.item() - (n1 * l1.item() + (n - n1) * l2.item()) / n) < 1e-5 * (1 + abs(loss.item()))
    lb, gb = flow.value_and_grad(flat, torch.full((1,), 0.7, device=DEV), x[:1000])   # broadcast t
    lr_, gr = flow.value_and_grad(flat, torch.full((1000,), 0.7, device=DEV), x[:1000])
    assert lb.item() == lr_.item() and torch.equal(gb, gr)
    with pytest.raises(ValueError):
        flow.value_and_grad(flat, t[:0], x[:0])
    tanh_flow = RealNVP(MNF(dim, 4, "loop", 1.0, False, "tanh", E), Gaussian(np.zeros(dim), np.eye(dim)).logdensity)
    with pytest.raises(NotImplementedError):
        tanh_flow.value_and_grad(flat, t[:10], x[:10])
