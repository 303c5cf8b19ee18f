"""CPU tests: the oracle restatement against closed forms, the reference's own finite-difference
check (test_partial_s_log_density.py, now asserted), Random123 KATs and the golden fixtures.
No GPU needed."""
import glob
import os

import numpy as np
import pytest

from oracle import numpy_ref as nr

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Random123 philox4x32-10 known answers
KATS = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_philox_kat_c_oracle(oracle_lib, ctr, key, want):
    assert tuple(int(x) for x in oracle_lib.philox(ctr, key)) == want


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_philox_kat_host_prng(ctr, key, want):
    from utils import prng
    assert prng.philox4x32_10(ctr, key) == want


def test_box_muller_normals_moments(oracle_lib):
    z = np.concatenate([oracle_lib.sim_normals(11, p, 3, 8) for p in range(20000)])
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    assert abs(np.mean(z ** 4) - 3) < 0.1


@pytest.mark.parametrize("d", [1, 2, 4, 8])
def test_c_oracle_equals_numpy_restatement(oracle_lib, d):
    rng = np.random.default_rng(d)
    N, n = 50, 60
    F = nr.problem_constants(d)
    z0 = rng.standard_normal((N, 2 * d)).astype(np.float32)
    xi = rng.standard_normal((n + 1, N, d)).astype(np.float32)
    u = rng.random(N).astype(np.float32)
    o = oracle_lib.sde_simulate(z0, n, 0.02, 1.0, "quadratic", F, noise=xi, shift_u=u)
    last, traj, _ = nr.sde_scan(z0, n, 0.02, 1.0, nr.grad_quadratic(F), xi, u)
    assert np.max(np.abs(o["traj"] - traj) / (np.abs(traj).max() + 1)) < 1e-5


def test_chain_law_matches_sample_paths():
    """em_chain_moments is the exact law of sde_scan: check on 2e5 paths (5 sigma)."""
    d, N, n = 2, 200000, 20
    F = nr.problem_constants(d)
    rng = np.random.default_rng(0)
    z0 = rng.standard_normal((N, 2 * d))
    xi = rng.standard_normal((n + 1, N, d))
    u = rng.random(N)
    last, traj, _ = nr.sde_scan(z0, n, 0.05, 1.0, nr.grad_quadratic(F), xi, u)
    mt, st, ml, sl = nr.em_chain_moments(F, 1.0, 0.05, n, np.zeros(2 * d), np.eye(2 * d))
    for s in (0, n - 1):
        emp = traj[s].T @ traj[s] / N
        sig = np.sqrt((np.outer(np.diag(st[s]), np.diag(st[s])) + st[s] ** 2) / N)
        assert np.max(np.abs(emp - st[s]) / sig) < 5
    emp = last.T @ last / N
    sig = np.sqrt((np.outer(np.diag(sl), np.diag(sl)) + sl ** 2) / N)
    assert np.max(np.abs(emp - sl) / sig) < 5


def test_chain_converges_to_ou_weak_order_one():
    """the terminal-covariance gap to the continuous OU law ~ dt."""
    d, T = 4, 2.0
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F)
    _, P = nr.ou_mean_cov(T, cfg)
    gaps = []
    for n in (100, 200, 400):
        _, _, _, sl = nr.em_chain_moments(F, 1.0, T / n, n, np.zeros(2 * d), np.eye(2 * d))
        gaps.append(np.abs(sl - P).max())
    assert 1.7 < gaps[0] / gaps[1] < 2.3 and 1.7 < gaps[1] / gaps[2] < 2.3


def test_ou_closed_form_matches_ode():
    """ou_mean_cov (Van Loan) == the reference's moment ODE (…_OU.py:78-86) integrated by RK45."""
    from scipy.integrate import solve_ivp
    F = nr.problem_constants(3)
    cfg = nr.ou_configuration(F)
    cfg["m_0"] = np.array([1.0, -0.5, 0.2, 0.0, 0.3, 0.0])
    n = 6

    def rhs(t, y):
        m, P = y[:n], y[n:].reshape(n, n)
        return np.concatenate([cfg["F"] @ m, (cfg["F"] @ P + P @ cfg["F"].T + cfg["L"]).ravel()])

    sol = solve_ivp(rhs, (0, 1.3), np.concatenate([cfg["m_0"], cfg["P_0"].ravel()]), rtol=1e-10, atol=1e-12)
    m, P = nr.ou_mean_cov(1.3, cfg)
    assert np.allclose(m, sol.y[:n, -1], atol=1e-7) and np.allclose(P, sol.y[n:, -1].reshape(n, n), atol=1e-7)


def test_quadratic_residual_moments_identity_and_gradient():
    rng = np.random.default_rng(0)
    d = 3
    F = nr.problem_constants(d)
    K, b = rng.standard_normal((d, d)), rng.standard_normal(d)
    zi, zt, z0 = (rng.standard_normal((m, 2 * d)) for m in (300, 200, 1000))
    loss, gt, _ = nr.kfp_quadratic_samples(K, b, zi, zt, z0, F, 0.7, 2.0)
    l2, gt2, gK, gb, _ = nr.kfp_quadratic_from_moments(K, b, nr.moments(zi), nr.moments(z0), nr.moments(zt), F, 0.7, 2.0)
    assert abs(loss - l2) < 1e-9 * (1 + abs(loss)) and abs(gt - gt2) < 1e-9 * (1 + abs(gt))
    g_fd = nr.fd_grad(lambda th: nr.kfp_quadratic_samples(th[:9].reshape(3, 3), th[9:], zi, zt, z0, F, 0.7, 2.0)[0],
                      np.concatenate([K.ravel(), b]))
    assert np.allclose(np.concatenate([gK.ravel(), gb]), g_fd, rtol=1e-6, atol=1e-6)


def test_loss_equals_ground_truth_on_exact_stationary_data():
    """kinetic_fokker_planck.py:33-58 identity: E[loss] = E[loss gt] for exact OU data with
    time-uniform 0T samples (checked through moments, no sampling noise)."""
    d, T = 2, 2.0
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F)
    ts = (np.arange(4000) + 0.5) * T / 4000
    M0 = np.mean([nr.ou_mean_cov(t, cfg)[1] for t in ts], 0)
    PT = nr.ou_mean_cov(T, cfg)[1]

    def mom(P):  # exact moments in the packed layout (mean 0)
        m = P.shape[0]
        return np.concatenate([[1.0], np.zeros(m), P[np.triu_indices(m)]])
    rng = np.random.default_rng(3)
    K, b = rng.standard_normal((d, d)), rng.standard_normal(d) * 0.1
    loss, gt, *_ = nr.kfp_quadratic_from_moments(K, b, mom(cfg["P_0"]), mom(M0), mom(PT), F, 1.0, T)
    assert abs(loss - gt) < 1e-5 * (1 + abs(gt))


def test_gmm_analytic_adjoint_vs_finite_differences():
    rng = np.random.default_rng(1)
    d, K = 3, 4
    mus_true, mus = nr.gmm_centres(d, 5), rng.standard_normal((K, d))
    zi, zt, z0 = (1.5 * rng.standard_normal((m, 2 * d)) for m in (200, 150, 800))
    G = nr.kfp_gmm_grad_analytic(mus, zi, zt, z0, mus_true, 0.5, 2.0)
    g_fd = nr.fd_grad(lambda th: nr.kfp_gmm_loss(th, zi, zt, z0, mus_true, 0.5, 2.0)[0], mus)
    assert np.allclose(G, g_fd, rtol=1e-6, atol=1e-7)


def test_kmv_moment_form_equals_pairwise():
    rng = np.random.default_rng(2)
    d, n, n_t = 3, 120, 3
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F)
    x, v = rng.standard_normal((n, n_t, d)), rng.standard_normal((n, n_t, d))
    tau = np.array([0.2, 0.9, 1.7])
    K, b = 0.3 * rng.standard_normal((d, d)), 0.2 * rng.standard_normal(d)
    l1, g1 = nr.kmv_pairwise_loss(K, b, x, v, tau, cfg)
    l2, g2, gK, gb = nr.kmv_from_moments(K, b, x, v, tau, cfg)
    assert abs(l1 - l2) < 1e-9 * (1 + abs(l1)) and abs(g1 - g2) < 1e-9 * (1 + abs(g1))
    g_fd = nr.fd_grad(lambda th: nr.kmv_pairwise_loss(th[:9].reshape(3, 3), th[9:], x, v, tau, cfg)[0],
                      np.concatenate([K.ravel(), b]))
    assert np.allclose(np.concatenate([gK.ravel(), gb]), g_fd, rtol=1e-5, atol=1e-6)


def test_partial_s_log_density_fd_kat():
    """test_partial_s_log_density.py:241-311 (d = 10, s = 0.1, delta 1e-4 / 1e-3), asserted."""
    g = np.load(os.path.join(GOLD, "dlogrho_d10.npz"))
    cfg = nr.ou_configuration(g["F"], gamma=1.0)
    x, s = g["x"], float(g["s"])
    fd1 = (nr.log_density(s + 1e-4, x, cfg) - nr.log_density(s - 1e-4, x, cfg)) / 2e-4
    fd2 = (nr.partial_s_log_density(s + 1e-3, x, cfg) - nr.partial_s_log_density(s - 1e-3, x, cfg)) / 2e-3
    assert np.sqrt(np.mean(((g["ds"] - fd1) / fd1) ** 2)) < 1e-3
    assert np.sqrt(np.mean(((g["ds2"] - fd2) / fd2) ** 2)) < 1e-3
    assert np.allclose(nr.partial_s_log_density(s, x, cfg), g["ds"], rtol=1e-12)


def test_partial_s_log_density_fd_kat_reference_configuration():
    """test_partial_s_log_density.py at its own configuration (:9-62: gamma = 0.1, P_v0 = 0.1; d = 10,
    s = 0.1, x ~ U[0, 1)): the restatement's analytic ds / ds2 vs central differences (delta 1e-4 / 1e-3),
    relative RMSE < 1e-3, and the build's host coefficient rows (the kernel's inputs) reproduce them."""
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    from example_problems.kinetic_fokker_planck_example_OU import initialize_configuration
    g = np.load(os.path.join(GOLD, "dlogrho_d10_refcfg.npz"))
    assert float(g["gamma"]) == 0.1 and float(g["P_v0"]) == 0.1 and float(g["T"]) == 1.0
    cfg = nr.ou_configuration(g["F"], gamma=0.1, P_x0=1.0, P_v0=0.1)
    x, s = g["x"], float(g["s"])
    fd1 = (nr.log_density(s + 1e-4, x, cfg) - nr.log_density(s - 1e-4, x, cfg)) / 2e-4
    fd2 = (nr.partial_s_log_density(s + 1e-3, x, cfg) - nr.partial_s_log_density(s - 1e-3, x, cfg)) / 2e-3
    assert np.sqrt(np.mean(((g["ds"] - fd1) / fd1) ** 2)) < 1e-3
    assert np.sqrt(np.mean(((g["ds2"] - fd2) / fd2) ** 2)) < 1e-3
    assert np.allclose(nr.partial_s_log_density(s, x, cfg), g["ds"], rtol=1e-12)
    # the coefficient rows the GPU kernel consumes: ds = a1 + beta1.r + r^T G1 r, r = m1 - x
    d = x.shape[1]
    ic = initialize_configuration(d, gamma_friction=0.1, P_x_0_scale=1.0, P_v_0_scale=0.1)
    c = dlogrho_coefficients([s], ic, d)[0]
    m1, a1, b1, G1 = c[:d], c[d], c[d + 1:2 * d + 1], c[2 * d + 1:2 * d + 1 + d * d].reshape(d, d)
    o = 2 * d + 1 + d * d
    a2, b2, G2 = c[o], c[o + 1:o + 1 + d], c[o + 1 + d:o + 1 + d + d * d].reshape(d, d)
    r = m1 - x
    assert np.allclose(a1 + r @ b1 + np.einsum("ni,ij,nj->n", r, G1, r), g["ds"], rtol=1e-9, atol=1e-9)
    assert np.allclose(a2 + r @ b2 + np.einsum("ni,ij,nj->n", r, G2, r), g["ds2"], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "sde_*.npz"))))
def test_oracle_reproduces_sde_golden(oracle_lib, path):
    g = np.load(path)
    F = g["params"]
    grad = nr.grad_quadratic(F) if str(g["kind"]) == "quadratic" else nr.grad_gmm(F)
    n = g["xi"].shape[0] - 1
    last, traj, _ = nr.sde_scan(g["z0"], n, float(g["dt"]), float(g["gamma"]), grad, g["xi"], g["u"])
    assert np.allclose(traj[g["keep"]], g["traj"], rtol=1e-12, atol=1e-12)
    kind = str(g["kind"])
    o = oracle_lib.sde_simulate(g["z0"], n, float(g["dt"]), float(g["gamma"]), kind, F, n_centers=F.shape[0] if kind == "gmm" else 0,
                                noise=g["xi"], shift_u=g["u"])
    assert np.array_equal(o["tau"], g["tau"])
    scale = np.abs(g["traj"]).max() + 1
    assert np.max(np.abs(o["traj"][g["keep"]] - g["traj"])) / scale < 2e-5


def test_residual_goldens():
    g = np.load(os.path.join(GOLD, "kfp_quadratic.npz"))
    loss, gt, _ = nr.kfp_quadratic_samples(g["K"], g["b"], g["zi"], g["zt"], g["z0"], g["F"], 1.0, 2.0)
    assert np.isclose(loss, g["loss"], rtol=1e-12) and np.isclose(gt, g["loss_gt"], rtol=1e-12)
    g = np.load(os.path.join(GOLD, "kfp_gmm.npz"))
    loss, gt, _ = nr.kfp_gmm_loss(g["mus"], g["zi"], g["zt"], g["z0"], g["mus_true"], 0.5, 2.0)
    assert np.isclose(loss, g["loss"], rtol=1e-12)
    G = nr.kfp_gmm_grad_analytic(g["mus"], g["zi"], g["zt"], g["z0"], g["mus_true"], 0.5, 2.0)
    assert np.allclose(G, g["grad"], rtol=1e-5, atol=1e-7)
    for name in ("kmv_pairwise.npz", "kmv_pairwise_d8.npz", "kmv_pairwise_recipe.npz"):
        # the moment form (what kmv.hip implements) == the literal O(n^2) pair tensor of the fixture
        g = np.load(os.path.join(GOLD, name))
        cfg = nr.ou_configuration(g["F"])
        loss, gt, gK, gb = nr.kmv_from_moments(g["K"], g["b"], g["x"], g["v"], g["tau"], cfg)
        assert np.isclose(loss, g["loss"], rtol=1e-9), name
        assert np.isclose(gt, g["loss_gt"], rtol=1e-9), name
        assert np.allclose(np.concatenate([gK.ravel(), gb]), g["grad"], rtol=1e-5, atol=1e-6), name


def test_constants_recipe():
    g = np.load(os.path.join(GOLD, "constants.npz"))
    from example_problems.kinetic_fokker_planck_example_OU import problem_matrix
    for d in (2, 4, 8, 10):
        assert np.array_equal(problem_matrix(d), g[f"tilde_F_d{d}"])
        assert np.array_equal(nr.problem_constants(d), g[f"tilde_F_d{d}"])


def test_kmv_mlp_two_pass_adjoint_vs_finite_differences():
    """General-Phi KMV (Phi_theta = V_hypothesis): the two-pass adjoint the HIP path runs
    (gbar = mean_j grad Phi, then per-pair seeds) equals central differences of the literal
    pair-tensor loss of kinetic_mckean_vlasov.py:74-97 (tiny net, fp64)."""
    rng = np.random.default_rng(4)
    d, n, n_t = 2, 9, 2
    dims = [d, 5, 5, 3]
    flat = rng.standard_normal(sum(dims[i] * dims[i + 1] + dims[i + 1] for i in range(3))) * 0.5
    cfg = nr.ou_configuration(nr.problem_constants(d))
    x, v = rng.standard_normal((n, n_t, d)), rng.standard_normal((n, n_t, d))
    tau = np.array([0.4, 1.3])
    f = lambda fl: nr.kmv_mlp_pairwise_loss(nr.mlp_unflat(fl, dims), x, v, tau, cfg)[0]
    ga = nr.mlp_flat(nr.kmv_mlp_grad_analytic(nr.mlp_unflat(flat, dims), x, v, tau, cfg))
    assert np.allclose(ga, nr.fd_grad(f, flat, eps=1e-6), rtol=1e-6, atol=1e-8)


def test_mlp_taylor_terms_and_adjoint_vs_finite_differences():
    """The MLP residual's per-sample terms (grad, V', V'') and the analytic parameter adjoint that
    mlp.hip implements, against central differences (tiny net, fp64)."""
    rng = np.random.default_rng(1)
    dims = [2, 5, 4, 3]
    flat = rng.standard_normal(sum(dims[i] * dims[i + 1] + dims[i + 1] for i in range(3))) * 0.6
    P = nr.mlp_unflat(flat, dims)
    x, v = rng.standard_normal((7, 2)), rng.standard_normal((7, 2))
    V, g, Vd, Vdd = nr.mlp_forward_terms(P, x, v)
    e = 1e-5
    Vp, Vm = nr.mlp_forward_terms(P, x + e * v, v)[0], nr.mlp_forward_terms(P, x - e * v, v)[0]
    assert np.allclose((Vp - Vm) / (2 * e), Vd, atol=1e-7)
    assert np.allclose((Vp - 2 * V + Vm) / e ** 2, Vdd, atol=1e-3)
    zi, zt, z0 = (rng.standard_normal((m, 4)) for m in (20, 15, 60))
    gt = nr.grad_gmm(nr.gmm_centres(2, 3))
    f = lambda fl: nr.kfp_mlp_loss(nr.mlp_unflat(fl, dims), zi, zt, z0, gt, 0.5, 2.0)[0]
    ga = nr.mlp_flat(nr.kfp_mlp_grad_analytic(P, zi, zt, z0, 0.5, 2.0))
    assert np.allclose(ga, nr.fd_grad(f, flat, eps=1e-6), rtol=1e-6, atol=1e-8)


def test_fp_mlp_laplacian_and_adjoint_vs_finite_differences():
    """Overdamped FP residual (fokker_planck.py:33-63): the Laplacian as d Taylor directions against
    second differences, and the analytic adjoint (rows [x | e_k] + value-weighted boundary rows, the
    layout pdeinv_fp_rows builds) against central differences of the loss (tiny net, fp64)."""
    rng = np.random.default_rng(3)
    dims = [3, 5, 4, 3]
    flat = rng.standard_normal(sum(dims[i] * dims[i + 1] + dims[i + 1] for i in range(3))) * 0.6
    P = nr.mlp_unflat(flat, dims)
    x = rng.standard_normal((6, 3))
    e = 1e-4
    V = lambda y: nr.mlp_forward_terms(P, y, np.zeros_like(y))[0]
    lap_fd = sum((V(x + e * np.eye(3)[k]) - 2 * V(x) + V(x - e * np.eye(3)[k])) / e ** 2 for k in range(3))
    lap = sum(nr.mlp_forward_terms(P, x, np.tile(np.eye(3)[k], (6, 1)))[3] for k in range(3))
    assert np.allclose(lap, lap_fd, atol=1e-5)
    F = nr.problem_constants(3)
    xi, xt, x0 = (rng.standard_normal((m, 3)) for m in (20, 15, 40))
    f = lambda fl: nr.fp_mlp_loss(nr.mlp_unflat(fl, dims), xi, xt, x0, F, 2.0)[0]
    ga = nr.mlp_flat(nr.fp_mlp_grad_analytic(P, xi, xt, x0, 2.0))
    assert np.allclose(ga, nr.fd_grad(f, flat, eps=1e-6), rtol=1e-6, atol=1e-8)


def test_fp_closed_form_matches_moment_ode():
    """fokker_planck_example.py:101-116 (test_OU, printed only in the reference): the closed form
    of OU_process against the moment ODE dm/dt = -F m, dP/dt = -FP - PF + L — asserted here."""
    from scipy.integrate import solve_ivp
    cfg = nr.fp_configuration(nr.problem_constants(4))
    F, L = cfg["F"], cfg["L"]

    def rhs(t, y):
        m, Pm = y[:4], y[4:].reshape(4, 4)
        return np.concatenate([-F @ m, (-F @ Pm - Pm @ F + L).ravel()])
    ts = np.linspace(0, 2.0, 11)
    sol = solve_ivp(rhs, (0, 2.0), np.concatenate([cfg["m_0"], cfg["P_0"].ravel()]), t_eval=ts, rtol=1e-10,
                    atol=1e-12)
    for k, t in enumerate(ts):
        m, Pc = nr.fp_mean_cov(t, cfg)
        assert np.abs(m - sol.y[:4, k]).max() < 1e-7 and np.abs(Pc - sol.y[4:, k].reshape(4, 4)).max() < 1e-7


def test_shared_clock_stamp_times_match_c_oracle(oracle_lib):
    """utils.mean_field.stamp_times (host, no device sync) reproduces the interacting simulator's
    shared-clock tau rows bit for bit (C oracle of pdeinv_mf_step's tau0 + k dt)."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pde-inverse-problem_amd"))
    from utils.mean_field import stamp_times
    A = nr.problem_constants(2)
    z0 = np.random.default_rng(1).standard_normal((64, 4)).astype(np.float32)
    for seed, ctr in ((0xABCDEF, 5), (0x5EED_0004, 101 * 7), (2**40 + 3, 0)):
        o = oracle_lib.sde_simulate(z0, 30, 0.02, 1.0, "meanfield", A, seed=seed, counter_offset=ctr)
        assert np.array_equal(o["tau"][:, 0], stamp_times(seed, ctr, 30, 0.02))


@pytest.mark.parametrize("d,N,n,explicit", [(2, 300, 25, False), (3, 257, 12, True), (8, 130, 20, False)])
def test_mean_field_closed_form_mean_path_matches_interacting_oracle(oracle_lib, d, N, n, explicit):
    """The fused McKean–Vlasov driver's premise, pinned on the CPU: the mean path unrolled from
    [count, sum z0, sum of each update's noise] (numpy_ref.mf_mean_path) equals the mean of the
    interacting C-oracle simulation, whose every update recomputes xbar from all fp32 states
    (oracle_sde_simulate kind=meanfield). Both the Philox and the explicit-noise stream. Tolerance 2e-6
    of the state scale (the oracle's fp32 states vs the fp64 recursion)."""
    A = nr.problem_constants(d)
    rng = np.random.default_rng(d + N)
    z0 = (rng.standard_normal((N, 2 * d)) + 0.7).astype(np.float32)  # non-centred: the mean moves
    seed, ctr, dt = 0x5EED_0004 + d, 17, 0.02
    noise = rng.standard_normal((n + 1, N, d)).astype(np.float32) if explicit else None
    o = oracle_lib.sde_simulate(z0, n, dt, 1.0, "meanfield", A, seed=seed, counter_offset=ctr, noise=noise)
    if explicit:
        xi_sum = noise.astype(np.float64).sum(1)
    else:
        xi_sum = np.array([[oracle_lib.sim_normals(seed, i, ctr + s, d) for i in range(N)] for s in range(n + 1)],
                          np.float64).sum(1)
    sums = np.concatenate([[N], z0[:, :d].astype(np.float64).sum(0), z0[:, d:].astype(np.float64).sum(0),
                           xi_sum.ravel()])
    tau0 = float(o["tau"][0, 0])
    path = nr.mf_mean_path(sums, d, n, dt, tau0, 1.0)
    actual = np.concatenate([z0[None, :, :d], o["traj"][:, :, :d], o["last"][None, :, :d]]).astype(np.float64).mean(1)
    scale = 1 + np.abs(o["traj"]).max()
    assert np.abs(path - actual).max() < 2e-6 * scale, np.abs(path - actual).max()


@pytest.mark.parametrize("dim,mask_type,E,soft_init,act", [(1, "loop", 10, 1.0, "celu"), (2, "loop", 10, 1.0, "celu"),
                                                           (2, "random", 0, 0.0, "tanh"), (2, "loop", 6, 1.0, "silu")])
def test_realnvp_restatement_is_a_normalised_invertible_density(dim, mask_type, E, soft_init, act):
    """Pins the RealNVP restatement (normalizing_flow.py:115-229) without JAX: the sampling direction
    inverts the likelihood direction (x -> x0 -> x) with opposite log-det-Jacobians, and exp(log p_t)
    integrates to 1 over x (change of variables; 1-D and 2-D quadrature)."""
    couple = 4 if mask_type == "loop" else 3
    masks = nr.nvp_masks(dim, couple, mask_type)
    flat = nr.nvp_init(dim, masks.shape[0], E, False, seed=dim, scale=1.5, perturb=True)
    kw = dict(dim=dim, masks=masks, E=E, soft_init=soft_init, act=act)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((200, dim))
    t = rng.uniform(0, 2, 200)
    x0, ldj_r = nr.realnvp_apply(flat, t, x, reverse=True, **kw)
    x1, ldj_f = nr.realnvp_apply(flat, t, x0, reverse=False, **kw)
    assert np.max(np.abs(x1 - x)) < 1e-10 and np.max(np.abs(ldj_r + ldj_f)) < 1e-10
    mean, cov = np.full(dim, 0.3), np.eye(dim) * 1.7
    g = np.linspace(-60, 60, 12001) if dim == 1 else np.linspace(-60, 60, 801)
    pts = g[:, None] if dim == 1 else np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
    for tt in (0.0, 0.7):
        p = np.exp(nr.realnvp_logdensity(flat, tt, pts, base_mean=mean, base_cov=cov, **kw))
        integral = p.sum() * (g[1] - g[0]) ** dim
        assert abs(integral - 1.0) < 2e-3, integral


@pytest.mark.parametrize("dim,E,soft_init,ignore_time,act", [(2, 10, 1.0, False, "celu"), (3, 0, 0.0, False, "celu"),
                                                             (1, 4, 1.0, True, "tanh")])
def test_realnvp_nll_gradient_restatement(dim, E, soft_init, ignore_time, act):
    """The maximum-likelihood value_and_grad restatement (log_density_estimation.py:47-58): its value
    is the NumPy log-density restatement's negative mean, and its autograd gradient matches central
    differences of that NumPy restatement (fp64) on random coordinates."""
    masks = nr.nvp_masks(dim, 2, "loop")
    flat = nr.nvp_init(dim, masks.shape[0], E, ignore_time, seed=7, scale=1.3, perturb=True)
    rng = np.random.default_rng(3)
    x = rng.standard_normal((64, dim))
    t = rng.uniform(0, 2, 64)
    mean, cov = np.full(dim, 0.2), np.eye(dim) * 1.4
    kw = dict(dim=dim, masks=masks, E=E, ignore_time=ignore_time, soft_init=soft_init, act=act)
    loss, grad = nr.realnvp_nll_value_and_grad(flat, t, x, base_mean=mean, base_cov=cov, **kw)

    def nll(th):
        return -nr.realnvp_logdensity(th, t, x, base_mean=mean, base_cov=cov, **kw).mean()

    assert abs(loss - nll(flat)) < 1e-12 * (1 + abs(loss))
    idx = rng.choice(flat.size, 40, replace=False)
    h = 1e-6
    for k in idx:
        e = np.zeros_like(flat)
        e[k] = h
        fd = (nll(flat + e) - nll(flat - e)) / (2 * h)
        assert abs(fd - grad[k]) < 1e-6 * (1 + abs(fd)), (k, fd, grad[k])
