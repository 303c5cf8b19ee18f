"""GPU tests of the reference-shaped host API (registry / problems / method / trainer) and of
the McKean–Vlasov path, against the CPU oracle (oracle/numpy_ref.py, oracle/pdeinv_oracle.c).

Tolerances: residual terms 1e-4 relative (fp32 sums, fp64 across blocks); ds log rho 1e-4
relative to the term scale; mean-field trajectories 2e-4 absolute vs the C oracle.
"""
import numpy as np
import pytest
import torch

from oracle import numpy_ref as nr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


def _cfg(overrides):
    from utils import config
    return config.compose("config", overrides)


def test_kmv_residual_vs_pairwise_restatement(native):
    """Moment-form KMV residual == the reference's literal O(n^2) pairwise formulation."""
    from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov
    from methods.consistency_instances import kinetic_mckean_vlasov as kmv
    from core.model import QuadraticModel
    from utils import prng
    d, n, n_t = 3, 300, 4
    cfg = _cfg(["pde_instance=kinetic_mckean_vlasov", f"pde_instance.domain_dim={d}"])
    pi = KineticMcKeanVlasov(cfg, prng.PRNGKey(0))
    rng = np.random.default_rng(1)
    x = rng.standard_normal((n, n_t, d)); v = rng.standard_normal((n, n_t, d))
    tau = np.array([0.3, 0.7, 1.1, 1.9])
    K = rng.standard_normal((d, d)) * 0.3; b = rng.standard_normal(d) * 0.2
    z = np.concatenate([x, v], -1).reshape(-1, 2 * d)  # reference order rows (i, t)
    model = QuadraticModel(d)
    params = model.unflat(_t(np.concatenate([K.ravel(), b])))
    res = kmv.value_and_grad_fn(model.apply, params, {"0T": _t(z), "tau_0T": tau}, None, pi)
    cfg_np = nr.ou_configuration(pi.initial_configuration["tilde_F"], gamma=1.0)
    loss, loss_gt = nr.kmv_pairwise_loss(K, b, x, v, tau, cfg_np)
    assert abs(float(res["loss"]) - loss) < 2e-4 * (1 + abs(loss))
    assert abs(float(res["loss ground truth"]) - loss_gt) < 2e-4 * (1 + abs(loss_gt))
    g_fd = nr.fd_grad(lambda th: nr.kmv_pairwise_loss(th[:d * d].reshape(d, d), th[d * d:], x, v, tau, cfg_np)[0],
                      np.concatenate([K.ravel(), b]), eps=1e-5)
    g = torch.cat([res["grad"]["params"]["tilde_F"]["kernel"].reshape(-1), res["grad"]["params"]["tilde_F"]["bias"]])
    assert np.allclose(g.cpu().numpy(), g_fd, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("d", [2, 8])
def test_kmv_sde_stamp_sums_product_path(native, d):
    """The product path of the McKean-Vlasov SDE scheme with a quadratic model: sample_data takes the per-stamp sums
    from the simulator (simulate_interacting(stamp_sums=True): pdeinv_sde_simulate_mf_kmv, no trajectory written),
    value_and_grad_fn consumes data["kmv_sums"]; the same simulate with its trajectory written and the residual's own
    pass over it gives the same loss / loss ground truth / gradient (fp32 reassociation: 1e-5 relative) and the same
    stamps."""
    from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov
    from methods.consistency_instances import kinetic_mckean_vlasov as kmv
    from core.model import QuadraticModel
    from utils import prng
    cfg = _cfg(["pde_instance=kinetic_mckean_vlasov", f"pde_instance.domain_dim={d}"])
    pi = KineticMcKeanVlasov(cfg, prng.PRNGKey(0))
    rng = np.random.default_rng(d)
    model = QuadraticModel(d)
    params = model.unflat(_t(np.concatenate([rng.standard_normal(d * d) * 0.3, rng.standard_normal(d) * 0.2])))
    ctr = pi._counter
    _, ra = pi.simulate_interacting(prng.PRNGKey(21), 3000)
    pi._counter = ctr
    _, rb = pi.simulate_interacting(prng.PRNGKey(21), 3000, stamp_sums=True)
    assert "traj" not in rb
    tau_a = ra["tau"][:, 0].double().cpu().numpy()
    assert np.array_equal(tau_a, rb["tau_0T"])
    res_a = kmv.value_and_grad_fn(model.apply, params, {"0T_tm": ra["traj"], "tau_0T": tau_a, "shared_time": True},
                                  None, pi)
    res_b = kmv.value_and_grad_fn(model.apply, params, {"kmv_sums": (rb["kmv_mom"], rb["kmv_wst"]),
                                                        "tau_0T": rb["tau_0T"], "shared_time": True}, None, pi)
    for k in ("loss", "loss ground truth"):
        a, b = float(res_a[k]), float(res_b[k])
        assert abs(a - b) < 1e-5 * (1 + abs(a)), (k, a, b)
    ga = torch.cat([res_a["grad"]["params"]["tilde_F"]["kernel"].reshape(-1), res_a["grad"]["params"]["tilde_F"]["bias"]])
    gb = torch.cat([res_b["grad"]["params"]["tilde_F"]["kernel"].reshape(-1), res_b["grad"]["params"]["tilde_F"]["bias"]])
    assert (ga - gb).abs().max().item() < 1e-5 * (1 + ga.abs().max().item())
    assert torch.equal(ra["last"], rb["last"])


@pytest.mark.parametrize("d,n,chunk,W,L,impl", [(2, 40, 1 << 18, 20, 3, 0), (4, 37, 300, 20, 3, 1),
                                                (4, 37, 300, 20, 3, 2), (3, 70, 300, 10, 2, 2),
                                                (2, 130, 300, 20, 8, 2), (8, 65, 300, 28, 2, 2),
                                                (1, 66, 300, 16, 4, 2), (2, 530, 300, 20, 2, 2),
                                                (2, 70, 300, 28, 12, 2), (2, 60, 300, 64, 2, 2),
                                                (8, 40, 1 << 18, 256, 2, 0), (4, 45, 500, 100, 3, 2),
                                                (4, 33, 256, 32, 2, 0), (8, 45, 300, 20, 3, -2), (3, 70, 300, 10, 2, -2),
                                                (2, 300, 300, 20, 3, -2),
                                                # dims other than 2 / 4 / 8 and one hidden layer on the fused
                                                # wide-net path (pair rows zero-padded; no rocBLAS)
                                                (3, 45, 300, 64, 2, 2), (5, 40, 300, 32, 2, 0),
                                                (2, 50, 300, 64, 1, 2),
                                                # dims 9..16 on the fused wide-net path (pair rows padded to 16)
                                                (12, 40, 300, 64, 2, 0), (16, 30, 300, 32, 1, 2)])
def test_kmv_general_phi_mlp_vs_pairwise_restatement(native, d, n, chunk, W, L, impl):
    """General Phi_theta = V_hypothesis (non-parametric KMV, kinetic_mckean_vlasov.py:11-120) == the
    literal pair-tensor restatement (loss, loss ground truth, terms) and its FD-checked analytic gradient
    (oracle kmv_mlp_grad_analytic), on both implementations: impl 2 / auto = the narrow-net pair kernels
    (pairs built in registers, MFMA weight gradients; odd widths / dims zero-padded; n not a multiple of
    the 64-pair tile), impl 1 = pair rows through rocBLAS (chunk = 300 forces partial i-blocks and
    j-chunking). (2, 130, ..., 20, 8) is the reference's default net (MLP.yaml: width 20, 8 layers);
    n = 530 spans two of pass 2's 512-reference work units (a partial second one). (2, 70, ..., 28, 12)
    pads to more than 8 192 parameters, so pass 2 takes its global-memory weight-gradient slab
    (kmvp_grad_kernel<D, W, false>) instead of the LDS slab. Widths >= 32 (64, 256 = the C5 width, 100
    zero-padded to 128, 32) run the pair rows through the fused fp32-MFMA residual kernels (no rocBLAS),
    chunked (300 / 500 / 256 rows: partial i-blocks and j-chunks).
    impl = -2: impl 2 with every parameter perturbed by 0.15 N(0, 1) (non-zero biases: the initialiser's
    are zero), on the MFMA pair-tile kernels (widths <= 20: mlp_pairs_mfma.hip).
    Tolerance 2e-4 relative (fp32)."""
    from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov
    from methods.consistency_instances import kinetic_mckean_vlasov as kmv
    from core.model import V_hypothesis
    from utils import native as nat, prng
    perturb = impl < 0
    impl = abs(impl)
    n_t = 3
    cfg = _cfg(["pde_instance=kinetic_mckean_vlasov", f"pde_instance.domain_dim={d}"])
    pi = KineticMcKeanVlasov(cfg, prng.PRNGKey(0))
    rng = np.random.default_rng(7)
    x = rng.standard_normal((n, n_t, d)); v = rng.standard_normal((n, n_t, d))
    tau = np.array([0.3, 0.9, 1.6])
    net = V_hypothesis(output_dim=1, hidden_dims=[W] * L)
    params = net.init(prng.PRNGKey(11), np.zeros(d), device=DEV)
    dims = net.dims(d)
    flat = net.flat(params)
    if perturb:
        flat = flat + torch.as_tensor(0.15 * rng.standard_normal(flat.numel()), dtype=flat.dtype, device=flat.device)
    P = nr.mlp_unflat(flat.double().cpu().numpy(), dims)
    cfg_np = nr.ou_configuration(pi.initial_configuration["tilde_F"], gamma=1.0)
    loss, loss_gt, parts = nr.kmv_mlp_pairwise_loss(P, x, v, tau, cfg_np)
    ga = nr.mlp_flat(nr.kmv_mlp_grad_analytic(P, x, v, tau, cfg_np))
    z = _t(np.concatenate([x, v], -1).reshape(-1, 2 * d))  # reference order rows (i, t)
    if chunk == 1 << 18:
        res = kmv.value_and_grad_fn(net.apply, params, {"0T": z, "tau_0T": tau}, None, pi)
        out, g = None, torch.cat([t.reshape(-1) for lay in res["grad"]["params"].values()
                                  for t in (lay["kernel"], lay["bias"])])
        got_loss, got_gt = float(res["loss"]), float(res["loss ground truth"])
    else:
        coef = pi.coefficients(tau, z.device)
        _, ds = nat.kmv_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d, want_ds=True)
        acc, g = nat.residual_kmv_mlp(dims, flat, z, n_t, n, 2 * d, n_t * 2 * d, ds,
                                      pi.initial_configuration["tilde_F"], 1.0, chunk_rows=chunk, impl=impl)
        out = nat.kfp_terms_finalize(acc, g, 1.0).cpu().numpy()
        got_loss, got_gt = float(out[nat.KFP_SLOTS.index("loss")]), float(out[nat.KFP_SLOTS.index("loss ground truth")])
        assert abs(out[nat.KFP_SLOTS.index("loss_Hessian")] - parts["hessian"]) < 2e-4 * (1 + abs(parts["hessian"]))
        assert abs(out[nat.KFP_SLOTS.index("loss_nabla")] - parts["nabla"]) < 2e-4 * (1 + abs(parts["nabla"]))
    assert abs(got_loss - loss) < 2e-4 * (1 + abs(loss))
    assert abs(got_gt - loss_gt) < 2e-4 * (1 + abs(loss_gt))
    g = g.double().cpu().numpy()
    assert np.abs(g - ga).max() < 2e-4 * (1 + np.abs(ga).max())


def test_kmv_general_phi_pair_kernels_golden_1400(native):
    """The pair kernels at a size where pass 1's persistent grid (2 048 waves over n * n_time items)
    iterates: d = 2, n = 1 400, 3 stamps (4 200 items), the reference's default 20 x 8 net, against the
    committed fp64 restatement (tests/golden/kmv_mlp_pairs_1400.npz, oracle/make_golden.py
    kmv_mlp_large: the literal pair tensor of kinetic_mckean_vlasov.py:20-23, 74-97, evaluated 250
    references at a time). Tolerance 2e-4 relative (fp32)."""
    import os
    from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov
    from utils import native as nat, prng
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "kmv_mlp_pairs_1400.npz"))
    x, v, tau, dims = g["x"], g["v"], g["tau"], [int(t) for t in g["dims"]]
    n, n_t, d = x.shape
    cfg = _cfg(["pde_instance=kinetic_mckean_vlasov", f"pde_instance.domain_dim={d}"])
    pi = KineticMcKeanVlasov(cfg, prng.PRNGKey(0))
    assert np.allclose(np.asarray(pi.initial_configuration["tilde_F"], np.float64), g["F"])
    z = _t(np.concatenate([x, v], -1).reshape(-1, 2 * d))
    coef = pi.coefficients(tau, z.device)
    _, ds = nat.kmv_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d, want_ds=True)
    acc, grad = nat.residual_kmv_mlp(dims, _t(g["flat"]), z, n_t, n, 2 * d, n_t * 2 * d, ds, g["F"], 1.0,
                                     impl=nat.MLP_IMPL_FUSED)
    out = nat.kfp_terms_finalize(acc, grad, 1.0).cpu().numpy()
    for key, slot in (("loss", "loss"), ("loss_gt", "loss ground truth"), ("hessian", "loss_Hessian"),
                      ("nabla", "loss_nabla")):
        ref = float(g[key])
        assert abs(out[nat.KFP_SLOTS.index(slot)] - ref) < 2e-4 * (1 + abs(ref)), (key, out[nat.KFP_SLOTS.index(slot)], ref)
    ga = g["grad"]
    gg = grad.double().cpu().numpy()
    assert np.abs(gg - ga).max() < 2e-4 * (1 + np.abs(ga).max()), np.abs(gg - ga).max()


@pytest.mark.parametrize("scale", [3e-4, 0.005])
def test_kmv_general_phi_output_near_zero(native, scale):
    """The regime training drives the interaction net into (Phi*(0) = 0): the output layer's bias is set to
    b = -K_L^T h(0), so the net's output y vanishes at the origin, and the particles sit close together
    (x ~ scale N(0, 1)), so every pair's |y| is small against |b|. The MFMA pair tiles fold the output
    layer into a quadratic form expanded at h(0) (mlp_pairs_mfma.hip): the value term, the Hessian term
    and the gradient must keep their RELATIVE accuracy against the fp64 pair-tensor restatement (an
    unshifted fold h^T M h + 2 c^T h + |b|^2 loses it to cancellation, ~eps |b|^2 / |y|^2). Reference
    default net (20 x 8, out 40), perturbed. Tolerances 2e-4 relative to each term / the gradient norm."""
    from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov
    from core.model import V_hypothesis
    from utils import native as nat, prng
    d, n, n_t, W, L = 2, 160, 2, 20, 8
    cfg = _cfg(["pde_instance=kinetic_mckean_vlasov", f"pde_instance.domain_dim={d}"])
    pi = KineticMcKeanVlasov(cfg, prng.PRNGKey(0))
    rng = np.random.default_rng(21)
    x = (scale * rng.standard_normal((n, n_t, d))).astype(np.float32).astype(np.float64)
    v = rng.standard_normal((n, n_t, d)).astype(np.float32).astype(np.float64)
    tau = np.array([0.4, 1.2])
    net = V_hypothesis(output_dim=1, hidden_dims=[W] * L)
    dims = net.dims(d)
    flat = net.flat(net.init(prng.PRNGKey(11), np.zeros(d), device=DEV)).double().cpu().numpy()
    flat = flat + 0.15 * rng.standard_normal(flat.size)
    P = nr.mlp_unflat(flat.astype(np.float32).astype(np.float64), dims)
    h0 = np.zeros(d)
    for K, b in P[:-1]:
        h0 = np.tanh(h0 @ K + b)
    Ko, _ = P[-1]
    P[-1] = (Ko, (-(h0 @ Ko)).astype(np.float32).astype(np.float64))
    flat = nr.mlp_flat(P)
    cfg_np = nr.ou_configuration(pi.initial_configuration["tilde_F"], gamma=1.0)
    loss, loss_gt, parts = nr.kmv_mlp_pairwise_loss(P, x, v, tau, cfg_np)
    ga = nr.mlp_flat(nr.kmv_mlp_grad_analytic(P, x, v, tau, cfg_np))
    z = _t(np.concatenate([x, v], -1).reshape(-1, 2 * d))
    coef = pi.coefficients(tau, z.device)
    _, ds = nat.kmv_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d, want_ds=True)
    acc, g = nat.residual_kmv_mlp(dims, _t(flat), z, n_t, n, 2 * d, n_t * 2 * d, ds,
                                  pi.initial_configuration["tilde_F"], 1.0, impl=nat.MLP_IMPL_FUSED)
    out = nat.kfp_terms_finalize(acc, g, 1.0).cpu().numpy()
    fric = out[nat.KFP_SLOTS.index("loss_friction")]
    hess = out[nat.KFP_SLOTS.index("loss_Hessian")]
    assert abs(fric - 2 * parts["value"]) < 2e-4 * abs(2 * parts["value"]), (fric, 2 * parts["value"])
    assert abs(hess - parts["hessian"]) < 2e-4 * abs(parts["hessian"]), (hess, parts["hessian"])
    gg = g.double().cpu().numpy()
    assert np.linalg.norm(gg - ga) < 2e-4 * np.linalg.norm(ga), np.linalg.norm(gg - ga) / np.linalg.norm(ga)


def test_kmv_general_phi_mfma_tiles_vs_ring_at_recipe_size(native, monkeypatch):
    """The reference's KMV recipe size (scripts/parametric/KMV/run_quadratic_online.sh: d = 2, one stamp,
    n = 5 000 -> 25 M pairs; the default 20 x 8 net, every parameter perturbed so the biases are non-zero):
    the MFMA pair tiles (mlp_pairs_mfma.hip: 20 reference chunks per particle, every persistent wave over
    many work units, the folded output layer) against the register-ring kernels (mlp_pairs.hip,
    impl = MLP_IMPL_PAIRS_RING), both checked against the pairwise restatement at smaller sizes above.
    Loss slots and gradient to 2e-5 relative (fp32 sums over 25 M pairs in different orders)."""
    from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov
    from core.model import V_hypothesis
    from utils import native as nat, prng
    d, n, n_t = 2, 5000, 1
    cfg = _cfg(["pde_instance=kinetic_mckean_vlasov", f"pde_instance.domain_dim={d}"])
    pi = KineticMcKeanVlasov(cfg, prng.PRNGKey(0))
    rng = np.random.default_rng(11)
    z = _t(rng.standard_normal((n * n_t, 2 * d)))
    tau = np.array([0.7])
    net = V_hypothesis(output_dim=1, hidden_dims=[20] * 8)
    params = net.init(prng.PRNGKey(11), np.zeros(d), device=DEV)
    dims = net.dims(d)
    flat = net.flat(params)
    flat = flat + torch.as_tensor(0.1 * rng.standard_normal(flat.numel()), dtype=flat.dtype, device=flat.device)
    coef = pi.coefficients(tau, z.device)
    _, ds = nat.kmv_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d, want_ds=True)
    run = lambda impl: nat.residual_kmv_mlp(dims, flat, z, n_t, n, 2 * d, n_t * 2 * d, ds,
                                            pi.initial_configuration["tilde_F"], 1.0, impl=impl)
    acc_q, g_q = run(nat.MLP_IMPL_FUSED)
    acc_r, g_r = run(nat.MLP_IMPL_PAIRS_RING)
    a_q, a_r = acc_q.cpu().numpy(), acc_r.cpu().numpy()
    assert np.abs(a_q - a_r).max() < 2e-5 * (1 + np.abs(a_r).max()), (a_q, a_r)
    gq, gr = g_q.double().cpu().numpy(), g_r.double().cpu().numpy()
    assert np.abs(gq - gr).max() < 2e-5 * np.abs(gr).max(), np.abs(gq - gr).max() / np.abs(gr).max()


def test_partial_s_log_density_kat(native):
    """test_partial_s_log_density.py:241-311 re-created and ASSERTED: d = 10, s = 0.1,
    central differences delta = 1e-4 (ds) and 1e-3 (ds2), relative RMSE < 1e-3; plus a direct
    comparison with the fp64 restatement."""
    from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov
    from utils import prng
    d = 10
    cfg = _cfg(["pde_instance=kinetic_mckean_vlasov", f"pde_instance.domain_dim={d}",
                "pde_instance.total_evolving_time=1.0"])
    pi = KineticMcKeanVlasov(cfg, prng.PRNGKey(0))
    x = np.random.default_rng(0).uniform(size=(3, d))
    s = 0.1
    ds = pi.partial_s_log_density_fn(s, _t(x)).double().cpu().numpy()
    ds2 = pi.partial_s2_log_density_fn(s, _t(x)).double().cpu().numpy()
    cfg_np = nr.ou_configuration(pi.initial_configuration["tilde_F"], gamma=1.0)
    fd1 = (nr.log_density(s + 1e-4, x, cfg_np) - nr.log_density(s - 1e-4, x, cfg_np)) / 2e-4
    fd2 = (nr.partial_s_log_density(s + 1e-3, x, cfg_np) - nr.partial_s_log_density(s - 1e-3, x, cfg_np)) / 2e-3
    ref1 = nr.partial_s_log_density(s, x, cfg_np); ref2 = nr.partial_s2_log_density(s, x, cfg_np)
    assert np.sqrt(np.mean(((ref1 - fd1) / fd1) ** 2)) < 1e-3
    assert np.sqrt(np.mean(((ref2 - fd2) / fd2) ** 2)) < 1e-3
    assert np.max(np.abs(ds - ref1) / (1 + np.abs(ref1))) < 1e-4
    assert np.max(np.abs(ds2 - ref2) / (1 + np.abs(ref2))) < 1e-3
    # vector s, matrix x -> [n_x, n_s] like the reference's vmap order
    both = pi.partial_s_log_density_fn(np.array([0.1, 0.5]), _t(x))
    assert tuple(both.shape) == (3, 2)


def test_mean_field_simulator_vs_c_oracle(native, oracle_lib):
    from utils.mean_field import simulate_mean_field
    from core.potential import MeanFieldQuadraticPotential
    from utils import prng
    d, N, n = 2, 2000, 50
    A = nr.problem_constants(d)
    z0 = np.random.default_rng(3).standard_normal((N, 2 * d)).astype(np.float32) + 0.5
    key = prng.Key(0xABCDEF)
    r = simulate_mean_field(_t(z0), n, 0.02, key, MeanFieldQuadraticPotential(A), 1.0, counter_offset=5)
    o = oracle_lib.sde_simulate(z0, n, 0.02, 1.0, "meanfield", A, seed=key.seed, counter_offset=5)
    assert np.array_equal(r["tau"].cpu().numpy(), o["tau"])
    from utils.mean_field import stamp_times
    assert np.array_equal(r["tau"][:, 0].cpu().numpy(), stamp_times(key.seed, 5, n, 0.02))
    assert np.max(np.abs(r["traj"].cpu().numpy() - o["traj"])) < 2e-4
    assert np.max(np.abs(r["last"].cpu().numpy() - o["last"])) < 2e-4


def test_mean_field_equals_ou_for_centred_ensemble(native):
    """with xbar_0 = vbar_0 = 0 the MV system's covariance is the OU chain's."""
    from utils.mean_field import simulate_mean_field
    from core.potential import MeanFieldQuadraticPotential
    from utils import prng
    d, N, n = 2, 1 << 17, 50
    A = nr.problem_constants(d)
    z0 = native.gaussian_sample(N, _t(np.zeros(2 * d)), _t(np.eye(2 * d)), seed=5)
    z0 = z0 - z0.mean(0)
    r = simulate_mean_field(z0, n, 0.02, prng.Key(9), MeanFieldQuadraticPotential(A), 1.0, random_shift=False)
    P0 = (z0.double().T @ z0.double() / N).cpu().numpy()
    mt, st, _, _ = nr.em_chain_moments(A, 1.0, 0.02, n, np.zeros(2 * d), P0, random_shift=False)
    z = r["traj"][n - 1].double()
    emp = (z.T @ z / N).cpu().numpy()
    P = st[n - 1]
    sig = np.sqrt((np.outer(np.diag(P), np.diag(P)) + P ** 2) / N)
    assert np.max(np.abs(emp - P) / sig) < 5.5


def _run(overrides, iters=3):
    import main
    cfg = _cfg(overrides + ["train.optimizer.learning_rate.initial=1e-2", "test.frequency=1000000"])
    trainer, params = main.run(cfg, number_of_iterations=iters)
    return trainer


def test_trainer_kou_exact(native):
    tr = _run(["pde_instance=kinetic_fokker_planck", "solver.train.batch_size_0T=20000",
               "solver.train.batch_size_init=2000", "solver.train.batch_size_terminal=2000"])
    assert len(tr.history) == 3 and all(np.isfinite(h["loss"]) for h in tr.history)


def test_trainer_kou_sde_fused_converges(native):
    """The fused simulate+moments path trains: loss ground truth decreases."""
    tr = _run(["pde_instance=kinetic_fokker_planck", "pde_instance.sample_scheme=SDE",
               "solver.train.batch_size_0T=50000", "train.optimizer.learning_rate.initial=5e-2"], iters=60)
    gt = [h["loss ground truth"] for h in tr.history]
    assert gt[-1] < 0.5 * gt[0]


def test_trainer_gmm_online_and_offline(native):
    for mode in ("online", "offline"):
        tr = _run(["pde_instance=kinetic_fokker_planck", "pde_instance.potential=GMM", f"pde_instance.sample_mode={mode}",
                   "pde_instance.n_steps=20", "solver.train.batch_size_0T=500", "pde_instance.sample_initial_size=5000",
                   "pde_instance.sample_terminal_size=2000", "pde_instance.sample_0T_size=1000",
                   "pde_instance.n_steps_terminal=40", "pde_instance.n_steps_0T=40"])
        assert all(np.isfinite(h["loss"]) for h in tr.history)


def test_trainer_kmv_exact_and_sde(native):
    base = ["pde_instance=kinetic_mckean_vlasov", "pde_instance.domain_dim=2", "solver.train.sample_mode=grid_time",
            "solver.train.sample_per_time=5000", "solver.train.n_time_stamps=1", "pde_instance.total_evolving_time=1"]
    tr = _run(base)
    assert all(np.isfinite(h["loss"]) for h in tr.history)
    tr = _run(base + ["pde_instance.sample_scheme=SDE", "pde_instance.n_steps=20"])
    assert all(np.isfinite(h["loss"]) for h in tr.history)


def test_trainer_kmv_sde_stamp_sums_route(native, monkeypatch):
    """The SDE scheme's two routes for a quadratic model (methods/consistency.py): the simulator's own stamp sums
    (default) and trajectory + KMV pass (STAMP_SUMS_MIN_BYTES raised past the trajectory) train to the same losses (fp32
    reassociation of the sums carried through the updates: 1e-4 relative)."""
    import methods.consistency as mc
    base = ["pde_instance=kinetic_mckean_vlasov", "pde_instance.domain_dim=2", "solver.train.sample_mode=grid_time",
            "solver.train.sample_per_time=5000", "solver.train.n_time_stamps=1", "pde_instance.total_evolving_time=1",
            "pde_instance.sample_scheme=SDE", "pde_instance.n_steps=20"]
    ta = _run(base)
    monkeypatch.setattr(mc, "STAMP_SUMS_MIN_BYTES", 1 << 62)
    tb = _run(base)
    la, lb = [h["loss"] for h in ta.history], [h["loss"] for h in tb.history]
    assert len(la) == len(lb) > 0
    assert np.allclose(la, lb, rtol=1e-4, atol=1e-6), (la, lb)


def test_trainer_kmv_non_parametric(native):
    """estimation_mode=non-parametric under KMV (get_model -> V_hypothesis, the MLP.yaml net of
    width 20 x 8 layers): the general-Phi pair-row residual drives the trainer end to end."""
    base = ["pde_instance=kinetic_mckean_vlasov", "pde_instance.domain_dim=2", "solver.train.sample_mode=grid_time",
            "solver.train.sample_per_time=300", "solver.train.n_time_stamps=1", "pde_instance.total_evolving_time=1",
            "estimation_mode=non-parametric"]
    tr = _run(base)
    assert all(np.isfinite(h["loss"]) for h in tr.history)


def test_no_cpu_fallback_for_callables(native):
    from utils.sampling_utils import underdamped_langevin_dynamics_scan
    from utils import prng
    with pytest.raises(NotImplementedError):
        underdamped_langevin_dynamics_scan(_t(np.zeros((4, 4))), 5, 0.1, prng.Key(1), lambda q: q, 1.0)


def test_reference_shaped_scan_outputs(native):
    from utils.sampling_utils import underdamped_langevin_dynamics_scan
    from core.potential import GMMPotential
    from utils import prng
    pot = GMMPotential(nr.gmm_centres(4, 3), 1.0)
    last, traj, tau = underdamped_langevin_dynamics_scan(_t(np.zeros((64, 8))), 30, 0.05, prng.Key(3), pot.gradient, 0.5)
    assert tuple(last.shape) == (64, 8) and tuple(traj.shape) == (64, 30, 8) and tuple(tau.shape) == (64, 30)
    # tau = tau0 + k dt with tau0 in [0, dt)  (sampling_utils.py:32, 48)
    t = tau.cpu().numpy()
    assert np.all((t[:, 0] >= 0) & (t[:, 0] < 0.05)) and np.allclose(np.diff(t, axis=1), 0.05, atol=1e-6)


def test_estimate_log_density_trains_on_offline_dataset(native):
    """core/log_density_estimation.py:13-100 on a small offline GMM dataset: the per-epoch strided
    subsample (1 in 5 time stamps, 1 in 5 trajectories), the native value_and_grad and Adam with the
    reference's schedule. The negative log-likelihood must fall, and the learned density must beat the
    untrained flow on held-out rows of the dataset."""
    from core import log_density_estimation as lde
    from registry import get_pde_instance
    from utils import prng
    cfg = _cfg(["pde_instance=kinetic_fokker_planck", "pde_instance.potential=GMM", "pde_instance.sample_mode=offline",
                "pde_instance.domain_dim=2", "pde_instance.sample_initial_size=2000",
                "pde_instance.sample_terminal_size=1000", "pde_instance.sample_0T_size=2000",
                "pde_instance.n_steps_terminal=40", "pde_instance.n_steps_0T=40"])
    rng = prng.PRNGKey(int(cfg.seed))
    pi = get_pde_instance(cfg)(cfg=cfg, rng=rng)
    fn = lde.estimate_log_density(cfg, pi, prng.PRNGKey(3), num_epochs=300, frequency=100, verbose=False)
    h = fn.history
    assert len(h) == 3 and all(np.isfinite(h)) and h[-1] < h[0] - 0.05, h
    rows = pi.dataset["0T"][:, 1::5, :2].reshape(-1, 2)
    times = pi.dataset["tau_0T"][:, 1::5].reshape(-1)
    fresh = lde.create_normalizing_flow_fn(pi.distribution_initial_x.logdensity, 2)
    p0 = fresh.init(prng.split(prng.PRNGKey(3), 2)[0], 0.0, np.zeros(2))
    assert fn(times, rows).mean().item() > fresh.apply(p0, times, rows).mean().item()
