"""The accuracy half of BASELINE.json's metric, asserted on the GPU path.

* Recovered drift (north_star: "recovered drift parameters within 1e-3 of the analytic ground truth"):
  config C2 (kinetic OU, d = 4, 2^21 particles, T = 2, gamma = 1). The quadratic model's exact loss
  minimiser S = K + K^T (what Adam converges to on this convex loss; kinetic_fokker_planck_example_OU.py:
  209-220, kinetic_fokker_planck.py:33-61) from Philox EM moments at n = 100 / 200 / 400, two Richardson
  levels (the EM bias is O(dt)). Tolerance: max |S - tilde_F| <= 1e-3 (the north_star figure).
  Budget: 512 ensembles per level (5.4e8 trajectories per level; ~3 s on one MI355X), about 4x the
  bench's, so the Monte-Carlo error (~3.5e-4) sits well inside the bar.
* test_partial_s_log_density.py at ITS OWN configuration (:9-62, :241-311): d = 10, gamma = 0.1,
  P_v0 = 0.1, P_x0 = 1, m0 = 0, T = 1, s = 0.1, x ~ U[0, 1) — the lightly damped regime. The GPU kernel
  (kmv_weights, coefficient rows from dlogrho_coefficients) against central differences of the fp64
  log density (delta 1e-4 / 1e-3, relative RMSE < 1e-3, the reference's printed check, now asserted) and
  against the committed fixture tests/golden/dlogrho_d10_refcfg.npz (1e-4 / 1e-3 of the term scale).
"""
import os

import numpy as np
import pytest
import torch

from oracle import numpy_ref as nr

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device="cuda")


def test_c2_drift_recovery_within_1e3(native):
    from example_problems.kinetic_fokker_planck_example_OU import problem_matrix
    from methods.consistency_instances.kinetic_fokker_planck import recover_drift_richardson
    d, N, n, T, gamma = 4, 1 << 21, 100, 2.0, 1.0
    F = problem_matrix(d)
    z0 = native.gaussian_sample(N, torch.zeros(2 * d, device="cuda"), torch.eye(2 * d, device="cuda"),
                                seed=0x5EED_0001 ^ 0xA5A5)
    rec = recover_drift_richardson(z0, F, gamma, T, n, seed=0x5EED_0001, passes=512)
    err_em = np.abs(rec["S_n"] - F).max()
    err = np.abs(rec["S_rich"] - F).max()
    assert err_em > 0.02, err_em           # the O(dt) EM bias is really there at n = 100 ...
    assert err <= 1e-3, (err, rec["S_rich"], F)   # ... and Richardson removes it to the north_star bar
    assert np.abs(rec["S_rich1"] - F).max() <= 2e-3


def _refcfg():
    g = np.load(os.path.join(GOLD, "dlogrho_d10_refcfg.npz"))
    cfg = nr.ou_configuration(g["F"], gamma=float(g["gamma"]), P_x0=float(g["P_x0"]), P_v0=float(g["P_v0"]))
    return g, cfg


def test_partial_s_log_density_reference_configuration(native):
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    from example_problems.kinetic_fokker_planck_example_OU import initialize_configuration
    g, cfg = _refcfg()
    x, s = g["x"], float(g["s"])
    d = x.shape[1]
    ic = initialize_configuration(d, gamma_friction=float(g["gamma"]), P_x_0_scale=float(g["P_x0"]),
                                  P_v_0_scale=float(g["P_v0"]))
    assert np.allclose(ic["tilde_F"], g["F"]) and np.allclose(ic["P_0"], cfg["P_0"]) and np.allclose(ic["F"], cfg["F"])
    coef = _t(dlogrho_coefficients([s], ic, d))
    _, ds = native.kmv_weights(d, float(g["gamma"]), coef, _t(x), 1, len(x), 0, d, want_ds=True)
    ds = ds[0].double().cpu().numpy()
    fd1 = (nr.log_density(s + 1e-4, x, cfg) - nr.log_density(s - 1e-4, x, cfg)) / 2e-4
    fd2 = (nr.partial_s_log_density(s + 1e-3, x, cfg) - nr.partial_s_log_density(s - 1e-3, x, cfg)) / 2e-3
    assert np.sqrt(np.mean(((ds[:, 0] - fd1) / fd1) ** 2)) < 1e-3
    assert np.sqrt(np.mean(((ds[:, 1] - fd2) / fd2) ** 2)) < 1e-3
    assert np.max(np.abs(ds[:, 0] - g["ds"]) / (1 + np.abs(g["ds"]))) < 1e-4
    assert np.max(np.abs(ds[:, 1] - g["ds2"]) / (1 + np.abs(g["ds2"]))) < 1e-3


def test_partial_s_log_density_reference_configuration_host_api(native):
    """The same KAT through the reference-shaped method (KineticMcKeanVlasov.partial_s[2]_log_density_fn)
    with the reference test's configuration put in through the problem's initial_configuration."""
    from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov
    from example_problems.kinetic_fokker_planck_example_OU import initialize_configuration
    from utils import config, prng
    g, cfg = _refcfg()
    x, s = g["x"], float(g["s"])
    d = x.shape[1]
    c = config.compose("config", ["pde_instance=kinetic_mckean_vlasov", f"pde_instance.domain_dim={d}",
                                  "pde_instance.total_evolving_time=1.0"])
    pi = KineticMcKeanVlasov(c, prng.PRNGKey(0))
    pi.initial_configuration = initialize_configuration(d, gamma_friction=float(g["gamma"]),
                                                        P_x_0_scale=float(g["P_x0"]), P_v_0_scale=float(g["P_v0"]))
    ds = pi.partial_s_log_density_fn(s, _t(x)).double().cpu().numpy()
    ds2 = pi.partial_s2_log_density_fn(s, _t(x)).double().cpu().numpy()
    assert np.max(np.abs(ds - g["ds"]) / (1 + np.abs(g["ds"]))) < 1e-4
    assert np.max(np.abs(ds2 - g["ds2"]) / (1 + np.abs(g["ds2"]))) < 1e-3
