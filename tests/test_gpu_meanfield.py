"""BASELINE config C4 (kinetic McKean–Vlasov, quadratic interaction, d = 8) on the GPU, against the
CPU oracle (oracle/pdeinv_oracle.c, oracle/numpy_ref.py) and the committed golden fixtures.

Reference: methods/consistency_instances/kinetic_mckean_vlasov.py:11-120 (pairwise residual),
example_problems/kinetic_mckean_vlasov_example_quadratic.py:18-216 (d_s log rho, Phi*), README.md:55-80
(the mean-field equivalence). Tolerances (written per test): Philox-mode trajectories 2e-4 absolute vs
the C oracle (hardware v_log / v_sin / v_cos vs libm in the normals); explicit-noise trajectories 2e-5
of the state scale; the two McKean–Vlasov drivers against each other 2e-5 of the state scale; moment
sums 1e-5 relative (fp32 per thread / block, fp64 across blocks); residual 1e-4 relative, gradient 1e-3.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import numpy_ref as nr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


def _sim(z0, n, A, exchange, seed=0x5EED_0004, ctr=5, noise=None, random_shift=True, dt=0.02):
    from core.potential import MeanFieldQuadraticPotential
    from utils import prng
    from utils.mean_field import simulate_mean_field
    return simulate_mean_field(z0, n, dt, prng.Key(seed), MeanFieldQuadraticPotential(A), 1.0, counter_offset=ctr,
                               noise=noise, random_shift=random_shift, exchange=exchange)


@pytest.mark.parametrize("exchange", ["fused", "per_update"])
@pytest.mark.parametrize("d,N", [(8, 4099), (8, 6000), (2, 2000), (3, 333)])
def test_mean_field_vs_c_oracle(native, oracle_lib, exchange, d, N):
    """Both McKean–Vlasov drivers vs the interacting C oracle (which recomputes xbar from all fp32 states
    before every update), n = 100. N = 4099 / 6000 leave whole waves of the last block past N (the staged
    row load/store of mf_step_kernel and its zero-initialised lanes); d = 3 takes the unstaged rows."""
    n = 100
    A = nr.problem_constants(d)
    z0 = (np.random.default_rng(d * 7 + N).standard_normal((N, 2 * d)) + 0.5).astype(np.float32)
    r = _sim(_t(z0), n, A, exchange)
    o = oracle_lib.sde_simulate(z0, n, 0.02, 1.0, "meanfield", A, seed=0x5EED_0004, counter_offset=5)
    assert np.array_equal(r["tau"].cpu().numpy(), o["tau"])
    assert np.max(np.abs(r["traj"].cpu().numpy() - o["traj"])) < 2e-4
    assert np.max(np.abs(r["last"].cpu().numpy() - o["last"])) < 2e-4
    assert torch.isfinite(r["xsum"]).all()


@pytest.mark.parametrize("d,N", [(8, 4099), (4, 777)])
def test_mean_field_explicit_noise_vs_c_oracle(native, oracle_lib, d, N):
    """Explicit-noise parity mode (no transcendental differences): the fused driver (noise sums from the
    noise buffer) and the per-update driver vs the C oracle on the same xi: 2e-5 of the state scale."""
    n = 100
    A = nr.problem_constants(d)
    rng = np.random.default_rng(N)
    z0 = (rng.standard_normal((N, 2 * d)) - 0.3).astype(np.float32)
    xi = rng.standard_normal((n + 1, N, d)).astype(np.float32)
    o = oracle_lib.sde_simulate(z0, n, 0.02, 1.0, "meanfield", A, seed=0x5EED_0004, counter_offset=5, noise=xi)
    scale = 1 + np.abs(o["traj"]).max()
    for exchange in ("fused", "per_update"):
        r = _sim(_t(z0), n, A, exchange, noise=_t(xi))
        assert np.max(np.abs(r["traj"].cpu().numpy() - o["traj"])) < 2e-5 * scale, exchange
        assert np.max(np.abs(r["last"].cpu().numpy() - o["last"])) < 2e-5 * scale, exchange


def test_mean_field_drivers_agree(native):
    """The closed-form mean path (one all-reduce per simulate) and the per-update exchange (xbar from the
    fp32 states) give the same ensemble: trajectories to 2e-5 of the state scale, the recorded
    [count, sum x] per update to 1e-6 relative."""
    d, N, n = 8, 50_000, 100
    A = nr.problem_constants(d)
    z0 = native.gaussian_sample(N, _t(np.full(2 * d, 0.4)), _t(np.eye(2 * d)), seed=3)
    a = _sim(z0, n, A, "fused")
    b = _sim(z0, n, A, "per_update")
    scale = 1 + b["traj"].abs().max().item()
    assert (a["traj"] - b["traj"]).abs().max().item() < 2e-5 * scale
    assert (a["last"] - b["last"]).abs().max().item() < 2e-5 * scale
    xa, xb = a["xsum"].cpu().numpy(), b["xsum"].cpu().numpy()
    assert np.array_equal(xa[:, 0], xb[:, 0])
    assert np.max(np.abs(xa[:, 1:] - xb[:, 1:])) < 1e-6 * N * (1 + np.abs(xb[:, 1:] / N).max())


def test_mean_field_full_size_centred_law(native):
    """SURVEY.md §8(c) P4 at the C4 size (2^21 particles per GPU, d = 8, n = 100, fused driver): with a
    centred initial ensemble the interacting system's second moments are the EM chain's with
    tilde_F = A (em_chain_moments) — every entry of E[z z^T] at three time stamps and at T within 5.5
    sigma_MC. The closed-form mean path also matches the actual mean of the simulated states (1e-6)."""
    d, N, n = 8, 1 << 21, 100
    A = nr.problem_constants(d)
    z0 = native.gaussian_sample(N, _t(np.zeros(2 * d)), _t(np.eye(2 * d)), seed=5)
    z0 = z0 - z0.mean(0)
    r = _sim(z0, n, A, "fused", seed=9, random_shift=False)
    P0 = (z0.double().T @ z0.double() / N).cpu().numpy()
    _, sec, _, sec_last = nr.em_chain_moments(A, 1.0, 0.02, n, np.zeros(2 * d), P0, random_shift=False)
    xbar = r["xbar"].double().cpu().numpy()
    for s in (9, 49, 99, n):
        z = r["last"] if s == n else r["traj"][s]
        mom = native.moments(z).cpu().numpy()
        _, mean, M = nr.unpack_moments(mom, 2 * d)
        P = sec_last if s == n else sec[s]
        sig = np.sqrt((np.outer(np.diag(P), np.diag(P)) + P ** 2) / N)
        assert np.max(np.abs(M - P) / sig) < 5.5, (s, np.max(np.abs(M - P) / sig))
        if s < n:  # xbar row s + 1 = the mean after update s
            assert np.max(np.abs(mean[:d] - xbar[s + 1])) < 1e-6, (s, np.abs(mean[:d] - xbar[s + 1]).max())


def test_moments_batched_m16(native):
    """moments_batched_kernel<16> (the C4 per-time-stamp moments of z = [x, v], d = 8) vs fp64 sums."""
    rng = np.random.default_rng(16)
    n_t, n = 5, 3001
    z = rng.standard_normal((n_t, n, 16)).astype(np.float32) + 0.2
    out = native.moments_batched(_t(z), n_t, n, 16, n * 16, 16).cpu().numpy()
    for t in range(n_t):
        ref = nr.moments(z[t].astype(np.float64))
        assert np.allclose(out[t], ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())


def _coef(d, tau):
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    cfg = nr.ou_configuration(nr.problem_constants(d))
    return cfg, _t(dlogrho_coefficients(np.asarray(tau, np.float64), cfg, d))


def test_kmv_weights_d8(native):
    """kmv_weights_kernel<8>: per-particle (d_s log rho, d_s^2 log rho) vs the fp64 restatement
    (…_quadratic.py:18-191) and the per-stamp c-weighted moments (c = ds2 + ds^2 + gamma ds)."""
    d, n = 8, 2500
    tau = [0.3, 1.1, 1.9]
    cfg, coef = _coef(d, tau)
    rng = np.random.default_rng(8)
    z = rng.standard_normal((len(tau), n, 2 * d)).astype(np.float32)
    wst, ds = native.kmv_weights(d, 1.0, coef, _t(z), len(tau), n, n * 2 * d, 2 * d, want_ds=True)
    wst, ds = wst.cpu().numpy(), ds.double().cpu().numpy()
    for t, s in enumerate(tau):
        x = z[t, :, :d].astype(np.float64)
        r1, r2 = nr.partial_s_log_density(s, x, cfg), nr.partial_s2_log_density(s, x, cfg)
        assert np.max(np.abs(ds[t, :, 0] - r1) / (1 + np.abs(r1))) < 1e-4
        assert np.max(np.abs(ds[t, :, 1] - r2) / (1 + np.abs(r2))) < 1e-3
        c = r2 + r1 ** 2 + 1.0 * r1
        ref = np.concatenate([[c.sum()], c @ x, ((x * c[:, None]).T @ x)[np.triu_indices(d)]])
        assert np.allclose(wst[t], ref, rtol=1e-3, atol=1e-3 * np.abs(ref).max())


@pytest.mark.parametrize("d,n_t,n", [(8, 7, 50_001), (2, 3, 999), (5, 2, 4096)])
def test_kmv_moments_weights_fused_equals_separate(native, d, n_t, n):
    """The fused one-read pass == moments_batched(2d) + kmv_weights(d) on the same rows (the sums are
    reassociated differently: 1e-5 relative)."""
    rng = np.random.default_rng(d + n)
    tau = np.linspace(0.2, 1.8, n_t)
    _, coef = _coef(d, tau)
    z = _t(rng.standard_normal((n_t, n, 2 * d)) * 1.3 + 0.1)
    mom, wst = native.kmv_moments_weights(d, 1.0, coef, z, n_t, n, n * 2 * d, 2 * d)
    mom_s = native.moments_batched(z, n_t, n, 2 * d, n * 2 * d, 2 * d)
    wst_s, _ = native.kmv_weights(d, 1.0, coef, z, n_t, n, n * 2 * d, 2 * d)
    for a, b in ((mom, mom_s), (wst, wst_s)):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        assert np.allclose(a, b, rtol=1e-5, atol=1e-5 * np.abs(b).max())


def test_kmv_moments_weights_set_beyond_32bit_offsets(native):
    """A set of 2^26 + 77 rows at d = 8 (4.3 GB, byte offsets past 2^32): the packed pass rebases its buffer
    descriptor per row block (the r04 single-descriptor form had to fall back to lane-private loads above
    2^24 rows) and still equals moments_batched + kmv_weights (lane-private loads) on the same rows."""
    d, n_t, n = 8, 1, (1 << 26) + 77
    _, coef = _coef(d, np.array([0.9]))
    g = torch.Generator(device=DEV)
    g.manual_seed(26)
    z = torch.randn((n, 2 * d), device=DEV, generator=g) * 1.3 + 0.1
    mom, wst = native.kmv_moments_weights(d, 1.0, coef, z, n_t, n, n * 2 * d, 2 * d)
    mom_s = native.moments_batched(z, n_t, n, 2 * d, n * 2 * d, 2 * d)
    wst_s, _ = native.kmv_weights(d, 1.0, coef, z, n_t, n, n * 2 * d, 2 * d)
    assert mom[0, 0].item() == n
    for a, b in ((mom, mom_s), (wst, wst_s)):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        assert np.allclose(a, b, rtol=1e-5, atol=1e-5 * np.abs(b).max())
    del z


@pytest.mark.parametrize("d,n_t,n,n_steps,poff", [(8, 100, 50_001, 100, 0), (8, 7, 4099, 30, 123_456_789_012),
                                                  (2, 3, 999, 2, 5), (5, 4, 4096, 3, 0)])
def test_kmv_pass_fused_with_next_mf_sums(native, d, n_t, n, n_steps, poff):
    """pdeinv_kmv_moments_weights_mf_sums (the C4 steady state: the KMV pass also sums the NEXT simulate's
    mean-path noise): mom / wst bit-identical to the plain pass (same kernel code), sums_next == mf_sums of
    the next simulate to fp32 partial-sum reassociation (1e-6 relative of the term scale), incl. more updates
    than stamps (the tail launch), particle ids past 2^32 and partial blocks."""
    rng = np.random.default_rng(d + n)
    tau = np.linspace(0.2, 1.8, n_t)
    _, coef = _coef(d, tau)
    z = _t(rng.standard_normal((n_t, n, 2 * d)) * 1.3 + 0.1)
    z0n = _t(rng.standard_normal((n, 2 * d)) + 0.25)
    A = nr.problem_constants(d)
    desc, keep = native.mf_desc(n, d, n_steps, 0.02, 1.0, A, seed=0x5EED_0004, counter_offset=777,
                                particle_offset=poff)
    mom, wst = native.kmv_moments_weights(d, 1.0, coef, z, n_t, n, n * 2 * d, 2 * d)
    mom2, wst2, sums = native.kmv_moments_weights_mf_sums(d, 1.0, coef, z, n_t, n, n * 2 * d, 2 * d, desc, z0n)
    assert torch.equal(mom, mom2) and torch.equal(wst, wst2)
    ref = native.mf_sums(desc, z0n).cpu().numpy()
    got = sums.cpu().numpy()
    assert got.shape == ref.shape
    assert got[0] == ref[0] == n
    assert np.allclose(got[1:1 + 2 * d], ref[1:1 + 2 * d], rtol=1e-6, atol=1e-6 * n)  # [x0, v0] sums
    noise_scale = np.sqrt(n)  # |sum of n normals| ~ sqrt(n): absolute tolerance on that scale
    assert np.max(np.abs(got[1 + 2 * d:] - ref[1 + 2 * d:])) < 1e-5 * noise_scale
    del keep


@pytest.mark.parametrize("d,n,n_steps,poff", [(8, 50_001, 100, 0), (8, 4099, 30, 123_456_789_012), (2, 999, 2, 5),
                                            (4, 37, 127, 0), (6, 4096, 64, 77)])
def test_simulate_mf_next_sums(native, d, n, n_steps, poff):
    """pdeinv_sde_simulate_mf_next (C4: the next simulate's mean-path noise sums drawn inside the simulator):
    the trajectory, tau and last bit-identical to the plain fused McKean-Vlasov simulate; sums_next ==
    mf_sums of the next simulate — count and z0 sums exactly (the same z0 pass), the noise sums to fp32
    partial-sum reassociation — incl. partial waves (n = 37 < 64), n_steps + 1 = 128 (three sums per lane),
    ids past 2^32."""
    rng = np.random.default_rng(d + n + n_steps)
    z0 = _t(rng.standard_normal((n, 2 * d)) + 0.25)
    A = nr.problem_constants(d)
    desc, keep = native.mf_desc(n, d, n_steps, 0.02, 1.0, A, seed=0x5EED_0004, counter_offset=777,
                                particle_offset=poff)
    xbar, _ = native.mf_mean_path(desc, native.mf_sums(desc, z0), xsum=False)
    desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
    out = [{k: torch.empty(shape, device="cuda") for k, shape in
            (("traj", (n_steps, n, 2 * d)), ("tau", (n_steps, n)), ("last", (n, 2 * d)))} for _ in range(2)]
    native.sde_simulate_desc(desc, z0, out[0]["traj"], out[0]["tau"], out[0]["last"])
    nxt, keep_n = native.mf_desc(n, d, n_steps, 0.02, 1.0, A, seed=0x5EED_0004, counter_offset=777 + n_steps + 1,
                                 particle_offset=poff)
    sums = native.sde_simulate_mf_next(desc, z0, out[1]["traj"], out[1]["tau"], out[1]["last"], nxt, z0)
    for k in ("traj", "tau", "last"):
        assert torch.equal(out[0][k], out[1][k]), k
    ref = native.mf_sums(nxt, z0).cpu().numpy()
    got = sums.cpu().numpy()
    assert got.shape == ref.shape and got[0] == ref[0] == n
    assert np.array_equal(got[1:1 + 2 * d], ref[1:1 + 2 * d])
    assert np.max(np.abs(got[1 + 2 * d:] - ref[1 + 2 * d:])) < 1e-5 * np.sqrt(n)
    assert np.abs(got[1 + 2 * d:]).max() > 0.1  # the noise sums are there
    del keep, keep_n


@pytest.mark.parametrize("d,n,n_steps,poff", [(8, 50_001, 100, 0), (8, 4099, 30, 123_456_789_012), (2, 999, 2, 5),
                                            (4, 37, 127, 0), (6, 4096, 64, 77), (8, 70_000, 1, 3)])
def test_simulate_mf_kmv_equals_separate(native, d, n, n_steps, poff):
    """pdeinv_sde_simulate_mf_kmv (C4: the KMV residual's per-stamp sums formed inside the simulator from its
    LDS-staged rows, on the matrix pipe): trajectory / tau / last bit-identical to the plain fused simulate;
    mom / wst == kmv_moments_weights over the written trajectory to fp32 reassociation (1e-5 relative, as
    test_kmv_moments_weights_fused_equals_separate); with the next simulate, sums_next as
    test_simulate_mf_next_sums. Partial waves (n = 37), rows past N inside a block (4099, 999), ids past 2^32,
    one stamp (n_steps = 1), three running noise sums per lane (n_steps + 1 = 128)."""
    rng = np.random.default_rng(d + n + n_steps + 1)
    z0 = _t(rng.standard_normal((n, 2 * d)) * 0.8 + 0.25)
    A = nr.problem_constants(d)
    desc, keep = native.mf_desc(n, d, n_steps, 0.02, 1.0, A, seed=0x5EED_0004, counter_offset=777,
                                particle_offset=poff)
    xbar, _ = native.mf_mean_path(desc, native.mf_sums(desc, z0), xsum=False)
    desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
    out = [{k: torch.empty(shape, device="cuda") for k, shape in
            (("traj", (n_steps, n, 2 * d)), ("tau", (n_steps, n)), ("last", (n, 2 * d)))} for _ in range(3)]
    native.sde_simulate_desc(desc, z0, out[0]["traj"], out[0]["tau"], out[0]["last"])
    from utils.mean_field import stamp_times
    _, coef = _coef(d, stamp_times(0x5EED_0004, 777, n_steps, 0.02).astype(np.float64) + 0.05)
    mom_s, wst_s = native.kmv_moments_weights(d, 1.0, coef, out[0]["traj"], n_steps, n, n * 2 * d, 2 * d)
    nxt, keep_n = native.mf_desc(n, d, n_steps, 0.02, 1.0, A, seed=0x5EED_0004, counter_offset=777 + n_steps + 1,
                                 particle_offset=poff)
    mom, wst = native.sde_simulate_mf_kmv(desc, z0, out[1]["traj"], out[1]["tau"], out[1]["last"], 1.0, coef)
    mom2, wst2, sums = native.sde_simulate_mf_kmv(desc, z0, out[2]["traj"], out[2]["tau"], out[2]["last"], 1.0, coef,
                                                  nxt, z0)
    for k in ("traj", "tau", "last"):
        assert torch.equal(out[0][k], out[1][k]) and torch.equal(out[0][k], out[2][k]), k
    assert torch.equal(mom, mom2) and torch.equal(wst, wst2)  # the same stamp sums with and without the next sums
    assert np.array_equal(mom[:, 0].cpu().numpy(), np.full(n_steps, float(n)))
    for a, b in ((mom, mom_s), (wst, wst_s)):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        assert np.allclose(a, b, rtol=1e-5, atol=1e-5 * np.abs(b).max())
    ref = native.mf_sums(nxt, z0).cpu().numpy()
    got = sums.cpu().numpy()
    assert got.shape == ref.shape and got[0] == ref[0] == n
    assert np.array_equal(got[1:1 + 2 * d], ref[1:1 + 2 * d])
    assert np.max(np.abs(got[1 + 2 * d:] - ref[1 + 2 * d:])) < 1e-5 * np.sqrt(n)
    # no trajectory at all: the stamp sums still come out (nothing is read back)
    last = torch.empty((n, 2 * d), device="cuda")
    mom3, wst3 = native.sde_simulate_mf_kmv(desc, z0, None, None, last, 1.0, coef)
    assert torch.equal(mom3, mom) and torch.equal(wst3, wst) and torch.equal(last, out[0]["last"])
    del keep, keep_n


def test_simulate_mf_kmv_rejects(native):
    """Odd dims and long paths with next sums are UNSUPPORTED; a next simulate that differs in more than its
    counter, a coefficient table of the wrong shape and a non-McKean-Vlasov descriptor are INVALID."""
    n, d = 1000, 8
    A = nr.problem_constants(d)
    z0 = _t(np.zeros((n, 2 * d)))
    desc, keep = native.mf_desc(n, d, 10, 0.02, 1.0, A, seed=1, counter_offset=0)
    xbar, _ = native.mf_mean_path(desc, native.mf_sums(desc, z0), xsum=False)
    desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
    last = torch.empty((n, 2 * d), device="cuda")
    _, coef = _coef(d, np.linspace(0.1, 1.0, 10))
    other, keep2 = native.mf_desc(n, d, 10, 0.02, 1.0, A, seed=2, counter_offset=11)
    with pytest.raises(ValueError):
        native.sde_simulate_mf_kmv(desc, z0, None, None, last, 1.0, coef, other, z0)
    with pytest.raises(ValueError):
        native.sde_simulate_mf_kmv(desc, z0, None, None, last, 1.0, coef[:5].contiguous())
    long_desc, keep3 = native.mf_desc(n, d, 200, 0.02, 1.0, A, seed=1, counter_offset=0)
    long_next, keep4 = native.mf_desc(n, d, 200, 0.02, 1.0, A, seed=1, counter_offset=201)
    long_desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
    _, coef200 = _coef(d, np.linspace(0.01, 2.0, 200))
    with pytest.raises(NotImplementedError):
        native.sde_simulate_mf_kmv(long_desc, z0, None, None, last, 1.0, coef200, long_next, z0)
    d3 = 3
    A3 = nr.problem_constants(d3)
    z03 = _t(np.zeros((n, 2 * d3)))
    desc3, keep5 = native.mf_desc(n, d3, 10, 0.02, 1.0, A3, seed=1, counter_offset=0)
    xbar3, _ = native.mf_mean_path(desc3, native.mf_sums(desc3, z03), xsum=False)
    desc3.d_meanfield = ctypes.c_void_p(xbar3.data_ptr())
    _, coef3 = _coef(d3, np.linspace(0.1, 1.0, 10))
    with pytest.raises(NotImplementedError):
        native.sde_simulate_mf_kmv(desc3, z03, None, None, torch.empty((n, 2 * d3), device="cuda"), 1.0, coef3)
    del keep, keep2, keep3, keep4, keep5


def test_simulate_mf_next_rejects(native):
    """The next simulate must differ in its counter only; odd dims / long paths are UNSUPPORTED (pdeinv_mf_sums)."""
    n, d = 1000, 8
    A = nr.problem_constants(d)
    z0 = _t(np.zeros((n, 2 * d)))
    desc, keep = native.mf_desc(n, d, 10, 0.02, 1.0, A, seed=1, counter_offset=0)
    xbar, _ = native.mf_mean_path(desc, native.mf_sums(desc, z0), xsum=False)
    desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
    traj, last = torch.empty((10, n, 2 * d), device="cuda"), torch.empty((n, 2 * d), device="cuda")
    other, keep2 = native.mf_desc(n, d, 10, 0.02, 1.0, A, seed=2, counter_offset=11)
    with pytest.raises(ValueError):
        native.sde_simulate_mf_next(desc, z0, traj, None, last, other, z0)
    long_desc, keep3 = native.mf_desc(n, d, 200, 0.02, 1.0, A, seed=1, counter_offset=0)
    long_next, keep4 = native.mf_desc(n, d, 200, 0.02, 1.0, A, seed=1, counter_offset=201)
    long_desc.d_meanfield = ctypes.c_void_p(xbar.data_ptr())
    with pytest.raises(NotImplementedError):
        native.sde_simulate_mf_next(long_desc, z0, torch.empty((200, n, 2 * d), device="cuda"), None, last,
                                    long_next, z0)
    del keep, keep2, keep3, keep4


@pytest.mark.parametrize("name", ["kmv_pairwise_d8.npz", "kmv_pairwise_recipe.npz"])
def test_kmv_residual_vs_pairwise_golden(native, name):
    """residual_kmv at the C4 dimension (d = 8, 2 time stamps) and on the reference's runnable recipe
    (scripts/parametric/KMV/run_quadratic_online.sh: d = 2, one stamp, 5 000 exact OU samples) against
    the literal O(n^2) pair-tensor restatement frozen in tests/golden (oracle/make_golden.py), gradient
    against its central differences. Both the separate and the fused moment passes."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name))
    x, v, tau = g["x"], g["v"], g["tau"]
    n, n_t, d = x.shape
    z = _t(np.concatenate([x, v], -1).reshape(-1, 2 * d))  # reference row order (i, t)
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    coef = _t(dlogrho_coefficients(tau, nr.ou_configuration(g["F"]), d))
    theta = _t(np.concatenate([g["K"].ravel(), g["b"]]))
    fused = native.kmv_moments_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d)
    sep = (native.moments_batched(z, n_t, n, 2 * d, 2 * d, n_t * 2 * d),
           native.kmv_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d)[0])
    for mom, wst in (fused, sep):
        out, grad = native.residual_kmv(mom, wst, theta, g["F"], 1.0)
        out = out.cpu().numpy()
        assert abs(out[0] - g["loss"]) < 1e-4 * (1 + abs(g["loss"])), (out[0], g["loss"])
        assert abs(out[1] - g["loss_gt"]) < 1e-4 * (1 + abs(g["loss_gt"]))
        assert np.allclose(grad.cpu().numpy(), g["grad"], rtol=1e-3, atol=1e-3 * (1 + np.abs(g["grad"]).max()))
