"""CPU tests of the host-side mirror: config composition, PRNG keys, registry, sharding,
model init, the drift-recovery solve, and the C-ABI library's exported symbols."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_compose_defaults_and_overrides():
    from utils import config
    c = config.compose("config", [])
    assert c.pde_instance.name == "Fokker-Planck" and c.solver.name == "ConsistencyBased"
    assert c.train.optimizer.learning_rate.initial == 0.001 and c.seed == 1
    c = config.compose("config", ["pde_instance=kinetic_mckean_vlasov", "pde_instance.domain_dim=2",
                                  "train.optimizer.learning_rate.initial=1e-2", "backend.use_pmap_train=True",
                                  "solver.train.sample_mode=grid_time", "estimation_mode=parametric", "seed=2"])
    assert c.pde_instance.name == "Kinetic-McKean-Vlasov" and c.pde_instance.domain_dim == 2
    assert c.train.optimizer.learning_rate.initial == 0.01 and c.backend.use_pmap_train is True
    assert c.solver.train.sample_mode == "grid_time" and c.seed == 2
    with pytest.raises(ValueError):
        config.compose("config", ["pde_instance=nope"])


@pytest.mark.parametrize("script", ["run_KOU.sh", "run_KGMM.sh", "parametric/KMV/run_quadratic_online.sh"])
def test_reference_script_overrides_compose(script):
    """The override lists of the reference's scripts/*.sh compose unchanged."""
    from utils import config
    overrides = {
        "run_KOU.sh": ["pde_instance.domain_dim=4", "pde_instance.name=Kinetic-Fokker-Planck", "train.batch_size=250000",
                       "solver.train.sample_per_time=250", "solver.train.n_time_stamps=100",
                       "solver.train.batch_size_0T=250000", "solver.train.sample_mode=grid_time",
                       "neural_network.hidden_dim=32", "train.optimizer.learning_rate.scheduling=cosine"],
        "run_KGMM.sh": ["pde_instance.domain_dim=4", "pde_instance=kinetic_fokker_planck", "pde_instance.sample_mode=online",
                        "pde_instance.potential=GMM", "pde_instance.n_steps=200", "solver.train.batch_size_0T=2500"],
        "parametric/KMV/run_quadratic_online.sh": ["pde_instance.domain_dim=2", "pde_instance=kinetic_mckean_vlasov",
                                                   "pde_instance.potential=Quadratic", "solver.train.sample_per_time=5000",
                                                   "solver.train.n_time_stamps=1", "solver.train.batch_size_init=0"],
    }[script]
    c = config.compose("config", overrides)
    assert c.pde_instance.domain_dim in (2, 4)


def test_prng_split_is_deterministic_and_distinct():
    from utils import prng
    k = prng.PRNGKey(1)
    a, b = prng.split(k)
    assert prng.split(k) == [a, b] and a != b
    assert len({x.seed for x in prng.split(k, 64)}) == 64
    assert prng.fold_in(k, 0) != prng.fold_in(k, 1)


def test_registry():
    import registry
    from utils import config
    c = config.compose("config", ["pde_instance=kinetic_fokker_planck", "pde_instance.potential=GMM"])
    assert registry.get_pde_instance(c).__module__.endswith("_GMM")
    c = config.compose("config", [])  # the reference's default: overdamped Fokker-Planck
    assert registry.get_pde_instance(c).__name__ == "FokkerPlanck"
    c = config.compose("config", ["pde_instance.name=Heat"])
    with pytest.raises(NotImplementedError):
        registry.get_pde_instance(c)
    c = config.compose("config", ["solver=PINN"])
    with pytest.raises(NotImplementedError):
        registry.get_method(c)


@pytest.mark.parametrize("n,w", [(10, 3), (2 ** 21 * 8, 8), (5, 8), (0, 2)])
def test_shard_partitions(n, w):
    from utils import distributed as dist
    parts = [dist.shard(n, r, w) for r in range(w)]
    assert sum(p[1] for p in parts) == n
    off = 0
    for o, m in parts:
        assert o == off
        off += m


def test_drift_recovery_is_exact_on_continuous_moments():
    from methods.consistency_instances.kinetic_fokker_planck import recover_quadratic_drift
    from oracle import numpy_ref as nr
    d, T = 4, 2.0
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F)
    ts = (np.arange(2000) + 0.5) * T / 2000
    M0 = np.mean([nr.ou_mean_cov(t, cfg)[1] for t in ts], 0)

    def mom(P):
        m = P.shape[0]
        return np.concatenate([[1.0], np.zeros(m), P[np.triu_indices(m)]])
    S, b = recover_quadratic_drift(np.stack([mom(cfg["P_0"]), mom(M0), mom(nr.ou_mean_cov(T, cfg)[1])]), 1.0, T, d)
    assert np.abs(S - F).max() < 1e-5 and np.abs(b).max() < 1e-9


def test_ou_moments_batched_match_oracle():
    """The batched exact-sampler moments (one vectorised Van Loan pass) vs the oracle's
    per-time closed form of the reference's odeint ODE (…_OU.py:73-106)."""
    from example_problems.kinetic_fokker_planck_example_OU import (initialize_configuration, ou_moments_batched,
                                                                   sym_sqrt_batched)
    from oracle import numpy_ref as nr
    for d in (2, 4, 8):
        ic = initialize_configuration(d)
        cfg = nr.ou_configuration(ic["tilde_F"])
        ts = np.concatenate([[0.0, 1e-4], np.random.default_rng(d).uniform(0, 2, 50), [2.0, 5.0]])
        m, P = ou_moments_batched(ts, ic)
        for g, t in enumerate(ts):
            mr, Pr = nr.ou_mean_cov(t, cfg) if t > 0 else (cfg["m_0"], cfg["P_0"])
            assert np.abs(m[g] - mr).max() < 1e-10
            assert np.abs(P[g] - Pr).max() < 1e-9 * (1 + np.abs(Pr).max())
        C = sym_sqrt_batched(P)
        assert np.abs(C @ C - P).max() < 1e-9 * (1 + np.abs(P).max())
        assert np.allclose(C, np.transpose(C, (0, 2, 1)))


def test_ou_exact_sampler_abi_validation_and_van_loan_scaling():
    """pdeinv_ou_exact_sample rejects a null descriptor, an unsupported dimension, a bad Taylor degree and
    t_min > t_max before any HIP call; the host's per-problem constants keep |B|_1 t_max / 2^s <= 1 (the scaled
    Taylor sum's truncation bound) and B^0 = I."""
    import ctypes
    from example_problems.kinetic_fokker_planck_example_OU import initialize_configuration, van_loan_powers
    from utils import native
    L = native.lib()
    assert ctypes.sizeof(native.OuDesc) == 56
    call = lambda d: L.pdeinv_ou_exact_sample(d, 1, 1, 1, 0, 0, 0, None, None, None, None, None, None)
    assert call(None) == native.PDEINV_ERR_INVALID
    for kw, err in (({"n": 3}, native.PDEINV_ERR_UNSUPPORTED), ({"n": 34}, native.PDEINV_ERR_UNSUPPORTED),
                    ({"taylor_degree": 0}, native.PDEINV_ERR_INVALID), ({"t_min": 2.0, "t_max": 1.0}, native.PDEINV_ERR_INVALID),
                    ({}, native.PDEINV_ERR_INVALID)):  # ({}: valid shape, null device pointers)
        d = native.OuDesc(8, 18, 3, 1e-4, 2.0, None, None, None)
        for k, v in kw.items():
            setattr(d, k, v)
        assert call(ctypes.byref(d)) == err, (kw, L.pdeinv_last_error())
    for dim in (1, 4, 16):
        ic = initialize_configuration(dim)
        pw, s = van_loan_powers(ic, 2.0)
        n2 = 4 * dim
        assert pw.shape == (19, n2, n2) and np.array_equal(pw[0], np.eye(n2))
        assert np.abs(pw[1]).sum(axis=0).max() * 2.0 / 2.0 ** s <= 1.0


def test_adam_matches_optax_semantics():
    import torch
    from core.trainer import Adam, cosine_decay_schedule
    opt = Adam(0.1, weight_decay=0.01, eps=1e-4)
    p = {"w": torch.tensor([1.0, -2.0])}
    st = opt.init(p)
    g = {"w": torch.tensor([0.5, 0.25])}
    p1, st = opt.update(g, st, p)
    gw = np.array([0.5, 0.25]) + 0.01 * np.array([1.0, -2.0])
    m, v = 0.1 * gw, 0.001 * gw ** 2
    want = np.array([1.0, -2.0]) - 0.1 * (m / 0.1) / (np.sqrt(v / 0.001) + 1e-4)
    assert np.allclose(p1["w"].numpy(), want, rtol=1e-6)
    f = cosine_decay_schedule(1.0, 20000, 1e-3)
    assert f(0) == 1.0 and abs(f(20000) - 1e-3) < 1e-12 and abs(f(10000) - (0.5 * 0.999 + 1e-3)) < 1e-9


def test_trainer_ema_matches_optax_restatement():
    """core/trainer.py:87-103 (use_ema) across a lowered switch epoch, against an fp64 restatement of
    optax.adam + optax.ema(0.999): at the switch epoch EmaState(count=0, ema=params) is taken from the
    params before that step's update; every later step sets ema <- 0.999 ema + 0.001 params and the
    params become the raw ema (no debias division). The parameters must stay O(1)."""
    import torch
    from core.trainer import Adam, JaxTrainer
    from utils import config, prng

    cfg = config.compose("config", ["train.optimizer.use_ema=True", "test.frequency=1000"])
    c = np.array([0.7, -1.3, 2.1])

    class Quadratic:  # loss 0.5 |p - c|^2, grad p - c
        def value_and_grad_fn(self, forward_fn, params, rng):
            p = params["w"]
            g = p - torch.as_tensor(c, dtype=p.dtype)
            return {"loss": 0.5 * (g * g).sum(), "grad": {"w": g}, "grad_norm": g.norm(),
                    "loss ground truth": 0.5 * (g * g).sum()}

        def test_fn(self, forward_fn, params, rng):
            return {}

    start, iters, lr, wd = 3, 9, 0.1, 0.0
    tr = JaxTrainer(cfg, Quadratic(), prng.PRNGKey(0), Adam(lr, weight_decay=wd), None,
                    {"w": torch.zeros(3, dtype=torch.float64)})
    tr.ema_start = start
    out = tr.fit(number_of_iterations=iters)["w"].numpy()

    p, mu, nu, ema = np.zeros(3), np.zeros(3), np.zeros(3), None
    for k in range(iters):
        g = p - c
        if k == start:
            ema = p.copy()
        mu, nu = 0.9 * mu + 0.1 * g, 0.999 * nu + 0.001 * g * g
        p = p - lr * (mu / (1 - 0.9 ** (k + 1))) / (np.sqrt(nu / (1 - 0.999 ** (k + 1))) + 1e-4)
        if ema is not None:
            ema = 0.999 * ema + 0.001 * p
            p = ema.copy()
    assert np.abs(out - p).max() < 1e-12, (out, p)
    assert np.abs(out).max() < 1.0  # O(1): the old debiased branch blew the params up ~1000x


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "pdeinv.h")).read()
    return set(re.findall(r"^(?:int|int64_t|size_t|const char\*)\s+(pdeinv_\w+)\(", txt, flags=re.M))


def test_header_and_binding_agree():
    from utils import native
    assert _header_functions() == set(native.EXPORTED_SYMBOLS)


def test_library_exports_every_header_symbol():
    """The C-ABI shared library loads without a GPU and exports everything include/pdeinv.h declares."""
    from utils import native
    if not os.path.exists(native.LIB_PATH):
        native.build()
    lib = ctypes.CDLL(native.LIB_PATH)
    missing = [s for s in _header_functions() if not hasattr(lib, s)]
    assert not missing
    lib.pdeinv_moment_len.restype = ctypes.c_int
    assert lib.pdeinv_moment_len(8) == 45 and lib.pdeinv_abi_version() == native.ABI_VERSION == 10


def test_loader_fails_loudly_without_gpu():
    import torch
    from utils import native
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    with pytest.raises(RuntimeError):
        native.sde_simulate(torch.zeros((4, 4)), 3, 0.1, 1.0, dict(kind=0, params=np.eye(2)), seed=1)


def test_abi_argument_validation_without_gpu():
    """The C ABI rejects bad descriptors before touching the HIP runtime (negative
    status + thread-local pdeinv_last_error()), so these run on a GPU-less host: a null descriptor,
    an unsupported dim, n_steps = 0, a non-finite dt, ld_z0 < 2d, a null RealNVP descriptor."""
    import ctypes
    from utils import native
    L = native.lib()

    def sde(**kw):
        d = native.SdeDesc()
        d.n_particles, d.dim, d.n_steps, d.dt, d.gamma, d.noise_scale = 16, 4, 10, 0.02, 1.0, 1.41
        for k, v in kw.items():
            setattr(d, k, v)
        return L.pdeinv_sde_simulate(ctypes.byref(d), None, None, None, None, None, None, None)

    assert L.pdeinv_sde_simulate(None, None, None, None, None, None, None, None) == native.PDEINV_ERR_INVALID
    assert b"null descriptor" in L.pdeinv_last_error()
    assert sde(dim=0) == native.PDEINV_ERR_UNSUPPORTED and b"dim" in L.pdeinv_last_error()
    assert sde(dim=17) == native.PDEINV_ERR_UNSUPPORTED
    assert sde(n_steps=0) == native.PDEINV_ERR_INVALID and b"n_steps" in L.pdeinv_last_error()
    assert sde(dt=float("nan")) == native.PDEINV_ERR_INVALID
    assert sde(n_particles=-1) == native.PDEINV_ERR_INVALID
    assert sde(ld_z0=5) == native.PDEINV_ERR_INVALID and b"ld_z0" in L.pdeinv_last_error()
    assert L.pdeinv_realnvp_value_and_grad(None, None, None, 0, None, 0, 0, None, None, None, 0, None) \
        == native.PDEINV_ERR_INVALID
    # the query reports the AUTO path: compiled shapes and the zero-padded envelope (d = 3 -> 4, width 20 -> 32);
    # width > 1024 is rejected under AUTO (only the explicit LIBRARY cross-check reaches rocBLAS)
    assert L.pdeinv_mlp_fused_supported(3, 2, 256, 40) == 1 and L.pdeinv_mlp_fused_supported(8, 2, 256, 40) == 1
    assert L.pdeinv_mlp_fused_supported(8, 1, 256, 40) == 1 and L.pdeinv_mlp_fused_supported(8, 2, 256, 80) == 1
    assert L.pdeinv_mlp_fused_supported(2, 8, 20, 40) == 1 and L.pdeinv_mlp_fused_supported(8, 2, 1024, 40) == 1
    assert L.pdeinv_mlp_fused_supported(8, 2, 1025, 40) == 0 and L.pdeinv_mlp_fused_supported(12, 2, 1000, 40) == 1
    assert L.pdeinv_mlp_fused_supported(17, 2, 256, 40) == 0
    assert native.kmv_mlp_path([2] + [20] * 8 + [40]) == "pair_tiles_mfma"
    assert native.kmv_mlp_path([2, 24, 24, 40]) == "pair_ring"
    assert native.kmv_mlp_path([2, 64, 64, 40]) == "fused_rows_mfma"
    assert native.kmv_mlp_path([2, 64, 64, 40], native.MLP_IMPL_LIBRARY) == "library_rocblas"
    # LIBRARY only where the rocBLAS path runs (dim <= 8); AUTO never resolves to it
    with pytest.raises(NotImplementedError):
        native.kmv_mlp_path([12, 64, 64, 40], native.MLP_IMPL_LIBRARY)
    with pytest.raises(NotImplementedError):
        native.kmv_mlp_path([4, 2048, 2048, 40])
    with pytest.raises(NotImplementedError):
        native.kmv_mlp_path([17, 64, 64, 40])
    for dims in ([2] + [20] * 8 + [40], [2, 24, 24, 40], [2, 64, 64, 40], [12, 1000, 1000, 40], [16, 1024, 40]):
        assert native.kmv_mlp_path(dims) != "library_rocblas"
    # impl is validated (PDEINV_MLP_IMPL_PAIRS_RING selects the register-ring pair kernels, kmv_mlp only)
    F = (ctypes.c_float * 4)(1, 0, 0, 1)
    km = native.KmvMlpDesc()
    km.dim, km.n_layers, km.width, km.out_features, km.n_sets, km.n_rows, km.gamma = 2, 8, 20, 40, 1, 64, 1.0
    km.tilde_F = ctypes.cast(F, ctypes.c_void_p)
    dummy = ctypes.c_void_p(16)
    call = lambda: L.pdeinv_residual_kmv_mlp(ctypes.byref(km), dummy, 0, 4, dummy, dummy, dummy, dummy, dummy, None)
    km.impl = 7
    assert call() == native.PDEINV_ERR_INVALID and b"impl" in L.pdeinv_last_error()
    km.impl, km.width = native.MLP_IMPL_PAIRS_RING, 64
    assert call() == native.PDEINV_ERR_UNSUPPORTED and b"PAIRS_RING" in L.pdeinv_last_error()
    fm = native.KfpMlpDesc()
    fm.dim, fm.n_layers, fm.width, fm.out_features, fm.impl = 4, 2, 256, 40, native.MLP_IMPL_PAIRS_RING
    assert L.pdeinv_residual_kfp_mlp(ctypes.byref(fm), None, 0, 0, None, 0, 0, None, 0, 0, None, None, None, None,
                                     None) == native.PDEINV_ERR_INVALID
    # AUTO past the hand-written envelope is UNSUPPORTED before any HIP call (no rocBLAS fallback)
    Fq = (ctypes.c_float * 16)(*np.eye(4, dtype=np.float32).ravel())
    fm.width, fm.impl, fm.true_kind, fm.true_params = 2048, native.MLP_IMPL_AUTO, native.POT_QUADRATIC, \
        ctypes.cast(Fq, ctypes.c_void_p)
    assert L.pdeinv_residual_kfp_mlp(ctypes.byref(fm), dummy, 64, 8, dummy, 64, 8, dummy, 64, 8, dummy, dummy, dummy,
                                     dummy, None) == native.PDEINV_ERR_UNSUPPORTED
    assert b"LIBRARY" in L.pdeinv_last_error()
    km.impl, km.width, km.n_layers = native.MLP_IMPL_AUTO, 2048, 2
    assert call() == native.PDEINV_ERR_UNSUPPORTED and b"LIBRARY" in L.pdeinv_last_error()


def test_bench_refuses_mismatched_world_size():
    """bench.py exits non-zero, printing no line, when torch.distributed.run's WORLD_SIZE disagrees with
    --gpus (checked before any GPU call, so it runs here), and rejects --gpus 0."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    for argv in (["--gpus", "1"], ["--gpus", "0"]):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv + ["--steps", "1", "--warmup", "0"],
                           env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode != 0 and "{" not in r.stdout, (r.stdout, r.stderr[-2000:])


def test_oracle_under_asan():
    """the host AddressSanitizer + UBSan build of the C oracle (oracle/Makefile `asan`,
    oracle/asan_driver.c) runs every oracle entry point on ragged inputs and the Philox KATs clean."""
    import shutil
    import subprocess
    if shutil.which(os.environ.get("CC", "gcc")) is None:
        pytest.skip("no host C compiler")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    r = subprocess.run([os.path.join(ROOT, "oracle", "_build", "oracle_asan")], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failed checks" in r.stdout
