"""Generate tests/golden/*.npz from the fp64 NumPy restatement (oracle/numpy_ref.py).

Test infrastructure only. The reference (JAX) cannot run in this image and ships no golden
vectors, so these fixtures freeze the restatement's answers on fixed
seeded inputs; the restatement itself is pinned by the closed-form checks in
tests/test_oracle.py (exact EM-chain law, continuous OU moments, finite differences).

    python oracle/make_golden.py        # rewrites tests/golden/
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle import numpy_ref as nr  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
N, n, T = 64, 100, 2.0
KEEP = np.r_[0, np.arange(9, n, 10)]  # stored trajectory rows


def sde_case(name, d, gamma, grad_fn, params, seed, z0_scale=(1.0, 1.0), **extra):
    rng = np.random.default_rng(seed)
    z0 = np.concatenate([z0_scale[0] * rng.standard_normal((N, d)), z0_scale[1] * rng.standard_normal((N, d))],
                        1).astype(np.float32)
    xi = rng.standard_normal((n + 1, N, d)).astype(np.float32)
    u = rng.random(N).astype(np.float32)
    last, traj, _ = nr.sde_scan(z0, n, T / n, gamma, grad_fn, xi, u)
    _, _, tau32 = nr.sde_scan(z0, n, T / n, gamma, grad_fn, xi, u, dtype=np.float32)
    np.savez_compressed(os.path.join(OUT, f"sde_{name}.npz"), z0=z0, xi=xi, u=u, dt=T / n, gamma=gamma,
                        params=np.asarray(params, np.float64), keep=KEEP, traj=traj[KEEP], last=last, tau=tau32,
                        **extra)


def main():
    os.makedirs(OUT, exist_ok=True)
    for d in (2, 4, 8):
        F = nr.problem_constants(d)
        sde_case(f"kou_d{d}", d, 1.0, nr.grad_quadratic(F), F, 100 + d, kind="quadratic")
    for K in (3, 8):
        mus = nr.gmm_centres(4, K)
        sde_case(f"gmm_d4_k{K}", 4, 0.5, nr.grad_gmm(mus), mus, 200 + K, z0_scale=(2.0, 0.3162), kind="gmm")

    # KFP residual, quadratic model (kinetic_fokker_planck.py:33-58)
    rng = np.random.default_rng(7)
    d = 4
    F = nr.problem_constants(d)
    K = 0.3 * rng.standard_normal((d, d)); b = 0.2 * rng.standard_normal(d)
    zi, zt, z0 = (rng.standard_normal((m, 2 * d)).astype(np.float32) for m in (500, 400, 3000))
    loss, loss_gt, parts = nr.kfp_quadratic_samples(K, b, zi, zt, z0, F, 1.0, T)
    g = nr.fd_grad(lambda th: nr.kfp_quadratic_samples(th[:16].reshape(4, 4), th[16:], zi, zt, z0, F, 1.0, T)[0],
                   np.concatenate([K.ravel(), b]), eps=1e-6)
    np.savez_compressed(os.path.join(OUT, "kfp_quadratic.npz"), K=K, b=b, zi=zi, zt=zt, z0=z0, F=F, gamma=1.0, T=T,
                        loss=loss, loss_gt=loss_gt, grad=g)

    # KFP residual, GMM model
    mus_true = nr.gmm_centres(4, 3)
    mus = rng.standard_normal((3, 4))
    zi, zt, z0 = (1.5 * rng.standard_normal((m, 8)).astype(np.float32) for m in (400, 300, 2000))
    loss, loss_gt, parts = nr.kfp_gmm_loss(mus, zi, zt, z0, mus_true, 0.5, T)
    g = nr.fd_grad(lambda th: nr.kfp_gmm_loss(th, zi, zt, z0, mus_true, 0.5, T)[0], mus, eps=1e-6)
    np.savez_compressed(os.path.join(OUT, "kfp_gmm.npz"), mus=mus, mus_true=mus_true, zi=zi, zt=zt, z0=z0, gamma=0.5,
                        T=T, loss=loss, loss_gt=loss_gt, hessian=parts["hessian"], grad=g)

    # KMV residual, literal pairwise formulation (kinetic_mckean_vlasov.py:11-120)
    d, m_, nt = 2, 200, 3
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F, gamma=1.0)
    x = rng.standard_normal((m_, nt, d)); v = rng.standard_normal((m_, nt, d))
    tau = np.array([0.25, 0.8, 1.6])
    K = 0.3 * rng.standard_normal((d, d)); b = 0.2 * rng.standard_normal(d)
    loss, loss_gt = nr.kmv_pairwise_loss(K, b, x, v, tau, cfg)
    g = nr.fd_grad(lambda th: nr.kmv_pairwise_loss(th[:4].reshape(2, 2), th[4:], x, v, tau, cfg)[0],
                   np.concatenate([K.ravel(), b]), eps=1e-6)
    np.savez_compressed(os.path.join(OUT, "kmv_pairwise.npz"), K=K, b=b, x=x, v=v, tau=tau, F=F, loss=loss,
                        loss_gt=loss_gt, grad=g)

    # the same at the C4 dimension d = 8 (BASELINE config C4: kinetic McKean-Vlasov, quadratic, d = 8)
    d, m_, nt = 8, 150, 2
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F, gamma=1.0)
    x = rng.standard_normal((m_, nt, d)); v = rng.standard_normal((m_, nt, d))
    tau = np.array([0.4, 1.3])
    K = 0.2 * rng.standard_normal((d, d)); b = 0.2 * rng.standard_normal(d)
    loss, loss_gt = nr.kmv_pairwise_loss(K, b, x, v, tau, cfg)
    g = nr.fd_grad(lambda th: nr.kmv_pairwise_loss(th[:64].reshape(8, 8), th[64:], x, v, tau, cfg)[0],
                   np.concatenate([K.ravel(), b]), eps=1e-6)
    np.savez_compressed(os.path.join(OUT, "kmv_pairwise_d8.npz"), K=K, b=b, x=x, v=v, tau=tau, F=F, loss=loss,
                        loss_gt=loss_gt, grad=g)

    # the reference's runnable KMV recipe (scripts/parametric/KMV/run_quadratic_online.sh:15-19: d = 2,
    # one time stamp, 5 000 samples per stamp, T = 1, exact OU samples at a uniform time s0): there the
    # reference's [n_time, n] -> [n, n_time] reshape of d_s log rho (kinetic_mckean_vlasov.py:57-72)
    # coincides with the build's transposed pairing, so this fixture is the reference's
    # own pairing. Pair tensor of 25 M pairs, built 500 particles at a time.
    d, m_ = 2, 5000
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F, gamma=1.0)
    s0 = 0.37
    mean, P = nr.ou_mean_cov(s0, cfg)
    z = rng.multivariate_normal(mean, P, size=m_).astype(np.float32).astype(np.float64)  # stored as fp32
    x, v = z[:, None, :d], z[:, None, d:]
    tau = np.array([s0])
    K = 0.3 * rng.standard_normal((d, d)); b = 0.2 * rng.standard_normal(d)
    loss, loss_gt = nr.kmv_pairwise_loss(K, b, x, v, tau, cfg, chunk=500)
    g = nr.fd_grad(lambda th: nr.kmv_pairwise_loss(th[:4].reshape(2, 2), th[4:], x, v, tau, cfg, chunk=500)[0],
                   np.concatenate([K.ravel(), b]), eps=1e-6)
    np.savez_compressed(os.path.join(OUT, "kmv_pairwise_recipe.npz"), K=K, b=b, x=x.astype(np.float32),
                        v=v.astype(np.float32), tau=tau, F=F, loss=loss, loss_gt=loss_gt, grad=g)

    # ds log rho KAT inputs/outputs (test_partial_s_log_density.py:241-311 shape: d = 10, s = 0.1)
    d = 10
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F, gamma=1.0)
    xs = np.random.default_rng(0).uniform(size=(3, d))
    np.savez_compressed(os.path.join(OUT, "dlogrho_d10.npz"), F=F, x=xs, s=0.1,
                        ds=nr.partial_s_log_density(0.1, xs, cfg), ds2=nr.partial_s2_log_density(0.1, xs, cfg),
                        logp=nr.log_density(0.1, xs, cfg))

    dlogrho_refcfg()

    # constants recipe
    np.savez_compressed(os.path.join(OUT, "constants.npz"), **{f"tilde_F_d{d}": nr.problem_constants(d)
                                                               for d in (2, 4, 8, 10)})
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


def dlogrho_refcfg():
    """test_partial_s_log_density.py at its own configuration (:9-62: gamma = 0.1, P_x0 = 1, P_v0 = 0.1,
    m0 = 0, tilde_L = 2; :243-261: d = 10, T = 1, s = 0.1, x ~ U[0, 1) of shape [3, d]). tilde_F is the
    build's recipe (the reference's PRNGKey(2217) normals need JAX). Writes
    tests/golden/dlogrho_d10_refcfg.npz only."""
    d, gamma, P_x0, P_v0, s = 10, 0.1, 1.0, 0.1, 0.1
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F, gamma=gamma, P_x0=P_x0, P_v0=P_v0)
    xs = np.random.default_rng(10).uniform(size=(3, d))
    np.savez_compressed(os.path.join(OUT, "dlogrho_d10_refcfg.npz"), F=F, x=xs, s=s, gamma=gamma, P_x0=P_x0,
                        P_v0=P_v0, T=1.0, ds=nr.partial_s_log_density(s, xs, cfg),
                        ds2=nr.partial_s2_log_density(s, xs, cfg), logp=nr.log_density(s, xs, cfg))
    print("dlogrho_d10_refcfg.npz", os.path.getsize(os.path.join(OUT, "dlogrho_d10_refcfg.npz")))


def kmv_mlp_large():
    """General-Phi KMV (V_hypothesis interaction, the reference's default 20 x 8 net) at a size where the
    pair kernels' persistent pass-1 grid (2 048 waves over n * n_time items, mlp_pairs.hip) iterates:
    d = 2, n = 1 400 particles x 3 stamps = 4 200 items. The literal pair tensor (5.9 M pairs) is built
    250 references at a time; loss terms and the analytic gradient (kmv_mlp_pairwise_loss /
    kmv_mlp_grad_analytic, the same formulas) are sums over references, so the chunked evaluation is
    exact. Writes tests/golden/kmv_mlp_pairs_1400.npz only (its own seed; the other fixtures untouched)."""
    rng = np.random.default_rng(1400)
    d, n, nt, W, L = 2, 1400, 3, 20, 8
    F = nr.problem_constants(d)
    cfg = nr.ou_configuration(F, gamma=1.0)
    x = rng.standard_normal((n, nt, d)).astype(np.float32).astype(np.float64)
    v = rng.standard_normal((n, nt, d)).astype(np.float32).astype(np.float64)
    tau = np.array([0.3, 0.9, 1.6])
    dims = [d] + [W] * L + [1]
    flat = np.concatenate([np.concatenate([(rng.standard_normal((i, o)) / np.sqrt(i)).ravel(),
                                           0.1 * rng.standard_normal(o)]) for i, o in zip(dims[:-1], dims[1:])])
    flat = flat.astype(np.float32).astype(np.float64)
    P = nr.mlp_unflat(flat, dims)
    c = nr.kmv_value_weights(x, tau, cfg)
    CH = 250
    sg = np.zeros((n, nt, d)); sgt = np.zeros((n, nt, d)); sphi = np.zeros((n, nt)); shvv = np.zeros((n, nt))
    for a0 in range(0, n, CH):
        y = x[None] - x[a0:a0 + CH, None]                        # [a, b, T, d] = x_b - x_a
        vv = np.broadcast_to(v[None], y.shape)
        Phi, g, _, Hvv = nr.mlp_forward_terms(P, y.reshape(-1, d), vv.reshape(-1, d))
        m = y.shape[0]
        sphi += Phi.reshape(m, n, nt).sum(0); shvv += Hvv.reshape(m, n, nt).sum(0)
        sg += g.reshape(m, n, nt, d).sum(0); sgt += (y @ F.T).sum(0)
    gbar, gtrue = sg / n, sgt / n
    parts = dict(nabla=np.mean(np.sum(gbar ** 2, -1)), hessian=np.mean(shvv / n), value=np.mean(sphi / n * c),
                 nabla_true=np.mean(np.sum(gtrue ** 2, -1)))
    loss = parts["nabla"] - 2 * parts["hessian"] + 2 * parts["value"] + parts["nabla_true"]
    loss_gt = np.mean(np.sum((gtrue - gbar) ** 2, -1))
    s = 1.0 / (n * n * nt)
    grad = np.zeros_like(flat)
    for a0 in range(0, n, CH):
        y = x[None] - x[a0:a0 + CH, None]
        m = y.shape[0]
        rows = np.concatenate([y.reshape(-1, d), np.broadcast_to(v[None], y.shape).reshape(-1, d)], 1)
        C = np.zeros((rows.shape[0], 4))
        C[:, 1] = -2 * s
        C[:, 3] = (2 * s * np.broadcast_to(c[None], (m, n, nt))).reshape(-1)
        U = (2 * s * np.broadcast_to(gbar[None], y.shape)).reshape(-1, d)
        grad += nr.mlp_flat(nr.mlp_grad_rows(P, rows, C, U))
    np.savez_compressed(os.path.join(OUT, "kmv_mlp_pairs_1400.npz"), x=x.astype(np.float32), v=v.astype(np.float32),
                        tau=tau, F=F, dims=np.asarray(dims), flat=flat.astype(np.float32), loss=loss, loss_gt=loss_gt,
                        hessian=parts["hessian"], nabla=parts["nabla"], value=parts["value"], grad=grad)
    print("kmv_mlp_pairs_1400.npz", os.path.getsize(os.path.join(OUT, "kmv_mlp_pairs_1400.npz")))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "kmv_mlp_large":
        kmv_mlp_large()
    elif len(sys.argv) > 1 and sys.argv[1] == "dlogrho_refcfg":
        dlogrho_refcfg()
    else:
        main()
