"""NumPy restatement of the reference hot path — CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker / CPU baseline. The product package (pde-inverse-problem_amd/) never does.

Parity status: the reference is JAX, which is absent from this image, so no
reference output can be produced here and the reference ships no golden vectors
(SURVEY.md §4). This restatement is pinned instead by closed-form known answers:
  * the exact law of the semi-implicit Euler–Maruyama chain (em_chain_moments), which the
    sample-path restatement must reproduce — an identity, not a tolerance fit;
  * the continuous OU moments (ou_mean_cov), i.e. the reference's own odeint solution
    (…_OU.py:73-106) in closed form, to which the chain converges at O(dt);
  * the finite-difference checks of the reference's only test script
    (test_partial_s_log_density.py:241-311), here asserted;
  * the loss == "loss ground truth" identity in expectation (kinetic_fokker_planck.py:33-58).
Bit-level parity with JAX's threefry streams is "parity unpinned".

Functions cite the reference file:line they follow (paths relative to the reference root).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.linalg import expm

SQRT2 = math.sqrt(2.0)


# --------------------------------------------------------------------------------------
# simulator: utils/sampling_utils.py:6-52
# --------------------------------------------------------------------------------------
def grad_quadratic(A, c=None):
    """grad U(q) = A (q - c) — V_true_fn of …_OU.py:130-138 is 0.5 x^T tilde_F x."""
    A = np.asarray(A)

    def g(q):
        y = q if c is None else q - c
        return y @ A.T

    return g


def gmm_value_grad(x, mus, sigma=1.0):
    """core/potential.py:32-37: V = -logsumexp_k(-|x-mu_k|^2/(2 sigma^2)), grad = sum_k w_k (x-mu_k)/sigma^2."""
    x = np.asarray(x)
    diff = x[..., None, :] - mus  # [..., K, d]
    a = -np.sum(diff * diff, axis=-1) / (2.0 * sigma * sigma)
    amax = np.max(a, axis=-1, keepdims=True)
    e = np.exp(a - amax)
    den = np.sum(e, axis=-1, keepdims=True)
    w = e / den
    value = -(amax[..., 0] + np.log(den[..., 0]))
    grad = np.sum(w[..., None] * diff, axis=-2) / (sigma * sigma)
    return value, grad


def grad_gmm(mus, sigma=1.0):
    mus = np.asarray(mus)
    return lambda q: gmm_value_grad(q, mus, sigma)[1]


def update_step(q, p, h, grad_fn, gamma, xi, noise_scale=SQRT2):
    """utils/sampling_utils.py:6-22 (h may be per-particle [N,1])."""
    g = grad_fn(q)
    noise = noise_scale * xi
    p_new = p - h * g + np.sqrt(h) * noise - gamma * p * h
    q_new = q + h * p_new
    return q_new, p_new


def sde_scan(z0, n_steps, dt, gamma, grad_fn, xi, u, noise_scale=SQRT2, dtype=np.float64,
             random_shift=True):
    """utils/sampling_utils.py:25-52 for all particles at once, with explicit noise.

    z0 [N, 2d]; xi [n_steps+1, N, d] standard normals (update s uses xi[s]); u [N] in [0,1).
    Returns (last [N,2d], traj [n_steps, N, 2d] time-major, tau [n_steps, N]).
    """
    z0 = np.asarray(z0, dtype=dtype)
    N, m = z0.shape
    d = m // 2
    dt = dtype(dt)
    gamma = dtype(gamma)
    ns = dtype(noise_scale)
    q, p = z0[:, :d].copy(), z0[:, d:].copy()
    tau0 = (np.asarray(u, dtype=dtype) * dt) if random_shift else np.zeros(N, dtype=dtype)
    traj = np.empty((n_steps, N, m), dtype=dtype)
    for s in range(n_steps + 1):
        if s == 0:
            h = tau0[:, None]
        elif s == n_steps:
            h = (dt - tau0)[:, None]
        else:
            h = dt
        q, p = update_step(q, p, h, grad_fn, gamma, np.asarray(xi[s], dtype=dtype), ns)
        if s < n_steps:
            traj[s, :, :d] = q
            traj[s, :, d:] = p
    last = np.concatenate([q, p], axis=1)
    tau = (tau0[None, :] + (np.arange(n_steps, dtype=dtype) * dt)[:, None]).astype(dtype)
    return last, traj, tau


# --------------------------------------------------------------------------------------
# KOU problem constants and analytic moments: example_problems/kinetic_fokker_planck_example_OU.py
# --------------------------------------------------------------------------------------
def ou_configuration(tilde_F, gamma=1.0, P_x0=1.0, P_v0=1.0, L_scale=2.0):
    """…_OU.py:15-70: F = [[0, I], [-tilde_F, -gamma I]], L = diag(0, L_scale I), m0 = 0."""
    tilde_F = np.asarray(tilde_F, dtype=np.float64)
    d = tilde_F.shape[0]
    I = np.eye(d)
    Z = np.zeros((d, d))
    F = np.block([[Z, I], [-tilde_F, -gamma * I]])
    L = np.block([[Z, Z], [Z, L_scale * I]])
    m0 = np.zeros(2 * d)
    P0 = np.block([[P_x0 * I, Z], [Z, P_v0 * I]])
    return dict(gamma_friction=gamma, tilde_F=tilde_F, F=F, L=L, m_0=m0, P_0=P0,
                m_x_0=np.zeros(d), P_x_0=P_x0 * I)


def ou_mean_cov(t, cfg):
    """Closed form of OU_process (…_OU.py:73-93): m' = F m, P' = F P + P F^T + L.

    m(t) = e^{Ft} m0; P(t) = e^{Ft} P0 e^{F^T t} + int_0^t e^{Fs} L e^{F^T s} ds, the integral by
    Van Loan's block exponential (exact to rounding, where the reference uses dopri5 odeint).
    """
    F, L, m0, P0 = cfg["F"], cfg["L"], cfg["m_0"], cfg["P_0"]
    n = F.shape[0]
    E = expm(F * t)
    blk = np.zeros((2 * n, 2 * n))
    blk[:n, :n] = -F
    blk[:n, n:] = L
    blk[n:, n:] = F.T
    V = expm(blk * t)
    Q = V[n:, n:].T @ V[:n, n:]
    m = E @ m0
    P = E @ P0 @ E.T + Q
    return m, 0.5 * (P + P.T)


def em_step_matrices(tilde_F, gamma, h, noise_scale=SQRT2):
    """Exact law of one semi-implicit update with grad U = tilde_F q (sampling_utils.py:17-20):
    z' = A(h) z + B(h) xi, A = [[I - h^2 F~, h(1-gamma h) I], [-h F~, (1-gamma h) I]], B = sqrt(h) ns [h I; I]."""
    d = tilde_F.shape[0]
    I = np.eye(d)
    A = np.block([[I - h * h * tilde_F, h * (1 - gamma * h) * I], [-h * tilde_F, (1 - gamma * h) * I]])
    B = math.sqrt(h) * noise_scale * np.vstack([h * I, I])
    return A, B


def em_chain_moments(tilde_F, gamma, dt, n_steps, m0, P0, noise_scale=SQRT2, random_shift=True,
                     n_gl=8):
    """Exact mean / second moment of every traj row and of `last` for the chain restated by
    sde_scan with grad U = tilde_F q, averaged over tau0 = u dt, u ~ U(0,1).

    Entries are polynomials in tau0 of degree <= 8, so n_gl >= 5 Gauss–Legendre nodes are exact.
    Returns (mean_traj [n,2d], second_traj [n,2d,2d], mean_last [2d], second_last [2d,2d]).
    """
    tilde_F = np.asarray(tilde_F, dtype=np.float64)
    m = 2 * tilde_F.shape[0]
    nodes, weights = np.polynomial.legendre.leggauss(n_gl)
    us = 0.5 * (nodes + 1.0) if random_shift else np.array([0.0])
    ws = 0.5 * weights if random_shift else np.array([1.0])
    A_dt, B_dt = em_step_matrices(tilde_F, gamma, dt, noise_scale)
    mean_tr = np.zeros((n_steps, m))
    sec_tr = np.zeros((n_steps, m, m))
    mean_last = np.zeros(m)
    sec_last = np.zeros((m, m))
    for u, w in zip(us, ws):
        t0 = u * dt
        A0, B0 = em_step_matrices(tilde_F, gamma, t0, noise_scale)
        mu = A0 @ m0
        P = A0 @ P0 @ A0.T + B0 @ B0.T
        for s in range(n_steps):
            if s > 0:
                mu = A_dt @ mu
                P = A_dt @ P @ A_dt.T + B_dt @ B_dt.T
            mean_tr[s] += w * mu
            sec_tr[s] += w * (P + np.outer(mu, mu))
        A1, B1 = em_step_matrices(tilde_F, gamma, dt - t0, noise_scale)
        mu_l = A1 @ mu
        P_l = A1 @ P @ A1.T + B1 @ B1.T
        mean_last += w * mu_l
        sec_last += w * (P_l + np.outer(mu_l, mu_l))
    return mean_tr, sec_tr, mean_last, sec_last


def mf_mean_path(sums, d, n_steps, dt, tau0, gamma, noise_scale=SQRT2):
    """Closed-form mean path of the interacting (McKean–Vlasov) ensemble — the restatement behind
    utils/mean_field.py's fused driver (sde.hip mf_path_kernel). The quadratic interaction's drift
    A (x_i - xbar) (kinetic_mckean_vlasov.py:20-23 for Phi* = x^T A x / 2) averages to zero over the
    ensemble, so the update of sampling_utils.py:17,20 averaged over particles is
        vbar' = (1 - gamma h) vbar + sqrt(h) ns xibar_s ,  xbar' = xbar + h vbar'.
    sums = [count, sum x0 (d), sum v0 (d), sum_i xi_{i,s} (d) for s = 0..n]. Returns xbar [n+2, d]:
    row s is the mean before update s (row n+1: after the last update). h_s = tau0, dt, ..., dt - tau0
    (the particles' fp32 step sizes)."""
    sums = np.asarray(sums, np.float64)
    cnt = sums[0]
    inv = 1.0 / cnt if cnt > 0 else 0.0
    xb, vb = sums[1:1 + d] * inv, sums[1 + d:1 + 2 * d] * inv
    xi = sums[1 + 2 * d:].reshape(n_steps + 1, d) * inv
    out = np.zeros((n_steps + 2, d))
    dt32, t032 = np.float32(dt), np.float32(tau0)
    for s in range(n_steps + 1):
        out[s] = xb
        h = t032 if s == 0 else (dt32 - t032 if s == n_steps else dt32)
        sh = float(np.sqrt(np.float32(h)) * np.float32(noise_scale))
        vb = vb - gamma * float(h) * vb + sh * xi[s]
        xb = xb + float(h) * vb
    out[n_steps + 1] = xb
    return out


# --------------------------------------------------------------------------------------
# moments layout of include/pdeinv.h
# --------------------------------------------------------------------------------------
def moments(z):
    """[count, sum z, sum z_i z_j (i<=j)] in fp64."""
    z = np.asarray(z, dtype=np.float64).reshape(-1, np.shape(z)[-1])
    m = z.shape[1]
    iu = np.triu_indices(m)
    S2 = z.T @ z
    return np.concatenate([[z.shape[0]], z.sum(0), S2[iu]])


def unpack_moments(vec, m):
    vec = np.asarray(vec, dtype=np.float64)
    n = vec[0]
    mean = vec[1:1 + m] / n
    S = np.zeros((m, m))
    iu = np.triu_indices(m)
    S[iu] = vec[1 + m:]
    S = S + S.T - np.diag(np.diag(S))
    return n, mean, S / n


# --------------------------------------------------------------------------------------
# KFP residual: methods/consistency_instances/kinetic_fokker_planck.py:11-69
# --------------------------------------------------------------------------------------
def kfp_quadratic_samples(K, b, z_init, z_term, z_0T, tilde_F, gamma, T):
    """Per-sample fp64 restatement of loss_fn (:33-50) and loss_ground_truth_fn (:52-58) for
    V_theta(x) = x . (x K + b) (…_OU.py:209-220): grad V = (K+K^T) x + b, Hessian K+K^T."""
    K = np.asarray(K, np.float64); b = np.asarray(b, np.float64)
    S = K + K.T
    d = K.shape[0]

    def split(z):
        z = np.asarray(z, np.float64)
        return z[:, :d], z[:, d:]

    xi, vi = split(z_init); xt, vt = split(z_term); x0, v0 = split(z_0T)
    gV = lambda x: x @ S.T + b
    gT = lambda x: x @ np.asarray(tilde_F, np.float64).T
    parts = dict(
        initial=np.mean(np.sum(gV(xi) * vi, -1)) if len(xi) else 0.0,
        terminal=np.mean(np.sum(gV(xt) * vt, -1)) if len(xt) else 0.0,
        nabla=np.mean(np.sum(gV(x0) ** 2, -1)),
        hessian=np.mean(np.einsum("ni,ij,nj->n", v0, S, v0)),
        friction=np.mean(np.sum(gV(x0) * v0, -1)) * gamma,
        nabla_true=np.mean(np.sum(gT(x0) ** 2, -1)),
    )
    loss = (parts["nabla"] - 2 * parts["hessian"] + 2 * parts["friction"] + parts["nabla_true"]
            + (-2 * parts["initial"] + 2 * parts["terminal"]) / T)
    loss_gt = np.mean(np.sum((gT(x0) - gV(x0)) ** 2, -1))
    return loss, loss_gt, parts


def kfp_quadratic_from_moments(K, b, mom_init, mom_0T, mom_term, tilde_F, gamma, T):
    """The same loss and its exact gradient d/d(K,b) from the three moment sets."""
    K = np.asarray(K, np.float64); b = np.asarray(b, np.float64)
    F = np.asarray(tilde_F, np.float64)
    d = K.shape[0]
    S = K + K.T

    def blocks(mom):
        n, mean, M = unpack_moments(mom, 2 * d)
        return mean[:d], mean[d:], M[:d, :d], M[:d, d:], M[d:, d:]

    ex, ev, Mxx, Mxv, Mvv = blocks(mom_0T)
    _, evi, _, Mxvi, _ = blocks(mom_init)
    _, evt, _, Mxvt, _ = blocks(mom_term)
    nabla = np.trace(S @ Mxx @ S) + 2 * b @ S @ ex + b @ b
    hess = np.trace(S @ Mvv)
    fric_raw = np.trace(S @ Mxv) + b @ ev
    init = np.trace(S @ Mxvi) + b @ evi
    term = np.trace(S @ Mxvt) + b @ evt
    true = np.trace(F @ Mxx @ F.T)
    loss = nabla - 2 * hess + 2 * gamma * fric_raw + true + (-2 * init + 2 * term) / T
    D = F - S
    loss_gt = np.trace(D @ Mxx @ D.T) - 2 * b @ D @ ex + b @ b
    G = (S @ Mxx + Mxx @ S + 2 * np.outer(b, ex)) - 2 * Mvv + 2 * gamma * Mxv.T \
        + (-2 * Mxvi.T + 2 * Mxvt.T) / T
    gK = G + G.T
    gb = (2 * S @ ex + 2 * b) + 2 * gamma * ev + (-2 * evi + 2 * evt) / T
    parts = dict(nabla=nabla, hessian=hess, friction=gamma * fric_raw, nabla_true=true,
                 initial=init, terminal=term)
    return loss, loss_gt, gK, gb, parts


# --------------------------------------------------------------------------------------
# KFP residual with the parametric GMM model (…_GMM.py:214-234)
# --------------------------------------------------------------------------------------
def gmm_terms(x, v, mus, sigma=1.0):
    """Per-sample grad V, v^T Hess V v for V = -logsumexp (analytic: H = I/s^2 - Cov_w(mu)/s^4)."""
    x = np.asarray(x, np.float64); v = np.asarray(v, np.float64)
    diff = x[:, None, :] - mus[None]
    a = -np.sum(diff ** 2, -1) / (2 * sigma ** 2)
    a -= a.max(-1, keepdims=True)
    w = np.exp(a); w /= w.sum(-1, keepdims=True)
    s2 = 1.0 / sigma ** 2
    mbar = w @ mus
    g = s2 * (x - mbar)
    pk = v @ mus.T
    pbar = np.sum(w * pk, -1)
    vHv = s2 * np.sum(v * v, -1) - s2 * s2 * (np.sum(w * pk * pk, -1) - pbar ** 2)
    return g, vHv


def kfp_gmm_loss(mus, z_init, z_term, z_0T, mus_true, gamma, T, sigma=1.0, sigma_true=1.0):
    """loss_fn (:33-50) / loss_ground_truth_fn (:52-58) with V_theta = GMM(mus), V* = GMM(mus_true)."""
    mus = np.asarray(mus, np.float64)
    d = mus.shape[1]
    z_init = np.asarray(z_init, np.float64); z_term = np.asarray(z_term, np.float64)
    z_0T = np.asarray(z_0T, np.float64)
    x0, v0 = z_0T[:, :d], z_0T[:, d:]
    g0, h0 = gmm_terms(x0, v0, mus, sigma)
    gt = gmm_value_grad(x0, np.asarray(mus_true, np.float64), sigma_true)[1]
    parts = dict(nabla=np.mean(np.sum(g0 ** 2, -1)), hessian=np.mean(h0),
                 friction=gamma * np.mean(np.sum(g0 * v0, -1)),
                 nabla_true=np.mean(np.sum(gt ** 2, -1)))
    for name, z in (("initial", z_init), ("terminal", z_term)):
        if len(z):
            gz, _ = gmm_terms(z[:, :d], z[:, d:], mus, sigma)
            parts[name] = np.mean(np.sum(gz * z[:, d:], -1))
        else:
            parts[name] = 0.0
    loss = (parts["nabla"] - 2 * parts["hessian"] + 2 * parts["friction"] + parts["nabla_true"]
            + (-2 * parts["initial"] + 2 * parts["terminal"]) / T)
    loss_gt = np.mean(np.sum((gt - g0) ** 2, -1))
    return loss, loss_gt, parts


def fd_grad(fn, theta, eps=1e-5):
    """Central finite differences in fp64 (replaces jax.value_and_grad as the checker)."""
    theta = np.asarray(theta, np.float64)
    g = np.zeros_like(theta)
    it = np.nditer(theta, flags=["multi_index"])
    for _ in it:
        idx = it.multi_index
        tp = theta.copy(); tp[idx] += eps
        tm = theta.copy(); tm[idx] -= eps
        g[idx] = (fn(tp) - fn(tm)) / (2 * eps)
    return g


# --------------------------------------------------------------------------------------
# score / log-density terms: kinetic_mckean_vlasov_example_quadratic.py:18-191,
# test_partial_s_log_density.py:142-164
# --------------------------------------------------------------------------------------
def _xmarginal(s, cfg):
    d = cfg["tilde_F"].shape[0]
    mean, cov = ou_mean_cov(s, cfg)
    F, L = cfg["F"], cfg["L"]
    dm = F @ mean
    d2m = F @ dm
    dP = F @ cov + cov @ F.T + L
    d2P = F @ dP + dP @ F.T
    return (mean[:d], cov[:d, :d], dm[:d], d2m[:d], dP[:d, :d], d2P[:d, :d])


def log_density(s, x, cfg):
    """test_partial_s_log_density.py:142-153: log N(x; m_1(s), P_11(s))."""
    m1, P11, *_ = _xmarginal(s, cfg)
    Pinv = np.linalg.inv(P11)
    r = m1 - np.asarray(x, np.float64)
    quad = np.einsum("...i,ij,...j->...", r, Pinv, r)
    return -0.5 * quad - 0.5 * np.log(np.linalg.det(2 * np.pi * P11))


def partial_s_log_density(s, x, cfg):
    """kinetic_mckean_vlasov_example_quadratic.py:51-69."""
    m1, P11, dm1, _, dP11, _ = _xmarginal(s, cfg)
    Pinv = np.linalg.inv(P11)
    dPinv = -Pinv @ dP11 @ Pinv
    r = m1 - np.asarray(x, np.float64)
    term1 = -np.einsum("i,ij,...j->...", dm1, Pinv, r)
    term2 = -0.5 * np.trace(dP11 @ Pinv)
    term3 = -0.5 * np.einsum("...i,ij,...j->...", r, dPinv, r)
    return term1 + term2 + term3


def partial_s2_log_density(s, x, cfg):
    """kinetic_mckean_vlasov_example_quadratic.py:120-177."""
    m1, P11, dm1, d2m1, dP11, d2P11 = _xmarginal(s, cfg)
    Pinv = np.linalg.inv(P11)
    dPinv = -Pinv @ dP11 @ Pinv
    d2Pinv = -Pinv @ d2P11 @ Pinv + 2 * Pinv @ dP11 @ Pinv @ dP11 @ Pinv
    x = np.asarray(x, np.float64)
    r = m1 - x
    term1 = (-np.einsum("i,ij,...j->...", d2m1, Pinv, r) - np.einsum("i,ij,...j->...", dm1, dPinv, r)
             - dm1 @ Pinv @ dm1)
    term2 = -0.5 * np.einsum("...i,ij,...j->...", -r, d2Pinv, -r) - np.einsum("...i,ij,j->...", r, dPinv, dm1)
    term3 = 0.5 * np.trace(Pinv @ dP11 @ Pinv @ dP11) - 0.5 * np.trace(Pinv @ d2P11)
    return term1 + term2 + term3


# --------------------------------------------------------------------------------------
# KMV residual: methods/consistency_instances/kinetic_mckean_vlasov.py:11-120 (pairwise, O(n^2))
# --------------------------------------------------------------------------------------
def kmv_pairwise_loss(K, b, x, v, tau, cfg, chunk=None):
    """Literal restatement with the [m, n, n_time, d] pairwise tensor (:20-23, :74-97), for
    Phi_theta(y) = y . (y K + b) (…_quadratic.py:205-216), Phi* = 0.5 y^T tilde_F y (:193-203).
    x, v: [n, n_time, d]; tau [n_time]. `chunk` bounds memory for large n: the pair tensor is built
    for `chunk` particles i at a time (the means over the reference axis j are unchanged)."""
    K = np.asarray(K, np.float64); b = np.asarray(b, np.float64)
    S = K + K.T
    F = cfg["tilde_F"]
    gamma = cfg["gamma_friction"]
    x = np.asarray(x, np.float64); v = np.asarray(v, np.float64)
    n = x.shape[0]
    cb = n if chunk is None else int(chunk)
    mg, mP, mT = [], [], []
    for i0 in range(0, n, cb):
        y = x[None, i0:i0 + cb] - x[:, None]  # [m, chunk, T, d] (x_minus_ref, :23): y[j, i] = x_i - x_j
        mg.append(np.mean(y @ S.T + b, 0))
        mP.append(np.mean(np.einsum("...i,ij,...j->...", y, K, y) + y @ b, 0))
        mT.append(np.mean(y @ F.T, 0))
    gPhi_m, Phi_m, gTrue_m = (np.concatenate(a, 0) for a in (mg, mP, mT))
    loss_nabla = np.mean(np.sum(gPhi_m ** 2, -1))
    loss_hess = np.mean(np.einsum("nti,ij,ntj->nt", v, S, v))  # Hessian constant in j
    ps = np.stack([partial_s_log_density(t, x[:, k], cfg) for k, t in enumerate(tau)], 1)
    ps2 = np.stack([partial_s2_log_density(t, x[:, k], cfg) for k, t in enumerate(tau)], 1)
    loss_value = np.mean(Phi_m * (ps2 + ps ** 2 + gamma * ps))
    loss_true = np.mean(np.sum(gTrue_m ** 2, -1))
    loss = loss_nabla - 2 * loss_hess + 2 * loss_value + loss_true
    loss_gt = np.mean(np.sum((gTrue_m - gPhi_m) ** 2, -1))
    return loss, loss_gt


# --------------------------------------------------------------------------------------
# problem constants
# --------------------------------------------------------------------------------------
def problem_constants(d, seed=2217):
    """tilde_F = G G^T, G ~ N(0,1)^{d x (d+1)} (…_OU.py:16-19 distribution, numpy PCG64 stream)."""
    G = np.random.default_rng(seed).standard_normal((d, d + 1))
    return G @ G.T


def gmm_centres(d, K, seed=2217, lo=-4.0, hi=4.0):
    """mu_k ~ U[-4, 4]^d (…_GMM.py:22-23, 52-59 distribution)."""
    return np.random.default_rng(seed + 1).uniform(lo, hi, size=(K, d))


# --------------------------------------------------------------------------------------
# derivations used by the kernels, restated in fp64 so the CPU suite can check them
# --------------------------------------------------------------------------------------
def kfp_gmm_grad_analytic(mus, z_init, z_term, z_0T, mus_true, gamma, T, sigma=1.0):
    """The analytic adjoint of residual.hip kfp_gmm_kernel: d loss / d mu via the softmax chain
    rule (F_k = df/dw_k, explicit d/dmu_j), per sample, summed with the loss weights."""
    mus = np.asarray(mus, np.float64)
    d = mus.shape[1]
    s2 = 1.0 / sigma ** 2
    s4 = s2 * s2
    G = np.zeros_like(mus)

    def acc(z, c1, c2, c3):
        z = np.asarray(z, np.float64)
        if len(z) == 0:
            return
        x, v = z[:, :d], z[:, d:]
        diff = x[:, None, :] - mus[None]
        a = -np.sum(diff ** 2, -1) * 0.5 * s2
        a -= a.max(-1, keepdims=True)
        w = np.exp(a); w /= w.sum(-1, keepdims=True)
        mbar = w @ mus
        e = x - mbar
        pk = v @ mus.T
        em = e @ mus.T
        pbar = np.sum(w * pk, -1, keepdims=True)
        Fk = -2 * c1 * s4 * em - c2 * s4 * (pk * pk - 2 * pbar * pk) - c3 * s2 * pk
        Fbar = np.sum(w * Fk, -1, keepdims=True)
        cw = w * (Fk - Fbar) * s2
        ce = -2 * c1 * s4 * w
        cv = -w * (2 * c2 * s4 * (pk - pbar) + c3 * s2)
        G[:] += np.einsum("nk,nki->ki", cw, diff) + np.einsum("nk,ni->ki", ce, e) + np.einsum("nk,ni->ki", cv, v)

    M = len(z_0T)
    acc(z_0T, 1.0 / M, -2.0 / M, 2 * gamma / M)
    if len(z_init):
        acc(z_init, 0.0, 0.0, -2.0 / (T * len(z_init)))
    if len(z_term):
        acc(z_term, 0.0, 0.0, 2.0 / (T * len(z_term)))
    return G


def kmv_from_moments(K, b, x, v, tau, cfg):
    """kmv.hip's formulation: per time stamp moments + c-weighted moments -> loss, loss_gt, grad."""
    K = np.asarray(K, np.float64); b = np.asarray(b, np.float64)
    x = np.asarray(x, np.float64); v = np.asarray(v, np.float64)
    S = K + K.T
    F = cfg["tilde_F"]
    gamma = cfg["gamma_friction"]
    n, n_t, d = x.shape
    N = n * n_t
    nabla = hess = value = true = gt = 0.0
    G = np.zeros((d, d)); gb = 2 * b.copy()
    Mvv = np.einsum("nti,ntj->ij", v, v) / N
    for t in range(n_t):
        xt = x[:, t]
        xbar = xt.mean(0)
        M = xt.T @ xt / n
        C = M - np.outer(xbar, xbar)
        ds = partial_s_log_density(tau[t], xt, cfg)
        ds2 = partial_s2_log_density(tau[t], xt, cfg)
        c = ds2 + ds ** 2 + gamma * ds
        W, Wx, Wxx = c.sum(), c @ xt, (xt * c[:, None]).T @ xt
        w = n / N
        nabla += w * np.trace(S @ C @ S)
        true += w * np.trace(F @ C @ F.T)
        D = F - S
        gt += w * np.trace(D @ C @ D.T)
        value += (0.5 * np.trace(S @ Wxx) - xbar @ S @ Wx + 0.5 * W * np.trace(S @ M) + b @ (Wx - W * xbar)) / N
        G += w * (S @ C + C @ S) + 2 * (0.5 * Wxx - np.outer(xbar, Wx) + 0.5 * W * M) / N
        gb += 2 * (Wx - W * xbar) / N
    nabla += b @ b
    gt += b @ b
    hess = np.trace(S @ Mvv)
    G += -2 * Mvv
    loss = nabla - 2 * hess + 2 * value + true
    return loss, gt, G + G.T, gb


# --------------------------------------------------------------------------------------
# non-parametric hypothesis V_hypothesis (core/model.py:32-62): Dense(W) x L, tanh, Dense(40), sum y^2
# --------------------------------------------------------------------------------------
def mlp_forward_terms(params, x, v):
    """Per sample: V, g = grad_x V (reverse), Vd = grad V . v, Vdd = v^T Hess V v (Taylor mode).
    params = [(K_1, b_1), ..., (K_L, b_L), (K_o, b_o)] with flax kernels [in, out]."""
    x = np.asarray(x, np.float64); v = np.asarray(v, np.float64)
    h, hd, hdd = x, v, np.zeros_like(x)
    cache = []
    for K, b in params[:-1]:
        z, zd, zdd = h @ K + b, hd @ K, hdd @ K
        h = np.tanh(z)
        s1 = 1 - h * h
        s2 = -2 * h * s1
        hd, hdd = s1 * zd, s1 * zdd + s2 * zd * zd
        cache.append(s1)
    Ko, bo = params[-1]
    y, yd, ydd = h @ Ko + bo, hd @ Ko, hdd @ Ko
    V = np.sum(y * y, -1)
    Vd = 2 * np.sum(y * yd, -1)
    Vdd = 2 * np.sum(yd * yd + y * ydd, -1)
    a = (2 * y) @ Ko.T
    for (K, _), s1 in zip(reversed(params[:-1]), reversed(cache)):
        a = (s1 * a) @ K.T
    return V, a, Vd, Vdd


def kfp_mlp_loss(params, z_init, z_term, z_0T, grad_true, gamma, T):
    """loss_fn (kinetic_fokker_planck.py:33-50) / loss_ground_truth_fn (:52-58) for the MLP model;
    grad_true(x) -> grad V*(x)."""
    d = params[0][0].shape[0]
    z_0T = np.asarray(z_0T, np.float64)
    x0, v0 = z_0T[:, :d], z_0T[:, d:]
    _, g, Vd, Vdd = mlp_forward_terms(params, x0, v0)
    gt = grad_true(x0)
    parts = dict(nabla=np.mean(np.sum(g * g, -1)), hessian=np.mean(Vdd), friction=gamma * np.mean(Vd),
                 nabla_true=np.mean(np.sum(gt * gt, -1)))
    for name, z in (("initial", z_init), ("terminal", z_term)):
        z = np.asarray(z, np.float64)
        parts[name] = np.mean(mlp_forward_terms(params, z[:, :d], z[:, d:])[2]) if len(z) else 0.0
    loss = (parts["nabla"] - 2 * parts["hessian"] + 2 * parts["friction"] + parts["nabla_true"]
            + (-2 * parts["initial"] + 2 * parts["terminal"]) / T)
    return loss, np.mean(np.sum((gt - g) ** 2, -1)), parts


def mlp_flat(params):
    return np.concatenate([np.concatenate([K.ravel(), b.ravel()]) for K, b in params])


def mlp_unflat(flat, dims):
    """dims = [d, W_1, ..., W_L, out]."""
    out, o = [], 0
    for i in range(len(dims) - 1):
        K = flat[o:o + dims[i] * dims[i + 1]].reshape(dims[i], dims[i + 1]); o += dims[i] * dims[i + 1]
        b = flat[o:o + dims[i + 1]]; o += dims[i + 1]
        out.append((K, b))
    return out


def kfp_mlp_grad_analytic(params, z_init, z_term, z_0T, gamma, T):
    """d loss / d params for the MLP model by the adjoint mlp.hip implements: Taylor forward
    (h, hd, hdd), the grad_x reverse chain (a, zeta), its forward-mode adjoint (abar, zetabar),
    then reverse over the three forward streams; weight gradients are sums of outer products."""
    rows, coefs = [], []
    for z, c in ((z_0T, (1.0 / len(z_0T), -2.0 / len(z_0T), 2 * gamma / len(z_0T), 0.0)),
                 (z_init, (0.0, 0.0, -2.0 / (T * max(len(z_init), 1)), 0.0)),
                 (z_term, (0.0, 0.0, 2.0 / (T * max(len(z_term), 1)), 0.0))):
        z = np.asarray(z, np.float64)
        if len(z):
            rows.append(z)
            coefs.append(np.tile(np.asarray(c)[None], (len(z), 1)))
    return mlp_grad_rows(params, np.concatenate(rows), np.concatenate(coefs))


# --------------------------------------------------------------------------------------
# overdamped Fokker–Planck (example_problems/fokker_planck_example.py,
# methods/consistency_instances/fokker_planck.py:33-63)
# --------------------------------------------------------------------------------------
def fp_configuration(F, m0_scale=1.0, P0_scale=5.0, L_scale=2.0):
    """fokker_planck_example.py:20-46."""
    F = np.asarray(F, np.float64)
    d = F.shape[0]
    U, s, _ = np.linalg.svd(F)
    L, P0, m0 = np.eye(d) * L_scale, np.eye(d) * P0_scale, np.ones(d) * m0_scale
    return {"F": F, "L": L, "U": U, "s": s, "B": U.T @ L @ U, "B_0": U.T @ P0 @ U, "m_0": m0, "P_0": P0}


def fp_mean_cov(t, cfg):
    """OU_process (:48-55): dm/dt = -F m, dP/dt = -FP - PF + L in closed form."""
    e = np.diag(np.exp(-t * cfg["s"]))
    U = cfg["U"]
    ss = cfg["s"][:, None] + cfg["s"][None, :]
    BS = cfg["B"] / ss
    return U @ e @ U.T @ cfg["m_0"], U @ (e @ cfg["B_0"] @ e + BS - e @ BS @ e) @ U.T


def fp_mlp_loss(params, x_init, x_term, x_0T, F, T):
    """loss_fn (:48-55) / loss_ground_truth_fn (:57-58): lap V = sum_k e_k^T Hess V e_k."""
    x0 = np.asarray(x_0T, np.float64)
    d = x0.shape[1]
    _, g, _, _ = mlp_forward_terms(params, x0, np.zeros_like(x0))
    lap = sum(mlp_forward_terms(params, x0, np.tile(np.eye(d)[k], (len(x0), 1)))[3] for k in range(d))
    gt = x0 @ np.asarray(F, np.float64).T
    V = lambda x: mlp_forward_terms(params, x, np.zeros_like(x))[0] if len(x) else np.zeros(0)
    vi, vt = V(np.asarray(x_init, np.float64)), V(np.asarray(x_term, np.float64))
    parts = dict(nabla=np.mean(np.sum(g * g, -1)), laplacian=np.mean(lap), nabla_true=np.mean(np.sum(gt * gt, -1)),
                 initial=np.mean(vi) if len(vi) else 0.0, terminal=np.mean(vt) if len(vt) else 0.0)
    loss = parts["nabla"] - 2 * parts["laplacian"] + parts["nabla_true"] + 2 * (parts["terminal"] - parts["initial"]) / T
    return loss, np.mean(np.sum((gt - g) ** 2, -1)), parts


def fp_mlp_grad_analytic(params, x_init, x_term, x_0T, T):
    """d loss / d params of fp_mlp_loss through mlp_grad_rows: 0T rows [x | e_k] with
    (c1, c2) = (1/(dM), -2/M); boundary rows [x | 0] weighting V with c0 = -+2/(T n)."""
    x0 = np.asarray(x_0T, np.float64)
    M, d = x0.shape
    rows = [np.concatenate([np.repeat(x0, d, 0), np.tile(np.eye(d), (M, 1))], 1)]
    coefs = [np.tile([[1.0 / (d * M), -2.0 / M, 0.0, 0.0]], (M * d, 1))]
    for x, sgn in ((x_init, -1.0), (x_term, 1.0)):
        x = np.asarray(x, np.float64)
        if len(x):
            rows.append(np.concatenate([x, np.zeros_like(x)], 1))
            coefs.append(np.tile([[0.0, 0.0, 0.0, sgn * 2.0 / (T * len(x))]], (len(x), 1)))
    return mlp_grad_rows(params, np.concatenate(rows), np.concatenate(coefs))


def mlp_grad_rows(params, Z, C, U=None):
    """Gradient of sum_r [c1 |g|^2 + c2 V'' + c3 V' + c0 V + u . g](row r) over rows Z = [x | v] with
    per-row weights C = [c1, c2, c3, c0] and optional per-row input-gradient seeds U (the adjoint
    of mlp.hip / mlp_fused.hip; U is the KMV pass-2 seed of kmv_mlp_grad_analytic)."""
    d = params[0][0].shape[0]
    L = len(params) - 1
    c1, c2, c3, c0 = C[:, :1], C[:, 1:2], C[:, 2:3], C[:, 3:4]
    x, v = Z[:, :d], Z[:, d:]
    A = [(x, v, np.zeros_like(x))]          # (h, hd, hdd) per layer input
    Zs, S = [], []
    for K, b in params[:-1]:
        h, hd, hdd = A[-1]
        z, zd, zdd = h @ K + b, hd @ K, hdd @ K
        hn = np.tanh(z)
        s1 = 1 - hn * hn
        s2 = -2 * hn * s1
        s3 = -2 * s1 * s1 - 2 * hn * s2
        A.append((hn, s1 * zd, s1 * zdd + s2 * zd * zd))
        Zs.append((zd, zdd))
        S.append((s1, s2, s3))
    Ko, bo = params[-1]
    hL, hdL, hddL = A[-1]
    y, yd, ydd = hL @ Ko + bo, hdL @ Ko, hddL @ Ko
    # grad_x chain
    u = 2 * y
    a_l = [None] * (L + 1)
    zeta = [None] * (L + 1)
    a = u @ Ko.T
    for l in range(L, 0, -1):
        a_l[l] = a
        zeta[l] = S[l - 1][0] * a
        a = zeta[l] @ params[l - 1][0].T
    g = a
    # forward-mode adjoint of the grad chain
    abar = [None] * (L + 1)
    zetabar = [None] * (L + 1)
    abar[0] = 2 * c1 * g + (0.0 if U is None else U)
    for l in range(1, L + 1):
        zetabar[l] = abar[l - 1] @ params[l - 1][0]
        abar[l] = S[l - 1][0] * zetabar[l]
    ubar = abar[L] @ Ko
    ybar = 2 * c3 * yd + 2 * c2 * ydd + 2 * ubar + 2 * c0 * y
    ydbar = 2 * c3 * y + 4 * c2 * yd
    yddbar = 2 * c2 * y
    grads = [None] * (L + 1)
    gKo = hL.T @ ybar + hdL.T @ ydbar + hddL.T @ yddbar + abar[L].T @ u
    grads[L] = (gKo, ybar.sum(0))
    hb, hdb, hddb = ybar @ Ko.T, ydbar @ Ko.T, yddbar @ Ko.T
    for l in range(L, 0, -1):
        s1, s2, s3 = S[l - 1]
        zd, zdd = Zs[l - 1]
        zb = s1 * hb + s2 * zd * hdb + (s2 * zdd + s3 * zd * zd) * hddb + s2 * a_l[l] * zetabar[l]
        zdb = s1 * hdb + 2 * s2 * zd * hddb
        zddb = s1 * hddb
        hp, hdp, hddp = A[l - 1]
        K = params[l - 1][0]
        gK = hp.T @ zb + hdp.T @ zdb + hddp.T @ zddb + abar[l - 1].T @ zeta[l]
        grads[l - 1] = (gK, zb.sum(0))
        hb, hdb, hddb = zb @ K.T, zdb @ K.T, zddb @ K.T
    return grads


# --------------------------------------------------------------------------------------
# KMV residual for a general (MLP) interaction Phi_theta = V_hypothesis
# (methods/consistency_instances/kinetic_mckean_vlasov.py:11-120 with get_model non-parametric)
# --------------------------------------------------------------------------------------
def kmv_value_weights(x, tau, cfg):
    """c[i, t] = ds2 + ds^2 + gamma ds of log rho at (tau_t, x_it) (:62-90 of the residual)."""
    gamma = cfg["gamma_friction"]
    ps = np.stack([partial_s_log_density(t, x[:, k], cfg) for k, t in enumerate(tau)], 1)
    ps2 = np.stack([partial_s2_log_density(t, x[:, k], cfg) for k, t in enumerate(tau)], 1)
    return ps2 + ps ** 2 + gamma * ps


def kmv_mlp_pairwise_loss(params, x, v, tau, cfg, weights=None):
    """Literal restatement with the [m, n, n_time, d] pair tensor x_minus_ref[a, b] = x_b - x_a
    (:20-23; the particle is b, the reference a), Phi_theta = V_hypothesis, Phi* = 0.5 y^T F y:
    loss (:74-97) and loss ground truth (:99-110). x, v: [n, n_time, d]; tau [n_time]."""
    x = np.asarray(x, np.float64); v = np.asarray(v, np.float64)
    n, nt, d = x.shape
    F = cfg["tilde_F"]
    y = x[None] - x[:, None]                                    # [m, n, T, d]
    vv = np.broadcast_to(v[None], y.shape)                      # v_b
    Phi, g, _, Hvv = mlp_forward_terms(params, y.reshape(-1, d), vv.reshape(-1, d))
    Phi, Hvv = Phi.reshape(n, n, nt), Hvv.reshape(n, n, nt)
    g = g.reshape(n, n, nt, d)
    gbar = g.mean(0)                                            # [n, T, d]
    gtrue = (y @ F.T).mean(0)
    c = kmv_value_weights(x, tau, cfg) if weights is None else weights
    loss_nabla = np.mean(np.sum(gbar ** 2, -1))
    loss_hess = np.mean(Hvv.mean(0))
    loss_value = np.mean(Phi.mean(0) * c)
    loss_true = np.mean(np.sum(gtrue ** 2, -1))
    loss = loss_nabla - 2 * loss_hess + 2 * loss_value + loss_true
    loss_gt = np.mean(np.sum((gtrue - gbar) ** 2, -1))
    return loss, loss_gt, dict(nabla=loss_nabla, hessian=loss_hess, value=loss_value, nabla_true=loss_true)


def kmv_mlp_grad_analytic(params, x, v, tau, cfg, weights=None):
    """d loss / d theta of kmv_mlp_pairwise_loss in the two passes the HIP path runs:
    pass 1 gbar_i = mean_j grad Phi(x_i - x_j); pass 2 over the pair rows [x_i - x_j | v_i] with
    c2 = -2/(n^2 T), c0 = 2 c_it/(n^2 T) per row and the input-gradient seed u_i = 2 gbar_i/(n^2 T)
    (the |mean_j grad Phi|^2 term is quadratic in the mean, so its adjoint is linear per pair)."""
    x = np.asarray(x, np.float64); v = np.asarray(v, np.float64)
    n, nt, d = x.shape
    y = (x[None] - x[:, None])                                  # [j, i, T, d]
    _, g, _, _ = mlp_forward_terms(params, y.reshape(-1, d), np.zeros((y.size // d, d)))
    gbar = g.reshape(n, n, nt, d).mean(0)                       # [i, T, d]
    c = kmv_value_weights(x, tau, cfg) if weights is None else weights
    s = 1.0 / (n * n * nt)
    rows = np.concatenate([y.reshape(-1, d), np.broadcast_to(v[None], y.shape).reshape(-1, d)], 1)
    C = np.zeros((rows.shape[0], 4))
    C[:, 1] = -2 * s
    C[:, 3] = (2 * s * np.broadcast_to(c[None], (n, n, nt))).reshape(-1)
    U = (2 * s * np.broadcast_to(gbar[None], y.shape)).reshape(-1, d)
    return mlp_grad_rows(params, rows, C, U)


# --------------------------------------------------------------------------------------
# RealNVP log-density (core/normalizing_flow.py:8-229; core/log_density_estimation.py:103-114)
# --------------------------------------------------------------------------------------
def _nvp_act(name, x):
    if name == "celu":
        return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))
    if name == "relu":
        return np.maximum(x, 0)
    if name == "tanh":
        return np.tanh(x)
    if name == "elu":
        return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))
    if name == "silu":
        return x / (1 + np.exp(-x))
    if name == "softplus":
        return np.logaddexp(x, 0)
    if name == "gelu":  # flax nn.gelu(approximate=True)
        return 0.5 * x * (1 + np.tanh(np.sqrt(2 / np.pi) * (x + 0.044715 * x ** 3)))
    raise ValueError(name)


def nvp_masks(dim, couple_mul, mask_type):
    """MNF.setup (:174-199): 'loop' zeroes one coordinate per layer; 'random' draws Bernoulli(1/2)
    masks from RandomState(888), rejecting all-0 / all-1 and repeats of the previous mask."""
    if mask_type == "loop":
        out = []
        for i in range(dim * couple_mul):
            m = np.ones(dim)
            m[i % dim] = 0
            out.append(m)
        return np.stack(out)
    rng = np.random.RandomState(seed=888)
    prev = np.zeros(dim, dtype=int)
    out = []
    for _ in range(couple_mul):
        while True:
            m = rng.binomial(1, p=0.5, size=[dim])
            if not (m.sum() in [0, dim] or (m == prev).all()):
                prev = m
                break
        out.append(m.astype(np.float64))
    return np.stack(out)


def nvp_in_dim(dim, E, ignore_time):
    return dim if ignore_time else dim + (E if E > 0 else 1)


def nvp_param_count(dim, n_layers, E, ignore_time):
    i = nvp_in_dim(dim, E, ignore_time)
    mlp = i * 8 + 8 + 8 * 16 + 16 + 16 * 16 + 16 + 16 * dim + dim
    Et = 0 if ignore_time else E
    return (2 * (Et * Et + Et) if Et > 0 else 0) + n_layers * (dim + 2 * mlp)


def nvp_unflat(flat, dim, n_layers, E, ignore_time):
    """The flat layout of include/pdeinv.h (pdeinv_realnvp_desc) -> nested lists."""
    flat = np.asarray(flat, dtype=np.float64)
    o = [0]

    def take(*shape):
        n = int(np.prod(shape))
        v = flat[o[0]:o[0] + n].reshape(shape)
        o[0] += n
        return v

    Et = 0 if ignore_time else E
    temb = [(take(Et, Et), take(Et)), (take(Et, Et), take(Et))] if Et > 0 else None
    i = nvp_in_dim(dim, E, ignore_time)
    layers = []
    for _ in range(n_layers):
        sf = take(dim)
        nets = []
        for _ in range(2):
            nets.append([(take(i, 8), take(8)), (take(8, 16), take(16)), (take(16, 16), take(16)), (take(16, dim), take(dim))])
        layers.append((sf, nets[0], nets[1]))
    assert o[0] == flat.size
    return temb, layers


def nvp_time_embedding(temb, t, E, act):
    half = E // 2
    emb = np.exp(np.arange(half) * -(np.log(10000) / (half - 1)))   # SinusoidalEmbedding (:24-38)
    e = np.asarray(t)[..., None] * emb
    se = np.concatenate([np.sin(e), np.cos(e)], -1)
    (W1, b1), (W2, b2) = temb
    return _nvp_act(act, se @ W1 + b1) @ W2 + b2                      # TimeEmbedding (:8-22)


def _nvp_mlp(net, x, act):
    h = x
    for k, (W, b) in enumerate(net):
        h = h @ W + b
        if k < 3:
            h = _nvp_act(act, h)
    return h


def realnvp_apply(flat, t, x, *, dim, masks, E=10, ignore_time=False, soft_init=1.0, act="celu", reverse=True):
    """MNF.__call__ (:205-217) over a batch: returns (x_out, ldj). reverse=True is the likelihood
    direction (layers reversed, x <- (x + tr) e^s)."""
    n_layers = masks.shape[0]
    temb, layers = nvp_unflat(flat, dim, n_layers, E, ignore_time)
    x = np.asarray(x, dtype=np.float64).copy()
    t = np.broadcast_to(np.asarray(t, dtype=np.float64), x.shape[:1])
    if ignore_time:
        tcat = np.zeros((x.shape[0], 0))
    elif E > 0:
        tcat = nvp_time_embedding(temb, t, E, act)
    else:
        tcat = t[:, None]
    ldj = np.zeros(x.shape[0])
    order = range(n_layers - 1, -1, -1) if reverse else range(n_layers)
    for l in order:
        m = masks[l]
        sf, snet, tnet = layers[l]
        xt = np.concatenate([x * m, tcat], -1)                         # CouplingLayer (:133-163)
        s, tr = _nvp_mlp(snet, xt, act), _nvp_mlp(tnet, xt, act)
        if not ignore_time and soft_init == 0.0:
            s, tr = t[:, None] * s, t[:, None] * tr
        f = np.exp(sf)
        s = np.tanh(s / f) * f * (1 - m)
        tr = tr * (1 - m)
        if reverse:
            x = (x + tr) * np.exp(s)
            ldj += s.sum(-1)
        else:
            x = x * np.exp(-s) - tr
            ldj -= s.sum(-1)
    return x, ldj


def realnvp_logdensity(flat, t, x, *, dim, masks, base_mean, base_cov, **kw):
    """RealNVP.__call__ (:223-229): log p0(T^{-1}(x)) + ldj with p0 = Gaussian (distribution.py:52-81)."""
    x0, ldj = realnvp_apply(flat, t, x, dim=dim, masks=masks, reverse=True, **kw)
    off = x0 - base_mean
    quad = np.einsum("ni,ij,nj->n", off, np.linalg.inv(base_cov), off)
    log_det = np.log(np.linalg.det(base_cov * 2 * np.pi))
    return -0.5 * (log_det + quad) + ldj


def nvp_init(dim, n_layers, E, ignore_time, seed=0, scale=1.0, perturb=False):
    """Flax defaults (lecun_normal kernels, zero biases, zero scaling factors). perturb=True adds
    random biases and scaling factors (and `scale` multiplies the kernels) so tests see a
    non-trivial flow (a fresh init is close to the identity map)."""
    rng = np.random.default_rng(seed)
    parts = []
    Et = 0 if ignore_time else E

    def dense(i, o):
        k = rng.standard_normal((i, o))
        k = np.clip(k, -2, 2) / 0.87962566103423978 * np.sqrt(1.0 / i) * scale
        parts.extend([k.ravel(), 0.3 * rng.standard_normal(o) if perturb else np.zeros(o)])

    if Et > 0:
        dense(Et, Et)
        dense(Et, Et)
    i = nvp_in_dim(dim, E, ignore_time)
    for _ in range(n_layers):
        parts.append(-1.0 + 0.2 * rng.standard_normal(dim) if perturb else np.zeros(dim))
        for _ in range(2):
            dense(i, 8)
            dense(8, 16)
            dense(16, 16)
            dense(16, dim)
    flat = np.concatenate(parts)
    assert flat.size == nvp_param_count(dim, n_layers, E, ignore_time)
    return flat


def realnvp_nll_value_and_grad(flat, t, x, *, dim, masks, base_mean, base_cov, E=10, ignore_time=False,
                               soft_init=1.0, act="celu"):
    """(loss, grad) of the maximum-likelihood step (log_density_estimation.py:47-58):
    loss = -mean log p_t(x), grad = d loss / d params in the flat layout of include/pdeinv.h.
    The same restatement as realnvp_apply / realnvp_logdensity, written in torch fp64 (CPU) so
    autograd stands in for jax.value_and_grad; the value is checked against the NumPy
    restatement and the gradient against central differences in tests/test_oracle.py."""
    import torch

    acts = {"celu": torch.nn.functional.celu, "elu": torch.nn.functional.elu, "relu": torch.relu,
            "tanh": torch.tanh, "silu": torch.nn.functional.silu, "softplus": torch.nn.functional.softplus,
            "gelu": lambda z: torch.nn.functional.gelu(z, approximate="tanh")}
    f = acts[act]
    n_layers = masks.shape[0]
    p = torch.tensor(np.asarray(flat, dtype=np.float64), requires_grad=True)
    X = torch.tensor(np.asarray(x, dtype=np.float64))
    T = torch.tensor(np.broadcast_to(np.asarray(t, dtype=np.float64), X.shape[:1]).copy())
    o = [0]

    def take(*shape):
        k = int(np.prod(shape))
        v = p[o[0]:o[0] + k].reshape(shape)
        o[0] += k
        return v

    Et = 0 if ignore_time else E
    if Et > 0:
        W1, b1, W2, b2 = take(Et, Et), take(Et), take(Et, Et), take(Et)
        half = Et // 2
        freq = torch.exp(torch.arange(half, dtype=torch.float64) * -(math.log(10000) / (half - 1)))
        e = T[:, None] * freq
        se = torch.cat([torch.sin(e), torch.cos(e)], -1)
        tcat = f(se @ W1 + b1) @ W2 + b2
    elif ignore_time:
        tcat = torch.zeros((X.shape[0], 0), dtype=torch.float64)
    else:
        tcat = T[:, None]
    i_dim = nvp_in_dim(dim, E, ignore_time)
    layers = []
    for _ in range(n_layers):
        sf = take(dim)
        nets = [[(take(i_dim, 8), take(8)), (take(8, 16), take(16)), (take(16, 16), take(16)), (take(16, dim), take(dim))]
                for _ in range(2)]
        layers.append((sf, nets[0], nets[1]))
    assert o[0] == p.numel()

    def mlp(net, h):
        for k, (W, b) in enumerate(net):
            h = h @ W + b
            if k < 3:
                h = f(h)
        return h

    M = torch.tensor(np.asarray(masks, dtype=np.float64))
    ldj = torch.zeros(X.shape[0], dtype=torch.float64)
    hard = (not ignore_time) and soft_init == 0.0
    for l in range(n_layers - 1, -1, -1):   # likelihood direction (RealNVP.__call__, reverse=True)
        sf, snet, tnet = layers[l]
        m = M[l]
        xt = torch.cat([X * m, tcat], -1)
        s, tr = mlp(snet, xt), mlp(tnet, xt)
        if hard:
            s, tr = T[:, None] * s, T[:, None] * tr
        sfe = torch.exp(sf)
        s = torch.tanh(s / sfe) * sfe * (1 - m)
        tr = tr * (1 - m)
        X = (X + tr) * torch.exp(s)
        ldj = ldj + s.sum(-1)
    off = X - torch.tensor(np.asarray(base_mean, dtype=np.float64))
    icov = torch.tensor(np.linalg.inv(base_cov))
    quad = torch.einsum("ni,ij,nj->n", off, icov, off)
    log_det = float(np.log(np.linalg.det(base_cov * 2 * np.pi)))
    loss = -(-0.5 * (log_det + quad) + ldj).mean()
    loss.backward()
    return float(loss.detach()), p.grad.numpy().copy()
