/*
 * pdeinv.h — C ABI of the MI355X-native hot path of shenzebang/PDE-inverse-problem.
 *
 * The reference is pure Python/JAX: its hot path is XLA-generated code
 * behind Python callables. Each entry point below replaces one of those callables and
 * cites the reference interface it stands in for (paths relative to the reference root).
 *
 * Conventions:
 *   - every pointer named d_* / "device" is a device (HBM) pointer owned by the caller;
 *     the library never allocates on the hot path — workspace sizes are queried first;
 *   - work is enqueued on the caller's hipStream_t (passed as void*), nothing blocks;
 *   - return 0 on success, a negative pdeinv_status on failure; the message is in
 *     pdeinv_last_error() (thread-local). Python maps INVALID -> ValueError,
 *     UNSUPPORTED -> NotImplementedError, HIP -> RuntimeError, mirroring the reference's
 *     exception types (…_OU.py:138 ValueError, consistency.py:25 NotImplementedError);
 *   - all arithmetic the reference does in fp32 is fp32 here; cross-particle sums are
 *     accumulated fp32 per thread / block and fp64 across blocks;
 *   - results are deterministic given (seed, counter_offset, particle ids): no float
 *     atomics, every reduction has a fixed order.
 *
 * RNG stream layout (Philox4x32-10, Random123; replaces jax.random threefry, which
 * cannot be reproduced bit-for-bit without JAX — SURVEY.md §8(c) P7):
 *   key = {lo32(seed), hi32(seed)}
 *   simulator normals, update s (0..n_steps) of global particle p, 4-normal block j:
 *       ctr = {lo32(p), hi32(p), counter_offset + s, j}
 *   simulator time shift tau0 of particle p:
 *       ctr = {lo32(p), hi32(p), counter_offset, 0x80000000}
 *       (McKean–Vlasov: one shared tau0 for the interacting ensemble, p = UINT64_MAX;
 *        with d_shift_u, u[0] is used)
 *   Gaussian sampler, sample r (global row), 4-normal block j:
 *       ctr = {lo32(r), hi32(r), counter_offset, 0x40000000 | j}
 *   u32 -> uniform:  u = (x >> 8) * 2^-24 in [0,1)
 *   u32 pair (a,b) -> 2 normals (Box–Muller): f(x) = as_float((x & 0x7FFFFF) | 0x3F800000)
 *       in [1,2); u1 = 2 - f(a) in (0,1], u2 = f(b) - 1 in [0,1) (both exact in fp32),
 *       r = sqrt(-2 ln u1), (r cos 2πu2, r sin 2πu2)
 *   Philox block j = (x0,x1,x2,x3) yields normals 4j..4j+3 from pairs (x0,x1),(x2,x3).
 */
#ifndef PDEINV_H
#define PDEINV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDEINV_ABI_VERSION 10  /* 10: pdeinv_sde_simulate_mf_kmv; 9: pdeinv_ou_exact_sample, pdeinv_kmv_mlp_path */
#define PDEINV_MAX_DIM 16          /* d (configuration-space dimension) */
#define PDEINV_MAX_PARAMS 256      /* floats of potential parameters passed by value */

typedef enum {
  PDEINV_OK = 0,
  PDEINV_ERR_INVALID = -1,     /* bad argument / shape  -> ValueError          */
  PDEINV_ERR_UNSUPPORTED = -2, /* unsupported kind/dim  -> NotImplementedError */
  PDEINV_ERR_HIP = -3          /* HIP runtime failure   -> RuntimeError        */
} pdeinv_status;

typedef enum {
  /* grad U(q) = A (q - c); params = A[d*d] row-major, then c[d] (optional, see has_center).
     KOU: A = tilde_F (…_OU.py:15-19, V_true_fn :130-138). */
  PDEINV_POT_QUADRATIC = 0,
  /* GMM: U(x) = -logsumexp_k(-|x-mu_k|^2 / (2 sigma^2)); grad by the analytic softmax form.
     params = mu[K*d] row-major (core/potential.py:32-61). */
  PDEINV_POT_GMM = 1,
  /* McKean–Vlasov quadratic interaction: grad U(q_i) = A (q_i - xbar_s), xbar_s the ensemble mean
     of the positions before update s. params = A[d*d]. Two drivers:
     pdeinv_sde_simulate with d_meanfield = the precomputed mean path (pdeinv_mf_sums ->
     all-reduce -> pdeinv_mf_mean_path), or update by update with pdeinv_mf_step. */
  PDEINV_POT_MEANFIELD_QUADRATIC = 2,
  /* U = 0 (core/potential.py VoidPotential). */
  PDEINV_POT_NONE = 3
} pdeinv_potential_kind;

typedef struct {
  int32_t kind;        /* pdeinv_potential_kind */
  int32_t n_centers;   /* K for GMM (<= PDEINV_MAX_PARAMS / d) */
  float sigma;         /* GMM component std (reference: 1, …_GMM.py:76-78) */
  int32_t has_center;  /* QUADRATIC: params[d*d .. d*d+d) is c */
  const float* params; /* HOST pointer, copied by value into the kernel arguments */
} pdeinv_potential;

/* ---------------------------------------------------------------------------------------
 * Simulator — replaces utils/sampling_utils.py:25-52 underdamped_langevin_dynamics_scan
 * (vmapped per particle) and its update_step :6-22.
 *   per particle: tau0 = U*dt; one update of h = tau0, n_steps-1 updates of h = dt, one of
 *   h = dt - tau0 (total T = n_steps*dt); each update
 *       p' = p - h*gradU(q) + sqrt(h)*noise_scale*xi - gamma*p*h ;  q' = q + h*p'
 *   traj[s] is the state after update s (s = 0..n_steps-1), tau[s] = tau0 + s*dt,
 *   last = state after update n_steps.
 * Layout: z0 [N, 2d] (x first, v second; row stride ld_z0 floats, >= 2d).
 *         traj [n_steps, N, 2d] TIME-MAJOR (coalesced stores; the reference's [N, n, 2d]
 *         is traj.permute(1,0,2)); tau [n_steps, N]; last [N, 2d]. Each output nullable.
 * Moments (optional, fused — the KFP residual then needs no re-read of traj): when
 * d_moments != NULL the kernel accumulates, for the three sample sets
 *   set 0 = z0 ("initial"), set 1 = traj ("0T"), set 2 = last ("terminal"),
 * the fp64 vector [count, sum z (2d), sum z_i z_j (i<=j, row-major upper triangle)]
 * (pdeinv_moment_len(2d) doubles per set) into d_moments[3][len]. Requires d_workspace of
 * pdeinv_sde_workspace_bytes() bytes.
 * --------------------------------------------------------------------------------------- */
typedef struct {
  int64_t n_particles;      /* N in this call (may be 0) */
  int64_t particle_offset;  /* global id of row 0 (rank sharding: ids are rank-count invariant) */
  int32_t dim;              /* d, 1..PDEINV_MAX_DIM */
  int32_t n_steps;          /* n >= 1 */
  float dt;                 /* T / n */
  float gamma;              /* friction (KOU 1.0 …_OU.py:21; GMM 0.5 …_GMM.py:17) */
  float noise_scale;        /* sqrt(2) (sampling_utils.py:14) */
  int32_t random_shift;     /* 1: tau0 ~ U(0,dt) (reference); 0: tau0 = 0 */
  uint64_t seed;
  uint32_t counter_offset;  /* advance by n_steps+1 between calls */
  int64_t ld_z0;            /* row stride of z0 in floats (0 => 2d) */
  pdeinv_potential potential;
  const float* d_noise;     /* nullable: explicit xi [n_steps+1, N, d] (parity mode) */
  const float* d_shift_u;   /* nullable: explicit u [N] in [0,1) for tau0 = u*dt */
  const float* d_meanfield; /* MEANFIELD + pdeinv_sde_simulate: xbar [n_steps+1, d] fp32, the mean
                               path of pdeinv_mf_mean_path (row s is used by update s) */
} pdeinv_sde_desc;

int pdeinv_moment_len(int m); /* 1 + m + m(m+1)/2 */
size_t pdeinv_sde_workspace_bytes(const pdeinv_sde_desc* desc);
int pdeinv_sde_simulate(const pdeinv_sde_desc* desc, const float* d_z0, float* d_traj,
                        float* d_tau, float* d_last, void* d_workspace, double* d_moments,
                        void* stream);

/* McKean–Vlasov stepping (one update per call; the mean-field xbar of the current state is
 * an input so that ranks can all-reduce it between calls — SURVEY.md §8(e)).
 * Reads z [N,2d] (state before the update), writes z_out [N,2d] (may alias traj row), and
 * accumulates the fp64 partial [count, sum x (d)] of the NEW positions into d_xsum
 * (pdeinv_mf_workspace_bytes()). h selects the update kind: 0 = tau0 step, 1 = dt step,
 * 2 = final dt - tau0 step; s is the update index (RNG counter). */
size_t pdeinv_mf_workspace_bytes(const pdeinv_sde_desc* desc);
int pdeinv_mf_step(const pdeinv_sde_desc* desc, int32_t s, const float* d_z, float* d_z_out,
                   float* d_tau_row, const float* d_tau0, const double* d_xbar_sum,
                   void* d_workspace, double* d_xsum, void* stream);
/* McKean–Vlasov, fused multi-step path. For the quadratic interaction the ensemble mean obeys
 *   vbar' = (1 - gamma h) vbar + sqrt(h) noise_scale xibar_s,  xbar' = xbar + h vbar'
 * exactly (the drift A (x_i - xbar) averages to zero), xibar_s the mean of update s's noise — a
 * function of the particle ids and the RNG stream only. So the mean path needs ONE reduction:
 *   pdeinv_mf_sums:  d_sums [pdeinv_mf_sums_len(desc)] fp64 =
 *                    [count, sum x0 (d), sum v0 (d), sum_i xi_{i,s} (d) for s = 0..n_steps]
 *                    over this call's particles (rank-local; all-reduce(sum) it across ranks);
 *   pdeinv_mf_mean_path: the all-reduced sums -> d_xbar [n_steps+1, d] fp32 (mean before update s)
 *                    and optionally d_xsum [n_steps+2, 1+d] fp64 = [count, count * xbar_s]
 *                    (the closed-form path, a model quantity — not sums measured from the simulated
 *                    fp32 states; take pdeinv_moments of the trajectory for those);
 *   pdeinv_sde_simulate(desc with d_meanfield = d_xbar): all n_steps+1 updates in registers.
 * The explicit-noise mode (d_noise) is honoured by pdeinv_mf_sums and the simulator alike. */
int64_t pdeinv_mf_sums_len(const pdeinv_sde_desc* desc);
size_t pdeinv_mf_sums_workspace_bytes(const pdeinv_sde_desc* desc);
int pdeinv_mf_sums(const pdeinv_sde_desc* desc, const float* d_z0, void* d_workspace, double* d_sums,
                   void* stream);
int pdeinv_mf_mean_path(const pdeinv_sde_desc* desc, const double* d_sums, float* d_xbar, double* d_xsum,
                        void* stream);
/* ABI 8. pdeinv_sde_simulate (fused McKean–Vlasov path, desc->d_meanfield set) that also returns the NEXT
 * simulate's pdeinv_mf_sums(next, d_z0_next) in d_sums_next [pdeinv_mf_sums_len] fp64 (rank-local): the noise
 * sums are drawn inside the store-bound simulator instead of by a separate launch or the KMV pass. `next` may
 * differ from `desc` in counter_offset only (same seed, particles, particle_offset, dim, n_steps); Philox
 * noise; even dim <= 8, n_steps + 1 <= 128 (else PDEINV_ERR_UNSUPPORTED: use pdeinv_mf_sums). Equal to
 * pdeinv_mf_sums up to the fp32 partial-sum order; deterministic. Replaces the sums half of the reference's
 * per-update mean field (kinetic_mckean_vlasov.py:20-23 through sampling_utils.py:6-22). */
size_t pdeinv_sde_simulate_mf_next_workspace_bytes(const pdeinv_sde_desc* desc);
int pdeinv_sde_simulate_mf_next(const pdeinv_sde_desc* desc, const float* d_z0, float* d_traj, float* d_tau,
                                float* d_last, const pdeinv_sde_desc* next, const float* d_z0_next,
                                void* d_workspace, double* d_sums_next, void* stream);
/* ABI 10. pdeinv_sde_simulate (fused McKean–Vlasov path, desc->d_meanfield set) that also forms the quadratic-Φ
 * KMV residual's per-time-stamp sums of its own trajectory rows 0..n_steps-1 — exactly what
 * pdeinv_kmv_moments_weights(dim, gamma, d_coef, d_traj, n_steps, N, N*2d, 2d) returns (d_mom [n_steps,
 * moment_len(2d)], d_wstats [n_steps, moment_len(d)] fp64, rank-local), up to the fp32 summation order — from the
 * rows the simulator stages for its stores, so the trajectory is not read back (d_traj may be NULL). d_coef
 * [n_steps, 3d + 2 + 2d^2] as pdeinv_kmv_weights. With `next` non-NULL it also returns the next simulate's
 * pdeinv_mf_sums in d_sums_next as pdeinv_sde_simulate_mf_next (same restrictions: counter offset only,
 * n_steps + 1 <= 128). Even dim <= 8, Philox noise (else PDEINV_ERR_UNSUPPORTED); deterministic. Replaces the
 * simulate of sampling_utils.py:25-52 followed by the pair sums of kinetic_mckean_vlasov.py:11-120.
 * Workspace (256-byte aligned): pdeinv_sde_simulate_mf_kmv_workspace_bytes(desc, next != NULL). */
size_t pdeinv_sde_simulate_mf_kmv_workspace_bytes(const pdeinv_sde_desc* desc, int32_t with_next);
int pdeinv_sde_simulate_mf_kmv(const pdeinv_sde_desc* desc, const float* d_z0, float* d_traj, float* d_tau,
                               float* d_last, float gamma, const float* d_coef, double* d_mom, double* d_wstats,
                               const pdeinv_sde_desc* next, const float* d_z0_next, double* d_sums_next,
                               void* d_workspace, void* stream);
/* tau0 per particle (u*dt from the shift stream, or d_shift_u) -> d_tau0 [N]. */
int pdeinv_sde_tau0(const pdeinv_sde_desc* desc, float* d_tau0, void* stream);

/* ---------------------------------------------------------------------------------------
 * Generic moment reduction of a sample set (rows of m floats, row stride ld floats) —
 * the reduction behind every parametric-quadratic residual term
 * (methods/consistency_instances/kinetic_fokker_planck.py:33-58) for data that did not come
 * out of the fused simulator (offline subsample, exact Gaussian samples).
 * Output: d_out[pdeinv_moment_len(m)] fp64 (count, sums, upper-triangle products).
 * --------------------------------------------------------------------------------------- */
size_t pdeinv_moments_workspace_bytes(int64_t n_rows, int32_t m);
int pdeinv_moments(const float* d_z, int64_t n_rows, int32_t m, int64_t ld, void* d_workspace,
                   double* d_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * KFP residual, parametric quadratic V_theta(x) = x . Dense_d(x) = x^T K x + b^T x
 * (…_OU.py:209-220), grad V = S x + b, Hessian S = K + K^T.
 * Replaces kinetic_fokker_planck.py:11-69 value_and_grad_fn for this model: every term of
 * loss_fn (:33-50) and loss_ground_truth_fn (:52-58) is an expectation of a polynomial of
 * degree <= 2 in z, so all of them — and d loss / d(K,b) — follow exactly from the three
 * moment sets (init, 0T, terminal). d_moments: [3][pdeinv_moment_len(2d)] fp64 sums
 * (possibly all-reduced over ranks). d_theta = [K (d*d, flax layout [in,out]), b (d)] fp32.
 * Outputs: d_out[PDEINV_KFP_NOUT] fp32, d_grad [d*d + d] fp32 (same layout as theta).
 * --------------------------------------------------------------------------------------- */
enum {
  PDEINV_KFP_LOSS = 0,
  PDEINV_KFP_LOSS_GT = 1,        /* "loss ground truth" */
  PDEINV_KFP_GRAD_NORM = 2,
  PDEINV_KFP_NABLA = 3,          /* E_0T |grad V_theta|^2 */
  PDEINV_KFP_HESSIAN = 4,        /* E_0T v^T H v */
  PDEINV_KFP_FRICTION = 5,       /* gamma * E_0T grad V_theta . v */
  PDEINV_KFP_NABLA_TRUE = 6,     /* E_0T |grad V*|^2 */
  PDEINV_KFP_INITIAL = 7,        /* E_init grad V_theta . v */
  PDEINV_KFP_TERMINAL = 8,       /* E_term grad V_theta . v */
  PDEINV_KFP_NOUT = 9
};

typedef struct {
  int32_t dim;
  float gamma;
  float total_time;          /* T (divides the boundary terms, :48-50) */
  const float* tilde_F;      /* HOST [d*d]: grad V* = tilde_F x (V_true, …_OU.py:130-138) */
} pdeinv_kfp_quad_desc;

int pdeinv_residual_kfp_quadratic(const pdeinv_kfp_quad_desc* desc, const double* d_moments,
                                  const float* d_theta, float* d_out, float* d_grad,
                                  void* stream);

/* ---------------------------------------------------------------------------------------
 * KFP residual, parametric GMM V_theta(x) = -logsumexp_k(-|x-mu_k|^2/(2 sigma^2)) with
 * learnable mu [K,d] (…_GMM.py:214-234), true potential GMM(mu*) (…_GMM.py:94-102).
 * Fused per-sample forward (grad V, v^T H v, grad V . v, grad V*) and the analytic adjoint
 * d/d mu (replaces jax.value_and_grad, kinetic_fokker_planck.py:60-61).
 * Sets: initial [n_init,2d], terminal [n_term,2d], 0T [n_0T,2d], each with its row stride.
 * Coefficients (c_*) weight the per-sample terms so that the accumulators are the loss and
 * gradient directly:  loss = sum_0T(c_nabla T1 + c_hess T2 + c_fric T3 + c_true Tt)
 *                          + c_init sum_init T3 + c_term sum_term T3.
 * (reference: c_nabla = 1/M, c_hess = -2/M, c_fric = 2 gamma/M, c_true = 1/M,
 *  c_init = -2/(T B_i), c_term = 2/(T B_t)). The fp64 accumulator d_acc has
 * PDEINV_GMM_NACC + K*d entries and may be all-reduced before pdeinv_residual_kfp_gmm_finalize.
 * --------------------------------------------------------------------------------------- */
enum {
  PDEINV_GMM_ACC_LOSS = 0,     /* weighted loss (all terms) */
  PDEINV_GMM_ACC_LOSS_GT = 1,  /* c_true * sum |grad V* - grad V|^2 */
  PDEINV_GMM_ACC_NABLA = 2,    /* c_true * sum T1 (unweighted mean when c_true = 1/M) */
  PDEINV_GMM_ACC_HESSIAN = 3,  /* c_true * sum T2 */
  PDEINV_GMM_ACC_FRICTION = 4, /* c_true * sum T3 */
  PDEINV_GMM_ACC_NABLA_TRUE = 5,
  PDEINV_GMM_ACC_INITIAL = 6,  /* sum_init T3 / n_init */
  PDEINV_GMM_ACC_TERMINAL = 7, /* sum_term T3 / n_term */
  PDEINV_GMM_NACC = 8
};

typedef struct {
  int32_t dim;
  int32_t n_centers;         /* K of the model */
  float sigma;               /* model sigma (reference 1) */
  int32_t n_centers_true;    /* K* */
  float sigma_true;
  const float* mus_true;     /* HOST [K* * d] */
  float gamma;               /* friction (…_GMM.py:17), reported in the FRICTION slot */
  float c_nabla, c_hess, c_fric, c_true, c_init, c_term;
} pdeinv_kfp_gmm_desc;

size_t pdeinv_residual_kfp_gmm_workspace_bytes(const pdeinv_kfp_gmm_desc* desc, int64_t n_init,
                                               int64_t n_term, int64_t n_0T);
int pdeinv_residual_kfp_gmm(const pdeinv_kfp_gmm_desc* desc, const float* d_init,
                            int64_t n_init, int64_t ld_init, const float* d_term,
                            int64_t n_term, int64_t ld_term, const float* d_0T, int64_t n_0T,
                            int64_t ld_0T, const float* d_mus, void* d_workspace,
                            double* d_acc, void* stream);
/* d_acc -> d_out[PDEINV_KFP_NOUT] (same slots as the quadratic residual), d_grad [K*d]. */

/* The GMM simulator with this residual fused in (the reference's online KFP-GMM iteration:
 * …_GMM.py:104-142 simulate, then kinetic_fokker_planck.py:11-69 over initial = z0, 0T = every
 * trajectory row, terminal = last). Each particle's rows are consumed in registers as they are
 * produced (no re-read of the trajectory); grad V* of a 0T row is the simulator's grad U at that
 * state, so the residual's true GMM (n_centers_true, sigma_true, mus_true) must be the simulated
 * potential (checked: PDEINV_ERR_INVALID otherwise). d_mus = the model centres [K*d] (device).
 * Coefficients as above with n_init = n_term = N, n_0T = N * n_steps (global counts over ranks);
 * the INITIAL / TERMINAL slots hold sum T3 / N of this call. Outputs: the simulator's (each nullable)
 * and d_acc [PDEINV_GMM_NACC + K*d] fp64 (all-reduce, then pdeinv_residual_kfp_gmm_finalize).
 * dim <= 8, model n_centers * dim <= 64. */
size_t pdeinv_sde_simulate_kfp_gmm_workspace_bytes(const pdeinv_sde_desc* desc, const pdeinv_kfp_gmm_desc* res);
int pdeinv_sde_simulate_kfp_gmm(const pdeinv_sde_desc* desc, const pdeinv_kfp_gmm_desc* res, const float* d_mus,
                                const float* d_z0, float* d_traj, float* d_tau, float* d_last, void* d_workspace,
                                double* d_acc, void* stream);
int pdeinv_residual_kfp_gmm_finalize(const pdeinv_kfp_gmm_desc* desc, const double* d_acc,
                                     float* d_out, float* d_grad, void* stream);

/* ---------------------------------------------------------------------------------------
 * Batched moments: n_sets sample sets of n_rows rows each; row r of set t starts at
 * z + t*set_stride + r*ld (floats). out [n_sets][pdeinv_moment_len(m)] fp64.
 * The per-time-stamp moments behind the McKean–Vlasov residual (one set per time stamp):
 * mean_j grad Phi(x_i - x_j) = S (x_i - xbar_t) + b for quadratic Phi
 * (kinetic_mckean_vlasov.py:20-23, 74-97), so xbar_t and Cov_t replace the O(n^2) pairs.
 * --------------------------------------------------------------------------------------- */
size_t pdeinv_moments_batched_workspace_bytes(int64_t n_sets, int64_t n_rows, int32_t m);
int pdeinv_moments_batched(const float* d_z, int64_t n_sets, int64_t n_rows, int32_t m,
                           int64_t set_stride, int64_t ld, void* d_workspace, double* d_out,
                           void* stream);

/* ---------------------------------------------------------------------------------------
 * Score / log-density time derivatives of the Gaussian X-marginal N(m1(s), P11(s)) —
 * partial_s_log_density_fn / partial_s2_log_density_fn
 * (kinetic_mckean_vlasov_example_quadratic.py:18-191). Per time stamp t the host passes
 * (from the closed-form OU moments) the coefficient row
 *   [m1 (d), a1, beta1 (d), Gamma1 (d*d), a2, beta2 (d), Gamma2 (d*d)]   (PDEINV_KMV_NCOEF(d))
 * with  ds log rho  = a1 + beta1 . r + r^T Gamma1 r,  ds2 log rho = a2 + beta2 . r + r^T Gamma2 r,
 * r = m1 - x. Per particle the kernel evaluates both, c = ds2 + ds^2 + gamma ds (the weight
 * of the Phi term, kinetic_mckean_vlasov.py:243-248), and accumulates per time stamp the
 * fp64 vector [sum c, sum c x (d), sum c x_i x_j (i<=j)] (pdeinv_moment_len(d) doubles).
 * Optional per-particle output d_ds [n_sets, n_rows, 2] = (ds log rho, ds2 log rho).
 * --------------------------------------------------------------------------------------- */
#define PDEINV_KMV_NCOEF(d) (3 * (d) + 2 + 2 * (d) * (d))
size_t pdeinv_kmv_weights_workspace_bytes(int64_t n_sets, int64_t n_rows, int32_t dim);
int pdeinv_kmv_weights(int32_t dim, float gamma, const float* d_coef, const float* d_z,
                       int64_t n_sets, int64_t n_rows, int64_t set_stride, int64_t ld,
                       float* d_ds, void* d_workspace, double* d_out, void* stream);

/* Fused pdeinv_moments_batched(m = 2d) + pdeinv_kmv_weights: one read of each row z = [x, v] gives
 * d_mom [n_sets][pdeinv_moment_len(2d)] and d_wstats [n_sets][pdeinv_moment_len(d)] (the same sums,
 * the same layout). dim <= 8. Workspace: pdeinv_kmv_moments_weights_workspace_bytes(). */
size_t pdeinv_kmv_moments_weights_workspace_bytes(int64_t n_sets, int64_t n_rows, int32_t dim);
int pdeinv_kmv_moments_weights(int32_t dim, float gamma, const float* d_coef, const float* d_z, int64_t n_sets,
                               int64_t n_rows, int64_t set_stride, int64_t ld, void* d_workspace, double* d_mom,
                               double* d_wstats, void* stream);

/* The same pass fused with the NEXT McKean–Vlasov simulate's mean-path input (the steady state of the
 * KMV training loop, config C4): besides d_mom / d_wstats it writes d_sums_next =
 * pdeinv_mf_sums(next, d_z0_next) — the noise sums of updates t < n_sets are generated inside the
 * HBM-bound pass (stamp t's rows are the particles next->particle_offset + r, next->n_particles ==
 * n_rows, dim equal, Philox noise only), the remaining updates and the [count, x0, v0] block by a
 * tail launch. Equal to pdeinv_mf_sums up to the fp32 partial-sum order (different block tiling).
 * Workspace: pdeinv_kmv_moments_weights_mf_sums_workspace_bytes(). */
size_t pdeinv_kmv_moments_weights_mf_sums_workspace_bytes(int64_t n_sets, int64_t n_rows, int32_t dim,
                                                          const pdeinv_sde_desc* next);
int pdeinv_kmv_moments_weights_mf_sums(int32_t dim, float gamma, const float* d_coef, const float* d_z,
                                       int64_t n_sets, int64_t n_rows, int64_t set_stride, int64_t ld,
                                       void* d_workspace, double* d_mom, double* d_wstats,
                                       const pdeinv_sde_desc* next, const float* d_z0_next, double* d_sums_next,
                                       void* stream);

/* KMV residual for Phi_theta(y) = y . Dense_d(y) (…_quadratic.py:205-216) from the per-time-stamp
 * moments of z (mom [n_sets][moment_len(2d)]) and weighted stats (wst [n_sets][moment_len(d)]):
 * loss (:74-97 of kinetic_mckean_vlasov.py), loss ground truth (:256-266) and d loss/d(K,b).
 * Outputs d_out[PDEINV_KFP_NOUT] (INITIAL/TERMINAL slots unused = 0; FRICTION slot = the
 * "2 * loss_value" term) and d_grad [d*d + d]. */
typedef struct {
  int32_t dim;
  int32_t n_sets;
  float gamma;
  const float* tilde_F;  /* HOST [d*d]: Phi* = 0.5 y^T tilde_F y (…_quadratic.py:193-203) */
} pdeinv_kmv_desc;
size_t pdeinv_residual_kmv_workspace_bytes(const pdeinv_kmv_desc* desc);
int pdeinv_residual_kmv(const pdeinv_kmv_desc* desc, const double* d_mom, const double* d_wstats,
                        const float* d_theta, void* d_workspace, float* d_out, float* d_grad, void* stream);

/* ---------------------------------------------------------------------------------------
 * KFP residual for the non-parametric hypothesis V_hypothesis (core/model.py:32-62):
 * V(x) = sum_o y_o^2, y = Dense_out(tanh(Dense_W(... tanh(Dense_W(x))))), out = 40.
 * Fused value + d loss / d theta over the three sample sets (same loss and coefficients as the
 * GMM residual): Taylor-mode forward streams, the grad_x reverse chain, its forward adjoint, the
 * reverse sweep and the weight-gradient outer products, as dense GEMMs (rocBLAS sgemm, fp32) plus
 * fused element-wise kernels, chunked over chunk_rows rows. impl selects the implementation:
 * PDEINV_MLP_IMPL_AUTO and PDEINV_MLP_IMPL_FUSED take the hand-written fused path for every d <= 16,
 * 1 <= L <= 16, W <= 1024 and any out_features: fp32 MFMA GEMMs whose prologues and epilogues carry all of
 * the element-wise algebra (layer 1 is recomputed from the rows, never stored; L = 1 runs the output layer
 * off the layer-1 prologue). The kernels are compiled for d in {2, 4, 8, 16} and W in {32, 64, 128, 256,
 * 512, 1024}; other d / W (e.g. the reference default 20 x 8 layers, MLP.yaml) run zero-padded to the next
 * compiled one (exact; rows, parameters and the true potential padded, the gradient unpadded, on the
 * device). PDEINV_MLP_IMPL_LIBRARY forces the rocBLAS + element-wise-kernel path (explicit opt-in, the
 * only way rocBLAS is loaded); AUTO and FUSED on a shape outside the above return PDEINV_ERR_UNSUPPORTED.
 * d_params / d_grad: flat flax order [K_1 (d x W), b_1, K_2 (W x W), b_2, ..., K_o (W x out), b_o]
 * (pdeinv_mlp_param_count floats). d_acc [PDEINV_GMM_NACC] and d_grad are ACCUMULATED (+=): zero
 * them first. pdeinv_kfp_terms_finalize turns (acc, grad) into the PDEINV_KFP_* slots.
 * --------------------------------------------------------------------------------------- */
typedef struct {
  int32_t dim;            /* d */
  int32_t n_layers;       /* hidden layers L >= 1 (neural_network.layers) */
  int32_t width;          /* hidden width W (neural_network.hidden_dim) */
  int32_t out_features;   /* 40 in the reference */
  int32_t true_kind;      /* PDEINV_POT_QUADRATIC (tilde_F, d*d) or PDEINV_POT_GMM (mus, K*d) */
  int32_t n_centers_true;
  float sigma_true;
  const float* true_params; /* HOST */
  float gamma;
  float c_nabla, c_hess, c_fric, c_true, c_init, c_term;
  int64_t chunk_rows;     /* rows per GEMM chunk (workspace grows with it); 0 => 2^18 */
  int32_t impl;           /* PDEINV_MLP_IMPL_* */
  int32_t boundary_value; /* 0: boundary sets weight V' = grad V . v (kinetic FP, :49-50);
                             1: they weight V itself (overdamped FP, fokker_planck.py:48-52) —
                             see pdeinv_fp_rows for the overdamped residual's row layout */
} pdeinv_kfp_mlp_desc;
#define PDEINV_MLP_IMPL_AUTO 0
#define PDEINV_MLP_IMPL_LIBRARY 1 /* rocBLAS sgemm path (cross-check; librocblas.so.5 loaded at run time) */
#define PDEINV_MLP_IMPL_FUSED 2
#define PDEINV_MLP_IMPL_PAIRS_RING 3 /* pdeinv_residual_kmv_mlp only: force the register-ring pair kernels
                                        (width <= 28) instead of the MFMA pair tiles — A/B and cross-checks */
/* 1 when impl = AUTO runs this V_hypothesis shape on the hand-written fused fp32-MFMA kernels (compiled shapes and
   the zero-padded envelope: dim <= 16, width <= 1024, depth 1..16, any out_features), 0 when AUTO rejects it
   (PDEINV_ERR_UNSUPPORTED: only the explicit impl = LIBRARY cross-check runs such shapes, on rocBLAS) */
int pdeinv_mlp_fused_supported(int32_t dim, int32_t n_layers, int32_t width, int32_t out_features);
/* Residual calls (pdeinv_residual_kfp_mlp / pdeinv_residual_kmv_mlp) served by rocBLAS in this process so far: only
   impl = LIBRARY ever adds to it (ABI 10). */
int64_t pdeinv_rocblas_calls(void);
int64_t pdeinv_mlp_param_count(int32_t dim, int32_t n_layers, int32_t width, int32_t out_features);
size_t pdeinv_residual_kfp_mlp_workspace_bytes(const pdeinv_kfp_mlp_desc* desc);
int pdeinv_residual_kfp_mlp(const pdeinv_kfp_mlp_desc* desc, const float* d_init, int64_t n_init,
                            int64_t ld_init, const float* d_term, int64_t n_term, int64_t ld_term,
                            const float* d_0T, int64_t n_0T, int64_t ld_0T, const float* d_params,
                            void* d_workspace, double* d_acc, float* d_grad, void* stream);
int pdeinv_kfp_terms_finalize(const double* d_acc, const float* d_grad, int64_t n_grad, float gamma,
                              float* d_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * KMV residual for a general interaction Phi_theta = V_hypothesis (the non-parametric model of
 * core/model.py:109-131 under kinetic_mckean_vlasov.py:11-120): every pair (i, j) of the n_rows
 * particles of each of the n_sets time stamps, y = x_i - x_j (x_minus_ref, :20-23). Two passes over
 * pair rows built chunk by chunk (gbar_i = mean_j grad Phi, then the per-pair adjoint with seed
 * 2 gbar_i / (n^2 n_sets)) on the library MLP path. d_z: rows [x | v] of stamp t at
 * d_z + t*set_stride + i*ld; d_ds [n_sets][n_rows][2] = (ds log rho, ds2 log rho) from
 * pdeinv_kmv_weights. d_acc [PDEINV_GMM_NACC] and d_grad are ACCUMULATED (+=, zero them first);
 * pdeinv_kfp_terms_finalize(acc, grad, P, gamma = 1) gives the PDEINV_KFP_* slots (HESSIAN = the
 * pair mean of v^T Hess Phi v, FRICTION = 2 x the weighted value mean, as pdeinv_residual_kmv).
 * Multi-GPU: pairs are formed within each rank's particles (the reference's per-device batch under
 * pmap, trainer.py:44-53); average the finalized outputs over ranks.
 * --------------------------------------------------------------------------------------- */
typedef struct {
  int32_t dim;            /* d <= 16 (the pair kernels and LIBRARY: d <= 8) */
  int32_t n_layers;       /* hidden layers (neural_network.layers) */
  int32_t width;          /* hidden width (neural_network.hidden_dim) */
  int32_t out_features;   /* 40 in the reference */
  int32_t n_sets;         /* time stamps */
  int64_t n_rows;         /* particles per time stamp */
  float gamma;            /* friction (weights c = ds2 + ds^2 + gamma ds) */
  const float* tilde_F;   /* HOST [d*d]: Phi* = 0.5 y^T tilde_F y (…_quadratic.py:193-203) */
  int64_t chunk_rows;     /* pair rows per GEMM chunk (library path); 0 => 2^18 */
  int32_t impl;           /* PDEINV_MLP_IMPL_*: AUTO / FUSED = the hand-written paths — width <= 20 with
                             n_layers <= 8 and dim <= 8 (the reference default 20 x 8): 16-pair fp32 MFMA
                             tiles (mlp_pairs_mfma.hip; any out_features — routed before the ring limits;
                             workspace ~ CUs x 4 waves x P floats + the weight image, ~15 MB for the default
                             net); other widths <= 28 (or every width <= 28 under PAIRS_RING):
                             the register-ring pair kernels (pairs built in registers, MFMA weight
                             gradients; dim <= 8, n_layers <= 16, out <= 64; workspace ~ 2048 waves x
                             (5 W L x 64 + P) floats); width >= 32 (dim <= 16 zero-padded to 2/4/8/16,
                             1 <= n_layers <= 16, width <= 1024 zero-padded to 32/64/.../1024, any out):
                             chunks of pair rows through the fused fp32-MFMA residual kernels of
                             pdeinv_residual_kfp_mlp; LIBRARY = pair rows through rocBLAS (explicit opt-in, loaded
                             at run time: libpdeinv.so does not link rocBLAS) */
} pdeinv_kmv_mlp_desc;
/* The path pdeinv_residual_kmv_mlp takes for this descriptor (shape + impl): PDEINV_KMV_PATH_PAIR_TILES (the
   16-pair MFMA tiles), _PAIR_RING (the register-ring pair kernels), _FUSED_ROWS (pair rows through the fused
   fp32-MFMA residual kernels), _LIBRARY (pair rows through rocBLAS), or -1 when the shape is unsupported. */
#define PDEINV_KMV_PATH_PAIR_TILES 0
#define PDEINV_KMV_PATH_PAIR_RING 1
#define PDEINV_KMV_PATH_FUSED_ROWS 2
#define PDEINV_KMV_PATH_LIBRARY 3
int pdeinv_kmv_mlp_path(const pdeinv_kmv_mlp_desc* desc);
size_t pdeinv_residual_kmv_mlp_workspace_bytes(const pdeinv_kmv_mlp_desc* desc);
int pdeinv_residual_kmv_mlp(const pdeinv_kmv_mlp_desc* desc, const float* d_z, int64_t set_stride, int64_t ld,
                            const float* d_ds, const float* d_params, void* d_workspace, double* d_acc,
                            float* d_grad, void* stream);

/* ---------------------------------------------------------------------------------------
 * Exact kinetic-OU sampler (example_problems/kinetic_fokker_planck_example_OU.py:140-156, the reference's
 * default KOU data: groups of rows, each from N(m(t_g), P(t_g)) at its own time t_g ~ U(t_min, t_max)),
 * entirely on the device: per group the Van Loan exponential X = exp(B t_g), B = [[-F, L], [0, F^T]]
 * (scaled Taylor sum of degree taylor_degree over the host-precomputed powers B^0..B^K, then `squarings`
 * squarings — the host's ou_moments_batched recipe), m = e^{Ft} m0, P = e^{Ft}(P0 e^{F^T t} + X[:n, n:]),
 * its lower Cholesky factor R (fp64), and the rows m + R xi with the grouped Gaussian sampler's noise stream
 * (pdeinv_gaussian_sample_grouped with the same seed / ctr_z / row_off and these means / factors gives the
 * same rows). t_g = t_min + (t_max - t_min) u_g, u_g = 24 bits of Philox(seed; (g, 0, ctr_t, 0xD0000000)),
 * unless t_in gives them. Outputs t_out [G], mean_out [G, n], factor_out [G, n, n] are optional (null).
 * n = 2d, any even n <= 32 (d = 1..16); d_powers [(taylor_degree + 1), 2n, 2n], d_m0 [n], d_P0 [n, n] fp64.
 * --------------------------------------------------------------------------------------- */
typedef struct {
  int32_t n;              /* 2d */
  int32_t taylor_degree;  /* K (<= 30) */
  int32_t squarings;      /* s: |B|_1 t_max / 2^s <= 1 */
  double t_min, t_max;
  const double* d_powers; /* B^0 .. B^K */
  const double* d_m0;
  const double* d_P0;
} pdeinv_ou_desc;
int pdeinv_ou_exact_sample(const pdeinv_ou_desc* desc, int64_t n_groups, int64_t rows_per_group, uint64_t seed,
                           uint32_t ctr_t, uint32_t ctr_z, int64_t row_off, const float* d_t_in, float* d_t_out,
                           float* d_mean_out, float* d_factor_out, float* d_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Overdamped Fokker–Planck (example_problems/fokker_planck_example.py,
 * methods/consistency_instances/fokker_planck.py:33-63) — the reference's default pde_instance.
 *
 * Residual: loss = E_0T|grad V|^2 - 2 E_0T[lap V] + E_0T|grad V*|^2 + (2/T)(E_T V - E_0 V) for the
 * V_hypothesis MLP, through pdeinv_residual_kfp_mlp with boundary_value = 1 on rows built here:
 *   unit_directions = 1: out[r*d + k] = [x_r | e_k]  (lap V = sum_k e_k^T Hess V e_k: the 0T set
 *                        with c_nabla = c_true = 1/(d M), c_hess = -2/M, c_fric = 0);
 *   unit_directions = 0: out[r] = [x_r | 0]          (boundary sets: only V is weighted).
 * x [n, ldx] rows of d floats (device) -> out [n * (unit_directions ? d : 1), 2d].
 * --------------------------------------------------------------------------------------- */
int pdeinv_fp_rows(const float* d_x, int64_t n, int64_t ldx, int32_t dim, int32_t unit_directions,
                   float* d_out, void* stream);

/* Exact sampler of the overdamped OU law (fokker_planck_example.py:48-61, sample_ground_truth
 * :88-96): sample r draws its own time t_r ~ U(t_lo, t_hi) (t_lo == t_hi: a fixed time), then
 * x_r ~ N(m(t_r), P(t_r)) with, in the eigenbasis F = U diag(s) U^T,
 *   U^T m(t) = e^{-ts} o (U^T m0),  U^T P(t) U = e B0 e + (B / (s_i + s_j)) o (1 - e_i e_j),
 *   e = diag(e^{-ts}), B0 = U^T P0 U, B = U^T L U                                  (:48-55)
 * — moments, Cholesky factor and sample all in registers, one thread per sample. Host arrays
 * (row-major): U [d*d], s [d], Um0 [d], B0 [d*d], B [d*d]; d <= 8. out [n, d]; t_out [n] nullable.
 * Stream: time u from ctr {row, counter_offset, 0x10000000}, normals as pdeinv_gaussian_sample. */
int pdeinv_fp_exact_sample(int64_t n, int32_t dim, uint64_t seed, uint32_t counter_offset, int64_t row_offset,
                           float t_lo, float t_hi, const float* U_host, const float* s_host, const float* Um0_host,
                           const float* B0_host, const float* B_host, float* d_out, float* d_t_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * GMM potential value and gradient over a batch — GMMPotential.value/.gradient
 * (core/potential.py:48-61; V_true_fn of …_GMM.py:94-102). Either output nullable.
 * --------------------------------------------------------------------------------------- */
int pdeinv_gmm_potential(int32_t dim, int32_t n_centers, float sigma, const float* mus_host,
                         const float* d_x, int64_t n, int64_t ld, float* d_value,
                         float* d_grad, void* stream);

/* ---------------------------------------------------------------------------------------
 * Exact Gaussian sampler — core/distribution.py:52-65 Gaussian.sample: z = C^{1/2} xi + mu.
 * d_mean [m], d_cov_half [m*m] row-major (device); out [n, m]; rows are global ids
 * row_offset + r (rank sharding). m <= 2*PDEINV_MAX_DIM.
 * --------------------------------------------------------------------------------------- */
int pdeinv_gaussian_sample(int64_t n, int32_t m, uint64_t seed, uint32_t counter_offset,
                           int64_t row_offset, const float* d_mean, const float* d_cov_half,
                           float* d_out, void* stream);
/* Grouped form — the KOU exact sampler (…_OU.py:140-190: one Gaussian N(m(t_g), P(t_g)) per
 * random time, `sample_per_time` rows each) in one launch: rows [g*rows_per_group, (g+1)*...)
 * use d_means[g] ([n_groups, m]) and d_cov_halves[g] ([n_groups, m, m]). Same row stream as
 * pdeinv_gaussian_sample (global row = row_offset + r). */
int pdeinv_gaussian_sample_grouped(int64_t n_groups, int64_t rows_per_group, int32_t m, uint64_t seed,
                                   uint32_t counter_offset, int64_t row_offset, const float* d_means,
                                   const float* d_cov_halves, float* d_out, void* stream);

/* Raw Philox4x32-10 blocks for the KAT / stream tests: block i uses
 * ctr = {lo32(i), hi32(i), ctr_z, ctr_w}; out [n_blocks, 4] u32. */
int pdeinv_philox_fill(uint64_t seed, uint32_t ctr_z, uint32_t ctr_w, int64_t n_blocks,
                       uint32_t* d_out, void* stream);

/* Strided time/trajectory subsample gather (consistency.py:97-118, offline mode):
 * out[r*n_t + t] = traj_tm[time_idx[t], traj_idx[r]] for a time-major traj [n, N, m]. */
int pdeinv_gather_subsample(const float* d_traj, int64_t n_particles, int32_t n_steps,
                            int32_t m, const int32_t* d_traj_idx, int64_t n_traj_sel,
                            const int32_t* d_time_idx, int32_t n_time_sel, float* d_out,
                            void* stream);

/* One uniformly drawn step per particle (Philox stream ctr.w = 0x20000000): out[p] =
 * traj_tm[t_p, p], optional t_out[p] = t_p. The per-particle 0T batch of BASELINE config 5. */
int pdeinv_gather_random_step(const float* d_traj, int64_t n_particles, int32_t n_steps, int32_t m,
                              uint64_t seed, uint32_t ctr, float* d_out, int32_t* d_t_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Time-conditioned RealNVP log-density (core/normalizing_flow.py:8-229, the model built by
 * core/log_density_estimation.py:103-114): log p_t(x) = log p0(T_t^{-1}(x)) + sum ldj, the
 * coupling layers applied in reverse order (MNF.__call__(reverse=True), :205-217).
 * Each CouplingLayer (:115-163): xt = [x * mask, temb(t)] (or [x * mask, t], or x * mask),
 * s = scale_net(xt), tr = translate_net(xt) (BasicMLP: Dense 8, act, Dense 16, act, Dense 16,
 * act, Dense dim), [soft_init == 0: s, tr *= t], sf = exp(scaling_factor), s = tanh(s / sf) sf,
 * s, tr *= (1 - mask); x = (x + tr) exp(s), ldj += sum s.
 * temb (TimeEmbedding, :8-22): Dense_E(act(Dense_E(SinusoidalEmbedding_E(t)))).
 * Flat parameter layout (d_params, fp32, flax kernels [in, out] row-major):
 *   [E > 0] temb: W1 [E x E], b1 [E], W2 [E x E], b2 [E]
 *   per layer l (forward order): scaling_factor [dim]; scale_net: W0 [in x 8], b0, W1 [8 x 16], b1,
 *   W2 [16 x 16], b2, W3 [16 x dim], b3; translate_net: the same; in = dim + (E > 0 ? E : 1)
 *   (dim only when ignore_time). pdeinv_realnvp_param_count gives the total.
 * --------------------------------------------------------------------------------------- */
#define PDEINV_ACT_CELU 0
#define PDEINV_ACT_RELU 1
#define PDEINV_ACT_TANH 2
#define PDEINV_ACT_ELU 3
#define PDEINV_ACT_SILU 4
#define PDEINV_ACT_SOFTPLUS 5
#define PDEINV_ACT_GELU 6 /* tanh approximation (flax nn.gelu default) */
#define PDEINV_REALNVP_MAX_LAYERS 64
typedef struct {
  int32_t dim;             /* 1..8 */
  int32_t n_layers;        /* coupling layers, <= PDEINV_REALNVP_MAX_LAYERS */
  int32_t embed_time_dim;  /* E: 0 => the raw t is appended; even, <= 16 */
  int32_t ignore_time;
  float soft_init;         /* 0 => hard parameterisation (s, tr scaled by t) */
  int32_t activation;      /* PDEINV_ACT_* */
  const float* masks;      /* HOST [n_layers * dim], 1 = keep */
  const float* base_mean;  /* HOST [dim]: log p0 = -1/2 (log_det + (x - m)^T inv_cov (x - m)) */
  const float* base_inv_cov; /* HOST [dim * dim] */
  float base_log_det;      /* log det(2 pi cov) (distribution.py:60) */
} pdeinv_realnvp_desc;
int64_t pdeinv_realnvp_param_count(const pdeinv_realnvp_desc* desc);
/* out[i] = log p_{t_i}(x_i); t_stride 0 broadcasts d_t[0]. */
int pdeinv_realnvp_logdensity(const pdeinv_realnvp_desc* desc, const float* d_params, const float* d_t,
                              int64_t t_stride, const float* d_x, int64_t n, int64_t ld_x, float* d_out,
                              void* stream);

/* Maximum-likelihood value_and_grad of the flow (replaces jax.value_and_grad(loss_fn) in
 * core/log_density_estimation.py:47-58): *d_loss = -mean_i log p_{t_i}(x_i), d_grad[param_count]
 * = d loss / d params (same flat layout as d_params). d_workspace: pdeinv_realnvp_grad_workspace
 * bytes (a per-block partial slab; reduced in a fixed order, deterministic). n >= 1. */
int64_t pdeinv_realnvp_grad_workspace(const pdeinv_realnvp_desc* desc, int64_t n);
int pdeinv_realnvp_value_and_grad(const pdeinv_realnvp_desc* desc, const float* d_params, const float* d_t,
                                  int64_t t_stride, const float* d_x, int64_t n, int64_t ld_x, float* d_loss,
                                  float* d_grad, void* d_workspace, int64_t workspace_bytes, void* stream);

/* Fused optimizer step of the trainer (core/trainer.py:85-86 + main.py:11-29):
 * optax.chain(add_decayed_weights(weight_decay), adam(lr, b1, b2, eps)) then apply_updates, in
 * place over a flat parameter vector; count = the step number after increment (>= 1). */
int pdeinv_adam_update(float* d_params, const float* d_grad, float* d_mu, float* d_nu, int64_t n, float lr,
                       float b1, float b2, float eps, float weight_decay, int32_t count, void* stream);

int pdeinv_abi_version(void);
const char* pdeinv_last_error(void);
/* HIP runtime version the library is running against (detects a second HIP runtime). */
int pdeinv_runtime_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PDEINV_H */
