/*
 * pdeinv_oracle.c — CPU ORACLE (test infrastructure only).
 *
 * Plain-C, single-threaded restatement of the reference's hot path, used ONLY by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker / CPU baseline.
 * Nothing in the product path (pde-inverse-problem_amd/) links or calls this file.
 *
 * Parity status: the reference is Python/JAX and JAX is not installed in this image
 * (SURVEY.md §0, §8(c)); its threefry bit-stream is therefore unobtainable and this oracle
 * is pinned instead by (i) the Random123 Philox4x32-10 known-answer vectors, (ii) the exact
 * discrete-chain / analytic OU moments (oracle/numpy_ref.py) and (iii) fixtures generated
 * by oracle/make_golden.py. Bit parity with JAX streams: "parity unpinned" (DESIGN.md §3).
 *
 * Follows:
 *   utils/sampling_utils.py:6-22   update_step
 *   utils/sampling_utils.py:25-52  underdamped_langevin_dynamics_scan (tau0 shift, n+1 updates)
 *   core/potential.py:32-46        gmm_V / g_gmm_V (grad of -logsumexp, analytic softmax form
 *                                  of the commented code at :39-43)
 *   example_problems/kinetic_fokker_planck_example_OU.py:130-138  grad V* = tilde_F x
 *   core/distribution.py:64-65     Gaussian.sample
 * RNG: the stream layout documented in include/pdeinv.h.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

/* Random123 philox4x32 with R = 10 rounds. */
void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2],
                          uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
    uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    if (r < 9) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline float u32_to_unit(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }

/* Box–Muller of one u32 pair (include/pdeinv.h): the low 23 bits of each word are the mantissa
 * of a float f in [1, 2); u1 = 2 - f1 in (0, 1] and the angle is f2 - 1 revolutions (both exact in
 * fp32); transcendentals in double, rounded once. */
static inline float unit_1_2(uint32_t x) {
  union { uint32_t u; float f; } c;
  c.u = (x & 0x007FFFFFu) | 0x3F800000u;
  return c.f;
}
static inline void box_muller(uint32_t a, uint32_t b, float* z0, float* z1) {
  float u1 = 2.0f - unit_1_2(a);
  float rev = unit_1_2(b) - 1.0f;
  double r = sqrt(-2.0 * log((double)u1));
  double th = 2.0 * M_PI * (double)rev;
  *z0 = (float)(r * cos(th));
  *z1 = (float)(r * sin(th));
}

static void normals_block(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                          float z[4]) {
  uint32_t ctr[4] = {c0, c1, c2, c3};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  oracle_philox4x32_10(ctr, key, o);
  box_muller(o[0], o[1], &z[0], &z[1]);
  box_muller(o[2], o[3], &z[2], &z[3]);
}

/* d normals of update s of global particle p. */
void oracle_sim_normals(uint64_t seed, uint64_t p, uint32_t ctr_z, int d, float* out) {
  for (int j = 0; 4 * j < d; ++j) {
    float z[4];
    normals_block(seed, (uint32_t)p, (uint32_t)(p >> 32), ctr_z, (uint32_t)j, z);
    for (int k = 0; k < 4 && 4 * j + k < d; ++k) out[4 * j + k] = z[k];
  }
}

float oracle_shift_u(uint64_t seed, uint64_t p, uint32_t counter_offset) {
  uint32_t ctr[4] = {(uint32_t)p, (uint32_t)(p >> 32), counter_offset, 0x80000000u};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  oracle_philox4x32_10(ctr, key, o);
  return u32_to_unit(o[0]);
}

/* ---- potentials ------------------------------------------------------------------ */
enum { POT_QUADRATIC = 0, POT_GMM = 1, POT_MEANFIELD = 2, POT_NONE = 3 };

/* grad of V(x) = -logsumexp_k(a_k), a_k = -|x-mu_k|^2/(2 s^2)  (core/potential.py:32-37) */
void oracle_gmm_grad(int d, int K, float sigma, const float* mus, const float* x, float* g,
                     float* value) {
  double a[64];
  double amax = -INFINITY;
  double inv2s2 = 1.0 / (2.0 * (double)sigma * (double)sigma);
  for (int k = 0; k < K; ++k) {
    double s = 0.0;
    for (int i = 0; i < d; ++i) {
      double t = (double)x[i] - (double)mus[k * d + i];
      s += t * t;
    }
    a[k] = -s * inv2s2;
    if (a[k] > amax) amax = a[k];
  }
  double den = 0.0;
  for (int k = 0; k < K; ++k) { a[k] = exp(a[k] - amax); den += a[k]; }
  if (value) *value = (float)(-(amax + log(den)));
  if (g) {
    for (int i = 0; i < d; ++i) {
      double acc = 0.0;
      for (int k = 0; k < K; ++k) acc += a[k] * ((double)x[i] - (double)mus[k * d + i]);
      g[i] = (float)(acc / den / ((double)sigma * (double)sigma));
    }
  }
}

static void grad_u(int kind, int d, int K, float sigma, const float* params, int has_center,
                   const float* xbar, const float* q, float* g) {
  if (kind == POT_QUADRATIC || kind == POT_MEANFIELD) {
    float c[16];
    for (int i = 0; i < d; ++i) {
      float ci = 0.0f;
      if (kind == POT_MEANFIELD) ci = xbar[i];
      else if (has_center) ci = params[d * d + i];
      c[i] = q[i] - ci;
    }
    for (int i = 0; i < d; ++i) {
      float acc = 0.0f;
      for (int j = 0; j < d; ++j) acc += params[i * d + j] * c[j];
      g[i] = acc;
    }
  } else if (kind == POT_GMM) {
    oracle_gmm_grad(d, K, sigma, params, q, g, NULL);
  } else {
    for (int i = 0; i < d; ++i) g[i] = 0.0f;
  }
}

/*
 * underdamped_langevin_dynamics_scan restated (sampling_utils.py:25-52), all particles,
 * fp32 state. traj time-major [n, N, 2d]; tau [n, N]; last [N, 2d]; any output may be NULL.
 * noise (nullable): explicit xi [n+1, N, d]; shift_u (nullable): explicit u [N].
 * meanfield (nullable, POT_MEANFIELD): xbar is computed here, exactly, from the current
 * fp32 positions of ALL N particles before each update (the interacting-particle system).
 */
int oracle_sde_simulate(int64_t N, int64_t particle_offset, int d, int n_steps, float dt,
                        float gamma, float noise_scale, int random_shift, uint64_t seed,
                        uint32_t counter_offset, int kind, int K, float sigma,
                        const float* params, int has_center, const float* noise,
                        const float* shift_u, const float* z0, int64_t ld_z0, float* traj,
                        float* tau, float* last) {
  if (d < 1 || d > 16 || n_steps < 1 || N < 0) return -1;
  if (ld_z0 == 0) ld_z0 = 2 * d;
  const int m = 2 * d;
  float* st = (float*)malloc(sizeof(float) * (size_t)(N > 0 ? N : 1) * m);
  float* t0 = (float*)malloc(sizeof(float) * (size_t)(N > 0 ? N : 1));
  if (!st || !t0) { free(st); free(t0); return -3; }
  for (int64_t i = 0; i < N; ++i) {
    memcpy(st + i * m, z0 + i * ld_z0, sizeof(float) * m);
    float u = 0.0f;
    /* McKean–Vlasov particles interact, so they must share one clock: a single tau0 drawn
       from the global id UINT64_MAX (include/pdeinv.h). */
    int64_t idx = (kind == POT_MEANFIELD) ? 0 : i;
    uint64_t gid = (kind == POT_MEANFIELD) ? UINT64_MAX : (uint64_t)(particle_offset + i);
    if (random_shift) u = shift_u ? shift_u[idx] : oracle_shift_u(seed, gid, counter_offset);
    t0[i] = random_shift ? u * dt : 0.0f;
  }
  float xbar[16];
  for (int s = 0; s <= n_steps; ++s) {
    if (kind == POT_MEANFIELD) {
      for (int k = 0; k < d; ++k) {
        double acc = 0.0;
        for (int64_t i = 0; i < N; ++i) acc += st[i * m + k];
        xbar[k] = (float)(N > 0 ? acc / (double)N : 0.0);
      }
    }
    for (int64_t i = 0; i < N; ++i) {
      float* q = st + i * m;
      float* p = q + d;
      float h = (s == 0) ? t0[i] : ((s == n_steps) ? dt - t0[i] : dt);
      float g[16], xi[16];
      grad_u(kind, d, K, sigma, params, has_center, xbar, q, g);
      if (noise) {
        for (int k = 0; k < d; ++k) xi[k] = noise[((int64_t)s * N + i) * d + k];
      } else {
        oracle_sim_normals(seed, (uint64_t)(particle_offset + i), counter_offset + (uint32_t)s, d, xi);
      }
      float sh = sqrtf(h) * noise_scale;
      for (int k = 0; k < d; ++k) {
        /* p_new = p - dt*grad_U + sqrt(dt)*noise - gamma*p*dt  (sampling_utils.py:17) */
        p[k] = p[k] - h * g[k] + sh * xi[k] - gamma * p[k] * h;
      }
      for (int k = 0; k < d; ++k) q[k] = q[k] + h * p[k]; /* :20, new p */
      if (s < n_steps) {
        if (traj) memcpy(traj + ((int64_t)s * N + i) * m, q, sizeof(float) * m);
        if (tau) tau[(int64_t)s * N + i] = t0[i] + (float)s * dt;
      } else if (last) {
        memcpy(last + i * m, q, sizeof(float) * m);
      }
    }
  }
  free(st);
  free(t0);
  return 0;
}

/* [count, sum z (m), sum z_i z_j (i<=j)] in fp64 — the moment layout of include/pdeinv.h */
void oracle_moments(const float* z, int64_t n, int m, int64_t ld, double* out) {
  int len = 1 + m + m * (m + 1) / 2;
  memset(out, 0, sizeof(double) * len);
  if (ld == 0) ld = m;
  out[0] = (double)n;
  for (int64_t r = 0; r < n; ++r) {
    const float* row = z + r * ld;
    for (int i = 0; i < m; ++i) out[1 + i] += row[i];
    int o = 1 + m;
    for (int i = 0; i < m; ++i)
      for (int j = i; j < m; ++j) out[o++] += (double)row[i] * (double)row[j];
  }
}

/* Gaussian.sample restated (distribution.py:64-65) with the sampler stream. */
void oracle_gaussian_sample(int64_t n, int m, uint64_t seed, uint32_t counter_offset,
                            int64_t row_offset, const float* mean, const float* cov_half,
                            float* out) {
  float xi[32];
  for (int64_t r = 0; r < n; ++r) {
    uint64_t g = (uint64_t)(row_offset + r);
    for (int j = 0; 4 * j < m; ++j) {
      float z[4];
      normals_block(seed, (uint32_t)g, (uint32_t)(g >> 32), counter_offset, 0x40000000u | (uint32_t)j, z);
      for (int k = 0; k < 4 && 4 * j + k < m; ++k) xi[4 * j + k] = z[k];
    }
    for (int i = 0; i < m; ++i) {
      float acc = 0.0f;
      for (int j = 0; j < m; ++j) acc += cov_half[i * m + j] * xi[j];
      out[r * m + i] = acc + mean[i];
    }
  }
}

void oracle_philox_fill(uint64_t seed, uint32_t ctr_z, uint32_t ctr_w, int64_t n_blocks,
                        uint32_t* out) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  for (int64_t i = 0; i < n_blocks; ++i) {
    uint32_t ctr[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), ctr_z, ctr_w};
    oracle_philox4x32_10(ctr, key, out + 4 * i);
  }
}
