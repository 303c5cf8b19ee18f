// common.h — device helpers shared by the pdeinv HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <string>

#include "../../include/pdeinv.h"

namespace pdeinv {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kBlock = 256;          // 4 waves of 64
constexpr int kWave = 64;
constexpr int kWavesPerBlock = kBlock / kWave;

// ---- A/B switches of the measurement tools ------------------------------------------------
// Only a tools/build_var.sh build with -DPDEINV_AB_ENV=1 reads them: the default library reads no environment
// variable, so a stray variable in a user's shell cannot change which kernels run.
#ifndef PDEINV_AB_ENV
#define PDEINV_AB_ENV 0
#endif
inline const char* ab_env(const char* name) {
#if PDEINV_AB_ENV
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// ---- error plumbing (host) ------------------------------------------------------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

#define PDEINV_REQUIRE(cond, code, msg) \
  do {                                  \
    if (!(cond)) return ::pdeinv::fail((code), (msg)); \
  } while (0)

// ---- Philox4x32-10 (Random123) ----------------------------------------------------------
constexpr uint32_t kM0 = 0xD2511F53u, kM1 = 0xCD9E8D57u;
constexpr uint32_t kW0 = 0x9E3779B9u, kW1 = 0xBB67AE85u;

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product (hi and lo together) instead of v_mul_hi + v_mul_lo
    // and one v_bitop3_b32 (LUT 0x96 = a ^ b ^ c, gfx950) per three-way xor instead of two v_xor
    const uint64_t p0 = (uint64_t)kM0 * c.x, p1 = (uint64_t)kM1 * c.z;
    c = make_uint4(__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
                   __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0);
    k0 += kW0;
    k1 += kW1;
  }
  return c;
}

// u32 -> [0,1) with 24 random bits (exact in fp32; identical on host and device).
__device__ __forceinline__ float u32_unit(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }

// Box–Muller on the hardware transcendentals (v_log_f32 is log2, v_sin/v_cos take revolutions).
// Each u32 becomes a float in [1, 2) with one v_and_or_b32 (the low 23 bits as the mantissa):
// u1 = 2 - f1 in (0, 1] (exact), and the angle f2 in [1, 2) revolutions is the same angle as
// f2 - 1 in [0, 1) — no shift / convert / scale per uniform.
__device__ __forceinline__ float unit_1_2(uint32_t x) { return __uint_as_float((x & 0x007FFFFFu) | 0x3F800000u); }
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float u1 = 2.0f - unit_1_2(a);  // (0, 1]
  const float th = unit_1_2(b);         // [1, 2) revolutions
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  z0 = r * __builtin_amdgcn_cosf(th);
  z1 = r * __builtin_amdgcn_sinf(th);
}

// d standard normals of update counter `ctr` of particle (plo, phi): the simulator's noise stream
// (include/pdeinv.h: Philox4x32-10 block j = (plo, phi, ctr, j), Box–Muller on each pair).
template <int D>
__device__ __forceinline__ void stream_normals(uint32_t k0, uint32_t k1, uint32_t ctr, uint32_t plo, uint32_t phi,
                                               float* xi) {
#pragma unroll
  for (int j = 0; 4 * j < D; ++j) {
    const uint4 r = philox4x32_10(make_uint4(plo, phi, ctr, (uint32_t)j), k0, k1);
    float z[4];
    box_muller(r.x, r.y, z[0], z[1]);
    box_muller(r.z, r.w, z[2], z[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * j + k < D) xi[4 * j + k] = z[k];
  }
}

// The McKean–Vlasov mean-path noise stream of one simulate (pdeinv_mf_sums), for kernels that sum
// it outside the simulator (the fused KMV pass, kmv.hip). Filled / validated by mf_noise_of (sde.hip).
struct MfNoise {
  uint32_t k0, k1, ctr_off;
  int64_t poff;
};
int mf_noise_of(const pdeinv_sde_desc* d, int dim, int64_t n_particles, MfNoise& out);
// pdeinv_mf_sums restricted to updates y0..n_steps and the [count, x0, v0] block: writes those columns of
// `sums` (the columns of updates < y0 are left to the caller). Workspace: pdeinv_mf_sums_workspace_bytes.
int mf_sums_tail(const pdeinv_sde_desc* d, const float* z0, int y0, void* ws, double* sums, hipStream_t st);

// ---- wave / block reductions ------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Reduce the N per-thread values over the block and store the block sum of value c < n_write
// to partials[c * n_blocks + block] (column-major slab: the fp64 reducer then reads each
// column contiguously). N is compile-time so `vals` stays in VGPRs (a runtime index would
// demote the whole array to scratch). `lds` holds kWavesPerBlock * N floats. All threads call.
template <int N>
__device__ __forceinline__ void block_reduce_to_slab(const float (&vals)[N], int n_write, float* lds,
                                                     float* partials, int block, int n_blocks) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  __syncthreads();  // lds may still be read by a previous call
#pragma unroll
  for (int c = 0; c < N; ++c) {
    if (c < n_write) {
      const float s = wave_sum(vals[c]);
      if (lane == 0) lds[wave * N + c] = s;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < n_write; c += kBlock) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) s += lds[w * N + c];
    partials[(int64_t)c * n_blocks + block] = s;
  }
}

// ---- moments layout -----------------------------------------------------------------------
__host__ __device__ constexpr int moment_len(int m) { return 1 + m + m * (m + 1) / 2; }

template <int M>
struct MomentAcc {
  float v[moment_len(M)];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < moment_len(M); ++i) v[i] = 0.f;
  }
  __device__ __forceinline__ void add(const float* z, float w) {  // w = 1 (active) or 0
    v[0] += w;
#pragma unroll
    for (int i = 0; i < M; ++i) v[1 + i] = fmaf(w, z[i], v[1 + i]);
    int o = 1 + M;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const float wz = w * z[i];
#pragma unroll
      for (int j = i; j < M; ++j) {
        v[o] = fmaf(wz, z[j], v[o]);
        ++o;
      }
    }
  }
};

// Step-loop moment accumulator: sum z and the Gram sum z z^T of one particle's rows, laid out so
// that every packed FMA (v_pk_fma_f32) multiplies an ALIGNED register pair (z[2p], z[2p+1]) by a
// broadcast z[i]: row i keeps pairs p = i/2 .. M/2-1 (for odd i the first pair's low lane
// duplicates entry (i-1, i) and is dropped). No register shuffles on the hot loop; finish() maps
// the pairs onto the MomentAcc triangle (count, sums, i <= j) and applies the 0/1 lane weight.
template <int M>
struct PairGram {
  static constexpr int P = M / 2;
  static constexpr int npairs() {
    int n = 0;
    for (int i = 0; i < M; ++i) n += P - i / 2;
    return n;
  }
  f32x2 s[P];
  f32x2 g[npairs()];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int p = 0; p < P; ++p) s[p] = f32x2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < npairs(); ++k) g[k] = f32x2{0.f, 0.f};
  }
  __device__ __forceinline__ void add(const float* z) {
    f32x2 zp[P];
#pragma unroll
    for (int p = 0; p < P; ++p) zp[p] = f32x2{z[2 * p], z[2 * p + 1]};
#pragma unroll
    for (int p = 0; p < P; ++p) s[p] += zp[p];
    int k = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const f32x2 zi = f32x2{z[i], z[i]};
#pragma unroll
      for (int p = i / 2; p < P; ++p) {
        g[k] = zi * zp[p] + g[k];
        ++k;
      }
    }
  }
  __device__ __forceinline__ void finish(float rows, float w, float* v) const {
    v[0] = rows * w;
#pragma unroll
    for (int i = 0; i < M; ++i) v[1 + i] = w * s[i / 2][i % 2];
    int o = 1 + M, k = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
#pragma unroll
      for (int p = i / 2; p < P; ++p) {
#pragma unroll
        for (int l = 0; l < 2; ++l)
          if (2 * p + l >= i) v[o++] = w * g[k][l];
        ++k;
      }
    }
  }
};

// softmax weights w_k of a_k = -|x - mu_k|^2 / (2 s^2) = (x.mu_k - |mu_k|^2/2)/s^2 + const(x)
// (the |x|^2 term cancels in the softmax); returns w, mbar = sum_k w_k mu_k and t_k = x.mu_k.
// l2s = log2(e)/s^2, nh[k] = -|mu_k|^2/2. Even d runs on packed pairs (v_pk_fma_f32).
template <int D>
__device__ __forceinline__ float dotd(const float* a, const float* b) {
  if constexpr (D % 2 == 0) {
    f32x2 t = {0.f, 0.f};
#pragma unroll
    for (int p = 0; p < D / 2; ++p) t = f32x2{a[2 * p], a[2 * p + 1]} * f32x2{b[2 * p], b[2 * p + 1]} + t;
    return t[0] + t[1];
  } else {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < D; ++i) t = fmaf(a[i], b[i], t);
    return t;
  }
}

// ---- GMM softmax and KFP-GMM residual, packed over centre pairs ---------------------------
// A KM-slot GMM is held as KM/2 centre pairs: pair p keeps (mu_{2p,i}, mu_{2p+1,i}) for every
// coordinate i and the two logit constants c_k = -l2s |mu_k|^2 / 2 (log2 units, l2s = log2 e / s^2;
// -inf in empty slots, whose weight is then exactly 0 with no per-centre branch). Every per-centre
// scalar of the softmax and of the residual adjoint is one half of a v_pk_* instruction, and the
// d-term dots x . mu_k accumulate two centres at once with no horizontal add. (The previous layout
// packed over coordinates and spent one scalar instruction per centre on every softmax / adjoint
// scalar: 527 -> see DESIGN.md §4.4 for the instruction counts of the fused C3 step loop.)
template <int D, int KM>
struct GmmPairs {
  static_assert(KM % 2 == 0, "GMM centre slots come in pairs");
  static constexpr int KP = KM / 2;
  f32x2 mu[KP][D];
  f32x2 c[KP];
  // slot k of a K-centre GMM (mus [K, D] row-major); empty slots: mu = 0, c = -inf. For an object in
  // memory (LDS), one thread per slot: scalar stores, so the two threads of a pair never race.
  __device__ __forceinline__ void set(int k, int K, const float* mus, float l2s) {
    float n2 = 0.f;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const float m = k < K ? mus[k * D + i] : 0.f;
      reinterpret_cast<float*>(&mu[k / 2][i])[k % 2] = m;
      n2 = fmaf(m, m, n2);
    }
    reinterpret_cast<float*>(&c[k / 2])[k % 2] = k < K ? -0.5f * l2s * n2 : -INFINITY;
  }
};

__device__ __forceinline__ f32x2 bc2(float s) { return f32x2{s, s}; }

// E_k = 2^(a_k - max a) for a_k = l2s (x . mu_k) + c_k (the softmax logits of -|x - mu_k|^2 / (2 s^2)
// up to the k-independent -|x|^2 / (2 s^2)); returns sum_k E_k.
template <int D, int KM>
__device__ __forceinline__ float gmm_exp_weights(const f32x2 (*mu)[D], const f32x2* c, float l2s, const float* x,
                                                 f32x2* E) {
  constexpr int KP = KM / 2;
  float amax = -INFINITY;
  // coordinate-outer: the KP pair chains advance side by side, so no packed FMA waits on the one just issued
  // (a dependent v_pk_* read costs a wait state on gfx950); each chain keeps its i = 0..D-1 order
  f32x2 t[KP];
#pragma unroll
  for (int p = 0; p < KP; ++p) t[p] = bc2(x[0]) * mu[p][0];
#pragma unroll
  for (int i = 1; i < D; ++i)
#pragma unroll
    for (int p = 0; p < KP; ++p) t[p] = bc2(x[i]) * mu[p][i] + t[p];
#pragma unroll
  for (int p = 0; p < KP; ++p) {
    E[p] = t[p] * bc2(l2s) + c[p];
    amax = fmaxf(amax, fmaxf(E[p][0], E[p][1]));
  }
  f32x2 S = {0.f, 0.f};
#pragma unroll
  for (int p = 0; p < KP; ++p) {
    const f32x2 a = E[p] - bc2(amax);
    E[p] = f32x2{__builtin_amdgcn_exp2f(a[0]), __builtin_amdgcn_exp2f(a[1])};
    S += E[p];
  }
  return S[0] + S[1];
}

// sum_k E_k mu_k[i] for every coordinate (two centre chains, added at the end)
template <int D, int KM>
__device__ __forceinline__ void gmm_mix(const f32x2 (*mu)[D], const f32x2* E, float* out) {
  constexpr int KP = KM / 2;
  f32x2 s[D];  // centre-outer: the D coordinate chains side by side (each keeps its p = 0..KP-1 order)
#pragma unroll
  for (int i = 0; i < D; ++i) s[i] = E[0] * mu[0][i];
#pragma unroll
  for (int p = 1; p < KP; ++p)
#pragma unroll
    for (int i = 0; i < D; ++i) s[i] = E[p] * mu[p][i] + s[i];
#pragma unroll
  for (int i = 0; i < D; ++i) out[i] = s[i][0] + s[i][1];
}

// grad of U = -logsumexp_k(-|q - mu_k|^2 / (2 s^2)) = (q - sum_k w_k mu_k) / s^2 (core/potential.py:32-37;
// the softmax form of the commented analytic gradient :39-43).
template <int D, int KM>
__device__ __forceinline__ void gmm_grad(const f32x2 (*mu)[D], const f32x2* c, float l2s, float inv_s2,
                                         const float* q, float* g) {
  f32x2 E[KM / 2];
  const float inv = __builtin_amdgcn_rcpf(gmm_exp_weights<D, KM>(mu, c, l2s, q, E));
  float acc[D];
  gmm_mix<D, KM>(mu, E, acc);
#pragma unroll
  for (int i = 0; i < D; ++i) g[i] = inv_s2 * fmaf(-acc[i], inv, q[i]);
}

// Accumulators of the analytic mu-adjoint, per lane: G[p][i] = sum cw_k x_i + ce_k e_i + cv_k v_i over
// the lane's samples and CW[p] = sum cw_k; the gradient is G_k - mu_k CW_k (gmm_adjoint_flat).
template <int D, int KM>
struct GmmAdjAcc {
  static constexpr int KP = KM / 2;
  f32x2 G[KP][D];
  f32x2 CW[KP];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      CW[p] = f32x2{0.f, 0.f};
#pragma unroll
      for (int i = 0; i < D; ++i) G[p][i] = f32x2{0.f, 0.f};
    }
  }
};

// One sample (x, v) of the KFP residual for the GMM model V_theta = -logsumexp_k(-|x-mu_k|^2/(2 s^2))
// (kinetic_fokker_planck.py:33-50 per sample, …_GMM.py:214-234): returns grad V_theta = s2 (x - mbar) in g,
// T1 = |g|^2, T2 = v^T Hess V_theta v, T3 = g . v, and adds the analytic adjoint of c1 T1 + c2 T2 + c3 T3
// with respect to mu (softmax chain rule; derivation and FD check: oracle/numpy_ref.py
// kfp_gmm_grad_analytic) to `acc`. With w the softmax weights, p_k = mu_k . v, e = x - mbar,
// em_k = e . mu_k, pbar = sum w p, A1 = -2 c1 s^4, A2 = -c2 s^4, A3 = -c3 s^2, B = A3 - 2 A2 pbar:
//   F_k = A1 em_k + p_k (A2 p_k + B),   Fbar = sum w F,
//   d/d mu_k = cw_k (x - mu_k) + ce_k e + cv_k v,  cw = w s2 (F - Fbar), ce = A1 w, cv = w (2 A2 p_k + B).
// Shared by the standalone residual (residual.hip kfp_gmm_kernel) and the simulator-fused one (sde.hip).
template <int D, int KM>
__device__ __forceinline__ void gmm_residual_sample(const f32x2 (*mu)[D], const f32x2* c, float s2, float l2s,
                                                    const float* x, const float* v, float c1, float c2, float c3,
                                                    GmmAdjAcc<D, KM>& acc, float* g, float& T1, float& T2,
                                                    float& T3) {
  constexpr int KP = KM / 2;
  f32x2 W[KP];
  const float inv = __builtin_amdgcn_rcpf(gmm_exp_weights<D, KM>(mu, c, l2s, x, W));
#pragma unroll
  for (int p = 0; p < KP; ++p) W[p] *= bc2(inv);
  float e[D];
  gmm_mix<D, KM>(mu, W, e);
#pragma unroll
  for (int i = 0; i < D; ++i) {
    e[i] = x[i] - e[i];
    g[i] = s2 * e[i];
  }
  const float ee = dotd<D>(e, e), ev = dotd<D>(e, v), vv = dotd<D>(v, v);
  T1 = s2 * s2 * ee;
  T3 = s2 * ev;
  f32x2 PK[KP], EM[KP];
  f32x2 pb = {0.f, 0.f}, wq = {0.f, 0.f};
#pragma unroll
  for (int p = 0; p < KP; ++p) {
    PK[p] = bc2(v[0]) * mu[p][0];
    EM[p] = bc2(e[0]) * mu[p][0];
  }
#pragma unroll
  for (int i = 1; i < D; ++i)  // coordinate-outer (independent packed FMAs back to back, same per-chain order)
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      PK[p] = bc2(v[i]) * mu[p][i] + PK[p];
      EM[p] = bc2(e[i]) * mu[p][i] + EM[p];
    }
#pragma unroll
  for (int p = 0; p < KP; ++p) {
    const f32x2 wp = W[p] * PK[p];
    pb += wp;
    wq = wp * PK[p] + wq;
  }
  const float pbar = pb[0] + pb[1], wp2 = wq[0] + wq[1];
  const float s4 = s2 * s2;
  T2 = s2 * vv - s4 * (wp2 - pbar * pbar);  // v^T (I/s^2 - Cov_w(mu)/s^4) v
  const float A1 = -2.f * c1 * s4, A2 = -c2 * s4, A3 = -c3 * s2;
  const float B = fmaf(-2.f * A2, pbar, A3);
  f32x2 F[KP], fb = {0.f, 0.f};
#pragma unroll
  for (int p = 0; p < KP; ++p) {
    F[p] = bc2(A1) * EM[p] + PK[p] * (bc2(A2) * PK[p] + bc2(B));
    fb = W[p] * F[p] + fb;
  }
  const float nsF = -s2 * (fb[0] + fb[1]);
  f32x2 cw[KP], ce[KP], cv[KP];
#pragma unroll
  for (int p = 0; p < KP; ++p) {
    cw[p] = W[p] * (bc2(s2) * F[p] + bc2(nsF));
    ce[p] = bc2(A1) * W[p];
    cv[p] = W[p] * (bc2(2.f * A2) * PK[p] + bc2(B));
    acc.CW[p] += cw[p];
  }
  // G += cw x, then + ce e, then + cv v (the same rounding order per entry as one cv v + (ce e + (cw x + G))),
  // term-outer so that consecutive packed FMAs are independent
#pragma unroll
  for (int p = 0; p < KP; ++p)
#pragma unroll
    for (int i = 0; i < D; ++i) acc.G[p][i] = cw[p] * bc2(x[i]) + acc.G[p][i];
#pragma unroll
  for (int p = 0; p < KP; ++p)
#pragma unroll
    for (int i = 0; i < D; ++i) acc.G[p][i] = ce[p] * bc2(e[i]) + acc.G[p][i];
#pragma unroll
  for (int p = 0; p < KP; ++p)
#pragma unroll
    for (int i = 0; i < D; ++i) acc.G[p][i] = cv[p] * bc2(v[i]) + acc.G[p][i];
}

// the lane's mu-gradient in the reference parameter order (k * D + i): G_k - mu_k CW_k
template <int D, int KM>
__device__ __forceinline__ void gmm_adjoint_flat(const GmmAdjAcc<D, KM>& acc, const f32x2 (*mu)[D], float* out) {
#pragma unroll
  for (int k = 0; k < KM; ++k)
#pragma unroll
    for (int i = 0; i < D; ++i) out[k * D + i] = fmaf(-mu[k / 2][i][k % 2], acc.CW[k / 2][k % 2], acc.G[k / 2][i][k % 2]);
}

// V_hypothesis parameters zero-padded to wider compiled shapes (exact: a padded hidden unit has zero
// incoming and outgoing weights, z = 0, h = tanh 0 = 0, so it changes no output and no real gradient).
constexpr int kMlpPadMaxL = 16;
// Padded <-> real flat parameter index (flax order: per layer kernel [in, out] then bias [out]).
struct MlpPadMap {
  int L;
  int din[kMlpPadMaxL + 1], dout[kMlpPadMaxL + 1];     // real dims of layer l
  int pin[kMlpPadMaxL + 1], pout[kMlpPadMaxL + 1];     // padded dims
  int64_t roff[kMlpPadMaxL + 1], poff[kMlpPadMaxL + 1];  // kernel offsets (real / padded); bias follows the kernel
  __host__ __device__ int64_t real_of(int64_t q) const {  // padded index -> real index or -1
    for (int l = 0; l <= L; ++l) {
      const int64_t kb = poff[l], bb = kb + (int64_t)pin[l] * pout[l], be = bb + pout[l];
      if (q < kb || q >= be) continue;
      if (q >= bb) {
        const int n = (int)(q - bb);
        return n < dout[l] ? roff[l] + (int64_t)din[l] * dout[l] + n : -1;
      }
      const int m = (int)((q - kb) / pout[l]), n = (int)((q - kb) % pout[l]);
      return (m < din[l] && n < dout[l]) ? roff[l] + (int64_t)m * dout[l] + n : -1;
    }
    return -1;
  }
};


// fp64 column reducer launched after any kernel that wrote a partial slab.
void launch_slab_reduce(const float* partials, int n_blocks, int n_cols, double* out,
                        hipStream_t stream);

inline int grid_for(int64_t n, int64_t per_block = kBlock) {
  return (int)((n + per_block - 1) / per_block);
}

}  // namespace pdeinv
