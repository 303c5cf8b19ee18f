// common.h — device helpers shared by the pdeinv HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/pdeinv.h"

namespace pdeinv {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kBlock = 256;          // 4 waves of 64
constexpr int kWave = 64;
constexpr int kWavesPerBlock = kBlock / kWave;

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

// out[i] += s * a[i] (packed pairs for even d)
template <int D>
__device__ __forceinline__ void axpyd(float s, const float* a, float* out) {
  if constexpr (D % 2 == 0) {
#pragma unroll
    for (int p = 0; p < D / 2; ++p) {
      const f32x2 r = f32x2{s, s} * f32x2{a[2 * p], a[2 * p + 1]} + f32x2{out[2 * p], out[2 * p + 1]};
      out[2 * p] = r[0];
      out[2 * p + 1] = r[1];
    }
  } else {
#pragma unroll
    for (int i = 0; i < D; ++i) out[i] = fmaf(s, a[i], out[i]);
  }
}

template <int D, int KM>
__device__ __forceinline__ void gmm_softmax(const float* x, const float (*mu)[D], const float* nh, float l2s,
                                            float* w, float* mbar, float* t) {
  // unused centre slots carry nh = -inf: weight exactly 0, no per-centre branches
  float amax = -INFINITY;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    t[k] = dotd<D>(x, mu[k]);
    w[k] = (t[k] + nh[k]) * l2s;
    amax = fmaxf(amax, w[k]);
  }
  float den = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    w[k] = __builtin_amdgcn_exp2f(w[k] - amax);
    den += w[k];
  }
  const float inv = __builtin_amdgcn_rcpf(den);
#pragma unroll
  for (int i = 0; i < D; ++i) mbar[i] = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    w[k] *= inv;
    axpyd<D>(w[k], mu[k], mbar);
  }
}

// One sample (x, v) of the KFP residual for the GMM model V_theta = -logsumexp_k(-|x-mu_k|^2/(2 s^2))
// (kinetic_fokker_planck.py:33-50 per sample, …_GMM.py:214-234): returns grad V_theta = s2 (x - mbar) in g,
// T1 = |g|^2, T2 = v^T Hess V_theta v, T3 = g . v, and adds the analytic adjoint of
// c1 T1 + c2 T2 + c3 T3 with respect to mu (softmax chain rule; derivation and FD check:
// oracle/numpy_ref.py kfp_gmm_grad_analytic) to gacc[K*D]. Shared by the standalone residual
// (residual.hip kfp_gmm_kernel) and the simulator-fused one (sde.hip). The d-vector work runs on
// packed pairs for even d; the per-centre scalars are folded so that each costs one or two FMAs.
template <int D, int KM>
__device__ __forceinline__ void gmm_residual_sample(const float (*mu)[D], const float* nh, float s2, float l2s,
                                                    const float* x, const float* v, float c1, float c2, float c3,
                                                    float* gacc, float* g, float& T1, float& T2, float& T3) {
  float w[KM], mbar[D], xm[KM];
  gmm_softmax<D, KM>(x, mu, nh, l2s, w, mbar, xm);
  float e[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    e[i] = x[i] - mbar[i];
    g[i] = s2 * e[i];
  }
  const float ee = dotd<D>(e, e), ev = dotd<D>(e, v), vv = dotd<D>(v, v);
  T1 = s2 * s2 * ee;
  T3 = s2 * ev;
  float pk[KM], em[KM], pbar = 0.f, wp2 = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    pk[k] = dotd<D>(mu[k], v);
    em[k] = dotd<D>(e, mu[k]);  // e.mu_k
    pbar = fmaf(w[k], pk[k], pbar);
    wp2 = fmaf(w[k] * pk[k], pk[k], wp2);
  }
  const float s4 = s2 * s2;
  T2 = s2 * vv - s4 * (wp2 - pbar * pbar);  // v^T (I/s^2 - Cov_w(mu)/s^4) v
  // adjoint: F_k = d f / d w_k = A1 em_k + pk_k (A2 (pk_k - 2 pbar) + A3), then the softmax chain rule
  const float A1 = -2.f * c1 * s4, A2 = -c2 * s4, A3 = -c3 * s2;
  float Fk[KM], Fbar = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    Fk[k] = fmaf(A1, em[k], pk[k] * fmaf(A2, pk[k] - 2.f * pbar, A3));
    Fbar = fmaf(w[k], Fk[k], Fbar);
  }
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    // cw (x - mu_k) + ce e + cv v with cw = w (F_k - Fbar) s2, ce = A1 w, cv = w (2 A2 (pk_k - pbar) + A3)
    const float cw = w[k] * s2 * (Fk[k] - Fbar);
    const float ce = A1 * w[k];
    const float cv = w[k] * fmaf(2.f * A2, pk[k] - pbar, A3);
    float* gk = gacc + k * D;
    if constexpr (D % 2 == 0) {
#pragma unroll
      for (int p = 0; p < D / 2; ++p) {
        const f32x2 xp = f32x2{x[2 * p], x[2 * p + 1]}, mp = f32x2{mu[k][2 * p], mu[k][2 * p + 1]};
        f32x2 r = f32x2{gk[2 * p], gk[2 * p + 1]};
        r = f32x2{cw, cw} * (xp - mp) + r;
        r = f32x2{ce, ce} * f32x2{e[2 * p], e[2 * p + 1]} + r;
        r = f32x2{cv, cv} * f32x2{v[2 * p], v[2 * p + 1]} + r;
        gk[2 * p] = r[0];
        gk[2 * p + 1] = r[1];
      }
    } else {
#pragma unroll
      for (int i = 0; i < D; ++i) gk[i] += cw * (x[i] - mu[k][i]) + ce * e[i] + cv * v[i];
    }
  }
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
