// realnvp.hip — time-conditioned RealNVP log-density (core/normalizing_flow.py:8-229).
// One thread per (t, x) sample; all tiny MLPs (widths 8 / 16 / 16) run in
// VGPRs on the VALU. The weights are read at wave-uniform addresses (scalar loads, one fetch
// serves the 64 samples of a wave); masks and the base Gaussian travel in the kernel arguments.
#include <math.h>

#include "common.h"

namespace pdeinv {

struct NvpArgs {
  int n_layers, E, in_dim, ignore_time, act;
  float soft_init, log_det;
  float mean[8], inv_cov[64];
  float masks[PDEINV_REALNVP_MAX_LAYERS * 8];
};

__device__ __forceinline__ float nvp_act(int act, float x) {
  switch (act) {
    case PDEINV_ACT_CELU: return x > 0.f ? x : expm1f(x);  // jax.nn.celu, alpha = 1
    case PDEINV_ACT_RELU: return fmaxf(x, 0.f);
    case PDEINV_ACT_TANH: return tanhf(x);
    case PDEINV_ACT_ELU: return x > 0.f ? x : expm1f(x);
    case PDEINV_ACT_SILU: return x / (1.f + expf(-x));
    case PDEINV_ACT_SOFTPLUS: return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x)));
    default: {  // gelu, tanh approximation
      const float c = 0.7978845608028654f;  // sqrt(2 / pi)
      return 0.5f * x * (1.f + tanhf(c * (x + 0.044715f * x * x * x)));
    }
  }
}

// y[out] = act?(b + in @ W), W [n_in x n_out] row-major at p, b right after it.
template <int NI, int NO>
__device__ __forceinline__ const float* dense(const float* __restrict__ p, const float (&in)[NI], int n_in,
                                              float (&out)[NO], int act, bool apply_act) {
  const float* b = p + n_in * NO;
#pragma unroll
  for (int o = 0; o < NO; ++o) out[o] = b[o];
  for (int i = 0; i < n_in; ++i) {
    const float v = in[i];
#pragma unroll
    for (int o = 0; o < NO; ++o) out[o] = fmaf(v, p[i * NO + o], out[o]);
  }
  if (apply_act) {
#pragma unroll
    for (int o = 0; o < NO; ++o) out[o] = nvp_act(act, out[o]);
  }
  return b + NO;
}

template <int D>
__device__ __forceinline__ const float* basic_mlp(const float* p, const float (&in)[D + 16], int n_in, int act,
                                                  float (&out)[D]) {
  float h0[8], h1[16], h2[16];
  p = dense<D + 16, 8>(p, in, n_in, h0, act, true);
  p = dense<8, 16>(p, h0, 8, h1, act, true);
  p = dense<16, 16>(p, h1, 16, h2, act, true);
  return dense<16, D>(p, h2, 16, out, act, false);
}

template <int D>
__global__ __launch_bounds__(kBlock) void realnvp_logdensity_kernel(NvpArgs a, const float* __restrict__ params,
                                                                    const float* __restrict__ tv, int64_t t_stride,
                                                                    const float* __restrict__ xv, int64_t n,
                                                                    int64_t ld, int64_t layer_stride,
                                                                    float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float t = tv[i * t_stride];
  float x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = xv[i * ld + k];
  // time embedding (shared by every coupling layer)
  float temb[16];
  const float* p = params;
  if (!a.ignore_time) {
    if (a.E > 0) {
      const int half = a.E / 2;
      const float step = logf(10000.f) / (float)(half - 1);
      float se[16], h[16];
      for (int k = 0; k < half; ++k) {
        const float e = t * expf(-step * (float)k);
        se[k] = sinf(e);
        se[half + k] = cosf(e);
      }
      // two E x E dense layers (runtime E <= 16)
      for (int o = 0; o < a.E; ++o) h[o] = p[a.E * a.E + o];
      for (int q = 0; q < a.E; ++q)
        for (int o = 0; o < a.E; ++o) h[o] = fmaf(se[q], p[q * a.E + o], h[o]);
      for (int o = 0; o < a.E; ++o) h[o] = nvp_act(a.act, h[o]);
      p += a.E * a.E + a.E;
      for (int o = 0; o < a.E; ++o) temb[o] = p[a.E * a.E + o];
      for (int q = 0; q < a.E; ++q)
        for (int o = 0; o < a.E; ++o) temb[o] = fmaf(h[q], p[q * a.E + o], temb[o]);
      p += a.E * a.E + a.E;
    } else {
      temb[0] = t;
    }
  }
  const float* layers = p;
  float ldj = 0.f;
  for (int l = a.n_layers - 1; l >= 0; --l) {  // likelihood direction: reversed layers
    const float* lp = layers + (int64_t)l * layer_stride;
    const float* m = a.masks + l * D;
    float in[D + 16];
#pragma unroll
    for (int k = 0; k < D; ++k) in[k] = x[k] * m[k];
    const int n_t = a.in_dim - D;
    for (int q = 0; q < n_t; ++q) in[D + q] = temb[q];
    float s[D], tr[D];
    const float* sfp = lp;
    const float* q = basic_mlp<D>(lp + D, in, a.in_dim, a.act, s);
    basic_mlp<D>(q, in, a.in_dim, a.act, tr);
    const bool hard = !a.ignore_time && a.soft_init == 0.f;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      float sk = hard ? t * s[k] : s[k];
      float tk = hard ? t * tr[k] : tr[k];
      const float sf = expf(sfp[k]);
      sk = tanhf(sk / sf) * sf;
      sk *= 1.f - m[k];
      tk *= 1.f - m[k];
      x[k] = (x[k] + tk) * expf(sk);
      ldj += sk;
    }
  }
  float quad = 0.f;
#pragma unroll
  for (int r = 0; r < D; ++r) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) acc = fmaf(a.inv_cov[r * D + c], x[c] - a.mean[c], acc);
    quad = fmaf(x[r] - a.mean[r], acc, quad);
  }
  out[i] = -0.5f * (a.log_det + quad) + ldj;
}


// ---------------------------------------------------------------------------------------------
// Value and parameter gradient of the maximum-likelihood loss (log_density_estimation.py:47-58):
// loss = -mean_i log p_{t_i}(x_i), replacing jax.value_and_grad(loss_fn). One thread per sample,
// one 256-sample tile per block.
// * The backward pass walks the coupling layers in the opposite order of the likelihood pass and
//   rebuilds each layer's input from its output by inverting the layer (x_in = x_out e^{-s} - tr;
//   the masked coordinates, which feed s and tr, pass through unchanged and exact): no per-layer
//   state is stored.
// * Parameters are staged in LDS in a zero-padded canonical layout (x rows padded to DM, time rows
//   to 16, output columns to DM, the time embedding to 16 x 16), so every per-sample loop has
//   compile-time trip counts and no predicates: padded inputs are 0 and meet zero weights. Every
//   lane reads the same weight (a broadcast ds_read).
// * Each dense layer's weight gradient sum_samples a_i delta_o is formed per tile in LDS (rows of
//   a and delta staged; items = (row i, 4 outputs) x sample slices; fixed-order slice combine)
//   and written to the tile's row of a [tiles x (P + 1)] slab (column P = sum log p). A
//   fixed-order fp64 column reduce (chunked over at most kNvpMaxRows tiles) gives
//   grad = -1/n sum. No float atomics: bit-reproducible run to run.
// Compiled for DM in {2, 4, 8} with the runtime dim d <= DM (padded coordinates are x = 0,
// mask = 1, so they never move) and for the celu / elu activation (the flow of
// log_density_estimation.py:103-114).
// ---------------------------------------------------------------------------------------------
constexpr int kNvpAst = 25;        // LDS row stride of a (<= 8 + 16 values; odd: conflict-free row writes)
constexpr int kNvpGst = 17;        // LDS row stride of delta (<= 16 values)
constexpr int kNvpMaxRows = 2048;  // tiles per slab chunk

// Activation derivative from the post-activation value h.
template <int ACT>
__device__ __forceinline__ float nvp_act_grad_h(float h) {
  static_assert(ACT != PDEINV_ACT_SILU && ACT != PDEINV_ACT_GELU, "derivative needs the pre-activation");
  if (ACT == PDEINV_ACT_CELU || ACT == PDEINV_ACT_ELU) return h > 0.f ? 1.f : h + 1.f;  // e^z = h + 1
  if (ACT == PDEINV_ACT_RELU) return h > 0.f ? 1.f : 0.f;
  if (ACT == PDEINV_ACT_TANH) return 1.f - h * h;
  return 1.f - expf(-h);  // softplus: sigmoid(z) = 1 - e^{-h}
}

// Canonical (padded) LDS layout of one BasicMLP and one coupling layer.
template <int DM>
struct NvpCanon {
  static constexpr int W0x = 0, W0t = DM * 8, B0 = W0t + 16 * 8, W1 = B0 + 8, B1 = W1 + 8 * 16, W2 = B1 + 16,
                       B2 = W2 + 16 * 16, W3 = B2 + 16, B3 = W3 + 16 * DM, MLP = B3 + DM;
  static constexpr int SF = 0, SNET = DM, TNET = DM + MLP, LAYER = DM + 2 * MLP;
};
constexpr int kTembCanon = 2 * (16 * 16 + 16);  // W1 [16x16], b1, W2 [16x16], b2

struct NvpLds {
  float a[kBlock * kNvpAst];
  float g[kBlock * kNvpGst];
  float part[kBlock * 4];
};

// row[off + r * n_out + o] = sum over the tile of a_r * g_o (r < n_in) and of g_o (the bias row
// r = n_in). The caller has written its a row (L.a) after a barrier. All threads call.
template <int NO>
__device__ __forceinline__ void nvp_wgrad(NvpLds& L, const float (&g)[NO], int n_in, int n_out,
                                          float* __restrict__ row, int64_t off) {
  // Opaque copies: without them LICM hoists every call site's per-lane item / slice / address
  // math out of the layer loop and keeps it live across the whole kernel (> 1 KB of spills).
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  asm volatile("" : "+s"(n_in), "+s"(n_out));
#pragma unroll
  for (int o = 0; o < NO; ++o) L.g[tid * kNvpGst + o] = g[o];  // columns >= n_out are never stored
  __syncthreads();
  const int og_n = (n_out + 3) >> 2;
  const int items = (n_in + 1) * og_n;
  int S = 1;
  while (S < 8 && 2 * S * items <= kBlock) S *= 2;
  const int span = kBlock / S;
  const int slice = tid / items, item = tid - slice * items;
  const int r = item / og_n, o0 = (item - r * og_n) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (slice < S) {
    const int s0 = slice * span;
    for (int s = s0; s < s0 + span; ++s) {
      const float av = r < n_in ? L.a[s * kNvpAst + r] : 1.f;
      const float* gs = L.g + s * kNvpGst + o0;
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = fmaf(av, gs[c], acc[c]);
    }
  }
  if (S > 1) {
    if (slice < S) {
#pragma unroll
      for (int c = 0; c < 4; ++c) L.part[(slice * items + item) * 4 + c] = acc[c];
    }
    __syncthreads();
    if (tid < items) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float v = 0.f;
        for (int q = 0; q < S; ++q) v += L.part[(q * items + tid) * 4 + c];
        acc[c] = v;
      }
    }
  }
  if (tid < items) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (o0 + c < n_out) row[off + r * n_out + o0 + c] = acc[c];
  }
}

template <int NA>
__device__ __forceinline__ void nvp_put_a(NvpLds& L, const float (&av)[NA]) {
#pragma unroll
  for (int i = 0; i < NA; ++i) L.a[threadIdx.x * kNvpAst + i] = av[i];  // slots >= n_in are never read
}

// Keeps the scheduler from hoisting whole weight matrices' LDS loads into VGPRs ahead of use
// (without it the kernel spills > 1 KB per lane).
#define NVP_ROW_FENCE() __builtin_amdgcn_sched_barrier(0)

// BasicMLP (:97-111) forward on the canonical layout; keeps the post-activations.
template <int DM, int ACT>
__device__ __forceinline__ void nvp_mlp_fwd(const float* __restrict__ p, const float (&xm)[DM],
                                            const float (&temb)[16], float (&h0)[8], float (&h1)[16],
                                            float (&h2)[16], float (&out)[DM]) {
  using C = NvpCanon<DM>;
#pragma unroll
  for (int o = 0; o < 8; ++o) h0[o] = p[C::B0 + o];
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < 8; ++o) h0[o] = fmaf(xm[k], p[C::W0x + k * 8 + o], h0[o]);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < 8; ++o) h0[o] = fmaf(temb[q], p[C::W0t + q * 8 + o], h0[o]);
  }
#pragma unroll
  for (int o = 0; o < 8; ++o) h0[o] = nvp_act(ACT, h0[o]);
#pragma unroll
  for (int o = 0; o < 16; ++o) h1[o] = p[C::B1 + o];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < 16; ++o) h1[o] = fmaf(h0[i], p[C::W1 + i * 16 + o], h1[o]);
  }
#pragma unroll
  for (int o = 0; o < 16; ++o) h1[o] = nvp_act(ACT, h1[o]);
#pragma unroll
  for (int o = 0; o < 16; ++o) h2[o] = p[C::B2 + o];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < 16; ++o) h2[o] = fmaf(h1[i], p[C::W2 + i * 16 + o], h2[o]);
  }
#pragma unroll
  for (int o = 0; o < 16; ++o) h2[o] = nvp_act(ACT, h2[o]);
#pragma unroll
  for (int o = 0; o < DM; ++o) out[o] = p[C::B3 + o];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < DM; ++o) out[o] = fmaf(h2[j], p[C::W3 + j * DM + o], out[o]);
  }
}

// BasicMLP backward: weight gradients into the tile's slab row at `off` (the net's first float
// in the reference layout; n_in = d + n_t), input gradients added into gxm / gtemb.
template <int DM, int ACT>
__device__ __forceinline__ void nvp_mlp_bwd(NvpLds& L, const float* __restrict__ p, int64_t off, int d, int n_t,
                                            const float (&xm)[DM], const float (&temb)[16], const float (&h0)[8],
                                            const float (&h1)[16], const float (&h2)[16], const float (&dout)[DM],
                                            float (&gxm)[DM], float (&gtemb)[16], float* __restrict__ row) {
  using C = NvpCanon<DM>;
  const int n_in = d + n_t;
  const int64_t o1 = (int64_t)n_in * 8 + 8, o2 = o1 + 8 * 16 + 16, o3 = o2 + 16 * 16 + 16;
  __syncthreads();
  nvp_put_a(L, h2);
  nvp_wgrad(L, dout, 16, d, row, off + o3);
  float d2[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    NVP_ROW_FENCE();
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < DM; ++o) s = fmaf(p[C::W3 + j * DM + o], dout[o], s);
    d2[j] = s * nvp_act_grad_h<ACT>(h2[j]);
  }
  __syncthreads();
  nvp_put_a(L, h1);
  nvp_wgrad(L, d2, 16, 16, row, off + o2);
  float d1[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    NVP_ROW_FENCE();
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < 16; ++o) s = fmaf(p[C::W2 + j * 16 + o], d2[o], s);
    d1[j] = s * nvp_act_grad_h<ACT>(h1[j]);
  }
  __syncthreads();
  nvp_put_a(L, h0);
  nvp_wgrad(L, d1, 8, 16, row, off + o1);
  float d0[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    NVP_ROW_FENCE();
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < 16; ++o) s = fmaf(p[C::W1 + j * 16 + o], d1[o], s);
    d0[j] = s * nvp_act_grad_h<ACT>(h0[j]);
  }
  __syncthreads();
  nvp_put_a(L, xm);  // reference row order: x rows 0..d-1, then the time rows
#pragma unroll
  for (int q = 0; q < 16; ++q) L.a[threadIdx.x * kNvpAst + d + q] = temb[q];
  nvp_wgrad(L, d0, n_in, 8, row, off);
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < 8; ++o) gxm[k] = fmaf(p[C::W0x + k * 8 + o], d0[o], gxm[k]);  // padded rows are 0
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < 8; ++o) gtemb[q] = fmaf(p[C::W0t + q * 8 + o], d0[o], gtemb[q]);
  }
}

// TimeEmbedding (:8-22) on the padded 16 x 16 copy: se = SinusoidalEmbedding(t) (:24-38) from the
// per-slot (frequency, is_sin) table (0 past E), he = act(se W1 + b1), temb = he W2 + b2.
template <int ACT>
__device__ __forceinline__ void nvp_time_embed(const float* __restrict__ tw, const float* __restrict__ freq,
                                               float t, float (&se)[16], float (&he)[16], float (&temb)[16]) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float e = t * freq[q];
    se[q] = freq[16 + q] * sinf(e) + freq[32 + q] * cosf(e);
  }
#pragma unroll
  for (int o = 0; o < 16; ++o) he[o] = tw[256 + o];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < 16; ++o) he[o] = fmaf(se[q], tw[q * 16 + o], he[o]);
  }
#pragma unroll
  for (int o = 0; o < 16; ++o) he[o] = nvp_act(ACT, he[o]);  // padded: act(0) = 0 (celu / elu)
#pragma unroll
  for (int o = 0; o < 16; ++o) temb[o] = tw[272 + 256 + o];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    NVP_ROW_FENCE();
#pragma unroll
    for (int o = 0; o < 16; ++o) temb[o] = fmaf(he[q], tw[272 + q * 16 + o], temb[o]);
  }
}

template <int DM, int ACT>
__global__ __launch_bounds__(kBlock) void realnvp_grad_kernel(NvpArgs a, int d, const float* __restrict__ params,
                                                              const float* __restrict__ tv, int64_t t_stride,
                                                              const float* __restrict__ xv, int64_t n, int64_t ld,
                                                              int64_t layer_stride, int64_t n_params,
                                                              int64_t tile0, float* __restrict__ slab,
                                                              int64_t slab_ld) {
  using C = NvpCanon<DM>;
  __shared__ NvpLds L;
  __shared__ float sW[C::LAYER];   // current coupling layer, canonical layout
  __shared__ float sT[kTembCanon];  // time embedding, canonical layout
  __shared__ float sF[48];          // sinusoid table: frequency, sin weight, cos weight (0 past E)
  __shared__ float sM[PDEINV_REALNVP_MAX_LAYERS * DM];  // masks, padded with 1
  __shared__ float sB[DM + DM * DM];                     // base mean, inverse covariance (0-padded)
  const int E = a.E;
  const int n_in = a.in_dim, n_t = n_in - d;
  const int mlp_n = n_in * 8 + 8 + 8 * 16 + 16 + 16 * 16 + 16 + 16 * d + d;
  const int64_t temb_params = E > 0 ? 2 * ((int64_t)E * E + E) : 0;
  const float* layers = params + temb_params;
  const bool hard = !a.ignore_time && a.soft_init == 0.f;
  const int tid = threadIdx.x;
  // ---- per-block staging of the small tables ----
  for (int q = tid; q < kTembCanon; q += kBlock) {
    const int part = q / 272, r = q - part * 272;  // [W (16x16) | b (16)] x 2
    float v = 0.f;
    if (E > 0) {
      const float* src = params + part * (E * E + E);
      if (r < 256) {
        const int i = r / 16, o = r % 16;
        v = (i < E && o < E) ? src[i * E + o] : 0.f;
      } else {
        v = (r - 256 < E) ? src[E * E + (r - 256)] : 0.f;
      }
    }
    sT[q] = v;
  }
  if (tid < 16) {
    const int half = E / 2;
    const bool on = E > 0 && tid < E;
    const bool is_sin = tid < half;
    const float step = E > 0 ? logf(10000.f) / (float)(half - 1) : 0.f;
    sF[tid] = on ? expf(-step * (float)(is_sin ? tid : tid - half)) : 0.f;
    sF[16 + tid] = on && is_sin ? 1.f : 0.f;
    sF[32 + tid] = on && !is_sin ? 1.f : 0.f;
  }
  for (int q = tid; q < a.n_layers * DM; q += kBlock) {
    const int l = q / DM, k = q % DM;
    sM[q] = k < d ? a.masks[l * d + k] : 1.f;
  }
  for (int q = tid; q < DM + DM * DM; q += kBlock) {
    float v = 0.f;
    if (q < DM) {
      v = q < d ? a.mean[q] : 0.f;
    } else {
      const int r = (q - DM) / DM, c = (q - DM) % DM;
      v = (r < d && c < d) ? a.inv_cov[r * d + c] : 0.f;
    }
    sB[q] = v;
  }
  // Stage layer l in the canonical layout (zero padding).
  auto stage = [&](int l) {
    __syncthreads();
    const float* lp = layers + (int64_t)l * layer_stride;
    for (int q = tid; q < C::LAYER; q += kBlock) {
      float v = 0.f;
      if (q < DM) {
        v = q < d ? lp[q] : 0.f;
      } else {
        const int net = (q - DM) / C::MLP, r = (q - DM) - net * C::MLP;
        const float* np = lp + d + net * mlp_n;
        if (r < C::W0t) {
          const int k = r / 8, o = r % 8;
          v = k < d ? np[k * 8 + o] : 0.f;
        } else if (r < C::B0) {
          const int qq = (r - C::W0t) / 8, o = (r - C::W0t) % 8;
          v = qq < n_t ? np[(d + qq) * 8 + o] : 0.f;
        } else if (r < C::W3) {  // b0, W1, b1, W2, b2: same order and size as the reference
          v = np[n_in * 8 + (r - C::B0)];
        } else if (r < C::B3) {
          const int j = (r - C::W3) / DM, o = (r - C::W3) % DM;
          v = o < d ? np[n_in * 8 + (C::W3 - C::B0) + j * d + o] : 0.f;
        } else {
          const int o = r - C::B3;
          v = o < d ? np[n_in * 8 + (C::W3 - C::B0) + 16 * d + o] : 0.f;
        }
      }
      sW[q] = v;
    }
    __syncthreads();
  };
  float* row = slab + (int64_t)blockIdx.x * slab_ld;
  const int64_t i = (tile0 + blockIdx.x) * kBlock + tid;
  const bool active = i < n;
  const float w = active ? 1.f : 0.f;
  const float t = active ? tv[i * t_stride] : 0.f;
  float x[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) x[k] = (active && k < d) ? xv[i * ld + k] : 0.f;
  __syncthreads();
  float temb[16];
  {
    float se[16], he[16];
    nvp_time_embed<ACT>(sT, sF, t, se, he, temb);
    if (E == 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) temb[q] = 0.f;
      if (!a.ignore_time) temb[0] = t;  // the raw time appended (CouplingLayer :137)
    }
  }
  // ---- likelihood pass (layers L-1 .. 0): x <- (x + tr) e^s ----
  float ldj = 0.f;
  for (int l = a.n_layers - 1; l >= 0; --l) {
    stage(l);
    float m[DM], xm[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      m[k] = sM[l * DM + k];
      xm[k] = x[k] * m[k];
    }
    float h0[8], h1[16], h2[16], so[DM], to[DM];
    nvp_mlp_fwd<DM, ACT>(sW + C::SNET, xm, temb, h0, h1, h2, so);
    nvp_mlp_fwd<DM, ACT>(sW + C::TNET, xm, temb, h0, h1, h2, to);
#pragma unroll
    for (int k = 0; k < DM; ++k) {  // padded k: keep = 0, so x stays 0 and ldj is unchanged
      const float keep = 1.f - m[k];
      const float sf = expf(sW[C::SF + k]);
      const float sk = tanhf((hard ? t * so[k] : so[k]) / sf) * sf * keep;
      x[k] = (x[k] + (hard ? t * to[k] : to[k]) * keep) * expf(sk);
      ldj += sk;
    }
  }
  // ---- base density log p0(x0) and its gradient ----
  float gx[DM], diff[DM], quad = 0.f;
#pragma unroll
  for (int c = 0; c < DM; ++c) diff[c] = x[c] - sB[c];  // padded: 0 - 0
#pragma unroll
  for (int r = 0; r < DM; ++r) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < DM; ++c) acc = fmaf(sB[DM + r * DM + c], diff[c], acc);
    quad = fmaf(diff[r], acc, quad);
    gx[r] = -w * acc;
  }
  const float logp = -0.5f * (a.log_det + quad) + ldj;
  // ---- backward through layers 0 .. L-1, rebuilding each layer's input ----
  float gtemb[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) gtemb[q] = 0.f;
  for (int l = 0; l < a.n_layers; ++l) {
    stage(l);
    const int64_t loff = temb_params + (int64_t)l * layer_stride;
    float m[DM], xm[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      m[k] = sM[l * DM + k];
      xm[k] = x[k] * m[k];
    }
    float h0[8], h1[16], h2[16], out[DM];
    nvp_mlp_fwd<DM, ACT>(sW + C::SNET, xm, temb, h0, h1, h2, out);
    float s[DM], es[DM], gso[DM], gto[DM], galpha[DM], gacc[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      const float keep = 1.f - m[k];
      const float spre = hard ? t * out[k] : out[k];
      const float sf = expf(sW[C::SF + k]);
      const float th = tanhf(spre / sf);
      s[k] = th * sf * keep;
      es[k] = expf(s[k]);
      const float gs = (gx[k] * x[k] + w) * keep;         // d(log p0 + ldj)/ds via x_out and ldj
      const float dth = 1.f - th * th;
      galpha[k] = gs * (th * sf - dth * spre);            // d/d scaling_factor (sf = e^alpha)
      gso[k] = (hard ? t : 1.f) * gs * dth;                // d/d scale_net output
      gto[k] = (hard ? t : 1.f) * gx[k] * es[k] * keep;  // d/d translate_net output
      gacc[k] = 0.f;
    }
    __syncthreads();
    nvp_wgrad(L, galpha, 0, d, row, loff);
    nvp_mlp_bwd<DM, ACT>(L, sW + C::SNET, loff + d, d, n_t, xm, temb, h0, h1, h2, gso, gacc, gtemb, row);
    nvp_mlp_fwd<DM, ACT>(sW + C::TNET, xm, temb, h0, h1, h2, out);
    nvp_mlp_bwd<DM, ACT>(L, sW + C::TNET, loff + d + mlp_n, d, n_t, xm, temb, h0, h1, h2, gto, gacc, gtemb, row);
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      const float tr = (hard ? t * out[k] : out[k]) * (1.f - m[k]);
      x[k] = x[k] * expf(-s[k]) - tr;
      gx[k] = gx[k] * es[k] + m[k] * gacc[k];
    }
  }
  // ---- time-embedding backward ----
  if (E > 0) {
    float se[16], he[16], temb2[16];
    nvp_time_embed<ACT>(sT, sF, t, se, he, temb2);
    __syncthreads();
    nvp_put_a(L, he);
    nvp_wgrad(L, gtemb, E, E, row, (int64_t)E * E + E);
    float gz[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float v = 0.f;
#pragma unroll
      for (int o = 0; o < 16; ++o) v = fmaf(sT[272 + q * 16 + o], gtemb[o], v);  // padded W2 is 0
      gz[q] = v * nvp_act_grad_h<ACT>(he[q]);
    }
    __syncthreads();
    nvp_put_a(L, se);
    nvp_wgrad(L, gz, E, E, row, 0);
  }
  float lw[1] = {w * logp};
  __syncthreads();
  nvp_wgrad(L, lw, 0, 1, row, n_params);
}

// acc[c] (+)= sum_r slab[r][c] over one chunk (fp64, fixed order: 4 row groups of a column, then
// the groups in order); on the last chunk grad[c] = scale * acc[c] (c < n_params), loss = ...[n_params].
__global__ __launch_bounds__(kBlock) void nvp_grad_reduce_kernel(const float* __restrict__ slab, int rows,
                                                                  int64_t ld, int64_t n_params, double* acc64,
                                                                  int first, int last, double scale,
                                                                  float* __restrict__ grad,
                                                                  float* __restrict__ loss) {
  __shared__ double part[kBlock];
  const int64_t c = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  double acc = 0.0;
  if (c <= n_params)
    for (int r = g; r < rows; r += 4) acc += (double)slab[(int64_t)r * ld + c];
  part[threadIdx.x] = acc;
  __syncthreads();
  if (g == 0 && c <= n_params) {
    double v = ((part[threadIdx.x] + part[threadIdx.x + 64]) + part[threadIdx.x + 128]) + part[threadIdx.x + 192];
    if (!first) v += acc64[c];
    acc64[c] = v;
    if (last) {
      if (c < n_params) grad[c] = (float)(scale * v);
      else *loss = (float)(scale * v);
    }
  }
}

static int64_t layer_params(int D, int in_dim) {
  const int64_t mlp = (int64_t)in_dim * 8 + 8 + 8 * 16 + 16 + 16 * 16 + 16 + 16 * D + D;
  return D + 2 * mlp;
}

static int in_dim_of(const pdeinv_realnvp_desc* d) {
  return d->ignore_time ? d->dim : d->dim + (d->embed_time_dim > 0 ? d->embed_time_dim : 1);
}

}  // namespace pdeinv

using namespace pdeinv;

extern "C" int64_t pdeinv_realnvp_param_count(const pdeinv_realnvp_desc* d) {
  if (!d || d->dim < 1 || d->dim > 8 || d->n_layers < 1 || d->embed_time_dim < 0) return -1;
  const int E = d->ignore_time ? 0 : d->embed_time_dim;
  return (E > 0 ? 2 * ((int64_t)E * E + E) : 0) + (int64_t)d->n_layers * layer_params(d->dim, in_dim_of(d));
}

extern "C" int pdeinv_realnvp_logdensity(const pdeinv_realnvp_desc* d, const float* params, const float* t,
                                         int64_t t_stride, const float* x, int64_t n, int64_t ld, float* out,
                                         void* stream) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "realnvp: null descriptor");
  PDEINV_REQUIRE(d->dim >= 1 && d->dim <= 8, PDEINV_ERR_UNSUPPORTED, "realnvp: dim must be in [1, 8]");
  PDEINV_REQUIRE(d->n_layers >= 1 && d->n_layers <= PDEINV_REALNVP_MAX_LAYERS, PDEINV_ERR_UNSUPPORTED,
                 "realnvp: 1 <= n_layers <= 64");
  PDEINV_REQUIRE(d->embed_time_dim >= 0 && d->embed_time_dim <= 16 && d->embed_time_dim % 2 == 0 &&
                     d->embed_time_dim != 2,
                 PDEINV_ERR_UNSUPPORTED, "realnvp: embed_time_dim must be 0 or even in [4, 16]");
  PDEINV_REQUIRE(d->activation >= PDEINV_ACT_CELU && d->activation <= PDEINV_ACT_GELU, PDEINV_ERR_UNSUPPORTED,
                 "realnvp: unknown activation");
  PDEINV_REQUIRE(d->masks && d->base_mean && d->base_inv_cov, PDEINV_ERR_INVALID, "realnvp: null host array");
  PDEINV_REQUIRE(n >= 0 && ld >= d->dim && t_stride >= 0, PDEINV_ERR_INVALID, "realnvp: bad sizes");
  if (n == 0) return PDEINV_OK;
  PDEINV_REQUIRE(params && t && x && out, PDEINV_ERR_INVALID, "realnvp: null device pointer");
  const int D = d->dim;
  NvpArgs a{};
  a.n_layers = d->n_layers;
  a.ignore_time = d->ignore_time ? 1 : 0;
  a.E = a.ignore_time ? 0 : d->embed_time_dim;
  a.in_dim = in_dim_of(d);
  a.act = d->activation;
  a.soft_init = d->soft_init;
  a.log_det = d->base_log_det;
  for (int k = 0; k < D; ++k) a.mean[k] = d->base_mean[k];
  for (int k = 0; k < D * D; ++k) a.inv_cov[k] = d->base_inv_cov[k];
  for (int k = 0; k < d->n_layers * D; ++k) a.masks[k] = d->masks[k];
  const int64_t ls = layer_params(D, a.in_dim);
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid_for(n));
  switch (D) {
#define CASE(DD) case DD: hipLaunchKernelGGL(realnvp_logdensity_kernel<DD>, g, dim3(kBlock), 0, st, a, params, t, t_stride, x, n, ld, ls, out); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
  }
  return check_launch("realnvp_logdensity_kernel");
}

static int64_t nvp_grad_rows(int64_t n) {
  const int64_t tiles = (n + kBlock - 1) / kBlock;
  return tiles < kNvpMaxRows ? tiles : kNvpMaxRows;
}

extern "C" int64_t pdeinv_realnvp_grad_workspace(const pdeinv_realnvp_desc* d, int64_t n) {
  const int64_t P = pdeinv_realnvp_param_count(d);
  if (P < 0 || n < 0) return -1;
  const int64_t slab = (nvp_grad_rows(n) * (P + 1) * (int64_t)sizeof(float) + 15) / 16 * 16;
  return slab + (P + 1) * (int64_t)sizeof(double);
}
extern "C" int pdeinv_realnvp_value_and_grad(const pdeinv_realnvp_desc* d, const float* params, const float* t,
                                             int64_t t_stride, const float* x, int64_t n, int64_t ld, float* loss,
                                             float* grad, void* workspace, int64_t workspace_bytes, void* stream) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "realnvp: null descriptor");
  PDEINV_REQUIRE(d->dim >= 1 && d->dim <= 8, PDEINV_ERR_UNSUPPORTED, "realnvp: dim must be in [1, 8]");
  PDEINV_REQUIRE(d->n_layers >= 1 && d->n_layers <= PDEINV_REALNVP_MAX_LAYERS, PDEINV_ERR_UNSUPPORTED,
                 "realnvp: 1 <= n_layers <= 64");
  PDEINV_REQUIRE(d->embed_time_dim >= 0 && d->embed_time_dim <= 16 && d->embed_time_dim % 2 == 0 &&
                     d->embed_time_dim != 2,
                 PDEINV_ERR_UNSUPPORTED, "realnvp: embed_time_dim must be 0 or even in [4, 16]");
  PDEINV_REQUIRE(d->activation >= PDEINV_ACT_CELU && d->activation <= PDEINV_ACT_GELU, PDEINV_ERR_UNSUPPORTED,
                 "realnvp: unknown activation");
  PDEINV_REQUIRE(d->activation == PDEINV_ACT_CELU || d->activation == PDEINV_ACT_ELU, PDEINV_ERR_UNSUPPORTED,
                 "realnvp: value_and_grad is built for celu / elu (the flow of log_density_estimation.py:103-114)");
  PDEINV_REQUIRE(d->masks && d->base_mean && d->base_inv_cov, PDEINV_ERR_INVALID, "realnvp: null host array");
  PDEINV_REQUIRE(n >= 1 && ld >= d->dim && t_stride >= 0, PDEINV_ERR_INVALID,
                 "realnvp: value_and_grad needs n >= 1 rows (the loss is a mean)");
  PDEINV_REQUIRE(params && t && x && loss && grad && workspace, PDEINV_ERR_INVALID, "realnvp: null device pointer");
  PDEINV_REQUIRE(workspace_bytes >= pdeinv_realnvp_grad_workspace(d, n), PDEINV_ERR_INVALID,
                 "realnvp: workspace too small (pdeinv_realnvp_grad_workspace)");
  const int D = d->dim;
  NvpArgs a{};
  a.n_layers = d->n_layers;
  a.ignore_time = d->ignore_time ? 1 : 0;
  a.E = a.ignore_time ? 0 : d->embed_time_dim;
  a.in_dim = in_dim_of(d);
  a.act = d->activation;
  a.soft_init = d->soft_init;
  a.log_det = d->base_log_det;
  for (int k = 0; k < D; ++k) a.mean[k] = d->base_mean[k];
  for (int k = 0; k < D * D; ++k) a.inv_cov[k] = d->base_inv_cov[k];
  for (int k = 0; k < d->n_layers * D; ++k) a.masks[k] = d->masks[k];
  const int64_t ls = layer_params(D, a.in_dim);
  const int64_t P = pdeinv_realnvp_param_count(d);
  const int64_t rows_max = nvp_grad_rows(n);
  float* slab = (float*)workspace;
  double* acc64 = (double*)((char*)workspace + (rows_max * (P + 1) * (int64_t)sizeof(float) + 15) / 16 * 16);
  hipStream_t st = (hipStream_t)stream;
  const int64_t tiles = (n + kBlock - 1) / kBlock;
  // DM in {2, 4, 8} covers d = 1..8 (padded coordinates stay fixed); celu and elu are the same map.
  for (int64_t tile0 = 0; tile0 < tiles; tile0 += rows_max) {
    const int64_t rows = tiles - tile0 < rows_max ? tiles - tile0 : rows_max;
    const dim3 g((unsigned)rows);
    if (D <= 2)
      hipLaunchKernelGGL((realnvp_grad_kernel<2, PDEINV_ACT_CELU>), g, dim3(kBlock), 0, st, a, D, params, t,
                         t_stride, x, n, ld, ls, P, tile0, slab, P + 1);
    else if (D <= 4)
      hipLaunchKernelGGL((realnvp_grad_kernel<4, PDEINV_ACT_CELU>), g, dim3(kBlock), 0, st, a, D, params, t,
                         t_stride, x, n, ld, ls, P, tile0, slab, P + 1);
    else
      hipLaunchKernelGGL((realnvp_grad_kernel<8, PDEINV_ACT_CELU>), g, dim3(kBlock), 0, st, a, D, params, t,
                         t_stride, x, n, ld, ls, P, tile0, slab, P + 1);
    int rc = check_launch("realnvp_grad_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(nvp_grad_reduce_kernel, dim3((unsigned)((P + 1 + 63) / 64)), dim3(kBlock), 0, st, slab,
                       (int)rows, P + 1, P, acc64, tile0 == 0 ? 1 : 0, tile0 + rows >= tiles ? 1 : 0,
                       -1.0 / (double)n, grad, loss);
    rc = check_launch("nvp_grad_reduce_kernel");
    if (rc) return rc;
  }
  return PDEINV_OK;
}
