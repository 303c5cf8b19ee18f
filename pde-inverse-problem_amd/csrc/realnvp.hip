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
// loss = -mean_i log p_{t_i}(x_i), replacing jax.value_and_grad(loss_fn).
//
// Matrix-core formulation (v_mfma_f32_16x16x4_f32, exact fp32). Samples go in tiles of 16; every
// per-sample 16-vector (x, its gradient, the time embedding, each hidden layer) lives in the
// MFMA accumulator layout: lane (g = lane / 16, s = lane % 16) holds components 4g .. 4g + 3 of
// sample s. A dense layer out = W^T in is four MFMAs whose B operand at k-step j is register j of
// that same layout — k-slot (j, g) stands for input component 4g + j, and the A operand (the
// weights, read from LDS) is permuted to match — so layers chain with no data movement at all.
// The input-gradient product W d uses the transposed read of the same LDS matrix. Weight
// gradients sum_s a_s d_s^T take the samples as the reduction dimension: each tile goes through a
// per-wave swizzled LDS stage (one 16-byte write per lane, one read per k-step) into four MFMAs
// whose accumulators (ΔW in the same layout, rows = inputs) stay in registers over the wave's
// tiles. Bias and scaling-factor gradients are per-lane sums, summed over the samples at the flush
// (a reduce-scatter butterfly for a net's four bias vectors).
// All widths are padded to 16 (the net's first layer: 8 outputs; x: d <= 8 coordinates; time:
// n_t <= 16 features) with zero weights, so padded components stay exactly 0.
// * The backward pass walks the coupling layers in the opposite order of the likelihood pass and
//   rebuilds each layer's input by inverting the layer (x_in = x_out e^{-s} - tr; the masked
//   coordinates, which feed s and tr, pass through unchanged and exact): no per-layer state.
// * Per coupling layer the block sums its four waves' compact partial blocks (NvC) as float4 into its
//   slab row; the split reduce reads slab column nv_slab_col(c) for reference parameter c (the loss
//   after the time embedding's columns), and a fixed-order fp64 column reduce gives grad = -1/n sum.
//   No float atomics: bit-reproducible run to run.
// * Packed layout (d <= 4, time features <= 12): 49 KB of LDS per block and 168 VGPRs, three waves per
//   SIMD.
// Built for the celu / elu activation (the flow of log_density_estimation.py:103-114).
// ---------------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kNvpMaxRows = 8192;  // slab rows (128-sample blocks) per launch + reduce chunk
#ifndef PDEINV_NVT
#define PDEINV_NVT 2
#endif
#ifndef PDEINV_NVW_PK
#define PDEINV_NVW_PK 3  // waves per SIMD of the packed-layout gradient kernel (49 KB LDS per block)
#endif
#ifndef PDEINV_NVW
#define PDEINV_NVW 2
#endif
constexpr int kNvT = PDEINV_NVT;   // 16-sample tiles per wave (32 samples; 128 per block)
constexpr int kNvSPB = kWavesPerBlock * 16 * kNvT;  // samples per block = per slab row
constexpr int kNvWS = 20;          // LDS row stride of a padded 16 x 16 weight matrix
// Per-wave sample stage: [16 samples][16 components] dense, the 4-float chunk c of sample row r stored at chunk
// c ^ nv_swz(r). Its 16-byte writes (8-lane groups, rows s = 0..7 of one chunk) and its 4-byte reads (32-lane
// groups, rows 4t + {0, 1}, 16 components each) then cover the 32 banks of each lane group exactly once.
constexpr int kNvSS = 16;
__device__ __forceinline__ int nv_swz(int r) { return (r >> 1) & 3; }
constexpr int kNvRaw = 8 + 2 * (24 * 8 + 8 + 128 + 16 + 256 + 16 + 16 * 8 + 8);  // one layer's params, d <= 8
constexpr int kNvPre = (kNvRaw + kBlock - 1) / kBlock;

// Activation derivative from the post-activation value h (celu / elu: e^z = h + 1): min(h + 1, 1).
__device__ __forceinline__ float nvp_celu_grad_h(float h) { return fminf(h + 1.f, 1.f); }
// hardware exp2 / rcp (v_exp_f32, v_rcp_f32: ~1 ulp; the grad kernel's transcendentals)
__device__ __forceinline__ float nv_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float nv_tanh(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(nv_exp(2.f * x) + 1.f); }
// celu(z) = median(z, e^z - 1, 0): e^z - 1 >= z everywhere, so the median is z for z > 0 and e^z - 1 for
// z <= 0 (one v_med3 instead of a compare and a select).
__device__ __forceinline__ float nvp_celu(float z) { return __builtin_amdgcn_fmed3f(z, nv_exp(z) - 1.f, 0.f); }

// Padded LDS layout of one BasicMLP (weights [in][out] with row stride kNvWS), one coupling layer
// and the time embedding.
// Each matrix is also stored transposed (suffix T): the input-gradient product W d then reads it with
// the same bank-conflict-free pattern as the forward (a transposed read of W itself is 4-way).
// Packed layout: no W0X (the joined first layer is W0T). The layer image carries the layer's mask (by
// position, padded with 1) after sf. The time embedding's matrices use the same LDS array before the first
// and after the last coupling layer (TEMB floats at its start).
template <bool PK>
struct NvM {
  static constexpr int MAT = 16 * kNvWS;
  static constexpr int W0T = 0, W0X = PK ? 0 : MAT, W1 = W0X + MAT, W2 = W1 + MAT, W3 = W2 + MAT,
                       TR = W3 + MAT,  // W^T at +TR
                       B0 = 2 * TR, B1 = B0 + 16, B2 = B1 + 16, B3 = B2 + 16, NET = B3 + 16;
  static constexpr int SF = 0, MASK = 16, SNET = 32, TNET = 32 + NET, LAYER = 32 + 2 * NET;
  static constexpr int E_W1 = 0, E_B1 = MAT, E_W2 = MAT + 16, E_B2 = 2 * MAT + 16, E_W2T = 2 * MAT + 32,
                       TEMB = 3 * MAT + 32;
  static_assert(TEMB <= LAYER, "time embedding inside the layer image");
};
// Per-wave partial-gradient block of one coupling layer, compact (only the entries a parameter maps to):
// [t-net | s-net | sf (16, by position)]. Per net, packed layout: W0 [16 input positions][8 hidden units],
// W1 [8][16], W2 [16][16], W3 [16][4 coordinates], b0..b3 by position (16 each); identity layout: W0T
// [16 time rows][8], W0X [8 coordinates][8], W1 [8][16], W2, W3 [16][8], b0..b3. The block is also the layer's
// slab-row segment (the flush sums the four waves' blocks as float4 into it); the reduce maps it to the
// reference parameter order (nv_slab_col). In LDS the t-net part aliases the wave's sample stage (it is written
// after the t-net's last weight gradient) and the s-net part + sf sit behind the stage (written as soon as the
// s-net's backward is done, so its accumulators are dead during the t-net's). The time embedding's flush reuses
// the first 2 x 272 floats.
template <bool PK>
struct NvC {
  static constexpr int W0T = 0, W0X = 128, W1 = PK ? 128 : 192, W2 = W1 + 128, W3 = W2 + 256,
                       B0 = W3 + (PK ? 64 : 128), B1 = B0 + 16, B2 = B1 + 16, B3 = B2 + 16, NET = B3 + 16;
  static constexpr int TNET = 0, SNET = NET, SF = 2 * NET, LAYER = 2 * NET + 16;  // 1296 / 1552 floats
};
constexpr int kNvStageF = 2 * 16 * kNvSS;  // per-wave sample stage (floats): one tile's two operands
// Per-wave scratch: [t-net block / sample stage (kNvTR floats) | s-net block | sf]
template <bool PK>
struct NvScr {
  static constexpr int TR = NvC<PK>::NET > kNvStageF ? NvC<PK>::NET : kNvStageF;
  static constexpr int SIZE = TR + NvC<PK>::NET + 16;
};
// LDS offset (in the wave's scratch) of compact-block entry o
template <bool PK>
__device__ __forceinline__ int nv_flush_lds(int o) { return o < NvC<PK>::NET ? o : o - NvC<PK>::NET + NvScr<PK>::TR; }

struct NvLane {
  int g, s;    // component group, sample within the tile
  int sw, sr;  // sample-stage offsets: this lane's 16-byte write (row s, chunk g); its read of row g, component s
};

// Position of a component in the padded 16-vectors. Packed layout (PK: d <= 4, n_t <= 12): coordinate c
// at 4c (register 0 of lane group c), time-embedding component e at 4(e / 3) + 1 + e % 3 (registers 1..3),
// the first hidden layer's 8 units at 4(o / 2) + o % 2 (registers 0, 1). So [x | temb] is ONE 16-vector
// with no data movement (register 0 from x, 1..3 from temb: the net's first layer is one 16 x 16 product,
// not two), and the k-steps whose inputs are all padding are skipped: W1 reads 2 of 4, the input-gradient
// products of W3 and W0 1 and 2 of 4. The matrices are permuted to match when a layer is staged (a
// dense layer's output order is the A operand's row order, free to choose). Identity layout otherwise.
template <bool PK> __device__ __forceinline__ int nv_xpos(int c) { return PK ? 4 * c : c; }
template <bool PK> __device__ __forceinline__ int nv_tpos(int e) { return PK ? 4 * (e / 3) + 1 + e % 3 : e; }
template <bool PK> __device__ __forceinline__ int nv_hpos(int o) { return PK ? 4 * (o / 2) + o % 2 : o; }
// inverses: position -> component, or -1 (padding); n = the component count
template <bool PK> __device__ __forceinline__ int nv_xinv(int p, int n) {
  const int c = PK ? ((p & 3) == 0 ? p >> 2 : -1) : p;
  return c < n ? c : -1;
}
template <bool PK> __device__ __forceinline__ int nv_tinv(int p, int n) {
  const int e = PK ? ((p & 3) != 0 ? 3 * (p >> 2) + (p & 3) - 1 : -1) : p;
  return e < n ? e : -1;
}
template <bool PK> __device__ __forceinline__ int nv_hinv(int p) {
  const int o = PK ? ((p & 3) < 2 ? 2 * (p >> 2) + (p & 3) : -1) : p;
  return o < 8 ? o : -1;
}

__device__ __forceinline__ f32x4 nv_vec(const float* b, const NvLane& ln) {
  return *reinterpret_cast<const f32x4*>(b + 4 * ln.g);
}
__device__ __forceinline__ f32x4 nv_celu4(f32x4 z) {
  return f32x4{nvp_celu(z[0]), nvp_celu(z[1]), nvp_celu(z[2]), nvp_celu(z[3])};
}
__device__ __forceinline__ f32x4 nv_dact4(f32x4 d, f32x4 h) {
  return f32x4{d[0] * nvp_celu_grad_h(h[0]), d[1] * nvp_celu_grad_h(h[1]), d[2] * nvp_celu_grad_h(h[2]),
               d[3] * nvp_celu_grad_h(h[3])};
}
// Order the wave's own LDS stage accesses (a wave's LDS instructions execute in order, so a lane
// reads what another lane of the same wave wrote before it) without fencing the MFMA / VALU
// stream: a compiler memory barrier only, so independent matrix work still moves across it.
__device__ __forceinline__ void nv_wave_sync() { asm volatile("" ::: "memory"); }
// The wave's kNvT tiles go through every dense layer together: one A-operand (weight) read feeds
// kNvT independent MFMAs, so the accumulation chains of the tiles interleave.
typedef f32x4 NvV[kNvT];

// k-steps j with JM bit j clear carry only padding inputs (all zero) and are skipped.
template <int JM = 0xF>
__device__ __forceinline__ void nv_fwdT(const float* W, const NvLane& ln, const NvV& x, NvV& c) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!((JM >> j) & 1)) continue;
    const float av = W[(4 * ln.g + j) * kNvWS + ln.s];
#pragma unroll
    for (int u = 0; u < kNvT; ++u) c[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, x[u][j], c[u], 0, 0, 0);
  }
}
__device__ __forceinline__ void nv_bcast(NvV& c, const f32x4& b) {
#pragma unroll
  for (int u = 0; u < kNvT; ++u) c[u] = b;
}

// acc += sum over the wave's samples of a_s d_s^T (rows = a components): per-wave LDS stage
// [2][16 samples][kNvSS] (swizzled chunks, nv_swz) holding one tile at a time (a wave's LDS instructions run
// in order, so the next tile's writes follow this tile's reads): one 16-byte write per lane and operand, one
// read per operand and k-step.
__device__ __forceinline__ f32x4 nv_wgrad(float* stage, const NvLane& ln, const NvV& a, const NvV& d, f32x4 acc) {
#pragma unroll
  for (int u = 0; u < kNvT; ++u) {
    nv_wave_sync();  // the previous reads of the stage are issued
    *reinterpret_cast<f32x4*>(stage + ln.sw) = a[u];
    *reinterpret_cast<f32x4*>(stage + 16 * kNvSS + ln.sw) = d[u];
    nv_wave_sync();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      // row 4t + g: nv_swz(4t + g) = nv_swz(g) ^ 2 (t & 1), i.e. component s ^ 8 on odd t
      const int r = 4 * t * kNvSS + (ln.sr ^ (t & 1 ? 8 : 0));
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(stage[r], stage[16 * kNvSS + r], acc, 0, 0, 0);
    }
  }
  return acc;
}

// Gradient accumulators of one BasicMLP over the wave's tiles.
struct NvNetAcc {
  f32x4 w0t, w0x, w1, w2, w3, b0, b1, b2, b3;
  __device__ void zero() { w0t = w0x = w1 = w2 = w3 = b0 = b1 = b2 = b3 = f32x4{0.f, 0.f, 0.f, 0.f}; }
};

struct NvAct {
  NvV h0, h1, h2;
};

// Packed layout: the net input [xm | temb] as one vector (register 0 from xm, 1..3 from temb).
__device__ __forceinline__ void nv_join(const NvV& xm, const NvV& temb, NvV& in) {
#pragma unroll
  for (int u = 0; u < kNvT; ++u) in[u] = f32x4{xm[u][0], temb[u][1], temb[u][2], temb[u][3]};
}

// BasicMLP (:97-111) forward: input [temb | xm], hidden 8 / 16 / 16, output d (all padded to 16).
// Packed layout: the first layer is one product over the joined input, stored at W0T.
template <bool PK>
__device__ __forceinline__ void nv_mlp_fwd(const float* p, const NvLane& ln, const NvV& temb, const NvV& xm,
                                           NvAct& h, NvV& out) {
  NvV z;
  nv_bcast(z, nv_vec(p + NvM<PK>::B0, ln));
  if constexpr (PK) {
    NvV in;
    nv_join(xm, temb, in);
    nv_fwdT(p + NvM<PK>::W0T, ln, in, z);
  } else {
    nv_fwdT(p + NvM<PK>::W0T, ln, temb, z);
    nv_fwdT(p + NvM<PK>::W0X, ln, xm, z);
  }
#pragma unroll
  for (int u = 0; u < kNvT; ++u) {
    if constexpr (PK)  // registers 2, 3: padding units (zero weights and bias), celu(0) = 0
      h.h0[u] = f32x4{nvp_celu(z[u][0]), nvp_celu(z[u][1]), 0.f, 0.f};
    else
      h.h0[u] = nv_celu4(z[u]);
  }
  nv_bcast(z, nv_vec(p + NvM<PK>::B1, ln));
  nv_fwdT<PK ? 0x3 : 0xF>(p + NvM<PK>::W1, ln, h.h0, z);
#pragma unroll
  for (int u = 0; u < kNvT; ++u) h.h1[u] = nv_celu4(z[u]);
  nv_bcast(z, nv_vec(p + NvM<PK>::B2, ln));
  nv_fwdT(p + NvM<PK>::W2, ln, h.h1, z);
#pragma unroll
  for (int u = 0; u < kNvT; ++u) h.h2[u] = nv_celu4(z[u]);
  nv_bcast(out, nv_vec(p + NvM<PK>::B3, ln));
  nv_fwdT(p + NvM<PK>::W3, ln, h.h2, out);
}

// BasicMLP backward from d(out): parameter gradients into acc, input gradients added to gtemb
// (time rows) and gx (x rows). The input-gradient products W d read the transposed copies.
// Packed layout: acc.w0t holds the joined first-layer gradient (acc.w0x unused).
template <bool PK>
__device__ __forceinline__ void nv_mlp_bwd(const float* p, const NvLane& ln, float* stage, const NvV& temb,
                                           const NvV& xm, const NvAct& h, const NvV& dout, NvNetAcc& acc,
                                           NvV& gtemb, NvV& gx) {
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  NvV d, e;
  acc.w3 = nv_wgrad(stage, ln, h.h2, dout, acc.w3);
  nv_bcast(e, z4);
  nv_fwdT<PK ? 0x1 : 0xF>(p + NvM<PK>::TR + NvM<PK>::W3, ln, dout, e);
#pragma unroll
  for (int u = 0; u < kNvT; ++u) {
    acc.b3 += dout[u];
    d[u] = nv_dact4(e[u], h.h2[u]);
  }
  acc.w2 = nv_wgrad(stage, ln, h.h1, d, acc.w2);
  nv_bcast(e, z4);
  nv_fwdT(p + NvM<PK>::TR + NvM<PK>::W2, ln, d, e);
#pragma unroll
  for (int u = 0; u < kNvT; ++u) {
    acc.b2 += d[u];
    d[u] = nv_dact4(e[u], h.h1[u]);
  }
  acc.w1 = nv_wgrad(stage, ln, h.h0, d, acc.w1);
  nv_bcast(e, z4);
  nv_fwdT(p + NvM<PK>::TR + NvM<PK>::W1, ln, d, e);
#pragma unroll
  for (int u = 0; u < kNvT; ++u) {
    acc.b1 += d[u];
    if constexpr (PK)  // padding units: their gradient feeds only padding entries (dropped by the flush)
      d[u] = f32x4{e[u][0] * nvp_celu_grad_h(h.h0[u][0]), e[u][1] * nvp_celu_grad_h(h.h0[u][1]), 0.f, 0.f};
    else
      d[u] = nv_dact4(e[u], h.h0[u]);
  }
  if constexpr (PK) {
    NvV in;
    nv_join(xm, temb, in);
    acc.w0t = nv_wgrad(stage, ln, in, d, acc.w0t);
#pragma unroll
    for (int u = 0; u < kNvT; ++u) acc.b0 += d[u];
    nv_bcast(e, z4);
    nv_fwdT<0x3>(p + NvM<PK>::TR + NvM<PK>::W0T, ln, d, e);
#pragma unroll
    for (int u = 0; u < kNvT; ++u) {
      gx[u][0] += e[u][0];
#pragma unroll
      for (int c = 1; c < 4; ++c) gtemb[u][c] += e[u][c];
    }
  } else {
    acc.w0t = nv_wgrad(stage, ln, temb, d, acc.w0t);
    acc.w0x = nv_wgrad(stage, ln, xm, d, acc.w0x);
#pragma unroll
    for (int u = 0; u < kNvT; ++u) acc.b0 += d[u];
    nv_fwdT(p + NvM<PK>::TR + NvM<PK>::W0T, ln, d, gtemb);
    nv_fwdT(p + NvM<PK>::TR + NvM<PK>::W0X, ln, d, gx);
  }
}

// Sum of v over the 16 samples of each component group: DPP inside 16-lane rows (quad_perm xor 1,
// xor 2, row_half_mirror, row_mirror), every lane of the row ends with the row total.
template <int CTRL>
__device__ __forceinline__ float nv_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ f32x4 nv_sum16(f32x4 v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] += nv_dpp<0xB1>(v[i]);
    v[i] += nv_dpp<0x4E>(v[i]);
    v[i] += nv_dpp<0x141>(v[i]);
    v[i] += nv_dpp<0x140>(v[i]);
  }
  return v;
}

// The four bias vectors of a net summed over the 16 samples of each component group at once: a reduce-scatter
// butterfly over the 16 values (b0..b3, registers 0..3) — row mirror, half-row mirror, quad xor 2, quad xor 1,
// each stage keeping the half of the values selected by one lane bit — leaves lane s with the total of value s
// (45 VALU instead of 4 x nv_sum16). Written to r[16 (s / 4) + 4 g + s % 4] (b_{s/4} by position).
__device__ __forceinline__ void nv_put_bias4(float* r, const NvLane& ln, const f32x4& b0, const f32x4& b1,
                                             const f32x4& b2, const f32x4& b3) {
  float v[16];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v[c] = b0[c];
    v[4 + c] = b1[c];
    v[8 + c] = b2[c];
    v[12 + c] = b3[c];
  }
  auto stage = [&](auto dpp, int half, bool hi) {
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float send = hi ? v[i] : v[i + half], keep = hi ? v[i + half] : v[i];
      v[i] = keep + dpp(send);
    }
  };
  stage([](float x) { return nv_dpp<0x140>(x); }, 8, (ln.s & 8) != 0);  // partner 15 - s (row mirror)
  stage([](float x) { return nv_dpp<0x141>(x); }, 4, (ln.s & 4) != 0);  // partner s ^ 7 (half-row mirror)
  stage([](float x) { return nv_dpp<0x4E>(x); }, 2, (ln.s & 2) != 0);   // s ^ 2
  stage([](float x) { return nv_dpp<0xB1>(x); }, 1, (ln.s & 1) != 0);   // s ^ 1
  r[(ln.s >> 2) * 16 + 4 * ln.g + (ln.s & 3)] = v[0];
}

// A wave's partials into its LDS flush block: matrices in the accumulator layout (row 4g + i,
// column s), vectors summed over samples.
__device__ __forceinline__ void nv_put_mat(float* r, const NvLane& ln, const f32x4& m) {
#pragma unroll
  for (int i = 0; i < 4; ++i) r[(4 * ln.g + i) * 16 + ln.s] = m[i];
}
// Compact matrix put (NvC): row 4g + i -> row map R (-1: padding), column s -> column map C, width NC.
template <int NC, typename RM, typename CM>
__device__ __forceinline__ void nv_put_cmat(float* r, const NvLane& ln, const f32x4& m, RM rm, CM cm) {
  const int c = cm(ln.s);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = rm(4 * ln.g + i);
    if (q >= 0 && c >= 0) r[q * NC + c] = m[i];
  }
}
__device__ __forceinline__ void nv_put_vec(float* r, const NvLane& ln, const f32x4& v) {
  const f32x4 t = nv_sum16(v);
  if (ln.s == 0) *reinterpret_cast<f32x4*>(r + 4 * ln.g) = t;
}
template <bool PK>
__device__ __forceinline__ void nv_put_net(float* r, const NvLane& ln, const NvNetAcc& a) {
  using C = NvC<PK>;
  auto all = [](int p) { return p; };
  auto hid = [](int p) { return PK ? ((p & 3) < 2 ? 2 * (p >> 2) + (p & 1) : -1) : (p < 8 ? p : -1); };  // h0 unit
  if constexpr (PK) {
    nv_put_cmat<8>(r + C::W0T, ln, a.w0t, all, hid);
  } else {
    nv_put_cmat<8>(r + C::W0T, ln, a.w0t, all, hid);
    nv_put_cmat<8>(r + C::W0X, ln, a.w0x, [](int p) { return p < 8 ? p : -1; }, hid);
  }
  nv_put_cmat<16>(r + C::W1, ln, a.w1, hid, all);
  nv_put_cmat<16>(r + C::W2, ln, a.w2, all, all);
  if constexpr (PK)
    nv_put_cmat<4>(r + C::W3, ln, a.w3, all, [](int p) { return (p & 3) == 0 ? p >> 2 : -1; });
  else
    nv_put_cmat<8>(r + C::W3, ln, a.w3, all, [](int p) { return p < 8 ? p : -1; });
  static_assert(C::B1 == C::B0 + 16 && C::B2 == C::B1 + 16 && C::B3 == C::B2 + 16, "bias vectors contiguous");
  nv_put_bias4(r + C::B0, ln, a.b0, a.b1, a.b2, a.b3);
}

// Flat (reference-order) parameter f of one BasicMLP -> its index in the compact net block (NvC).
template <bool PK>
__host__ __device__ __forceinline__ int nv_cb_src(int f, int d, int n_t) {
  using C = NvC<PK>;
  const int n_in = d + n_t;
  if (f < n_in * 8) {
    const int r = f / 8, o = f - r * 8;
    if (PK) return C::W0T + (r < d ? 4 * r : 4 * ((r - d) / 3) + 1 + (r - d) % 3) * 8 + o;
    return r < d ? C::W0X + r * 8 + o : C::W0T + (r - d) * 8 + o;
  }
  f -= n_in * 8;
  if (f < 8) return C::B0 + (PK ? 4 * (f / 2) + f % 2 : f);
  f -= 8;
  if (f < 128) return C::W1 + f;  // [h0 unit][16]
  f -= 128;
  if (f < 16) return C::B1 + f;
  f -= 16;
  if (f < 256) return C::W2 + f;
  f -= 256;
  if (f < 16) return C::B2 + f;
  f -= 16;
  if (f < 16 * d) return C::W3 + (f / d) * (PK ? 4 : 8) + f % d;
  f -= 16 * d;
  return C::B3 + (PK ? 4 * f : f);
}

// Slab-row layout of the gradient kernel: [L compact layer blocks (NvC::LAYER each) | time embedding (reference
// order) | loss], row stride rounded up to 4 floats (the layer blocks are stored as float4).
struct NvSlabMap {
  int d, n_t, pk, n_layers;
  int64_t layer_stride, temb_params, n_params, cb;
};
__host__ __device__ __forceinline__ int64_t nv_slab_col(const NvSlabMap& m, int64_t c) {
  const int64_t lcb = (int64_t)m.n_layers * m.cb;
  if (c >= m.n_params) return lcb + m.temb_params;  // loss
  if (c < m.temb_params) return lcb + c;
  c -= m.temb_params;
  const int64_t l = c / m.layer_stride;
  int k = (int)(c - l * m.layer_stride);
  const int64_t base = l * m.cb;
  if (k < m.d) return base + (m.pk ? NvC<true>::SF + 4 * k : NvC<false>::SF + k);  // sf by position
  k -= m.d;
  const int mlp_n = (m.d + m.n_t) * 8 + 8 + 8 * 16 + 16 + 16 * 16 + 16 + 16 * m.d + m.d;
  const int net = k >= mlp_n ? 1 : 0;
  k -= net * mlp_n;
  if (m.pk) return base + (net ? NvC<true>::TNET : NvC<true>::SNET) + nv_cb_src<true>(k, m.d, m.n_t);
  return base + (net ? NvC<false>::TNET : NvC<false>::SNET) + nv_cb_src<false>(k, m.d, m.n_t);
}
__host__ __device__ __forceinline__ int64_t nv_slab_ld(const NvSlabMap& m) {
  return ((int64_t)m.n_layers * m.cb + m.temb_params + 1 + 3) / 4 * 4;
}

// Raw coupling-layer parameter k (reference order: sf, s-net, t-net) -> its LDS position(s) in the padded layer
// image: dst | dstT << 16 (the transposed copy of a matrix entry; 0xFFFF for vectors). Layer-invariant, so a
// block computes it once and every staging is a scatter of the prefetched registers through this table.
template <bool PK>
__device__ __forceinline__ uint32_t nv_layer_dst(int k, int d, int n_t) {
  const int n_in = d + n_t, mlp_n = n_in * 8 + 8 + 8 * 16 + 16 + 16 * 16 + 16 + 16 * d + d;
  if (k < d) return (uint32_t)(NvM<PK>::SF + nv_xpos<PK>(k)) | 0xFFFF0000u;
  k -= d;
  const int net = k >= mlp_n ? 1 : 0;
  int f = k - net * mlp_n;
  const int base = net ? NvM<PK>::TNET : NvM<PK>::SNET;
  auto mat = [&](int M, int pr, int pc) {
    return (uint32_t)(base + M + pr * kNvWS + pc) | ((uint32_t)(base + NvM<PK>::TR + M + pc * kNvWS + pr) << 16);
  };
  auto vec = [&](int B, int p) { return (uint32_t)(base + B + p) | 0xFFFF0000u; };
  if (f < n_in * 8) {
    const int r = f / 8, o = f - r * 8;
    if (PK) return mat(NvM<PK>::W0T, r < d ? nv_xpos<PK>(r) : nv_tpos<PK>(r - d), nv_hpos<PK>(o));
    return r < d ? mat(NvM<PK>::W0X, r, o) : mat(NvM<PK>::W0T, r - d, o);
  }
  f -= n_in * 8;
  if (f < 8) return vec(NvM<PK>::B0, nv_hpos<PK>(f));
  f -= 8;
  if (f < 128) return mat(NvM<PK>::W1, nv_hpos<PK>(f / 16), f % 16);
  f -= 128;
  if (f < 16) return vec(NvM<PK>::B1, f);
  f -= 16;
  if (f < 256) return mat(NvM<PK>::W2, f / 16, f % 16);
  f -= 256;
  if (f < 16) return vec(NvM<PK>::B2, f);
  f -= 16;
  if (f < 16 * d) return mat(NvM<PK>::W3, f / d, nv_xpos<PK>(f % d));
  f -= 16 * d;
  return vec(NvM<PK>::B3, nv_xpos<PK>(f));
}

template <int ACT, bool PK>
__global__ __launch_bounds__(kBlock, PK ? PDEINV_NVW_PK : PDEINV_NVW) void realnvp_grad_kernel(NvpArgs a, int d, const float* __restrict__ params,
                                                                 const float* __restrict__ tv, int64_t t_stride,
                                                                 const float* __restrict__ xv, int64_t n, int64_t ld,
                                                                 int64_t layer_stride, int64_t n_params,
                                                                 int64_t tile0, float* __restrict__ slab,
                                                                 int64_t slab_ld) {
  static_assert(ACT == PDEINV_ACT_CELU, "celu / elu flow");
  __shared__ float sW[NvM<PK>::LAYER];  // current coupling layer (padded); the time embedding before / after
  float* const sT = sW;
  __shared__ float sF[48];              // sinusoid table: frequency, sin weight, cos weight
  __shared__ float sB[16 + 16 * 16];    // base mean, inverse covariance (0-padded)
  // per-wave sample stages and flush blocks (NvScr)
  __shared__ float sScr[kWavesPerBlock][NvScr<PK>::SIZE];
  __shared__ uint32_t sDst[kNvRaw];                  // raw layer parameter -> LDS position(s), nv_layer_dst
  using C = NvC<PK>;
  const int E = a.E;
  const int n_in = a.in_dim, n_t = n_in - d;
  const int64_t lcb = (int64_t)a.n_layers * C::LAYER;  // slab-row offset of the time-embedding columns
  const int64_t temb_params = E > 0 ? 2 * ((int64_t)E * E + E) : 0;
  const float* layers = params + temb_params;
  const bool hard = !a.ignore_time && a.soft_init == 0.f;
  const int tid = threadIdx.x, wave = tid >> 6;
  NvLane ln;
  {
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));  // opaque: keeps per-use address math out of long-lived registers
    ln.g = lane >> 4;
    ln.s = lane & 15;
    ln.sw = ln.s * kNvSS + 4 * (ln.g ^ nv_swz(ln.s));
    ln.sr = ln.g * kNvSS + (ln.s ^ (4 * nv_swz(ln.g)));
  }
  float* stage = sScr[wave];
  float* red = sScr[wave];
  // ---- per-block tables ----
  // padded [16][kNvWS] (and its transpose): position (r, c) <- src[rm(r)][cm(c)], 0 where a map gives -1
  auto put_mat = [&](float* dst, float* dst_t, const float* src, int ld_src, auto rm, auto cm) {
    for (int q = tid; q < 16 * kNvWS; q += kBlock) {
      const int r = q / kNvWS, c = q - r * kNvWS;
      const int sr = c < 16 ? rm(r) : -1, sc = c < 16 ? cm(c) : -1;
      dst[q] = (sr >= 0 && sc >= 0) ? src[sr * ld_src + sc] : 0.f;
      if (dst_t) {
        const int tr = c < 16 ? rm(c) : -1, tc = c < 16 ? cm(r) : -1;
        dst_t[q] = (tr >= 0 && tc >= 0) ? src[tr * ld_src + tc] : 0.f;
      }
    }
  };
  auto put_vec = [&](float* dst, const float* src, auto m) {
    for (int q = tid; q < 16; q += kBlock) {
      const int k = m(q);
      dst[q] = k >= 0 ? src[k] : 0.f;
    }
  };
  auto idn = [](int len) { return [len](int p) { return p < len ? p : -1; }; };
  auto put_temb = [&] {  // the time embedding's matrices into sT (= the start of sW)
    auto tmap = [E](int p) { return nv_tinv<PK>(p, E); };
    put_mat(sT + NvM<PK>::E_W1, nullptr, params, E, idn(E), idn(E));
    put_vec(sT + NvM<PK>::E_B1, params + E * E, idn(E));
    put_mat(sT + NvM<PK>::E_W2, sT + NvM<PK>::E_W2T, params + E * E + E, E, idn(E), tmap);  // temb at its positions
    put_vec(sT + NvM<PK>::E_B2, params + 2 * E * E + E, tmap);
  };
  if (tid < 16) {
    const int half = E / 2;
    const bool on = E > 0 && tid < E;
    const bool is_sin = tid < half;
    const float step = E > 0 ? logf(10000.f) / (float)(half - 1) : 0.f;
    sF[tid] = on ? expf(-step * (float)(is_sin ? tid : tid - half)) : 0.f;
    sF[16 + tid] = on && is_sin ? 1.f : 0.f;
    sF[32 + tid] = on && !is_sin ? 1.f : 0.f;
  }
  for (int k = tid; k < layer_stride; k += kBlock) sDst[k] = nv_layer_dst<PK>(k, d, n_t);
  for (int q = tid; q < NvM<PK>::LAYER; q += kBlock) sW[q] = 0.f;  // padding: never written again
  for (int q = tid; q < 16 + 256; q += kBlock) {  // mean at the x positions; inv_cov rows by position, columns by coordinate
    float v = 0.f;
    if (q < 16) {
      const int k = nv_xinv<PK>(q, d);
      v = k >= 0 ? a.mean[k] : 0.f;
    } else {
      const int r = nv_xinv<PK>((q - 16) / 16, d), c = (q - 16) % 16;
      v = (r >= 0 && c < d) ? a.inv_cov[r * d + c] : 0.f;
    }
    sB[q] = v;
  }
  // Layer parameters are prefetched one staged layer ahead into registers (one coalesced load per
  // thread and slot, in flight under the previous layer's math) and scattered into the padded /
  // transposed layer image through the sDst table. Staging order: L-1 .. 0 (likelihood), 0 .. L-1.
  float pre[kNvPre];
  auto prefetch = [&](int l) {
    const float* lp = layers + (int64_t)l * layer_stride;
#pragma unroll
    for (int k = 0; k < kNvPre; ++k) {
      const int q = tid + k * kBlock;
      pre[k] = q < layer_stride ? lp[q] : 0.f;
    }
  };
  int staged = 0;  // layers staged so far
  auto stage_layer = [&](int l) {
    __syncthreads();  // every wave is done with the previous layer
    if (tid < 16) {  // the layer's mask by position, padded with 1
      const int k = nv_xinv<PK>(tid, d);
      sW[NvM<PK>::MASK + tid] = k >= 0 ? a.masks[l * d + k] : 1.f;
    }
#pragma unroll
    for (int k = 0; k < kNvPre; ++k) {
      const int q = tid + k * kBlock;
      if (q < layer_stride) {
        const uint32_t t = sDst[q];
        sW[t & 0xFFFFu] = pre[k];
        if ((t >> 16) != 0xFFFFu) sW[t >> 16] = pre[k];
      }
    }
    ++staged;
    if (staged < 2 * a.n_layers) prefetch(staged < a.n_layers ? a.n_layers - 1 - staged : staged - a.n_layers);
    __syncthreads();
  };
  prefetch(a.n_layers - 1);
  float* row = slab + (int64_t)blockIdx.x * slab_ld;
  // write this block's reduced partials for the flat range [off, off + len): src(f) -> flush index
  auto flush = [&](int64_t off, int len, auto src) {
    __syncthreads();  // every wave's partials are in its flush block
    for (int f = tid; f < len; f += kBlock) {
      const int k = src(f);
      float v = 0.f;
      if (k >= 0) v = ((sScr[0][k] + sScr[1][k]) + sScr[2][k]) + sScr[3][k];
      row[off + f] = v;
    }
    __syncthreads();  // the flush blocks are free again
  };

  // ---- the wave's tiles ----
  NvV x, gx, temb, gtemb;
  float tt[kNvT], w[kNvT], ldj[kNvT];
  const int64_t base = (tile0 + blockIdx.x) * kNvSPB + wave * 16 * kNvT;
  __syncthreads();  // sW zeroed
  if (E > 0) put_temb();
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kNvT; ++u) {
    const int64_t i = base + 16 * u + ln.s;
    const bool active = i < n;
    w[u] = active ? 1.f : 0.f;
    tt[u] = active ? tv[i * t_stride] : 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = nv_xinv<PK>(4 * ln.g + c, d);
      x[u][c] = (active && k >= 0 && (!PK || c == 0)) ? xv[i * ld + k] : 0.f;  // packed: registers 1..3 are 0
      gtemb[u][c] = 0.f;
    }
    ldj[u] = 0.f;
  }
  // TimeEmbedding (:8-22): se = SinusoidalEmbedding(t) (:24-38), he = act(se W1 + b1), temb = he W2 + b2
  auto sinusoid = [&](NvV& se) {
#pragma unroll
    for (int u = 0; u < kNvT; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int q = 4 * ln.g + c;
        const float e = tt[u] * sF[q];
        se[u][c] = sF[16 + q] * sinf(e) + sF[32 + q] * cosf(e);
      }
  };
  if (E > 0) {
    NvV se, he;
    sinusoid(se);
    nv_bcast(he, nv_vec(sT + NvM<PK>::E_B1, ln));
    nv_fwdT(sT + NvM<PK>::E_W1, ln, se, he);
#pragma unroll
    for (int u = 0; u < kNvT; ++u) he[u] = nv_celu4(he[u]);
    nv_bcast(temb, nv_vec(sT + NvM<PK>::E_B2, ln));
    nv_fwdT(sT + NvM<PK>::E_W2, ln, he, temb);
    __syncthreads();  // every wave has read the time embedding: back to the zero-padded layer image
    for (int q = tid; q < NvM<PK>::TEMB; q += kBlock) sW[q] = 0.f;
  } else {
#pragma unroll
    for (int u = 0; u < kNvT; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) temb[u][c] = (!a.ignore_time && 4 * ln.g + c == nv_tpos<PK>(0)) ? tt[u] : 0.f;
  }
  // Packed layout: the coordinates live in register 0 only (registers 1..3 of x, gx stay exactly 0 through
  // every coupling layer), so the per-coordinate coupling math runs over NC = 1 register.
  constexpr int NC = PK ? 1 : 4;
  // ---- likelihood pass (layers L-1 .. 0): x <- (x + tr) e^s ----
  for (int l = a.n_layers - 1; l >= 0; --l) {
    stage_layer(l);
    const f32x4 m = nv_vec(sW + NvM<PK>::MASK, ln), sfw = nv_vec(sW + NvM<PK>::SF, ln);
    f32x4 sf, isf;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      sf[c] = nv_exp(sfw[c]);
      isf[c] = __builtin_amdgcn_rcpf(sf[c]);
    }
    NvV xm, so, to;
#pragma unroll
    for (int u = 0; u < kNvT; ++u) xm[u] = PK ? f32x4{x[u][0] * m[0], 0.f, 0.f, 0.f} : x[u] * m;
    {
      NvAct h;
      nv_mlp_fwd<PK>(sW + NvM<PK>::SNET, ln, temb, xm, h, so);
      nv_mlp_fwd<PK>(sW + NvM<PK>::TNET, ln, temb, xm, h, to);
    }
#pragma unroll
    for (int u = 0; u < kNvT; ++u) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {  // padded / masked k: keep = 0, x unchanged
        const float keep = 1.f - m[c];
        const float sk = nv_tanh((hard ? tt[u] * so[u][c] : so[u][c]) * isf[c]) * sf[c] * keep;
        x[u][c] = (x[u][c] + (hard ? tt[u] * to[u][c] : to[u][c]) * keep) * nv_exp(sk);
        ldj[u] += sk;
      }
    }
  }
  // ---- base density log p0(x0) and its gradient (per-wave stage holds the tile's x rows) ----
  float lsum = 0.f;  // sum over the wave's samples of w log p (lane-partial)
#pragma unroll
  for (int u = 0; u < kNvT; ++u) {
    const f32x4 diff = x[u] - nv_vec(sB, ln);
    nv_wave_sync();
    *reinterpret_cast<f32x4*>(stage + ln.sw) = diff;
    nv_wave_sync();
    float quad = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int r = 4 * ln.g + c;
      float acc = 0.f;
      for (int q = 0; q < d; ++q)
        acc = fmaf(sB[16 + r * 16 + q], stage[ln.s * kNvSS + (nv_xpos<PK>(q) ^ (4 * nv_swz(ln.s)))], acc);
      quad = fmaf(diff[c], acc, quad);
      gx[u][c] = PK && c > 0 ? 0.f : -w[u] * acc;
    }
    float part = ldj[u] - 0.5f * quad;  // the four groups' parts sum to log p + 0.5 log_det
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    if (ln.g == 0) lsum += w[u] * (part - 0.5f * a.log_det);
  }
  // ---- backward through layers 0 .. L-1, rebuilding each layer's input ----
  for (int l = 0; l < a.n_layers; ++l) {
    stage_layer(l);
    const f32x4 m = nv_vec(sW + NvM<PK>::MASK, ln), sfw = nv_vec(sW + NvM<PK>::SF, ln);
    f32x4 sfv, isf;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      sfv[c] = nv_exp(sfw[c]);
      isf[c] = __builtin_amdgcn_rcpf(sfv[c]);
    }
    NvNetAcc as, at;
    as.zero();
    at.zero();
    f32x4 galpha = {0.f, 0.f, 0.f, 0.f};
    NvV xm, out, s, es, gso, gto, gacc;
    NvAct h;
#pragma unroll
    for (int u = 0; u < kNvT; ++u) xm[u] = PK ? f32x4{x[u][0] * m[0], 0.f, 0.f, 0.f} : x[u] * m;
    nv_mlp_fwd<PK>(sW + NvM<PK>::SNET, ln, temb, xm, h, out);
#pragma unroll
    for (int u = 0; u < kNvT; ++u) {
      gso[u] = gto[u] = gacc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float keep = 1.f - m[c];
        const float spre = hard ? tt[u] * out[u][c] : out[u][c];
        const float sf = sfv[c];
        const float th = nv_tanh(spre * isf[c]);
        s[u][c] = th * sf * keep;
        es[u][c] = nv_exp(s[u][c]);
        const float gs = (gx[u][c] * x[u][c] + w[u]) * keep;  // d(log p0 + ldj)/ds via x_out and ldj
        const float dth = 1.f - th * th;
        galpha[c] += gs * (th * sf - dth * spre);              // d/d scaling_factor (sf = e^alpha)
        gso[u][c] = (hard ? tt[u] : 1.f) * gs * dth;           // d/d scale_net output
        gto[u][c] = (hard ? tt[u] : 1.f) * gx[u][c] * es[u][c] * keep;  // d/d translate_net output
      }
    }
    nv_mlp_bwd<PK>(sW + NvM<PK>::SNET, ln, stage, temb, xm, h, gso, as, gtemb, gacc);
    nv_put_vec(red + NvScr<PK>::TR + NvC<PK>::NET, ln, galpha);  // behind the stage (nv_flush_lds)
    nv_put_net<PK>(red + NvScr<PK>::TR, ln, as);
    nv_mlp_fwd<PK>(sW + NvM<PK>::TNET, ln, temb, xm, h, out);
    nv_mlp_bwd<PK>(sW + NvM<PK>::TNET, ln, stage, temb, xm, h, gto, at, gtemb, gacc);
#pragma unroll
    for (int u = 0; u < kNvT; ++u)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float tr = (hard ? tt[u] * out[u][c] : out[u][c]) * (1.f - m[c]);
        x[u][c] = x[u][c] * __builtin_amdgcn_rcpf(es[u][c]) - tr;
        gx[u][c] = gx[u][c] * es[u][c] + m[c] * gacc[u][c];
      }
    // the t-net partials into the wave's compact block (it aliases only the wave's own stage: no barrier), then
    // the block's four wave blocks summed as float4 into the layer's slab-row segment. The next stage_layer's
    // barrier orders these reads before any wave's next stage writes.
    nv_wave_sync();
    nv_put_net<PK>(red + C::TNET, ln, at);
    __syncthreads();
    for (int q = tid; q < C::LAYER / 4; q += kBlock) {
      const int o = nv_flush_lds<PK>(4 * q);
      const f32x4 v = ((*reinterpret_cast<const f32x4*>(&sScr[0][o]) + *reinterpret_cast<const f32x4*>(&sScr[1][o])) +
                       *reinterpret_cast<const f32x4*>(&sScr[2][o])) +
                      *reinterpret_cast<const f32x4*>(&sScr[3][o]);
      *reinterpret_cast<f32x4*>(row + (int64_t)l * C::LAYER + 4 * q) = v;
    }
  }
  __syncthreads();  // the last layer's sums are read: the stages and the layer image are free again
  if (E > 0) {
    put_temb();
    __syncthreads();
  }
  // ---- time-embedding backward and the loss column ----
  if (E > 0) {
    f32x4 w1 = {0.f, 0.f, 0.f, 0.f}, w2 = w1, b1 = w1, b2 = w1;
    NvV se, he, gz;
    sinusoid(se);
    nv_bcast(he, nv_vec(sT + NvM<PK>::E_B1, ln));
    nv_fwdT(sT + NvM<PK>::E_W1, ln, se, he);
#pragma unroll
    for (int u = 0; u < kNvT; ++u) he[u] = nv_celu4(he[u]);
    w2 = nv_wgrad(stage, ln, he, gtemb, w2);
    nv_bcast(gz, f32x4{0.f, 0.f, 0.f, 0.f});
    nv_fwdT(sT + NvM<PK>::E_W2T, ln, gtemb, gz);
#pragma unroll
    for (int u = 0; u < kNvT; ++u) {
      b2 += gtemb[u];
      gz[u] = nv_dact4(gz[u], he[u]);
      b1 += gz[u];
    }
    w1 = nv_wgrad(stage, ln, se, gz, w1);
    __syncthreads();  // stages done (flush blocks alias them)
    nv_put_mat(red + 0, ln, w1);
    nv_put_vec(red + 256, ln, b1);
    nv_put_mat(red + 272, ln, w2);
    nv_put_vec(red + 528, ln, b2);
    const int EE = E * E + E;
    flush(lcb, 2 * EE, [&](int f) {
      const int part = f >= EE, r = f - part * EE;
      const int o = part * 272;  // W2 / b2 columns at the temb positions
      if (r < E * E) return o + (r / E) * 16 + (part ? nv_tpos<PK>(r % E) : r % E);
      return o + 256 + (part ? nv_tpos<PK>(r - E * E) : r - E * E);
    });
  }
  lsum += __shfl_xor(lsum, 1, 64);
  lsum += __shfl_xor(lsum, 2, 64);
  lsum += __shfl_xor(lsum, 4, 64);
  lsum += __shfl_xor(lsum, 8, 64);
  if (tid % 64 == 0) red[0] = lsum;
  flush(lcb + temb_params, 1, [&](int) { return 0; });
}

// Slab column sums in two fixed-order fp64 stages (bit-reproducible): kNvSplits row splits of the
// chunk, each summed by 4 row phases of a 64-column block (4 independent loads in flight per
// lane), then the splits in order. Column c of parts is reference parameter c (n_params: the loss),
// read from slab column nv_slab_col(c). On the last chunk grad[c] = scale * acc[c] (c < n_params) and
// loss = scale * acc[n_params].
constexpr int kNvSplits = 16;
__global__ __launch_bounds__(kBlock) void nvp_slab_split_kernel(const float* __restrict__ slab_base, int rows,
                                                                 int64_t ld, NvSlabMap map, int64_t n_cols,
                                                                 double* __restrict__ parts) {
  __shared__ double part[kBlock];
  const int64_t c = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const float* slab = slab_base + (c < n_cols ? nv_slab_col(map, c) : 0);
  const int g = threadIdx.x >> 6;
  const int rps = (rows + kNvSplits - 1) / kNvSplits;
  const int r0 = blockIdx.y * rps, r1 = r0 + rps < rows ? r0 + rps : rows;
  double acc = 0.0;
  if (c < n_cols) {
    int r = r0 + g;
    for (; r + 12 < r1; r += 16) {
      const float v0 = slab[(int64_t)r * ld], v1 = slab[(int64_t)(r + 4) * ld];
      const float v2 = slab[(int64_t)(r + 8) * ld], v3 = slab[(int64_t)(r + 12) * ld];
      acc += (double)v0;
      acc += (double)v1;
      acc += (double)v2;
      acc += (double)v3;
    }
    for (; r < r1; r += 4) acc += (double)slab[(int64_t)r * ld];
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  if (g == 0 && c < n_cols)
    parts[blockIdx.y * n_cols + c] =
        ((part[threadIdx.x] + part[threadIdx.x + 64]) + part[threadIdx.x + 128]) + part[threadIdx.x + 192];
}

__global__ __launch_bounds__(kBlock) void nvp_grad_reduce_kernel(const double* __restrict__ parts,
                                                                  int64_t n_params, double* acc64,
                                                                  int first, int last, double scale,
                                                                  float* __restrict__ grad,
                                                                  float* __restrict__ loss) {
  const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (c <= n_params) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < kNvSplits; ++q) v += parts[q * (n_params + 1) + c];
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

// Packed layout where [x | temb] fits one 16-vector with x in register 0 (PDEINV_NVP_PACK=0 forces the
// identity layout, A/B).
static bool nvp_packed(const pdeinv_realnvp_desc* d) {
  static const bool pack_env = [] { const char* e = ab_env("PDEINV_NVP_PACK"); return !(e && e[0] == '0'); }();
  return pack_env && d->dim <= 4 && in_dim_of(d) - d->dim <= 12;
}
static NvSlabMap nvp_slab_map(const pdeinv_realnvp_desc* d) {
  NvSlabMap m{};
  const int E = d->ignore_time ? 0 : d->embed_time_dim;
  m.d = d->dim;
  m.n_t = in_dim_of(d) - d->dim;
  m.pk = nvp_packed(d) ? 1 : 0;
  m.n_layers = d->n_layers;
  m.layer_stride = layer_params(d->dim, in_dim_of(d));
  m.temb_params = E > 0 ? 2 * ((int64_t)E * E + E) : 0;
  m.n_params = m.temb_params + (int64_t)d->n_layers * m.layer_stride;
  m.cb = m.pk ? NvC<true>::LAYER : NvC<false>::LAYER;
  return m;
}

static int64_t nvp_grad_rows(int64_t n) {
  const int64_t tiles = (n + kNvSPB - 1) / kNvSPB;
  return tiles < kNvpMaxRows ? tiles : kNvpMaxRows;
}

extern "C" int64_t pdeinv_realnvp_grad_workspace(const pdeinv_realnvp_desc* d, int64_t n) {
  const int64_t P = pdeinv_realnvp_param_count(d);
  if (P < 0 || n < 0) return -1;
  const int64_t slab = nvp_grad_rows(n) * nv_slab_ld(nvp_slab_map(d)) * (int64_t)sizeof(float);
  return slab + (1 + kNvSplits) * (P + 1) * (int64_t)sizeof(double);
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
  const NvSlabMap map = nvp_slab_map(d);
  const int64_t sld = nv_slab_ld(map);
  float* slab = (float*)workspace;
  double* acc64 = (double*)((char*)workspace + rows_max * sld * (int64_t)sizeof(float));
  double* parts = acc64 + (P + 1);
  hipStream_t st = (hipStream_t)stream;
  const int64_t tiles = (n + kNvSPB - 1) / kNvSPB;
  // any d <= 8 (padded coordinates stay fixed); celu and elu are the same map.
  const bool packed = map.pk != 0;
  for (int64_t tile0 = 0; tile0 < tiles; tile0 += rows_max) {
    const int64_t rows = tiles - tile0 < rows_max ? tiles - tile0 : rows_max;
    const dim3 g((unsigned)rows);
    if (packed)
      hipLaunchKernelGGL((realnvp_grad_kernel<PDEINV_ACT_CELU, true>), g, dim3(kBlock), 0, st, a, D, params, t,
                         t_stride, x, n, ld, ls, P, tile0, slab, sld);
    else
      hipLaunchKernelGGL((realnvp_grad_kernel<PDEINV_ACT_CELU, false>), g, dim3(kBlock), 0, st, a, D, params, t,
                         t_stride, x, n, ld, ls, P, tile0, slab, sld);
    int rc = check_launch("realnvp_grad_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(nvp_slab_split_kernel, dim3((unsigned)((P + 1 + 63) / 64), kNvSplits), dim3(kBlock), 0, st,
                       slab, (int)rows, sld, map, P + 1, parts);
    rc = check_launch("nvp_slab_split_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(nvp_grad_reduce_kernel, dim3((unsigned)((P + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       parts, P, acc64, tile0 == 0 ? 1 : 0, tile0 + rows >= tiles ? 1 : 0, -1.0 / (double)n, grad,
                       loss);
    rc = check_launch("nvp_grad_reduce_kernel");
    if (rc) return rc;
  }
  return PDEINV_OK;
}
