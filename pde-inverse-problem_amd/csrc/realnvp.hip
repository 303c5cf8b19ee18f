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
