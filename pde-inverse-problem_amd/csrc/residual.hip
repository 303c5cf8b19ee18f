// residual.hip — PDE-consistency residuals and their parameter gradients (gfx950).
//
// Replaces methods/consistency_instances/kinetic_fokker_planck.py:11-69 (value_and_grad_fn):
// the reference evaluates grad V_theta (vmap(grad)), v^T Hess V_theta v (vmap(jvp∘grad)) and
// grad V* per sample and then differentiates the whole loss with jax.value_and_grad. Here
//  * the parametric quadratic model reduces exactly to moments (moments.hip / the fused
//    simulator) plus this O(d^3) finalize, and
//  * the parametric GMM model runs one fused per-sample pass with the analytic adjoint
//    d loss / d mu, HBM-bound on the 8d bytes per sample.
#include <math.h>

#include "common.h"

namespace pdeinv {

// =========================================================================================
// KFP residual, V_theta(x) = x^T K x + b^T x — finalize from the three moment sets
// =========================================================================================
struct KfpQuadArgs {
  int d;
  float gamma, T;
  float F[PDEINV_MAX_DIM * PDEINV_MAX_DIM];
};

// Moment accessors over the packed fp64 layout [count, sum z (m), sum z_i z_j (i<=j)].
struct MomView {
  const double* v;
  int m;
  double inv;
  __device__ MomView(const double* p, int m_) : v(p), m(m_), inv(p[0] > 0 ? 1.0 / p[0] : 0.0) {}
  __device__ double mean(int i) const { return v[1 + i] * inv; }
  __device__ double M(int i, int j) const {  // E[z_i z_j]
    if (i > j) { const int t = i; i = j; j = t; }
    return v[1 + m + i * m - i * (i - 1) / 2 + (j - i)] * inv;
  }
};

// One block; thread t < d*d owns entry (i, j) = (t / d, t % d) of every d x d quantity, the
// scalar terms are block sums. Gradient derivation: oracle/numpy_ref.py
// kfp_quadratic_from_moments (checked there against central finite differences).
__global__ __launch_bounds__(kBlock) void kfp_quadratic_finalize_kernel(KfpQuadArgs a,
                                                                        const double* __restrict__ mom,
                                                                        const float* __restrict__ theta,
                                                                        float* __restrict__ out,
                                                                        float* __restrict__ grad) {
  const int d = a.d, m = 2 * d, L = moment_len(m);
  const MomView si(mom, m), s0(mom + L, m), st(mom + 2 * L, m);
  auto S = [&](int i, int j) { return (double)theta[i * d + j] + (double)theta[j * d + i]; };
  auto b = [&](int i) { return (double)theta[d * d + i]; };
  auto F = [&](int i, int j) { return (double)a.F[i * d + j]; };
  const double g = a.gamma, T = a.T;
  // scalars: nabla, hess, fric(raw), init, term, true, gt, |grad|^2
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int t = threadIdx.x;
  if (t < d * d) {
    const int i = t / d, j = t % d;
    double SM = 0, MS = 0, SMji = 0, MSji = 0, FMF = 0, DMD = 0;
    for (int k = 0; k < d; ++k) {
      SM += S(i, k) * s0.M(k, j);
      MS += s0.M(i, k) * S(k, j);
      SMji += S(j, k) * s0.M(k, i);
      MSji += s0.M(j, k) * S(k, i);
      FMF += s0.M(j, k) * F(i, k);
      DMD += s0.M(j, k) * (F(i, k) - S(i, k));
    }
    acc[0] = SM * S(j, i);                    // tr(S Mxx S)
    acc[1] = S(i, j) * s0.M(d + j, d + i);    // tr(S Mvv)
    acc[2] = S(i, j) * s0.M(j, d + i);        // tr(S Mxv), Mxv[j][i] = E[x_j v_i]
    acc[3] = S(i, j) * si.M(j, d + i);
    acc[4] = S(i, j) * st.M(j, d + i);
    acc[5] = F(i, j) * FMF;                   // tr(F Mxx F^T)
    acc[6] = (F(i, j) - S(i, j)) * DMD;       // tr(D Mxx D^T), D = F - S
    // d loss / d S entries, then d/dK = G + G^T
    const double Gij = SM + MS + 2 * b(i) * s0.mean(j) - 2 * s0.M(d + i, d + j) + 2 * g * s0.M(d + i, j) +
                       (-2 * si.M(d + i, j) + 2 * st.M(d + i, j)) / T;
    const double Gji = SMji + MSji + 2 * b(j) * s0.mean(i) - 2 * s0.M(d + j, d + i) + 2 * g * s0.M(d + j, i) +
                       (-2 * si.M(d + j, i) + 2 * st.M(d + j, i)) / T;
    const double gk = Gij + Gji;
    grad[i * d + j] = (float)gk;
    acc[7] = gk * gk;
  }
  if (t < d) {
    const int i = t;
    double Sex = 0, De = 0;
    for (int k = 0; k < d; ++k) {
      Sex += S(i, k) * s0.mean(k);
      De += (F(i, k) - S(i, k)) * s0.mean(k);
    }
    acc[0] += 2 * b(i) * Sex + b(i) * b(i);
    acc[2] += b(i) * s0.mean(d + i);
    acc[3] += b(i) * si.mean(d + i);
    acc[4] += b(i) * st.mean(d + i);
    acc[6] += -2 * b(i) * De + b(i) * b(i);
    const double gb = 2 * Sex + 2 * b(i) + 2 * g * s0.mean(d + i) + (-2 * si.mean(d + i) + 2 * st.mean(d + i)) / T;
    grad[d * d + i] = (float)gb;
    acc[7] += gb * gb;
  }
  __shared__ double red[kWavesPerBlock][8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    double v = acc[c];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((t & 63) == 0) red[t >> 6][c] = v;
  }
  __syncthreads();
  if (t == 0) {
    double r[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) r[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    const double nabla = r[0], hess = r[1], fric = r[2], init = r[3], term = r[4], tru = r[5];
    out[PDEINV_KFP_LOSS] = (float)(nabla - 2 * hess + 2 * g * fric + tru + (-2 * init + 2 * term) / T);
    out[PDEINV_KFP_LOSS_GT] = (float)r[6];
    out[PDEINV_KFP_GRAD_NORM] = (float)sqrt(r[7]);
    out[PDEINV_KFP_NABLA] = (float)nabla;
    out[PDEINV_KFP_HESSIAN] = (float)hess;
    out[PDEINV_KFP_FRICTION] = (float)(g * fric);
    out[PDEINV_KFP_NABLA_TRUE] = (float)tru;
    out[PDEINV_KFP_INITIAL] = (float)init;
    out[PDEINV_KFP_TERMINAL] = (float)term;
  }
}

// =========================================================================================
// KFP residual, V_theta = GMM(mu) — fused per-sample forward + analytic adjoint
// =========================================================================================
struct GmmResArgs {
  int K, KT;
  float s2, l2s, s2t, l2st;  // 1/sigma^2 and log2(e)/sigma^2
  int64_t n0, ni, nt, ld0, ldi, ldt;
  const float* z0T;
  const float* zi;
  const float* zt;
  float c_nabla, c_hess, c_fric, c_true, c_init, c_term, inv_ni, inv_nt;
  float mus_true[PDEINV_MAX_PARAMS];
};

constexpr int kGmmGridCap = 1024;

template <int D, int KM>
__global__ __launch_bounds__(kBlock) void kfp_gmm_kernel(GmmResArgs a, const float* __restrict__ mus,
                                                         float* __restrict__ partials) {
  constexpr int NS = PDEINV_GMM_NACC;
  // model and true GMM in centre-pair layout (common.h GmmPairs) in LDS, read with wave-uniform
  // broadcasts: pinned in VGPRs they took 2 (K d + K) registers beside the adjoint accumulators
  // (155 VGPRs, occupancy 3)
  __shared__ GmmPairs<D, KM> cen[2];
  GmmPairs<D, KM>& cm = cen[0];
  GmmPairs<D, KM>& ct = cen[1];
  for (int k = threadIdx.x; k < KM; k += kBlock) {
    cm.set(k, a.K, mus, a.l2s);
    ct.set(k, a.KT, a.mus_true, a.l2st);
  }
  __syncthreads();
  float acc[NS];
#pragma unroll
  for (int c = 0; c < NS; ++c) acc[c] = 0.f;
  GmmAdjAcc<D, KM> adj;
  adj.zero();

  const int64_t total = a.n0 + a.ni + a.nt;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const float s2 = a.s2;
  auto row_of = [&](int64_t r, int& set) -> const float* {
    if (r < a.n0) { set = 0; return a.z0T + r * a.ld0; }
    if (r < a.n0 + a.ni) { set = 1; return a.zi + (r - a.n0) * a.ldi; }
    set = 2;
    return a.zt + (r - a.n0 - a.ni) * a.ldt;
  };
  // software pipeline: the next row is loaded before the current one is processed (only a few
  // waves fit per SIMD at this register count, so the load latency must hide behind ALU work)
  int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  int set_n = 0;
  float xn[D], vn[D];
  if (r < total) {
    const float* row = row_of(r, set_n);
#pragma unroll
    for (int i = 0; i < D; ++i) { xn[i] = row[i]; vn[i] = row[D + i]; }
  }
  for (; r < total; r += stride) {
    // re-read the LDS centres every sample (hoisted out of the loop they take the registers the LDS
    // layout exists to save)
    asm volatile("" ::: "memory");
    const int set = set_n;
    float x[D], v[D];
#pragma unroll
    for (int i = 0; i < D; ++i) { x[i] = xn[i]; v[i] = vn[i]; }
    if (r + stride < total) {
      const float* row = row_of(r + stride, set_n);
#pragma unroll
      for (int i = 0; i < D; ++i) { xn[i] = row[i]; vn[i] = row[D + i]; }
    }

    const float c1 = set == 0 ? a.c_nabla : 0.f;
    const float c2 = set == 0 ? a.c_hess : 0.f;
    const float c3 = set == 0 ? a.c_fric : (set == 1 ? a.c_init : a.c_term);
    float g[D], T1, T2, T3;
    gmm_residual_sample<D, KM>(cm.mu, cm.c, s2, a.l2s, x, v, c1, c2, c3, adj, g, T1, T2, T3);
    acc[PDEINV_GMM_ACC_LOSS] += c1 * T1 + c2 * T2 + c3 * T3;
    if (set == 0) {
      float gt[D];
      gmm_grad<D, KM>(ct.mu, ct.c, a.l2st, a.s2t, x, gt);
      float Tt = 0.f, Tgt = 0.f;
#pragma unroll
      for (int i = 0; i < D; ++i) {
        Tt = fmaf(gt[i], gt[i], Tt);
        Tgt = fmaf(gt[i] - g[i], gt[i] - g[i], Tgt);
      }
      acc[PDEINV_GMM_ACC_LOSS] += a.c_true * Tt;
      acc[PDEINV_GMM_ACC_LOSS_GT] += a.c_true * Tgt;
      acc[PDEINV_GMM_ACC_NABLA] += a.c_true * T1;
      acc[PDEINV_GMM_ACC_HESSIAN] += a.c_true * T2;
      acc[PDEINV_GMM_ACC_FRICTION] += a.c_true * T3;
      acc[PDEINV_GMM_ACC_NABLA_TRUE] += a.c_true * Tt;
    } else if (set == 1) {
      acc[PDEINV_GMM_ACC_INITIAL] += a.inv_ni * T3;
    } else {
      acc[PDEINV_GMM_ACC_TERMINAL] += a.inv_nt * T3;
    }
  }
  float flat[NS + KM * D];
#pragma unroll
  for (int c = 0; c < NS; ++c) flat[c] = acc[c];
  gmm_adjoint_flat<D, KM>(adj, cm.mu, flat + NS);
  __shared__ float lds[kWavesPerBlock * (NS + KM * D)];
  block_reduce_to_slab(flat, NS + a.K * D, lds, partials, blockIdx.x, gridDim.x);
}

__global__ void kfp_gmm_finalize_kernel(int n_grad, float gamma, const double* __restrict__ acc,
                                        float* __restrict__ out, float* __restrict__ grad) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double gn = 0.0;
  for (int k = 0; k < n_grad; ++k) {
    const double g = acc[PDEINV_GMM_NACC + k];
    grad[k] = (float)g;
    gn += g * g;
  }
  out[PDEINV_KFP_LOSS] = (float)acc[PDEINV_GMM_ACC_LOSS];
  out[PDEINV_KFP_LOSS_GT] = (float)acc[PDEINV_GMM_ACC_LOSS_GT];
  out[PDEINV_KFP_GRAD_NORM] = (float)sqrt(gn);
  out[PDEINV_KFP_NABLA] = (float)acc[PDEINV_GMM_ACC_NABLA];
  out[PDEINV_KFP_HESSIAN] = (float)acc[PDEINV_GMM_ACC_HESSIAN];
  out[PDEINV_KFP_FRICTION] = (float)(gamma * acc[PDEINV_GMM_ACC_FRICTION]);
  out[PDEINV_KFP_NABLA_TRUE] = (float)acc[PDEINV_GMM_ACC_NABLA_TRUE];
  out[PDEINV_KFP_INITIAL] = (float)acc[PDEINV_GMM_ACC_INITIAL];
  out[PDEINV_KFP_TERMINAL] = (float)acc[PDEINV_GMM_ACC_TERMINAL];
}

// =========================================================================================
// GMM potential value / gradient over a batch (core/potential.py:48-61)
// =========================================================================================
struct GmmPotArgs {
  int K;
  float s2, nh_s2_l2e;
  int64_t n, ld;
  float mus[PDEINV_MAX_PARAMS];
};

template <int D>
__global__ __launch_bounds__(kBlock) void gmm_potential_kernel(GmmPotArgs a, const float* __restrict__ x_in,
                                                               float* __restrict__ value,
                                                               float* __restrict__ grad) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= a.n) return;
  float x[D];
#pragma unroll
  for (int i = 0; i < D; ++i) x[i] = x_in[r * a.ld + i];
  float al[16], amax = -INFINITY;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k < a.K) {
      float d2 = 0.f;
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const float t = x[i] - a.mus[k * D + i];
        d2 = fmaf(t, t, d2);
      }
      al[k] = d2 * a.nh_s2_l2e;
      amax = fmaxf(amax, al[k]);
    }
  }
  float den = 0.f, accm[D];
#pragma unroll
  for (int i = 0; i < D; ++i) accm[i] = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k < a.K) {
      const float e = __builtin_amdgcn_exp2f(al[k] - amax);
      den += e;
#pragma unroll
      for (int i = 0; i < D; ++i) accm[i] = fmaf(e, a.mus[k * D + i], accm[i]);
    }
  }
  // V = -logsumexp(a) = -(amax + log(den)) in natural units
  if (value) value[r] = -(amax + __builtin_amdgcn_logf(den)) * 0.6931471805599453f;
  if (grad) {
    const float inv = 1.f / den;
#pragma unroll
    for (int i = 0; i < D; ++i) grad[r * D + i] = a.s2 * (x[i] - accm[i] * inv);
  }
}

}  // namespace pdeinv

using namespace pdeinv;

extern "C" int pdeinv_residual_kfp_quadratic(const pdeinv_kfp_quad_desc* d, const double* mom,
                                             const float* theta, float* out, float* grad,
                                             void* stream) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "kfp_quadratic: null descriptor");
  PDEINV_REQUIRE(d->dim >= 1 && d->dim <= PDEINV_MAX_DIM, PDEINV_ERR_UNSUPPORTED,
                 "kfp_quadratic: dim must be in [1, 16]");
  PDEINV_REQUIRE(mom && theta && out && grad, PDEINV_ERR_INVALID, "kfp_quadratic: null pointer");
  PDEINV_REQUIRE(d->tilde_F != nullptr, PDEINV_ERR_INVALID, "kfp_quadratic: tilde_F is null");
  PDEINV_REQUIRE(std::isfinite(d->total_time) && d->total_time > 0.f, PDEINV_ERR_INVALID,
                 "kfp_quadratic: total_time must be > 0");
  KfpQuadArgs a{};
  a.d = d->dim;
  a.gamma = d->gamma;
  a.T = d->total_time;
  for (int k = 0; k < d->dim * d->dim; ++k) a.F[k] = d->tilde_F[k];
  hipLaunchKernelGGL(kfp_quadratic_finalize_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, a,
                     mom, theta, out, grad);
  return check_launch("kfp_quadratic_finalize_kernel");
}

static int gmm_grid(int64_t total) {
  int g = grid_for(total);
  return g < 1 ? 1 : (g > kGmmGridCap ? kGmmGridCap : g);
}

static int gmm_km(int D, int K) {
  int km = K <= 4 ? 4 : (K <= 8 ? 8 : 16);
  while (km * D > 128 && km > 4) km /= 2;
  return (K <= km) ? km : 0;
}

extern "C" size_t pdeinv_residual_kfp_gmm_workspace_bytes(const pdeinv_kfp_gmm_desc* d, int64_t ni,
                                                          int64_t nt, int64_t n0) {
  if (!d || d->dim < 1 || d->n_centers < 1) return 0;
  return (size_t)(PDEINV_GMM_NACC + d->n_centers * d->dim) * gmm_grid(ni + nt + n0) * sizeof(float);
}

template <int D, int KM>
static void launch_gmm(const GmmResArgs& a, const float* mus, float* ws, int g, hipStream_t st) {
  hipLaunchKernelGGL((kfp_gmm_kernel<D, KM>), dim3(g), dim3(kBlock), 0, st, a, mus, ws);
}

template <int D>
static int dispatch_gmm(int km, const GmmResArgs& a, const float* mus, float* ws, int g, hipStream_t st) {
  if (km == 4) launch_gmm<D, 4>(a, mus, ws, g, st);
  else if (km == 8) launch_gmm<D, 8>(a, mus, ws, g, st);
  else if constexpr (D <= 8) launch_gmm<D, 16>(a, mus, ws, g, st);
  else return fail(PDEINV_ERR_UNSUPPORTED, "kfp_gmm: n_centers too large for dim");
  return PDEINV_OK;
}

extern "C" int pdeinv_residual_kfp_gmm(const pdeinv_kfp_gmm_desc* d, const float* zi, int64_t ni,
                                       int64_t ldi, const float* zt, int64_t nt, int64_t ldt,
                                       const float* z0, int64_t n0, int64_t ld0, const float* mus,
                                       void* ws, double* acc, void* stream) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "kfp_gmm: null descriptor");
  const int D = d->dim;
  PDEINV_REQUIRE(D >= 1 && D <= 16, PDEINV_ERR_UNSUPPORTED, "kfp_gmm: dim must be in [1, 16]");
  PDEINV_REQUIRE(d->n_centers >= 1 && d->n_centers_true >= 1 && d->n_centers_true <= 16,
                 PDEINV_ERR_UNSUPPORTED, "kfp_gmm: need 1 <= n_centers, n_centers_true <= 16");
  const int km = gmm_km(D, d->n_centers >= d->n_centers_true ? d->n_centers : d->n_centers_true);
  PDEINV_REQUIRE(km > 0, PDEINV_ERR_UNSUPPORTED, "kfp_gmm: n_centers * dim exceeds 128 registers");
  PDEINV_REQUIRE(ni >= 0 && nt >= 0 && n0 >= 1, PDEINV_ERR_INVALID, "kfp_gmm: 0T set must be non-empty");
  PDEINV_REQUIRE(mus && ws && acc && z0 && (ni == 0 || zi) && (nt == 0 || zt), PDEINV_ERR_INVALID,
                 "kfp_gmm: null pointer");
  PDEINV_REQUIRE(d->mus_true != nullptr, PDEINV_ERR_INVALID, "kfp_gmm: mus_true is null");
  PDEINV_REQUIRE(d->sigma > 0.f && d->sigma_true > 0.f, PDEINV_ERR_INVALID, "kfp_gmm: sigma must be > 0");
  GmmResArgs a{};
  a.K = d->n_centers;
  a.KT = d->n_centers_true;
  a.s2 = 1.f / (d->sigma * d->sigma);
  a.l2s = a.s2 * 1.4426950408889634f;
  a.s2t = 1.f / (d->sigma_true * d->sigma_true);
  a.l2st = a.s2t * 1.4426950408889634f;
  a.n0 = n0; a.ni = ni; a.nt = nt;
  a.ld0 = ld0 ? ld0 : 2 * D; a.ldi = ldi ? ldi : 2 * D; a.ldt = ldt ? ldt : 2 * D;
  PDEINV_REQUIRE(a.ld0 >= 2 * D && a.ldi >= 2 * D && a.ldt >= 2 * D, PDEINV_ERR_INVALID,
                 "kfp_gmm: row stride < 2*dim");
  a.z0T = z0; a.zi = zi; a.zt = zt;
  a.c_nabla = d->c_nabla; a.c_hess = d->c_hess; a.c_fric = d->c_fric; a.c_true = d->c_true;
  a.c_init = d->c_init; a.c_term = d->c_term;
  a.inv_ni = ni ? 1.f / (float)ni : 0.f;
  a.inv_nt = nt ? 1.f / (float)nt : 0.f;
  for (int k = 0; k < d->n_centers_true * D; ++k) a.mus_true[k] = d->mus_true[k];
  hipStream_t st = (hipStream_t)stream;
  const int g = gmm_grid(n0 + ni + nt);
  float* wsf = (float*)ws;
  int rc = PDEINV_OK;
  switch (D) {
#define CASE(DD) case DD: rc = dispatch_gmm<DD>(km, a, mus, wsf, g, st); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(10) CASE(12) CASE(16)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "kfp_gmm: dim must be one of 1-8, 10, 12, 16");
  }
  if (rc) return rc;
  rc = check_launch("kfp_gmm_kernel");
  if (rc) return rc;
  launch_slab_reduce(wsf, g, PDEINV_GMM_NACC + a.K * D, acc, st);
  return check_launch("slab_reduce_kernel");
}

extern "C" int pdeinv_residual_kfp_gmm_finalize(const pdeinv_kfp_gmm_desc* d, const double* acc,
                                                float* out, float* grad, void* stream) {
  PDEINV_REQUIRE(d && acc && out && grad, PDEINV_ERR_INVALID, "kfp_gmm_finalize: null pointer");
  hipLaunchKernelGGL(kfp_gmm_finalize_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     d->n_centers * d->dim, d->gamma, acc, out, grad);
  return check_launch("kfp_gmm_finalize_kernel");
}

extern "C" int pdeinv_gmm_potential(int32_t D, int32_t K, float sigma, const float* mus_host,
                                    const float* x, int64_t n, int64_t ld, float* value,
                                    float* grad, void* stream) {
  PDEINV_REQUIRE(D >= 1 && D <= 16 && K >= 1 && K <= 16 && K * D <= PDEINV_MAX_PARAMS,
                 PDEINV_ERR_UNSUPPORTED, "gmm_potential: need dim <= 16, 1 <= K <= 16");
  PDEINV_REQUIRE(sigma > 0.f && mus_host != nullptr, PDEINV_ERR_INVALID, "gmm_potential: bad sigma / mus");
  PDEINV_REQUIRE(n >= 0, PDEINV_ERR_INVALID, "gmm_potential: n < 0");
  if (n == 0) return PDEINV_OK;
  PDEINV_REQUIRE(x != nullptr, PDEINV_ERR_INVALID, "gmm_potential: x is null");
  GmmPotArgs a{};
  a.K = K;
  a.s2 = 1.f / (sigma * sigma);
  a.nh_s2_l2e = -0.5f * a.s2 * 1.4426950408889634f;
  a.n = n;
  a.ld = ld ? ld : D;
  PDEINV_REQUIRE(a.ld >= D, PDEINV_ERR_INVALID, "gmm_potential: ld < dim");
  for (int k = 0; k < K * D; ++k) a.mus[k] = mus_host[k];
  hipStream_t st = (hipStream_t)stream;
  switch (D) {
#define CASE(DD) case DD: hipLaunchKernelGGL(gmm_potential_kernel<DD>, dim3(grid_for(n)), dim3(kBlock), 0, st, a, x, value, grad); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(10) CASE(12) CASE(16)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "gmm_potential: dim must be one of 1-8, 10, 12, 16");
  }
  return check_launch("gmm_potential_kernel");
}
