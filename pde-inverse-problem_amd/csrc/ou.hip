// ou.hip — the exact kinetic-OU sampler on the device (example_problems/kinetic_fokker_planck_example_OU.py:140-156).
//
// The reference's default KOU data (sample_scheme "exact", random_time mode) are groups of 100 rows, each group
// drawn from N(m(t_g), P(t_g)) at its own random time t_g ~ U(1e-4, T): it integrates m' = F m,
// P' = F P + P F^T + L with odeint per time (:73-106) and takes an SVD square root per group (distribution.py:52-65).
// Here one workgroup per group does all of it in fp64 in LDS — no host round trip per iteration:
//   t_g     = tmin + (tmax - tmin) u_g, u_g from Philox (seed; g, ctr, 0xD0000000) (24 random bits), or given;
//   X       = exp(B t_g), B = [[-F, L], [0, F^T]] (Van Loan), by the same scaled Taylor sum as the host
//             ou_moments_batched: X = (sum_k (t_g / 2^s)^k / k! B^k)^(2^s), the powers B^k precomputed once
//             per problem on the host (a (K+1) x 2n x 2n fp64 table, read through L2 by every group);
//   E       = exp(F t_g) = X[n:, n:]^T, m = E m0, P = E (P0 E^T + X[:n, n:]), symmetrised;
//   R       = the lower Cholesky factor of P (R R^T = P; a non-positive pivot zeroes its column: the PSD limit);
//   rows    = m + R xi, xi the grouped Gaussian sampler's own Philox / Box–Muller stream (sampling.hip), so the
//             rows equal pdeinv_gaussian_sample_grouped(means, factors) given the same means and factors.
#include <math.h>

#include "common.h"

namespace pdeinv {

struct OuArgs {
  int32_t n, K, s;            // n = 2d (<= 32); Taylor degree K; squarings s
  int64_t G, rows_per_group, row_off;
  double tmin, tspan;
  uint32_t k0, k1, ctr_t, ctr_z;
  const double* pw;           // [(K + 1), 2n, 2n]
  const double* m0;           // [n]
  const double* P0;           // [n, n]
  const float* t_in;          // [G] or null (draw)
  float* t_out;               // [G] or null
  float* mean_out;            // [G, n] or null
  float* factor_out;          // [G, n, n] or null
  float* out;                 // [G * rows_per_group, n]
};

// one row of the grouped sampler (gaussian_sample_kernel<M>, sampling.hip): same Philox blocks, same FMA order
template <int M>
__device__ __forceinline__ void ou_row(uint32_t k0, uint32_t k1, uint32_t ctr_z, uint64_t gid, const float* mean,
                                       const float* ch, float* dst) {
  float xi[M];
#pragma unroll
  for (int j = 0; 4 * j < M; ++j) {
    const uint4 b = philox4x32_10(make_uint4((uint32_t)gid, (uint32_t)(gid >> 32), ctr_z, 0x40000000u | (uint32_t)j),
                                  k0, k1);
    float z[4];
    box_muller(b.x, b.y, z[0], z[1]);
    box_muller(b.z, b.w, z[2], z[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * j + k < M) xi[4 * j + k] = z[k];
  }
#pragma unroll M <= 16 ? M : 1
  for (int i = 0; i < M; ++i) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < M; ++j) acc = fmaf(ch[i * M + j], xi[j], acc);
    dst[i] = acc + mean[i];
  }
}

// M = n = 2d (compile-time: LDS sizes and the row sampler)
template <int M>
__global__ __launch_bounds__(kBlock) void ou_exact_sample_kernel(OuArgs a) {
  constexpr int n = M, n2 = 2 * M;
  __shared__ double X[n2 * n2], Y[n2 * n2];
  __shared__ double Pm[n * n];
  __shared__ double mv[n];
  __shared__ float meanf[n], chf[n * n];
  __shared__ double coef[32];
  const int64_t g = blockIdx.x;
  const int tid = threadIdx.x;
  double t;
  if (a.t_in) {
    t = (double)a.t_in[g];
  } else {
    const uint4 r = philox4x32_10(make_uint4((uint32_t)g, (uint32_t)((uint64_t)g >> 32), a.ctr_t, 0xD0000000u), a.k0,
                                  a.k1);
    t = (double)(float)(a.tmin + a.tspan * (double)u32_unit(r.x));  // the fp32 time t_out reports is the one used
  }
  if (tid == 0) {
    if (a.t_out) a.t_out[g] = (float)t;
    const double tau = t / (double)(1 << a.s);
    double c = 1.0;
    coef[0] = 1.0;
    for (int k = 1; k <= a.K; ++k) {
      c = c * tau / (double)k;
      coef[k] = c;
    }
  }
  __syncthreads();
  // X = sum_k coef_k B^k
  for (int e = tid; e < n2 * n2; e += kBlock) {
    double acc = 0.0;
    for (int k = 0; k <= a.K; ++k) acc = fma(coef[k], a.pw[(int64_t)k * n2 * n2 + e], acc);
    X[e] = acc;
  }
  __syncthreads();
  double* src = X;
  double* dst = Y;
  for (int q = 0; q < a.s; ++q) {  // X <- X X
    for (int e = tid; e < n2 * n2; e += kBlock) {
      const int i = e / n2, j = e - i * n2;
      double acc = 0.0;
      for (int k = 0; k < n2; ++k) acc = fma(src[i * n2 + k], src[k * n2 + j], acc);
      dst[e] = acc;
    }
    __syncthreads();
    double* t2 = src;
    src = dst;
    dst = t2;
  }
  // E[i][j] = src[(n + j) * n2 + n + i];  Gv[i][j] = src[i * n2 + n + j]
  auto E = [&](int i, int j) { return src[(n + j) * n2 + n + i]; };
  // T1 = P0 E^T + Gv  -> dst (n x n)
  for (int e = tid; e < n * n; e += kBlock) {
    const int i = e / n, j = e - i * n;
    double acc = src[i * n2 + n + j];
    for (int k = 0; k < n; ++k) acc = fma(a.P0[i * n + k], E(j, k), acc);
    dst[e] = acc;
  }
  if (tid < n) {
    double acc = 0.0;
    for (int k = 0; k < n; ++k) acc = fma(E(tid, k), a.m0[k], acc);
    mv[tid] = acc;
  }
  __syncthreads();
  for (int e = tid; e < n * n; e += kBlock) {  // P = E T1
    const int i = e / n, j = e - i * n;
    double acc = 0.0;
    for (int k = 0; k < n; ++k) acc = fma(E(i, k), dst[k * n + j], acc);
    Pm[e] = acc;
  }
  __syncthreads();
  // symmetrise into src (free now: E was consumed), then Cholesky in place (lower), one column per step
  double* C = src == X ? Y : X;  // not dst (holds T1, done) — any free buffer of n*n: use the one E is not in
  for (int e = tid; e < n * n; e += kBlock) {
    const int i = e / n, j = e - i * n;
    C[e] = 0.5 * (Pm[i * n + j] + Pm[j * n + i]);
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    if (tid == 0) {
      double dd = C[j * n + j];
      for (int k = 0; k < j; ++k) dd -= C[j * n + k] * C[j * n + k];
      C[j * n + j] = dd > 0.0 ? sqrt(dd) : 0.0;
    }
    __syncthreads();
    const double piv = C[j * n + j];
    for (int i = j + 1 + tid; i < n; i += kBlock) {
      double v = C[i * n + j];
      for (int k = 0; k < j; ++k) v -= C[i * n + k] * C[j * n + k];
      C[i * n + j] = piv > 0.0 ? v / piv : 0.0;
    }
    __syncthreads();
  }
  for (int e = tid; e < n * n; e += kBlock) {
    const int i = e / n, j = e - i * n;
    const float v = j <= i ? (float)C[e] : 0.f;
    chf[e] = v;
    if (a.factor_out) a.factor_out[g * n * n + e] = v;
  }
  if (tid < n) {
    meanf[tid] = (float)mv[tid];
    if (a.mean_out) a.mean_out[g * n + tid] = (float)mv[tid];
  }
  __syncthreads();
  for (int64_t r = tid; r < a.rows_per_group; r += kBlock) {  // factor and mean read from LDS (broadcast)
    const int64_t row = g * a.rows_per_group + r;
    ou_row<M>(a.k0, a.k1, a.ctr_z, (uint64_t)(a.row_off + row), meanf, chf, a.out + row * M);
  }
}

}  // namespace pdeinv

using namespace pdeinv;

extern "C" int pdeinv_ou_exact_sample(const pdeinv_ou_desc* d, int64_t n_groups, int64_t rows_per_group,
                                      uint64_t seed, uint32_t ctr_t, uint32_t ctr_z, int64_t row_off,
                                      const float* t_in, float* t_out, float* mean_out, float* factor_out, float* out,
                                      void* stream) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "ou_exact_sample: null descriptor");
  PDEINV_REQUIRE(d->n >= 2 && d->n <= 2 * PDEINV_MAX_DIM && d->n % 2 == 0, PDEINV_ERR_UNSUPPORTED,
                 "ou_exact_sample: dim must be in [1, 16]");
  PDEINV_REQUIRE(d->taylor_degree >= 1 && d->taylor_degree <= 30 && d->squarings >= 0 && d->squarings <= 30,
                 PDEINV_ERR_INVALID, "ou_exact_sample: need 1 <= taylor_degree <= 30, 0 <= squarings <= 30");
  PDEINV_REQUIRE(n_groups >= 0 && rows_per_group >= 0 && row_off >= 0 && n_groups <= 0x7FFFFFFF, PDEINV_ERR_INVALID,
                 "ou_exact_sample: bad group sizes");
  PDEINV_REQUIRE(std::isfinite(d->t_min) && std::isfinite(d->t_max) && d->t_max >= d->t_min, PDEINV_ERR_INVALID,
                 "ou_exact_sample: need t_min <= t_max");
  if (n_groups == 0) return PDEINV_OK;
  PDEINV_REQUIRE(d->d_powers && d->d_m0 && d->d_P0 && (out || rows_per_group == 0), PDEINV_ERR_INVALID,
                 "ou_exact_sample: null pointer");
  OuArgs a{};
  a.n = d->n;
  a.K = d->taylor_degree;
  a.s = d->squarings;
  a.G = n_groups;
  a.rows_per_group = rows_per_group;
  a.row_off = row_off;
  a.tmin = d->t_min;
  a.tspan = d->t_max - d->t_min;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.ctr_t = ctr_t;
  a.ctr_z = ctr_z;
  a.pw = d->d_powers;
  a.m0 = d->d_m0;
  a.P0 = d->d_P0;
  a.t_in = t_in;
  a.t_out = t_out;
  a.mean_out = mean_out;
  a.factor_out = factor_out;
  a.out = out;
  hipStream_t st = (hipStream_t)stream;
  switch (d->n) {
#define CASE(MM) case MM: hipLaunchKernelGGL(ou_exact_sample_kernel<MM>, dim3((unsigned)n_groups), dim3(kBlock), 0, st, a); break;
    CASE(2) CASE(4) CASE(6) CASE(8) CASE(10) CASE(12) CASE(14) CASE(16) CASE(18) CASE(20) CASE(22) CASE(24)
    CASE(26) CASE(28) CASE(30) CASE(32)
#undef CASE
  }
  return check_launch("ou_exact_sample_kernel");
}
