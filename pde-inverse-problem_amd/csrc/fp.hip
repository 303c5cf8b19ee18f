// fp.hip — overdamped Fokker–Planck pieces (gfx950): the exact per-sample-time sampler and the
// row layout that turns the overdamped residual's Laplacian into Taylor-mode directions.
//
// Reference: example_problems/fokker_planck_example.py (OU_process :48-55, sample_ground_truth
// :88-96 — one random time per sample, vmapped) and methods/consistency_instances/
// fokker_planck.py:33-63 (loss with laplacian_V = trace(jacfwd(grad V))).
#include <math.h>

#include "common.h"

namespace pdeinv {

constexpr int kFpMaxDim = 8;

struct FpArgs {
  int64_t n, row_off;
  uint32_t k0, k1, ctr;
  float t_lo, t_span;
  float U[kFpMaxDim * kFpMaxDim], s[kFpMaxDim], Um0[kFpMaxDim];
  float B0[kFpMaxDim * kFpMaxDim], B[kFpMaxDim * kFpMaxDim];
};

// One sample per thread: t ~ U(t_lo, t_lo + t_span); eigenbasis moments (fp32, d^2 terms);
// in-register Cholesky C = L L^T; y = U^T m + L xi; x = U y.
template <int D>
__global__ __launch_bounds__(kBlock) void fp_exact_sample_kernel(FpArgs a, float* __restrict__ out,
                                                                 float* __restrict__ t_out) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= a.n) return;
  const uint64_t gid = (uint64_t)(a.row_off + r);
  const uint32_t lo = (uint32_t)gid, hi = (uint32_t)(gid >> 32);
  const uint4 tb = philox4x32_10(make_uint4(lo, hi, a.ctr, 0x10000000u), a.k0, a.k1);
  const float t = fmaf(u32_unit(tb.x), a.t_span, a.t_lo);
  float e[D];
#pragma unroll
  for (int i = 0; i < D; ++i) e[i] = __expf(-t * a.s[i]);
  float C[D][D];
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      const float ee = e[i] * e[j];
      C[i][j] = ee * a.B0[i * D + j] + a.B[i * D + j] * (1.f - ee) / (a.s[i] + a.s[j]);
    }
  // Cholesky (lower), C is SPD for t > 0 (and = B0 at t = 0)
#pragma unroll
  for (int j = 0; j < D; ++j) {
    float dj = C[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) dj = fmaf(-C[j][k], C[j][k], dj);
    dj = sqrtf(fmaxf(dj, 0.f));
    C[j][j] = dj;
    const float inv = dj > 0.f ? 1.f / dj : 0.f;
#pragma unroll
    for (int i = j + 1; i < D; ++i) {
      float v = C[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) v = fmaf(-C[i][k], C[j][k], v);
      C[i][j] = v * inv;
    }
  }
  float xi[D];
#pragma unroll
  for (int j = 0; 4 * j < D; ++j) {
    const uint4 b = philox4x32_10(make_uint4(lo, hi, a.ctr, 0x40000000u | (uint32_t)j), a.k0, a.k1);
    float z[4];
    box_muller(b.x, b.y, z[0], z[1]);
    box_muller(b.z, b.w, z[2], z[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * j + k < D) xi[4 * j + k] = z[k];
  }
  float y[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    float v = e[i] * a.Um0[i];
#pragma unroll
    for (int k = 0; k <= i; ++k) v = fmaf(C[i][k], xi[k], v);
    y[i] = v;
  }
#pragma unroll
  for (int i = 0; i < D; ++i) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < D; ++k) v = fmaf(a.U[i * D + k], y[k], v);
    out[r * D + i] = v;
  }
  if (t_out) t_out[r] = t;
}

// [x_r | e_k] rows (unit_directions) or [x_r | 0] rows; one output row per thread.
__global__ void fp_rows_kernel(const float* __restrict__ x, int64_t n, int64_t ldx, int d, int dirs,
                               float* __restrict__ out) {
  const int64_t o = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int per = dirs ? d : 1;
  if (o >= n * per) return;
  const int64_t r = o / per;
  const int k = (int)(o - r * per);
  float* dst = out + o * 2 * d;
  for (int i = 0; i < d; ++i) dst[i] = x[r * ldx + i];
  for (int i = 0; i < d; ++i) dst[d + i] = (dirs && i == k) ? 1.f : 0.f;
}

}  // namespace pdeinv

using namespace pdeinv;

extern "C" int pdeinv_fp_rows(const float* x, int64_t n, int64_t ldx, int32_t d, int32_t dirs, float* out,
                              void* stream) {
  PDEINV_REQUIRE(d >= 1 && d <= PDEINV_MAX_DIM, PDEINV_ERR_UNSUPPORTED, "fp_rows: dim must be in [1, 16]");
  PDEINV_REQUIRE(n >= 0 && ldx >= d, PDEINV_ERR_INVALID, "fp_rows: n < 0 or ldx < dim");
  if (n == 0) return PDEINV_OK;
  PDEINV_REQUIRE(x && out, PDEINV_ERR_INVALID, "fp_rows: null pointer");
  const int64_t rows = n * (dirs ? d : 1);
  hipLaunchKernelGGL(fp_rows_kernel, dim3(grid_for(rows)), dim3(kBlock), 0, (hipStream_t)stream, x, n, ldx, d,
                     dirs ? 1 : 0, out);
  return check_launch("fp_rows_kernel");
}

extern "C" int pdeinv_fp_exact_sample(int64_t n, int32_t d, uint64_t seed, uint32_t ctr, int64_t row_off, float t_lo,
                                      float t_hi, const float* U, const float* s, const float* Um0, const float* B0,
                                      const float* B, float* out, float* t_out, void* stream) {
  PDEINV_REQUIRE(d >= 1 && d <= kFpMaxDim, PDEINV_ERR_UNSUPPORTED, "fp_exact_sample: dim must be in [1, 8]");
  PDEINV_REQUIRE(n >= 0 && row_off >= 0, PDEINV_ERR_INVALID, "fp_exact_sample: n / row_offset < 0");
  PDEINV_REQUIRE(std::isfinite(t_lo) && std::isfinite(t_hi) && t_hi >= t_lo && t_lo >= 0.f, PDEINV_ERR_INVALID,
                 "fp_exact_sample: need 0 <= t_lo <= t_hi");
  if (n == 0) return PDEINV_OK;
  PDEINV_REQUIRE(U && s && Um0 && B0 && B && out, PDEINV_ERR_INVALID, "fp_exact_sample: null pointer");
  FpArgs a{};
  a.n = n;
  a.row_off = row_off;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.ctr = ctr;
  a.t_lo = t_lo;
  a.t_span = t_hi - t_lo;
  for (int i = 0; i < d; ++i) {
    PDEINV_REQUIRE(std::isfinite(s[i]) && s[i] > 0.f, PDEINV_ERR_INVALID, "fp_exact_sample: F must be SPD (s > 0)");
    a.s[i] = s[i];
    a.Um0[i] = Um0[i];
  }
  for (int k = 0; k < d * d; ++k) {
    a.U[k] = U[k];
    a.B0[k] = B0[k];
    a.B[k] = B[k];
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid_for(n));
  switch (d) {
#define CASE(DD) case DD: hipLaunchKernelGGL(fp_exact_sample_kernel<DD>, g, dim3(kBlock), 0, st, a, out, t_out); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "fp_exact_sample: dim must be in [1, 8]");
  }
  return check_launch("fp_exact_sample_kernel");
}
