// sampling.hip — exact Gaussian sampler, raw Philox stream and the offline subsample gather.
#include "common.h"

namespace pdeinv {

// core/distribution.py:64-65  Gaussian.sample: z = C^{1/2} xi + mu (one row per thread).
// Grouped form (the exact sampler of …_OU.py:140-190, one Gaussian per random time): row r
// uses mean[g], ch[g] with g = r / rows_per_group; one group is the plain sampler.
template <int M>
__global__ __launch_bounds__(kBlock) void gaussian_sample_kernel(int64_t n, uint32_t k0, uint32_t k1,
                                                                 uint32_t ctr_z, int64_t row_off,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ ch,
                                                                 float* __restrict__ out,
                                                                 int64_t rows_per_group) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  if (rows_per_group < n) {
    const int64_t g = r / rows_per_group;
    mean += g * M;
    ch += g * M * M;
  }
  const uint64_t gid = (uint64_t)(row_off + r);
  float xi[M];
#pragma unroll
  for (int j = 0; 4 * j < M; ++j) {
    const uint4 b = philox4x32_10(make_uint4((uint32_t)gid, (uint32_t)(gid >> 32), ctr_z,
                                             0x40000000u | (uint32_t)j), k0, k1);
    float z[4];
    box_muller(b.x, b.y, z[0], z[1]);
    box_muller(b.z, b.w, z[2], z[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * j + k < M) xi[4 * j + k] = z[k];
  }
  float y[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < M; ++j) acc = fmaf(ch[i * M + j], xi[j], acc);
    y[i] = acc + mean[i];
  }
  float* dst = out + r * M;
  if constexpr (M % 4 == 0) {
#pragma unroll
    for (int k = 0; k < M; k += 4)
      *reinterpret_cast<float4*>(dst + k) = make_float4(y[k], y[k + 1], y[k + 2], y[k + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < M; ++k) dst[k] = y[k];
  }
}

__global__ void philox_fill_kernel(int64_t n, uint32_t k0, uint32_t k1, uint32_t cz, uint32_t cw,
                                   uint4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  out[i] = philox4x32_10(make_uint4((uint32_t)i, (uint32_t)((uint64_t)i >> 32), cz, cw), k0, k1);
}

// consistency.py:97-118 — data_0T = dataset["0T"][traj_idx][:, time_idx, :] flattened, read
// from the time-major trajectory [n_steps, N, m]. One output row per thread; an index out of
// range produces a NaN row (loud in the loss) instead of an out-of-bounds read.
__global__ void gather_kernel(const float* __restrict__ traj, int64_t N, int n_steps, int m,
                              const int32_t* __restrict__ traj_idx, int64_t n_sel,
                              const int32_t* __restrict__ time_idx, int n_t,
                              float* __restrict__ out) {
  const int64_t o = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (o >= n_sel * n_t) return;
  const int64_t r = o / n_t;
  const int t = (int)(o - r * n_t);
  const int32_t p = traj_idx[r], s = time_idx[t];
  float* dst = out + o * m;
  if (p < 0 || p >= N || s < 0 || s >= n_steps) {
    for (int k = 0; k < m; ++k) dst[k] = __builtin_nanf("");
    return;
  }
  const float* src = traj + ((int64_t)s * N + p) * m;
  for (int k = 0; k < m; ++k) dst[k] = src[k];
}

// One uniformly drawn trajectory row per particle: out[p] = traj[t_p, p], t_p = Philox(seed;
// p, ctr) mod n_steps (the C5 residual batch). Coalesced: consecutive particles
// read consecutive rows of their (different) time slabs.
__global__ void gather_random_step_kernel(const float* __restrict__ traj, int64_t N, int n_steps, int m,
                                          uint32_t k0, uint32_t k1, uint32_t ctr, float* __restrict__ out,
                                          int32_t* __restrict__ t_out) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= N) return;
  const uint4 b = philox4x32_10(make_uint4((uint32_t)p, (uint32_t)((uint64_t)p >> 32), ctr, 0x20000000u), k0, k1);
  const int t = (int)(((uint64_t)b.x * (uint64_t)n_steps) >> 32);  // unbiased-enough range reduction
  if (t_out) t_out[p] = t;
  const float* src = traj + ((int64_t)t * N + p) * m;
  float* dst = out + p * m;
  for (int k = 0; k < m; ++k) dst[k] = src[k];
}

// m % 4 == 0 and 16-byte aligned rows (the C5 batch: m = 2d = 16): one thread per 16-byte quad of a
// row, so a row is one contiguous 4-lane run per load / store instead of m scalar accesses strided by
// the row length across the wave (each thread of a row recomputes the row's Philox draw: cheap).
__global__ void gather_random_step_vec_kernel(const float* __restrict__ traj, int64_t N, int n_steps, int m,
                                              uint32_t k0, uint32_t k1, uint32_t ctr, float* __restrict__ out,
                                              int32_t* __restrict__ t_out) {
  const int nq = m >> 2;
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= N * nq) return;
  const int64_t p = e / nq;
  const int q = (int)(e - p * nq);
  const uint4 b = philox4x32_10(make_uint4((uint32_t)p, (uint32_t)((uint64_t)p >> 32), ctr, 0x20000000u), k0, k1);
  const int t = (int)(((uint64_t)b.x * (uint64_t)n_steps) >> 32);  // same draw as the scalar kernel
  if (t_out && q == 0) t_out[p] = t;
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(traj + ((int64_t)t * N + p) * m) + q);
  reinterpret_cast<f32x4*>(out + p * m)[q] = v;
}

}  // namespace pdeinv

using namespace pdeinv;

extern "C" int pdeinv_gather_random_step(const float* traj, int64_t N, int32_t n_steps, int32_t m, uint64_t seed,
                                         uint32_t ctr, float* out, int32_t* t_out, void* stream) {
  PDEINV_REQUIRE(N >= 0 && n_steps >= 1 && m >= 1, PDEINV_ERR_INVALID, "gather_random_step: bad sizes");
  if (N == 0) return PDEINV_OK;
  PDEINV_REQUIRE(traj && out, PDEINV_ERR_INVALID, "gather_random_step: null pointer");
  if (m % 4 == 0 && ((uintptr_t)traj & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    hipLaunchKernelGGL(gather_random_step_vec_kernel, dim3(grid_for(N * (m / 4))), dim3(kBlock), 0,
                       (hipStream_t)stream, traj, N, n_steps, m, (uint32_t)seed, (uint32_t)(seed >> 32), ctr, out,
                       t_out);
    return check_launch("gather_random_step_vec_kernel");
  }
  hipLaunchKernelGGL(gather_random_step_kernel, dim3(grid_for(N)), dim3(kBlock), 0, (hipStream_t)stream, traj, N,
                     n_steps, m, (uint32_t)seed, (uint32_t)(seed >> 32), ctr, out, t_out);
  return check_launch("gather_random_step_kernel");
}

extern "C" int pdeinv_gaussian_sample_grouped(int64_t n_groups, int64_t rows_per_group, int32_t m, uint64_t seed,
                                              uint32_t ctr, int64_t row_off, const float* mean, const float* ch,
                                              float* out, void* stream) {
  PDEINV_REQUIRE(m >= 1 && m <= 2 * PDEINV_MAX_DIM, PDEINV_ERR_UNSUPPORTED,
                 "gaussian_sample: dim must be in [1, 32]");
  PDEINV_REQUIRE(n_groups >= 0 && rows_per_group >= 0 && row_off >= 0, PDEINV_ERR_INVALID,
                 "gaussian_sample: n_groups / rows_per_group / row_offset < 0");
  const int64_t n = n_groups * rows_per_group;
  if (n == 0) return PDEINV_OK;
  PDEINV_REQUIRE(mean && ch && out, PDEINV_ERR_INVALID, "gaussian_sample: null pointer");
  PDEINV_REQUIRE(m % 4 != 0 || ((uintptr_t)out % 16) == 0, PDEINV_ERR_INVALID,
                 "gaussian_sample: out must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const dim3 g(grid_for(n));
  switch (m) {
#define CASE(MM) case MM: hipLaunchKernelGGL(gaussian_sample_kernel<MM>, g, dim3(kBlock), 0, st, n, k0, k1, ctr, row_off, mean, ch, out, rows_per_group); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10) CASE(11)
    CASE(12) CASE(13) CASE(14) CASE(15) CASE(16) CASE(18) CASE(20) CASE(22) CASE(24) CASE(26) CASE(28) CASE(30)
    CASE(32)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "gaussian_sample: dim must be 1-16 or an even number up to 32");
  }
  return check_launch("gaussian_sample_kernel");
}

extern "C" int pdeinv_gaussian_sample(int64_t n, int32_t m, uint64_t seed, uint32_t ctr,
                                      int64_t row_off, const float* mean, const float* ch,
                                      float* out, void* stream) {
  PDEINV_REQUIRE(n >= 0, PDEINV_ERR_INVALID, "gaussian_sample: n / row_offset < 0");
  return pdeinv_gaussian_sample_grouped(n ? 1 : 0, n, m, seed, ctr, row_off, mean, ch, out, stream);
}

extern "C" int pdeinv_philox_fill(uint64_t seed, uint32_t cz, uint32_t cw, int64_t n, uint32_t* out,
                                  void* stream) {
  PDEINV_REQUIRE(n >= 0, PDEINV_ERR_INVALID, "philox_fill: n < 0");
  if (n == 0) return PDEINV_OK;
  PDEINV_REQUIRE(out && ((uintptr_t)out % 16) == 0, PDEINV_ERR_INVALID,
                 "philox_fill: out must be non-null and 16-byte aligned");
  hipLaunchKernelGGL(philox_fill_kernel, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, n,
                     (uint32_t)seed, (uint32_t)(seed >> 32), cz, cw, reinterpret_cast<uint4*>(out));
  return check_launch("philox_fill_kernel");
}

extern "C" int pdeinv_gather_subsample(const float* traj, int64_t N, int32_t n_steps, int32_t m,
                                       const int32_t* traj_idx, int64_t n_sel,
                                       const int32_t* time_idx, int32_t n_t, float* out,
                                       void* stream) {
  PDEINV_REQUIRE(N >= 0 && n_steps >= 1 && m >= 1 && n_sel >= 0 && n_t >= 0, PDEINV_ERR_INVALID,
                 "gather_subsample: bad sizes");
  if (n_sel == 0 || n_t == 0) return PDEINV_OK;
  PDEINV_REQUIRE(traj && traj_idx && time_idx && out, PDEINV_ERR_INVALID, "gather_subsample: null pointer");
  hipLaunchKernelGGL(gather_kernel, dim3(grid_for(n_sel * n_t)), dim3(kBlock), 0, (hipStream_t)stream,
                     traj, N, n_steps, m, traj_idx, n_sel, time_idx, n_t, out);
  return check_launch("gather_kernel");
}
