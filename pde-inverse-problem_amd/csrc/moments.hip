// moments.hip — sample-set moment reduction and the shared fp64 slab reducer (gfx950).
//
// Every term of the KFP residual for a parametric quadratic V_theta, and of its gradient,
// is an expectation of a polynomial of degree <= 2 in z = [x, v]
// (methods/consistency_instances/kinetic_fokker_planck.py:33-58), so one streaming pass that
// accumulates [count, sum z, sum z z^T] replaces the reference's vmap(grad) / vmap(jvp∘grad)
// / value_and_grad over every sample. HBM-bound: 4*m bytes read per row.
#include <mutex>
#include <string>

#include "common.h"

namespace pdeinv {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(PDEINV_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return PDEINV_OK;
}

// One block per column: fixed-order fp64 sum of partials[c * n_blocks + 0 .. n_blocks).
__global__ __launch_bounds__(kBlock) void slab_reduce_kernel(const float* __restrict__ partials,
                                                             int n_blocks,
                                                             double* __restrict__ out) {
  const int c = blockIdx.x;
  const float* col = partials + (int64_t)c * n_blocks;
  double s = 0.0;
  for (int b = threadIdx.x; b < n_blocks; b += kBlock) s += (double)col[b];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  __shared__ double w[kWavesPerBlock];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < kWavesPerBlock; ++k) t += w[k];
    out[c] = t;
  }
}

void launch_slab_reduce(const float* partials, int n_blocks, int n_cols, double* out,
                        hipStream_t stream) {
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(n_cols), dim3(kBlock), 0, stream, partials, n_blocks,
                     out);
}

constexpr int kMomGridCap = 2048;  // memory-bound: cap and grid-stride (8 blocks per CU)

static int mom_grid(int64_t n_rows) {
  int g = grid_for(n_rows);
  return g < 1 ? 1 : (g > kMomGridCap ? kMomGridCap : g);
}

template <int M>
__global__ __launch_bounds__(kBlock) void moments_kernel(const float* __restrict__ z, int64_t n,
                                                         int64_t ld, float* __restrict__ partials) {
  MomentAcc<M> acc;
  acc.zero();
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const bool vec4 = (M % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)z & 15) == 0);
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n; r += stride) {
    const float* row = z + r * ld;
    float v[M];
    if (vec4) {
#pragma unroll
      for (int k = 0; k < M; k += 4) {
        const float4 t = *reinterpret_cast<const float4*>(row + k);
        v[k] = t.x; v[k + 1] = t.y; v[k + 2] = t.z; v[k + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < M; ++k) v[k] = row[k];
    }
    acc.add(v, 1.f);
  }
  __shared__ float lds[kWavesPerBlock * moment_len(M)];
  block_reduce_to_slab(acc.v, moment_len(M), lds, partials, blockIdx.x, gridDim.x);
}

}  // namespace pdeinv

using namespace pdeinv;

extern "C" const char* pdeinv_last_error(void) { return g_last_error.c_str(); }
extern "C" int pdeinv_abi_version(void) { return PDEINV_ABI_VERSION; }
extern "C" int pdeinv_runtime_version(void) {
  int v = 0;
  if (hipRuntimeGetVersion(&v) != hipSuccess) return -1;
  return v;
}

extern "C" size_t pdeinv_moments_workspace_bytes(int64_t n_rows, int32_t m) {
  if (m < 1 || m > 16 || n_rows < 0) return 0;
  return (size_t)moment_len(m) * mom_grid(n_rows) * sizeof(float);
}

extern "C" int pdeinv_moments(const float* z, int64_t n, int32_t m, int64_t ld, void* ws,
                              double* out, void* stream) {
  PDEINV_REQUIRE(m >= 1 && m <= 16, PDEINV_ERR_UNSUPPORTED, "moments: m must be in [1, 16]");
  PDEINV_REQUIRE(n >= 0, PDEINV_ERR_INVALID, "moments: n_rows must be >= 0");
  if (ld == 0) ld = m;
  PDEINV_REQUIRE(ld >= m, PDEINV_ERR_INVALID, "moments: ld < m");
  PDEINV_REQUIRE(out != nullptr && ws != nullptr, PDEINV_ERR_INVALID, "moments: null out/workspace");
  PDEINV_REQUIRE(n == 0 || z != nullptr, PDEINV_ERR_INVALID, "moments: z is null");
  hipStream_t st = (hipStream_t)stream;
  const int g = mom_grid(n);
  float* p = (float*)ws;
  switch (m) {
#define CASE(MM) case MM: hipLaunchKernelGGL(moments_kernel<MM>, dim3(g), dim3(kBlock), 0, st, z, n, ld, p); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
  }
  int rc = check_launch("moments_kernel");
  if (rc) return rc;
  launch_slab_reduce(p, g, moment_len(m), out, st);
  return check_launch("slab_reduce_kernel");
}
