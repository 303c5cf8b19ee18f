// mlp.hip — KFP residual for the non-parametric hypothesis V_hypothesis (gfx950).
//
// V(x) = sum_o y_o^2, y = h_L K_o + b_o, h_l = tanh(h_{l-1} K_l + b_l), h_0 = x   (core/model.py:32-62)
// Per sample the residual (kinetic_fokker_planck.py:33-58) needs g = grad_x V, V' = g.v and
// V'' = v^T Hess V v, and the trainer needs d loss / d theta (jax.value_and_grad, :60-61).
// Batched over samples this is a chain of dense GEMMs — [rows x W] x [W x W] — plus per-element
// Taylor / adjoint algebra:
//   F1  Taylor-mode forward, three streams (h, h', h'') through every layer        3P MACs / sample
//   R1  reverse chain of grad_x V (a_l, zeta_l)                                     1P
//   F2  forward-mode adjoint of that chain (abar_l, zetabar_l)                      1P
//   R2  reverse over the three forward streams                                      3P
//   G   weight gradients: sums of outer products over samples (4 stream pairs)      4P
// (24P FLOP per sample). The GEMMs are plain library GEMMs (rocBLAS sgemm, fp32
// on the MFMA f32 path); every element-wise step, the per-row loss terms and the reductions are
// the kernels below. The derivation is oracle/numpy_ref.py kfp_mlp_grad_analytic, checked against
// central finite differences.
#include <dlfcn.h>

#include <atomic>
#include <math.h>
#include <rocblas/rocblas.h>

#include <mutex>

#include "common.h"
#include "mlp_fused.h"

namespace pdeinv {

// ---- rocBLAS plumbing ------------------------------------------------------------------------
// rocBLAS serves only the explicit opt-in impl = LIBRARY (a cross-check of the hand-written kernels): every AUTO /
// FUSED shape runs on this library's own kernels. So libpdeinv.so does not link it: the first LIBRARY call loads
// librocblas.so.5 with dlopen and resolves the five entry points it uses; without it that call fails loudly
// (PDEINV_ERR_UNSUPPORTED), and no other path notices. (rocblas.h supplies the types only.)
struct BlasApi {
  decltype(&rocblas_create_handle) create_handle = nullptr;
  decltype(&rocblas_destroy_handle) destroy_handle = nullptr;
  decltype(&rocblas_set_stream) set_stream = nullptr;
  decltype(&rocblas_sgemm) sgemm = nullptr;
  decltype(&rocblas_sgemm_strided_batched) sgemm_strided_batched = nullptr;
  bool ok = false;
};

// residual calls served by rocBLAS in this process (pdeinv_rocblas_calls: AUTO / FUSED never add to it)
static std::atomic<int64_t> g_rocblas_calls{0};

static const BlasApi& blas_api() {
  static const BlasApi api = [] {
    BlasApi a{};
    void* lib = nullptr;
    for (const char* name : {"librocblas.so.5", "/opt/rocm/lib/librocblas.so.5", "librocblas.so"}) {
      lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (lib) break;
    }
    if (!lib) return a;
    a.create_handle = (decltype(a.create_handle))dlsym(lib, "rocblas_create_handle");
    a.destroy_handle = (decltype(a.destroy_handle))dlsym(lib, "rocblas_destroy_handle");
    a.set_stream = (decltype(a.set_stream))dlsym(lib, "rocblas_set_stream");
    a.sgemm = (decltype(a.sgemm))dlsym(lib, "rocblas_sgemm");
    a.sgemm_strided_batched = (decltype(a.sgemm_strided_batched))dlsym(lib, "rocblas_sgemm_strided_batched");
    a.ok = a.create_handle && a.destroy_handle && a.set_stream && a.sgemm && a.sgemm_strided_batched;
    return a;
  }();
  return api;
}

// One handle per (host thread, device): a rocBLAS handle carries its stream, so a handle shared
// between threads lets one thread's rocblas_set_stream retarget another thread's GEMMs (the ABI
// promises reentrancy across distinct streams, include/pdeinv.h). Thread-local handles need no lock
// around set_stream + the GEMM sequence; they are destroyed when the thread exits.
struct ThreadBlasHandles {
  rocblas_handle h[64] = {};
  ~ThreadBlasHandles() {
    for (rocblas_handle& x : h)
      if (x) blas_api().destroy_handle(x);
  }
};

static rocblas_handle blas_handle(int device) {
  thread_local ThreadBlasHandles handles;
  if (device < 0 || device >= 64 || !blas_api().ok) return nullptr;
  if (!handles.h[device]) {
    if (blas_api().create_handle(&handles.h[device]) != rocblas_status_success) handles.h[device] = nullptr;
  }
  return handles.h[device];
}

// K-split factor of the weight-gradient GEMMs: the reduction runs over 4 x chunk rows while the
// output is only n_in x n_out (<= 256 x 256), so one GEMM launches a few dozen workgroups. Slicing
// the rows into up to kMaxKSplit batched GEMMs (>= kMinKSlice rows each) fills the chip; the fp32
// partial slabs are summed in a fixed order (deterministic, no atomics).
constexpr int kMaxKSplit = 256;
constexpr int64_t kMinKSlice = 4096;
constexpr int kColsumBlocks = 512;

// out[i] += sum_k part[k * n + i]. A block owns kSumCols outputs; its kBlock / kSumCols thread
// groups each sum a strided subset of the S slices (independent loads in flight), then the group
// partials are added in a fixed order through LDS — deterministic, and fast for the small n
// (a few thousand weights) and large S of the weight / bias gradients.
constexpr int kSumCols = 32;
__global__ __launch_bounds__(kBlock) void sum_slices_kernel(const float* __restrict__ part, int S, int64_t n,
                                                            float* __restrict__ out) {
  constexpr int G = kBlock / kSumCols;
  __shared__ float red[G][kSumCols];
  const int c = threadIdx.x % kSumCols, g = threadIdx.x / kSumCols;
  const int64_t i = (int64_t)blockIdx.x * kSumCols + c;
  float s = 0.f;
  if (i < n)
    for (int k = g; k < S; k += G) s += part[(int64_t)k * n + i];
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < G; ++q) t += red[q][c];
    out[i] += t;
  }
}

// partial column sums of B[R x n] (row-major): block b sums rows [b*rpb, (b+1)*rpb). For n < kBlock
// the block's threads cover kBlock / n rows at a time (lane t: column t % n, row offset t / n), so
// every thread is busy and a wave reads contiguous bytes; the row-lanes are combined in a fixed
// order through LDS. Wider outputs use blockIdx.y column tiles of kBlock.
__global__ __launch_bounds__(kBlock) void colsum_partial_kernel(const float* __restrict__ B, int64_t R, int n,
                                                                int64_t rpb, float* __restrict__ part) {
  __shared__ float red[kBlock];
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < R ? r0 + rpb : R;
  if (n >= kBlock) {
    const int c = blockIdx.y * kBlock + threadIdx.x;
    if (c >= n) return;
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) s += B[r * n + c];
    part[(int64_t)blockIdx.x * n + c] = s;
    return;
  }
  const int lanes = kBlock / n;  // row-lanes (>= 1)
  const int c = threadIdx.x % n, q = threadIdx.x / n;
  float s = 0.f;
  if (q < lanes)
    for (int64_t r = r0 + q; r < r1; r += lanes) s += B[r * n + c];
  red[threadIdx.x] = s;
  __syncthreads();
  if (q == 0) {
    float t = 0.f;
    for (int k = 0; k < lanes; ++k) t += red[k * n + c];
    part[(int64_t)blockIdx.x * n + c] = t;
  }
}

struct Blas {
  rocblas_handle h;
  hipStream_t st;
  float* part;  // >= kMaxKSplit * max(n_in * n_out) floats (also holds the colsum partials)
  int status = 0;
  // row-major C[R x n_out] = A[R x n_in] . K[n_in x n_out]
  void fwd(const float* A, const float* K, float* C, int64_t R, int n_in, int n_out) {
    const float one = 1.f, zero = 0.f;
    if (blas_api().sgemm(h, rocblas_operation_none, rocblas_operation_none, n_out, (rocblas_int)R, n_in, &one, K,
                      n_out, A, n_in, &zero, C, n_out) != rocblas_status_success)
      status = 1;
  }
  // row-major C[R x n_in] = A[R x n_out] . K^T
  void bwd(const float* A, const float* K, float* C, int64_t R, int n_in, int n_out) {
    const float one = 1.f, zero = 0.f;
    if (blas_api().sgemm(h, rocblas_operation_transpose, rocblas_operation_none, n_in, (rocblas_int)R, n_out, &one, K,
                      n_out, A, n_out, &zero, C, n_in) != rocblas_status_success)
      status = 1;
  }
  // Kbar[n_in x n_out] += A[R x n_in]^T . B[R x n_out]  (K-split into S batched slices + slab sum)
  void wgrad(const float* A, const float* B, float* Kbar, int64_t R, int n_in, int n_out) {
    const float one = 1.f, zero = 0.f;
    int64_t S = R / kMinKSlice;
    S = S < 1 ? 1 : (S > kMaxKSplit ? kMaxKSplit : S);
    const int64_t Ks = R / S, rem = R - S * Ks;
    const int64_t nout = (int64_t)n_in * n_out;
    if (blas_api().sgemm_strided_batched(h, rocblas_operation_none, rocblas_operation_transpose, n_out, n_in,
                                      (rocblas_int)Ks, &one, B, n_out, Ks * n_out, A, n_in, Ks * n_in, &zero, part,
                                      n_out, nout, (rocblas_int)S) != rocblas_status_success)
      status = 1;
    hipLaunchKernelGGL(sum_slices_kernel, dim3(grid_for(nout, kSumCols)), dim3(kBlock), 0, st, part, (int)S, nout, Kbar);
    if (rem > 0 && blas_api().sgemm(h, rocblas_operation_none, rocblas_operation_transpose, n_out, n_in,
                                 (rocblas_int)rem, &one, B + S * Ks * n_out, n_out, A + S * Ks * n_in, n_in, &one,
                                 Kbar, n_out) != rocblas_status_success)
      status = 1;
  }
  // bbar[n] += sum over the R rows of B[R x n]
  void colsum(const float* B, float* bbar, int64_t R, int n) {
    const int64_t rpb = (R + kColsumBlocks - 1) / kColsumBlocks;
    const int nb = (int)((R + rpb - 1) / rpb);
    hipLaunchKernelGGL(colsum_partial_kernel, dim3(nb, n >= kBlock ? (n + kBlock - 1) / kBlock : 1), dim3(kBlock), 0,
                       st, B, R, n, rpb, part);
    hipLaunchKernelGGL(sum_slices_kernel, dim3(grid_for(n, kSumCols)), dim3(kBlock), 0, st, part, nb, (int64_t)n, bbar);
  }
};

// ---- element-wise kernels --------------------------------------------------------------------
__device__ __forceinline__ float fast_tanh(float z) {
  // tanh(z) = 1 - 2 / (exp(2z) + 1); exp2 on the hardware unit, saturates cleanly at +-1
  const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * z);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

// F1: z (+bias), z', z'' -> h = tanh z, h' = s1 z', h'' = s1 z'' + s2 z'^2
__global__ void mlp_act_fwd(const float* __restrict__ Z, float* __restrict__ A, const float* __restrict__ bias,
                            int64_t R, int n) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t S = R * n;
  if (e >= S) return;
  const int j = (int)(e % n);
  const float z = Z[e] + bias[j], zd = Z[S + e], zdd = Z[2 * S + e];
  const float h = fast_tanh(z);
  const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
  A[e] = h;
  A[S + e] = s1 * zd;
  A[2 * S + e] = fmaf(s1, zdd, s2 * zd * zd);
}

// output layer: y (+bias) stored back; u = 2y (seed of the grad_x chain); per row
// terms = {V' = 2 y.y', V'' = 2(y'.y' + y.y''), V = y.y, 0}
// A block owns rb consecutive rows = rb*O consecutive elements of each plane: phase 1 is
// element-wise and coalesced, the per-element products go to LDS, phase 2 sums them per row.
__global__ __launch_bounds__(kBlock) void mlp_out(float* __restrict__ Y, const float* __restrict__ bias,
                                                  float* __restrict__ YB, float4* __restrict__ terms, int64_t R,
                                                  int O, int rb) {
  extern __shared__ float prod[];  // [3][rb*O]
  const int64_t S = R * O;
  const int64_t r0 = (int64_t)blockIdx.x * rb;
  const int nr = (int)((R - r0) < rb ? (R - r0) : rb);
  const int ne = nr * O;
  const int64_t e0 = r0 * O;
  for (int k = threadIdx.x; k < ne; k += kBlock) {
    const int64_t e = e0 + k;
    const float y = Y[e] + bias[k % O], yd = Y[S + e], ydd = Y[2 * S + e];
    Y[e] = y;
    YB[3 * S + e] = 2.f * y;
    prod[k] = y * yd;
    prod[rb * O + k] = fmaf(yd, yd, y * ydd);
    prod[2 * rb * O + k] = y * y;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < nr; r += kBlock) {
    float vd = 0.f, vdd = 0.f, v = 0.f;
    for (int o = 0; o < O; ++o) {
      vd += prod[r * O + o];
      vdd += prod[rb * O + r * O + o];
      v += prod[2 * rb * O + r * O + o];
    }
    terms[r0 + r] = make_float4(2.f * vd, 2.f * vdd, v, 0.f);
  }
}

// R1: zeta = tanh'(z) * a   (a = GEMM output, kept for R2)
__global__ void mlp_gchain(const float* __restrict__ a, const float* __restrict__ h, float* __restrict__ zeta,
                           int64_t S) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= S) return;
  const float hv = h[e];
  zeta[e] = (1.f - hv * hv) * a[e];
}

// F2: abar = tanh'(z) * zetabar
__global__ void mlp_gadj(const float* __restrict__ zetabar, const float* __restrict__ h, float* __restrict__ abar,
                         int64_t S) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= S) return;
  const float hv = h[e];
  abar[e] = (1.f - hv * hv) * zetabar[e];
}

struct MlpLossArgs {
  int d, set, true_kind, KT, bval;
  int uw;  // rows carry [x | v | u | w]: input-gradient seed u (added to abar_0) and value weight w
           // (KMV pair rows, set 3: pdeinv_residual_kmv_mlp)
  float c1, c2, c3, c0, c_true, inv_n;
  float s2t, l2st;
  float tp[PDEINV_MAX_PARAMS];  // tilde_F [d*d] or true GMM centres [K*d]
};

// per row: T1 = |g|^2, T2 = V'', T3 = V', T0 = V, true-potential terms (0T rows); seeds
// abar_0 = 2 c1 g; block partial sums of the 8 accumulator slots of pdeinv.h (PDEINV_GMM_ACC_*).
// The boundary slots report the set mean of V' (kinetic FP) or of V (bval: overdamped FP).
template <int D>
__global__ __launch_bounds__(kBlock) void mlp_loss(MlpLossArgs a, const float* __restrict__ G,
                                                   const float* __restrict__ X, int64_t ldx,
                                                   const float4* __restrict__ terms, float* __restrict__ abar0,
                                                   int64_t R, float* __restrict__ partials) {
  float acc[PDEINV_GMM_NACC] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < R; r += stride) {
    float g[D], x[D], T1 = 0.f;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      g[i] = G[r * D + i];
      x[i] = X[r * ldx + i];
      T1 = fmaf(g[i], g[i], T1);
      abar0[r * D + i] = 2.f * a.c1 * g[i] + (a.uw ? X[r * ldx + 2 * D + i] : 0.f);
    }
    const float4 t = terms[r];
    const float T2 = t.y, T3 = t.x, T0 = t.z;
    const float wr = a.uw ? X[r * ldx + 3 * D] : 1.f;
    acc[PDEINV_GMM_ACC_LOSS] += a.c1 * T1 + a.c2 * T2 + a.c3 * T3 + a.c0 * wr * T0;
    if (a.set == 3) {  // KMV pair rows: -2 x Hessian mean and 2 x value mean (scaled by c2, c0)
      acc[PDEINV_GMM_ACC_HESSIAN] += -0.5f * a.c2 * T2;
      acc[PDEINV_GMM_ACC_FRICTION] += a.c0 * wr * T0;
    } else if (a.set == 0) {
      float gt[D];
      if (a.true_kind == PDEINV_POT_QUADRATIC) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < D; ++j) s = fmaf(a.tp[i * D + j], x[j], s);
          gt[i] = s;
        }
      } else {
        float w[16], amax = -INFINITY;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          if (k < a.KT) {
            float d2 = 0.f;
#pragma unroll
            for (int i = 0; i < D; ++i) {
              const float u = x[i] - a.tp[k * D + i];
              d2 = fmaf(u, u, d2);
            }
            w[k] = -0.5f * d2 * a.l2st;
            amax = fmaxf(amax, w[k]);
          }
        }
        float den = 0.f, m[D];
#pragma unroll
        for (int i = 0; i < D; ++i) m[i] = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          if (k < a.KT) {
            const float e = __builtin_amdgcn_exp2f(w[k] - amax);
            den += e;
#pragma unroll
            for (int i = 0; i < D; ++i) m[i] = fmaf(e, a.tp[k * D + i], m[i]);
          }
        }
        const float inv = 1.f / den;
#pragma unroll
        for (int i = 0; i < D; ++i) gt[i] = a.s2t * (x[i] - m[i] * inv);
      }
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
    } else if (a.set == 1) {
      acc[PDEINV_GMM_ACC_INITIAL] += a.inv_n * (a.bval ? T0 : T3);
    } else {
      acc[PDEINV_GMM_ACC_TERMINAL] += a.inv_n * (a.bval ? T0 : T3);
    }
  }
  __shared__ float lds[kWavesPerBlock * PDEINV_GMM_NACC];
  block_reduce_to_slab(acc, PDEINV_GMM_NACC, lds, partials, blockIdx.x, gridDim.x);
}

// seeds of the reverse sweep over the forward streams (c0: weight of the value V = y.y):
//   ybar = 2 c3 y' + 2 c2 y'' + 2 ubar + 2 c0 y,  y'bar = 2 c3 y + 4 c2 y',  y''bar = 2 c2 y
// (rw: optional per-row weight of the value term, rw[r * ldw] for element e = r * O + o)
__global__ void mlp_seeds(const float* __restrict__ Y, const float* __restrict__ UB, float* __restrict__ YB,
                          float c2, float c3, float c0, int64_t S, const float* __restrict__ rw, int64_t ldw, int O) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= S) return;
  const float y = Y[e], yd = Y[S + e], ydd = Y[2 * S + e];
  const float cv = rw ? c0 * rw[(e / O) * ldw] : c0;
  YB[e] = 2.f * c3 * yd + 2.f * c2 * ydd + 2.f * UB[e] + 2.f * cv * y;
  YB[S + e] = 2.f * c3 * y + 4.f * c2 * yd;
  YB[2 * S + e] = 2.f * c2 * y;
}

// R2 element-wise step through tanh (s1 = tanh', s2 = tanh'', s3 = tanh'''):
//   zbar   = s1 hbar + s2 z' h'bar + (s2 z'' + s3 z'^2) h''bar + s2 a zetabar   (last: grad_x chain)
//   z'bar  = s1 h'bar + 2 s2 z' h''bar ;   z''bar = s1 h''bar
__global__ void mlp_act_bwd(const float* __restrict__ HB, const float* __restrict__ h, const float* __restrict__ Z,
                            const float* __restrict__ aL, const float* __restrict__ zb, float* __restrict__ ZB,
                            int64_t S) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= S) return;
  const float hv = h[e];
  const float s1 = 1.f - hv * hv, s2 = -2.f * hv * s1, s3 = -2.f * s1 * s1 - 2.f * hv * s2;
  const float zd = Z[S + e], zdd = Z[2 * S + e];
  const float hb = HB[e], hdb = HB[S + e], hddb = HB[2 * S + e];
  ZB[e] = s1 * hb + s2 * zd * hdb + (s2 * zdd + s3 * zd * zd) * hddb + s2 * aL[e] * zb[e];
  ZB[S + e] = s1 * hdb + 2.f * s2 * zd * hddb;
  ZB[2 * S + e] = s1 * hddb;
}

// copy the (x, v) rows of a sample set into the stream-0 / stream-1 input planes of layer 1
__global__ void mlp_load_rows(const float* __restrict__ z, int64_t ld, int d, float* __restrict__ A0, int64_t R) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= R * d) return;
  const int64_t r = e / d;
  const int i = (int)(e - r * d);
  A0[e] = z[r * ld + i];
  A0[R * d + e] = z[r * ld + d + i];
}

__global__ void slab_reduce_accum_kernel(const float* __restrict__ partials, int n_blocks,
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
  if (threadIdx.x == 0) out[c] += w[0] + w[1] + w[2] + w[3];
}

__global__ void kfp_terms_finalize_kernel(const double* __restrict__ acc, const float* __restrict__ grad,
                                          int64_t n_grad, float gamma, float* __restrict__ out) {
  double s = 0.0;
  for (int64_t k = threadIdx.x; k < n_grad; k += kBlock) s += (double)grad[k] * (double)grad[k];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  __shared__ double w[kWavesPerBlock];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[PDEINV_KFP_LOSS] = (float)acc[PDEINV_GMM_ACC_LOSS];
    out[PDEINV_KFP_LOSS_GT] = (float)acc[PDEINV_GMM_ACC_LOSS_GT];
    out[PDEINV_KFP_GRAD_NORM] = (float)sqrt(w[0] + w[1] + w[2] + w[3]);
    out[PDEINV_KFP_NABLA] = (float)acc[PDEINV_GMM_ACC_NABLA];
    out[PDEINV_KFP_HESSIAN] = (float)acc[PDEINV_GMM_ACC_HESSIAN];
    out[PDEINV_KFP_FRICTION] = (float)(gamma * acc[PDEINV_GMM_ACC_FRICTION]);
    out[PDEINV_KFP_NABLA_TRUE] = (float)acc[PDEINV_GMM_ACC_NABLA_TRUE];
    out[PDEINV_KFP_INITIAL] = (float)acc[PDEINV_GMM_ACC_INITIAL];
    out[PDEINV_KFP_TERMINAL] = (float)acc[PDEINV_GMM_ACC_TERMINAL];
  }
}

// ---- workspace plan -------------------------------------------------------------------------
constexpr int kLossGrid = 512;

struct MlpPlan {
  int d, L, W, O;
  int64_t Bc;
  size_t off_A0, off_Y, off_YB, off_UB, off_G, off_kpart, off_terms, off_part, total;
  size_t off_layer0, layer_stride;  // per hidden layer: A(4) Z(3) ZB(4) HB(3) aL(1) zb(1) planes of Bc*W
};

static MlpPlan make_plan(const pdeinv_kfp_mlp_desc* d) {
  MlpPlan p{};
  p.d = d->dim; p.L = d->n_layers; p.W = d->width; p.O = d->out_features;
  p.Bc = d->chunk_rows > 0 ? d->chunk_rows : (1 << 18);
  size_t o = 0;
  auto take = [&](size_t floats) { const size_t at = o; o += (floats + 63) & ~(size_t)63; return at; };
  p.off_A0 = take(4 * p.Bc * p.d);
  p.off_Y = take(3 * p.Bc * p.O);
  p.off_YB = take(4 * p.Bc * p.O);
  p.off_UB = take(p.Bc * p.O);
  p.off_G = take(p.Bc * p.d);
  const int64_t wmax = (int64_t)p.W * (p.W > p.d ? (p.W > p.O ? p.W : p.O) : p.d);
  const int64_t cmax = (int64_t)kColsumBlocks * (p.W > p.O ? p.W : p.O);
  p.off_kpart = take((size_t)(kMaxKSplit * wmax > cmax ? kMaxKSplit * wmax : cmax));
  p.off_terms = take(4 * p.Bc);
  p.off_part = take((size_t)PDEINV_GMM_NACC * kLossGrid);
  p.layer_stride = 16 * p.Bc * p.W;
  p.off_layer0 = take(p.layer_stride * p.L);
  p.total = o * sizeof(float);
  return p;
}

}  // namespace pdeinv

using namespace pdeinv;

// The shapes the fused fp32-MFMA path takes. The kernels are compiled for dim in {2, 4, 8, 16} and width in
// {32, 64, 128, 256, 512, 1024} (any depth 1..16, any out_features: mlpf::supported); every other dim <= 16 and
// width <= 1024 runs zero-padded to the next compiled one — exact: padded inputs and K1 rows are zero, padded
// hidden units have zero weights in and out (common.h MlpPadMap) — at the cost of the padded MACs. The
// reference's default V_hypothesis is 20 wide (configurations/neural_network/MLP.yaml:4-5). Only the explicit
// impl = LIBRARY reaches the rocBLAS path; an AUTO / FUSED shape outside the envelope is UNSUPPORTED.
struct FusedShape {
  int Dp = 0, Wp = 0;
  bool pad = false;
};
static int pad_dim(int D) { return D <= 2 ? 2 : (D <= 4 ? 4 : (D <= 8 ? 8 : 16)); }
static bool fused_shape(const pdeinv_kfp_mlp_desc* d, FusedShape* f = nullptr) {
  if (d->impl == PDEINV_MLP_IMPL_LIBRARY || d->dim < 1 || d->dim > 16 || d->n_layers < 1 ||
      d->n_layers > kMlpPadMaxL || d->out_features < 1)
    return false;
  int Wp = 0;
  for (int w : {32, 64, 128, 256, 512, 1024})
    if (w >= d->width) { Wp = w; break; }
  const int Dp = pad_dim(d->dim);
  if (!Wp || !mlpf::supported(Dp, d->n_layers, Wp, d->out_features)) return false;
  if (f) { f->Dp = Dp; f->Wp = Wp; f->pad = Dp != d->dim || Wp != d->width; }
  return true;
}

// The shape runs the hand-written fused fp32-MFMA path under impl = AUTO: the padded envelope of fused_shape (dims
// and widths zero-padded to the compiled ones), not only the compiled shapes themselves.
extern "C" int64_t pdeinv_rocblas_calls(void) { return g_rocblas_calls.load(std::memory_order_relaxed); }

extern "C" int pdeinv_mlp_fused_supported(int32_t dim, int32_t n_layers, int32_t width, int32_t out_features) {
  pdeinv_kfp_mlp_desc d{};
  d.dim = dim; d.n_layers = n_layers; d.width = width; d.out_features = out_features;
  d.impl = PDEINV_MLP_IMPL_AUTO;
  return fused_shape(&d) ? 1 : 0;
}

// PDEINV_MLP_FIRST_ORDER=0 (A/B): the boundary sets take the full second-order chain as the 0T set does
static bool first_order_enabled() {
  static const bool on = [] {
    const char* e = ab_env("PDEINV_MLP_FIRST_ORDER");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

static MlpPadMap width_pad_map(const pdeinv_kfp_mlp_desc* d, const FusedShape& f) {
  MlpPadMap pm{};
  pm.L = d->n_layers;
  int64_t ro = 0, po = 0;
  for (int l = 0; l <= pm.L; ++l) {
    pm.din[l] = l == 0 ? d->dim : d->width;
    pm.dout[l] = l == pm.L ? d->out_features : d->width;
    pm.pin[l] = l == 0 ? f.Dp : f.Wp;
    pm.pout[l] = l == pm.L ? d->out_features : f.Wp;
    pm.roff[l] = ro;
    pm.poff[l] = po;
    ro += (int64_t)pm.din[l] * pm.dout[l] + pm.dout[l];
    po += (int64_t)pm.pin[l] * pm.pout[l] + pm.pout[l];
  }
  return pm;
}

static int64_t pad_param_count(const MlpPadMap& pm) {
  return pm.poff[pm.L] + (int64_t)pm.pin[pm.L] * pm.pout[pm.L] + pm.pout[pm.L];
}

__global__ void mlp_pad_params_kernel(MlpPadMap pm, const float* __restrict__ src, int64_t P, float* __restrict__ dst) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P) return;
  const int64_t r = pm.real_of(q);
  dst[q] = r >= 0 ? src[r] : 0.f;
}

__global__ void mlp_unpad_grad_kernel(MlpPadMap pm, const float* __restrict__ gp, int64_t P, float* __restrict__ grad) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P) return;
  const int64_t r = pm.real_of(q);
  if (r >= 0) grad[r] += gp[q];
}

static int64_t chunk_rows_of(const pdeinv_kfp_mlp_desc* d) { return d->chunk_rows > 0 ? d->chunk_rows : (1 << 18); }

// fused-path workspace (floats): [run_chunk workspace | loss partials | padded params | padded gradient |
// padded rows (dim padding)]
struct FusedWs {
  size_t fl, part, pbuf, gbuf, rows, total;
  int64_t PP;
};
static FusedWs fused_ws(const pdeinv_kfp_mlp_desc* d, const FusedShape& f) {
  FusedWs w{};
  const int64_t Bc = chunk_rows_of(d);
  size_t o = 0;
  auto take = [&](size_t n) { const size_t at = o; o += (n + 63) & ~(size_t)63; return at; };
  w.fl = take(mlpf::workspace_floats(f.Dp, d->n_layers, f.Wp, d->out_features, Bc));
  w.part = take((size_t)PDEINV_GMM_NACC * kLossGrid);
  w.PP = f.pad ? pad_param_count(width_pad_map(d, f)) : 0;
  w.pbuf = take((size_t)w.PP);
  w.gbuf = take((size_t)w.PP);
  w.rows = take(f.Dp != d->dim ? (size_t)Bc * 2 * f.Dp : 0);
  w.total = o;
  return w;
}

// rows [x | v] of d floats -> [x, 0.. | v, 0..] of Dp (the fused path's dim padding)
__global__ void mlp_pad_rows_kernel(const float* __restrict__ src, int64_t ld, int64_t R, int D, int Dp,
                                    float* __restrict__ dst) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= R * 2 * Dp) return;
  const int64_t r = q / (2 * Dp);
  const int c = (int)(q - r * 2 * Dp), half = c / Dp, k = c - half * Dp;
  dst[q] = k < D ? src[r * ld + half * D + k] : 0.f;
}

extern "C" size_t pdeinv_residual_kfp_mlp_workspace_bytes(const pdeinv_kfp_mlp_desc* d) {
  if (!d || d->dim < 1 || d->n_layers < 1 || d->width < 1 || d->out_features < 1) return 0;
  FusedShape f;
  if (fused_shape(d, &f)) return fused_ws(d, f).total * sizeof(float);
  return make_plan(d).total;
}

namespace pdeinv {
struct LossCtx {
  MlpLossArgs la;
  const float* zr;
  int64_t ld;
  float* part;
  double* acc;
  int D;
};

static int fused_loss_hook(void* p, const float* G, const float4* terms, float* abar0, int64_t R, hipStream_t st) {
  LossCtx* c = (LossCtx*)p;
  const int lg = grid_for(R) < kLossGrid ? grid_for(R) : kLossGrid;
  switch (c->D) {
#define CASE(DD) case DD: hipLaunchKernelGGL(mlp_loss<DD>, dim3(lg), dim3(kBlock), 0, st, c->la, G, c->zr, c->ld, terms, abar0, R, c->part); break;
    CASE(2) CASE(4) CASE(8) CASE(16)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "kfp_mlp fused: dim must be 2, 4, 8 or 16");
  }
  hipLaunchKernelGGL(slab_reduce_accum_kernel, dim3(PDEINV_GMM_NACC), dim3(kBlock), 0, st, c->part, lg, c->acc);
  return check_launch("kfp_mlp fused loss");
}
}  // namespace pdeinv

namespace pdeinv {
// parameter offsets (flax order: K_1, b_1, ..., K_L, b_L, K_o, b_o)
static void param_offsets(int D, int W, int O, int L, int64_t* poff, int64_t* boff) {
  int64_t o = 0;
  for (int l = 0; l <= L; ++l) {
    const int n_in = (l == 0) ? D : W, n_out = (l == L) ? O : W;
    poff[l] = o; o += (int64_t)n_in * n_out;
    boff[l] = o; o += n_out;
  }
}

// One chunk of R rows through the library path: F1 Taylor forward, R1 grad_x chain, the loss
// terms (mlp_loss, accumulated into acc), F2 forward adjoint, R2 + weight gradients (accumulated
// into grad). grad_only stops after R1 and leaves g = grad_x V of every row in G (KMV pass 1).
struct LibRun {
  MlpPlan p;
  Blas* blas;
  float* w;
  const float* params;
  float* grad;
  const int64_t* poff;
  const int64_t* boff;
  hipStream_t st;
  double* acc;
  int64_t R = 0;
  float* layer(int l, int plane) const {
    return w + p.off_layer0 + p.layer_stride * (l - 1) + (size_t)plane * R * p.W;
  }
  float* G() const { return w + p.off_G; }
  int chunk(const float* zr, int64_t ld, int64_t rows, const MlpLossArgs& la, bool grad_only) {
    R = rows;
    const int D = p.d, W = p.W, O = p.O, L = p.L;
    float* A0 = w + p.off_A0;
    float* Y = w + p.off_Y;
    float* YB = w + p.off_YB;
    float* UB = w + p.off_UB;
    float* Gp = G();
    float4* terms = (float4*)(w + p.off_terms);
    float* part = w + p.off_part;
    Blas& b = *blas;
    // planes per hidden layer l: A 0-3, Z 4-6, ZB 7-10, HB 11-13, aL 14, zb 15. Inside a chunk of R
    // rows the planes are packed at stride R*W so that consecutive streams form one [k*R x W] operand.
    const int64_t SD = R * D, SW = R * W, SO = R * O;
    // ---- F1: Taylor-mode forward --------------------------------------------------------
    hipLaunchKernelGGL(mlp_load_rows, dim3(grid_for(SD)), dim3(kBlock), 0, st, zr, ld, D, A0, R);
    if (hipMemsetAsync(A0 + 2 * SD, 0, sizeof(float) * SD, st) != hipSuccess) return fail(PDEINV_ERR_HIP, "memset");
    for (int l = 1; l <= L; ++l) {
      const int n_in = (l == 1) ? D : W;
      const float* Ain = (l == 1) ? A0 : layer(l - 1, 0);
      float* Z = layer(l, 4);
      b.fwd(Ain, params + poff[l - 1], Z, 3 * R, n_in, W);  // three streams: one GEMM with 3R rows
      hipLaunchKernelGGL(mlp_act_fwd, dim3(grid_for(SW)), dim3(kBlock), 0, st, Z, layer(l, 0), params + boff[l - 1],
                         R, W);
    }
    b.fwd(layer(L, 0), params + poff[L], Y, 3 * R, W, O);
    {
      const int rb = O >= 2048 ? 1 : 2048 / O;  // 24 KB of LDS products per block
      hipLaunchKernelGGL(mlp_out, dim3((unsigned)((R + rb - 1) / rb)), dim3(kBlock), 3 * rb * O * sizeof(float), st,
                         Y, params + boff[L], YB, terms, R, O, rb);
    }
    // ---- R1: grad_x chain ---------------------------------------------------------------
    b.bwd(YB + 3 * SO, params + poff[L], layer(L, 14), R, W, O);  // a_L = u K_o^T
    for (int l = L; l >= 1; --l) {
      hipLaunchKernelGGL(mlp_gchain, dim3(grid_for(SW)), dim3(kBlock), 0, st, layer(l, 14), layer(l, 0),
                         layer(l, 10), SW);  // zeta_l -> ZB plane 3
      if (l > 1) b.bwd(layer(l, 10), params + poff[l - 1], layer(l - 1, 14), R, W, W);
      else b.bwd(layer(1, 10), params + poff[0], Gp, R, D, W);  // g = zeta_1 K_1^T
    }
    if (grad_only) {
      if (b.status) return fail(PDEINV_ERR_HIP, "mlp: rocBLAS call failed");
      return check_launch("mlp grad_x kernels");
    }
    // ---- loss terms, seed abar_0 = 2 c1 g (+ u) ------------------------------------------
    const int lg = grid_for(R) < kLossGrid ? grid_for(R) : kLossGrid;
    switch (D) {
#define CASE(DD) case DD: hipLaunchKernelGGL(mlp_loss<DD>, dim3(lg), dim3(kBlock), 0, st, la, Gp, zr, ld, terms, A0 + 3 * SD, R, part); break;
      CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(10) CASE(12) CASE(16)
#undef CASE
      default:
        return fail(PDEINV_ERR_UNSUPPORTED, "mlp: dim must be one of 1-8, 10, 12, 16");
    }
    hipLaunchKernelGGL(slab_reduce_accum_kernel, dim3(PDEINV_GMM_NACC), dim3(kBlock), 0, st, part, lg, acc);
    // ---- F2: forward-mode adjoint of the grad_x chain --------------------------------------
    for (int l = 1; l <= L; ++l) {
      const float* abar_prev = (l == 1) ? A0 + 3 * SD : layer(l - 1, 3);
      b.fwd(abar_prev, params + poff[l - 1], layer(l, 15), R, (l == 1) ? D : W, W);  // zetabar_l
      hipLaunchKernelGGL(mlp_gadj, dim3(grid_for(SW)), dim3(kBlock), 0, st, layer(l, 15), layer(l, 0),
                         layer(l, 3), SW);  // abar_l -> A plane 3
    }
    b.fwd(layer(L, 3), params + poff[L], UB, R, W, O);  // ubar = abar_L K_o
    hipLaunchKernelGGL(mlp_seeds, dim3(grid_for(SO)), dim3(kBlock), 0, st, Y, UB, YB, la.c2, la.c3, la.c0, SO,
                       la.uw ? zr + 3 * D : nullptr, ld, O);
    // ---- R2 + G: reverse over the three forward streams, weight gradients ---------------------
    b.wgrad(layer(L, 0), YB, grad + poff[L], 4 * R, W, O);  // K_o += [h;h';h'';abar]^T [ybar;..;u]
    b.colsum(YB, grad + boff[L], R, O);
    b.bwd(YB, params + poff[L], layer(L, 11), 3 * R, W, O);  // hbar streams of layer L
    for (int l = L; l >= 1; --l) {
      hipLaunchKernelGGL(mlp_act_bwd, dim3(grid_for(SW)), dim3(kBlock), 0, st, layer(l, 11), layer(l, 0),
                         layer(l, 4), layer(l, 14), layer(l, 15), layer(l, 7), SW);
      const int n_in = (l == 1) ? D : W;
      const float* Ain = (l == 1) ? A0 : layer(l - 1, 0);
      b.wgrad(Ain, layer(l, 7), grad + poff[l - 1], 4 * R, n_in, W);
      b.colsum(layer(l, 7), grad + boff[l - 1], R, W);
      if (l > 1) b.bwd(layer(l, 7), params + poff[l - 1], layer(l - 1, 11), 3 * R, W, W);
    }
    if (b.status) return fail(PDEINV_ERR_HIP, "mlp: rocBLAS call failed");
    return check_launch("mlp kernels");
  }
};
}  // namespace pdeinv

extern "C" int64_t pdeinv_mlp_param_count(int32_t dim, int32_t n_layers, int32_t width, int32_t out_features) {
  int64_t n = (int64_t)dim * width + width;
  for (int l = 1; l < n_layers; ++l) n += (int64_t)width * width + width;
  return n + (int64_t)width * out_features + out_features;
}

extern "C" int pdeinv_residual_kfp_mlp(const pdeinv_kfp_mlp_desc* d, const float* zi, int64_t ni, int64_t ldi,
                                       const float* zt, int64_t nt, int64_t ldt, const float* z0, int64_t n0,
                                       int64_t ld0, const float* params, void* ws, double* acc, float* grad,
                                       void* stream) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "kfp_mlp: null descriptor");
  const int D = d->dim;
  PDEINV_REQUIRE(D >= 1 && D <= 16, PDEINV_ERR_UNSUPPORTED, "kfp_mlp: dim must be in [1, 16]");
  PDEINV_REQUIRE(d->n_layers >= 1 && d->width >= 1 && d->out_features >= 1, PDEINV_ERR_INVALID,
                 "kfp_mlp: need n_layers, width, out_features >= 1");
  PDEINV_REQUIRE(d->impl >= PDEINV_MLP_IMPL_AUTO && d->impl <= PDEINV_MLP_IMPL_FUSED, PDEINV_ERR_INVALID,
                 "kfp_mlp: impl must be AUTO, LIBRARY or FUSED");
  PDEINV_REQUIRE(d->true_kind == PDEINV_POT_QUADRATIC || d->true_kind == PDEINV_POT_GMM, PDEINV_ERR_UNSUPPORTED,
                 "kfp_mlp: true potential must be QUADRATIC or GMM");
  PDEINV_REQUIRE(d->true_params != nullptr, PDEINV_ERR_INVALID, "kfp_mlp: true_params is null");
  PDEINV_REQUIRE(d->true_kind != PDEINV_POT_GMM || (d->n_centers_true >= 1 && d->n_centers_true <= 16 &&
                                                   d->n_centers_true * D <= PDEINV_MAX_PARAMS && d->sigma_true > 0.f),
                 PDEINV_ERR_UNSUPPORTED, "kfp_mlp: true GMM needs 1..16 centres");
  PDEINV_REQUIRE(n0 >= 1 && ni >= 0 && nt >= 0, PDEINV_ERR_INVALID, "kfp_mlp: 0T set must be non-empty");
  PDEINV_REQUIRE(params && ws && acc && grad && z0 && (ni == 0 || zi) && (nt == 0 || zt), PDEINV_ERR_INVALID,
                 "kfp_mlp: null pointer");
  // rocBLAS serves the explicit impl = LIBRARY only: AUTO / FUSED outside the hand-written envelope are rejected
  PDEINV_REQUIRE(d->impl == PDEINV_MLP_IMPL_LIBRARY || fused_shape(d), PDEINV_ERR_UNSUPPORTED,
                 "kfp_mlp: the hand-written path takes dim <= 16, 1 <= n_layers <= 16, width <= 1024 (zero-padded to "
                 "the compiled dims / widths), any out_features; impl = LIBRARY (rocBLAS) is the opt-in cross-check");
  const MlpPlan p = make_plan(d);
  PDEINV_REQUIRE(p.Bc <= (1 << 26), PDEINV_ERR_INVALID, "kfp_mlp: chunk_rows too large");
  hipStream_t st = (hipStream_t)stream;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(PDEINV_ERR_HIP, "kfp_mlp: hipGetDevice failed");
  float* w = (float*)ws;
  const int W = p.W, O = p.O, L = p.L;
  PDEINV_REQUIRE(L <= 16, PDEINV_ERR_UNSUPPORTED, "kfp_mlp: at most 16 hidden layers");
  int64_t poff[18], boff[18];
  param_offsets(D, W, O, L, poff, boff);

  MlpLossArgs la{};
  la.d = D;
  la.true_kind = d->true_kind;
  la.KT = d->n_centers_true;
  la.s2t = d->sigma_true > 0.f ? 1.f / (d->sigma_true * d->sigma_true) : 1.f;
  la.l2st = la.s2t * 1.4426950408889634f;
  const int ntp = d->true_kind == PDEINV_POT_QUADRATIC ? D * D : d->n_centers_true * D;
  for (int k = 0; k < ntp; ++k) la.tp[k] = d->true_params[k];

  // boundary sets weight V' (kinetic FP, :49-50) or V itself (overdamped FP, fokker_planck.py:48-52)
  const bool bval = d->boundary_value != 0;
  la.bval = bval ? 1 : 0;
  struct Set { const float* z; int64_t n, ld; int id; float c1, c2, c3, c0; } sets[3] = {
      {z0, n0, ld0 ? ld0 : 2 * D, 0, d->c_nabla, d->c_hess, d->c_fric, 0.f},
      {zi, ni, ldi ? ldi : 2 * D, 1, 0.f, 0.f, bval ? 0.f : d->c_init, bval ? d->c_init : 0.f},
      {zt, nt, ldt ? ldt : 2 * D, 2, 0.f, 0.f, bval ? 0.f : d->c_term, bval ? d->c_term : 0.f}};
  FusedShape fs;
  if (fused_shape(d, &fs)) {
    const int64_t Bc = chunk_rows_of(d);
    const int Wf = fs.Wp, Dp = fs.Dp;
    const FusedWs fw = fused_ws(d, fs);
    float* wsf = (float*)ws;
    const float* fparams = params;
    float* fgrad = grad;
    MlpPadMap pm{};
    if (fs.pad) {  // zero-padded copy of the parameters and a padded gradient accumulator behind the workspace
      pm = width_pad_map(d, fs);
      float* pbuf = wsf + fw.pbuf;
      float* gbuf = wsf + fw.gbuf;
      hipLaunchKernelGGL(mlp_pad_params_kernel, dim3((unsigned)((fw.PP + 255) / 256)), dim3(256), 0, st, pm, params,
                         fw.PP, pbuf);
      if (hipMemsetAsync(gbuf, 0, sizeof(float) * fw.PP, st) != hipSuccess)
        return fail(PDEINV_ERR_HIP, "kfp_mlp: memset");
      fparams = pbuf;
      fgrad = gbuf;
      param_offsets(Dp, Wf, O, L, poff, boff);
    }
    LossCtx lc{};
    lc.la = la;
    if (Dp != D) {  // the true potential on padded rows: zero rows / columns of tilde_F, zero coordinates of mu_k
      lc.la.d = Dp;
      for (int k = 0; k < PDEINV_MAX_PARAMS; ++k) lc.la.tp[k] = 0.f;
      if (d->true_kind == PDEINV_POT_QUADRATIC) {
        for (int i = 0; i < D; ++i)
          for (int j = 0; j < D; ++j) lc.la.tp[i * Dp + j] = d->true_params[i * D + j];
      } else {
        PDEINV_REQUIRE(d->n_centers_true * Dp <= PDEINV_MAX_PARAMS, PDEINV_ERR_UNSUPPORTED,
                       "kfp_mlp: padded true GMM exceeds PDEINV_MAX_PARAMS");
        for (int k = 0; k < d->n_centers_true; ++k)
          for (int i = 0; i < D; ++i) lc.la.tp[k * Dp + i] = d->true_params[k * D + i];
      }
    }
    lc.part = wsf + fw.part;
    lc.acc = acc;
    lc.D = Dp;
    for (const Set& s : sets) {
      PDEINV_REQUIRE(s.n == 0 || s.ld >= 2 * D, PDEINV_ERR_INVALID, "kfp_mlp: row stride < 2*dim");
      lc.la.set = s.id; lc.la.c1 = s.c1; lc.la.c2 = s.c2; lc.la.c3 = s.c3; lc.la.c0 = s.c0; lc.la.c_true = d->c_true;
      lc.la.inv_n = s.n ? 1.f / (float)s.n : 0.f;
      for (int64_t r0 = 0; r0 < s.n; r0 += Bc) {
        mlpf::Chunk c{};
        c.d = Dp; c.L = L; c.W = Wf; c.O = p.O;
        c.R = (s.n - r0) < Bc ? (s.n - r0) : Bc;
        c.z = s.z + r0 * s.ld;
        c.ldz = s.ld;
        if (Dp != D) {
          float* rows = wsf + fw.rows;
          const int64_t nq = c.R * 2 * Dp;
          hipLaunchKernelGGL(mlp_pad_rows_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, c.z, s.ld, c.R,
                             D, Dp, rows);
          c.z = rows;
          c.ldz = 2 * Dp;
        }
        c.params = fparams; c.grad = fgrad; c.poff = poff; c.boff = boff;
        c.c2 = s.c2; c.c3 = s.c3; c.c0 = s.c0;
        c.ws = wsf; c.Bc = Bc;
        // the initial / terminal sets weight V' (or V) only: no R1 / F2 (kinetic_fokker_planck.py:34-39)
        c.first_order = s.id != 0 && s.c1 == 0.f && s.c2 == 0.f && first_order_enabled();
        lc.zr = c.z;
        lc.ld = c.ldz;
        const int rc = mlpf::run_chunk(c, mlpf::LossHook{fused_loss_hook, &lc}, st);
        if (rc) return rc;
      }
    }
    if (fs.pad) {
      hipLaunchKernelGGL(mlp_unpad_grad_kernel, dim3((unsigned)((fw.PP + 255) / 256)), dim3(256), 0, st, pm, fgrad,
                         fw.PP, grad);
      return check_launch("mlp_unpad_grad_kernel");
    }
    return PDEINV_OK;
  }
  Blas blas{blas_handle(dev), st, w + p.off_kpart};
  PDEINV_REQUIRE(blas_api().ok, PDEINV_ERR_UNSUPPORTED,
                 "kfp_mlp: impl = LIBRARY needs rocBLAS (librocblas.so.5 could not be loaded)");
  if (!blas.h) return fail(PDEINV_ERR_HIP, "kfp_mlp: rocblas_create_handle failed");
  if (blas_api().set_stream(blas.h, st) != rocblas_status_success) return fail(PDEINV_ERR_HIP, "kfp_mlp: rocblas_set_stream");
  g_rocblas_calls.fetch_add(1, std::memory_order_relaxed);
  LibRun run{p, &blas, w, params, grad, poff, boff, st, acc};
  for (const Set& s : sets) {
    PDEINV_REQUIRE(s.n == 0 || s.ld >= 2 * D, PDEINV_ERR_INVALID, "kfp_mlp: row stride < 2*dim");
    la.set = s.id; la.c1 = s.c1; la.c2 = s.c2; la.c3 = s.c3; la.c0 = s.c0; la.c_true = d->c_true;
    la.inv_n = s.n ? 1.f / (float)s.n : 0.f;
    for (int64_t r0 = 0; r0 < s.n; r0 += p.Bc) {
      const int64_t R = (s.n - r0) < p.Bc ? (s.n - r0) : p.Bc;
      const int rc = run.chunk(s.z + r0 * s.ld, s.ld, R, la, false);
      if (rc) return rc;
    }
  }
  return PDEINV_OK;
}

// ---- KMV residual for a general (MLP) interaction Phi_theta = V_hypothesis ----------------------
// (methods/consistency_instances/kinetic_mckean_vlasov.py:11-120 under get_model non-parametric.)
// Per time stamp t the reference forms every pair (i, j) of its particles, y = x_i - x_j
// (x_minus_ref, :20-23), and needs  gbar_i = mean_j grad Phi(y_ij),  mean_j v_i^T Hess Phi(y_ij) v_i
// and  mean_j Phi(y_ij)  weighted by c_it = ds2 + ds^2 + gamma ds of log rho. The loss is quadratic
// in gbar, so its parameter adjoint is per pair once gbar is known — two passes over pair rows
// [y_ij | v_i | u_i | w_it] (built chunk by chunk, never the whole n^2 tensor):
//   pass 1  grad_x V of the pair rows (F1 + R1 of the library path), mean over j -> gbar (fp32 ws);
//           |gbar|^2, |gbar*|^2, |gbar* - gbar|^2 with gbar* = tilde_F (x_i - xbar_t) (Phi* quadratic);
//   pass 2  the full library path with c2 = -2 s, c0 = 2 s w_it and the input-gradient seed
//           u_i = 2 s gbar_i, s = 1 / (n^2 n_time)  (oracle/numpy_ref.py kmv_mlp_grad_analytic).
// rows of DP >= D floats per block: the particles' D coordinates, zeros past them (the fused path's dim padding)
template <int D, int DP = D>
__global__ void kmv_pair_rows_kernel(const float* __restrict__ z, int64_t set_stride, int64_t ld, int64_t t,
                                     int64_t i0, int64_t ni, int64_t j0, int64_t nj, int64_t n_rows,
                                     const float* __restrict__ gbar, const float* __restrict__ ds, float gamma,
                                     float u_scale, float* __restrict__ rows) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= ni * nj) return;
  const int64_t il = r / nj, i = i0 + il, j = j0 + (r - il * nj);
  const float* zi = z + t * set_stride + i * ld;
  const float* zj = z + t * set_stride + j * ld;
  float* o = rows + r * (3 * DP + 1);
  const int64_t p = t * n_rows + i;
#pragma unroll
  for (int k = 0; k < DP; ++k) {
    o[k] = k < D ? zi[k] - zj[k] : 0.f;
    o[DP + k] = k < D ? zi[D + k] : 0.f;
    o[2 * DP + k] = (k < D && gbar) ? u_scale * gbar[p * D + k] : 0.f;
  }
  float wv = 0.f;
  if (ds) {
    const float a = ds[2 * p], b2 = ds[2 * p + 1];
    wv = b2 + a * a + gamma * a;  // ds2 + ds^2 + gamma ds (kinetic_mckean_vlasov.py:84-89)
  }
  o[3 * DP] = wv;
}

// gbar[t][i0 + il] += inv_n * sum_jl G[il * nj + jl] (one block per il; fixed-order LDS tree)
template <int D, int DP = D>
__global__ __launch_bounds__(kBlock) void kmv_group_mean_kernel(const float* __restrict__ G, int64_t nj, float inv_n,
                                                                float* __restrict__ gbar_rows) {
  const int64_t il = blockIdx.x;
  float s[D];
#pragma unroll
  for (int k = 0; k < D; ++k) s[k] = 0.f;
  for (int64_t jl = threadIdx.x; jl < nj; jl += kBlock) {
#pragma unroll
    for (int k = 0; k < D; ++k) s[k] += G[(il * nj + jl) * DP + k];  // G rows of DP (padded dims dropped)
  }
  __shared__ float red[kBlock];
  for (int k = 0; k < D; ++k) {
    red[threadIdx.x] = s[k];
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
      if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) gbar_rows[il * D + k] += inv_n * red[0];
    __syncthreads();
  }
}

struct KmvTrueArgs {
  float F[PDEINV_MAX_DIM * PDEINV_MAX_DIM];
};

// per time stamp t (one block): xbar_t, then sum_i |gbar|^2, |gbar*|^2, |gbar* - gbar|^2 -> part[t][3]
template <int D>
__global__ __launch_bounds__(kBlock) void kmv_stamp_terms_kernel(KmvTrueArgs a, const float* __restrict__ z,
                                                                int64_t set_stride, int64_t ld, int64_t n_rows,
                                                                const float* __restrict__ gbar,
                                                                double* __restrict__ part) {
  const int64_t t = blockIdx.x;
  const float* zt = z + t * set_stride;
  __shared__ double red[kBlock];
  __shared__ float xbar[D];
  for (int k = 0; k < D; ++k) {
    double sk = 0.0;
    for (int64_t i = threadIdx.x; i < n_rows; i += kBlock) sk += (double)zt[i * ld + k];
    red[threadIdx.x] = sk;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
      if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) xbar[k] = (float)(red[0] / (double)n_rows);
    __syncthreads();
  }
  double acc[3] = {0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < n_rows; i += kBlock) {
    float y[D];
#pragma unroll
    for (int k = 0; k < D; ++k) y[k] = zt[i * ld + k] - xbar[k];
    const float* g = gbar + (t * n_rows + i) * D;
    float n1 = 0.f, n2 = 0.f, n3 = 0.f;
#pragma unroll
    for (int r = 0; r < D; ++r) {
      float gt = 0.f;
#pragma unroll
      for (int c = 0; c < D; ++c) gt = fmaf(a.F[r * D + c], y[c], gt);
      n1 = fmaf(g[r], g[r], n1);
      n2 = fmaf(gt, gt, n2);
      n3 = fmaf(gt - g[r], gt - g[r], n3);
    }
    acc[0] += n1; acc[1] += n2; acc[2] += n3;
  }
  for (int c = 0; c < 3; ++c) {
    red[threadIdx.x] = acc[c];
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
      if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) part[t * 3 + c] = red[0];
    __syncthreads();
  }
}

// fixed-order combine of the per-stamp sums into the PDEINV_GMM_ACC_* slots (+=)
__global__ void kmv_stamp_combine_kernel(const double* __restrict__ part, int64_t n_sets, double inv,
                                         double* __restrict__ acc) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double n1 = 0.0, n2 = 0.0, n3 = 0.0;
  for (int64_t t = 0; t < n_sets; ++t) {
    n1 += part[t * 3];
    n2 += part[t * 3 + 1];
    n3 += part[t * 3 + 2];
  }
  acc[PDEINV_GMM_ACC_LOSS] += (n1 + n2) * inv;
  acc[PDEINV_GMM_ACC_LOSS_GT] += n3 * inv;
  acc[PDEINV_GMM_ACC_NABLA] += n1 * inv;
  acc[PDEINV_GMM_ACC_NABLA_TRUE] += n2 * inv;
}

namespace {
struct KmvPlan {
  MlpPlan lib;
  int64_t ni, nj;           // pair-row block: ni particles x nj references
  size_t off_rows, off_gbar, off_part, total;  // floats past the library plan (part: doubles)
};

KmvPlan kmv_plan(const pdeinv_kmv_mlp_desc* d) {
  pdeinv_kfp_mlp_desc m{};
  m.dim = d->dim; m.n_layers = d->n_layers; m.width = d->width; m.out_features = d->out_features;
  m.chunk_rows = d->chunk_rows > 0 ? d->chunk_rows : (1 << 18);
  KmvPlan k{};
  k.lib = make_plan(&m);
  const int64_t Bc = k.lib.Bc, n = d->n_rows;
  k.nj = n <= Bc ? n : Bc;
  k.ni = n <= Bc ? (Bc / n < n ? Bc / n : n) : 1;
  size_t o = k.lib.total / sizeof(float);
  auto take = [&](size_t floats) { const size_t at = o; o += (floats + 63) & ~(size_t)63; return at; };
  k.off_rows = take((size_t)Bc * (3 * d->dim + 1));
  k.off_gbar = take((size_t)d->n_sets * n * d->dim);
  k.off_part = take((size_t)d->n_sets * 3 * 2);
  k.total = o * sizeof(float);
  return k;
}
}  // namespace

template <int D>
static int kmv_mlp_run(const pdeinv_kmv_mlp_desc* d, const KmvPlan& k, const float* z, int64_t set_stride,
                       int64_t ld, const float* ds, const float* params, float* w, double* acc, float* grad,
                       hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(PDEINV_ERR_HIP, "kmv_mlp: hipGetDevice failed");
  Blas blas{blas_handle(dev), st, w + k.lib.off_kpart};
  PDEINV_REQUIRE(blas_api().ok, PDEINV_ERR_UNSUPPORTED,
                 "kmv_mlp: impl = LIBRARY needs rocBLAS (librocblas.so.5 could not be loaded)");
  if (!blas.h) return fail(PDEINV_ERR_HIP, "kmv_mlp: rocblas_create_handle failed");
  if (blas_api().set_stream(blas.h, st) != rocblas_status_success) return fail(PDEINV_ERR_HIP, "kmv_mlp: rocblas_set_stream");
  g_rocblas_calls.fetch_add(1, std::memory_order_relaxed);
  int64_t poff[18], boff[18];
  param_offsets(D, d->width, d->out_features, d->n_layers, poff, boff);
  LibRun run{k.lib, &blas, w, params, grad, poff, boff, st, acc};
  const int64_t n = d->n_rows, T = d->n_sets, rld = 3 * D + 1;
  float* rows = w + k.off_rows;
  float* gbar = w + k.off_gbar;
  double* part = (double*)(w + k.off_part);
  const double s = 1.0 / ((double)n * (double)n * (double)T);
  if (hipMemsetAsync(gbar, 0, sizeof(float) * (size_t)T * n * D, st) != hipSuccess)
    return fail(PDEINV_ERR_HIP, "kmv_mlp: memset");
  MlpLossArgs la{};
  la.d = D;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      la.set = 3; la.uw = 1;
      la.c1 = 0.f; la.c3 = 0.f; la.c2 = (float)(-2.0 * s); la.c0 = (float)(2.0 * s);
    }
    for (int64_t t = 0; t < T; ++t) {
      for (int64_t i0 = 0; i0 < n; i0 += k.ni) {
        const int64_t ni = (n - i0) < k.ni ? (n - i0) : k.ni;
        for (int64_t j0 = 0; j0 < n; j0 += k.nj) {
          const int64_t nj = (n - j0) < k.nj ? (n - j0) : k.nj;
          const int64_t R = ni * nj;
          hipLaunchKernelGGL(kmv_pair_rows_kernel<D>, dim3(grid_for(R)), dim3(kBlock), 0, st, z, set_stride, ld, t,
                             i0, ni, j0, nj, n, pass ? gbar : nullptr, pass ? ds : nullptr, d->gamma,
                             (float)(2.0 * s), rows);
          const int rc = run.chunk(rows, rld, R, la, pass == 0);
          if (rc) return rc;
          if (pass == 0)
            hipLaunchKernelGGL(kmv_group_mean_kernel<D>, dim3((unsigned)ni), dim3(kBlock), 0, st, run.G(), nj,
                               (float)(1.0 / (double)n), gbar + (t * n + i0) * D);
        }
      }
    }
    if (pass == 0) {
      KmvTrueArgs ta{};
      for (int q = 0; q < D * D; ++q) ta.F[q] = d->tilde_F[q];
      hipLaunchKernelGGL(kmv_stamp_terms_kernel<D>, dim3((unsigned)T), dim3(kBlock), 0, st, ta, z, set_stride, ld, n,
                         gbar, part);
      hipLaunchKernelGGL(kmv_stamp_combine_kernel, dim3(1), dim3(64), 0, st, part, T, 1.0 / ((double)n * (double)T),
                         acc);
    }
  }
  return check_launch("kmv_mlp kernels");
}

// the narrow-net pair kernels (mlp_pairs.hip): pairs generated in registers, MFMA weight gradients
namespace pdeinv {
bool kmv_pairs_supported(const pdeinv_kmv_mlp_desc* d);
bool kmvq_supported(const pdeinv_kmv_mlp_desc* d);
size_t kmv_pairs_workspace_bytes(const pdeinv_kmv_mlp_desc* d);
int kmv_pairs_run(const pdeinv_kmv_mlp_desc* d, const float* z, int64_t set_stride, int64_t ld, const float* ds,
                  const float* params, void* ws, double* acc, float* grad, float** gbar_out, int pass, hipStream_t st);
}  // namespace pdeinv

static bool kmv_use_pairs(const pdeinv_kmv_mlp_desc* d) {
  return d->impl != PDEINV_MLP_IMPL_LIBRARY && kmv_pairs_supported(d);
}

// ---- wide general-Phi nets (width >= 32): the pair rows through the fused fp32-MFMA path ------------
// Pair rows [y_ij | v_i | u_i | w_it] are built chunk by chunk exactly as for the library path, then run
// through mlpf::run_chunk (the C5 machinery: B-resident row GEMMs, LDS-free weight gradients) — pass 1 in
// its grad-only mode (g = grad_x Phi per pair -> mean over j), pass 2 with the per-row value weight
// w_it on c0 and the input-gradient seed u_i in the loss hook. Widths between the compiled ones are
// zero-padded (exact, common.h MlpPadMap). No rocBLAS on this path.
static pdeinv_kfp_mlp_desc kmv_as_kfp(const pdeinv_kmv_mlp_desc* d) {
  pdeinv_kfp_mlp_desc m{};
  m.dim = d->dim; m.n_layers = d->n_layers; m.width = d->width; m.out_features = d->out_features;
  m.chunk_rows = d->chunk_rows > 0 ? d->chunk_rows : (1 << 18);
  m.impl = d->impl;
  return m;
}

static bool kmv_use_fused(const pdeinv_kmv_mlp_desc* d) {
  if (d->impl == PDEINV_MLP_IMPL_LIBRARY || kmv_use_pairs(d)) return false;
  if (d->dim < 1 || d->dim > 16) return false;
  const pdeinv_kfp_mlp_desc m = kmv_as_kfp(d);
  return fused_shape(&m);
}

namespace {
struct KmvFusedPlan {
  int Wf, Dp;
  bool pad;
  int64_t Bc, ni, nj, PP;
  MlpPadMap pm;
  size_t fl, off_part, off_pbuf, off_gbuf, off_rows, off_gbar, off_spart, total;  // floats
};

KmvFusedPlan kmv_fused_plan(const pdeinv_kmv_mlp_desc* d) {
  const pdeinv_kfp_mlp_desc m = kmv_as_kfp(d);
  KmvFusedPlan k{};
  FusedShape fs;
  fused_shape(&m, &fs);
  k.Wf = fs.Wp;
  k.Dp = fs.Dp;
  k.pad = fs.pad;
  k.Bc = m.chunk_rows;
  const int64_t n = d->n_rows;
  k.nj = n <= k.Bc ? n : k.Bc;
  k.ni = n <= k.Bc ? (k.Bc / n < n ? k.Bc / n : n) : 1;
  if (k.pad) {
    k.pm = width_pad_map(&m, fs);
    k.PP = pad_param_count(k.pm);
  }
  size_t o = 0;
  auto take = [&](size_t floats) { const size_t at = o; o += (floats + 63) & ~(size_t)63; return at; };
  k.fl = take(mlpf::workspace_floats(k.Dp, d->n_layers, k.Wf, d->out_features, k.Bc));
  k.off_part = take((size_t)PDEINV_GMM_NACC * kLossGrid);
  k.off_pbuf = take((size_t)k.PP);
  k.off_gbuf = take((size_t)k.PP);
  k.off_rows = take((size_t)k.Bc * (3 * k.Dp + 1));
  k.off_gbar = take((size_t)d->n_sets * n * d->dim);
  k.off_spart = take((size_t)d->n_sets * 3 * 2);
  k.total = o * sizeof(float);
  return k;
}
}  // namespace

// D = the particles' dim, DP = the fused kernels' (D zero-padded to 2 / 4 / 8: the pair rows carry the padding)
template <int D, int DP>
static int kmv_fused_run(const pdeinv_kmv_mlp_desc* d, const KmvFusedPlan& k, const float* z, int64_t set_stride,
                         int64_t ld, const float* ds, const float* params, float* w, double* acc, float* grad,
                         hipStream_t st) {
  const int L = d->n_layers, O = d->out_features;
  int64_t poff[18], boff[18];
  param_offsets(DP, k.Wf, O, L, poff, boff);
  const float* fparams = params;
  float* fgrad = grad;
  if (k.pad) {
    float* pbuf = w + k.off_pbuf;
    fgrad = w + k.off_gbuf;
    hipLaunchKernelGGL(mlp_pad_params_kernel, dim3((unsigned)((k.PP + 255) / 256)), dim3(256), 0, st, k.pm, params,
                       k.PP, pbuf);
    if (hipMemsetAsync(fgrad, 0, sizeof(float) * k.PP, st) != hipSuccess) return fail(PDEINV_ERR_HIP, "kmv_mlp: memset");
    fparams = pbuf;
  }
  const int64_t n = d->n_rows, T = d->n_sets, rld = 3 * DP + 1;
  float* rows = w + k.off_rows;
  float* gbar = w + k.off_gbar;
  double* part = (double*)(w + k.off_spart);
  const double s = 1.0 / ((double)n * (double)n * (double)T);
  if (hipMemsetAsync(gbar, 0, sizeof(float) * (size_t)T * n * D, st) != hipSuccess)
    return fail(PDEINV_ERR_HIP, "kmv_mlp: memset");
  LossCtx lc{};
  lc.la.d = DP;
  lc.la.set = 3;
  lc.la.uw = 1;
  lc.la.c2 = (float)(-2.0 * s);
  lc.la.c0 = (float)(2.0 * s);
  lc.part = w + k.off_part;
  lc.acc = acc;
  lc.D = DP;
  lc.zr = rows;
  lc.ld = rld;
  mlpf::Chunk c{};
  c.d = DP; c.L = L; c.W = k.Wf; c.O = O;
  c.z = rows; c.ldz = rld;
  c.params = fparams; c.grad = fgrad; c.poff = poff; c.boff = boff;
  c.ws = w; c.Bc = k.Bc;
  for (int pass = 0; pass < 2; ++pass) {
    c.grad_only = pass == 0;
    c.c2 = pass ? lc.la.c2 : 0.f;
    c.c3 = 0.f;
    c.c0 = pass ? lc.la.c0 : 0.f;
    c.wrow = pass ? rows + 3 * DP : nullptr;
    c.ldw = rld;
    for (int64_t t = 0; t < T; ++t) {
      for (int64_t i0 = 0; i0 < n; i0 += k.ni) {
        const int64_t ni = (n - i0) < k.ni ? (n - i0) : k.ni;
        for (int64_t j0 = 0; j0 < n; j0 += k.nj) {
          const int64_t nj = (n - j0) < k.nj ? (n - j0) : k.nj;
          c.R = ni * nj;
          hipLaunchKernelGGL((kmv_pair_rows_kernel<D, DP>), dim3(grid_for(c.R)), dim3(kBlock), 0, st, z, set_stride, ld,
                             t, i0, ni, j0, nj, n, pass ? gbar : nullptr, pass ? ds : nullptr, d->gamma,
                             (float)(2.0 * s), rows);
          const int rc = mlpf::run_chunk(c, mlpf::LossHook{fused_loss_hook, &lc}, st);
          if (rc) return rc;
          if (pass == 0)
            hipLaunchKernelGGL((kmv_group_mean_kernel<D, DP>), dim3((unsigned)ni), dim3(kBlock), 0, st,
                               mlpf::grad_rows(c), nj, (float)(1.0 / (double)n), gbar + (t * n + i0) * D);
        }
      }
    }
    if (pass == 0) {
      KmvTrueArgs ta{};
      for (int q = 0; q < D * D; ++q) ta.F[q] = d->tilde_F[q];
      hipLaunchKernelGGL(kmv_stamp_terms_kernel<D>, dim3((unsigned)T), dim3(kBlock), 0, st, ta, z, set_stride, ld, n,
                         gbar, part);
      hipLaunchKernelGGL(kmv_stamp_combine_kernel, dim3(1), dim3(64), 0, st, part, T, 1.0 / ((double)n * (double)T),
                         acc);
    }
  }
  if (k.pad)
    hipLaunchKernelGGL(mlp_unpad_grad_kernel, dim3((unsigned)((k.PP + 255) / 256)), dim3(256), 0, st, k.pm, fgrad,
                       k.PP, grad);
  return check_launch("kmv_mlp fused kernels");
}

static size_t kmv_pairs_part_offset(const pdeinv_kmv_mlp_desc* d) { return (kmv_pairs_workspace_bytes(d) + 255) & ~(size_t)255; }

extern "C" int pdeinv_kmv_mlp_path(const pdeinv_kmv_mlp_desc* d) {
  if (!d || d->dim < 1 || d->n_layers < 1 || d->n_layers > 16 || d->width < 1 || d->out_features < 1) return -1;
  if (kmv_use_pairs(d)) return kmvq_supported(d) ? PDEINV_KMV_PATH_PAIR_TILES : PDEINV_KMV_PATH_PAIR_RING;
  if (d->impl == PDEINV_MLP_IMPL_PAIRS_RING) return -1;
  if (kmv_use_fused(d)) return PDEINV_KMV_PATH_FUSED_ROWS;
  // rocBLAS only on the explicit opt-in, and only for the shapes its kernels take (dim 1..8)
  return d->impl == PDEINV_MLP_IMPL_LIBRARY && d->dim <= 8 ? PDEINV_KMV_PATH_LIBRARY : -1;
}

extern "C" size_t pdeinv_residual_kmv_mlp_workspace_bytes(const pdeinv_kmv_mlp_desc* d) {
  if (!d || d->dim < 1 || d->n_layers < 1 || d->width < 1 || d->out_features < 1 || d->n_sets < 1 || d->n_rows < 1)
    return 0;
  if (kmv_use_pairs(d)) return kmv_pairs_part_offset(d) + sizeof(double) * (size_t)d->n_sets * 3;
  if (kmv_use_fused(d)) return kmv_fused_plan(d).total;
  return kmv_plan(d).total;
}

template <int D>
static int kmv_pairs_orchestrate(const pdeinv_kmv_mlp_desc* d, const float* z, int64_t set_stride, int64_t ld,
                                 const float* ds, const float* params, void* ws, double* acc, float* grad,
                                 hipStream_t st) {
  float* gbar = nullptr;
  int rc = kmv_pairs_run(d, z, set_stride, ld, ds, params, ws, acc, grad, &gbar, 0, st);
  if (rc) return rc;
  double* part = (double*)((char*)ws + kmv_pairs_part_offset(d));
  KmvTrueArgs ta{};
  for (int q = 0; q < D * D; ++q) ta.F[q] = d->tilde_F[q];
  const int64_t n = d->n_rows, T = d->n_sets;
  hipLaunchKernelGGL(kmv_stamp_terms_kernel<D>, dim3((unsigned)T), dim3(kBlock), 0, st, ta, z, set_stride, ld, n, gbar,
                     part);
  hipLaunchKernelGGL(kmv_stamp_combine_kernel, dim3(1), dim3(64), 0, st, part, T, 1.0 / ((double)n * (double)T), acc);
  rc = check_launch("kmv_stamp kernels");
  if (rc) return rc;
  return kmv_pairs_run(d, z, set_stride, ld, ds, params, ws, acc, grad, nullptr, 1, st);
}

extern "C" int pdeinv_residual_kmv_mlp(const pdeinv_kmv_mlp_desc* d, const float* z, int64_t set_stride, int64_t ld,
                                       const float* ds, const float* params, void* ws, double* acc, float* grad,
                                       void* stream) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "kmv_mlp: null descriptor");
  PDEINV_REQUIRE(d->n_layers >= 1 && d->n_layers <= 16 && d->width >= 1 && d->out_features >= 1, PDEINV_ERR_INVALID,
                 "kmv_mlp: need 1 <= n_layers <= 16, width, out_features >= 1");
  PDEINV_REQUIRE(d->n_sets >= 1 && d->n_rows >= 1, PDEINV_ERR_INVALID, "kmv_mlp: need n_sets, n_rows >= 1");
  PDEINV_REQUIRE(ld >= 2 * d->dim && set_stride >= 0, PDEINV_ERR_INVALID, "kmv_mlp: row stride < 2*dim");
  PDEINV_REQUIRE(z && ds && params && ws && acc && grad && d->tilde_F, PDEINV_ERR_INVALID, "kmv_mlp: null pointer");
  PDEINV_REQUIRE(d->impl >= PDEINV_MLP_IMPL_AUTO && d->impl <= PDEINV_MLP_IMPL_PAIRS_RING, PDEINV_ERR_INVALID,
                 "kmv_mlp: impl must be AUTO, LIBRARY, FUSED or PAIRS_RING");
  PDEINV_REQUIRE(d->impl != PDEINV_MLP_IMPL_PAIRS_RING || kmv_use_pairs(d), PDEINV_ERR_UNSUPPORTED,
                 "kmv_mlp: PAIRS_RING needs dim <= 8, width <= 28, n_layers <= 16, out_features <= 64");
  PDEINV_REQUIRE(pdeinv_kmv_mlp_path(d) >= 0, PDEINV_ERR_UNSUPPORTED,
                 "kmv_mlp: the hand-written paths need dim <= 8 with width <= 28 (pair kernels), or dim <= 16 with "
                 "1 <= n_layers <= 16, width <= 1024 (fused MFMA path); impl = LIBRARY (rocBLAS, dim <= 8) is the "
                 "opt-in cross-check");
  hipStream_t st = (hipStream_t)stream;
  if (kmv_use_pairs(d)) {
    switch (d->dim) {
#define CASE(DD) case DD: return kmv_pairs_orchestrate<DD>(d, z, set_stride, ld, ds, params, ws, acc, grad, st);
      CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
    }
  }
  if (kmv_use_fused(d)) {
    const KmvFusedPlan k = kmv_fused_plan(d);
    switch (d->dim) {
#define CASE(DD, DDP) \
  case DD: return kmv_fused_run<DD, DDP>(d, k, z, set_stride, ld, ds, params, (float*)ws, acc, grad, st);
      CASE(1, 2) CASE(2, 2) CASE(3, 4) CASE(4, 4) CASE(5, 8) CASE(6, 8) CASE(7, 8) CASE(8, 8)
      CASE(9, 16) CASE(10, 16) CASE(11, 16) CASE(12, 16) CASE(13, 16) CASE(14, 16) CASE(15, 16) CASE(16, 16)
#undef CASE
    }
  }
  const KmvPlan k = kmv_plan(d);
  switch (d->dim) {
#define CASE(DD) case DD: return kmv_mlp_run<DD>(d, k, z, set_stride, ld, ds, params, (float*)ws, acc, grad, st);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "kmv_mlp: dim must be in [1, 8]");
  }
}

extern "C" int pdeinv_kfp_terms_finalize(const double* acc, const float* grad, int64_t n_grad, float gamma,
                                         float* out, void* stream) {
  PDEINV_REQUIRE(acc && grad && out && n_grad >= 0, PDEINV_ERR_INVALID, "kfp_terms_finalize: bad arguments");
  hipLaunchKernelGGL(kfp_terms_finalize_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, acc, grad, n_grad,
                     gamma, out);
  return check_launch("kfp_terms_finalize_kernel");
}
