// kmv.hip — McKean–Vlasov residual path (gfx950): per-time-stamp moments, the Gaussian
// score / log-density time derivatives per particle, and the residual finalize.
//
// The reference forms all pairs x_i - x_j per time stamp ([m, n, n_time, d],
// kinetic_mckean_vlasov.py:20-23) and triple-vmaps autodiff over them. For the quadratic
// interaction Phi_theta(y) = y^T K y + b^T y every pairwise mean is a function of the time
// stamp's moments, so the O(n^2) tensor becomes two streaming passes (moments, weights)
// plus an O(n_time d^3) finalize — exact, not an approximation.
#include <math.h>
#include <stdlib.h>

#include "common.h"

namespace pdeinv {

constexpr int kBatchedGridTarget = 4096;  // C4 KMV pass: r02 2.88 ms at 2048, 2.785 at 3072; r04 (buffer loads) 2.52 at 3072, 2.486 at 4096, 2.51 at 6144 (profiles/r04_kmv_grid_ab.txt)

static int64_t grid_target() {
  static const int64_t t = [] {
    const char* e = ab_env("PDEINV_KMV_GRID");  // A/B experiments (tools)
    return e ? (int64_t)atol(e) : (int64_t)kBatchedGridTarget;
  }();
  return t;
}

static int batched_bx(int64_t n_sets, int64_t n_rows) {
  int64_t bx = (grid_target() + n_sets - 1) / (n_sets > 0 ? n_sets : 1);
  const int64_t need = (n_rows + kBlock - 1) / kBlock;
  if (bx > need) bx = need;
  if (bx < 1) bx = 1;
  return (int)bx;
}

template <int M>
__global__ __launch_bounds__(kBlock) void moments_batched_kernel(const float* __restrict__ z, int64_t n_rows,
                                                                 int64_t set_stride, int64_t ld,
                                                                 float* __restrict__ partials) {
  MomentAcc<M> acc;
  acc.zero();
  const float* base = z + (int64_t)blockIdx.y * set_stride;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n_rows; r += stride) {
    const float* row = base + r * ld;
    float v[M];
#pragma unroll
    for (int k = 0; k < M; ++k) v[k] = row[k];
    acc.add(v, 1.f);
  }
  __shared__ float lds[kWavesPerBlock * moment_len(M)];
  // set t owns columns [t*L, (t+1)*L) of the slab
  block_reduce_to_slab(acc.v, moment_len(M), lds, partials + (int64_t)blockIdx.y * moment_len(M) * gridDim.x,
                       blockIdx.x, gridDim.x);
}

// ds log rho = a1 + beta1.r + r^T G1 r ; ds2 log rho = a2 + beta2.r + r^T G2 r ; r = m1 - x.
template <int D>
__global__ __launch_bounds__(kBlock) void kmv_weights_kernel(float gamma, const float* __restrict__ coef,
                                                             const float* __restrict__ z, int64_t n_rows,
                                                             int64_t set_stride, int64_t ld,
                                                             float* __restrict__ ds_out,
                                                             float* __restrict__ partials) {
  constexpr int NC = 3 * D + 2 + 2 * D * D;
  const int t = blockIdx.y;
  const float* c = coef + (int64_t)t * NC;  // wave-uniform: scalar loads
  const float* m1 = c;
  const float a1 = c[D];
  const float* b1 = c + D + 1;
  const float* G1 = c + 2 * D + 1;
  const float a2 = c[2 * D + 1 + D * D];
  const float* b2 = c + 2 * D + 2 + D * D;
  const float* G2 = c + 3 * D + 2 + D * D;
  MomentAcc<D> acc;
  acc.zero();
  const float* base = z + (int64_t)t * set_stride;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n_rows; r += stride) {
    const float* row = base + r * ld;
    float x[D], rr[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      x[k] = row[k];
      rr[k] = m1[k] - x[k];
    }
    float q1 = a1, q2 = a2;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      float g1 = b1[i], g2 = b2[i];
#pragma unroll
      for (int j = 0; j < D; ++j) {
        g1 = fmaf(G1[i * D + j], rr[j], g1);
        g2 = fmaf(G2[i * D + j], rr[j], g2);
      }
      q1 = fmaf(g1, rr[i], q1);
      q2 = fmaf(g2, rr[i], q2);
    }
    if (ds_out) {
      float* o = ds_out + ((int64_t)t * n_rows + r) * 2;
      o[0] = q1;
      o[1] = q2;
    }
    const float w = q2 + q1 * q1 + gamma * q1;  // kinetic_mckean_vlasov.py:243-248
    acc.add(x, w);
  }
  __shared__ float lds[kWavesPerBlock * moment_len(D)];
  block_reduce_to_slab(acc.v, moment_len(D), lds, partials + (int64_t)t * moment_len(D) * gridDim.x, blockIdx.x,
                       gridDim.x);
}

// Fused per-time-stamp pass: one read of each row z = [x, v] (2D floats) yields both the moments of
// z (the moments_batched sums) and the c-weighted sums of x (the kmv_weights sums): the McKean–Vlasov
// residual then reads its 2^21 x 100 x 64 B trajectory once instead of 1.5 times. Slab columns of set
// t: [moment_len(2D) | moment_len(D)].
//  * the Gram sum z z^T of a wave's 64 rows is 16 v_mfma_f32_16x16x4_f32 (A = B = the rows, K = rows,
//    features zero-padded to 16) into 4 accumulator registers per lane, fed through a per-wave LDS
//    transpose (row stride 20 floats: conflict-free 16-byte row writes); the lane-private alternative
//    (136 packed accumulators) left room for 2 waves per SIMD only;
//  * the per-row quadratic forms of d_s log rho and d_s^2 log rho run as packed pairs over coefficient
//    pairs (Gamma1_ij, Gamma2_ij) broadcast from LDS (as kernel SGPRs the 2 d^2 + 2 d coefficients spill),
//    over the symmetrised upper triangle: d(d+1)/2 LDS reads and packed FMAs per row instead of d^2
//    (this pass is bound by its per-row VALU / LDS work, not by HBM: 3.40 -> 2.81 ms at C4);
//  * packed rows (ld == 2d): the wave's 64 rows are read as one contiguous block (2d/4 coalesced
//    1 KiB loads) straight into the row stage, each lane then takes its own row back (3.80 -> 3.40 ms);
//  * count, sum z and the weighted moments stay lane-private (wave / block reduction at the end).
constexpr int kMwStride = 20;  // floats per staged row (16 features + pad)

//  * MF (pdeinv_kmv_moments_weights_mf_sums): the pass also sums the NEXT McKean–Vlasov simulate's
//    update-t noise over the stamp's particles (row r = particle poff + r), i.e. the mean-path input of
//    pdeinv_mf_sums for updates t < n_sets: that kernel is pure Philox / Box–Muller VALU work and this
//    pass is HBM-bound, so the RNG rides in the pass's idle issue slots instead of a separate launch.
template <int D, bool PACKED, bool MF = false>
__global__ __launch_bounds__(kBlock) void kmv_moments_weights_kernel(float gamma, const float* __restrict__ coef,
                                                                     const float* __restrict__ z, int64_t n_rows,
                                                                     int64_t set_stride, int64_t ld,
                                                                     float* __restrict__ partials,
                                                                     MfNoise mf = MfNoise{},
                                                                     float* __restrict__ mf_partials = nullptr) {
  constexpr int M = 2 * D, NC = 3 * D + 2 + 2 * D * D, LZ = moment_len(M), LW = moment_len(D);
  static_assert(M <= 16, "the 16x16 MFMA Gram holds 2d <= 16 features");
  const int t = blockIdx.y;
  const int lane = threadIdx.x & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const float* c = coef + (int64_t)t * NC;  // [m1 (D), a1, b1 (D), G1 (D*D), a2, b2 (D), G2 (D*D)]
  constexpr int NT = D * (D + 1) / 2;       // upper triangle of the symmetrised (G1, G2)
  __shared__ f32x2 cpair[NT + D];           // (G1_ij + G1_ji, G2_ij + G2_ji) for i < j, (G_ii) on the
                                            // diagonal, row-major over i <= j; then (b1_i, b2_i)
  __shared__ float stage[kWavesPerBlock][kWave * kMwStride];
  __shared__ float gram[kWavesPerBlock][16 * 16];
  for (int e = threadIdx.x; e < NT + D; e += kBlock) {
    if (e < NT) {  // triangle index e -> (i, j), i <= j
      int i = 0, rem = e;
      while (rem >= D - i) { rem -= D - i; ++i; }
      const int j = i + rem;
      const float* G1 = c + 2 * D + 1;
      const float* G2 = c + 3 * D + 2 + D * D;
      cpair[e] = i == j ? f32x2{G1[i * D + i], G2[i * D + i]}
                        : f32x2{G1[i * D + j] + G1[j * D + i], G2[i * D + j] + G2[j * D + i]};
    } else {
      cpair[e] = f32x2{c[D + 1 + (e - NT)], c[2 * D + 2 + D * D + (e - NT)]};
    }
  }
  float* srow = &stage[wave][lane * kMwStride];
#pragma unroll
  for (int k = M; k < 16; ++k) srow[k] = 0.f;  // padding features read as 0 by the MFMA
  __syncthreads();
  float m1[D];
#pragma unroll
  for (int k = 0; k < D; ++k) m1[k] = c[k];
  const f32x2 a12 = f32x2{c[D], c[2 * D + 1 + D * D]};

  f32x4 g4 = {0.f, 0.f, 0.f, 0.f};
  [[maybe_unused]] float xis[MF ? D : 1] = {};
  float zs[M] = {};
  float rows = 0.f;
  MomentAcc<D> acc;
  acc.zero();
  const float* base = z + (int64_t)t * set_stride;
  const bool vec4 = (M % 4 == 0) && (ld % 4 == 0) && (set_stride % 4 == 0) && (((uintptr_t)z & 15) == 0);
  // Packed rows (ld == 2d): the wave's 64 rows are one contiguous 256·M-byte block, loaded with M/4
  // fully coalesced 1 KiB dwordx4 instructions and transposed into the row stage through LDS (a
  // lane-private row load spans 64 rows per instruction and touches every line M/4 times).
  // PACKED (host-checked: 16-byte aligned, ld == 2d; any n_rows — the buffer descriptor is rebased per row block)
  constexpr int NQ = M % 4 == 0 ? M / 4 : 1;
  auto stage_packed = [&](const f32x4* q, float* v) {
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int p = k * 256 + lane * 4;
      *reinterpret_cast<f32x4*>(&stage[wave][(p / M) * kMwStride + p % M]) = q[k];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < M; k += 4) {
      const f32x4 t4 = *reinterpret_cast<const f32x4*>(srow + k);
      v[k] = t4[0]; v[k + 1] = t4[1]; v[k + 2] = t4[2]; v[k + 3] = t4[3];
    }
  };
  auto load = [&](int64_t r, float* v) {
    if (r < n_rows) {
      const float* row = base + r * ld;
      if (vec4) {
#pragma unroll
        for (int k = 0; k < M; k += 4) {
          const f32x4 q = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + k));
          v[k] = q[0]; v[k + 1] = q[1]; v[k + 2] = q[2]; v[k + 3] = q[3];
        }
      } else {
#pragma unroll
        for (int k = 0; k < M; ++k) v[k] = row[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < M; ++k) v[k] = 0.f;
    }
  };
  // wave-uniform trip count: every lane joins every MFMA (rows past the end are zeros, weight 0)
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t r0 = (int64_t)blockIdx.x * kBlock + wave * kWave;
  // one row block of the wave: its rows are in stage[wave], v = this lane's row
  auto consume = [&](const float* v, int64_t r0) {
    const bool active = r0 + lane < n_rows;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float a = stage[wave][(4 * j + lane / 16) * kMwStride + (lane & 15)];
      g4 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, g4, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    rows += active ? 1.f : 0.f;
#pragma unroll
    for (int k = 0; k < M; ++k) zs[k] += v[k];
    // (ds log rho, ds2 log rho) = (a1, a2) + (b1, b2) . r + r^T (G1, G2) r, r = m1 - x
    float rr[D];
#pragma unroll
    for (int k = 0; k < D; ++k) rr[k] = m1[k] - v[k];
    f32x2 q = a12;
    int o = 0;
#pragma unroll
    for (int i = 0; i < D; ++i) {  // q += r_i (b_i + sum_{j >= i} Gsym_ij r_j)
      f32x2 g = cpair[NT + i];
#pragma unroll
      for (int j = i; j < D; ++j, ++o) g = cpair[o] * f32x2{rr[j], rr[j]} + g;
      q = g * f32x2{rr[i], rr[i]} + q;
    }
    const float w = active ? q[1] + q[0] * q[0] + gamma * q[0] : 0.f;  // kinetic_mckean_vlasov.py:243-248
    acc.add(v, w);
    if constexpr (MF) {  // the next simulate's update-t normals of this lane's particle
      if (active) {
        const uint64_t gid = (uint64_t)(mf.poff + r0 + lane);
        float xi[D];
        stream_normals<D>(mf.k0, mf.k1, mf.ctr_off + (uint32_t)t, (uint32_t)gid, (uint32_t)(gid >> 32), xi);
#pragma unroll
        for (int k = 0; k < D; ++k) xis[k] += xi[k];
      }
    }
  };
  if constexpr (PACKED) {
    // The set's rows through a buffer descriptor: rows at or past n_rows read as zero (the hardware range
    // check), so the prefetch loads are unconditional — no per-load compare, zero fill and exec-masked branch
    // (2.74 -> 2.54 ms at C4, tools/kmv_time.py, profiles/r04_kmv_buffer_ab.txt; prefetching two blocks ahead
    // instead cost the third wave per SIMD and measured no faster). The descriptor is rebased on every row block
    // (64-bit base = the block's first row, records = the block's bytes that exist), so the 32-bit offsets stay
    // below 64 * 2d * 4 bytes for a set of any size; r0w is wave-uniform (scalar descriptor, no waterfall).
    auto load_buf = [&](int64_t r0w, f32x4* q) {
      const int64_t left = n_rows - r0w;
      const int nrec = left <= 0 ? 0 : (int)((left < kWave ? left : (int64_t)kWave) * M * 4);
      const float* bp = base + (left > 0 ? r0w * M : 0);
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bp), 0, nrec, 0x00020000);
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const uint32_t off = (uint32_t)((k * 256 + lane * 4) * 4);
        q[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 2));  // nt
      }
    };
    f32x4 qa[NQ];
    load_buf(r0, qa);
    for (; r0 < n_rows; r0 += stride) {
      asm volatile("" ::: "memory");  // keep the coefficient pairs in LDS (hoisted: 2 d^2 + 2 d VGPRs)
      float v[M];
      __builtin_amdgcn_wave_barrier();  // the previous block's stage reads are done
      stage_packed(qa, v);
      load_buf(r0 + stride, qa);  // software prefetch of the wave's next row block
      consume(v, r0);
    }
  } else {
    float vn[M];
    load(r0 + lane, vn);
    for (; r0 < n_rows; r0 += stride) {
      asm volatile("" ::: "memory");
      float v[M];
#pragma unroll
      for (int k = 0; k < M; ++k) v[k] = vn[k];
      load(r0 + stride + lane, vn);  // software prefetch of the next row
#pragma unroll
      for (int k = 0; k < M; k += 2) *reinterpret_cast<f32x2*>(srow + k) = f32x2{v[k], v[k + 1]};
      consume(v, r0);
    }
  }
  // the wave's 16 x 16 Gram: lane holds rows 4 (lane / 16) + i, column lane % 16 (symmetric, so the
  // row / column convention of the accumulator layout does not matter)
#pragma unroll
  for (int i = 0; i < 4; ++i) gram[wave][(4 * (lane / 16) + i) * 16 + (lane & 15)] = g4[i];
  float* slab = partials + (int64_t)t * (LZ + LW) * gridDim.x;
  float cs[1 + M];
  cs[0] = rows;
#pragma unroll
  for (int k = 0; k < M; ++k) cs[1 + k] = zs[k];
  __shared__ float lds[kWavesPerBlock * LW];
  block_reduce_to_slab(cs, 1 + M, lds, slab, blockIdx.x, gridDim.x);  // syncs: gram[] is complete
  for (int o = threadIdx.x; o < M * (M + 1) / 2; o += kBlock) {
    int i = 0, rem = o;
    while (rem >= M - i) { rem -= M - i; ++i; }
    const int j = i + rem;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) s += gram[w][i * 16 + j];
    slab[(int64_t)(1 + M + o) * gridDim.x + blockIdx.x] = s;
  }
  block_reduce_to_slab(acc.v, LW, lds, slab + (int64_t)LZ * gridDim.x, blockIdx.x, gridDim.x);
  if constexpr (MF) {
    __shared__ float lds2[kWavesPerBlock * D];
    block_reduce_to_slab(xis, D, lds2, mf_partials + (int64_t)t * D * gridDim.x, blockIdx.x, gridDim.x);
  }
}

// slab [n_sets][LZ + LW] (fp64, after slab_reduce) -> mom [n_sets][LZ], wst [n_sets][LW]
__global__ void kmv_split_kernel(const double* __restrict__ both, int64_t n_sets, int lz, int lw,
                                 double* __restrict__ mom, double* __restrict__ wst) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n_sets * (lz + lw)) return;
  const int64_t t = e / (lz + lw);
  const int c = (int)(e % (lz + lw));
  if (c < lz) mom[t * lz + c] = both[e];
  else wst[t * lw + (c - lz)] = both[e];
}

struct KmvArgs {
  int d, n_sets;
  float gamma;
  float F[PDEINV_MAX_DIM * PDEINV_MAX_DIM];
};

// Per time stamp t: n_t, xbar_t, M_t = E_t[x x^T], C_t = M_t - xbar xbar^T from mom (z moments);
// W_t, Wx_t, Wxx_t (sums) from wst. N = sum_t n_t.
//   nabla = (1/N) sum_t n_t tr(S C_t S) + b.b        hess = tr(S Mvv)
//   value = (1/N) sum_t [ 1/2 tr(S Wxx_t) - xbar_t^T S Wx_t + 1/2 W_t tr(S M_t) + b.(Wx_t - W_t xbar_t) ]
//   true  = (1/N) sum_t n_t tr(F C_t F)              gt = (1/N) sum_t n_t tr(D C_t D^T) + b.b, D = F - S
//   loss  = nabla - 2 hess + 2 value + true
// Two launches: one block per time stamp (C_t, S, F staged in LDS, thread per (i, j)) writes the
// per-t terms to a slab; one block sums the slab in a fixed order and assembles loss and grad.
constexpr int kKmvScalars = 4;  // nabla, value, true, gt (per-t contributions)

__host__ __device__ inline int kmv_slots(int d) { return d * d + d + kKmvScalars; }

__device__ __forceinline__ int tri_idx(int i, int j, int mm) {
  if (i > j) { const int t = i; i = j; j = t; }
  return i * mm - i * (i - 1) / 2 + (j - i);
}

__global__ __launch_bounds__(kBlock) void kmv_terms_kernel(KmvArgs a, const double* __restrict__ mom,
                                                           const double* __restrict__ wst,
                                                           const float* __restrict__ theta,
                                                           double* __restrict__ slab) {
  const int d = a.d, m = 2 * d, Lz = moment_len(m), Lw = moment_len(d), t = blockIdx.x, tid = threadIdx.x;
  __shared__ double sS[PDEINV_MAX_DIM * PDEINV_MAX_DIM], sF[PDEINV_MAX_DIM * PDEINV_MAX_DIM];
  __shared__ double sM[PDEINV_MAX_DIM * PDEINV_MAX_DIM], sC[PDEINV_MAX_DIM * PDEINV_MAX_DIM];
  __shared__ double sxb[PDEINV_MAX_DIM], sWx[PDEINV_MAX_DIM];
  __shared__ double red[kWavesPerBlock][kKmvScalars];
  const double* v = mom + (int64_t)t * Lz;
  const double* w = wst + (int64_t)t * Lw;
  double Ntot = 0;
  for (int u = 0; u < a.n_sets; ++u) Ntot += mom[(int64_t)u * Lz];
  const double invN = Ntot > 0 ? 1.0 / Ntot : 0.0;
  const double cnt = v[0], inv_c = cnt > 0 ? 1.0 / cnt : 0.0;
  if (tid < d) {
    sxb[tid] = v[1 + tid] * inv_c;
    sWx[tid] = w[1 + tid];
  }
  if (tid < d * d) {
    const int i = tid / d, j = tid % d;
    sS[tid] = (double)theta[i * d + j] + (double)theta[j * d + i];
    sF[tid] = (double)a.F[tid];
    sM[tid] = v[1 + m + tri_idx(i, j, m)] * inv_c;
  }
  __syncthreads();
  if (tid < d * d) sC[tid] = sM[tid] - sxb[tid / d] * sxb[tid % d];
  __syncthreads();
  double c[kKmvScalars] = {0, 0, 0, 0};
  double* out = slab + (int64_t)t * kmv_slots(d);
  if (tid < d * d) {
    const int i = tid / d, j = tid % d;
    const double nt = cnt * invN;
    double SC_ij = 0, CS_ij = 0, FC = 0, DC = 0;
    for (int k = 0; k < d; ++k) {
      const double ckj = sC[k * d + j];
      SC_ij += sS[i * d + k] * ckj;
      CS_ij += sC[i * d + k] * sS[k * d + j];
      FC += sF[i * d + k] * ckj;
      DC += (sF[i * d + k] - sS[i * d + k]) * ckj;
    }
    const double Wt = w[0], Wxx_ji = w[1 + d + tri_idx(j, i, d)];
    c[0] = nt * SC_ij * sS[j * d + i];                                    // tr(S C S)
    c[2] = nt * FC * sF[i * d + j];                                       // tr(F C F^T)
    c[3] = nt * DC * (sF[i * d + j] - sS[i * d + j]);                     // tr(D C D^T)
    c[1] = invN * (0.5 * sS[i * d + j] * Wxx_ji - sxb[i] * sS[i * d + j] * sWx[j] +
                   0.5 * Wt * sS[i * d + j] * sM[j * d + i]);              // value
    // d/dK_ij of the t terms (the (j, i) transpose is added in the combine)
    out[tid] = nt * (SC_ij + CS_ij) +
               2 * invN * (0.5 * Wxx_ji - sxb[i] * sWx[j] + 0.5 * Wt * sM[i * d + j]);
  }
  if (tid < d) out[d * d + tid] = sWx[tid] - w[0] * sxb[tid];  // bias weights (Wx_t - W_t xbar_t)
#pragma unroll
  for (int q = 0; q < kKmvScalars; ++q) {
    double x = c[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if ((tid & 63) == 0) red[tid >> 6][q] = x;
  }
  __syncthreads();
  if (tid < kKmvScalars) out[d * d + d + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
}

__global__ __launch_bounds__(kBlock) void kmv_combine_kernel(KmvArgs a, const double* __restrict__ mom,
                                                             const double* __restrict__ slab,
                                                             const float* __restrict__ theta,
                                                             float* __restrict__ out, float* __restrict__ grad) {
  const int d = a.d, m = 2 * d, Lz = moment_len(m), ns = kmv_slots(d), tid = threadIdx.x;
  __shared__ double tot[PDEINV_MAX_DIM * PDEINV_MAX_DIM + PDEINV_MAX_DIM + kKmvScalars];
  double Ntot = 0;
  for (int u = 0; u < a.n_sets; ++u) Ntot += mom[(int64_t)u * Lz];
  const double invN = Ntot > 0 ? 1.0 / Ntot : 0.0;
  for (int q = tid; q < ns; q += kBlock) {
    double s = 0;
    for (int t = 0; t < a.n_sets; ++t) s += slab[(int64_t)t * ns + q];  // fixed order
    tot[q] = s;
  }
  __syncthreads();
  auto S = [&](int i, int j) { return (double)theta[i * d + j] + (double)theta[j * d + i]; };
  double acc[7] = {0, 0, 0, 0, 0, 0, 0};  // nabla, hess, value, true, gt, |grad|^2
  if (tid < d * d) {
    const int i = tid / d, j = tid % d;
    double mvv = 0;
    for (int t = 0; t < a.n_sets; ++t) mvv += mom[(int64_t)t * Lz + 1 + m + tri_idx(d + i, d + j, m)];
    mvv *= invN;
    acc[1] = S(i, j) * mvv;
    const double gk = tot[i * d + j] + tot[j * d + i] - 4 * mvv;
    grad[i * d + j] = (float)gk;
    acc[5] = gk * gk;
  }
  if (tid < d) {
    const double b = (double)theta[d * d + tid], wsum = tot[d * d + tid];
    acc[0] += b * b;
    acc[4] += b * b;
    acc[2] += invN * b * wsum;
    const double gb = 2 * b + 2 * invN * wsum;
    grad[d * d + tid] = (float)gb;
    acc[5] += gb * gb;
  }
  if (tid == 0) {
    const double* sc = tot + d * d + d;
    acc[0] += sc[0];
    acc[2] += sc[1];
    acc[3] += sc[2];
    acc[4] += sc[3];
  }
  __shared__ double red[kWavesPerBlock][7];
#pragma unroll
  for (int c = 0; c < 7; ++c) {
    double v = acc[c];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((tid & 63) == 0) red[tid >> 6][c] = v;
  }
  __syncthreads();
  if (tid == 0) {
    double r[7];
#pragma unroll
    for (int c = 0; c < 7; ++c) r[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    out[PDEINV_KFP_LOSS] = (float)(r[0] - 2 * r[1] + 2 * r[2] + r[3]);
    out[PDEINV_KFP_LOSS_GT] = (float)r[4];
    out[PDEINV_KFP_GRAD_NORM] = (float)sqrt(r[5]);
    out[PDEINV_KFP_NABLA] = (float)r[0];
    out[PDEINV_KFP_HESSIAN] = (float)r[1];
    out[PDEINV_KFP_FRICTION] = (float)r[2];
    out[PDEINV_KFP_NABLA_TRUE] = (float)r[3];
    out[PDEINV_KFP_INITIAL] = 0.f;
    out[PDEINV_KFP_TERMINAL] = 0.f;
  }
}

}  // namespace pdeinv

using namespace pdeinv;

extern "C" size_t pdeinv_moments_batched_workspace_bytes(int64_t n_sets, int64_t n_rows, int32_t m) {
  if (m < 1 || m > 16 || n_sets < 1 || n_rows < 0) return 0;
  return (size_t)n_sets * moment_len(m) * batched_bx(n_sets, n_rows) * sizeof(float);
}

extern "C" int pdeinv_moments_batched(const float* z, int64_t n_sets, int64_t n_rows, int32_t m,
                                      int64_t set_stride, int64_t ld, void* ws, double* out, void* stream) {
  PDEINV_REQUIRE(m >= 1 && m <= 16, PDEINV_ERR_UNSUPPORTED, "moments_batched: m must be in [1, 16]");
  PDEINV_REQUIRE(n_sets >= 1 && n_sets <= 65535 && n_rows >= 0, PDEINV_ERR_INVALID,
                 "moments_batched: need 1 <= n_sets <= 65535, n_rows >= 0");
  if (ld == 0) ld = m;
  PDEINV_REQUIRE(ld >= m && set_stride >= 0, PDEINV_ERR_INVALID, "moments_batched: bad strides");
  PDEINV_REQUIRE(out && ws && (n_rows == 0 || z), PDEINV_ERR_INVALID, "moments_batched: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int bx = batched_bx(n_sets, n_rows);
  const dim3 g(bx, (unsigned)n_sets);
  float* p = (float*)ws;
  switch (m) {
#define CASE(MM) case MM: hipLaunchKernelGGL(moments_batched_kernel<MM>, g, dim3(kBlock), 0, st, z, n_rows, set_stride, ld, p); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
  }
  int rc = check_launch("moments_batched_kernel");
  if (rc) return rc;
  launch_slab_reduce(p, bx, (int)(n_sets * moment_len(m)), out, st);
  return check_launch("slab_reduce_kernel");
}

extern "C" size_t pdeinv_kmv_weights_workspace_bytes(int64_t n_sets, int64_t n_rows, int32_t dim) {
  if (dim < 1 || dim > 16 || n_sets < 1 || n_rows < 0) return 0;
  return (size_t)n_sets * moment_len(dim) * batched_bx(n_sets, n_rows) * sizeof(float);
}

extern "C" int pdeinv_kmv_weights(int32_t D, float gamma, const float* coef, const float* z, int64_t n_sets,
                                  int64_t n_rows, int64_t set_stride, int64_t ld, float* ds, void* ws,
                                  double* out, void* stream) {
  PDEINV_REQUIRE(D >= 1 && D <= 16, PDEINV_ERR_UNSUPPORTED, "kmv_weights: dim must be in [1, 16]");
  PDEINV_REQUIRE(n_sets >= 1 && n_sets <= 65535 && n_rows >= 0, PDEINV_ERR_INVALID,
                 "kmv_weights: need 1 <= n_sets <= 65535");
  if (ld == 0) ld = 2 * D;
  PDEINV_REQUIRE(ld >= D && set_stride >= 0, PDEINV_ERR_INVALID, "kmv_weights: bad strides");
  PDEINV_REQUIRE(coef && out && ws && (n_rows == 0 || z), PDEINV_ERR_INVALID, "kmv_weights: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int bx = batched_bx(n_sets, n_rows);
  const dim3 g(bx, (unsigned)n_sets);
  float* p = (float*)ws;
  switch (D) {
#define CASE(DD) case DD: hipLaunchKernelGGL(kmv_weights_kernel<DD>, g, dim3(kBlock), 0, st, gamma, coef, z, n_rows, set_stride, ld, ds, p); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(10) CASE(12) CASE(16)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "kmv_weights: dim must be one of 1-8, 10, 12, 16");
  }
  int rc = check_launch("kmv_weights_kernel");
  if (rc) return rc;
  launch_slab_reduce(p, bx, (int)(n_sets * moment_len(D)), out, st);
  return check_launch("slab_reduce_kernel");
}

extern "C" size_t pdeinv_residual_kmv_workspace_bytes(const pdeinv_kmv_desc* d) {
  if (!d || d->dim < 1 || d->dim > 8 || d->n_sets < 1) return 0;
  return (size_t)d->n_sets * kmv_slots(d->dim) * sizeof(double);
}

extern "C" int pdeinv_residual_kmv(const pdeinv_kmv_desc* d, const double* mom, const double* wst,
                                   const float* theta, void* ws, float* out, float* grad, void* stream) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "residual_kmv: null descriptor");
  PDEINV_REQUIRE(d->dim >= 1 && d->dim <= 8, PDEINV_ERR_UNSUPPORTED, "residual_kmv: dim must be in [1, 8]");
  PDEINV_REQUIRE(d->n_sets >= 1 && d->n_sets <= 65535, PDEINV_ERR_INVALID, "residual_kmv: need 1 <= n_sets <= 65535");
  PDEINV_REQUIRE(mom && wst && theta && ws && out && grad && d->tilde_F, PDEINV_ERR_INVALID,
                 "residual_kmv: null pointer");
  KmvArgs a{};
  a.d = d->dim;
  a.n_sets = d->n_sets;
  a.gamma = d->gamma;
  for (int k = 0; k < d->dim * d->dim; ++k) a.F[k] = d->tilde_F[k];
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(kmv_terms_kernel, dim3((unsigned)d->n_sets), dim3(kBlock), 0, st, a, mom, wst, theta,
                     (double*)ws);
  int rc = check_launch("kmv_terms_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(kmv_combine_kernel, dim3(1), dim3(kBlock), 0, st, a, mom, (const double*)ws, theta, out, grad);
  return check_launch("kmv_combine_kernel");
}

// fp32 partial slab, rounded up to 256 B so that the fp64 column sums behind it are aligned
static size_t kmv_mw_slab_bytes(int64_t cols, int bx) { return ((size_t)cols * bx * sizeof(float) + 255) & ~(size_t)255; }

static int kmv_mw_launch(int32_t D, float gamma, const float* coef, const float* z, int64_t n_sets, int64_t n_rows,
                         int64_t set_stride, int64_t ld, void* ws, double* mom, double* wst, hipStream_t st,
                         const MfNoise* mf, float* mf_partials) {
  const int bx = batched_bx(n_sets, n_rows);
  const int lz = moment_len(2 * D), lw = moment_len(D);
  const int64_t cols = n_sets * (lz + lw);
  float* p = (float*)ws;
  double* both = (double*)((char*)ws + kmv_mw_slab_bytes(cols, bx));
  const dim3 g(bx, (unsigned)n_sets);
  // packed rows (ld == 2d, 16-byte aligned, even d): the coalesced block-load variant
  const bool packed = (2 * D) % 4 == 0 && ld == 2 * D && set_stride % 4 == 0 && ((uintptr_t)z & 15) == 0;
  const MfNoise m = mf ? *mf : MfNoise{};
  switch (D) {
#define CASE(DD)                                                                                              \
  case DD:                                                                                                    \
    if (mf && packed)                                                                                         \
      hipLaunchKernelGGL((kmv_moments_weights_kernel<DD, (2 * DD) % 4 == 0, true>), g, dim3(kBlock), 0, st,    \
                         gamma, coef, z, n_rows, set_stride, ld, p, m, mf_partials);                          \
    else if (mf)                                                                                              \
      hipLaunchKernelGGL((kmv_moments_weights_kernel<DD, false, true>), g, dim3(kBlock), 0, st, gamma, coef, z, \
                         n_rows, set_stride, ld, p, m, mf_partials);                                          \
    else if (packed)                                                                                          \
      hipLaunchKernelGGL((kmv_moments_weights_kernel<DD, (2 * DD) % 4 == 0>), g, dim3(kBlock), 0, st, gamma, coef, \
                         z, n_rows, set_stride, ld, p, MfNoise{}, nullptr);                                   \
    else                                                                                                      \
      hipLaunchKernelGGL((kmv_moments_weights_kernel<DD, false>), g, dim3(kBlock), 0, st, gamma, coef, z, n_rows, \
                         set_stride, ld, p, MfNoise{}, nullptr);                                              \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
  }
  int rc = check_launch("kmv_moments_weights_kernel");
  if (rc) return rc;
  launch_slab_reduce(p, bx, (int)cols, both, st);
  rc = check_launch("slab_reduce_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(kmv_split_kernel, dim3(grid_for(cols)), dim3(kBlock), 0, st, both, n_sets, lz, lw, mom, wst);
  return check_launch("kmv_split_kernel");
}

extern "C" size_t pdeinv_kmv_moments_weights_workspace_bytes(int64_t n_sets, int64_t n_rows, int32_t dim) {
  if (dim < 1 || dim > 8 || n_sets < 1 || n_rows < 0) return 0;
  const int64_t cols = n_sets * (moment_len(2 * dim) + moment_len(dim));
  return kmv_mw_slab_bytes(cols, batched_bx(n_sets, n_rows)) + (size_t)cols * sizeof(double);
}

extern "C" int pdeinv_kmv_moments_weights(int32_t D, float gamma, const float* coef, const float* z, int64_t n_sets,
                                          int64_t n_rows, int64_t set_stride, int64_t ld, void* ws, double* mom,
                                          double* wst, void* stream) {
  PDEINV_REQUIRE(D >= 1 && D <= 8, PDEINV_ERR_UNSUPPORTED, "kmv_moments_weights: dim must be in [1, 8]");
  PDEINV_REQUIRE(n_sets >= 1 && n_sets <= 65535 && n_rows >= 0, PDEINV_ERR_INVALID,
                 "kmv_moments_weights: need 1 <= n_sets <= 65535, n_rows >= 0");
  if (ld == 0) ld = 2 * D;
  PDEINV_REQUIRE(ld >= 2 * D && set_stride >= 0, PDEINV_ERR_INVALID, "kmv_moments_weights: bad strides");
  PDEINV_REQUIRE(coef && mom && wst && ws && (n_rows == 0 || z), PDEINV_ERR_INVALID,
                 "kmv_moments_weights: null pointer");
  return kmv_mw_launch(D, gamma, coef, z, n_sets, n_rows, set_stride, ld, ws, mom, wst, (hipStream_t)stream,
                       nullptr, nullptr);
}

extern "C" size_t pdeinv_kmv_moments_weights_mf_sums_workspace_bytes(int64_t n_sets, int64_t n_rows, int32_t dim,
                                                                     const pdeinv_sde_desc* next) {
  const size_t a = pdeinv_kmv_moments_weights_workspace_bytes(n_sets, n_rows, dim);
  if (a == 0 || !next) return 0;
  const size_t b = (size_t)n_sets * dim * batched_bx(n_sets, n_rows) * sizeof(float);
  return ((a + 255) & ~(size_t)255) + ((b + 255) & ~(size_t)255) + pdeinv_mf_sums_workspace_bytes(next);
}

extern "C" int pdeinv_kmv_moments_weights_mf_sums(int32_t D, float gamma, const float* coef, const float* z,
                                                  int64_t n_sets, int64_t n_rows, int64_t set_stride, int64_t ld,
                                                  void* ws, double* mom, double* wst, const pdeinv_sde_desc* next,
                                                  const float* z0_next, double* sums_next, void* stream) {
  PDEINV_REQUIRE(D >= 1 && D <= 8, PDEINV_ERR_UNSUPPORTED, "kmv_moments_weights_mf_sums: dim must be in [1, 8]");
  PDEINV_REQUIRE(n_sets >= 1 && n_sets <= 65535 && n_rows >= 1, PDEINV_ERR_INVALID,
                 "kmv_moments_weights_mf_sums: need 1 <= n_sets <= 65535, n_rows >= 1");
  if (ld == 0) ld = 2 * D;
  PDEINV_REQUIRE(ld >= 2 * D && set_stride >= 0, PDEINV_ERR_INVALID, "kmv_moments_weights_mf_sums: bad strides");
  PDEINV_REQUIRE(coef && mom && wst && ws && z && next && z0_next && sums_next, PDEINV_ERR_INVALID,
                 "kmv_moments_weights_mf_sums: null pointer");
  MfNoise mf;
  int rc = mf_noise_of(next, D, n_rows, mf);
  if (rc) return rc;
  PDEINV_REQUIRE(n_sets <= (int64_t)next->n_steps + 1, PDEINV_ERR_INVALID,
                 "kmv_moments_weights_mf_sums: more stamps than updates of the next simulate");
  hipStream_t st = (hipStream_t)stream;
  const size_t a = (pdeinv_kmv_moments_weights_workspace_bytes(n_sets, n_rows, D) + 255) & ~(size_t)255;
  const int bx = batched_bx(n_sets, n_rows);
  const size_t b = ((size_t)n_sets * D * bx * sizeof(float) + 255) & ~(size_t)255;
  float* mfp = (float*)((char*)ws + a);
  rc = kmv_mw_launch(D, gamma, coef, z, n_sets, n_rows, set_stride, ld, ws, mom, wst, st, &mf, mfp);
  if (rc) return rc;
  // updates t < n_sets: the pass's slab -> sums columns 1 + 2D + t D + k
  launch_slab_reduce(mfp, bx, (int)(n_sets * D), sums_next + 1 + 2 * D, st);
  rc = check_launch("slab_reduce_kernel");
  if (rc) return rc;
  // updates n_sets .. n_steps and [count, sum x0, sum v0] of the next simulate
  return mf_sums_tail(next, z0_next, (int)n_sets, (char*)ws + a + b, sums_next, st);
}
