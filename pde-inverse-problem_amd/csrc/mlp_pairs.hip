// mlp_pairs.hip — the general-Phi KMV residual for narrow hypothesis nets, pairs generated in
// registers (gfx950).
//
// Replaces, for width <= 28 (the reference's default V_hypothesis is width 20 x 8 layers,
// configurations/neural_network/MLP.yaml:4-5), the pair-row + rocBLAS path of mlp.hip for
// methods/consistency_instances/kinetic_mckean_vlasov.py:11-120 with a non-parametric Phi_theta:
// every pair (i, j) of a time stamp's particles, y_ij = x_i - x_j (x_minus_ref, :20-23), needs
// grad Phi(y_ij), v_i^T Hess Phi(y_ij) v_i and Phi(y_ij), and the loss' parameter gradient.
//
// One lane owns one pair; a wave walks the 64-wide tiles of references j of one particle i. The
// narrow layers are per-lane VALU matvecs whose weights stream through scalar loads (wave-uniform
// addresses: no LDS copy, no VGPRs held for them). Nothing of the n^2 pair set touches HBM except
// a per-wave scratch ring of the tile's per-layer checkpoints (h, z', z'', a, zetabar: 5 W floats per
// layer per pair, written and read back coalesced, lane-fastest). Weight gradients — sums over pairs
// of outer products — run on the matrix pipe: v_mfma_f32_32x32x2_f32 with the tile's 64 pairs as the
// reduction dimension, fed through a per-wave LDS transpose (row stride 33: conflict-free 64-lane
// row writes); a constant-1 input feature carries the bias gradients through the same MFMA. Each
// wave folds its tile sums into a private global slab; a fixed-order reduction over waves gives the
// gradient (deterministic, no atomics).
//   pass 1 (kmvp_gbar_kernel)  value stream + grad_x chain -> gbar_i = mean_j grad Phi(y_ij)
//   pass 2 (kmvp_grad_kernel)  Taylor streams, grad_x chain, its forward adjoint (seed u_i = 2 s gbar_i),
//                              reverse sweep with c2 = -2 s, c0 = 2 s w_it  (the adjoint of
//                              oracle/numpy_ref.py mlp_grad_rows / kmv_mlp_grad_analytic)
// Widths / dims between the compiled ones are zero-padded on the device (exact: padded units carry
// z = 0, h = tanh 0 = 0 and zero outgoing weights).
#include <math.h>
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace pdeinv {
namespace mlpp {

constexpr int kSR = 33;   // LDS stage row stride (floats)
constexpr int kOC = 8;    // output-layer chunk
constexpr int kMaxL = 16;
constexpr int kWavesPB = 2;  // waves per block (each wave independent)

typedef float f32x16 __attribute__((ext_vector_type(16)));
// the parameters are read at wave-uniform addresses through the constant address space, so the
// compiler issues scalar (s_load) reads into SGPRs: every FMA takes its weight as an SGPR operand
typedef const __attribute__((address_space(4))) float cfloat;

struct Args {
  int L, O, Dr;                   // layers, outputs, real input dim (<= the compiled D)
  int64_t n, n_items;             // particles per stamp; items = n_sets * n
  int64_t set_stride, ld;         // rows of z: z + t*set_stride + i*ld
  const float* z;
  const float* ds;                // [n_sets, n, 2] (ds log rho, ds2 log rho)
  float gamma, s, inv_n;          // s = 1 / (n^2 n_sets)
  cfloat* prm;                    // padded flat params (device, constant address space)
  int P;                          // padded param count
  float* gbar;                    // [n_sets * n, Dr]
  float* scratch;                 // per wave: 5 * W * L * 64 floats
  float* gslab;                   // [n_waves][P]
  float* aslab;                   // [n_waves][8]
};

// kernel / bias offsets of layer l in the padded flat layout (computed, not tabled: a table indexed by
// the runtime layer would sit in SGPRs for the whole kernel)
template <int D, int W>
__device__ __forceinline__ int kofs(int l) { return l == 0 ? 0 : D * W + W + (l - 1) * (W * W + W); }
template <int D, int W>
__device__ __forceinline__ int bofs(int l, int L, int O) { return kofs<D, W>(l) + (l == 0 ? D * W : (l == L ? W * O : W * W)); }

__device__ __forceinline__ float ftanh(float z) {
  const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * z);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

typedef const __attribute__((address_space(4))) f32x2 cfloat2;

// out[n] = sum_k in[k] K[k][n] (+ b[n]) for S streams sharing the weights: K row-major [NI][NO] (NO even, 8-byte
// aligned) at a wave-uniform address. k-outer with packed pairs of outputs: one weight row (NO / 2 SGPR pairs)
// in flight at a time — the fence keeps the scheduler from hoisting every row's scalar loads (SGPR spills).
template <int NI, int NO, int S>
__device__ __forceinline__ void mv(cfloat* K, cfloat* b, const float (*in)[NI], float (*out)[NO]) {
  static_assert(NO % 2 == 0, "packed pairs");
  f32x2 acc[S][NO / 2];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int p = 0; p < NO / 2; ++p) acc[s][p] = (b && s == 0) ? f32x2{b[2 * p], b[2 * p + 1]} : f32x2{0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    __builtin_amdgcn_sched_barrier(0);
    cfloat2* row = reinterpret_cast<cfloat2*>(K + k * NO);
#pragma unroll
    for (int p = 0; p < NO / 2; ++p) {
      const f32x2 w = row[p];
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s][p] = f32x2{in[s][k], in[s][k]} * w + acc[s][p];
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int p = 0; p < NO / 2; ++p) {
      out[s][2 * p] = acc[s][p][0];
      out[s][2 * p + 1] = acc[s][p][1];
    }
}

// out[k] = sum_n in[n] K[k][n] (the transposed product), K row-major [NI][NO]: a packed dot per row
template <int NI, int NO, int S>
__device__ __forceinline__ void mvT(cfloat* K, const float (*in)[NO], float (*out)[NI]) {
  static_assert(NO % 2 == 0, "packed pairs");
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    __builtin_amdgcn_sched_barrier(0);
    cfloat2* row = reinterpret_cast<cfloat2*>(K + k * NO);
    f32x2 acc[S];
#pragma unroll
    for (int s = 0; s < S; ++s) acc[s] = f32x2{0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NO / 2; ++p) {
      const f32x2 w = row[p];
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s] = f32x2{in[s][2 * p], in[s][2 * p + 1]} * w + acc[s];
    }
#pragma unroll
    for (int s = 0; s < S; ++s) out[s][k] = acc[s][0] + acc[s][1];
  }
}

// per-wave scratch: [layer][var][feature][lane], var 0..4 = h, z', z'', a, zetabar
template <int W>
struct Ring {
  float* base;
  int lane;
  __device__ __forceinline__ float* at(int l, int var, int k) const {
    return base + ((int64_t)(l * 5 + var) * W + k) * kWave + lane;
  }
  __device__ __forceinline__ void put(int l, int var, const float* v) const {
#pragma unroll
    for (int k = 0; k < W; ++k) *at(l, var, k) = v[k];
  }
  __device__ __forceinline__ void get(int l, int var, float* v) const {
#pragma unroll
    for (int k = 0; k < W; ++k) v[k] = *at(l, var, k);
  }
};

// Outer-product accumulation C[m][n] += sum_p A_p[m] B_p[n] over the wave's 64 pairs on the matrix
// pipe. A / B rows are staged [pair][kSR] in LDS; the operand of k-step s is pair 2s + (lane >> 5),
// feature lane & 31 (v_mfma_f32_32x32x2_f32: A[m = lane & 31][k = lane >> 5], B[k][n = lane & 31]).
__device__ __forceinline__ void mfma_tile(const float* As, const float* Bs, f32x16& acc) {
  const int lane = threadIdx.x & (kWave - 1);
  const int l31 = lane & 31, hi = lane >> 5;
#pragma unroll 8
  for (int s = 0; s < kWave / 2; ++s) {
    const float av = As[(2 * s + hi) * kSR + l31];
    const float bv = Bs[(2 * s + hi) * kSR + l31];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
  }
}

// stage row of this lane: v[0..N) then (optionally) the constant feature 1 at index N, zeros to 32
template <int N>
__device__ __forceinline__ void stage_row(float* S, const float* v, bool one, bool active) {
  const int lane = threadIdx.x & (kWave - 1);
  float* r = S + lane * kSR;
#pragma unroll
  for (int k = 0; k < N; ++k) r[k] = active ? v[k] : 0.f;
#pragma unroll
  for (int k = N; k < 32; ++k) r[k] = (k == N && one && active) ? 1.f : 0.f;
}

// slab[goff + m * NO + n] += C[m][n] (m < NI), slab[bof + n] += C[NI][n]; n < nvalid of this column tile
// (C map: acc register q is row (q & 3) + 8 (q >> 2) + 4 (lane >> 5), column lane & 31)
template <int NI>
__device__ __forceinline__ void fold(float* slab, int64_t goff, int64_t bof, int NO, int n0, const f32x16& acc) {
  const int lane = threadIdx.x & (kWave - 1);
  const int n = n0 + (lane & 31);
  if (n >= NO) return;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int m = (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
    if (m < NI) slab[goff + (int64_t)m * NO + n] += acc[q];
    else if (m == NI && bof >= 0) slab[bof + n] += acc[q];
  }
}

__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_wave_barrier(); }

// -------------------------------------------------------------------------------------------------
// pass 1: gbar_i = (1/n) sum_j grad_y Phi(x_i - x_j)
// -------------------------------------------------------------------------------------------------
template <int D, int W>
__global__ __launch_bounds__(kWavesPB * kWave) void kmvp_gbar_kernel(Args a) {
  const int lane = threadIdx.x & (kWave - 1);
  // wave-uniform by construction; readfirstlane makes the compiler see it, so every per-wave base
  // (ring, slab) lives in SGPRs and each ring access is SGPR base + one lane-offset VGPR + immediate
  const int64_t wave = (int64_t)blockIdx.x * kWavesPB + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t n_waves = (int64_t)gridDim.x * kWavesPB;
  const Ring<W> ring{a.scratch + wave * (int64_t)5 * W * a.L * kWave, lane};
  cfloat* Ko = a.prm + kofs<D, W>(a.L);
  cfloat* bo = a.prm + bofs<D, W>(a.L, a.L, a.O);
  for (int64_t it = wave; it < a.n_items; it += n_waves) {
    const int64_t t = it / a.n, i = it - t * a.n;
    const float* zt = a.z + t * a.set_stride;
    float xi[D];
#pragma unroll
    for (int k = 0; k < D; ++k) xi[k] = k < a.Dr ? zt[i * a.ld + k] : 0.f;
    float gs[D] = {};
    for (int64_t j0 = 0; j0 < a.n; j0 += kWave) {
      const int64_t j = j0 + lane;
      const bool active = j < a.n;
      float y[1][D];
#pragma unroll
      for (int k = 0; k < D; ++k) y[0][k] = (active && k < a.Dr) ? xi[k] - zt[j * a.ld + k] : 0.f;
      // value stream, h_l kept in the ring
      float h[1][W];
      mv<D, W, 1>(a.prm + kofs<D, W>(0), a.prm + bofs<D, W>(0, a.L, a.O), y, h);
#pragma unroll
      for (int k = 0; k < W; ++k) h[0][k] = ftanh(h[0][k]);
      ring.put(0, 0, h[0]);
      for (int l = 1; l < a.L; ++l) {
        float zz[1][W];
        mv<W, W, 1>(a.prm + kofs<D, W>(l), a.prm + bofs<D, W>(l, a.L, a.O), h, zz);
#pragma unroll
        for (int k = 0; k < W; ++k) h[0][k] = ftanh(zz[0][k]);
        ring.put(l, 0, h[0]);
      }
      // a_L = (2 y_out) Ko^T, output chunks of kOC
      float av[1][W] = {};
      for (int o0 = 0; o0 < a.O; o0 += kOC) {
        float yo[kOC];
#pragma unroll
        for (int c = 0; c < kOC; ++c) yo[c] = bo[o0 + c];
#pragma unroll
        for (int k = 0; k < W; ++k) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int c = 0; c < kOC; ++c)
            yo[c] = fmaf(h[0][k], Ko[(int64_t)k * a.O + o0 + c], yo[c]);
        }
#pragma unroll
        for (int k = 0; k < W; ++k) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int c = 0; c < kOC; ++c)
            av[0][k] = fmaf(2.f * yo[c], Ko[(int64_t)k * a.O + o0 + c], av[0][k]);
        }
      }
      // grad_x chain: zeta = s1(z_l) a, a <- zeta K_l^T
      for (int l = a.L - 1; l >= 1; --l) {
        float hl[W];
        ring.get(l, 0, hl);
        float ze[1][W];
#pragma unroll
        for (int k = 0; k < W; ++k) ze[0][k] = (1.f - hl[k] * hl[k]) * av[0][k];
        mvT<W, W, 1>(a.prm + kofs<D, W>(l), ze, av);
      }
      float hl[W];
      ring.get(0, 0, hl);
      float ze[1][W], g[1][D];
#pragma unroll
      for (int k = 0; k < W; ++k) ze[0][k] = (1.f - hl[k] * hl[k]) * av[0][k];
      mvT<D, W, 1>(a.prm + kofs<D, W>(0), ze, g);
#pragma unroll
      for (int k = 0; k < D; ++k) gs[k] += active ? g[0][k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const float s = wave_sum(gs[k]);
      if (lane == 0 && k < a.Dr) a.gbar[it * a.Dr + k] = s * a.inv_n;
    }
  }
}

// -------------------------------------------------------------------------------------------------
// pass 2: d/dtheta of sum_ij [ u_i . grad Phi(y_ij) + c2 v_i^T Hess Phi(y_ij) v_i + c0_i Phi(y_ij) ]
// -------------------------------------------------------------------------------------------------
// Work units of pass 2: (item, block of kJB references) — finer than whole items, so the persistent
// grid's waves get equal shares (5 000 items over 2 048 waves left 2 or 3 items of 79 tiles per wave).
constexpr int kJB = 512;
constexpr int kRC = 4;  // checkpoint features loaded together in the reverse sweep

// LSLAB: the wave's weight-gradient slab lives in LDS for the whole kernel (every tile folds its 36
// outer-product tiles there with ds_* read-modify-writes) and is copied to the wave's global slab row
// once at the end; without it (nets whose padded parameter count does not fit) the folds go to the
// global slab row directly.
template <int D, int W, bool LSLAB>
__global__ __launch_bounds__(kWavesPB * kWave) void kmvp_grad_kernel(Args a) {
  static_assert(W < 32 && D < 32, "a constant-1 input feature must fit the 32-wide MFMA tile");
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // wave-uniform: SGPR bases
  const int64_t wave = (int64_t)blockIdx.x * kWavesPB + wib;
  const int64_t n_waves = (int64_t)gridDim.x * kWavesPB;
  __shared__ float stage[kWavesPB][2][kWave * kSR];
  extern __shared__ float lslab_all[];  // LSLAB: [kWavesPB][P]
  float* As = stage[wib][0];
  float* Bs = stage[wib][1];
  const Ring<W> ring{a.scratch + wave * (int64_t)5 * W * a.L * kWave, lane};
  float* gslab = a.gslab + wave * (int64_t)a.P;
  float* slab = LSLAB ? lslab_all + wib * a.P : gslab;
  if constexpr (LSLAB) {
    for (int q = lane; q < a.P; q += kWave) slab[q] = 0.f;
    wave_fence();
  }
  cfloat* Ko = a.prm + kofs<D, W>(a.L);
  cfloat* bo = a.prm + bofs<D, W>(a.L, a.L, a.O);
  const int L = a.L, O = a.O;
  const float c2 = -2.f * a.s;
  float accs[3] = {0.f, 0.f, 0.f};  // LOSS, HESSIAN, FRICTION slot partials
  const int64_t n_jb = (a.n + kJB - 1) / kJB;
  for (int64_t u = wave; u < a.n_items * n_jb; u += n_waves) {
    const int64_t it = u / n_jb, jb = u - it * n_jb;
    const int64_t t = it / a.n, i = it - t * a.n;
    const int64_t j_end = (jb + 1) * kJB < a.n ? (jb + 1) * kJB : a.n;
    const float* zt = a.z + t * a.set_stride;
    float xi[D], vi[D], u0[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      xi[k] = k < a.Dr ? zt[i * a.ld + k] : 0.f;
      vi[k] = k < a.Dr ? zt[i * a.ld + a.Dr + k] : 0.f;
      u0[k] = k < a.Dr ? 2.f * a.s * a.gbar[it * a.Dr + k] : 0.f;  // input-gradient seed u_i = 2 s gbar_i
    }
    const float dsa = a.ds[it * 2], dsb = a.ds[it * 2 + 1];
    const float c0 = 2.f * a.s * (dsb + dsa * dsa + a.gamma * dsa);  // 2 s w_it (:84-89)
    for (int64_t j0 = jb * kJB; j0 < j_end; j0 += kWave) {
      const int64_t j = j0 + lane;
      const bool active = j < j_end;
      float y[D];
#pragma unroll
      for (int k = 0; k < D; ++k) y[k] = (active && k < a.Dr) ? xi[k] - zt[j * a.ld + k] : 0.f;
      // ---- forward Taylor streams (h, h', h''), checkpoints h, z', z'' ----
      float hs[3][W];
      {
        float in[2][D], zz[2][W];
#pragma unroll
        for (int k = 0; k < D; ++k) { in[0][k] = y[k]; in[1][k] = vi[k]; }
        mv<D, W, 2>(a.prm + kofs<D, W>(0), a.prm + bofs<D, W>(0, a.L, a.O), in, zz);
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const float hn = ftanh(zz[0][k]), s1 = 1.f - hn * hn, s2 = -2.f * hn * s1;
          hs[0][k] = hn;
          hs[1][k] = s1 * zz[1][k];
          hs[2][k] = s2 * zz[1][k] * zz[1][k];
          zz[0][k] = 0.f;  // z'' of layer 1 is 0
        }
        ring.put(0, 0, hs[0]);
        ring.put(0, 1, zz[1]);
        ring.put(0, 2, zz[0]);
      }
      for (int l = 1; l < L; ++l) {
        float zz[3][W];
        mv<W, W, 3>(a.prm + kofs<D, W>(l), a.prm + bofs<D, W>(l, a.L, a.O), hs, zz);
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const float hn = ftanh(zz[0][k]), s1 = 1.f - hn * hn, s2 = -2.f * hn * s1;
          hs[0][k] = hn;
          hs[1][k] = s1 * zz[1][k];
          hs[2][k] = fmaf(s1, zz[2][k], s2 * zz[1][k] * zz[1][k]);
        }
        ring.put(l, 0, hs[0]);
        ring.put(l, 1, zz[1]);
        ring.put(l, 2, zz[2]);
      }
      // ---- output: V, V'', a_L = 2 y Ko^T ----
      float T0 = 0.f, T2 = 0.f;
      float av[1][W] = {};
      for (int o0 = 0; o0 < O; o0 += kOC) {
        float yo[3][kOC];
#pragma unroll
        for (int c = 0; c < kOC; ++c) {
          yo[0][c] = bo[o0 + c];
          yo[1][c] = yo[2][c] = 0.f;
        }
#pragma unroll
        for (int k = 0; k < W; ++k) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int c = 0; c < kOC; ++c)
            {
              const float w = Ko[(int64_t)k * O + o0 + c];
#pragma unroll
              for (int s = 0; s < 3; ++s) yo[s][c] = fmaf(hs[s][k], w, yo[s][c]);
            }
        }
#pragma unroll
        for (int c = 0; c < kOC; ++c) {
          T0 = fmaf(yo[0][c], yo[0][c], T0);
          T2 = fmaf(yo[1][c], yo[1][c], fmaf(yo[0][c], yo[2][c], T2));
        }
#pragma unroll
        for (int k = 0; k < W; ++k) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int c = 0; c < kOC; ++c)
            av[0][k] = fmaf(2.f * yo[0][c], Ko[(int64_t)k * O + o0 + c], av[0][k]);
        }
      }
      T2 *= 2.f;
      if (active) {
        accs[0] += c2 * T2 + c0 * T0;
        accs[1] += -0.5f * c2 * T2;
        accs[2] += c0 * T0;
      }
      // ---- grad_x chain (reverse): a_l, zeta = s1 a ----
      float g[1][D];
      for (int l = L - 1; l >= 0; --l) {
        ring.put(l, 3, av[0]);
        float hl[W];
        ring.get(l, 0, hl);
        float ze[1][W];
#pragma unroll
        for (int k = 0; k < W; ++k) ze[0][k] = (1.f - hl[k] * hl[k]) * av[0][k];
        if (l > 0) mvT<W, W, 1>(a.prm + kofs<D, W>(l), ze, av);
        else mvT<D, W, 1>(a.prm + kofs<D, W>(0), ze, g);
      }
      // ---- forward adjoint of the chain: abar_0 = u (c1 = 0 here), zetabar_l = abar_{l-1} K_l ----
      float ab0[D];
#pragma unroll
      for (int k = 0; k < D; ++k) ab0[k] = active ? u0[k] : 0.f;
      float abar[1][W];
      {
        float in[1][D];
#pragma unroll
        for (int k = 0; k < D; ++k) in[0][k] = ab0[k];
        float zb[1][W];
        mv<D, W, 1>(a.prm + kofs<D, W>(0), nullptr, in, zb);
        ring.put(0, 4, zb[0]);
        float hl[W];
        ring.get(0, 0, hl);
#pragma unroll
        for (int k = 0; k < W; ++k) abar[0][k] = (1.f - hl[k] * hl[k]) * zb[0][k];
      }
      for (int l = 1; l < L; ++l) {
        float zb[1][W];
        mv<W, W, 1>(a.prm + kofs<D, W>(l), nullptr, abar, zb);
        ring.put(l, 4, zb[0]);
        float hl[W];
        ring.get(l, 0, hl);
#pragma unroll
        for (int k = 0; k < W; ++k) abar[0][k] = (1.f - hl[k] * hl[k]) * zb[0][k];
      }
      // ---- output seeds, Ko / bo gradient, hb streams into layer L ----
      // ybar = 2 c2 y'' + 2 ubar + 2 c0 y,  y'bar = 4 c2 y',  y''bar = 2 c2 y,  u = 2 y (c1 = c3 = 0).
      // The four outer products (A = h_L + const 1 for bo, h'_L, h''_L, abar_L) run one type at a time,
      // compile-time unrolled (a runtime type index into register arrays would demote them to scratch);
      // the layer-L streams are re-read from the ring rather than held through the adjoint chains.
      float hb[3][W];
#pragma unroll
      for (int k = 0; k < W; ++k) hb[0][k] = hb[1][k] = hb[2][k] = 0.f;
      auto seed_type = [&](auto tyc) {
        constexpr int ty = decltype(tyc)::value;
        float st[3][W];  // the streams this type needs: h_L (0, 2, 3), h'_L (1), h''_L (0), abar_L (0, 3)
        {
          float hl[W], zd[W];
          ring.get(L - 1, 0, hl);
#pragma unroll
          for (int k = 0; k < W; ++k) st[0][k] = hl[k];
          if constexpr (ty == 1) {
            ring.get(L - 1, 1, zd);
#pragma unroll
            for (int k = 0; k < W; ++k) st[1][k] = (1.f - hl[k] * hl[k]) * zd[k];
          }
          if constexpr (ty == 0) {
            ring.get(L - 1, 1, zd);
            ring.get(L - 1, 2, st[1]);  // z''
#pragma unroll
            for (int k = 0; k < W; ++k) {
              const float s1 = 1.f - hl[k] * hl[k], s2 = -2.f * hl[k] * s1;
              st[1][k] = fmaf(s1, st[1][k], s2 * zd[k] * zd[k]);  // h''_L
            }
          }
          if constexpr (ty == 0 || ty == 3) {
            ring.get(L - 1, 4, st[2]);
#pragma unroll
            for (int k = 0; k < W; ++k) st[2][k] *= 1.f - hl[k] * hl[k];  // abar_L = s1 zetabar_L
          }
        }
        wave_fence();
        if constexpr (ty == 0) stage_row<W>(As, st[0], true, active);
        else if constexpr (ty == 1) stage_row<W>(As, st[1], false, active);
        else if constexpr (ty == 2) {
          // h''_L for the A operand
          float hl[W], zd[W], zdd[W];
          ring.get(L - 1, 0, hl);
          ring.get(L - 1, 1, zd);
          ring.get(L - 1, 2, zdd);
#pragma unroll
          for (int k = 0; k < W; ++k) {
            const float s1 = 1.f - hl[k] * hl[k], s2 = -2.f * hl[k] * s1;
            zdd[k] = fmaf(s1, zdd[k], s2 * zd[k] * zd[k]);
          }
          stage_row<W>(As, zdd, false, active);
        } else stage_row<W>(As, st[2], false, active);
        for (int n0 = 0; n0 < O; n0 += 32) {
          for (int o0 = n0; o0 < n0 + 32 && o0 < O; o0 += kOC) {
            // y (all types), y' (type 1), y'' and ubar (type 0) of this output chunk
            float y0[kOC], y1[kOC];
#pragma unroll
            for (int c = 0; c < kOC; ++c) {
              y0[c] = bo[o0 + c];
              y1[c] = 0.f;
            }
            [[maybe_unused]] float ub[kOC] = {};
#pragma unroll
            for (int k = 0; k < W; ++k) {
              __builtin_amdgcn_sched_barrier(0);
#pragma unroll
              for (int c = 0; c < kOC; ++c) {
                const float w = Ko[(int64_t)k * O + o0 + c];
                if constexpr (ty == 1) y1[c] = fmaf(st[1][k], w, y1[c]);
                else y0[c] = fmaf(st[0][k], w, y0[c]);
                if constexpr (ty == 0) {
                  y1[c] = fmaf(st[1][k], w, y1[c]);  // y''
                  ub[c] = fmaf(st[2][k], w, ub[c]);
                }
              }
            }
            float sb[kOC];
#pragma unroll
            for (int c = 0; c < kOC; ++c) {
              if constexpr (ty == 0) sb[c] = 2.f * c2 * y1[c] + 2.f * ub[c] + 2.f * c0 * y0[c];
              else if constexpr (ty == 1) sb[c] = 4.f * c2 * y1[c];
              else if constexpr (ty == 2) sb[c] = 2.f * c2 * y0[c];
              else sb[c] = 2.f * y0[c];
              if (!active) sb[c] = 0.f;
              Bs[lane * kSR + (o0 - n0) + c] = sb[c];
            }
            if constexpr (ty < 3) {
#pragma unroll
              for (int k = 0; k < W; ++k) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int c = 0; c < kOC; ++c) hb[ty][k] = fmaf(sb[c], Ko[(int64_t)k * O + o0 + c], hb[ty][k]);
              }
            }
          }
          for (int c = O - n0; c < 32; ++c) Bs[lane * kSR + c] = 0.f;  // columns past O in this tile
          wave_fence();
          f32x16 acc = {};
          mfma_tile(As, Bs, acc);
          fold<W>(slab, kofs<D, W>(L), ty == 0 ? bofs<D, W>(L, a.L, a.O) : -1, O, n0, acc);
          wave_fence();
        }
      };
      seed_type(std::integral_constant<int, 0>{});
      seed_type(std::integral_constant<int, 1>{});
      seed_type(std::integral_constant<int, 2>{});
      seed_type(std::integral_constant<int, 3>{});
      // ---- reverse sweep over the hidden layers (z-bars computed in place of the h-bars) ----
      for (int l = L - 1; l >= 0; --l) {
        float ze[W];
        // the layer's five checkpoint rows in chunks of kRC features: 5 kRC loads in flight per wait
        // (one wait per feature left every load's HBM latency exposed at one wave per SIMD)
        static_assert(W % kRC == 0, "ring chunk");
#pragma unroll
        for (int k0 = 0; k0 < W; k0 += kRC) {
          __builtin_amdgcn_sched_barrier(0);
          float hn[kRC], zd[kRC], zdd[kRC], al[kRC], zbar[kRC];
#pragma unroll
          for (int c = 0; c < kRC; ++c) {
            hn[c] = *ring.at(l, 0, k0 + c);
            zd[c] = *ring.at(l, 1, k0 + c);
            zdd[c] = *ring.at(l, 2, k0 + c);
            al[c] = *ring.at(l, 3, k0 + c);
            zbar[c] = *ring.at(l, 4, k0 + c);
          }
#pragma unroll
          for (int c = 0; c < kRC; ++c) {
            const int k = k0 + c;
            const float s1 = 1.f - hn[c] * hn[c], s2 = -2.f * hn[c] * s1, s3 = -2.f * s1 * s1 - 2.f * hn[c] * s2;
            const float b0 = hb[0][k], b1 = hb[1][k], b2 = hb[2][k];
            hb[0][k] = s1 * b0 + s2 * zd[c] * b1 + fmaf(s2, zdd[c], s3 * zd[c] * zd[c]) * b2 + s2 * al[c] * zbar[c];
            hb[1][k] = s1 * b1 + 2.f * s2 * zd[c] * b2;
            hb[2][k] = s1 * b2;
            ze[k] = s1 * al[c];
          }
        }
        // gK_l += [h, h', h'', abar]_{l-1}^T [zb, z'b, z''b, zeta]_l ; gb_l += zb (const-1 feature)
        auto outer = [&](auto tyc) {
          constexpr int ty = decltype(tyc)::value;
          wave_fence();
          if (l == 0) {
            float pv[D];
#pragma unroll
            for (int k = 0; k < D; ++k) pv[k] = ty == 0 ? y[k] : (ty == 1 ? vi[k] : (ty == 2 ? 0.f : ab0[k]));
            stage_row<D>(As, pv, ty == 0, active);
          } else {
            float pv[W];
#pragma unroll
            for (int k = 0; k < W; ++k) {
              const float hp = *ring.at(l - 1, 0, k), s1 = 1.f - hp * hp;
              if constexpr (ty == 0) pv[k] = hp;
              else if constexpr (ty == 1) pv[k] = s1 * *ring.at(l - 1, 1, k);
              else if constexpr (ty == 2) {
                const float zd = *ring.at(l - 1, 1, k);
                pv[k] = fmaf(s1, *ring.at(l - 1, 2, k), -2.f * hp * s1 * zd * zd);
              } else pv[k] = s1 * *ring.at(l - 1, 4, k);
            }
            stage_row<W>(As, pv, ty == 0, active);
          }
          if constexpr (ty < 3) stage_row<W>(Bs, hb[ty], false, active);
          else stage_row<W>(Bs, ze, false, active);
          wave_fence();
          f32x16 acc = {};
          mfma_tile(As, Bs, acc);
          if (l == 0) fold<D>(slab, kofs<D, W>(0), ty == 0 ? bofs<D, W>(0, a.L, a.O) : -1, W, 0, acc);
          else fold<W>(slab, kofs<D, W>(l), ty == 0 ? bofs<D, W>(l, a.L, a.O) : -1, W, 0, acc);
          wave_fence();
        };
        outer(std::integral_constant<int, 0>{});
        outer(std::integral_constant<int, 1>{});
        outer(std::integral_constant<int, 2>{});
        outer(std::integral_constant<int, 3>{});
        if (l > 0) {
          float nb[3][W];
          mvT<W, W, 3>(a.prm + kofs<D, W>(l), hb, nb);
#pragma unroll
          for (int k = 0; k < W; ++k) {
            hb[0][k] = nb[0][k];
            hb[1][k] = nb[1][k];
            hb[2][k] = nb[2][k];
          }
        }
      }
    }
  }
  if constexpr (LSLAB) {
    wave_fence();
    for (int q = lane; q < a.P; q += kWave) gslab[q] = slab[q];
  }
  float* as = a.aslab + wave * 8;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float v = wave_sum(accs[q]);
    if (lane == 0) as[q] = v;
  }
}

__global__ void kmvp_pad_kernel(MlpPadMap pm, const float* __restrict__ src, int64_t P, float* __restrict__ dst) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P) return;
  const int64_t r = pm.real_of(q);
  dst[q] = r >= 0 ? src[r] : 0.f;
}

// grad[real(q)] += sum_w slab[w][q] in a fixed order (fp64); acc slots likewise
__global__ void kmvp_reduce_kernel(MlpPadMap pm, const float* __restrict__ gslab, int64_t n_waves, int64_t P,
                                   const float* __restrict__ aslab, float* __restrict__ grad,
                                   double* __restrict__ acc) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < P) {
    const int64_t r = pm.real_of(q);
    if (r >= 0) {
      double s = 0.0;
      for (int64_t w = 0; w < n_waves; ++w) s += (double)gslab[w * P + q];
      grad[r] += (float)s;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 3) {
    double s = 0.0;
    for (int64_t w = 0; w < n_waves; ++w) s += (double)aslab[w * 8 + threadIdx.x];
    const int slot = threadIdx.x == 0 ? PDEINV_GMM_ACC_LOSS
                                      : (threadIdx.x == 1 ? PDEINV_GMM_ACC_HESSIAN : PDEINV_GMM_ACC_FRICTION);
    acc[slot] += s;
  }
}

}  // namespace mlpp

// ---- host driver ------------------------------------------------------------------------------
namespace {
constexpr int kPairWaves = 2048;  // persistent grid: 2 waves per SIMD of 256 CUs

int pair_waves() {
  static const int w = [] {
    const char* e = ab_env("PDEINV_PAIR_WAVES");  // A/B experiments (tools)
    const int v = e ? atoi(e) : kPairWaves;
    return v >= 2 ? v & ~1 : kPairWaves;
  }();
  return w;
}

int pad_dim(int d) { return d <= 2 ? 2 : (d <= 4 ? 4 : 8); }
int pad_width(int w) { return w <= 8 ? 8 : (w <= 16 ? 16 : (w <= 20 ? 20 : (w <= 24 ? 24 : 28))); }

struct PairPlan {
  MlpPadMap pm;
  int DP, WP;
  int64_t P, n_waves, items;
  size_t off_prm, off_gbar, off_scratch, off_gslab, off_aslab, total;  // bytes
};

PairPlan pair_plan(const pdeinv_kmv_mlp_desc* d) {
  PairPlan p{};
  p.DP = pad_dim(d->dim);
  p.WP = pad_width(d->width);
  const int L = d->n_layers;
  p.pm.L = L;
  int64_t ro = 0, po = 0;
  for (int l = 0; l <= L; ++l) {
    p.pm.din[l] = l == 0 ? d->dim : d->width;
    p.pm.dout[l] = l == L ? d->out_features : d->width;
    p.pm.pin[l] = l == 0 ? p.DP : p.WP;
    p.pm.pout[l] = l == L ? (d->out_features + mlpp::kOC - 1) / mlpp::kOC * mlpp::kOC : p.WP;
    p.pm.roff[l] = ro;
    p.pm.poff[l] = po;
    ro += (int64_t)p.pm.din[l] * p.pm.dout[l] + p.pm.dout[l];
    po += (int64_t)p.pm.pin[l] * p.pm.pout[l] + p.pm.pout[l];
  }
  p.P = po;
  p.items = (int64_t)d->n_sets * d->n_rows;
  p.n_waves = p.items < pair_waves() ? ((p.items + 1) / 2) * 2 : pair_waves();
  size_t o = 0;
  auto take = [&](size_t bytes) { const size_t at = o; o += (bytes + 255) & ~(size_t)255; return at; };
  p.off_prm = take(sizeof(float) * p.P);
  p.off_gbar = take(sizeof(float) * p.items * p.DP);
  p.off_scratch = take(sizeof(float) * (size_t)p.n_waves * 5 * p.WP * L * kWave);
  p.off_gslab = take(sizeof(float) * (size_t)p.n_waves * p.P);
  p.off_aslab = take(sizeof(float) * (size_t)p.n_waves * 8);
  p.total = o;
  return p;
}

constexpr size_t kLdsSlabMax = 64 * 1024;  // per block (the stage arrays take another 33 KB)

template <int D, int W>
void launch_pairs(const mlpp::Args& a, int64_t n_waves, hipStream_t st, bool pass2) {
  const dim3 g((unsigned)(n_waves / mlpp::kWavesPB)), b(mlpp::kWavesPB * kWave);
  const size_t lds = sizeof(float) * (size_t)mlpp::kWavesPB * a.P;
  if (pass2 && lds <= kLdsSlabMax) {
    static const bool attr = hipFuncSetAttribute((const void*)mlpp::kmvp_grad_kernel<D, W, true>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)kLdsSlabMax) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL((mlpp::kmvp_grad_kernel<D, W, true>), g, b, lds, st, a);
  }
  else if (pass2) hipLaunchKernelGGL((mlpp::kmvp_grad_kernel<D, W, false>), g, b, 0, st, a);
  else hipLaunchKernelGGL((mlpp::kmvp_gbar_kernel<D, W>), g, b, 0, st, a);
}

template <int D>
int dispatch_w(int WP, const mlpp::Args& a, int64_t nw, hipStream_t st, bool pass2) {
#ifdef PDEINV_PAIRS_QUICK  // development builds: one instantiation
  if (D == 2 && WP == 20) { launch_pairs<2, 20>(a, nw, st, pass2); return PDEINV_OK; }
  return fail(PDEINV_ERR_UNSUPPORTED, "quick build");
#else
  switch (WP) {
    case 8: launch_pairs<D, 8>(a, nw, st, pass2); break;
    case 16: launch_pairs<D, 16>(a, nw, st, pass2); break;
    case 20: launch_pairs<D, 20>(a, nw, st, pass2); break;
    case 24: launch_pairs<D, 24>(a, nw, st, pass2); break;
    case 28: launch_pairs<D, 28>(a, nw, st, pass2); break;
    default: return fail(PDEINV_ERR_UNSUPPORTED, "kmv_mlp pairs: width");
  }
  return PDEINV_OK;
#endif
}
}  // namespace

// the MFMA pair-tile kernels (mlp_pairs_mfma.hip) take the shapes they cover (dim <= 8, width <= 20,
// n_layers <= 8, any out_features: the reference default); the register-ring kernels here the rest of
// width <= 28 (n_layers <= 16, out_features <= 64), or every such shape under PDEINV_MLP_IMPL_PAIRS_RING
bool kmvq_supported(const pdeinv_kmv_mlp_desc* d);
size_t kmvq_workspace_bytes(const pdeinv_kmv_mlp_desc* d);
int kmvq_run(const pdeinv_kmv_mlp_desc* d, const float* z, int64_t set_stride, int64_t ld, const float* ds,
             const float* params, void* ws, double* acc, float* grad, float** gbar_out, int pass, hipStream_t st);

static bool ring_supported(const pdeinv_kmv_mlp_desc* d) {
  return d->dim >= 1 && d->dim <= 8 && d->width >= 1 && d->width <= 28 && d->n_layers >= 1 &&
         d->n_layers <= mlpp::kMaxL && d->out_features >= 1 && d->out_features <= 64;
}

bool kmv_pairs_supported(const pdeinv_kmv_mlp_desc* d) { return kmvq_supported(d) || ring_supported(d); }

size_t kmv_pairs_workspace_bytes(const pdeinv_kmv_mlp_desc* d) {
  return kmvq_supported(d) ? kmvq_workspace_bytes(d) : pair_plan(d).total;
}

// pass 1 (gbar) + the stamp terms (caller), then pass 2; grad and acc accumulate (+=)
int kmv_pairs_run(const pdeinv_kmv_mlp_desc* d, const float* z, int64_t set_stride, int64_t ld, const float* ds,
                  const float* params, void* ws, double* acc, float* grad, float** gbar_out, int pass,
                  hipStream_t st) {
  if (kmvq_supported(d)) return kmvq_run(d, z, set_stride, ld, ds, params, ws, acc, grad, gbar_out, pass, st);
  const PairPlan p = pair_plan(d);
  char* w = (char*)ws;
  float* prm = (float*)(w + p.off_prm);
  mlpp::Args a{};
  a.L = d->n_layers;
  a.O = p.pm.pout[a.L];  // padded to a multiple of kOC (zero columns)
  a.Dr = d->dim;
  a.n = d->n_rows;
  a.n_items = p.items;
  a.set_stride = set_stride;
  a.ld = ld;
  a.z = z;
  a.ds = ds;
  a.gamma = d->gamma;
  a.s = (float)(1.0 / ((double)d->n_rows * (double)d->n_rows * (double)d->n_sets));
  a.inv_n = (float)(1.0 / (double)d->n_rows);
  a.prm = (mlpp::cfloat*)prm;
  a.P = (int)p.P;
  a.gbar = (float*)(w + p.off_gbar);
  a.scratch = (float*)(w + p.off_scratch);
  a.gslab = (float*)(w + p.off_gslab);
  a.aslab = (float*)(w + p.off_aslab);
  if (gbar_out) *gbar_out = a.gbar;
  int rc = PDEINV_OK;
  if (pass == 0) {
    hipLaunchKernelGGL(mlpp::kmvp_pad_kernel, dim3((unsigned)((p.P + 255) / 256)), dim3(256), 0, st, p.pm, params,
                       p.P, prm);
    rc = check_launch("kmvp_pad_kernel");
    if (rc) return rc;
  } else {
    if (hipMemsetAsync(a.gslab, 0, sizeof(float) * (size_t)p.n_waves * p.P, st) != hipSuccess ||
        hipMemsetAsync(a.aslab, 0, sizeof(float) * (size_t)p.n_waves * 8, st) != hipSuccess)
      return fail(PDEINV_ERR_HIP, "kmv_mlp pairs: memset");
  }
  switch (p.DP) {
    case 2: rc = dispatch_w<2>(p.WP, a, p.n_waves, st, pass == 1); break;
    case 4: rc = dispatch_w<4>(p.WP, a, p.n_waves, st, pass == 1); break;
    case 8: rc = dispatch_w<8>(p.WP, a, p.n_waves, st, pass == 1); break;
    default: rc = fail(PDEINV_ERR_UNSUPPORTED, "kmv_mlp pairs: dim");
  }
  if (rc) return rc;
  rc = check_launch(pass ? "kmvp_grad_kernel" : "kmvp_gbar_kernel");
  if (rc || pass == 0) return rc;
  hipLaunchKernelGGL(mlpp::kmvp_reduce_kernel, dim3((unsigned)((p.P + 255) / 256)), dim3(256), 0, st, p.pm, a.gslab,
                     p.n_waves, p.P, a.aslab, grad, acc);
  return check_launch("kmvp_reduce_kernel");
}

}  // namespace pdeinv
