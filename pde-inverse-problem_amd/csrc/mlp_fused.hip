// mlp_fused.hip — the V_hypothesis KFP residual on hand-written fp32 MFMA kernels (gfx950).
//
// Same algebra as mlp.hip's library path (oracle/numpy_ref.py kfp_mlp_grad_analytic), but the
// element-wise steps ride in GEMM prologues (building the A operand in LDS) or epilogues (on the
// accumulators). The first hidden layer has K = d (<= 16) inputs, so its streams come from small
// VALU kernels over the sample rows (h1 planes, abar1, g, and the layer-1 parameter gradient).
//
// Row GEMMs (samples x features):  C_s[BM x BN] = A_s[BM x K] . B[K x BN], s < S streams sharing
// one weight tile. v_mfma_f32_32x32x2_f32 (exact fp32, 64 cycles / SIMD, 16 acc regs); 4 waves
// in a WGM x WGN grid; A and B staged k-major in LDS (As[s][k][m], Bs[k][n]) so both MFMA operand
// reads are 32 consecutive floats per half-wave. Workgroups loop over row blocks (persistent grid)
// so the epilogues that reduce over rows (bias gradients) keep register partials and write one
// slab row per workgroup; slabs are summed in a fixed order (deterministic). The next k-tile's
// global loads are issued before the current tile's MFMAs (register prefetch).
//
// Weight gradients (sum over samples of 4 stream-pair outer products): C[n_in x n_out] =
// sum_p A_p^T B_p, rows split into slices (one partial slab each); the 4 pairs of a 16-row block
// are staged together so every source plane is read once per tile.
//
// Per chunk (L = 2; deeper nets add the "middle" steps):
//   FWD   z2 streams = [h1, h1', h1''] K2      A: layer 1 from the rows   E: tanh -> h2, z2', z2''
//   OUT   y streams  = [h2, h2', h2''] Ko      A: h', h'' from planes   E: +bo, V' and V'' per row
//   R1    a2 = (2y) Ko^T                                                E: store
//   R1    a1 = (s1(h2) a2) K2^T                                         E: store
//   g     g = (s1(z1) a1) K1^T                 VALU, one wave per row (layer-1 recompute)
//   loss  (mlp.hip)  per-row terms, abar0 = 2 c1 g
//   F2    zetabar2 = abar1 K2                  A: abar1 = s1(z1) (abar0 K1) from the rows   E: store
//   UB    ubar = (s1(h2) zetabar2) Ko                                   E: seeds ybar.., bo grad
//   R2    hbar2 streams = ybar streams Ko^T                             E: act_bwd -> zbar2, b2 grad
//   R2    hbar1 streams = zbar2 streams K2^T                            E: store
//   L1    layer-1 act_bwd + K1 / b1 gradient   VALU, columns per thread, rows looped
//   G     Ko += [h2..abar2]^T [ybar..u];  K2 += [h1..abar1]^T [zbar2..zeta2] (layer-1 streams rebuilt
//         from the rows in the A prologue: the h1 / abar1 planes never exist)
// First-order chunks (the initial / terminal sets, c1 = c2 = 0; W in {128, 256}) run run_chunk_fo2 instead: the
// same steps on two streams [h, z'] / [zbar, z'bar], without R1, g, F2 and UB (see there).
#include <math.h>

#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include <vector>

#include "mlp_fused.h"

namespace pdeinv {
namespace mlpf {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;   // feature k-step of the row GEMMs
// Row-GEMM LDS tiles are k-major with a row pitch of BM + 1 (A) / BN + 1 (B) floats. ds_write_b32
// banks are (addr/4) mod 32 per 32-lane half: the transposing stores (A from row-major planes, B_NT
// from row-major weights) put 32 consecutive k of one row in a half, i.e. a stride of one pitch;
// a pitch = 1 (mod 32) maps them to 32 distinct banks (the old + 4 pitch made them 4-way
// conflicts: SQ_LDS_BANK_CONFLICT > SQ_ACTIVE_INST_LDS in profiles/r02_c5_pmc_sq_v2.txt). The
// MFMA operand reads (32 consecutive floats of one k row per half) are conflict-free at any pitch.
constexpr int kPitchPad = 1;
constexpr int BKG = 16;  // rows per weight-gradient step (4 pairs staged together)
constexpr int kT = 256;

__device__ __forceinline__ float ftanh(float z) {
  const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * z);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

// 32-bit byte offsets from a uniform base (saddr addressing): a chunk's planes stay at or below 2^30 floats
// (byte offsets < 2^32, unsigned; run_chunk checks Bc * max(W, out) <= 2^30)
// Plane accesses keep the default cache policy (non-temporal plane loads everywhere measured C5 +10 ms: the planes
// re-read by later products lose their cache hits; non-temporal epilogue stores everywhere were mixed,
// profiles/r05_c5_out16_nt_ab.txt), except two streams that are touched once:
__device__ __forceinline__ float ldo(const float* base, uint32_t idx) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + (idx << 2));
}
__device__ __forceinline__ void sto(float* base, uint32_t idx, float v) {
  *reinterpret_cast<float*>(reinterpret_cast<char*>(base) + (idx << 2)) = v;
}
// the hbar1 planes (written by R2b, read once by l1_grad_kernel): l1_grad 3.79 -> 3.60 ms, R2b 13.61 -> 13.49 ms
// (profiles/r05_c5_nt_hb1_ab.txt)
__device__ __forceinline__ void sto_h(float* base, uint32_t idx, float v) {
  __builtin_nontemporal_store(v, reinterpret_cast<float*>(reinterpret_cast<char*>(base) + (idx << 2)));
}
__device__ __forceinline__ float ld_h(const float* p) { return __builtin_nontemporal_load(p); }
// the streaming epilogue of the K = out_features reverse product (R2a: five planes in, three out, 1.3 B of plane
// traffic per FLOP): C5 R2a 8.01 -> 7.79 ms, the products that re-read its planes unchanged
// (profiles/r05_c5_nt_epi_ab.txt)
__device__ __forceinline__ float ldo_s(const float* base, uint32_t idx) {
  return __builtin_nontemporal_load(reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + (idx << 2)));
}
__device__ __forceinline__ void sto_s(float* base, uint32_t idx, float v) {
  __builtin_nontemporal_store(v, reinterpret_cast<float*>(reinterpret_cast<char*>(base) + (idx << 2)));
}

// Workgroup placement: the dispatcher hands linear workgroup b to XCD b % 8. xcd_linear(b, nb)
// renumbers so that each XCD runs one contiguous range of logical ids; kernels then split the
// logical id so that the workgroups that read the same rows (the column blocks of a row GEMM, the
// output tiles of a weight-gradient slice) are consecutive — same XCD, resident together, so the
// second reader of a plane hits that XCD's L2 instead of HBM. Pure renumbering (same results).
__device__ __forceinline__ int xcd_linear(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8, l = b / 8;
  return x < r ? x * (q + 1) + l : r * (q + 1) + (x - r) * q + l;
}

enum { A_RAW1 = 0, A_FWD, A_S1MUL, A_U, A_S3, A_L1F, A_L1A, A_FWD2, A_S2 };
// A_L1F / A_L1A build the layer-1 streams in the prologue from the sample rows (no h1 planes):
//   A_L1F: [h1, s1 z1', s2 z1'^2] with z1 = x K1 + b1, z1' = v K1      (the FWD operand)
//   A_L1A: abar1 = s1(z1) (abar0 K1)                                      (the F2 operand)
// A_FWD2 / A_S2 are the first-order chain's two-stream forms of A_FWD / A_S3 ([h, s1 z'] | two raw planes).
// One thread owns one row (x and v | abar0 in registers), K1^T and b1 sit in LDS (broadcast reads).
enum { B_NN = 0, B_NT };
enum { E_ACT_FWD = 0, E_OUT, E_STORE, E_STORE3, E_SEEDS, E_ACT_BWD, E_OUT_SEEDS1 };
// E_OUT_SEEDS1 (first-order chunks, S = 2): the output layer's E_OUT terms and, in the same epilogue, the reverse
// seeds ybar = 2 c3 y' + 2 c0 y, y'bar = 2 c3 y (c1 = c2 = 0 there, so ubar = 0 and y''bar = 0) with the output bias
// gradient partials — the UB product and the y planes are not needed. S = 2 epilogues carry only the h and z'
// streams (E_ACT_FWD / E_STORE3) and, in E_ACT_BWD, drop the z'' and adjoint (a zetabar) terms, which are zero there.

struct GemmArgs {
  int64_t R;
  int K, N;
  int n_mblocks;
  const float *pa0, *pa1, *pa2;           // A-source planes, ld K
  const float* Bw;                        // [K x N] (B_NN) or [N x K] (B_NT), row-major
  const float* bias;                      // [N], stream 0 (E_ACT_FWD, E_OUT)
  float *po0, *po1, *po2;                 // outputs, ld N
  const float *pe0, *pe1, *pe2, *pe3, *pe4;  // epilogue inputs, ld N
  float4* terms;  // per row {V', V'', V, 0}
  float c2, c3, c0;
  float* part;
  const float* xz;   // A_L1*: sample rows [x | v], stride ldxz
  int64_t ldxz;
  const float* ab0;  // A_L1A: abar0 [R x d]
  const float* k1;   // A_L1*: K1 [d x K] (flax [in, out]) and b1 [K]
  const float* b1;
  const float* wrow;  // E_SEEDS: per-row weight of c0 (KMV pair rows), stride ldw; nullptr = 1
  int64_t ldw;
};

template <int AM>
constexpr bool a_is_l1() { return AM == A_L1F || AM == A_L1A; }
template <int D>
constexpr int k1_stride() { return (D + 1 + 3) & ~3; }  // K1^T row: d weights, b1, pad to 16 B

// K1^T and b1 into LDS, row k = [K1[0][k] .. K1[d-1][k], b1[k], 0..]
template <int D>
__device__ __forceinline__ void stage_k1t(const float* __restrict__ k1, const float* __restrict__ b1, int K,
                                          float* k1s) {
  constexpr int SK = k1_stride<D>();
  for (int e = threadIdx.x; e < K * SK; e += kT) {
    const int k = e / SK, i = e - k * SK;
    k1s[e] = i < D ? k1[i * K + k] : (i == D ? b1[k] : 0.f);
  }
}

// layer-1 pre-activation z1 = x . K1[:, k] + b1[k] and the second projection y . K1[:, k]
template <int D>
__device__ __forceinline__ void l1_project(const float* x, const float* y, const float* kc, float& z, float& zy) {
  z = kc[D] + dotd<D>(x, kc);
  zy = dotd<D>(y, kc);
}

// ---- operand staging: global -> registers (issued one k-block ahead, in flight under the
//      MFMAs of the current block) -> prologue math -> LDS (k-major) ----------------------
template <int BM, int AM>
struct ARegs {
  static constexpr int NE = BM * BK / kT;  // elements per thread
  static constexpr int NV = (AM == A_FWD || AM == A_S3) ? 3 : ((AM == A_S1MUL || AM == A_FWD2 || AM == A_S2) ? 2 : 1);
  float v[NE][NV > 0 ? NV : 1];
};

// Loads are unconditional from a clamped 32-bit offset (a chunk's planes stay at or below 2^30 floats):
// no per-element exec-mask branches. The zeroing select of out-of-range elements happens in the
// store phase, after the MFMAs, so the loads stay in flight under the current tile's math.
template <int BM, int AM>
__device__ __forceinline__ void load_a(const GemmArgs& a, ARegs<BM, AM>& ra, int r0, int k0) {
#pragma unroll
  for (int j = 0; j < ARegs<BM, AM>::NE; ++j) {
    const int e = threadIdx.x + j * kT;
    const int m = e / BK, kk = e - m * BK;
    const int r = r0 + m, k = k0 + kk;
    const bool ok = r < a.R && k < a.K;
    const uint32_t o = ok ? (uint32_t)(r * a.K + k) : 0u;
    ra.v[j][0] = ldo(a.pa0, o);
    if constexpr (ARegs<BM, AM>::NV > 1) ra.v[j][1] = ldo(a.pa1, o);
    if constexpr (ARegs<BM, AM>::NV > 2) ra.v[j][2] = ldo(a.pa2, o);
  }
}

template <int S, int BM, int AM>
__device__ __forceinline__ void store_a(const GemmArgs& a, const ARegs<BM, AM>& ra, float* As, int r0, int k0,
                                        bool full) {
  constexpr int LDA = BM + kPitchPad;
#pragma unroll
  for (int j = 0; j < ARegs<BM, AM>::NE; ++j) {
    const int e = threadIdx.x + j * kT;
    const int m = e / BK, kk = e - m * BK;
    const bool ok = full || (r0 + m < a.R && k0 + kk < a.K);
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if constexpr (AM == A_FWD) {
      const float h = ra.v[j][0], zd = ra.v[j][1], zdd = ra.v[j][2];
      const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
      v0 = h;
      v1 = s1 * zd;
      v2 = fmaf(s1, zdd, s2 * zd * zd);
    } else if constexpr (AM == A_S1MUL) {
      const float h = ra.v[j][0];
      v0 = (1.f - h * h) * ra.v[j][1];
    } else if constexpr (AM == A_U) {
      v0 = 2.f * ra.v[j][0];
    } else if constexpr (AM == A_RAW1) {
      v0 = ra.v[j][0];
    } else if constexpr (AM == A_FWD2) {
      const float h = ra.v[j][0];
      v0 = h;
      v1 = (1.f - h * h) * ra.v[j][1];
    } else if constexpr (AM == A_S2) {
      v0 = ra.v[j][0];
      v1 = ra.v[j][1];
    } else {  // A_S3
      v0 = ra.v[j][0];
      v1 = ra.v[j][1];
      v2 = ra.v[j][2];
    }
    As[kk * LDA + m] = ok ? v0 : 0.f;
    if constexpr (S > 1) As[(BK + kk) * LDA + m] = ok ? v1 : 0.f;
    if constexpr (S > 2) As[(2 * BK + kk) * LDA + m] = ok ? v2 : 0.f;
  }
}

template <int BN, int BMD>
__device__ __forceinline__ void b_coords(int e, int& kk, int& nn) {
  if constexpr (BMD == B_NN) {
    kk = e / BN;
    nn = e - kk * BN;
  } else {
    nn = e / BK;
    kk = e - nn * BK;
  }
}

template <int BN, int BMD>
__device__ __forceinline__ void load_b(const GemmArgs& a, float (&rb)[BK * BN / kT], int k0, int n0) {
#pragma unroll
  for (int j = 0; j < BK * BN / kT; ++j) {
    int kk, nn;
    b_coords<BN, BMD>(threadIdx.x + j * kT, kk, nn);
    const int k = k0 + kk, n = n0 + nn;
    const bool ok = k < a.K && n < a.N;
    const uint32_t o = ok ? (uint32_t)(BMD == B_NN ? k * a.N + n : n * a.K + k) : 0u;
    rb[j] = ldo(a.Bw, o);
  }
}

template <int BN, int BMD>
__device__ __forceinline__ void store_b(const GemmArgs& a, const float (&rb)[BK * BN / kT], float* Bs, int k0, int n0,
                                        bool full) {
  constexpr int LDB = BN + kPitchPad;
#pragma unroll
  for (int j = 0; j < BK * BN / kT; ++j) {
    int kk, nn;
    b_coords<BN, BMD>(threadIdx.x + j * kT, kk, nn);
    const bool ok = full || (k0 + kk < a.K && n0 + nn < a.N);
    Bs[kk * LDB + nn] = ok ? rb[j] : 0.f;
  }
}

template <int S, int BM, int BN, int WGM, int AM, int BMD, int EM, int D = 0>
__global__ __launch_bounds__(kT, 2) void fgemm(GemmArgs a) {
  constexpr bool L1 = a_is_l1<AM>();
  static_assert(!L1 || (D > 0 && kT % BM == 0), "layer-1 prologue: D and one row per thread");
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 32, NI = WN / 32;
  static_assert(MI >= 1 && NI >= 1 && MI * 32 == WM && NI * 32 == WN, "wave tile must be 32-multiples");
  static_assert(EM != E_OUT || WGN == 1, "E_OUT reduces each row inside one wave");
  constexpr int LDA = BM + kPitchPad, LDB = BN + kPitchPad;
  constexpr int NP = (EM == E_SEEDS || EM == E_ACT_BWD) ? 1 : 0;
  extern __shared__ float lds[];
  float* As = lds;                  // [S][BK][LDA]
  float* Bs = As + S * BK * LDA;    // [BK][LDB]
  [[maybe_unused]] float* k1s = Bs + BK * LDB;  // L1 modes: [K][SK]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if constexpr (L1) stage_k1t<D>(a.k1, a.b1, a.K, k1s);  // visible after the k-loop's first barrier
  const int wm = wave / WGN, wn = wave - (wave / WGN) * WGN, l31 = lane & 31, hi = lane >> 5;
  const int gx = gridDim.x, gy = gridDim.y;
  const int lid = xcd_linear(blockIdx.x + blockIdx.y * gx, gx * gy);
  const int bx = lid / gy, by = lid - (lid / gy) * gy;  // column blocks of a row block adjacent
  const int n0 = by * BN;
  [[maybe_unused]] float pacc[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) pacc[ni] = 0.f;

  for (int mb = bx; mb < a.n_mblocks; mb += gx) {
    const int r0 = mb * BM;
    f32x16 acc[S][MI][NI];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int q = 0; q < 16; ++q) acc[s][mi][ni][q] = 0.f;

    ARegs<BM, L1 ? A_RAW1 : AM> ra;
    float rb[BK * BN / kT];
    [[maybe_unused]] float rx[L1 ? D : 1], ry[L1 ? D : 1];  // L1 modes: the thread's row (x, v | abar0)
    if constexpr (L1) {
      const int64_t r = std::min<int64_t>(r0 + tid % BM, a.R - 1);
#pragma unroll
      for (int i = 0; i < D; ++i) {
        rx[i] = a.xz[r * a.ldxz + i];
        ry[i] = AM == A_L1F ? a.xz[r * a.ldxz + D + i] : a.ab0[r * D + i];
      }
    } else {
      load_a<BM, AM>(a, ra, r0, 0);
    }
    load_b<BN, BMD>(a, rb, 0, n0);
    for (int k0 = 0; k0 < a.K; k0 += BK) {
      __syncthreads();  // every wave is done reading the previous tile
      if constexpr (L1) {
        const bool rok = r0 + tid % BM < a.R;
#pragma unroll
        for (int j = 0; j < BM * BK / kT; ++j) {
          const int m = tid % BM, kk = tid / BM + (kT / BM) * j;
          const bool ok = rok && k0 + kk < a.K;
          const float* kc = k1s + (ok ? k0 + kk : 0) * k1_stride<D>();
          float z, zy;
          l1_project<D>(rx, ry, kc, z, zy);
          const float h = ftanh(z), s1 = 1.f - h * h;
          if constexpr (AM == A_L1F) {
            As[kk * LDA + m] = ok ? h : 0.f;
            As[(BK + kk) * LDA + m] = ok ? s1 * zy : 0.f;
            As[(2 * BK + kk) * LDA + m] = ok ? -2.f * h * s1 * zy * zy : 0.f;
          } else {
            As[kk * LDA + m] = ok ? s1 * zy : 0.f;
          }
        }
      } else {
        store_a<S, BM, AM>(a, ra, As, r0, k0, r0 + BM <= a.R && k0 + BK <= a.K);
      }
      store_b<BN, BMD>(a, rb, Bs, k0, n0, k0 + BK <= a.K && n0 + BN <= a.N);
      __syncthreads();
      if (k0 + BK < a.K) {  // next tile's global loads fly under this tile's MFMAs
        if constexpr (!L1) load_a<BM, AM>(a, ra, r0, k0 + BK);
        load_b<BN, BMD>(a, rb, k0 + BK, n0);
      }
      // the last tile of a K that is not a BK multiple (the reverse K = out_features product, A_S3)
      // stops at its last valid k pair: a wave-uniform skip instead of MFMAs on the zero padding (in the
      // other modes the branch only added spills: not compiled there)
      const int kv = (AM == A_S3 || AM == A_S2) ? a.K - k0 : BK;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        if (kk < kv) {
          float bv[NI];
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) bv[ni] = Bs[(kk + hi) * LDB + wn * WN + ni * 32 + l31];
#pragma unroll
          for (int s = 0; s < S; ++s)
#pragma unroll
            for (int mi = 0; mi < MI; ++mi) {
              const float av = As[(s * BK + kk + hi) * LDA + wm * WM + mi * 32 + l31];
#pragma unroll
              for (int ni = 0; ni < NI; ++ni)
                acc[s][mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[ni], acc[s][mi][ni], 0, 0, 0);
            }
        }
      }
    }

    // ---- epilogue: acc register q of tile (mi, ni) is C[row][col] with
    //      row = (q & 3) + 8 (q >> 2) + 4 (lane >> 5), col = lane & 31 (32x32 C/D map)
    const bool full = r0 + BM <= a.R && n0 + BN <= a.N;  // interior tile: guard-free copy
    auto epilogue = [&](auto check) {
      constexpr bool CHECK = decltype(check)::value;
  #pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        [[maybe_unused]] float t0[16], t1[16], t2[16];
        if constexpr (EM == E_OUT) {
  #pragma unroll
          for (int q = 0; q < 16; ++q) t0[q] = t1[q] = t2[q] = 0.f;
        }
  #pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const int n = n0 + wn * WN + ni * 32 + l31;
          const bool nv = n < a.N;
          [[maybe_unused]] float bn = 0.f;
          if constexpr (EM == E_ACT_FWD || EM == E_OUT) bn = a.bias[nv ? n : 0];
  #pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int r = r0 + wm * WM + mi * 32 + (q & 3) + 8 * (q >> 2) + 4 * hi;
            const bool ok = !CHECK || (nv && r < a.R);
            const uint32_t o = (uint32_t)(r * a.N + n);
            if constexpr (EM == E_ACT_FWD) {
              if (ok) {
                sto(a.po0, o, ftanh(acc[0][mi][ni][q] + bn));
                sto(a.po1, o, acc[1][mi][ni][q]);
                if constexpr (S > 2) sto(a.po2, o, acc[S - 1][mi][ni][q]);
              }
            } else if constexpr (EM == E_STORE) {
              if (ok) sto(a.po0, o, acc[0][mi][ni][q]);
            } else if constexpr (EM == E_STORE3) {
              if (ok) {
                sto(a.po0, o, acc[0][mi][ni][q]);
                sto(a.po1, o, acc[1][mi][ni][q]);
                if constexpr (S > 2) sto(a.po2, o, acc[S - 1][mi][ni][q]);
              }
            } else if constexpr (EM == E_OUT) {
              if (ok) {
                const float y = acc[0][mi][ni][q] + bn, yd = acc[1][mi][ni][q], ydd = acc[2][mi][ni][q];
                sto(a.po0, o, y);
                sto(a.po1, o, yd);
                sto(a.po2, o, ydd);
                t0[q] = fmaf(y, y, t0[q]);
                t1[q] = fmaf(y, yd, t1[q]);
                t2[q] = fmaf(yd, yd, fmaf(y, ydd, t2[q]));
              }
            } else if constexpr (EM == E_SEEDS) {
              if (ok) {
                const float ub = acc[0][mi][ni][q];
                const float y = ldo(a.pe0, o), yd = ldo(a.pe1, o), ydd = ldo(a.pe2, o);
                const float c0r = a.wrow ? a.c0 * a.wrow[(int64_t)r * a.ldw] : a.c0;
                const float yb = 2.f * a.c3 * yd + 2.f * a.c2 * ydd + 2.f * ub + 2.f * c0r * y;
                sto(a.po0, o, yb);
                sto(a.po1, o, 2.f * a.c3 * y + 4.f * a.c2 * yd);
                sto(a.po2, o, 2.f * a.c2 * y);
                pacc[ni] += yb;
              }
            } else if constexpr (EM == E_ACT_BWD) {
              if (ok) {
                const float hb = acc[0][mi][ni][q], hdb = acc[1][mi][ni][q];
                const float h = ldo_s(a.pe0, o), zd = ldo_s(a.pe1, o);
                const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
                if constexpr (S > 2) {
                  const float hddb = acc[S - 1][mi][ni][q];
                  const float zdd = ldo_s(a.pe2, o), aL = ldo_s(a.pe3, o), zb = ldo_s(a.pe4, o);
                  const float s3 = -2.f * s1 * s1 - 2.f * h * s2;
                  const float zbar = s1 * hb + s2 * zd * hdb + (s2 * zdd + s3 * zd * zd) * hddb + s2 * aL * zb;
                  sto_s(a.po0, o, zbar);
                  sto_s(a.po1, o, s1 * hdb + 2.f * s2 * zd * hddb);
                  sto_s(a.po2, o, s1 * hddb);
                  pacc[ni] += zbar;
                } else {  // first-order chain: h'' bar = 0, a zetabar = 0
                  const float zbar = s1 * hb + s2 * zd * hdb;
                  sto(a.po0, o, zbar);
                  sto(a.po1, o, s1 * hdb);
                  pacc[ni] += zbar;
                }
              }
            }
          }
        }
        if constexpr (EM == E_OUT) {
  #pragma unroll
          for (int q = 0; q < 16; ++q) {
            float p0 = t0[q], p1 = t1[q], p2 = t2[q];
  #pragma unroll
            for (int off = 16; off > 0; off >>= 1) {
              p0 += __shfl_xor(p0, off, 64);
              p1 += __shfl_xor(p1, off, 64);
              p2 += __shfl_xor(p2, off, 64);
            }
            const int r = r0 + wm * WM + mi * 32 + (q & 3) + 8 * (q >> 2) + 4 * hi;
            // out_features > BN: one partial per column block (by), summed by terms_sum_kernel
            if (l31 == 0 && r < a.R) a.terms[(int64_t)by * a.R + r] = make_float4(2.f * p1, 2.f * p2, p0, 0.f);
          }
        }
      }
    };
    if (full) epilogue(std::false_type{});
    else epilogue(std::true_type{});
  }

  if constexpr (NP > 0) {
    __syncthreads();
    float* red = lds;  // [WGM][BN]
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const float v = pacc[ni] + __shfl_xor(pacc[ni], 32, 64);
      if (hi == 0) red[wm * BN + wn * WN + ni * 32 + l31] = v;
    }
    __syncthreads();
    for (int c = tid; c < BN; c += kT) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < WGM; ++w) s += red[w * BN + c];
      if (n0 + c < a.N) a.part[(int64_t)bx * a.N + n0 + c] = s;
    }
  }
}

// ---- layer-1 kernels (VALU; K1 is d x W, d <= 16) ------------------------------------------
// g = zeta1 K1^T with zeta1 = s1(z1) a1, z1 = x K1 + b1: one wave per row, lane owns columns
// lane + 64 j; the d partial sums are wave-reduced.
template <int D, int W>
__global__ __launch_bounds__(kT) void l1_g_kernel(const float* __restrict__ a1, const float* __restrict__ z,
                                                  int64_t ldz, const float* __restrict__ K1,
                                                  const float* __restrict__ b1, int64_t R, float* __restrict__ G) {
  constexpr int CPL = W >= 64 ? W / 64 : 1;  // W < 64: lanes >= W carry zero weights
  const int lane = threadIdx.x & 63;
  const bool cv = W >= 64 || lane < W;
  const int lc = cv ? lane : 0;
  float k1[CPL][D], bb[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    bb[j] = cv ? b1[lc + 64 * j] : 0.f;
#pragma unroll
    for (int i = 0; i < D; ++i) k1[j][i] = cv ? K1[i * W + lc + 64 * j] : 0.f;
  }
  const int64_t nw = (int64_t)gridDim.x * (kT / 64);
  for (int64_t r = (int64_t)blockIdx.x * (kT / 64) + (threadIdx.x >> 6); r < R; r += nw) {
    float x[D], g[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      x[i] = z[r * ldz + i];
      g[i] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      float zz = bb[j];
#pragma unroll
      for (int i = 0; i < D; ++i) zz = fmaf(x[i], k1[j][i], zz);
      const float h = ftanh(zz);
      const float zeta = cv ? (1.f - h * h) * a1[r * W + lc + 64 * j] : 0.f;
#pragma unroll
      for (int i = 0; i < D; ++i) g[i] = fmaf(zeta, k1[j][i], g[i]);
    }
#pragma unroll
    for (int i = 0; i < D; ++i) g[i] = wave_sum(g[i]);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < D; ++i) G[r * D + i] = g[i];
    }
  }
}

// The same g on the matrix pipe (W <= 256): per wave, 16 rows at a time and 16-column groups of
// layer 1. Z^T[c][row] = [K1; b1]^T[c][:] . [x; 1][row] as (D + 1) / 4 rounded-up v_mfma_f32_16x16x4_f32
// (A = the K1 columns, lane constants; B = the rows' x) leaves lane (row, h) with columns 4 h + t of the
// group in register t — exactly the (m = row, k-slot h) A layout of G[row][i] += zeta[row][c] K1[i][c]
// (4 MFMAs per group, B = K1[i][c] lane constants, i = lane & 15 < D), so zeta = s1(z) a1 never leaves
// the lane and the d-wide row sums need no cross-lane reduction (the VALU kernel above spends 8 wave
// reductions per row). a1 is read as one 16-byte run per lane (4 consecutive columns of its row).
template <int D, int W>
__global__ __launch_bounds__(kT) void l1_g_mfma_kernel(const float* __restrict__ a1, const float* __restrict__ z,
                                                       int64_t ldz, const float* __restrict__ K1,
                                                       const float* __restrict__ b1, int64_t R, float* __restrict__ G) {
  static_assert(W % 16 == 0 && W <= 256 && D <= 16, "l1_g_mfma: W <= 256, d <= 16");
  constexpr int NG = W / 16, NS = (D + 1 + 3) / 4;  // column groups; k-steps of [x; 1]
  const int lane = threadIdx.x & 63, c16 = lane & 15, rq = lane >> 4;
  float kz[NG][NS], kg[NG][4];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int c = 16 * g + c16;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int i = 4 * s + rq;
      kz[g][s] = i < D ? K1[i * W + c] : (i == D ? b1[c] : 0.f);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) kg[g][t] = c16 < D ? K1[c16 * W + 16 * g + 4 * rq + t] : 0.f;
  }
  const int64_t nw = (int64_t)gridDim.x * (kT / 64);
  for (int64_t r0 = ((int64_t)blockIdx.x * (kT / 64) + (threadIdx.x >> 6)) * 16; r0 < R; r0 += nw * 16) {
    const int64_t row = std::min<int64_t>(r0 + c16, R - 1);
    float xb[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int i = 4 * s + rq;
      xb[s] = i < D ? z[row * ldz + i] : (i == D ? 1.f : 0.f);
    }
    const f32x4* arow = reinterpret_cast<const f32x4*>(a1 + row * W + 4 * rq);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    f32x4 an = arow[0];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const f32x4 av = an;
      if (g + 1 < NG) an = arow[4 * (g + 1)];  // the next group's a1 run, in flight under this group
      f32x4 zt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) zt = __builtin_amdgcn_mfma_f32_16x16x4f32(kz[g][s], xb[s], zt, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float h = ftanh(zt[t]);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32((1.f - h * h) * av[t], kg[g][t], acc, 0, 0, 0);
      }
    }
    // acc: lane (i = c16, h) holds G[r0 + 4 h + q][i] in register q
    if (c16 < D) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = r0 + 4 * rq + q;
        if (r < R) G[r * D + c16] = acc[q];
      }
    }
  }
}

// Layer-1 reverse step and its parameter gradient, from hbar1 streams (R2 final GEMM) and a1:
//   zbar1 = s1 hb + s2 z1' h'b + s3 z1'^2 h''b + s2 a1 zetabar1,  z'bar1 = s1 h'b + 2 s2 z1' h''b,
//   zeta1 = s1 a1;  K1[i][k] += x_i zbar1 + v_i z'bar1 + abar0_i zeta1,  b1[k] += zbar1
// (the third input stream h0'' = 0 carries nothing). Thread owns columns, loops rows; per-block
// partial slab [(D + 1) x W] (K1 rows then b1 = the flat parameter order). FO (first-order chunks): h''bar = 0
// and a1 = abar0 = 0, so zbar1 = s1 hb + s2 z1' h'b, z'bar1 = s1 h'b — hb2, a1 and abar0 are not read.
constexpr int kL1Rows = 64;  // rows staged in LDS per step

template <int D, int W, bool FO = false>
__global__ __launch_bounds__(kT) void l1_grad_kernel(const float* __restrict__ hb0, const float* __restrict__ hb1,
                                                     const float* __restrict__ hb2, const float* __restrict__ a1,
                                                     const float* __restrict__ z, int64_t ldz,
                                                     const float* __restrict__ abar0, const float* __restrict__ K1,
                                                     const float* __restrict__ b1, int64_t R, int64_t rpb,
                                                     float* __restrict__ part) {
  constexpr int CW = W < kT ? W : kT;       // columns covered per pass
  constexpr int CPT = W / CW;               // columns per thread
  constexpr int RPH = kT / CW;              // row phases
  constexpr int XC = FO ? 2 * D : 3 * D;  // staged row: x | v (| abar0)
  __shared__ float xs[kL1Rows * XC];
  __shared__ float red[(RPH > 1 ? RPH : 1) * W];
  const int tid = threadIdx.x, c0 = tid % CW, ph = tid / CW;
  float k1[CPT][D], bb[CPT], pacc[CPT][D + 1];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    bb[j] = b1[c0 + CW * j];
#pragma unroll
    for (int i = 0; i < D; ++i) k1[j][i] = K1[i * W + c0 + CW * j];
#pragma unroll
    for (int i = 0; i <= D; ++i) pacc[j][i] = 0.f;
  }
  const int64_t rs = (int64_t)blockIdx.x * rpb;
  const int64_t re = rs + rpb < R ? rs + rpb : R;
  for (int64_t rb = rs; rb < re; rb += kL1Rows) {
    __syncthreads();
    for (int e = tid; e < kL1Rows * XC; e += kT) {
      const int m = e / XC, c = e - m * XC;
      const int64_t r = rb + m;
      xs[e] = r < re ? (c < 2 * D ? z[r * ldz + c] : abar0[r * D + c - 2 * D]) : 0.f;
    }
    __syncthreads();
    const int nr = (int)(re - rb < kL1Rows ? re - rb : kL1Rows);
    for (int m = ph; m < nr; m += RPH) {
      const float* x = xs + m * XC;
      const int64_t rowo = (rb + m) * W;
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int64_t o = rowo + c0 + CW * j;
        if constexpr (FO) {
          const float hb = ld_h(hb0 + o), hdb = ld_h(hb1 + o);
          float zz = bb[j], zd = 0.f;
#pragma unroll
          for (int i = 0; i < D; ++i) {
            zz = fmaf(x[i], k1[j][i], zz);
            zd = fmaf(x[D + i], k1[j][i], zd);
          }
          const float h = ftanh(zz);
          const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
          const float zbar = s1 * hb + s2 * zd * hdb, zdbar = s1 * hdb;
#pragma unroll
          for (int i = 0; i < D; ++i) pacc[j][i] = fmaf(x[i], zbar, fmaf(x[D + i], zdbar, pacc[j][i]));
          pacc[j][D] += zbar;
        } else {
          const float hb = ld_h(hb0 + o), hdb = ld_h(hb1 + o), hddb = ld_h(hb2 + o), aL = a1[o];
          float zz = bb[j], zd = 0.f, zb = 0.f;
#pragma unroll
          for (int i = 0; i < D; ++i) {
            zz = fmaf(x[i], k1[j][i], zz);
            zd = fmaf(x[D + i], k1[j][i], zd);
            zb = fmaf(x[2 * D + i], k1[j][i], zb);
          }
          const float h = ftanh(zz);
          const float s1 = 1.f - h * h, s2 = -2.f * h * s1, s3 = -2.f * s1 * s1 - 2.f * h * s2;
          const float zbar = s1 * hb + s2 * zd * hdb + s3 * zd * zd * hddb + s2 * aL * zb;
          const float zdbar = s1 * hdb + 2.f * s2 * zd * hddb;
          const float zeta = s1 * aL;
#pragma unroll
          for (int i = 0; i < D; ++i)
            pacc[j][i] = fmaf(x[i], zbar, fmaf(x[D + i], zdbar, fmaf(x[2 * D + i], zeta, pacc[j][i])));
          pacc[j][D] += zbar;
        }
      }
    }
  }
  float* out = part + (int64_t)blockIdx.x * (D + 1) * W;
#pragma unroll
  for (int i = 0; i <= D; ++i) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < CPT; ++j) red[ph * W + c0 + CW * j] = pacc[j][i];
    __syncthreads();
    for (int c = tid; c < W; c += kT) {
      float s = 0.f;
#pragma unroll
      for (int p = 0; p < RPH; ++p) s += red[p * W + c];
      out[i * W + c] = s;
    }
  }
}

// ---- weight gradients -------------------------------------------------------------------
// A streams: 4 stored planes | h, s1 z', s1 z'' + s2 z'^2, s1 zetabar | the layer-1 streams
// [h1, s1 z1', s2 z1'^2, s1 (abar0 K1)] rebuilt from the sample rows (thread owns one feature, its
// K1 column in registers; the 16 rows of a step staged in LDS one step ahead)
enum { GA_RAW4 = 0, GA_PL, GA_L1 };
enum { GB_PL = 0, GB_SM };    // B streams: zbar0..2, s1(h) a | ybar0..2, 2 y

struct WgradArgs {
  int64_t R;
  int n_in, n_out;
  int64_t rows_per_slice;
  const float *pa0, *pa1, *pa2, *pa3;        // A planes (ld n_in)
  const float *pb0, *pb1, *pb2, *pb3, *pb4;  // B planes (ld n_out): ZB0..2, H, A  |  YB0..2, Y0
  float* part;                               // [slices][n_in][n_out]
  const float* xz;                           // GA_L1: rows [x | v] (ld ldxz), abar0 [R x d], K1, b1
  int64_t ldxz;
  const float* ab0;
  const float* k1;
  const float* b1;
};

// Byte offsets inside one chunk's planes fit in 32 bits (run_chunk checks Bc * W <= 2^30), so the
// loads use a uniform base + 32-bit lane offset.
template <int D>
constexpr int xrow_stride() { return (3 * D + 3) & ~3; }  // [x | v | abar0] padded to 16 B

template <int BM, int BN, int GA, int GB, int D = 0>
__global__ __launch_bounds__(kT) void fwgrad(WgradArgs a) {
  static_assert(GA != GA_L1 || (D > 0 && kT % BM == 0), "GA_L1: D and one feature per thread");
  constexpr int XS = GA == GA_L1 ? xrow_stride<D>() : 1;
  constexpr int NX = GA == GA_L1 ? (BKG * XS + kT - 1) / kT : 1;
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 32, NI = WN / 32;
  static_assert(MI >= 1 && NI >= 1, "tile");
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int NEA = BKG * BM / kT, NEB = BKG * BN / kT;
  constexpr int NVB = GB == GB_PL ? 5 : 4;
  extern __shared__ float lds[];
  float* As = lds;                  // [4][BKG][LDA]  (k = sample row)
  float* Bs = As + 4 * BKG * LDA;   // [4][BKG][LDB]
  [[maybe_unused]] float* xs = Bs + 4 * BKG * LDB;  // GA_L1: [2][BKG][XS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, l31 = lane & 31, hi = lane >> 5;
  const int tiles_n = (a.n_out + BN - 1) / BN;
  const int n_tiles = gridDim.x;
  const int lid = xcd_linear(blockIdx.x + blockIdx.y * n_tiles, n_tiles * gridDim.y);
  const int tile = lid % n_tiles, slice = lid / n_tiles;  // the tiles of one row slice adjacent
  const int i0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int rs0 = (int)((int64_t)slice * a.rows_per_slice);
  const int rs1 = (int)(rs0 + a.rows_per_slice < a.R ? rs0 + a.rows_per_slice : a.R);
  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[mi][ni][q] = 0.f;

  float ra[GA == GA_L1 ? 1 : NEA][4], rb[NEB][NVB];
  [[maybe_unused]] float kc[GA == GA_L1 ? D + 1 : 1], xr[NX];
  if constexpr (GA == GA_L1) {
    const int i = std::min(i0 + tid % BM, a.n_in - 1);
#pragma unroll
    for (int q = 0; q < D; ++q) kc[q] = a.k1[q * a.n_in + i];
    kc[D] = a.b1[i];
  }
  auto load_x = [&](int rb0) {  // the step's sample rows -> registers (staged to LDS one step later)
#pragma unroll
    for (int t = 0; t < NX; ++t) {
      const int e = tid + t * kT, rr = e / XS, cc = e - rr * XS, r = rb0 + rr;
      float v = 0.f;
      if (e < BKG * XS && r < rs1 && cc < 3 * D)
        v = cc < 2 * D ? a.xz[(int64_t)r * a.ldxz + cc] : a.ab0[(int64_t)r * D + cc - 2 * D];
      xr[t] = v;
    }
  };
  auto stage_x = [&](int buf) {
#pragma unroll
    for (int t = 0; t < NX; ++t) {
      const int e = tid + t * kT;
      if (e < BKG * XS) xs[buf * BKG * XS + e] = xr[t];
    }
  };
  auto load = [&](int rb0) {
#pragma unroll
    for (int j = 0; j < (GA == GA_L1 ? 0 : NEA); ++j) {
      const int e = tid + j * kT, rr = e / BM, ii = e - rr * BM;
      const int r = rb0 + rr, i = i0 + ii;
      const bool ok = r < rs1 && i < a.n_in;
      const uint32_t o = ok ? (uint32_t)(r * a.n_in + i) : 0u;
      ra[j][0] = ldo(a.pa0, o);
      ra[j][1] = ldo(a.pa1, o);
      ra[j][2] = ldo(a.pa2, o);
      ra[j][3] = ldo(a.pa3, o);
    }
#pragma unroll
    for (int j = 0; j < NEB; ++j) {
      const int e = tid + j * kT, rr = e / BN, nn = e - rr * BN;
      const int r = rb0 + rr, n = n0 + nn;
      const bool ok = r < rs1 && n < a.n_out;
      const uint32_t o = ok ? (uint32_t)(r * a.n_out + n) : 0u;
      rb[j][0] = ldo(a.pb0, o);
      rb[j][1] = ldo(a.pb1, o);
      rb[j][2] = ldo(a.pb2, o);
      rb[j][3] = ldo(a.pb3, o);
      if constexpr (NVB > 4) rb[j][4] = ldo(a.pb4, o);
    }
  };
  auto store = [&](int rb0, int buf) {
    const bool rows_full = rb0 + BKG <= rs1;
#pragma unroll
    for (int j = 0; j < NEA; ++j) {
      const int e = tid + j * kT, rr = e / BM, ii = e - rr * BM;
      const bool ok = (rows_full || rb0 + rr < rs1) && i0 + ii < a.n_in;
      float v0, v1, v2, v3;
      if constexpr (GA == GA_L1) {
        const float* xrow = xs + (buf * BKG + rr) * XS;
        const float z = kc[D] + dotd<D>(xrow, kc), zd = dotd<D>(xrow + D, kc), zb = dotd<D>(xrow + 2 * D, kc);
        const float h = ftanh(z), s1 = 1.f - h * h;
        v0 = h;
        v1 = s1 * zd;
        v2 = -2.f * h * s1 * zd * zd;
        v3 = s1 * zb;
      } else {
        v0 = ra[j][0]; v1 = ra[j][1]; v2 = ra[j][2]; v3 = ra[j][3];
      }
      if constexpr (GA == GA_PL) {
        const float h = v0, zd = v1, zdd = v2, zeb = v3;
        const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
        v1 = s1 * zd;
        v2 = fmaf(s1, zdd, s2 * zd * zd);
        v3 = s1 * zeb;
      }
      As[(0 * BKG + rr) * LDA + ii] = ok ? v0 : 0.f;
      As[(1 * BKG + rr) * LDA + ii] = ok ? v1 : 0.f;
      As[(2 * BKG + rr) * LDA + ii] = ok ? v2 : 0.f;
      As[(3 * BKG + rr) * LDA + ii] = ok ? v3 : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NEB; ++j) {
      const int e = tid + j * kT, rr = e / BN, nn = e - rr * BN;
      const bool ok = (rows_full || rb0 + rr < rs1) && n0 + nn < a.n_out;
      float v3;
      if constexpr (GB == GB_PL) {
        const float h = rb[j][3];
        v3 = (1.f - h * h) * rb[j][4];
      } else {
        v3 = 2.f * rb[j][3];
      }
      Bs[(0 * BKG + rr) * LDB + nn] = ok ? rb[j][0] : 0.f;
      Bs[(1 * BKG + rr) * LDB + nn] = ok ? rb[j][1] : 0.f;
      Bs[(2 * BKG + rr) * LDB + nn] = ok ? rb[j][2] : 0.f;
      Bs[(3 * BKG + rr) * LDB + nn] = ok ? v3 : 0.f;
    }
  };

  if (rs0 < rs1) {
    load(rs0);
    if constexpr (GA == GA_L1) {
      load_x(rs0);
      stage_x(0);
      if (rs0 + BKG < rs1) load_x(rs0 + BKG);
    }
  }
  for (int rb0 = rs0, it = 0; rb0 < rs1; rb0 += BKG, ++it) {
    __syncthreads();
    store(rb0, it & 1);
    if constexpr (GA == GA_L1) stage_x((it & 1) ^ 1);  // next step's rows (buffer last read a step ago)
    __syncthreads();
    if (rb0 + BKG < rs1) load(rb0 + BKG);  // in flight under this block's MFMAs
    if constexpr (GA == GA_L1)
      if (rb0 + 2 * BKG < rs1) load_x(rb0 + 2 * BKG);
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int kk = 0; kk < BKG; kk += 2) {
        float bv[NI];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bv[ni] = Bs[(p * BKG + kk + hi) * LDB + wn * WN + ni * 32 + l31];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
          const float av = As[(p * BKG + kk + hi) * LDA + wm * WM + mi * 32 + l31];
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[ni], acc[mi][ni], 0, 0, 0);
        }
      }
  }
  float* out = a.part + (int64_t)slice * a.n_in * a.n_out;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = n0 + wn * WN + ni * 32 + l31;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = i0 + wm * WM + mi * 32 + (q & 3) + 8 * (q >> 2) + 4 * hi;
        if (i < a.n_in && n < a.n_out) out[(int64_t)i * a.n_out + n] = acc[mi][ni][q];
      }
    }
}

// Fixed-order slab sums: out[i] += sum_s part[s][i]. Many slabs are first folded in groups of
// kFold (more parallelism, same order every run), then the group sums are added.
constexpr int kFold = 16;

// E_OUT over ncb column blocks (out_features > 64): terms[r] = sum_cb terms[cb * R + r], fixed order
__global__ void terms_sum_kernel(float4* __restrict__ terms, int ncb, int64_t R) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  float4 t = terms[r];
  for (int cb = 1; cb < ncb; ++cb) {
    const float4 u = terms[(int64_t)cb * R + r];
    t.x += u.x; t.y += u.y; t.z += u.z;
  }
  terms[r] = t;
}

__global__ void fold_slabs_kernel(const float* __restrict__ part, int S, int64_t n, float* __restrict__ out2) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const int s0 = blockIdx.y * kFold, s1 = s0 + kFold < S ? s0 + kFold : S;
  float s = 0.f;
  for (int k = s0; k < s1; ++k) s += part[(int64_t)k * n + i];
  out2[(int64_t)blockIdx.y * n + i] = s;
}

__global__ void sum_slabs_kernel(const float* __restrict__ part, int S, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += part[(int64_t)k * n + i];
  out[i] += s;
}

// ---- B-resident row GEMMs and LDS-free weight gradients (W x W layers) -------------------
// Measured limit of fgemm / fwgrad above (r02-r03 SQ passes): two barriers per 32-k tile with the
// operand staging between them; the co-resident workgroup does not reliably cover that phase, so the
// big GEMMs held the fp32 MFMA pipe at ~0.6-0.7. These two kernels have no barrier in the main loop:
//
// rgemm: one persistent 8-wave workgroup per CU owns 128 output columns for its whole life; their B
//   slice (the whole K x 128 weight block, K <= 256: <= 129 KB) is staged into LDS ONCE. Each wave
//   computes a 32-row x 64-column tile (1 x 2 v_mfma_f32_32x32x2_f32 tiles per stream, S streams) of
//   row blocks of 128 rows; its A operand never touches LDS: lane (m = lane & 31, h = lane >> 5) owns
//   row m and, within each 32-k tile, the 16 k's [16h, 16h + 16) (the MFMA k slot of a lane is any
//   bijection shared by A and B), so it loads its 16 A values per plane as four 16-byte loads one tile
//   ahead (register double buffer) and applies the prologue transform in registers; layer-1 modes
//   rebuild A from the row's x / v | abar0 (registers) and K1^T (LDS, broadcast per half-wave).
// wgrad2: C[i][n] = sum_r sum_p A_p[r][i] B_p[r][n]: the sample rows are the MFMA reduction dimension
//   (lane (l = lane & 31, h) takes row 2s + h of step s), so every operand is one coalesced 128-byte
//   row segment per half-wave, loaded straight into registers one step ahead — no LDS, no barrier. One
//   8-wave workgroup per CU covers the whole [n_in x n_out] output for its slice of rows (waves 4 x 2,
//   each 32 MI x 32 NI); the repeat reads of a row's planes by the other waves hit the CU's L1.
constexpr int kRT = 512;            // 8 waves
constexpr int kRBN = 128;          // block columns (B slice resident in LDS)
constexpr int kRGridCap = 256;      // one workgroup per CU (LDS-bound)

template <int AM>
constexpr int rg_planes() {
  return (AM == A_FWD || AM == A_S3) ? 3
         : ((AM == A_S1MUL || AM == A_FWD2 || AM == A_S2) ? 2 : ((AM == A_U || AM == A_RAW1) ? 1 : 0));
}

bool rgemm_shape(int K, int N) { return K % 64 == 0 && K <= 256 && N % kRBN == 0; }

// V (schedule variant, A/B): 0 = Bt b128 reads, compiler schedule; 1 = + one fenced region per tile
// (prefetch one tile ahead); 2 = + loads / layer-1 VALU interleaved one per MFMA; 3 = Bs[k][n] with one
// ds_read_b32 per k-step and column tile, compiler schedule.
// BNC = block columns: 128 for the W x W layers; 64 for the output layer (N = out_features <= 64, one
// column block, columns past N zero in the staged B and never stored; E_OUT reduces a row's outputs
// inside one wave, E_SEEDS writes the seeds and the bias-gradient column sums).
template <int S, int NI, int AM, int BMD, int EM, int D = 0, int BNC = kRBN, int NW = 8>
__global__ __launch_bounds__(NW * 64, 1) void rgemm(GemmArgs a) {
  constexpr int NT = NW * 64;                                            // threads (NW waves)
  constexpr int WGN = BNC / (32 * NI), WGM = NW / WGN, BMR = 32 * WGM;  // waves along N / M, block rows
  static_assert((NI == 2 || NI == 4) && WGN >= 1 && WGN * WGM == NW, "rgemm wave grid");
  static_assert((EM != E_OUT && EM != E_OUT_SEEDS1) || WGN == 1, "E_OUT reduces each row inside one wave");
  constexpr bool L1 = a_is_l1<AM>();
  constexpr int NV = rg_planes<AM>();
  constexpr int SK = L1 ? k1_stride<D>() : 1;
  constexpr int NP = (EM == E_ACT_BWD || EM == E_SEEDS || EM == E_OUT_SEEDS1) ? 1 : 0;
  static_assert(!L1 || D > 0, "layer-1 modes need D");
  static_assert(EM == E_ACT_FWD || EM == E_STORE || EM == E_STORE3 || EM == E_ACT_BWD || EM == E_OUT ||
                    EM == E_SEEDS || EM == E_OUT_SEEDS1, "rgemm epilogues");
  static_assert(EM != E_OUT_SEEDS1 || S == 2, "the first-order output epilogue takes the h and z' streams");
  extern __shared__ float lds[];
  const int Kp = a.K + 4;                          // Bt row pitch: ds_read_b128 of 16 lanes' rows conflict-free
  float* Bt = lds;                                 // [BNC][Kp]: Bt[n][k] = B[k][n0 + n]
  [[maybe_unused]] float* k1s = Bt + (size_t)BNC * Kp;  // L1: [K][SK]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, l31 = lane & 31, hi = lane >> 5;
  const int K = a.K, N = a.N;
  const int ncb = (N + BNC - 1) / BNC;
  const int lid = xcd_linear(blockIdx.x, gridDim.x);  // the column blocks of a row stream adjacent: same XCD
  const int cb = lid % ncb, rs = lid / ncb, nrs = gridDim.x / ncb;
  const int n0 = cb * BNC;
  for (int e = tid; e < K * BNC; e += NT) {
    int k, n;
    float v;
    if constexpr (BMD == B_NN) {
      k = e / BNC;
      n = e - k * BNC;
      v = n0 + n < N ? a.Bw[(size_t)k * N + n0 + n] : 0.f;
    } else {
      n = e / K;
      k = e - n * K;
      v = n0 + n < N ? a.Bw[(size_t)(n0 + n) * K + k] : 0.f;
    }
    Bt[n * Kp + k] = v;
  }
  if constexpr (L1) {
    for (int e = tid; e < K * SK; e += NT) {
      const int k = e / SK, i = e - k * SK;
      k1s[e] = i < D ? a.k1[i * K + k] : (i == D ? a.b1[k] : 0.f);
    }
  }
  __syncthreads();
  [[maybe_unused]] float pacc[NI] = {};
  const int nk = K / 32;  // even: K % 64 == 0 (rgemm_shape)
  // The row-block loop is software-pipelined too: the last tile of a row block prefetches tile 0 (and,
  // layer-1 modes, the x / v | abar0 row) of the NEXT row block, so the epilogue and the next block's
  // first tile never wait on HBM.
  auto row_of = [&](int mb_) { return std::min<int64_t>((int64_t)mb_ * BMR + wm * 32 + l31, a.R - 1); };
  const float* pl[3] = {a.pa0, a.pa1, a.pa2};
  auto load_tile = [&](float (&t)[NV > 0 ? NV : 1][16], int kt, int64_t row) {
#pragma unroll
    for (int p = 0; p < NV; ++p) {
      const f32x4* src = reinterpret_cast<const f32x4*>(pl[p] + row * K + kt * 32 + 16 * hi);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = src[j];
        t[p][4 * j] = v[0]; t[p][4 * j + 1] = v[1]; t[p][4 * j + 2] = v[2]; t[p][4 * j + 3] = v[3];
      }
    }
  };
  [[maybe_unused]] float rx[L1 ? D : 1], ry[L1 ? D : 1], rxn[L1 ? D : 1], ryn[L1 ? D : 1];
  auto load_row = [&](float* x, float* y, int64_t row) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      x[i] = a.xz[row * a.ldxz + i];
      y[i] = AM == A_L1F ? a.xz[row * a.ldxz + D + i] : a.ab0[row * D + i];
    }
  };
  float t0[NV > 0 ? NV : 1][16], t1[NV > 0 ? NV : 1][16];
  if (rs < a.n_mblocks) {
    if constexpr (NV > 0) load_tile(t0, 0, row_of(rs));
    if constexpr (L1) load_row(rx, ry, row_of(rs));
  }
  for (int mb = rs; mb < a.n_mblocks; mb += nrs) {
    const int r0 = mb * BMR;
    const int64_t mr = row_of(mb);  // clamped row (stores are guarded)
    const int64_t mrn = mb + nrs < a.n_mblocks ? row_of(mb + nrs) : mr;
    // layer-1 modes: the B operand of the pre-activation MFMAs, [x, 1, 0] / y by c-pairs (half h: c = 2 j + h)
    [[maybe_unused]] float xsel[L1 ? (D + 2) / 2 : 1], ysel[L1 ? D / 2 : 1];
    if constexpr (L1) {
#pragma unroll
      for (int j = 0; j < (D + 2) / 2; ++j) {
        const float x0 = 2 * j < D ? rx[2 * j] : 1.f, x1 = 2 * j + 1 < D ? rx[2 * j + 1] : 0.f;
        xsel[j] = hi ? x1 : x0;
        if (j < D / 2) ysel[j] = hi ? ry[2 * j + 1] : ry[2 * j];
      }
      load_row(rxn, ryn, mrn);
    }
    f32x16 acc[S][NI];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[s][ni][q] = 0.f;
    auto steps = [&](const float (&t)[NV > 0 ? NV : 1][16], int kt) {
      float bt[NI][16];  // the lane's 16 k's of each B column: 4 ds_read_b128 per column tile
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // plane modes: the lane's k's are [16 hi, 16 hi + 16); layer-1 modes: the 32x32 MFMA result rows
          // (j & 3) + 8 (j >> 2) + 4 hi, i.e. 16-byte runs at 4 hi + 8 j
          const int ko = L1 ? 4 * hi + 8 * j : 16 * hi + 4 * j;
          const f32x4 v = *reinterpret_cast<const f32x4*>(Bt + (wn * 32 * NI + ni * 32 + l31) * Kp + kt * 32 + ko);
          bt[ni][4 * j] = v[0]; bt[ni][4 * j + 1] = v[1]; bt[ni][4 * j + 2] = v[2]; bt[ni][4 * j + 3] = v[3];
        }
      // layer-1 modes: the pre-activations of the lane's row for the tile's 32 k on the matrix pipe,
      //   Z^T[k][m] = sum_c [K1; b1][c][k] [x_m; 1][c],  Zy^T[k][m] = sum_c K1[c][k] y_m[c]
      // (A = the K1^T row of k = lane & 31 from LDS, B = the lane's own row): the 32x32 result leaves lane
      // (m, h) with k = (q & 3) + 8 (q >> 2) + 4 h for q < 16 — the lane's 16 A values of the tile, which
      // is why the B reads above use that k order. 5 + 4 MFMAs (d = 8) replace ~20 VALU per A value:
      // VALU in this kernel is not hidden under the MFMA pipe (profiles/r03_mfma_probe.txt).
      [[maybe_unused]] float at[L1 ? S : 1][L1 ? 16 : 1];
      if constexpr (L1) {
        constexpr int NZ = (D + 2) / 2;  // c-pairs of [x, 1]
        float kc[SK];
#pragma unroll
        for (int j = 0; j < SK / 4; ++j) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(k1s + (kt * 32 + l31) * SK + 4 * j);
          kc[4 * j] = v[0]; kc[4 * j + 1] = v[1]; kc[4 * j + 2] = v[2]; kc[4 * j + 3] = v[3];
        }
        f32x16 zt = {}, yt = {};
#pragma unroll
        for (int j = 0; j < NZ; ++j) {
          const float ka = hi ? (2 * j + 1 < SK ? kc[2 * j + 1] : 0.f) : kc[2 * j];
          zt = __builtin_amdgcn_mfma_f32_32x32x2f32(ka, xsel[j], zt, 0, 0, 0);
          if (j < D / 2) yt = __builtin_amdgcn_mfma_f32_32x32x2f32(ka, ysel[j], yt, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const float z = zt[q], zy = yt[q];
          const float h = ftanh(z), s1 = 1.f - h * h;
          if constexpr (AM == A_L1F) {
            at[0][q] = h;
            at[1][q] = s1 * zy;
            if constexpr (S > 2) at[S - 1][q] = -2.f * h * s1 * zy * zy;
          } else {
            at[0][q] = s1 * zy;
          }
        }
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        float av[3];
        if constexpr (L1) {
#pragma unroll
          for (int si = 0; si < S; ++si) av[si] = at[si][s];
        } else if constexpr (AM == A_FWD) {
          const float h = t[0][s], zd = t[1][s], zdd = t[2][s];
          const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
          av[0] = h;
          av[1] = s1 * zd;
          av[2] = fmaf(s1, zdd, s2 * zd * zd);
        } else if constexpr (AM == A_S1MUL) {
          const float h = t[0][s];
          av[0] = (1.f - h * h) * t[1][s];
        } else if constexpr (AM == A_U) {
          av[0] = 2.f * t[0][s];
        } else if constexpr (AM == A_RAW1) {
          av[0] = t[0][s];
        } else if constexpr (AM == A_FWD2) {
          const float h = t[0][s];
          av[0] = h;
          av[1] = (1.f - h * h) * t[1][s];
        } else if constexpr (AM == A_S2) {
          av[0] = t[0][s];
          av[1] = t[1][s];
        } else {  // A_S3
          av[0] = t[0][s];
          av[1] = t[1][s];
          av[2] = t[2][s];
        }
#pragma unroll
        for (int si = 0; si < S; ++si)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[si][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[si], bt[ni][s], acc[si][ni], 0, 0, 0);
      }
    };
    // Register double buffer, loads UNCONDITIONAL (the last prefetch re-reads tile 0 and is dropped): a
    // load under a branch makes the waitcnt pass merge the two paths and wait for the just-issued
    // prefetch before the current tile's MFMAs (measured: vmcnt(2) instead of vmcnt(12) in wgrad2).
    // One scheduling region per tile (sched_barrier around it): the B reads, the NEXT tile's A loads and
    // this tile's MFMAs. Without the region fence the machine scheduler sank each prefetch next to its first
    // use (vmcnt(0) before every k-step) to save registers; spreading the loads one per MFMA inside the region
    // (sched_group_barrier) measured slower (profiles/r03_c5_sched_ab.txt).
    auto tile = [&](const float (&tc)[NV > 0 ? NV : 1][16], float (&tn)[NV > 0 ? NV : 1][16], int kt, int ktn,
                    int64_t rown) {
      if constexpr (NV > 0) load_tile(tn, ktn, rown);
      steps(tc, kt);
      __builtin_amdgcn_sched_barrier(0);
    };
    __builtin_amdgcn_sched_barrier(0);
    for (int kt = 0; kt < nk; kt += 2) {  // t0 holds tile kt on entry (the last pair fetches the next block's tile 0)
      tile(t0, t1, kt, kt + 1, mr);
      tile(t1, t0, kt + 1, kt + 2 < nk ? kt + 2 : 0, kt + 2 < nk ? mr : mrn);
    }
    // ---- epilogue: acc register q of tile ni is C[row][col], row = (q & 3) + 8 (q >> 2) + 4 hi, col = l31
    const bool full = r0 + BMR <= a.R;
    auto epilogue = [&](auto check) {
      constexpr bool CHECK = decltype(check)::value;
      [[maybe_unused]] float t0[16], t1[16], t2[16];  // E_OUT: the row's sum y^2, y y', y'^2 + y y''
      if constexpr (EM == E_OUT || EM == E_OUT_SEEDS1) {
#pragma unroll
        for (int q = 0; q < 16; ++q) t0[q] = t1[q] = t2[q] = 0.f;
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int n = n0 + wn * 32 * NI + ni * 32 + l31;
        const bool nv = BNC == kRBN || n < N;  // output-layer blocks: columns past N are padding
        [[maybe_unused]] float bn = 0.f;
        if constexpr (EM == E_ACT_FWD || EM == E_OUT || EM == E_OUT_SEEDS1) bn = a.bias[nv ? n : 0];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int r = r0 + wm * 32 + (q & 3) + 8 * (q >> 2) + 4 * hi;
          const bool ok = (!CHECK || r < a.R) && nv;
          const uint32_t o = (uint32_t)(r * N + n);
          if constexpr (EM == E_ACT_FWD) {
            if (ok) {
              sto(a.po0, o, ftanh(acc[0][ni][q] + bn));
              sto(a.po1, o, acc[1][ni][q]);
              if constexpr (S > 2) sto(a.po2, o, acc[S - 1][ni][q]);
            }
          } else if constexpr (EM == E_STORE) {
            if (ok) sto(a.po0, o, acc[0][ni][q]);
          } else if constexpr (EM == E_STORE3) {  // hbar1 (R2b), read once by l1_grad_kernel
            if (ok) {
              sto_h(a.po0, o, acc[0][ni][q]);
              sto_h(a.po1, o, acc[1][ni][q]);
              if constexpr (S > 2) sto_h(a.po2, o, acc[S - 1][ni][q]);
            }
          } else if constexpr (EM == E_OUT_SEEDS1) {
            if (ok) {
              const float y = acc[0][ni][q] + bn, yd = acc[1][ni][q];
              t0[q] = fmaf(y, y, t0[q]);
              t1[q] = fmaf(y, yd, t1[q]);
              t2[q] = fmaf(yd, yd, t2[q]);
              const float c0r = a.wrow ? a.c0 * a.wrow[(int64_t)r * a.ldw] : a.c0;
              const float yb = 2.f * a.c3 * yd + 2.f * c0r * y;
              sto(a.po0, o, yb);
              sto(a.po1, o, 2.f * a.c3 * y);
              pacc[ni] += yb;
            }
          } else if constexpr (EM == E_OUT) {
            if (ok) {
              const float y = acc[0][ni][q] + bn, yd = acc[1][ni][q], ydd = acc[2][ni][q];
              sto(a.po0, o, y);
              sto(a.po1, o, yd);
              sto(a.po2, o, ydd);
              t0[q] = fmaf(y, y, t0[q]);
              t1[q] = fmaf(y, yd, t1[q]);
              t2[q] = fmaf(yd, yd, fmaf(y, ydd, t2[q]));
            }
          } else if constexpr (EM == E_SEEDS) {
            if (ok) {
              const float ub = acc[0][ni][q];
              const float y = ldo(a.pe0, o), yd = ldo(a.pe1, o), ydd = ldo(a.pe2, o);
              const float c0r = a.wrow ? a.c0 * a.wrow[(int64_t)r * a.ldw] : a.c0;
              const float yb = 2.f * a.c3 * yd + 2.f * a.c2 * ydd + 2.f * ub + 2.f * c0r * y;
              sto(a.po0, o, yb);
              sto(a.po1, o, 2.f * a.c3 * y + 4.f * a.c2 * yd);
              sto(a.po2, o, 2.f * a.c2 * y);
              pacc[ni] += yb;
            }
          } else {  // E_ACT_BWD
            if (ok) {
              const float hb = acc[0][ni][q], hdb = acc[1][ni][q];
              const float h = ldo(a.pe0, o), zd = ldo(a.pe1, o);
              const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
              if constexpr (S > 2) {
                const float hddb = acc[S - 1][ni][q];
                const float zdd = ldo(a.pe2, o), aL = ldo(a.pe3, o), zb = ldo(a.pe4, o);
                const float s3 = -2.f * s1 * s1 - 2.f * h * s2;
                const float zbar = s1 * hb + s2 * zd * hdb + (s2 * zdd + s3 * zd * zd) * hddb + s2 * aL * zb;
                sto(a.po0, o, zbar);
                sto(a.po1, o, s1 * hdb + 2.f * s2 * zd * hddb);
                sto(a.po2, o, s1 * hddb);
                pacc[ni] += zbar;
              } else {  // first-order chain: h'' bar = 0, a zetabar = 0
                const float zbar = s1 * hb + s2 * zd * hdb;
                sto(a.po0, o, zbar);
                sto(a.po1, o, s1 * hdb);
                pacc[ni] += zbar;
              }
            }
          }
        }
      }
      if constexpr (EM == E_OUT || EM == E_OUT_SEEDS1) {  // per-row reductions over the 32 lanes of each half-wave
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          float p0 = t0[q], p1 = t1[q], p2 = t2[q];
#pragma unroll
          for (int off = 16; off > 0; off >>= 1) {
            p0 += __shfl_xor(p0, off, 64);
            p1 += __shfl_xor(p1, off, 64);
            p2 += __shfl_xor(p2, off, 64);
          }
          const int r = r0 + wm * 32 + (q & 3) + 8 * (q >> 2) + 4 * hi;
          if (l31 == 0 && r < a.R) a.terms[r] = make_float4(2.f * p1, 2.f * p2, p0, 0.f);
        }
      }
    };
    if (full) epilogue(std::false_type{});
    else epilogue(std::true_type{});
    if constexpr (L1) {
#pragma unroll
      for (int i = 0; i < D; ++i) {
        rx[i] = rxn[i];
        ry[i] = ryn[i];
      }
    }
  }
  if constexpr (NP > 0) {  // bias-gradient column sums: one slab row per row stream
    __syncthreads();
    float* red = lds;  // [WGM][BNC] (Bt is dead)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const float v = pacc[ni] + __shfl_xor(pacc[ni], 32, 64);
      if (hi == 0) red[wm * BNC + wn * 32 * NI + ni * 32 + l31] = v;
    }
    __syncthreads();
    for (int c = tid; c < BNC; c += NT) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WGM; ++w) t += red[w * BNC + c];
      if (n0 + c < N) a.part[(int64_t)rs * N + n0 + c] = t;
    }
  }
}

// NPR = 2 (first-order chunks, GB_PL): only the pairs (h, zbar) and (s1 z', z'bar); the z'' and adjoint pairs are
// zero there, so their planes (and, GA_L1, abar0) are not read.
// rgemm16: the output layer (K = W <= 256, N = out_features <= 48) on v_mfma_f32_16x16x4_f32 — 16-column tiles, so
// 40 outputs take 48 MFMA columns instead of rgemm's 64 (the product was MFMA-bound on that padding). Same B-resident
// scheme as rgemm (the K x 48 slice of Ko in LDS once per workgroup, Bt[n][k], pitch K + 4), 8 waves of 32 rows x 48
// columns (2 M-tiles of 16 rows x 3 N-tiles), row blocks of 256. Lane (m = lane & 15, q = lane >> 4) owns rows
// m and m + 16 of its wave and, within each 32-k tile, the 8 k's [8q, 8q + 8) (the MFMA k-slot bijection is shared
// with B): two 16-byte loads per row and plane, one tile ahead. The C/D fragment leaves lane (n, q) with rows
// 4q + i (i < 4, register i) of column n; the per-row reductions of E_OUT / E_OUT_SEEDS1 run over the 16 lanes
// of a q-group.
template <int S, int AM, int EM>
__global__ __launch_bounds__(kRT, 1) void rgemm16(GemmArgs a) {
  constexpr int NT = 3, BNC = 16 * NT, MI = 2, NW = kRT / 64, BMR = 32 * NW;
  constexpr int NV = rg_planes<AM>();
  static_assert(EM == E_OUT || EM == E_SEEDS || EM == E_OUT_SEEDS1, "rgemm16: output-layer epilogues");
  static_assert(NV >= 1 && !a_is_l1<AM>(), "rgemm16: plane operands");
  constexpr int NP = (EM == E_SEEDS || EM == E_OUT_SEEDS1) ? 1 : 0;
  extern __shared__ float lds[];
  // Bt[n][k] at pitch K + 16 with the 16-byte chunks of each 32-k tile XOR-swizzled by n & 7: the 16-lane groups of a
  // ds_read_b128 (lanes {0-3, 12-15, 20-27} / {4-11, 16-19, 28-31}) then hit 64 distinct banks (the bank model of
  // tools/quad_gram_bank_model.py's rules: 8 read cycles per two k-halves instead of 16 at pitch K + 4)
  const int K = a.K, N = a.N, Kp = K + 16;
  float* Bt = lds;  // [BNC][Kp]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, qg = lane >> 4;
  for (int e = tid; e < K * BNC; e += kRT) {
    const int k = e / BNC, n = e - k * BNC;
    const int ks = (k & ~31) | ((((k >> 2) & 7) ^ (n & 7)) << 2) | (k & 3);
    Bt[n * Kp + ks] = n < N ? a.Bw[(size_t)k * N + n] : 0.f;
  }
  __syncthreads();
  const int rs = xcd_linear(blockIdx.x, gridDim.x), nrs = gridDim.x;
  [[maybe_unused]] float pacc[NT] = {};
  const int nk = K / 32;
  auto row_of = [&](int mb_, int mi) {
    return std::min<int64_t>((int64_t)mb_ * BMR + wave * 32 + mi * 16 + l16, a.R - 1);
  };
  const float* pl[3] = {a.pa0, a.pa1, a.pa2};
  auto load_tile = [&](float (&t)[NV][MI][8], int kt, int mb_) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int64_t row = row_of(mb_, mi);
#pragma unroll
      for (int p = 0; p < NV; ++p) {
        const f32x4* src = reinterpret_cast<const f32x4*>(pl[p] + row * K + kt * 32 + 8 * qg);
        const f32x4 v0 = src[0], v1 = src[1];
        t[p][mi][0] = v0[0]; t[p][mi][1] = v0[1]; t[p][mi][2] = v0[2]; t[p][mi][3] = v0[3];
        t[p][mi][4] = v1[0]; t[p][mi][5] = v1[1]; t[p][mi][6] = v1[2]; t[p][mi][7] = v1[3];
      }
    }
  };
  float t0[NV][MI][8], t1[NV][MI][8];
  if (rs < a.n_mblocks) load_tile(t0, 0, rs);
  for (int mb = rs; mb < a.n_mblocks; mb += nrs) {
    const int r0 = mb * BMR;
    const int mbn = mb + nrs < a.n_mblocks ? mb + nrs : mb;
    f32x4 acc[S][MI][NT];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[s][mi][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto steps = [&](const float (&t)[NV][MI][8], int kt) {
      float bt[NT][8];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(Bt + (nt * 16 + l16) * Kp + kt * 32 +
                                                          4 * ((2 * qg + h) ^ (l16 & 7)));
          bt[nt][4 * h] = v[0]; bt[nt][4 * h + 1] = v[1]; bt[nt][4 * h + 2] = v[2]; bt[nt][4 * h + 3] = v[3];
        }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float av[MI][3];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
          if constexpr (AM == A_FWD) {
            const float h = t[0][mi][j], zd = t[1][mi][j], zdd = t[2][mi][j];
            const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
            av[mi][0] = h;
            av[mi][1] = s1 * zd;
            av[mi][2] = fmaf(s1, zdd, s2 * zd * zd);
          } else if constexpr (AM == A_FWD2) {
            const float h = t[0][mi][j];
            av[mi][0] = h;
            av[mi][1] = (1.f - h * h) * t[1][mi][j];
          } else {  // A_S1MUL
            const float h = t[0][mi][j];
            av[mi][0] = (1.f - h * h) * t[1][mi][j];
          }
        }
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
              acc[s][mi][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mi][s], bt[nt][j], acc[s][mi][nt], 0, 0, 0);
      }
    };
    // register double buffer, loads unconditional (the last prefetch reads the next block's tile 0), one fenced
    // scheduling region per tile (rgemm's V = 1 schedule)
    __builtin_amdgcn_sched_barrier(0);
    for (int kt = 0; kt < nk; kt += 2) {
      load_tile(t1, kt + 1, mb);
      steps(t0, kt);
      __builtin_amdgcn_sched_barrier(0);
      load_tile(t0, kt + 2 < nk ? kt + 2 : 0, kt + 2 < nk ? mb : mbn);
      steps(t1, kt + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue: acc[s][mi][nt][i] = C[row = 16 mi + 4 q + i][col = 16 nt + n] of the wave's 32 rows
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      [[maybe_unused]] float tr0[4] = {}, tr1[4] = {}, tr2[4] = {};
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = nt * 16 + l16;
        const bool nv = n < N;
        [[maybe_unused]] float bn = 0.f;
        if constexpr (EM == E_OUT || EM == E_OUT_SEEDS1) bn = a.bias[nv ? n : 0];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = r0 + wave * 32 + mi * 16 + 4 * qg + i;
          const bool ok = r < a.R && nv;
          const uint32_t o = (uint32_t)(r * N + n);
          if constexpr (EM == E_OUT) {
            if (ok) {
              const float y = acc[0][mi][nt][i] + bn, yd = acc[1][mi][nt][i], ydd = acc[2][mi][nt][i];
              sto(a.po0, o, y);
              sto(a.po1, o, yd);
              sto(a.po2, o, ydd);
              tr0[i] = fmaf(y, y, tr0[i]);
              tr1[i] = fmaf(y, yd, tr1[i]);
              tr2[i] = fmaf(yd, yd, fmaf(y, ydd, tr2[i]));
            }
          } else if constexpr (EM == E_OUT_SEEDS1) {
            if (ok) {
              const float y = acc[0][mi][nt][i] + bn, yd = acc[1][mi][nt][i];
              tr0[i] = fmaf(y, y, tr0[i]);
              tr1[i] = fmaf(y, yd, tr1[i]);
              tr2[i] = fmaf(yd, yd, tr2[i]);
              const float c0r = a.wrow ? a.c0 * a.wrow[(int64_t)r * a.ldw] : a.c0;
              const float yb = 2.f * a.c3 * yd + 2.f * c0r * y;
              sto(a.po0, o, yb);
              sto(a.po1, o, 2.f * a.c3 * y);
              pacc[nt] += yb;
            }
          } else {  // E_SEEDS
            if (ok) {
              const float ub = acc[0][mi][nt][i];
              const float y = ldo(a.pe0, o), yd = ldo(a.pe1, o), ydd = ldo(a.pe2, o);
              const float c0r = a.wrow ? a.c0 * a.wrow[(int64_t)r * a.ldw] : a.c0;
              const float yb = 2.f * a.c3 * yd + 2.f * a.c2 * ydd + 2.f * ub + 2.f * c0r * y;
              sto(a.po0, o, yb);
              sto(a.po1, o, 2.f * a.c3 * y + 4.f * a.c2 * yd);
              sto(a.po2, o, 2.f * a.c2 * y);
              pacc[nt] += yb;
            }
          }
        }
      }
      if constexpr (EM == E_OUT || EM == E_OUT_SEEDS1) {  // per-row sums over the 16 lanes of the q-group
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float p0 = tr0[i], p1 = tr1[i], p2 = tr2[i];
#pragma unroll
          for (int off = 8; off > 0; off >>= 1) {
            p0 += __shfl_xor(p0, off, 64);
            p1 += __shfl_xor(p1, off, 64);
            p2 += __shfl_xor(p2, off, 64);
          }
          const int r = r0 + wave * 32 + mi * 16 + 4 * qg + i;
          if (l16 == 0 && r < a.R) a.terms[r] = make_float4(2.f * p1, 2.f * p2, p0, 0.f);
        }
      }
    }
  }
  if constexpr (NP > 0) {  // bias-gradient column sums: one slab row per row stream (fixed order)
    __syncthreads();
    float* red = lds;  // [NW][BNC] (Bt is dead)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float v = pacc[nt];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (qg == 0) red[wave * BNC + nt * 16 + l16] = v;
    }
    __syncthreads();
    for (int c = tid; c < BNC; c += kRT) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += red[w * BNC + c];
      if (c < N) a.part[(int64_t)rs * N + c] = t;
    }
  }
}

template <int MI, int NI, int GA, int GB, int D = 0, int NPR = 4>
__global__ __launch_bounds__(kRT, 1) void wgrad2(WgradArgs a) {
  static_assert(GA != GA_L1 || D > 0, "GA_L1 needs D");
  static_assert(GA != GA_RAW4, "wgrad2: A streams from planes (GA_PL) or rows (GA_L1)");
  static_assert(NPR == 4 || (NPR == 2 && GB == GB_PL), "wgrad2: 4 stream pairs, or 2 on the first-order chain");
  constexpr int NVA = GA == GA_PL ? NPR : 0;                 // raw A planes per feature group
  constexpr int NVB = NPR == 2 ? 2 : (GB == GB_PL ? 5 : 4);  // raw B planes per column group
  constexpr int NX = GA == GA_L1 ? (NPR == 2 ? 2 : 3) * D : 1;  // the row's [x | v (| abar0)]
  // GA_L1: a step's two rows [x | v (| abar0)] come in as NXE floats per lane (element lane + 64 j of the 2 x NXP
  // slab) and go through a wave-private LDS slab, read back by broadcast: one load per lane instead of NX per lane
  constexpr int NXP = (NX + 3) & ~3, NXE = GA == GA_L1 ? (2 * NXP + 63) / 64 : 1;
  __shared__ float xsl[GA == GA_L1 ? 8 * 2 * NXP : 1];  // [wave][2][NXP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, l31 = lane & 31, hi = lane >> 5;
  const int slice = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t rs0 = (int64_t)slice * a.rows_per_slice;
  const int64_t rs1 = std::min<int64_t>(rs0 + a.rows_per_slice, a.R);
  const int i0 = wm * 32 * MI, nb0 = wn * 32 * NI;
  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[mi][ni][q] = 0.f;
  [[maybe_unused]] float kc[GA == GA_L1 ? MI : 1][GA == GA_L1 ? D + 1 : 1];
  if constexpr (GA == GA_L1) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int i = i0 + mi * 32 + l31;
#pragma unroll
      for (int q = 0; q < D; ++q) kc[mi][q] = a.k1[q * a.n_in + i];
      kc[mi][D] = a.b1[i];
    }
  }
  struct Regs {
    float ra[NVA > 0 ? MI : 1][NVA > 0 ? NVA : 1];
    float rb[NI][NVB];
    float x[NXE];
  };
  [[maybe_unused]] float* xw = xsl + (GA == GA_L1 ? wave * 2 * NXP : 0);
  const float* pa[4] = {a.pa0, a.pa1, a.pa2, a.pa3};
  const float* pb[5] = {a.pb0, a.pb1, a.pb2, a.pb3, a.pb4};
  auto load = [&](Regs& g, int64_t rb0) {
    const int64_t r = std::min<int64_t>(rb0 + hi, a.R - 1);
#pragma unroll
    for (int mi = 0; mi < (NVA > 0 ? MI : 0); ++mi)
#pragma unroll
      for (int p = 0; p < NVA; ++p) g.ra[mi][p] = ldo(pa[p], (uint32_t)(r * a.n_in + i0 + mi * 32 + l31));
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int p = 0; p < NVB; ++p) g.rb[ni][p] = ldo(pb[p], (uint32_t)(r * a.n_out + nb0 + ni * 32 + l31));
    if constexpr (GA == GA_L1) {  // element e = lane + 64 j: row rb0 + e / NXP, column e % NXP (clamped, dropped)
#pragma unroll
      for (int j = 0; j < NXE; ++j) {
        const int e = lane + 64 * j, h = e / NXP < 2 ? e / NXP : 1, c = e - (e / NXP) * NXP;
        const int cc = c < NX ? c : NX - 1;
        const int64_t rr = std::min<int64_t>(rb0 + h, a.R - 1);
        g.x[j] = cc < 2 * D ? a.xz[rr * a.ldxz + cc] : a.ab0[rr * D + (cc - 2 * D)];
      }
    }
  };
  auto step = [&](const Regs& g, int64_t rb0) {
    const bool ok = rb0 + hi < rs1;
    float av[MI][4], bv[NI][4];
    [[maybe_unused]] float xv[GA == GA_L1 ? NXP : 1];
    if constexpr (GA == GA_L1) {  // through the wave's slab (LDS ops of one wave complete in order)
      __builtin_amdgcn_wave_barrier();  // the previous step's cross-lane reads of the slab stay before these stores
#pragma unroll
      for (int j = 0; j < NXE; ++j) {
        const int e = lane + 64 * j;
        if (e < 2 * NXP) xw[e] = g.x[j];
      }
      __builtin_amdgcn_wave_barrier();  // and these stores before the cross-lane reads below
#pragma unroll
      for (int j = 0; j < NXP / 4; ++j) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(xw + hi * NXP + 4 * j);
        xv[4 * j] = v[0]; xv[4 * j + 1] = v[1]; xv[4 * j + 2] = v[2]; xv[4 * j + 3] = v[3];
      }
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      if constexpr (GA == GA_L1) {
        const float z = kc[mi][D] + dotd<D>(xv, kc[mi]), zd = dotd<D>(xv + D, kc[mi]);
        const float h = ftanh(z), s1 = 1.f - h * h;
        av[mi][0] = h;
        av[mi][1] = s1 * zd;
        if constexpr (NPR > 2) {
          const float zb = dotd<D>(xv + 2 * D, kc[mi]);
          av[mi][2] = -2.f * h * s1 * zd * zd;
          av[mi][3] = s1 * zb;
        }
      } else {
        const float h = g.ra[mi][0], zd = g.ra[mi][1];
        const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
        av[mi][0] = h;
        av[mi][1] = s1 * zd;
        if constexpr (NPR > 2) {
          const float zdd = g.ra[mi][2], zeb = g.ra[mi][3];
          av[mi][2] = fmaf(s1, zdd, s2 * zd * zd);
          av[mi][3] = s1 * zeb;
        }
      }
#pragma unroll
      for (int p = 0; p < NPR; ++p) av[mi][p] = ok ? av[mi][p] : 0.f;  // rows past the slice add nothing
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      bv[ni][0] = g.rb[ni][0];
      bv[ni][1] = g.rb[ni][1];
      if constexpr (NPR > 2) {
        bv[ni][2] = g.rb[ni][2];
        if constexpr (GB == GB_PL) {
          const float h = g.rb[ni][3];
          bv[ni][3] = (1.f - h * h) * g.rb[ni][NVB - 1];
        } else {
          bv[ni][3] = 2.f * g.rb[ni][3];
        }
      }
    }
#pragma unroll
    for (int p = 0; p < NPR; ++p)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi][p], bv[ni][p], acc[mi][ni], 0, 0, 0);
  };
  // Two steps of 2 rows per iteration (register double buffer). Loads and steps are UNCONDITIONAL
  // (clamped rows; the ok mask zeroes rows past the slice): a load under a branch makes the waitcnt
  // pass merge both paths and wait for the just-issued prefetch (vmcnt(2)) before the MFMAs.
  // One scheduling region per step (sched_barrier on both sides of the step): the next step's loads stay ahead of
  // this step's MFMAs.
  auto region = [&](const Regs& gc, Regs& gn, int64_t rc, int64_t rn) {
    load(gn, rn);
    __builtin_amdgcn_sched_barrier(0);
    step(gc, rc);
    __builtin_amdgcn_sched_barrier(0);
  };
  Regs g0, g1;
  load(g0, rs0);
  __builtin_amdgcn_sched_barrier(0);
  for (int64_t rb = rs0; rb < rs1; rb += 4) {
    region(g0, g1, rb, rb + 2);
    region(g1, g0, rb + 2, rb + 4);
  }
  float* out = a.part + (int64_t)slice * a.n_in * a.n_out;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = nb0 + ni * 32 + l31;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = i0 + mi * 32 + (q & 3) + 8 * (q >> 2) + 4 * hi;
        out[(int64_t)i * a.n_out + n] = acc[mi][ni][q];
      }
    }
}

// wgrad_o: the output-layer weight gradient dKo[i][o] = sum_r sum_p A_p[r][i] B_p[r][o] (A = the last
// hidden layer's [h, s1 z', s1 z'' + s2 z'^2, s1 zetabar], B = [ybar0..2, 2 y], o < out_features <= 64)
// on v_mfma_f32_16x16x4_f32: 16-wide output tiles pad 40 outputs to 48 (32-wide tiles: 64), and the four
// sample rows of a k-step sit in the lane's 16-lane group (lane (c, g): row 4 s + g, column c), so every
// operand is a 64-byte row segment per lane group, loaded straight into registers one step ahead — no
// LDS, no barrier (the staged fwgrad kernel it replaces ran 2 barriers per 16 rows at 8 waves per CU).
// One wave per 64 hidden features (4 tiles) x all output tiles; workgroups = row slices.
// NPR = 2 (first-order chunks): only the pairs (h, ybar0) and (s1 z', ybar1) — the others are zero there.
template <int OT, int NPR = 4>
__global__ __launch_bounds__(kT) void wgrad_o(WgradArgs a) {
  static_assert(NPR == 2 || NPR == 4, "wgrad_o: 4 stream pairs, or 2 on the first-order chain");
  constexpr int FI = 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c16 = lane & 15, rq = lane >> 4;
  const int slice = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t rs0 = (int64_t)slice * a.rows_per_slice;
  const int64_t rs1 = std::min<int64_t>(rs0 + a.rows_per_slice, a.R);
  const int i0 = wave * 16 * FI;
  f32x4 acc[FI][OT];
#pragma unroll
  for (int fi = 0; fi < FI; ++fi)
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[fi][ot] = f32x4{0.f, 0.f, 0.f, 0.f};
  struct Regs {
    float a[FI][4], b[OT][4];
  };
  auto load = [&](Regs& g, int64_t rb) {  // clamped rows; columns past out_features read column 0 (dropped)
    const int64_t r = std::min<int64_t>(rb + rq, a.R - 1);
#pragma unroll
    for (int fi = 0; fi < FI; ++fi) {
      const uint32_t o = (uint32_t)(r * a.n_in + i0 + fi * 16 + c16);
      g.a[fi][0] = ldo(a.pa0, o);
      g.a[fi][1] = ldo(a.pa1, o);
      if constexpr (NPR > 2) {
        g.a[fi][2] = ldo(a.pa2, o);
        g.a[fi][3] = ldo(a.pa3, o);
      }
    }
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      const int oc = ot * 16 + c16;
      const uint32_t o = (uint32_t)(r * a.n_out + (oc < a.n_out ? oc : 0));
      g.b[ot][0] = ldo(a.pb0, o);
      g.b[ot][1] = ldo(a.pb1, o);
      if constexpr (NPR > 2) {
        g.b[ot][2] = ldo(a.pb2, o);
        g.b[ot][3] = ldo(a.pb3, o);
      }
    }
  };
  auto step = [&](const Regs& g, int64_t rb) {
    const bool ok = rb + rq < rs1;  // rows past the slice add nothing
    float av[FI][4];
#pragma unroll
    for (int fi = 0; fi < FI; ++fi) {
      const float h = g.a[fi][0], zd = g.a[fi][1];
      const float s1 = 1.f - h * h, s2 = -2.f * h * s1;
      av[fi][0] = ok ? h : 0.f;
      av[fi][1] = ok ? s1 * zd : 0.f;
      if constexpr (NPR > 2) {
        const float zdd = g.a[fi][2], zeb = g.a[fi][3];
        av[fi][2] = ok ? fmaf(s1, zdd, s2 * zd * zd) : 0.f;
        av[fi][3] = ok ? s1 * zeb : 0.f;
      }
    }
#pragma unroll
    for (int p = 0; p < NPR; ++p)
#pragma unroll
      for (int fi = 0; fi < FI; ++fi)
#pragma unroll
        for (int ot = 0; ot < OT; ++ot)
          acc[fi][ot] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[fi][p], p == 3 ? 2.f * g.b[ot][3] : g.b[ot][p],
                                                             acc[fi][ot], 0, 0, 0);
  };
  Regs g0, g1;
  load(g0, rs0);
  for (int64_t rb = rs0; rb < rs1; rb += 8) {  // loads unconditional (clamped), one step ahead
    load(g1, rb + 4);
    step(g0, rb);
    load(g0, rb + 8);
    step(g1, rb + 4);
  }
  float* out = a.part + (int64_t)slice * a.n_in * a.n_out;
#pragma unroll
  for (int fi = 0; fi < FI; ++fi)
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      const int oc = ot * 16 + c16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = i0 + fi * 16 + 4 * rq + q;
        if (oc < a.n_out) out[(int64_t)i * a.n_out + oc] = acc[fi][ot][q];
      }
    }
}

// ---- host side ------------------------------------------------------------------------
constexpr int kMaxWgradSlices = 256;
constexpr int kRowGridCap = 1024;  // workgroups per row GEMM launch (persistent over row blocks)

static int mblocks(int64_t R, int BM) { return (int)((R + BM - 1) / BM); }

static int sum_slabs(const float* part, int S, int64_t n, float* out, float* scratch, hipStream_t st) {
  const unsigned gx = (unsigned)((n + kT - 1) / kT);
  if (S > 2 * kFold) {
    const int G = (S + kFold - 1) / kFold;
    hipLaunchKernelGGL(fold_slabs_kernel, dim3(gx, G), dim3(kT), 0, st, part, S, n, scratch);
    part = scratch;
    S = G;
  }
  hipLaunchKernelGGL(sum_slabs_kernel, dim3(gx), dim3(kT), 0, st, part, S, n, out);
  return check_launch("kfp_mlp fused slab sum");
}

template <int S, int BM, int BN, int WGM, int AM, int BMD, int EM, int D = 0>
static int launch_gemm(GemmArgs a, hipStream_t st, int* grid_x_out = nullptr) {
  const size_t k1f = a_is_l1<AM>() ? (size_t)a.K * k1_stride<D>() : 0;
  const size_t bytes = ((size_t)S * BK * (BM + kPitchPad) + (size_t)BK * (BN + kPitchPad) + k1f) * sizeof(float);
  auto kern = fgemm<S, BM, BN, WGM, AM, BMD, EM, D>;
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  a.n_mblocks = mblocks(a.R, BM);
  const int gy = (a.N + BN - 1) / BN;
  const int gx = std::max(1, std::min(a.n_mblocks, kRowGridCap / gy));
  if (grid_x_out) *grid_x_out = gx;
  hipLaunchKernelGGL(kern, dim3(gx, gy), dim3(kT), bytes, st, a);
  return check_launch("kfp_mlp fused row GEMM");
}

// single-stream GEMM over N = W: full-width 256-column tiles when W allows (A built once per row)
// A_U (the R1 head a_L = (2y) Ko^T, K = out_features): 128 x 128 tiles, 4 x 1 waves — the 64 x 256 tile spilled
// (256 VGPRs + 44 B scratch); C5 1.97 -> 1.68 ms (profiles/r05_c5_g1_tile_ab.txt)
template <int AM, int BMD, int D = 0>
static int launch_gemm1(GemmArgs a, hipStream_t st) {
  if constexpr (AM == A_U) {
    if (a.N % 128 == 0) return launch_gemm<1, 128, 128, 4, AM, BMD, E_STORE, D>(a, st);
  }
  if (a.N % 256 == 0) return launch_gemm<1, 64, 256, 2, AM, BMD, E_STORE, D>(a, st);
  if (a.N > 64) return launch_gemm<1, 64, 128, 2, AM, BMD, E_STORE, D>(a, st);
  if (a.N > 32) return launch_gemm<1, 64, 64, 2, AM, BMD, E_STORE, D>(a, st);
  return launch_gemm<1, 128, 32, 4, AM, BMD, E_STORE, D>(a, st);
}

template <int BM, int BN, int GA, int GB, int D = 0>
static int launch_wgrad(WgradArgs a, float* grad_out, float* scratch, hipStream_t st) {
  const size_t xf = GA == GA_L1 ? (size_t)2 * BKG * xrow_stride<D>() : 0;
  const size_t bytes = ((size_t)4 * BKG * (BM + 4) + (size_t)4 * BKG * (BN + 4) + xf) * sizeof(float);
  auto kern = fwgrad<BM, BN, GA, GB, D>;
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  const int tiles = ((a.n_in + BM - 1) / BM) * ((a.n_out + BN - 1) / BN);
  int slices = std::max(1, std::min(kMaxWgradSlices, 1024 / tiles));
  int64_t rps = (a.R + slices - 1) / slices;
  rps = ((rps + BKG - 1) / BKG) * BKG;
  slices = (int)((a.R + rps - 1) / rps);
  a.rows_per_slice = rps;
  hipLaunchKernelGGL(kern, dim3(tiles, slices), dim3(kT), bytes, st, a);
  int rc = check_launch("kfp_mlp fused weight gradient");
  if (rc) return rc;
  return sum_slabs(a.part, slices, (int64_t)a.n_in * a.n_out, grad_out, scratch, st);
}


// S = 1 streams take 32 x 128 wave tiles (4 MFMA tiles per A value: the A prologue is the per-k VALU
// cost), S = 3 streams 32 x 64 (3 x 2 tiles, 96 accumulator registers).

template <int S, int AM, int BMD, int EM, int D, int NI, int NW>
static int launch_rgemm_t(GemmArgs a, hipStream_t st, int* grid_x_out) {
  constexpr int BMR = 32 * (NW / (kRBN / (32 * NI)));
  const size_t bytes = ((size_t)kRBN * (a.K + 4) +
                        (a_is_l1<AM>() ? (size_t)a.K * k1_stride<D>() : 0)) * sizeof(float);
  auto kern = rgemm<S, NI, AM, BMD, EM, D, kRBN, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  a.n_mblocks = mblocks(a.R, BMR);
  const int ncb = a.N / kRBN;
  const int nrs = std::max(1, std::min(a.n_mblocks, kRGridCap / ncb));
  if (grid_x_out) *grid_x_out = nrs;
  hipLaunchKernelGGL(kern, dim3(ncb * nrs), dim3(NW * 64), bytes, st, a);
  return check_launch("kfp_mlp fused B-resident row GEMM");
}

template <int S, int AM, int BMD, int EM, int D = 0>
static int launch_rgemm(GemmArgs a, hipStream_t st, int* grid_x_out = nullptr) {
  if (!rgemm_shape(a.K, a.N)) return fail(PDEINV_ERR_INVALID, "kfp_mlp rgemm: K % 64 == 0, K <= 256, N % 128 == 0");
  return launch_rgemm_t<S, AM, BMD, EM, D, (S == 1 ? 4 : 2), 8>(a, st, grid_x_out);
}

template <int MI, int NI, int GA, int GB, int D = 0, int NPR = 4>
static int launch_wgrad2(WgradArgs a, float* grad_out, float* scratch, hipStream_t st) {
  if (a.n_in != 128 * MI || a.n_out != 64 * NI) return fail(PDEINV_ERR_INVALID, "kfp_mlp wgrad2: tile / shape mismatch");
  const int slices = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxWgradSlices, (a.R + 63) / 64));
  int64_t rps = (a.R + slices - 1) / slices;
  rps = (rps + 1) & ~(int64_t)1;
  const int used = (int)((a.R + rps - 1) / rps);
  a.rows_per_slice = rps;
  auto kern = wgrad2<MI, NI, GA, GB, D, NPR>;
  hipLaunchKernelGGL(kern, dim3(used), dim3(kRT), 0, st, a);
  int rc = check_launch("kfp_mlp fused weight gradient (wgrad2)");
  if (rc) return rc;
  return sum_slabs(a.part, used, (int64_t)a.n_in * a.n_out, grad_out, scratch, st);
}

// output-layer weight gradient on wgrad_o (n_in a multiple of 64, <= 256; n_out <= 64)
template <int OT, int NPR = 4>
static int launch_wgrad_o(WgradArgs a, int64_t part_cap, float* grad_out, float* scratch, hipStream_t st) {
  const int waves = a.n_in / 64;
  if (a.n_in % 64 || waves < 1 || waves > kT / 64 || a.n_out > 16 * OT || a.n_out <= 16 * (OT - 1))
    return fail(PDEINV_ERR_INVALID, "kfp_mlp wgrad_o: shape mismatch");
  // slabs fit in part, and their kFold-group sums in part2 (part / kFold): cap a multiple of kFold
  int64_t cap = part_cap / ((int64_t)a.n_in * a.n_out);
  cap = cap >= kFold ? cap / kFold * kFold : std::max<int64_t>(1, cap);
  const int slices = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)kRowGridCap, cap, (a.R + 63) / 64}));
  int64_t rps = (a.R + slices - 1) / slices;
  rps = (rps + 7) & ~(int64_t)7;
  const int used = (int)((a.R + rps - 1) / rps);
  a.rows_per_slice = rps;
  hipLaunchKernelGGL((wgrad_o<OT, NPR>), dim3(used), dim3(64 * waves), 0, st, a);
  int rc = check_launch("kfp_mlp output-layer weight gradient (wgrad_o)");
  if (rc) return rc;
  return sum_slabs(a.part, used, (int64_t)a.n_in * a.n_out, grad_out, scratch, st);
}

// PDEINV_MLP_L1G=0: g = zeta1 K1^T on the VALU kernel (wave reductions) instead of l1_g_mfma_kernel
static bool use_l1g_mfma() {
  static const bool on = [] { const char* e = ab_env("PDEINV_MLP_L1G"); return !(e && e[0] == '0'); }();
  return on;
}

// PDEINV_MLP_WGO=0: the output-layer weight gradient on the staged fwgrad kernel (A/B measurements)
static bool use_wgo() {
  static const bool on = [] { const char* e = ab_env("PDEINV_MLP_WGO"); return !(e && e[0] == '0'); }();
  return on;
}

// B-resident row GEMMs / LDS-free weight gradients for W in {128, 256} (PDEINV_MLP_RGEMM=0: the
// staged fgemm / fwgrad kernels, for A/B measurements)
// The output layer (K = W, N = out_features <= 64) on the B-resident kernel: one 64-column block, 8 waves
// of 32 rows x 64 columns (NI = 2), row blocks of 256.
// PDEINV_MLP_OUT16=0 (A/B): the streamed output-layer products (out_features <= 48) on rgemm's 32-wide tiles instead
// of rgemm16
static bool use_out16() {
  static const bool on = [] { const char* e = ab_env("PDEINV_MLP_OUT16"); return !(e && e[0] == '0'); }();
  return on;
}

template <int S, int AM, int EM>
static int launch_rgemm16(GemmArgs a, hipStream_t st, int* grid_x_out) {
  constexpr int BNC = 48, BMR = 256;
  if (!(a.K % 64 == 0 && a.K <= 256 && a.N >= 1 && a.N <= BNC))
    return fail(PDEINV_ERR_INVALID, "kfp_mlp rgemm16 (output layer): K % 64 == 0, K <= 256, N <= 48");
  const size_t bytes = (size_t)BNC * (a.K + 16) * sizeof(float);
  auto kern = rgemm16<S, AM, EM>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  a.n_mblocks = mblocks(a.R, BMR);
  const int nrs = std::max(1, std::min(a.n_mblocks, kRGridCap));
  if (grid_x_out) *grid_x_out = nrs;
  hipLaunchKernelGGL(kern, dim3(nrs), dim3(kRT), bytes, st, a);
  return check_launch("kfp_mlp fused B-resident output-layer GEMM (16-wide)");
}

template <int S, int AM, int EM>
static int launch_rgemm_out(GemmArgs a, hipStream_t st, int* grid_x_out = nullptr) {
  // the streamed output products (S >= 2) on 16-wide tiles: C5 E_OUT 4.20 -> 3.44-3.56 ms; the one-stream UB product
  // measured no better on them (3.21 -> 3.23-3.45 ms at two workgroups per CU, 3.01 -> 3.04 at one) and stays on rgemm
  // (profiles/r05_c5_out16_nt_ab.txt, r05_c5_nt_hb1_ab.txt)
  if constexpr (S >= 2) {
    if (a.N <= 48 && use_out16()) return launch_rgemm16<S, AM, EM>(a, st, grid_x_out);
  }
  constexpr int NI = 2, BNC = 64, BMR = 256;
  if (!(a.K % 64 == 0 && a.K <= 256 && a.N >= 1 && a.N <= BNC))
    return fail(PDEINV_ERR_INVALID, "kfp_mlp rgemm (output layer): K % 64 == 0, K <= 256, N <= 64");
  const size_t bytes = (size_t)BNC * (a.K + 4) * sizeof(float);
  auto kern = rgemm<S, NI, AM, B_NN, EM, 0, BNC>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  a.n_mblocks = mblocks(a.R, BMR);
  const int nrs = std::max(1, std::min(a.n_mblocks, kRGridCap));
  if (grid_x_out) *grid_x_out = nrs;
  hipLaunchKernelGGL(kern, dim3(nrs), dim3(kRT), bytes, st, a);
  return check_launch("kfp_mlp fused B-resident output-layer GEMM");
}

// PDEINV_MLP_RGEMM_OUT=0: the output-layer products on fgemm (A/B)
static bool use_rgemm_out() {
  static const bool on = [] { const char* e = ab_env("PDEINV_MLP_RGEMM_OUT"); return !(e && e[0] == '0'); }();
  return on;
}

static bool use_rgemm(int W) {
  static const bool off = [] {
    const char* e = ab_env("PDEINV_MLP_RGEMM");
    return e && e[0] == '0';
  }();
  return !off && (W == 128 || W == 256);
}

// any out_features: the output layer's row reductions (E_OUT) take one partial per 64-column block when
// out_features > 64; L = 1 runs the output layer straight off the layer-1 prologue modes
bool supported(int d, int L, int W, int O) {
  return (d == 2 || d == 4 || d == 8 || d == 16) && L >= 1 && L <= 16 &&
         (W == 32 || W == 64 || W == 128 || W == 256 || W == 512 || W == 1024) && O >= 1;
}

// workspace layout (floats), chunk of Bc rows
struct Layout {
  size_t layer0, layer_stride, a1, hb1, ys, yb, terms, g, abar0, part, part2, total;
};
enum { P_H = 0, P_ZD, P_ZDD, P_A, P_ZETABAR, P_ZB0, P_ZB1, P_ZB2, kPlanes };

static size_t part_floats(int d, int W, int O) {
  size_t m = (size_t)kRowGridCap * (d + 1) * W;                  // layer-1 gradient slabs
  m = std::max(m, (size_t)kRowGridCap * std::max(W, O));         // bias slabs
  m = std::max(m, (size_t)kMaxWgradSlices * W * std::max(W, O)); // weight-gradient slabs
  return m;
}

static Layout layout(int d, int L, int W, int O, int64_t Bc) {
  Layout y{};
  size_t o = 0;
  auto take = [&](size_t n) { const size_t at = o; o += (n + 63) & ~(size_t)63; return at; };
  const size_t plane = ((size_t)Bc * W + 63) & ~(size_t)63;
  y.layer_stride = plane * kPlanes;
  y.layer0 = take(y.layer_stride * (L - 1));
  y.a1 = take(plane);
  y.hb1 = take(3 * plane);
  y.ys = take((size_t)3 * Bc * O);
  y.yb = take((size_t)3 * Bc * O);
  y.terms = take((size_t)4 * Bc * ((O + 63) / 64));  // E_OUT partials per 64-column block
  y.g = take((size_t)Bc * d);
  y.abar0 = take((size_t)Bc * d);
  y.part = take(part_floats(d, W, O));
  y.part2 = take(part_floats(d, W, O) / kFold + 64);
  y.total = o;
  return y;
}

size_t workspace_floats(int d, int L, int W, int O, int64_t Bc) { return layout(d, L, W, O, Bc).total; }

const float* grad_rows(const Chunk& c) { return c.ws + layout(c.d, c.L, c.W, c.O, c.Bc).g; }

// zero the first n floats of every plane and the first ng floats of g (first_order chunks)
static int zero_planes(const std::vector<float*>& planes, size_t n, float* g, size_t ng, hipStream_t st) {
  for (float* p : planes)
    if (hipMemsetAsync(p, 0, n * sizeof(float), st) != hipSuccess) return fail(PDEINV_ERR_HIP, "kfp_mlp fused: memset");
  if (hipMemsetAsync(g, 0, ng * sizeof(float), st) != hipSuccess) return fail(PDEINV_ERR_HIP, "kfp_mlp fused: memset");
  return 0;
}

// PDEINV_MLP_FO2=0 (A/B): first-order chunks run the full three-stream kernels on zeroed g / a / zetabar planes
static bool use_fo2() {
  static const bool on = [] { const char* e = ab_env("PDEINV_MLP_FO2"); return !(e && e[0] == '0'); }();
  return on;
}

// The first-order chain (initial / terminal sets: c1 = c2 = 0, kinetic_fokker_planck.py:34-39) on two streams, L >= 2,
// W in {128, 256}, out_features <= 64. Only V' = grad V . v and V enter the loss, so the chain carries [h, z'] forward
// and [zbar, z'bar] back: no z'' stream, no g / a chain, no forward adjoint (zetabar), no UB product (ubar = 0: the
// seeds ride in the output layer's epilogue, E_OUT_SEEDS1), and the weight gradients take 2 stream pairs of 4.
//   FWD   [h2, z2'] = [h1, s1 z1'] K2 (A_L1F, S = 2); middle layers A_FWD2
//   OUT   y, y' -> terms, seeds ybar = 2 c3 y' + 2 c0 y, y'bar = 2 c3 y, bo gradient     g := 0 (the loss reads it)
//   R2    [hbar_L, h'bar_L] = [ybar, y'bar] Ko^T, act_bwd (S = 2) ... [hbar1, h'bar1] = [zbar2, z'bar2] K2^T
//   L1    l1_grad_kernel<FO>;  G: wgrad_o / wgrad2 with 2 pairs
template <int D, int WB>
static int run_chunk_fo2(const Chunk& c, const LossHook& loss, hipStream_t st) {
  constexpr int TN = WB < 128 ? WB : 128;
  constexpr int TM = TN == 32 ? 128 : 64;
  constexpr int TG = TN == 32 ? 4 : 2;
  static_assert(WB == 128 || WB == 256, "first-order chain: the B-resident kernels");
  const int L = c.L, W = c.W, O = c.O;
  const int64_t R = c.R;
  const Layout y = layout(D, L, W, O, c.Bc);
  float* ws = c.ws;
  const size_t plane = ((size_t)c.Bc * W + 63) & ~(size_t)63;
  auto P = [&](int l, int k) { return ws + y.layer0 + y.layer_stride * (size_t)(l - 2) + plane * k; };
  float* HB1[2] = {ws + y.hb1, ws + y.hb1 + plane};
  float* YB[2] = {ws + y.yb, ws + y.yb + (size_t)c.Bc * O};
  float4* terms = (float4*)(ws + y.terms);
  float* G = ws + y.g;
  float* abar0 = ws + y.abar0;
  float* part = ws + y.part;
  float* part2 = ws + y.part2;
  const float* prm = c.params;
  auto Kw = [&](int l) { return prm + c.poff[l - 1]; };
  auto Bw = [&](int l) { return prm + c.boff[l - 1]; };
  const float* Ko = prm + c.poff[L];
  GemmArgs base{};
  base.R = R;
  base.c2 = 0.f;
  base.c3 = c.c3;
  base.c0 = c.c0;
  base.part = part;
  base.xz = c.z;
  base.ldxz = c.ldz;
  base.ab0 = abar0;
  base.k1 = Kw(1);
  base.b1 = Bw(1);
  base.wrow = c.wrow;
  base.ldw = c.ldw;
  int rc = 0;
#define RC(x)          \
  do {                 \
    rc = (x);          \
    if (rc) return rc; \
  } while (0)
  {
    GemmArgs a = base;
    a.K = W; a.N = W; a.Bw = Kw(2); a.bias = Bw(2);
    a.po0 = P(2, P_H); a.po1 = P(2, P_ZD);
    RC((launch_rgemm<2, A_L1F, B_NN, E_ACT_FWD, D>(a, st)));
  }
  for (int l = 3; l <= L; ++l) {
    GemmArgs a = base;
    a.K = W; a.N = W; a.Bw = Kw(l); a.bias = Bw(l);
    a.pa0 = P(l - 1, P_H); a.pa1 = P(l - 1, P_ZD);
    a.po0 = P(l, P_H); a.po1 = P(l, P_ZD);
    RC((launch_rgemm<2, A_FWD2, B_NN, E_ACT_FWD>(a, st)));
  }
  {
    GemmArgs a = base;
    a.K = W; a.N = O; a.Bw = Ko; a.bias = prm + c.boff[L];
    a.pa0 = P(L, P_H); a.pa1 = P(L, P_ZD);
    a.po0 = YB[0]; a.po1 = YB[1]; a.terms = terms;
    int gx = 0;
    RC((launch_rgemm_out<2, A_FWD2, E_OUT_SEEDS1>(a, st, &gx)));
    RC(sum_slabs(part, gx, O, c.grad + c.boff[L], part2, st));
  }
  if (hipMemsetAsync(G, 0, (size_t)R * D * sizeof(float), st) != hipSuccess)
    return fail(PDEINV_ERR_HIP, "kfp_mlp fused: memset");
  RC(loss.fn(loss.ctx, G, terms, abar0, R, st));
  {
    GemmArgs a = base;
    a.K = O; a.N = W; a.Bw = Ko;
    a.pa0 = YB[0]; a.pa1 = YB[1];
    a.pe0 = P(L, P_H); a.pe1 = P(L, P_ZD);
    a.po0 = P(L, P_ZB0); a.po1 = P(L, P_ZB1);
    int gx = 0;
    RC((launch_gemm<2, TM, TN, TG, A_S2, B_NT, E_ACT_BWD>(a, st, &gx)));
    RC(sum_slabs(part, gx, W, c.grad + c.boff[L - 1], part2, st));
  }
  for (int l = L; l >= 3; --l) {
    GemmArgs a = base;
    a.K = W; a.N = W; a.Bw = Kw(l);
    a.pa0 = P(l, P_ZB0); a.pa1 = P(l, P_ZB1);
    a.pe0 = P(l - 1, P_H); a.pe1 = P(l - 1, P_ZD);
    a.po0 = P(l - 1, P_ZB0); a.po1 = P(l - 1, P_ZB1);
    int gx = 0;
    RC((launch_rgemm<2, A_S2, B_NT, E_ACT_BWD>(a, st, &gx)));
    RC(sum_slabs(part, gx, W, c.grad + c.boff[l - 2], part2, st));
  }
  {
    GemmArgs a = base;
    a.K = W; a.N = W; a.Bw = Kw(2);
    a.pa0 = P(2, P_ZB0); a.pa1 = P(2, P_ZB1);
    a.po0 = HB1[0]; a.po1 = HB1[1];
    RC((launch_rgemm<2, A_S2, B_NT, E_STORE3>(a, st)));
    const int l1_blocks = (int)std::min<int64_t>((R + kL1Rows - 1) / kL1Rows, kRowGridCap);
    const int64_t l1_rpb = (R + l1_blocks - 1) / l1_blocks;
    hipLaunchKernelGGL((l1_grad_kernel<D, WB, true>), dim3(l1_blocks), dim3(kT), 0, st, HB1[0], HB1[1], nullptr,
                       nullptr, c.z, c.ldz, nullptr, Kw(1), Bw(1), R, l1_rpb, part);
    RC(check_launch("kfp_mlp fused layer-1 gradient (first order)"));
    RC(sum_slabs(part, l1_blocks, (int64_t)(D + 1) * W, c.grad + c.poff[0], part2, st));
  }
  {
    WgradArgs g{};
    g.R = R; g.n_in = W; g.n_out = O; g.part = part;
    g.pa0 = P(L, P_H); g.pa1 = P(L, P_ZD);
    g.pb0 = YB[0]; g.pb1 = YB[1];
    const int64_t cap = (int64_t)part_floats(D, W, O);
    switch ((O + 15) / 16) {
      case 1: RC((launch_wgrad_o<1, 2>(g, cap, c.grad + c.poff[L], part2, st))); break;
      case 2: RC((launch_wgrad_o<2, 2>(g, cap, c.grad + c.poff[L], part2, st))); break;
      case 3: RC((launch_wgrad_o<3, 2>(g, cap, c.grad + c.poff[L], part2, st))); break;
      default: RC((launch_wgrad_o<4, 2>(g, cap, c.grad + c.poff[L], part2, st))); break;
    }
  }
  for (int l = L; l >= 3; --l) {
    WgradArgs g{};
    g.R = R; g.n_in = W; g.n_out = W; g.part = part;
    g.pa0 = P(l - 1, P_H); g.pa1 = P(l - 1, P_ZD);
    g.pb0 = P(l, P_ZB0); g.pb1 = P(l, P_ZB1);
    RC((launch_wgrad2<WB / 128, WB / 64, GA_PL, GB_PL, 0, 2>(g, c.grad + c.poff[l - 1], part2, st)));
  }
  {
    WgradArgs g{};
    g.R = R; g.n_in = W; g.n_out = W; g.part = part;
    g.xz = c.z; g.ldxz = c.ldz; g.k1 = Kw(1); g.b1 = Bw(1);
    g.pb0 = P(2, P_ZB0); g.pb1 = P(2, P_ZB1);
    RC((launch_wgrad2<WB / 128, WB / 64, GA_L1, GB_PL, D, 2>(g, c.grad + c.poff[1], part2, st)));
  }
#undef RC
  return 0;
}

template <int D, int WB>
static int run_chunk_t(const Chunk& c, const LossHook& loss, hipStream_t st) {
  // hidden-width row-GEMM tiles: 64 x 128 (2 x 2 waves) for W >= 128; narrow nets get tiles no
  // wider than W (64: 64 x 64, 2 x 2 waves; 32: 128 x 32, 4 x 1 waves) so no MFMA column is padding
  constexpr int TN = WB < 128 ? WB : 128;
  constexpr int TM = TN == 32 ? 128 : 64;
  constexpr int TG = TN == 32 ? 4 : 2;
  // weight-gradient tiles (>= 64 per side: 2 x 2 waves of 32-multiples)
  constexpr int GW = WB < 128 ? 64 : 128;
  const int L = c.L, W = c.W, O = c.O;
  const int64_t R = c.R;
  const Layout y = layout(D, L, W, O, c.Bc);
  const bool RG = use_rgemm(WB);
  float* ws = c.ws;
  const size_t plane = ((size_t)c.Bc * W + 63) & ~(size_t)63;
  auto P = [&](int l, int k) { return ws + y.layer0 + y.layer_stride * (size_t)(l - 2) + plane * k; };
  float* A1 = ws + y.a1;
  float* HB1[3] = {ws + y.hb1, ws + y.hb1 + plane, ws + y.hb1 + 2 * plane};
  float* Ys[3] = {ws + y.ys, ws + y.ys + (size_t)c.Bc * O, ws + y.ys + 2 * (size_t)c.Bc * O};
  float* YB[3] = {ws + y.yb, ws + y.yb + (size_t)c.Bc * O, ws + y.yb + 2 * (size_t)c.Bc * O};
  float4* terms = (float4*)(ws + y.terms);
  float* G = ws + y.g;
  float* abar0 = ws + y.abar0;
  float* part = ws + y.part;
  float* part2 = ws + y.part2;
  const float* prm = c.params;
  auto Kw = [&](int l) { return prm + c.poff[l - 1]; };  // hidden layer l (1-based) kernel
  auto Bw = [&](int l) { return prm + c.boff[l - 1]; };
  const float* Ko = prm + c.poff[L];
  const float* bo = prm + c.boff[L];

  GemmArgs base{};
  base.R = R;
  base.c2 = c.c2;
  base.c3 = c.c3;
  base.c0 = c.c0;
  base.part = part;
  base.xz = c.z;
  base.ldxz = c.ldz;
  base.ab0 = abar0;
  base.k1 = Kw(1);
  base.b1 = Bw(1);
  base.wrow = c.wrow;
  base.ldw = c.ldw;
  int rc = 0;
#define RC(x)          \
  do {                 \
    rc = (x);          \
    if (rc) return rc; \
  } while (0)

  const int l1_blocks = (int)std::min<int64_t>((R + kL1Rows - 1) / kL1Rows, kRowGridCap);
  const int64_t l1_rpb = (R + l1_blocks - 1) / l1_blocks;
  auto sum_terms = [&]() {
    if (O <= 64) return 0;
    hipLaunchKernelGGL(terms_sum_kernel, dim3((unsigned)((R + kT - 1) / kT)), dim3(kT), 0, st, terms, (O + 63) / 64, R);
    return check_launch("kfp_mlp fused terms sum");
  };
  auto run_g = [&]() {  // g = zeta1 K1^T (grad_x V) from a1
    if constexpr (WB <= 256) {
      if (use_l1g_mfma()) {
        const int blocks = (int)std::min<int64_t>((R + 63) / 64, 2048);
        hipLaunchKernelGGL((l1_g_mfma_kernel<D, WB>), dim3(blocks), dim3(kT), 0, st, A1, c.z, c.ldz, Kw(1), Bw(1), R, G);
        return check_launch("kfp_mlp fused g (MFMA)");
      }
    }
    const int blocks = (int)std::min<int64_t>((R + 3) / 4, 2048);
    hipLaunchKernelGGL((l1_g_kernel<D, WB>), dim3(blocks), dim3(kT), 0, st, A1, c.z, c.ldz, Kw(1), Bw(1), R, G);
    return check_launch("kfp_mlp fused g");
  };
  if (L == 1) {
    // one hidden layer: the output layer reads the layer-1 streams straight from the prologue modes (h1,
    // s1 z1', s2 z1'^2 | s1 (abar0 K1)), the reverse product stops at hbar1 (l1_grad_kernel), and the
    // output-layer weight gradient rebuilds the layer-1 streams from the rows (GA_L1) — no plane of
    // layer 1 is stored
    {
      GemmArgs a = base;
      a.K = W; a.N = O; a.Bw = Ko; a.bias = bo;
      a.po0 = Ys[0]; a.po1 = Ys[1]; a.po2 = Ys[2]; a.terms = terms;
      RC((launch_gemm<3, 128, 64, 4, A_L1F, B_NN, E_OUT, D>(a, st)));
      RC(sum_terms());
    }
    if (c.first_order) {
      RC(zero_planes({A1}, (size_t)R * W, G, (size_t)R * D, st));
    } else {
      {
        GemmArgs a = base;
        a.K = O; a.N = W; a.Bw = Ko; a.pa0 = Ys[0]; a.po0 = A1;
        RC((launch_gemm1<A_U, B_NT>(a, st)));
      }
      RC(run_g());
    }
    if (c.grad_only) return 0;
    RC(loss.fn(loss.ctx, G, terms, abar0, R, st));
    {
      GemmArgs a = base;
      a.K = W; a.N = O; a.Bw = Ko;
      a.pe0 = Ys[0]; a.pe1 = Ys[1]; a.pe2 = Ys[2];
      a.po0 = YB[0]; a.po1 = YB[1]; a.po2 = YB[2];
      int gx = 0;
      RC((launch_gemm<1, 128, 64, 4, A_L1A, B_NN, E_SEEDS, D>(a, st, &gx)));
      RC(sum_slabs(part, gx, O, c.grad + c.boff[L], part2, st));
    }
    {
      GemmArgs a = base;
      a.K = O; a.N = W; a.Bw = Ko;
      a.pa0 = YB[0]; a.pa1 = YB[1]; a.pa2 = YB[2];
      a.po0 = HB1[0]; a.po1 = HB1[1]; a.po2 = HB1[2];
      RC((launch_gemm<3, TM, TN, TG, A_S3, B_NT, E_STORE3>(a, st)));
      hipLaunchKernelGGL((l1_grad_kernel<D, WB>), dim3(l1_blocks), dim3(kT), 0, st, HB1[0], HB1[1], HB1[2], A1, c.z,
                         c.ldz, abar0, Kw(1), Bw(1), R, l1_rpb, part);
      RC(check_launch("kfp_mlp fused layer-1 gradient"));
      RC(sum_slabs(part, l1_blocks, (int64_t)(D + 1) * W, c.grad + c.poff[0], part2, st));  // K1 then b1
    }
    {
      WgradArgs g{};
      g.R = R; g.n_in = W; g.n_out = O; g.part = part;
      g.xz = c.z; g.ldxz = c.ldz; g.ab0 = abar0; g.k1 = Kw(1); g.b1 = Bw(1);
      g.pb0 = YB[0]; g.pb1 = YB[1]; g.pb2 = YB[2]; g.pb3 = Ys[0];
      RC((launch_wgrad<GW, 64, GA_L1, GB_SM, D>(g, c.grad + c.poff[L], part2, st)));
    }
    return 0;
  }
  if constexpr (WB == 128 || WB == 256) {
    if (c.first_order && !c.grad_only && c.c2 == 0.f && RG && O <= 64 && use_rgemm_out() && use_wgo() && use_fo2())
      return run_chunk_fo2<D, WB>(c, loss, st);
  }
  // ---- F1 -------------------------------------------------------------------------------
  {  // layer 1 in the prologue (h1 streams never stored), layer 2 on MFMA
    GemmArgs a = base;
    a.K = W; a.N = W; a.Bw = Kw(2); a.bias = Bw(2);
    a.po0 = P(2, P_H); a.po1 = P(2, P_ZD); a.po2 = P(2, P_ZDD);
    if (RG) RC((launch_rgemm<3, A_L1F, B_NN, E_ACT_FWD, D>(a, st)));
    else RC((launch_gemm<3, TM, TN, TG, A_L1F, B_NN, E_ACT_FWD, D>(a, st)));
  }
  for (int l = 3; l <= L; ++l) {
    GemmArgs a = base;
    a.K = W; a.N = W; a.Bw = Kw(l); a.bias = Bw(l);
    a.pa0 = P(l - 1, P_H); a.pa1 = P(l - 1, P_ZD); a.pa2 = P(l - 1, P_ZDD);
    a.po0 = P(l, P_H); a.po1 = P(l, P_ZD); a.po2 = P(l, P_ZDD);
    if (RG) RC((launch_rgemm<3, A_FWD, B_NN, E_ACT_FWD>(a, st)));
    else RC((launch_gemm<3, TM, TN, TG, A_FWD, B_NN, E_ACT_FWD>(a, st)));
  }
  {
    GemmArgs a = base;
    a.K = W; a.N = O; a.Bw = Ko; a.bias = bo;
    a.pa0 = P(L, P_H); a.pa1 = P(L, P_ZD); a.pa2 = P(L, P_ZDD);
    a.po0 = Ys[0]; a.po1 = Ys[1]; a.po2 = Ys[2]; a.terms = terms;
    if (RG && use_rgemm_out() && O <= 64) RC((launch_rgemm_out<3, A_FWD, E_OUT>(a, st)));
    else RC((launch_gemm<3, 128, 64, 4, A_FWD, B_NN, E_OUT>(a, st)));
    RC(sum_terms());
  }
  // ---- R1: grad_x chain -------------------------------------------------------------------
  if (c.first_order) {  // no g, no forward adjoint: zeros where the later products read them
    std::vector<float*> z0{A1};
    for (int l = 2; l <= L; ++l) {
      z0.push_back(P(l, P_A));
      z0.push_back(P(l, P_ZETABAR));
    }
    RC(zero_planes(z0, (size_t)R * W, G, (size_t)R * D, st));
  } else {
    {
      GemmArgs a = base;
      a.K = O; a.N = W; a.Bw = Ko; a.pa0 = Ys[0]; a.po0 = P(L, P_A);
      RC((launch_gemm1<A_U, B_NT>(a, st)));
    }
    for (int l = L; l >= 2; --l) {
      GemmArgs a = base;
      a.K = W; a.N = W; a.Bw = Kw(l); a.pa0 = P(l, P_H); a.pa1 = P(l, P_A);
      a.po0 = l > 2 ? P(l - 1, P_A) : A1;
      if (RG) RC((launch_rgemm<1, A_S1MUL, B_NT, E_STORE>(a, st)));
      else RC((launch_gemm1<A_S1MUL, B_NT>(a, st)));
    }
    RC(run_g());
  }
  if (c.grad_only) return 0;  // KMV pass 1: g of every row is all that is needed
  RC(loss.fn(loss.ctx, G, terms, abar0, R, st));
  // ---- F2: forward adjoint ----------------------------------------------------------------
  if (!c.first_order) {
    {  // abar1 = s1(z1) (abar0 K1) in the prologue
      GemmArgs a = base;
      a.K = W; a.N = W; a.Bw = Kw(2); a.po0 = P(2, P_ZETABAR);
      if (RG) RC((launch_rgemm<1, A_L1A, B_NN, E_STORE, D>(a, st)));
      else RC((launch_gemm1<A_L1A, B_NN, D>(a, st)));
    }
    for (int l = 3; l <= L; ++l) {
      GemmArgs a = base;
      a.K = W; a.N = W; a.Bw = Kw(l); a.pa0 = P(l - 1, P_H); a.pa1 = P(l - 1, P_ZETABAR);
      a.po0 = P(l, P_ZETABAR);
      if (RG) RC((launch_rgemm<1, A_S1MUL, B_NN, E_STORE>(a, st)));
      else RC((launch_gemm1<A_S1MUL, B_NN>(a, st)));
    }
  }
  {
    GemmArgs a = base;
    a.K = W; a.N = O; a.Bw = Ko; a.pa0 = P(L, P_H); a.pa1 = P(L, P_ZETABAR);
    a.pe0 = Ys[0]; a.pe1 = Ys[1]; a.pe2 = Ys[2];
    a.po0 = YB[0]; a.po1 = YB[1]; a.po2 = YB[2];
    int gx = 0;
    if (RG && use_rgemm_out() && O <= 64) RC((launch_rgemm_out<1, A_S1MUL, E_SEEDS>(a, st, &gx)));
    else RC((launch_gemm<1, 128, 64, 4, A_S1MUL, B_NN, E_SEEDS>(a, st, &gx)));
    RC(sum_slabs(part, gx, O, c.grad + c.boff[L], part2, st));
  }
  // ---- R2: reverse over the forward streams -------------------------------------------------
  {
    GemmArgs a = base;
    a.K = O; a.N = W; a.Bw = Ko;
    a.pa0 = YB[0]; a.pa1 = YB[1]; a.pa2 = YB[2];
    a.pe0 = P(L, P_H); a.pe1 = P(L, P_ZD); a.pe2 = P(L, P_ZDD); a.pe3 = P(L, P_A); a.pe4 = P(L, P_ZETABAR);
    a.po0 = P(L, P_ZB0); a.po1 = P(L, P_ZB1); a.po2 = P(L, P_ZB2);
    int gx = 0;
    RC((launch_gemm<3, TM, TN, TG, A_S3, B_NT, E_ACT_BWD>(a, st, &gx)));
    RC(sum_slabs(part, gx, W, c.grad + c.boff[L - 1], part2, st));
  }
  for (int l = L; l >= 3; --l) {
    GemmArgs a = base;
    a.K = W; a.N = W; a.Bw = Kw(l);
    a.pa0 = P(l, P_ZB0); a.pa1 = P(l, P_ZB1); a.pa2 = P(l, P_ZB2);
    a.pe0 = P(l - 1, P_H); a.pe1 = P(l - 1, P_ZD); a.pe2 = P(l - 1, P_ZDD); a.pe3 = P(l - 1, P_A);
    a.pe4 = P(l - 1, P_ZETABAR);
    a.po0 = P(l - 1, P_ZB0); a.po1 = P(l - 1, P_ZB1); a.po2 = P(l - 1, P_ZB2);
    int gx = 0;
    if (RG) RC((launch_rgemm<3, A_S3, B_NT, E_ACT_BWD>(a, st, &gx)));
    else RC((launch_gemm<3, TM, TN, TG, A_S3, B_NT, E_ACT_BWD>(a, st, &gx)));
    RC(sum_slabs(part, gx, W, c.grad + c.boff[l - 2], part2, st));
  }
  {
    GemmArgs a = base;
    a.K = W; a.N = W; a.Bw = Kw(2);
    a.pa0 = P(2, P_ZB0); a.pa1 = P(2, P_ZB1); a.pa2 = P(2, P_ZB2);
    a.po0 = HB1[0]; a.po1 = HB1[1]; a.po2 = HB1[2];
    if (RG) RC((launch_rgemm<3, A_S3, B_NT, E_STORE3>(a, st)));
    else RC((launch_gemm<3, TM, TN, TG, A_S3, B_NT, E_STORE3>(a, st)));
    hipLaunchKernelGGL((l1_grad_kernel<D, WB>), dim3(l1_blocks), dim3(kT), 0, st, HB1[0], HB1[1], HB1[2], A1, c.z,
                       c.ldz, abar0, Kw(1), Bw(1), R, l1_rpb, part);
    RC(check_launch("kfp_mlp fused layer-1 gradient"));
    RC(sum_slabs(part, l1_blocks, (int64_t)(D + 1) * W, c.grad + c.poff[0], part2, st));  // K1 then b1
  }
  // ---- G: weight gradients ------------------------------------------------------------------
  {
    WgradArgs g{};
    g.R = R; g.n_in = W; g.n_out = O; g.part = part;
    g.pa0 = P(L, P_H); g.pa1 = P(L, P_ZD); g.pa2 = P(L, P_ZDD); g.pa3 = P(L, P_ZETABAR);
    g.pb0 = YB[0]; g.pb1 = YB[1]; g.pb2 = YB[2]; g.pb3 = Ys[0];
    const int64_t cap = (int64_t)part_floats(D, W, O);
    if (WB >= 64 && WB <= 256 && O <= 64 && use_wgo()) {
      switch ((O + 15) / 16) {
        case 1: RC((launch_wgrad_o<1>(g, cap, c.grad + c.poff[L], part2, st))); break;
        case 2: RC((launch_wgrad_o<2>(g, cap, c.grad + c.poff[L], part2, st))); break;
        case 3: RC((launch_wgrad_o<3>(g, cap, c.grad + c.poff[L], part2, st))); break;
        default: RC((launch_wgrad_o<4>(g, cap, c.grad + c.poff[L], part2, st))); break;
      }
    } else {
      RC((launch_wgrad<GW, 64, GA_PL, GB_SM>(g, c.grad + c.poff[L], part2, st)));
    }
  }
  for (int l = L; l >= 3; --l) {
    WgradArgs g{};
    g.R = R; g.n_in = W; g.n_out = W; g.part = part;
    g.pa0 = P(l - 1, P_H); g.pa1 = P(l - 1, P_ZD); g.pa2 = P(l - 1, P_ZDD); g.pa3 = P(l - 1, P_ZETABAR);
    g.pb0 = P(l, P_ZB0); g.pb1 = P(l, P_ZB1); g.pb2 = P(l, P_ZB2); g.pb3 = P(l, P_H); g.pb4 = P(l, P_A);
    if constexpr (WB == 128 || WB == 256) {
      if (RG) RC((launch_wgrad2<WB / 128, WB / 64, GA_PL, GB_PL>(g, c.grad + c.poff[l - 1], part2, st)));
      else RC((launch_wgrad<GW, GW, GA_PL, GB_PL>(g, c.grad + c.poff[l - 1], part2, st)));
    } else {
      RC((launch_wgrad<GW, GW, GA_PL, GB_PL>(g, c.grad + c.poff[l - 1], part2, st)));
    }
  }
  {
    WgradArgs g{};
    g.R = R; g.n_in = W; g.n_out = W; g.part = part;
    g.xz = c.z; g.ldxz = c.ldz; g.ab0 = abar0; g.k1 = Kw(1); g.b1 = Bw(1);
    g.pb0 = P(2, P_ZB0); g.pb1 = P(2, P_ZB1); g.pb2 = P(2, P_ZB2); g.pb3 = P(2, P_H); g.pb4 = P(2, P_A);
    if constexpr (WB == 128 || WB == 256) {
      if (RG) RC((launch_wgrad2<WB / 128, WB / 64, GA_L1, GB_PL, D>(g, c.grad + c.poff[1], part2, st)));
      else RC((launch_wgrad<GW, GW, GA_L1, GB_PL, D>(g, c.grad + c.poff[1], part2, st)));
    } else {
      RC((launch_wgrad<GW, GW, GA_L1, GB_PL, D>(g, c.grad + c.poff[1], part2, st)));
    }
  }
#undef RC
  return 0;
}

template <int D>
static int run_chunk_d(const Chunk& c, const LossHook& loss, hipStream_t st) {
  switch (c.W) {
    case 32: return run_chunk_t<D, 32>(c, loss, st);
    case 64: return run_chunk_t<D, 64>(c, loss, st);
    case 128: return run_chunk_t<D, 128>(c, loss, st);
    case 256: return run_chunk_t<D, 256>(c, loss, st);
    case 512: return run_chunk_t<D, 512>(c, loss, st);
    case 1024: return run_chunk_t<D, 1024>(c, loss, st);
    default: return fail(PDEINV_ERR_UNSUPPORTED, "kfp_mlp fused: width must be 32, 64, 128, 256, 512 or 1024");
  }
}

int run_chunk(const Chunk& c, const LossHook& loss, hipStream_t st) {
  if (!supported(c.d, c.L, c.W, c.O)) return fail(PDEINV_ERR_UNSUPPORTED, "kfp_mlp fused: unsupported shape");
  if (c.Bc * (int64_t)std::max(c.W, c.O) > ((int64_t)1 << 30))  // ldo / sto: 32-bit BYTE offsets into a plane
    return fail(PDEINV_ERR_INVALID, "kfp_mlp fused: chunk_rows * max(width, out_features) must stay at or below 2^30");
  if (c.R <= 0) return 0;
  switch (c.d) {
    case 2: return run_chunk_d<2>(c, loss, st);
    case 4: return run_chunk_d<4>(c, loss, st);
    case 8: return run_chunk_d<8>(c, loss, st);
    case 16: return run_chunk_d<16>(c, loss, st);
    default: return fail(PDEINV_ERR_UNSUPPORTED, "kfp_mlp fused: dim must be 2, 4, 8 or 16");
  }
}

}  // namespace mlpf
}  // namespace pdeinv

