// sde_kmv.hip — the McKean–Vlasov simulator fused with the KMV residual's per-time-stamp sums (gfx950).
#include "sde_common.h"

using namespace pdeinv;

// ---- McKean–Vlasov simulate + the KMV residual's per-time-stamp sums (ABI 10) -----------------------------
// The quadratic-Phi KMV residual (kinetic_mckean_vlasov.py:11-120, kmv.hip) reads, per time stamp t = trajectory
// row t, [count, sum z, sum z z^T] of z = [x, v] and the d_s log rho-weighted [sum w, sum w x, sum w x x^T] of x
// (w = d_s^2 log rho + (d_s log rho)^2 + gamma d_s log rho, kinetic_mckean_vlasov.py:243-248). The simulator stages
// each wave's 64 rows of update t in LDS for its coalesced store anyway; the same staged rows feed one
// v_mfma_f32_16x16x4_f32 tile per stamp over K = the wave's rows (sde_mf_kmv_kernel below), the waves of a block add
// their tiles in LDS in a fixed order (one barrier per 4 stamps), the block writes one partial column entry per sum
// and slab_reduce sums the blocks in fp64. Deterministic; no trajectory re-read. The two blocks the residual uses
// only summed over the stamps (sum w x x^T, the v v^T rest) come out as stamp totals.
// Measured (profiles/r06_c4_fused_single_tile.txt): the kernel spends more on the stamp sums
// (fp32 MFMA and the weight's VALU, which share the SIMD's issue) than the separate KMV pass spends streaming the
// trajectory back, so the product path takes it only for trajectories too large to keep (methods/consistency.py).
template <int D>
constexpr int kmv_ncp() { return D + 2 + 2 * (D * (D + 1) / 2 + D); }
template <int D>
constexpr int kmv_ncp_pad() { return (kmv_ncp<D>() + 15) / 16 * 16; }  // a stamp's row: whole 16-float chunks

struct KmvStamps {
  const float* cp;   // [n_steps][kmv_ncp_pad<D>()]: the stamp's coefficients in use order (kmv_coef_pairs_kernel)
  float* partials;   // [(n_steps * NS + NTOT) columns][gridDim.x]: every stamp's per-stamp sums, then the totals
  float gamma;
};

// The coefficients kmv_moments_weights_kernel builds in LDS per block (kmv.hip), once per stamp into global memory,
// in the order kmv_weight consumes them: m1 (D), (a1, a2), then per row i the pair (b1_i, b2_i) followed by the
// pairs (G1_ij + G1_ji, G2_ij + G2_ji), j = i .. D - 1 (G_ii on the diagonal); zero-padded to whole chunks.
template <int D>
__global__ void kmv_coef_pairs_kernel(const float* __restrict__ coef, float* __restrict__ cp) {
  constexpr int NC = 3 * D + 2 + 2 * D * D, NCP = kmv_ncp<D>(), NCPP = kmv_ncp_pad<D>();
  const float* c = coef + (int64_t)blockIdx.x * NC;  // [m1, a1, b1, G1, a2, b2, G2]
  float* o = cp + (int64_t)blockIdx.x * NCPP;
  for (int e = threadIdx.x; e < NCPP; e += blockDim.x) {
    float v = 0.f;
    if (e < D) {
      v = c[e];
    } else if (e == D) {
      v = c[D];
    } else if (e == D + 1) {
      v = c[2 * D + 1 + D * D];
    } else if (e < NCP) {
      int p = (e - D - 2) >> 1, i = 0;
      const int h = (e - D - 2) & 1;
      while (p >= D - i + 1) { p -= D - i + 1; ++i; }  // row i holds 1 + (D - i) pairs
      if (p == 0) {
        v = h ? c[2 * D + 2 + D * D + i] : c[D + 1 + i];  // (b1_i, b2_i)
      } else {
        const int j = i + p - 1;
        const float* G = h ? c + 3 * D + 2 + D * D : c + 2 * D + 1;
        v = i == j ? G[i * D + i] : G[i * D + j] + G[j * D + i];
      }
    }
    o[e] = v;
  }
}

// w of one row at stamp coefficients cp (uniform; scalar loads: no vmcnt wait, which on gfx950 would also wait for
// the trajectory stores in flight). Same operation order as kmv_moments_weights_kernel.
template <int D>
__device__ __forceinline__ float kmv_weight(const float* z, const float* cp, float gamma) {
  float rr[D] = {};
  f32x2 q = {0.f, 0.f}, g = {0.f, 0.f};
  f32x16 ch;
  int e = 0;  // the running coefficient index (a constant in every unrolled copy)
  auto next2 = [&]() -> f32x2 {
    if (e % 16 == 0) ch = sgpr_chunk16((kfloat*)(cp + e), g[0] + q[0] + rr[0]);  // one chunk live at a time
    const f32x2 v = {ch[e % 16], ch[e % 16 + 1]};
    e += 2;
    return v;
  };
#pragma unroll
  for (int k = 0; k < D; k += 2) {  // r = m1 - x
    const f32x2 m = next2();
    rr[k] = m[0] - z[k];
    rr[k + 1] = m[1] - z[k + 1];
  }
  q = next2();
#pragma unroll
  for (int i = 0; i < D; ++i) {  // q += r_i (b_i + sum_{j >= i} Gsym_ij r_j)
    g = next2();
#pragma unroll
    for (int j = i; j < D; ++j) g = next2() * f32x2{rr[j], rr[j]} + g;
    q = g * f32x2{rr[i], rr[i]} + q;
  }
  return q[1] + q[0] * q[0] + gamma * q[0];
}

// The per-stamp product. One v_mfma_f32_16x16x4_f32 tile per update, P = A^T Z over the wave's 64 rows (K), with
//   A = [x (D), one, w, v_0 .. v_{nA-1}, 0..]  (16 features, staged beside z by each row's own lane),  Z = [x, v]:
// rows x give sum x x^T and sum x v^T, row "one" sum z, row "w" sum w x, rows v_a sum v_a v^T. Every sum the
// KMV residual needs per stamp — [count, sum z, sum z z^T] and [sum w, sum w x] — comes out of it (the count is
// the block's rows, sum w a wave sum), except two blocks that the residual (kmv_terms / kmv_combine, kmv.hip) only
// uses summed over the stamps: sum w x x^T, and at d = 8 the v v^T entries the tile has no row for (a >= nA:
// (6,6), (6,7), (7,7)). Those are stamp totals, accumulated per lane over the whole simulate and reduced once.
// So the stamp's sums cost 16 MFMAs per wave-update (a second product for sum w x x^T per stamp doubled the
// kernel's matrix-pipe time and measured slower than the separate KMV pass).
template <int D>
constexpr int kmv_na() { return D < 14 - D ? D : 14 - D; }  // v rows in A (16 - D - 2 slots)
template <int D>
constexpr int kmv_vv_rest() {  // v v^T upper entries (a <= b) with a >= nA
  int n = 0;
  for (int a = kmv_na<D>(); a < D; ++a) n += D - a;
  return n;
}
template <int D>
constexpr int kmv_ntot() { return D * (D + 1) / 2 + kmv_vv_rest<D>(); }  // totals: [sum w x x^T | vv rest]

// Source of the [mom | wst] entry e (kmv_moments_weights order): >= 0 a tile word (entry (i, j) is accumulator
// register i % 4 of lane (i / 4) * 16 + j), -1 the count, -2 sum w, <= -3 the stamp total -(e + 3)... as -3 - k
template <int D>
__host__ __device__ constexpr int kmv_source(int e) {
  constexpr int M = 2 * D, LZ = moment_len(M), NA = kmv_na<D>();
  auto word = [](int i, int j) { return ((i >> 2) * 16 + j) * 4 + (i & 3); };
  auto tri = [](int t, int m, int& ii, int& jj) {
    ii = 0;
    while (t >= m - ii) { t -= m - ii; ++ii; }
    jj = ii + t;
  };
  if (e == 0) return -1;                             // count
  if (e <= M) return word(D, e - 1);                 // sum z_k: row "one"
  if (e < LZ) {                                      // sum z_i z_j, i <= j
    int i = 0, j = 0;
    tri(e - 1 - M, M, i, j);
    if (i < D) return word(i, j);                    // x x, x v
    const int va = i - D;
    if (va < NA) return word(D + 2 + va, j);         // v v
    int k = D * (D + 1) / 2;                         // the vv rest, in (a, b) order
    for (int aa = NA; aa < D; ++aa)
      for (int bb = aa; bb < D; ++bb, ++k)
        if (aa == va && bb == j - D) return -3 - k;
    return -3 - k;  // unreachable
  }
  if (e == LZ) return -2;                            // sum w
  if (e <= LZ + D) return word(D + 1, e - LZ - 1);   // sum w x_k: row "w"
  return -3 - (e - LZ - 1 - D);                      // sum w x_i x_j: a stamp total
}

// the per-stamp entries (source >= -2), in e order
template <int D>
constexpr int kmv_nstamp() {
  constexpr int M = 2 * D, LT = moment_len(M) + moment_len(D);
  int n = 0;
  for (int e = 0; e < LT; ++e) n += kmv_source<D>(e) >= -2;
  return n;
}

template <int D, int WAVES, bool NXT>
__global__ __launch_bounds__(64 * WAVES) void sde_mf_kmv_kernel(
    SdeArgs a, const float* __restrict__ z0, float* __restrict__ traj, float* __restrict__ tau,
    float* __restrict__ last, KmvStamps ks, MfNext nx) {
  constexpr int M = 2 * D, B = 64 * WAVES, NCP = kmv_ncp_pad<D>(), NA = kmv_na<D>();
  constexpr int LZ = moment_len(M), LW = moment_len(D), LT = LZ + LW;
  constexpr int NS = kmv_nstamp<D>(), NTOT = kmv_ntot<D>(), NVR = kmv_vv_rest<D>(), kRed = (NS + B - 1) / B;
  constexpr int KB = 4;  // stamps per block reduction, one barrier each (2: the same time; 8: one block per CU)
  static_assert(KB > 0 && (KB & (KB - 1)) == 0, "power-of-two batch");
  static_assert(D % 2 == 0 && D <= 8, "even dim <= 8: 16-byte staged rows, a 16-feature tile");
  static_assert(D + 2 + NA <= 16, "A = [x, one, w, v_0..v_{nA-1}] in 16 features");
  const int nb = gridDim.x;
  const int bid = a.remap ? xcd_block(blockIdx.x, nb) : (int)blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i_raw = (int64_t)bid * B + threadIdx.x;
  const bool active = i_raw < a.N;
  const int64_t i = active ? i_raw : a.N - 1;  // inactive lanes compute on a valid row, store nothing
  const uint64_t gid = (uint64_t)(a.poff + i);
  const uint32_t plo = (uint32_t)gid, phi = (uint32_t)(gid >> 32);
  const int64_t wave_row0 = i_raw - lane;
  const int n_valid = __builtin_amdgcn_readfirstlane((int)((a.N - wave_row0) < kWave ? (a.N - wave_row0) : kWave));
  const int64_t nblk = a.N - (int64_t)bid * B;
  const float block_rows = (float)(nblk < 0 ? 0 : (nblk > B ? B : nblk));

  __shared__ float stage[B * M + 2 * B];  // the waves' 64 rows of z (pitch M: store staging, both tile operands), w, one
  __shared__ f32x4 red[2][KB][WAVES][kWave];    // per batch of KB stamps (double-buffered): the waves' tiles
  __shared__ float wred[2][KB][WAVES];          // and their sums of w
  float* slot = stage + wave * kWave * M;
  float* wrow = stage + B * M + wave * kWave;

  float z[M];
#pragma unroll
  for (int k = 0; k < M; ++k) z[k] = z0[i * a.ld_z0 + k];

  const int c = lane & 15, rq = lane >> 4;  // operand roles: feature c of rows 4j + rq (A[c][rq] / Z[rq][c])
  const int ca = c < M ? c : 0;
  // the tile operands' LDS words of rows 4j + rq: Z = z row (stride 4M per j); A for c >= D its own word — one (the
  // one plane, stride 4), w (the w plane) or v_(c-D-2) (the z rows); A for c < D is the Z word itself
  const int a_off0 = wave * kWave * M + rq * M + ca;
  const int b_off0 = c == D ? B * M + B + wave * kWave + rq
                   : c == D + 1 ? B * M + wave * kWave + rq
                                : wave * kWave * M + rq * M + (c >= D + 2 && c < D + 2 + NA ? c - 2 : 0);
  const int b_str = c == D || c == D + 1 ? 4 : 4 * M;
  int srcs[kRed], cols[kRed];  // the per-stamp sums this thread adds (t-th: the compact entry threadIdx.x + B t)
#pragma unroll
  for (int t = 0; t < kRed; ++t) {
    srcs[t] = 0;
    cols[t] = -1;
    const int want = threadIdx.x + B * t;
    int n = 0;
    for (int e = 0; e < LT && want < NS; ++e) {
      const int sc = kmv_source<D>(e);
      if (sc < -2) continue;
      if (n == want) { srcs[t] = sc; cols[t] = n; break; }
      ++n;
    }
  }
  // the stamp totals, per lane over the whole simulate: sum w x_i x_j (i <= j) over PairGram pairs, the vv rest
  // sum w x x^T over all stamps on the matrix pipe (4 AGPRs, not D(D+1)/2 lane registers): a split-K tile, features
  // c < 8 carry rows 0..31 of the wave and c >= 8 rows 32..63, so its two diagonal 8 x 8 blocks are the two halves'
  // sums (the off-diagonal blocks are discarded): 8 MFMAs per stamp, A = w x_(c&7), B = x_(c&7) of the lane's row
  f32x4 pw = {0.f, 0.f, 0.f, 0.f};
  const int x_off0 = wave * kWave * M + (32 * (c >> 3) + rq) * M + ((c & 7) < D ? (c & 7) : 0);
  const int w_off0 = B * M + wave * kWave + 32 * (c >> 3) + rq;
  [[maybe_unused]] float vvr[NVR > 0 ? NVR : 1];
#pragma unroll
  for (int k = 0; k < (NVR > 0 ? NVR : 1); ++k) vvr[k] = 0.f;

  const float tau0 = a.tau0_mf;
  const float h_last = a.dt - tau0;
  float* tr = traj ? traj + wave_row0 * M : nullptr;
  float* ta = tau ? tau + i : nullptr;
  const int64_t tr_stride = a.N * M;

  [[maybe_unused]] float nacc[NXT ? 3 : 1][NXT ? D : 1];
  [[maybe_unused]] const int nbase = NXT ? lane * nx.np1 : 0;
  if constexpr (NXT) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < D; ++k) nacc[j][k] = 0.f;
  }

  auto update = [&](float h, float sh, uint32_t s) {
    float g[D], xi[D];
    grad_meanfield<D, true>(a, z, a.xbar + (int64_t)s * D, g);
    stream_normals<D>(a.k0, a.k1, a.ctr_off + s, plo, phi, xi);
    if constexpr (NXT) {  // pair q = nbase + s of the next simulate (sde_simulate_kernel NXT)
      const int q = nbase + (int)s;
      const int sp = q >> 6, j = sp - (nbase >> 6);
      const int64_t ip = wave_row0 + (q & 63);
      const uint64_t g2 = (uint64_t)(a.poff + ip);
      float xn[D];
      stream_normals<D>(a.k0, a.k1, nx.ctr_off + (uint32_t)sp, (uint32_t)g2, (uint32_t)(g2 >> 32), xn);
      const float wv = ip < a.N ? 1.f : 0.f;
      const float w0 = j == 0 ? wv : 0.f, w1 = j == 1 ? wv : 0.f, w2 = j == 2 ? wv : 0.f;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        nacc[0][k] = fmaf(w0, xn[k], nacc[0][k]);
        nacc[1][k] = fmaf(w1, xn[k], nacc[1][k]);
        nacc[2][k] = fmaf(w2, xn[k], nacc[2][k]);
      }
    }
    const float gh = a.gamma * h;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const float p = z[D + k];
      const float pn = fmaf(-gh, p, fmaf(sh, xi[k], fmaf(-h, g[k], p)));  // sampling_utils.py:17,20
      z[D + k] = pn;
      z[k] = fmaf(h, pn, z[k]);
    }
  };

  // trajectory row s (stamp s): stage z and A, store the row chunks, the stamp's tile of the wave's rows on the
  // matrix pipe, the lane's stamp totals, then the block's fixed-order sum of its waves' tiles -> one slab entry per sum
  auto stamp = [&](int s) {
    const float* cps = ks.cp + (int64_t)s * NCP;
    const bool live = n_valid == kWave || active;  // rows past N stage as zeros (weight 0, one = 0)
    const float w = live ? kmv_weight<D>(z, cps, ks.gamma) : 0.f;
    const float one = live ? 1.f : 0.f;
    if (n_valid == kWave) {
#pragma unroll
      for (int k = 0; k < M; k += 4)
        *reinterpret_cast<f32x4*>(slot + lane * M + k) = f32x4{z[k], z[k + 1], z[k + 2], z[k + 3]};
    } else {
#pragma unroll
      for (int k = 0; k < M; k += 4)
        *reinterpret_cast<f32x4*>(slot + lane * M + k) =
            active ? f32x4{z[k], z[k + 1], z[k + 2], z[k + 3]} : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    wrow[lane] = w;
    wrow[B + lane] = one;
    {  // the v v^T stamp totals the tile has no row for (one = 0 on rows past N)
      int r = 0;
#pragma unroll
      for (int va = NA; va < D; ++va)
#pragma unroll
        for (int vb = va; vb < D; ++vb, ++r) vvr[r] = fmaf(one * z[D + va], z[D + vb], vvr[r]);
    }
    const float wsum = wave_sum(w);
    __builtin_amdgcn_wave_barrier();
    if (tr) {  // 16-byte chunk q = k * 64 + lane of the wave's 64 * M floats: 1 KiB contiguous per instruction
      float* dst = tr + (int64_t)s * tr_stride;
      f32x4 v[M / 4];
#pragma unroll
      for (int k = 0; k < M / 4; ++k) v[k] = *reinterpret_cast<const f32x4*>(slot + 4 * (k * 64 + lane));
      if (n_valid == kWave) {
#pragma unroll
        for (int k = 0; k < M / 4; ++k)
          __builtin_nontemporal_store(v[k], reinterpret_cast<f32x4*>(dst + 4 * (k * 64 + lane)));
      } else {
#pragma unroll
        for (int k = 0; k < M / 4; ++k) {
          const int q = k * 64 + lane;
          if (4 * q < n_valid * M) __builtin_nontemporal_store(v[k], reinterpret_cast<f32x4*>(dst + 4 * q));
        }
      }
    }
    if (active && ta) __builtin_nontemporal_store(tau_value(tau0, s, a.dt), ta + (int64_t)s * a.N);
    f32x4 pt = {0.f, 0.f, 0.f, 0.f};
    int a_off = a_off0, b_off = b_off0;
    asm volatile("" : "+v"(a_off), "+v"(b_off));  // per stamp: not 32 addresses hoisted and held across stamps
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float av = stage[a_off + j * 4 * M];
      if constexpr (M < 16) av = c < M ? av : 0.f;
      // A[row][c] = [x (c < D) | one | w | v_(c-D-2)] from the same staged rows: x is av itself
      const float b = stage[b_off + j * b_str];
      const float a2 = c < D ? av : (c < D + 2 + NA ? b : 0.f);
      pt = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, av, pt, 0, 0, 0);
    }
    {
      int x_off = x_off0, w_off = w_off0;
      asm volatile("" : "+v"(x_off), "+v"(w_off));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float xv = stage[x_off + j * 4 * M];
        if constexpr (D < 8) xv = (c & 7) < D ? xv : 0.f;
        const float wv = stage[w_off + 4 * j];
        pw = __builtin_amdgcn_mfma_f32_16x16x4f32(wv * xv, xv, pw, 0, 0, 0);
      }
    }
    const int kb = s & (KB - 1), buf = (s / KB) & 1;
    __builtin_amdgcn_wave_barrier();
    red[buf][kb][wave][lane] = pt;
    if (lane == 0) wred[buf][kb][wave] = wsum;
    if (kb != KB - 1 && s != a.n_steps - 1) return;
    __syncthreads();  // the batch's tiles are in; the next batch writes the other buffer
    for (int k = 0; k <= kb; ++k) {
      const int64_t st = s - kb + k;
      const float* r = reinterpret_cast<const float*>(&red[buf][k][0][0]);
#pragma unroll
      for (int t = 0; t < kRed; ++t) {
        if (cols[t] >= 0) {
          float sum = 0.f;
          if (srcs[t] == -1) {
            sum = block_rows;
          } else if (srcs[t] == -2) {
#pragma unroll
            for (int w2 = 0; w2 < WAVES; ++w2) sum += wred[buf][k][w2];
          } else {
#pragma unroll
            for (int w2 = 0; w2 < WAVES; ++w2) sum += r[w2 * 256 + srcs[t]];
          }
          ks.partials[(st * NS + cols[t]) * nb + bid] = sum;
        }
      }
    }
  };

  // update 0: h = tau0 (sample at tau0)
  update(tau0, sqrtf(tau0) * a.ns, 0u);
  stamp(0);
  const float sh_dt = sqrtf(a.dt) * a.ns;
  for (int s = 1; s < a.n_steps; ++s) {
    update(a.dt, sh_dt, (uint32_t)s);
    stamp(s);
  }
  // final update: h = dt - tau0, lands exactly at T = n*dt (sampling_utils.py:44-46)
  update(h_last, sqrtf(h_last) * a.ns, (uint32_t)a.n_steps);
  if (active && last) store_row<D, kStoreNT>(last + i * M, z);
  {  // the stamp totals: [sum w x_i x_j (i <= j) | vv rest], one slab column each after the per-stamp ones
    constexpr int NT = D * (D + 1) / 2;
    // the waves' split-K tiles into the reduction buffer the last batch did not use (all its reads were before
    // the last barrier), the vv rest as wave sums
    f32x4* t2 = &red[(((a.n_steps - 1) / KB) & 1) ^ 1][0][0][0];
    t2[wave * kWave + lane] = pw;
    __shared__ float tlds[WAVES * (NVR > 0 ? NVR : 1)];
#pragma unroll
    for (int k = 0; k < NVR; ++k) {
      const float v = wave_sum(vvr[k]);
      if (lane == 0) tlds[wave * NVR + k] = v;
    }
    __syncthreads();
    const float* t2f = reinterpret_cast<const float*>(t2);
    const int64_t base = (int64_t)a.n_steps * NS;
    for (int k = threadIdx.x; k < NTOT; k += B) {
      float v = 0.f;
      if (k < NT) {  // (i, j): rows 0..31 at tile entry (i, j), rows 32..63 at (i + 8, j + 8)
        int i = 0, rem = k;
        while (rem >= D - i) { rem -= D - i; ++i; }
        const int j = i + rem;
        const int lo = ((i >> 2) * 16 + j) * 4 + (i & 3), hi = ((2 + (i >> 2)) * 16 + j + 8) * 4 + (i & 3);
#pragma unroll
        for (int w2 = 0; w2 < WAVES; ++w2) v += t2f[w2 * 256 + lo] + t2f[w2 * 256 + hi];
      } else {
#pragma unroll
        for (int w2 = 0; w2 < WAVES; ++w2) v += tlds[w2 * (NVR > 0 ? NVR : 1) + (k - NT)];
      }
      ks.partials[(base + k) * nb + bid] = v;
    }
  }
  if constexpr (NXT) {
    // the block's slab column per update, as sde_simulate_kernel NXT (fixed order: pass, wave, lane)
    float* rb = stage;
    constexpr int NE = (128 * D + B - 1) / B;
    float v[NE];
#pragma unroll
    for (int t = 0; t < NE; ++t) v[t] = 0.f;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int j0 = 2 * pass, nj = pass ? 1 : 2;
      __syncthreads();
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        if (jj < nj) {
#pragma unroll
          for (int k = 0; k < D; ++k) rb[((wave * kWave + lane) * 2 + jj) * D + k] = nacc[j0 + jj][k];
        }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < NE; ++t) {
        const int e = threadIdx.x + t * B;
        if (e < nx.np1 * D) {
          const int sp = e / D, k = e - sp * D;
          const int l0 = (64 * sp) / nx.np1, l1 = (64 * sp + 63) / nx.np1;
          for (int w2 = 0; w2 < WAVES; ++w2)
            for (int l = l0; l <= l1; ++l) {
              const int jj = sp - ((l * nx.np1) >> 6) - j0;
              if (jj >= 0 && jj < nj) v[t] += rb[((w2 * kWave + l) * 2 + jj) * D + k];
            }
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NE; ++t) {
      const int e = threadIdx.x + t * B;
      if (e < nx.np1 * D) nx.partials[(int64_t)e * nb + bid] = v[t];
    }
  }
}

constexpr int kMfKmvWaves = 4;  // waves per block of sde_mf_kmv_kernel
constexpr int kMfKmvBlock = 64 * kMfKmvWaves;

static int mf_kmv_grid(int64_t N) { return (int)((N + kMfKmvBlock - 1) / kMfKmvBlock); }

static size_t round256(size_t b) { return (b + 255) & ~(size_t)255; }

// workspace: [cp table | stamp partials | (next) noise-sum slab | (next) mf_sums tail workspace]
// per-stamp / total column counts of dim D (host)
static void mf_kmv_cols(int D, int& ns, int& ntot) {
  switch (D) {
#define CASE(DD) case DD: ns = kmv_nstamp<DD>(); ntot = kmv_ntot<DD>(); break;
    CASE(2) CASE(4) CASE(6) CASE(8)
#undef CASE
    default: ns = ntot = 0;
  }
}

// workspace: [cp table | partials (n NS + NTOT columns) | their fp64 sums | (next) noise-sum slab | (next) mf_sums tail]
static size_t mf_kmv_parts(const pdeinv_sde_desc* d, bool nxt, size_t off[5]) {
  const int D = d->dim;
  const int64_t n = d->n_steps;
  const int nb = mf_kmv_grid(d->n_particles);
  const int ncp = (D + 2 + 2 * (D * (D + 1) / 2 + D) + 15) / 16 * 16;  // kmv_ncp_pad
  int ns, ntot;
  mf_kmv_cols(D, ns, ntot);
  const size_t cols = (size_t)n * ns + ntot;
  off[0] = 0;
  off[1] = off[0] + round256((size_t)n * ncp * sizeof(float));
  off[2] = off[1] + round256(cols * nb * sizeof(float));
  off[3] = off[2] + round256(cols * sizeof(double));
  off[4] = off[3] + (nxt ? round256((size_t)(n + 1) * D * nb * sizeof(float)) : 0);
  return off[4] + (nxt ? pdeinv_mf_sums_workspace_bytes(d) : 0);
}

// compact sums -> [mom | wst] per stamp: the per-stamp entries from their columns, the stamp totals on stamp 0 (the
// residual uses them only summed over the stamps), the rest 0
template <int D>
__global__ void kmv_expand_kernel(const double* __restrict__ cs, int64_t n, double* __restrict__ mom,
                                  double* __restrict__ wst) {
  constexpr int M = 2 * D, LZ = moment_len(M), LW = moment_len(D), LT = LZ + LW, NS = kmv_nstamp<D>();
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n * LT) return;
  const int64_t t = q / LT;
  const int e = (int)(q - t * LT);
  const int sc = kmv_source<D>(e);
  double v;
  if (sc >= -2) {
    int col = 0;
    for (int f = 0; f < e; ++f) col += kmv_source<D>(f) >= -2;
    v = cs[t * NS + col];
  } else {
    v = t == 0 ? cs[n * NS + (-3 - sc)] : 0.0;
  }
  if (e < LZ) mom[t * LZ + e] = v;
  else wst[t * LW + (e - LZ)] = v;
}

extern "C" size_t pdeinv_sde_simulate_mf_kmv_workspace_bytes(const pdeinv_sde_desc* d, int32_t with_next) {
  if (!d || d->dim < 2 || d->dim > 8 || d->dim % 2 || d->n_particles <= 0 || d->n_steps < 1) return 0;
  size_t off[5];
  return mf_kmv_parts(d, with_next != 0, off);
}

template <int D, bool NXT>
static void launch_mf_kmv(const SdeArgs& a, const float* z0, float* traj, float* tau, float* last, const float* coef,
                          const KmvStamps& ks, const MfNext& nx, hipStream_t st) {
  hipLaunchKernelGGL(kmv_coef_pairs_kernel<D>, dim3((unsigned)a.n_steps), dim3(128), 0, st, coef, const_cast<float*>(ks.cp));
  hipLaunchKernelGGL((sde_mf_kmv_kernel<D, kMfKmvWaves, NXT>), dim3(mf_kmv_grid(a.N)), dim3(kMfKmvBlock), 0,
                     st, a, z0, traj, tau, last, ks, nx);
}

extern "C" int pdeinv_sde_simulate_mf_kmv(const pdeinv_sde_desc* d, const float* z0, float* traj, float* tau,
                                          float* last, float gamma, const float* coef, double* mom, double* wst,
                                          const pdeinv_sde_desc* next, const float* z0_next, double* sums_next,
                                          void* ws, void* stream) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  PDEINV_REQUIRE(d->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC, PDEINV_ERR_INVALID,
                 "sde_mf_kmv: the potential must be MEANFIELD_QUADRATIC");
  PDEINV_REQUIRE(d->d_meanfield != nullptr, PDEINV_ERR_INVALID,
                 "sde_mf_kmv: McKean–Vlasov needs d_meanfield (pdeinv_mf_mean_path)");
  PDEINV_REQUIRE(d->d_shift_u == nullptr, PDEINV_ERR_INVALID,
                 "sde_mf_kmv: McKean–Vlasov draws its shared tau0 from the stream (shift_u unsupported)");
  PDEINV_REQUIRE(d->d_noise == nullptr, PDEINV_ERR_UNSUPPORTED, "sde_mf_kmv: Philox noise only");
  const int D = d->dim;
  PDEINV_REQUIRE(D % 2 == 0 && D <= 8, PDEINV_ERR_UNSUPPORTED, "sde_mf_kmv: even dim <= 8");
  PDEINV_REQUIRE(std::isfinite(gamma), PDEINV_ERR_INVALID, "sde_mf_kmv: gamma must be finite");
  PDEINV_REQUIRE(d->n_steps <= 65535, PDEINV_ERR_INVALID, "sde_mf_kmv: more than 65535 time stamps");
  const bool nxt = next != nullptr;
  if (nxt) {
    PDEINV_REQUIRE(next->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC, PDEINV_ERR_INVALID,
                   "sde_mf_kmv: the next simulate must be MEANFIELD_QUADRATIC");
    PDEINV_REQUIRE(next->d_noise == nullptr, PDEINV_ERR_UNSUPPORTED, "sde_mf_kmv: Philox noise only");
    PDEINV_REQUIRE(next->dim == d->dim && next->n_particles == d->n_particles &&
                       next->particle_offset == d->particle_offset && next->seed == d->seed &&
                       next->n_steps == d->n_steps,
                   PDEINV_ERR_INVALID, "sde_mf_kmv: the next simulate must differ in its counter offset only");
    PDEINV_REQUIRE(d->n_steps + 1 <= 128, PDEINV_ERR_UNSUPPORTED, "sde_mf_kmv: next sums need n_steps + 1 <= 128");
    PDEINV_REQUIRE(sums_next != nullptr, PDEINV_ERR_INVALID, "sde_mf_kmv: sums_next is null");
  }
  PDEINV_REQUIRE(mom && wst && coef, PDEINV_ERR_INVALID, "sde_mf_kmv: null mom / wst / coef");
  a.xbar = d->d_meanfield;
  a.tau0_mf = shared_tau0_host(a, d);
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = d->n_steps;
  const int LZ = moment_len(2 * D), LW = moment_len(D);
  if (a.N == 0) {
    if (hipMemsetAsync(mom, 0, sizeof(double) * n * LZ, st) != hipSuccess ||
        hipMemsetAsync(wst, 0, sizeof(double) * n * LW, st) != hipSuccess ||
        (nxt && hipMemsetAsync(sums_next, 0, sizeof(double) * mf_sums_len(D, d->n_steps), st) != hipSuccess))
      return fail(PDEINV_ERR_HIP, "sde_mf_kmv: hipMemsetAsync failed");
    return PDEINV_OK;
  }
  PDEINV_REQUIRE(z0 && ws && (!nxt || z0_next), PDEINV_ERR_INVALID, "sde_mf_kmv: null pointer");
  PDEINV_REQUIRE(aligned(traj, 16) && aligned(last, 16) && aligned(tau, 4) && aligned(ws, 256), PDEINV_ERR_INVALID,
                 "sde_mf_kmv: traj/last must be 16-byte aligned, the workspace 256-byte aligned");
  size_t off[5];
  mf_kmv_parts(d, nxt, off);
  KmvStamps ks{};
  ks.cp = (const float*)((char*)ws + off[0]);
  ks.partials = (float*)((char*)ws + off[1]);
  ks.gamma = gamma;
  MfNext nx{};
  if (nxt) {
    nx.partials = (float*)((char*)ws + off[3]);
    nx.ctr_off = next->counter_offset;
    nx.np1 = d->n_steps + 1;
  }
  switch (D) {
#define CASE(DD)                                                                                   \
  case DD:                                                                                         \
    if (nxt) launch_mf_kmv<DD, true>(a, z0, traj, tau, last, coef, ks, nx, st);                    \
    else launch_mf_kmv<DD, false>(a, z0, traj, tau, last, coef, ks, nx, st);                       \
    break;
    CASE(2) CASE(4) CASE(6) CASE(8)
#undef CASE
  }
  rc = check_launch("sde_mf_kmv_kernel");
  if (rc) return rc;
  const int nb = mf_kmv_grid(a.N);
  int ns, ntot;
  mf_kmv_cols(D, ns, ntot);
  double* cs = (double*)((char*)ws + off[2]);
  launch_slab_reduce(ks.partials, nb, (int)(n * ns + ntot), cs, st);
  rc = check_launch("slab_reduce_kernel");
  if (rc) return rc;
  const unsigned eg = (unsigned)((n * (LZ + LW) + 255) / 256);
  switch (D) {
#define CASE(DD) case DD: hipLaunchKernelGGL(kmv_expand_kernel<DD>, dim3(eg), dim3(256), 0, st, cs, n, mom, wst); break;
    CASE(2) CASE(4) CASE(6) CASE(8)
#undef CASE
  }
  rc = check_launch("kmv_expand_kernel");
  if (rc || !nxt) return rc;
  launch_slab_reduce(nx.partials, nb, nx.np1 * D, sums_next + 1 + 2 * D, st);
  rc = check_launch("slab_reduce_kernel");
  if (rc) return rc;
  return mf_sums_tail(next, z0_next, d->n_steps + 1, (char*)ws + off[4], sums_next, st);
}
