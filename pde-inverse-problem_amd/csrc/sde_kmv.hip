// sde_kmv.hip — the McKean–Vlasov simulator fused with the KMV residual's per-time-stamp sums (gfx950).
#include "sde_common.h"

using namespace pdeinv;

// ---- McKean–Vlasov simulate + the KMV residual's per-time-stamp sums (ABI 10) -----------------------------
// The quadratic-Phi KMV residual (kinetic_mckean_vlasov.py:11-120, kmv.hip) reads, per time stamp t = trajectory
// row t, [count, sum z, sum z z^T] of z = [x, v] and the d_s log rho-weighted [sum w, sum w x, sum w x x^T] of x
// (w = d_s^2 log rho + (d_s log rho)^2 + gamma d_s log rho, kinetic_mckean_vlasov.py:243-248). The simulator stages
// each wave's 64 rows of update t in LDS for its coalesced store anyway; here the same staged rows feed two
// v_mfma_f32_16x16x4_f32 products over K = the wave's rows, once per update:
//   P1 = Z^T Z                            the Gram of z (features zero-padded to 16)
//   P2 = A^T Z,  A = [w x (D), w, one, 0..]   sum w x x^T (rows < D), sum w x (row D), sum z (row D + 1)
// (one = 1 on rows < N; staged rows past N are zero). A is staged beside z by each row's own lane, so the MFMA loop
// is two LDS reads and two MFMAs per 4 rows; sum w is a wave sum and the count the block's valid rows. The waves of
// a block add their tiles in LDS in a fixed order (one barrier per update, double-buffered) and the block writes one
// partial column entry per sum (198 at d = 8); slab_reduce sums the blocks in fp64. Deterministic; no trajectory
// re-read (the separate KMV pass reads the 13.4 GB C4 trajectory right after it was written).
// Measured at C4: 5.1 ms without the trajectory against 2.9 + 2.5 ms for simulate + KMV pass;
// the launch is bound by fp32 issue (the f32 MFMA shares the SIMD's issue with the simulator's VALU). A one-tile
// form with lane-private / split-K stamp totals and a spill-free form with chunked scalar operands measured slower.
template <int D>
constexpr int kmv_ncp() { return D + 2 + 2 * (D * (D + 1) / 2 + D); }

struct KmvStamps {
  const float* cp;   // [n_steps][kmv_ncp<D>()]: m1 (D), a1, a2, then (NT + D) coefficient pairs (kmv_coef_pairs_kernel)
  float* partials;   // [(n_steps * (LZ + LW)) columns][gridDim.x]: the mom columns of every stamp, then the wst ones
  float gamma;
};

// The coefficient pairs kmv_moments_weights_kernel builds in LDS per block (kmv.hip), once per stamp into global
// memory: (G1_ij + G1_ji, G2_ij + G2_ji) over the upper triangle (G_ii on the diagonal), then (b1_i, b2_i).
template <int D>
__global__ void kmv_coef_pairs_kernel(const float* __restrict__ coef, float* __restrict__ cp) {
  constexpr int NC = 3 * D + 2 + 2 * D * D, NT = D * (D + 1) / 2, NCP = kmv_ncp<D>();
  const float* c = coef + (int64_t)blockIdx.x * NC;  // [m1, a1, b1, G1, a2, b2, G2]
  float* o = cp + (int64_t)blockIdx.x * NCP;
  for (int e = threadIdx.x; e < NCP; e += blockDim.x) {
    float v;
    if (e < D) {
      v = c[e];
    } else if (e == D) {
      v = c[D];
    } else if (e == D + 1) {
      v = c[2 * D + 1 + D * D];
    } else {
      const int p = (e - D - 2) >> 1, h = (e - D - 2) & 1;
      if (p < NT) {
        int i = 0, rem = p;
        while (rem >= D - i) { rem -= D - i; ++i; }
        const int j = i + rem;
        const float* G = h ? c + 3 * D + 2 + D * D : c + 2 * D + 1;
        v = i == j ? G[i * D + i] : G[i * D + j] + G[j * D + i];
      } else {
        v = h ? c[2 * D + 2 + D * D + (p - NT)] : c[D + 1 + (p - NT)];
      }
    }
    o[e] = v;
  }
}

// w of one row at stamp coefficients cp (scalar loads from the constant address space: no vmcnt wait, which on
// gfx950 would also wait for the trajectory stores in flight). Same operation order as kmv_moments_weights_kernel.
template <int D>
__device__ __forceinline__ float kmv_weight(const float* z, kfloat* cp, float gamma) {
  constexpr int NT = D * (D + 1) / 2;
  float rr[D];
#pragma unroll
  for (int k = 0; k < D; ++k) rr[k] = cp[k] - z[k];  // r = m1 - x
  f32x2 q = f32x2{cp[D], cp[D + 1]};
  int o = 0;
#pragma unroll
  for (int i = 0; i < D; ++i) {  // q += r_i (b_i + sum_{j >= i} Gsym_ij r_j)
    f32x2 g = f32x2{cp[D + 2 + 2 * (NT + i)], cp[D + 3 + 2 * (NT + i)]};
#pragma unroll
    for (int j = i; j < D; ++j, ++o) g = f32x2{cp[D + 2 + 2 * o], cp[D + 3 + 2 * o]} * f32x2{rr[j], rr[j]} + g;
    q = g * f32x2{rr[i], rr[i]} + q;
  }
  return q[1] + q[0] * q[0] + gamma * q[0];
}

// stamp sum e (< LZ + LW, the [mom | wst] order of kmv_moments_weights) -> its word in a wave's two 16 x 16 tiles
// (tile p at p * 256; entry (i, j) is accumulator register i % 4 of lane (i / 4) * 16 + j); -1: the count, -2: sum w
// (neither is a tile entry: the block's valid rows, and a wave sum of w)
template <int D>
__device__ __forceinline__ int kmv_tile_word(int e) {
  constexpr int M = 2 * D, LZ = moment_len(M);
  int p = 1, i = 0, j = 0;
  auto tri = [](int t, int m, int& ii, int& jj) {
    ii = 0;
    while (t >= m - ii) { t -= m - ii; ++ii; }
    jj = ii + t;
  };
  if (e == 0) return -1;                                     // count
  if (e <= M) { i = D + 1; j = e - 1; }                      // sum z_k: the "one" row of A2 against B = z
  else if (e < LZ) { p = 0; tri(e - 1 - M, M, i, j); }       // sum z_i z_j, i <= j
  else if (e == LZ) return -2;                               // sum w
  else if (e <= LZ + D) { i = D; j = e - LZ - 1; }           // sum w x_j: the "w" row of A2
  else { tri(e - LZ - 1 - D, D, i, j); }                     // sum w x_i x_j
  return p * 256 + (((i >> 2) * 16 + j) * 4 + (i & 3));
}

#ifndef PDEINV_MF_KMV_MINW
#define PDEINV_MF_KMV_MINW 1
#endif
template <int D, int WAVES, bool NXT>
__global__ __launch_bounds__(64 * WAVES, PDEINV_MF_KMV_MINW) void sde_mf_kmv_kernel(
    SdeArgs a, const float* __restrict__ z0, float* __restrict__ traj, float* __restrict__ tau,
    float* __restrict__ last, KmvStamps ks, MfNext nx) {
  constexpr int M = 2 * D, B = 64 * WAVES, NCP = kmv_ncp<D>();
  constexpr int LZ = moment_len(M), LW = moment_len(D), LT = LZ + LW, kRed = (LT + B - 1) / B;
  static_assert(D % 2 == 0 && D <= 8, "even dim <= 8: 16-byte staged rows, a 16-feature Gram");
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

  __shared__ float stage[B * M];       // the wave's 64 rows of z (pitch M): store staging, MFMA operand A1 = B1 = B2
  __shared__ float astage[B * 16];     // the wave's 64 rows of A2 = [w x (D), w, one, 0..] (pitch 16)
  __shared__ f32x4 red[2][WAVES][2][kWave];  // per update (double-buffered, one barrier): the waves' two tiles
  __shared__ float wred[2][WAVES];           // per update: the waves' sum of w
  float* slot = stage + wave * kWave * M;
  float* aslot = astage + wave * kWave * 16;

  float z[M];
#pragma unroll
  for (int k = 0; k < M; ++k) z[k] = z0[i * a.ld_z0 + k];

  const int c = lane & 15, rq = lane >> 4;  // operand roles: feature c of rows 4j + rq (A[c][rq] / B[rq][c])
  const int ca = c < M ? c : 0;
  int srcs[kRed];  // the stamp sums this thread adds: e = threadIdx.x + B t
#pragma unroll
  for (int t = 0; t < kRed; ++t) srcs[t] = threadIdx.x + B * t < LT ? kmv_tile_word<D>(threadIdx.x + B * t) : 0;

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
    grad_meanfield<D>(a, z, a.xbar + (int64_t)s * D, g);
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

  // trajectory row s (stamp s): stage z and A2, store the row chunks, the stamp's two tiles of the wave's rows on
  // the matrix pipe, then the block's fixed-order sum of its waves' tiles -> one slab entry per sum
  auto stamp = [&](int s) {
    kfloat* cps = (kfloat*)(ks.cp + (int64_t)s * NCP);
    const bool live = n_valid == kWave || active;  // rows past N stage as zeros (weight 0, one = 0)
    const float w = live ? kmv_weight<D>(z, cps, ks.gamma) : 0.f;
    const float one = live ? 1.f : 0.f;
    float xw[D];
#pragma unroll
    for (int k = 0; k < D; ++k) xw[k] = w * z[k];
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
#pragma unroll
    for (int k = 0; k < 16; k += 4) {
      float q4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int f = k + u;
        q4[u] = f < D ? xw[f < D ? f : 0] : (f == D ? w : (f == D + 1 ? one : 0.f));
      }
      *reinterpret_cast<f32x4*>(aslot + lane * 16 + k) = f32x4{q4[0], q4[1], q4[2], q4[3]};
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
    f32x4 p1 = {0.f, 0.f, 0.f, 0.f}, p2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int row = 4 * j + rq;
      float av = slot[row * M + ca];
      if constexpr (M < 16) av = c < M ? av : 0.f;
      const float a2 = aslot[row * 16 + c];
      p1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, av, p1, 0, 0, 0);
      p2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, av, p2, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    red[s & 1][wave][0][lane] = p1;
    red[s & 1][wave][1][lane] = p2;
    if (lane == 0) wred[s & 1][wave] = wsum;
    __syncthreads();
    const float* r = reinterpret_cast<const float*>(&red[s & 1][0][0][0]);
#pragma unroll
    for (int t = 0; t < kRed; ++t) {
      const int e = threadIdx.x + B * t;
      if (e < LT) {
        float sum = 0.f;
        if (srcs[t] == -1) {
          sum = block_rows;
        } else if (srcs[t] == -2) {
#pragma unroll
          for (int w2 = 0; w2 < WAVES; ++w2) sum += wred[s & 1][w2];
        } else {
#pragma unroll
          for (int w2 = 0; w2 < WAVES; ++w2) sum += r[w2 * 512 + srcs[t]];
        }
        const int64_t cidx = e < LZ ? (int64_t)s * LZ + e : (int64_t)a.n_steps * LZ + (int64_t)s * LW + (e - LZ);
        ks.partials[cidx * nb + bid] = sum;
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

#ifndef PDEINV_MF_KMV_WAVES
#define PDEINV_MF_KMV_WAVES 4  // waves per block of sde_mf_kmv_kernel (the stamp partials shrink with the block)
#endif
constexpr int kMfKmvBlock = 64 * PDEINV_MF_KMV_WAVES;

static int mf_kmv_grid(int64_t N) { return (int)((N + kMfKmvBlock - 1) / kMfKmvBlock); }

static size_t round256(size_t b) { return (b + 255) & ~(size_t)255; }

// workspace: [cp table | stamp partials | (next) noise-sum slab | (next) mf_sums tail workspace]
static size_t mf_kmv_parts(const pdeinv_sde_desc* d, bool nxt, size_t off[4]) {
  const int D = d->dim;
  const int64_t n = d->n_steps;
  const int nb = mf_kmv_grid(d->n_particles);
  const int ncp = D + 2 + 2 * (D * (D + 1) / 2 + D);
  const size_t lt = (size_t)moment_len(2 * D) + moment_len(D);
  off[0] = 0;
  off[1] = off[0] + round256((size_t)n * ncp * sizeof(float));
  off[2] = off[1] + round256((size_t)n * lt * nb * sizeof(float));
  off[3] = off[2] + (nxt ? round256((size_t)(n + 1) * D * nb * sizeof(float)) : 0);
  return off[3] + (nxt ? pdeinv_mf_sums_workspace_bytes(d) : 0);
}

extern "C" size_t pdeinv_sde_simulate_mf_kmv_workspace_bytes(const pdeinv_sde_desc* d, int32_t with_next) {
  if (!d || d->dim < 2 || d->dim > 8 || d->dim % 2 || d->n_particles <= 0 || d->n_steps < 1) return 0;
  size_t off[4];
  return mf_kmv_parts(d, with_next != 0, off);
}

template <int D, bool NXT>
static void launch_mf_kmv(const SdeArgs& a, const float* z0, float* traj, float* tau, float* last, const float* coef,
                          const KmvStamps& ks, const MfNext& nx, hipStream_t st) {
  hipLaunchKernelGGL(kmv_coef_pairs_kernel<D>, dim3((unsigned)a.n_steps), dim3(128), 0, st, coef, const_cast<float*>(ks.cp));
  hipLaunchKernelGGL((sde_mf_kmv_kernel<D, PDEINV_MF_KMV_WAVES, NXT>), dim3(mf_kmv_grid(a.N)), dim3(kMfKmvBlock), 0,
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
  size_t off[4];
  mf_kmv_parts(d, nxt, off);
  KmvStamps ks{};
  ks.cp = (const float*)((char*)ws + off[0]);
  ks.partials = (float*)((char*)ws + off[1]);
  ks.gamma = gamma;
  MfNext nx{};
  if (nxt) {
    nx.partials = (float*)((char*)ws + off[2]);
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
  launch_slab_reduce(ks.partials, nb, (int)(n * LZ), mom, st);
  launch_slab_reduce(ks.partials + n * LZ * nb, nb, (int)(n * LW), wst, st);
  rc = check_launch("slab_reduce_kernel");
  if (rc || !nxt) return rc;
  launch_slab_reduce(nx.partials, nb, nx.np1 * D, sums_next + 1 + 2 * D, st);
  rc = check_launch("slab_reduce_kernel");
  if (rc) return rc;
  return mf_sums_tail(next, z0_next, d->n_steps + 1, (char*)ws + off[3], sums_next, st);
}
