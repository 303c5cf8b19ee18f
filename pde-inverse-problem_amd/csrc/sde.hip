// sde.hip — the Euler–Maruyama particle simulator (gfx950).
//
// Replaces utils/sampling_utils.py:25-52 (underdamped_langevin_dynamics_scan, vmapped over
// particles, lax.scan over steps) and update_step :6-22. XLA runs one scan body per step and
// round-trips the state through HBM each time; here one thread owns one particle for all
// n_steps+1 updates, the state lives in VGPRs, the noise is Philox4x32-10 in registers, and
// the only HBM traffic is the z0 read and the time-major trajectory / tau / last stores
// ((8d + 4) B per particle-update).
//
// Optionally the same kernel accumulates the moment sets (initial = z0, 0T = traj,
// terminal = last) that the parametric-quadratic residual needs, so the KFP residual
// (kinetic_fokker_planck.py:33-58) costs no second pass over the trajectory.
#include <math.h>
#include <stddef.h>
#include <stdlib.h>

#include <type_traits>

#include "sde_common.h"

namespace pdeinv {


template <int D>
__device__ __forceinline__ void grad_quadratic(const SdeArgs& a, const float* q, float* g) {
  if constexpr (D * D + D > 32) {
    kfloat* P = kernarg_params();
#pragma unroll
    for (int r = 0; r < D; ++r) {
      float acc = -P[D * D + r];
#pragma unroll
      for (int c = 0; c < D; ++c) acc = fmaf(P[r * D + c], q[c], acc);
      g[r] = acc;
    }
  } else {
#pragma unroll
    for (int r = 0; r < D; ++r) {
      float acc = -a.params[D * D + r];
#pragma unroll
      for (int c = 0; c < D; ++c) acc = fmaf(a.params[r * D + c], q[c], acc);
      g[r] = acc;
    }
  }
}

// grad of U = -logsumexp_k(-|q-mu_k|^2/(2 s^2)): gmm_grad (common.h), packed over centre pairs.
// Softmax logits are shift-invariant, so |q|^2 drops out: in log2 units
// a_k = l2s (q . mu_k) + c_k, l2s = log2e / s^2, c_k = -l2s |mu_k|^2 / 2 — one d-term dot per
// centre. The KM centres live in VGPRs for the whole kernel (pinned once: kept as kernel-argument
// SGPRs they overflow the scalar file and every use costs a v_readlane); unused slots carry
// c_k = -inf, so the softmax needs no per-centre branches.
template <int D, int KM>
struct GmmCentres {
  GmmPairs<D, KM> g;
  __device__ __forceinline__ void load(const SdeArgs& a) {
#pragma unroll
    for (int p = 0; p < KM / 2; ++p) {
#pragma unroll
      for (int i = 0; i < D; ++i) {
        g.mu[p][i] = f32x2{2 * p < a.K ? a.params[2 * p * D + i] : 0.f, 2 * p + 1 < a.K ? a.params[(2 * p + 1) * D + i] : 0.f};
        asm volatile("" : "+v"(g.mu[p][i]));
      }
      g.c[p] = f32x2{2 * p < a.K ? a.params[kMaxGmmK * D + 2 * p] : -INFINITY,
                     2 * p + 1 < a.K ? a.params[kMaxGmmK * D + 2 * p + 1] : -INFINITY};
      asm volatile("" : "+v"(g.c[p]));
    }
  }
};




// Wave-cooperative store of 64 consecutive rows [wave_row0, wave_row0 + 64) of M floats:
// row -> LDS (lane-private 4M bytes), then 16-byte chunk c = k*64 + lane -> global. Rows at or
// beyond n_valid are not stored. LDS traffic of one wave only: no barrier needed.
template <int D>
__device__ __forceinline__ void store_rows_staged(float* wave_dst, const float* z, float* slot,
                                                  int lane, int n_valid) {
  constexpr int M = 2 * D;
  static_assert(M % 4 == 0, "staged stores need 2d % 4 == 0");
#pragma unroll
  for (int k = 0; k < M; k += 4)
    *reinterpret_cast<f32x4*>(slot + lane * M + k) = f32x4{z[k], z[k + 1], z[k + 2], z[k + 3]};
  __builtin_amdgcn_wave_barrier();
  f32x4 v[M / 4];
#pragma unroll
  for (int k = 0; k < M / 4; ++k) v[k] = *reinterpret_cast<const f32x4*>(slot + 4 * (k * 64 + lane));
  if (n_valid == kWave) {  // wave-uniform: every full wave stores unguarded (one lgkmcnt wait)
#pragma unroll
    for (int k = 0; k < M / 4; ++k)
      __builtin_nontemporal_store(v[k], reinterpret_cast<f32x4*>(wave_dst + 4 * (k * 64 + lane)));
  } else {
#pragma unroll
    for (int k = 0; k < M / 4; ++k) {
      const int c = k * 64 + lane;  // 16-byte chunk within the wave's 64*M floats
      if (4 * c < n_valid * M) __builtin_nontemporal_store(v[k], reinterpret_cast<f32x4*>(wave_dst + 4 * c));
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// The mirror image: 16-byte chunks of the wave's 64 consecutive rows -> LDS (coalesced), then
// each lane reads its own row. Rows at or beyond n_valid read as zero.
template <int D>
__device__ __forceinline__ void load_rows_staged(const float* wave_src, float* z, float* slot, int lane,
                                                 int n_valid) {
  constexpr int M = 2 * D;
  static_assert(M % 4 == 0, "staged loads need 2d % 4 == 0");
#pragma unroll
  for (int k = 0; k < M / 4; ++k) {
    const int c = k * 64 + lane;
    const f32x4 v = (4 * c < n_valid * M) ? *reinterpret_cast<const f32x4*>(wave_src + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(slot + 4 * c) = v;
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < M; k += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(slot + lane * M + k);
    z[k] = v[0];
    z[k + 1] = v[1];
    z[k + 2] = v[2];
    z[k + 3] = v[3];
  }
  __builtin_amdgcn_wave_barrier();
}


__device__ __forceinline__ float shift_u(const SdeArgs& a, uint32_t plo, uint32_t phi, int64_t i) {
  if (a.shift_u) return a.shift_u[i];
  const uint4 r = philox4x32_10(make_uint4(plo, phi, a.ctr_off, 0x80000000u), a.k0, a.k1);
  return u32_unit(r.x);
}

// KFP residual of a GMM model fused into the GMM simulator (RES): the reference's online KFP-GMM
// iteration simulates (…_GMM.py:104-142) and then evaluates kinetic_fokker_planck.py:11-69 over
// initial = z0, 0T = every trajectory row, terminal = last. Here each particle's rows are consumed
// in registers as they are produced — the trajectory is never re-read — and grad V* of a 0T row is
// the simulator's own grad U at that state (computed by the next update anyway), so only the model
// softmax and its adjoint are extra work. Coefficients as pdeinv_kfp_gmm_desc.
struct GmmResFused {
  const float* mus;  // model centres [K, d] (device)
  int32_t K;
  float s2, l2s;     // model 1/sigma^2, log2(e)/sigma^2
  float c_nabla, c_hess, c_fric, c_true, c_init, c_term, inv_ni, inv_nt;
};


// SdeArgs must stay the FIRST parameter: kernarg_params() reads a.params at kernarg offset 0.
template <int D, int POT, bool MOM, int STORE, int KM = 1, bool NOISE = false, int MINW = 1, bool RES = false,
          bool NXT = false>
__global__ __launch_bounds__(kBlock, MINW) void sde_simulate_kernel(SdeArgs a, const float* __restrict__ z0,
                                                              float* __restrict__ traj,
                                                              float* __restrict__ tau,
                                                              float* __restrict__ last,
                                                              float* __restrict__ partials,
                                                              GmmResFused rf = GmmResFused{},
                                                              MfNext nx = MfNext{}) {
  constexpr int M = 2 * D;
  static_assert(!RES || (POT == PDEINV_POT_GMM && !MOM), "the fused residual is the GMM simulator's");
  static_assert(!NXT || (POT == PDEINV_POT_MEANFIELD_QUADRATIC && !NOISE && M % 4 == 0 && D <= 8),
                "next-simulate sums: McKean–Vlasov, Philox noise, even dim <= 8 (staged stores)");
  const int bid = a.remap ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int64_t i_raw = (int64_t)bid * kBlock + threadIdx.x;
  const bool active = i_raw < a.N;
  const int64_t i = active ? i_raw : a.N - 1;  // inactive lanes compute on a valid row, store nothing
  const float w = active ? 1.f : 0.f;
  const uint64_t gid = (uint64_t)(a.poff + i);
  const uint32_t plo = (uint32_t)gid, phi = (uint32_t)(gid >> 32);

  float z[M];
#pragma unroll
  for (int k = 0; k < M; ++k) z[k] = z0[i * a.ld_z0 + k];
  [[maybe_unused]] GmmCentres<D, (KM > 1 ? KM : 2)> centres;
  if constexpr (POT == PDEINV_POT_GMM && !RES) centres.load(a);

  __shared__ float lds[kWavesPerBlock * moment_len(M > 16 ? 2 : M)];
  const int nb = gridDim.x;
  constexpr int L = moment_len(M > 16 ? 2 : M);
  if constexpr (MOM) {
    MomentAcc<M> init;
    init.zero();
    init.add(z, w);
    block_reduce_to_slab(init.v, L, lds, partials, bid, nb);
  }

  // fused GMM residual state: the true (simulated) and the model GMM in centre-pair layout (common.h
  // GmmPairs) in LDS, read with wave-uniform broadcasts — in VGPRs they would take 2 (K d + K)
  // registers and, beside the adjoint accumulators, leave one wave per SIMD.
  __shared__ GmmPairs<D, (KM > 1 ? KM : 2)> lcen_s[RES ? 2 : 1];
  [[maybe_unused]] auto& lcen = lcen_s[0];
  [[maybe_unused]] auto& lmod = lcen_s[RES ? 1 : 0];
  constexpr int KR = KM > 1 ? KM : 2;
  [[maybe_unused]] float racc[PDEINV_GMM_NACC];
  [[maybe_unused]] GmmAdjAcc<D, KR> radj;
  if constexpr (RES) {
    for (int k = threadIdx.x; k < KM; k += kBlock) {
      // the simulator's packed constants (build_args) for the true GMM; the model's from its centres
      lcen.set(k, a.K, a.params, a.l2s);
      if (k < a.K) reinterpret_cast<float*>(&lcen.c[k / 2])[k % 2] = a.params[kMaxGmmK * D + k];
      lmod.set(k, rf.K, rf.mus, rf.l2s);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < PDEINV_GMM_NACC; ++c) racc[c] = 0.f;
    radj.zero();
  }
  // set 0 = 0T (gt = grad V* at the row), 1 = initial, 2 = terminal; w = 0 for lanes past N
  [[maybe_unused]] auto res_add = [&](const float* zz, const float* gt, int set) {
    if constexpr (RES) {
      const float c1 = set == 0 ? w * rf.c_nabla : 0.f;
      const float c2 = set == 0 ? w * rf.c_hess : 0.f;
      const float c3 = w * (set == 0 ? rf.c_fric : (set == 1 ? rf.c_init : rf.c_term));
      float gm[D], T1, T2, T3;
      gmm_residual_sample<D, KR>(lmod.mu, lmod.c, rf.s2, rf.l2s, zz, zz + D, c1, c2, c3, radj, gm, T1, T2, T3);
      racc[PDEINV_GMM_ACC_LOSS] += c1 * T1 + c2 * T2 + c3 * T3;
      if (set == 0) {
        float Tt = 0.f, Tgt = 0.f;
#pragma unroll
        for (int c = 0; c < D; ++c) {
          Tt = fmaf(gt[c], gt[c], Tt);
          Tgt = fmaf(gt[c] - gm[c], gt[c] - gm[c], Tgt);
        }
        const float ct = w * rf.c_true;
        racc[PDEINV_GMM_ACC_LOSS] += ct * Tt;
        racc[PDEINV_GMM_ACC_LOSS_GT] += ct * Tgt;
        racc[PDEINV_GMM_ACC_NABLA] += ct * T1;
        racc[PDEINV_GMM_ACC_HESSIAN] += ct * T2;
        racc[PDEINV_GMM_ACC_FRICTION] += ct * T3;
        racc[PDEINV_GMM_ACC_NABLA_TRUE] += ct * Tt;
      } else if (set == 1) {
        racc[PDEINV_GMM_ACC_INITIAL] += w * rf.inv_ni * T3;
      } else {
        racc[PDEINV_GMM_ACC_TERMINAL] += w * rf.inv_nt * T3;
      }
    }
  };

  const float tau0 = (POT == PDEINV_POT_MEANFIELD_QUADRATIC) ? a.tau0_mf
                                                              : (a.random_shift ? shift_u(a, plo, phi, i) * a.dt : 0.f);
  const float h_last = a.dt - tau0;

  constexpr bool kStaged = (STORE == kStoreStaged) && (M % 4 == 0);
  PairGram<(MOM ? M : 2)> acc;  // the 0T moments, lane-private (sharing them over lane quads measured slower, §4.6)
  acc.zero();

  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave_row0 = i_raw - lane;
  // wave-uniform by construction; readfirstlane lets the compiler branch on it with SALU
  const int n_valid = __builtin_amdgcn_readfirstlane((int)((a.N - wave_row0) < kWave ? (a.N - wave_row0) : kWave));
  __shared__ float stage[kStaged ? kBlock * M : 1];
  float* slot = stage + (threadIdx.x - lane) * M;
  float* tr = traj ? traj + (kStaged ? wave_row0 : i) * M : nullptr;
  float* ta = tau ? tau + i : nullptr;
  const int64_t tr_stride = a.N * M;
  auto put = [&](float* dst) {
    if constexpr (kStaged) store_rows_staged<D>(dst, z, slot, lane, n_valid);
    else if (active) store_row<D, STORE>(dst, z);
  };
  [[maybe_unused]] float nacc[NXT ? 3 : 1][NXT ? D : 1];
  [[maybe_unused]] const int nbase = NXT ? lane * nx.np1 : 0;  // the lane's first pair
  if constexpr (NXT) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < D; ++k) nacc[j][k] = 0.f;
  }

  auto update = [&](float h, float sh, uint32_t s) {
    // RES: re-read the LDS centres every update (hoisted out of the step loop they would take the
    // registers this layout exists to save)
    if constexpr (RES) asm volatile("" ::: "memory");
    float g[D], xi[D];
    if constexpr (POT == PDEINV_POT_GMM && RES) gmm_grad<D, KR>(lcen.mu, lcen.c, a.l2s, a.inv_s2, z, g);
    else if constexpr (POT == PDEINV_POT_GMM) gmm_grad<D, KR>(centres.g.mu, centres.g.c, a.l2s, a.inv_s2, z, g);
    else if constexpr (POT == PDEINV_POT_MEANFIELD_QUADRATIC) grad_meanfield<D>(a, z, a.xbar + (int64_t)s * D, g);
    else grad_quadratic<D>(a, z, g);
    if constexpr (RES) {
      if (s == 0) res_add(z, g, 1);  // z0: the initial set
      else res_add(z, g, 0);         // traj row s-1 (g = grad V* there): the 0T set
    }
    gen_normals<D, NOISE>(a, plo, phi, s, i, xi);
    if constexpr (NXT) {  // pair q = nbase + s of the next simulate: update q / 64 of particle wave_row0 + q % 64
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
      // p' = p - h*gradU + sqrt(h)*ns*xi - gamma*p*h ; q' = q + h*p'  (sampling_utils.py:17,20)
      const float pn = fmaf(-gh, p, fmaf(sh, xi[k], fmaf(-h, g[k], p)));
      z[D + k] = pn;
      z[k] = fmaf(h, pn, z[k]);
    }
  };

  // update 0: h = tau0 (sample at tau0)
  update(tau0, sqrtf(tau0) * a.ns, 0u);
  if (tr) put(tr);
  if (active && ta) __builtin_nontemporal_store(tau_value(tau0, 0, a.dt), ta);
  if constexpr (MOM) acc.add(z);

  const float sh_dt = sqrtf(a.dt) * a.ns;
  for (int s = 1; s < a.n_steps; ++s) {
    update(a.dt, sh_dt, (uint32_t)s);
    if (tr) put(tr + (int64_t)s * tr_stride);
    if (active && ta) __builtin_nontemporal_store(tau_value(tau0, s, a.dt), ta + (int64_t)s * a.N);
    if constexpr (MOM) acc.add(z);
  }

  // final update: h = dt - tau0, lands exactly at T = n*dt (sampling_utils.py:44-46)
  update(h_last, sqrtf(h_last) * a.ns, (uint32_t)a.n_steps);
  if (active && last) store_row<D, kStoreNT>(last + i * M, z);
  if constexpr (NXT) {
    // the block's slab column per update: through the (now free) staging buffer in two passes (running sums
    // 0-1, then 2; 4 waves x 64 lanes x 2 x D floats = the buffer), fixed order: pass, wave, lane
    float* red = stage;
    const int wv = threadIdx.x >> 6;
    constexpr int NE = (128 * D + kBlock - 1) / kBlock;
    float v[NE];
#pragma unroll
    for (int t = 0; t < NE; ++t) v[t] = 0.f;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int j0 = 2 * pass, nj = pass ? 1 : 2;
      __syncthreads();  // every wave is done with the buffer (its staged stores / the previous pass)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        if (jj < nj) {
#pragma unroll
          for (int k = 0; k < D; ++k) red[((wv * kWave + lane) * 2 + jj) * D + k] = nacc[j0 + jj][k];
        }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < NE; ++t) {
        const int e = threadIdx.x + t * kBlock;
        if (e < nx.np1 * D) {
          const int sp = e / D, k = e - sp * D;
          const int l0 = (64 * sp) / nx.np1, l1 = (64 * sp + 63) / nx.np1;  // the lanes that drew update sp
          for (int w2 = 0; w2 < kWavesPerBlock; ++w2)
            for (int l = l0; l <= l1; ++l) {
              const int jj = sp - ((l * nx.np1) >> 6) - j0;
              if (jj >= 0 && jj < nj) v[t] += red[((w2 * kWave + l) * 2 + jj) * D + k];
            }
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NE; ++t) {
      const int e = threadIdx.x + t * kBlock;
      if (e < nx.np1 * D) nx.partials[(int64_t)e * nb + bid] = v[t];
    }
  }
  if constexpr (RES) {
    res_add(z, z, 2);  // last: the terminal set
    constexpr int NR = PDEINV_GMM_NACC + KR * D;
    float flat[NR];
#pragma unroll
    for (int c = 0; c < PDEINV_GMM_NACC; ++c) flat[c] = racc[c];
    gmm_adjoint_flat<D, KR>(radj, lmod.mu, flat + PDEINV_GMM_NACC);
    __shared__ float rlds[kWavesPerBlock * NR];
    block_reduce_to_slab(flat, PDEINV_GMM_NACC + rf.K * D, rlds, partials, bid, nb);
  }

  if constexpr (MOM) {
    float mv[L];
    acc.finish((float)a.n_steps, w, mv);
    block_reduce_to_slab(mv, L, lds, partials + (int64_t)L * nb, bid, nb);
    MomentAcc<M> term;
    term.zero();
    term.add(z, w);
    block_reduce_to_slab(term.v, L, lds, partials + (int64_t)2 * L * nb, bid, nb);
  }
}

// Compile-time guard of the kernarg_params() invariant: the kernel's first parameter is SdeArgs (so its
// params field sits at kernarg offset offsetof(SdeArgs, params)), checked on a quadratic and a mean-field
// instantiation; the struct must be standard-layout for offsetof to be that offset.
template <typename F>
struct first_param;
template <typename R, typename A0, typename... As>
struct first_param<R (*)(A0, As...)> {
  using type = A0;
};
static_assert(std::is_standard_layout<SdeArgs>::value, "kernarg_params(): SdeArgs must be standard-layout");
static_assert(std::is_same<first_param<decltype(&sde_simulate_kernel<4, PDEINV_POT_QUADRATIC, false, 2>)>::type,
                           SdeArgs>::value &&
                  std::is_same<first_param<decltype(&sde_simulate_kernel<8, PDEINV_POT_MEANFIELD_QUADRATIC, false, 2>)>::type,
                               SdeArgs>::value,
              "kernarg_params() reads SdeArgs::params at its kernarg offset: SdeArgs must stay the first parameter "
              "of sde_simulate_kernel");

// ---- McKean–Vlasov single update ---------------------------------------------------------
// grad U(q_i) = A (q_i - xbar) with xbar = (sum x)/count of the ensemble BEFORE this update
// (the pairwise mean  mean_j grad Phi*(x_i - x_j) of kinetic_mckean_vlasov.py:20-23 for
// quadratic Phi*, evaluated in O(N)). Emits [count, sum x_new] partials for the next update.
template <int D>
__global__ __launch_bounds__(kBlock) void mf_step_kernel(SdeArgs a, int s, float tau0,
                                                         const float* __restrict__ zin,
                                                         float* __restrict__ zout,
                                                         float* __restrict__ tau_row,
                                                         const double* __restrict__ xbar_sum,
                                                         float* __restrict__ partials) {
  constexpr int M = 2 * D;
  constexpr bool kStaged = (M % 4 == 0);
  const int64_t i_raw = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = i_raw < a.N;
  const int64_t i = active ? i_raw : a.N - 1;
  const uint64_t gid = (uint64_t)(a.poff + i);
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave_row0 = i_raw - lane;
  const int n_valid = (int)((a.N - wave_row0) < kWave ? (a.N - wave_row0) : kWave);
  __shared__ float stage[kStaged ? kBlock * M : 1];
  float* slot = stage + (threadIdx.x - lane) * M;
  // zero-initialised: a wave wholly past N (n_valid <= 0) skips the staged load, and its lanes must
  // not feed garbage (0 * Inf = NaN) into the block's Σx partials below
  float z[M] = {};
  if constexpr (kStaged) {
    if (n_valid > 0) load_rows_staged<D>(zin + wave_row0 * M, z, slot, lane, n_valid);
  } else {
#pragma unroll
    for (int k = 0; k < M; ++k) z[k] = zin[i * M + k];
  }
  const double cnt = xbar_sum[0];
  float y[D];
#pragma unroll
  for (int k = 0; k < D; ++k) y[k] = z[k] - (float)(xbar_sum[1 + k] / cnt);
  float g[D];
#pragma unroll
  for (int r = 0; r < D; ++r) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) acc = fmaf(a.params[r * D + c], y[c], acc);
    g[r] = acc;
  }
  float xi[D];
  if (a.noise) gen_normals<D, true>(a, (uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)s, i, xi);
  else gen_normals<D, false>(a, (uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)s, i, xi);
  const float h = (s == 0) ? tau0 : ((s == a.n_steps) ? a.dt - tau0 : a.dt);
  const float sh = sqrtf(h) * a.ns;
  const float gh = a.gamma * h;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const float p = z[D + k];
    const float pn = fmaf(-gh, p, fmaf(sh, xi[k], fmaf(-h, g[k], p)));
    z[D + k] = pn;
    z[k] = fmaf(h, pn, z[k]);
  }
  if constexpr (kStaged) {
    if (n_valid > 0) store_rows_staged<D>(zout + wave_row0 * M, z, slot, lane, n_valid);
  } else if (active) {
    store_row<D, kStoreNT>(zout + i * M, z);
  }
  if (active && tau_row) tau_row[i] = tau_value(tau0, s, a.dt);
  float v[1 + D];
  v[0] = active ? 1.f : 0.f;
#pragma unroll
  for (int k = 0; k < D; ++k) v[1 + k] = active ? z[k] : 0.f;  // a select, not 0 * z
  __shared__ float lds[kWavesPerBlock * (1 + D)];
  block_reduce_to_slab(v, 1 + D, lds, partials, blockIdx.x, gridDim.x);
}

__global__ void tau0_kernel(SdeArgs a, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.N) return;
  const uint64_t gid = (uint64_t)(a.poff + i);
  out[i] = a.random_shift ? shift_u(a, (uint32_t)gid, (uint32_t)(gid >> 32), i) * a.dt : 0.f;
}

// ---- host side ----------------------------------------------------------------------------

static int sim_grid(int64_t N) { return grid_for(N); }

}  // namespace pdeinv

using namespace pdeinv;

extern "C" int pdeinv_moment_len(int m) { return moment_len(m); }

extern "C" size_t pdeinv_sde_workspace_bytes(const pdeinv_sde_desc* d) {
  if (!d || d->dim < 1 || d->dim > 8 || d->n_particles <= 0) return 0;
  return (size_t)3 * moment_len(2 * d->dim) * sim_grid(d->n_particles) * sizeof(float);
}

template <int D, int POT, bool MOM, int KM = 1>
static void launch_sim(const SdeArgs& a, const float* z0, float* traj, float* tau, float* last,
                       float* ws, hipStream_t st) {
  const dim3 g(sim_grid(a.N)), b(kBlock);
  if (a.noise)
    hipLaunchKernelGGL((sde_simulate_kernel<D, POT, MOM, kStoreStaged, KM, true>), g, b, 0, st, a, z0, traj, tau,
                       last, ws);
  else
    hipLaunchKernelGGL((sde_simulate_kernel<D, POT, MOM, kStoreStaged, KM, false>), g, b, 0, st, a, z0, traj, tau,
                       last, ws);
}

// Occupancy of the fused kernel: at d <= 4 the allocator fits 168 VGPRs (3 waves / SIMD) with a few
// dwords of spill; at d = 8 forcing it spills hundreds, so the compiler chooses.
template <int D> constexpr int kResMinWaves = D <= 4 ? 3 : 1;

template <int D, int KM>
static void launch_sim_res(const SdeArgs& a, const GmmResFused& rf, const float* z0, float* traj, float* tau,
                           float* last, float* ws, hipStream_t st) {
  const dim3 g(sim_grid(a.N)), b(kBlock);
  constexpr int W = kResMinWaves<D>;
  if (a.noise)
    hipLaunchKernelGGL((sde_simulate_kernel<D, PDEINV_POT_GMM, false, kStoreStaged, KM, true, W, true>), g, b, 0, st,
                       a, z0, traj, tau, last, ws, rf);
  else
    hipLaunchKernelGGL((sde_simulate_kernel<D, PDEINV_POT_GMM, false, kStoreStaged, KM, false, W, true>), g, b, 0,
                       st, a, z0, traj, tau, last, ws, rf);
}

template <int D, bool MOM>
static void launch_gmm_sim(const SdeArgs& a, const float* z0, float* traj, float* tau, float* last, float* ws,
                           hipStream_t st) {
  if (a.K <= 4) launch_sim<D, PDEINV_POT_GMM, MOM, 4>(a, z0, traj, tau, last, ws, st);
  else if (a.K <= 8) launch_sim<D, PDEINV_POT_GMM, MOM, 8>(a, z0, traj, tau, last, ws, st);
  else launch_sim<D, PDEINV_POT_GMM, MOM, 16>(a, z0, traj, tau, last, ws, st);
}

template <int D>
static int dispatch_sim(const SdeArgs& a, int pot, bool mom, const float* z0, float* traj,
                        float* tau, float* last, float* ws, hipStream_t st) {
  if (pot == PDEINV_POT_MEANFIELD_QUADRATIC) {
    launch_sim<D, PDEINV_POT_MEANFIELD_QUADRATIC, false>(a, z0, traj, tau, last, ws, st);
    return 0;
  }
  if (pot == PDEINV_POT_GMM) {
    if constexpr (D <= 8) {
      if (mom) { launch_gmm_sim<D, true>(a, z0, traj, tau, last, ws, st); return 0; }
    }
    launch_gmm_sim<D, false>(a, z0, traj, tau, last, ws, st);
  } else {
    if constexpr (D <= 8) {
      if (mom) { launch_sim<D, PDEINV_POT_QUADRATIC, true>(a, z0, traj, tau, last, ws, st); return 0; }
    }
    launch_sim<D, PDEINV_POT_QUADRATIC, false>(a, z0, traj, tau, last, ws, st);
  }
  return 0;
}



extern "C" int pdeinv_sde_simulate(const pdeinv_sde_desc* d, const float* z0, float* traj,
                                   float* tau, float* last, void* ws, double* moments,
                                   void* stream) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  const int D = d->dim;
  const bool mom = moments != nullptr;
  if (d->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC) {
    // the fused multi-step McKean–Vlasov path needs the mean path xbar [n+1, d] (pdeinv_mf_sums ->
    // all-reduce -> pdeinv_mf_mean_path); without it the ensemble runs update by update (pdeinv_mf_step)
    PDEINV_REQUIRE(d->d_meanfield != nullptr, PDEINV_ERR_INVALID,
                   "sde: McKean–Vlasov needs d_meanfield (pdeinv_mf_mean_path) or pdeinv_mf_step");
    PDEINV_REQUIRE(d->d_shift_u == nullptr, PDEINV_ERR_INVALID,
                   "sde: McKean–Vlasov draws its shared tau0 from the stream (shift_u unsupported)");
    PDEINV_REQUIRE(!mom, PDEINV_ERR_UNSUPPORTED, "sde: fused KFP moments are not defined for McKean–Vlasov");
    a.xbar = d->d_meanfield;
    a.tau0_mf = shared_tau0_host(a, d);
  }
  PDEINV_REQUIRE(!mom || D <= 8, PDEINV_ERR_UNSUPPORTED, "sde: fused moments need dim <= 8");
  hipStream_t st = (hipStream_t)stream;
  const int L = moment_len(2 * D);
  if (a.N == 0) {
    if (mom && hipMemsetAsync(moments, 0, sizeof(double) * 3 * L, st) != hipSuccess)
      return fail(PDEINV_ERR_HIP, "sde: hipMemsetAsync failed");
    return PDEINV_OK;
  }
  PDEINV_REQUIRE(z0 != nullptr, PDEINV_ERR_INVALID, "sde: z0 is null");
  PDEINV_REQUIRE(!mom || ws != nullptr, PDEINV_ERR_INVALID, "sde: moments need a workspace");
  const size_t va = (D % 2 == 0) ? 16 : 8;
  PDEINV_REQUIRE(aligned(traj, va) && aligned(last, va) && aligned(tau, 4), PDEINV_ERR_INVALID,
                 "sde: traj/last must be 16-byte (even dim) or 8-byte (odd dim) aligned");
  float* wsf = (float*)ws;
  switch (D) {
#define CASE(DD) case DD: dispatch_sim<DD>(a, d->potential.kind, mom, z0, traj, tau, last, wsf, st); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(10) CASE(12) CASE(16)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "sde: dim must be one of 1-8, 10, 12, 16");
  }
  rc = check_launch("sde_simulate_kernel");
  if (rc) return rc;
  if (mom) {
    launch_slab_reduce(wsf, sim_grid(a.N), 3 * L, moments, st);
    rc = check_launch("slab_reduce_kernel");
  }
  return rc;
}

static int gmm_res_km(int K) { return K <= 4 ? 4 : (K <= 8 ? 8 : 16); }

extern "C" size_t pdeinv_sde_simulate_kfp_gmm_workspace_bytes(const pdeinv_sde_desc* d, const pdeinv_kfp_gmm_desc* r) {
  if (!d || !r || d->dim < 1 || d->dim > 8 || d->n_particles <= 0 || r->n_centers < 1) return 0;
  return (size_t)(PDEINV_GMM_NACC + r->n_centers * d->dim) * sim_grid(d->n_particles) * sizeof(float);
}

extern "C" int pdeinv_sde_simulate_kfp_gmm(const pdeinv_sde_desc* d, const pdeinv_kfp_gmm_desc* r, const float* mus,
                                           const float* z0, float* traj, float* tau, float* last, void* ws, double* acc,
                                           void* stream) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  PDEINV_REQUIRE(r != nullptr, PDEINV_ERR_INVALID, "sde_kfp_gmm: null residual descriptor");
  const int D = d->dim;
  PDEINV_REQUIRE(d->potential.kind == PDEINV_POT_GMM, PDEINV_ERR_INVALID, "sde_kfp_gmm: the simulated potential must be GMM");
  PDEINV_REQUIRE(r->dim == D, PDEINV_ERR_INVALID, "sde_kfp_gmm: residual dim != simulator dim");
  PDEINV_REQUIRE(D <= 8, PDEINV_ERR_UNSUPPORTED, "sde_kfp_gmm: dim must be <= 8");
  PDEINV_REQUIRE(r->n_centers >= 1 && r->n_centers <= kMaxGmmK && r->n_centers * D <= 64, PDEINV_ERR_UNSUPPORTED,
                 "sde_kfp_gmm: need 1 <= model n_centers <= 16 and n_centers * dim <= 64");
  // grad V* of a 0T row is the simulator's grad U there: the true potential must be the simulated one
  bool same = r->n_centers_true == d->potential.n_centers && r->sigma_true == d->potential.sigma && r->mus_true;
  for (int k = 0; same && k < r->n_centers_true * D; ++k) same = r->mus_true[k] == d->potential.params[k];
  PDEINV_REQUIRE(same, PDEINV_ERR_INVALID, "sde_kfp_gmm: the residual's true GMM must be the simulated potential");
  PDEINV_REQUIRE(std::isfinite(r->sigma) && r->sigma > 0.f, PDEINV_ERR_INVALID, "sde_kfp_gmm: model sigma must be > 0");
  hipStream_t st = (hipStream_t)stream;
  PDEINV_REQUIRE(acc != nullptr, PDEINV_ERR_INVALID, "sde_kfp_gmm: acc is null");
  if (a.N == 0) {
    if (hipMemsetAsync(acc, 0, sizeof(double) * (PDEINV_GMM_NACC + r->n_centers * D), st) != hipSuccess)
      return fail(PDEINV_ERR_HIP, "sde_kfp_gmm: hipMemsetAsync failed");
    return PDEINV_OK;
  }
  PDEINV_REQUIRE(z0 && mus && ws, PDEINV_ERR_INVALID, "sde_kfp_gmm: null pointer");
  const size_t va = (D % 2 == 0) ? 16 : 8;
  PDEINV_REQUIRE(aligned(traj, va) && aligned(last, va) && aligned(tau, 4), PDEINV_ERR_INVALID,
                 "sde_kfp_gmm: traj/last must be 16-byte (even dim) or 8-byte (odd dim) aligned");
  GmmResFused rf{};
  rf.mus = mus;
  rf.K = r->n_centers;
  rf.s2 = 1.f / (r->sigma * r->sigma);
  rf.l2s = rf.s2 * 1.4426950408889634f;
  rf.c_nabla = r->c_nabla; rf.c_hess = r->c_hess; rf.c_fric = r->c_fric; rf.c_true = r->c_true;
  rf.c_init = r->c_init; rf.c_term = r->c_term;
  // the boundary sets are this call's z0 and last rows: their per-set means use the GLOBAL set sizes
  // folded into c_init / c_term by the caller; INITIAL / TERMINAL report sum T3 / N of this call
  rf.inv_ni = 1.f / (float)a.N;
  rf.inv_nt = 1.f / (float)a.N;
  const int km = gmm_res_km(a.K > rf.K ? a.K : rf.K);
  float* wsf = (float*)ws;
  switch (D) {
#define CASE(DD)                                                                          \
  case DD:                                                                                \
    if (km == 4) launch_sim_res<DD, 4>(a, rf, z0, traj, tau, last, wsf, st);              \
    else if (km == 8) launch_sim_res<DD, 8>(a, rf, z0, traj, tau, last, wsf, st);         \
    else launch_sim_res<DD, 16>(a, rf, z0, traj, tau, last, wsf, st);                     \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "sde_kfp_gmm: dim must be in [1, 8]");
  }
  rc = check_launch("sde_simulate_kernel<GMM, fused residual>");
  if (rc) return rc;
  launch_slab_reduce(wsf, sim_grid(a.N), PDEINV_GMM_NACC + r->n_centers * D, acc, st);
  return check_launch("slab_reduce_kernel");
}

extern "C" size_t pdeinv_mf_workspace_bytes(const pdeinv_sde_desc* d) {
  if (!d || d->dim < 1 || d->dim > PDEINV_MAX_DIM || d->n_particles <= 0) return 0;
  return (size_t)(1 + d->dim) * sim_grid(d->n_particles) * sizeof(float);
}

extern "C" int pdeinv_mf_step(const pdeinv_sde_desc* d, int32_t s, const float* z, float* z_out,
                              float* tau_row, const float* /*d_tau0*/, const double* xbar_sum,
                              void* ws, double* xsum, void* stream) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  PDEINV_REQUIRE(d->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC, PDEINV_ERR_INVALID,
                 "mf_step: potential must be MEANFIELD_QUADRATIC");
  PDEINV_REQUIRE(s >= 0 && s <= d->n_steps, PDEINV_ERR_INVALID, "mf_step: s out of range");
  PDEINV_REQUIRE(d->d_shift_u == nullptr, PDEINV_ERR_INVALID,
                 "mf_step: the shared tau0 is drawn from the stream (shift_u unsupported)");
  hipStream_t st = (hipStream_t)stream;
  if (a.N == 0) {
    if (xsum && hipMemsetAsync(xsum, 0, sizeof(double) * (1 + d->dim), st) != hipSuccess)
      return fail(PDEINV_ERR_HIP, "mf_step: hipMemsetAsync failed");
    return PDEINV_OK;
  }
  PDEINV_REQUIRE(z && z_out && xbar_sum && ws && xsum, PDEINV_ERR_INVALID, "mf_step: null pointer");
  const float tau0 = shared_tau0_host(a, d);
  const int D = d->dim;
  const int g = sim_grid(a.N);
  switch (D) {
#define CASE(DD)                                                                           \
  case DD:                                                                                 \
    hipLaunchKernelGGL(mf_step_kernel<DD>, dim3(g), dim3(kBlock), 0, st, a, s, tau0, z, z_out, \
                       tau_row, xbar_sum, (float*)ws);                                     \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(10) CASE(12) CASE(16)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "mf_step: dim must be one of 1-8, 10, 12, 16");
  }
  rc = check_launch("mf_step_kernel");
  if (rc) return rc;
  launch_slab_reduce((float*)ws, g, 1 + D, xsum, st);
  return check_launch("slab_reduce_kernel");
}


// ---- McKean–Vlasov, fused multi-step path ----------------------------------------------------
// The quadratic interaction makes the ensemble mean exactly solvable: averaged over the particles
// the drift A (x_i - xbar) vanishes, so one update of the ensemble mean is
//     vbar' = (1 - gamma h) vbar + sqrt(h) ns xibar_s ,   xbar' = xbar + h vbar'
// with xibar_s = (1/N) sum_i xi_{i,s}, the mean of the update's noise. The noise is a function of
// (global particle id, update) only, so the whole mean path xbar_0..xbar_n follows from ONE reduction
// over the ensemble — [count, sum x0, sum v0, sum_i xi_{i,s} for every s] — done before the
// simulation (pdeinv_mf_sums), all-reduced once across ranks, and unrolled in fp64
// (pdeinv_mf_mean_path). The simulator then runs all n+1 updates of a particle in registers like the
// uncoupled kernels (no per-update state re-read, no per-update collective), reading xbar_s per update.
// The per-update exchange (pdeinv_mf_step) computes the same xbar_s from the fp32 states; the two
// agree to fp32 rounding (tests/test_gpu_meanfield.py).
constexpr int kMfSumsPerThread = 16;  // particles per thread in pdeinv_mf_sums


// grid.x: particle tiles of kBlock*kMfSumsPerThread; grid.y = n_steps + 2: y <= n_steps sums the update-y
// noise, y = n_steps + 1 sums [count, x0, v0]. Slab columns: [count, x0 (D), v0 (D), xi_0 (D), ..., xi_n (D)].
template <int D, bool EXPLICIT>
__global__ __launch_bounds__(kBlock) void mf_sums_kernel(SdeArgs a, const float* __restrict__ z0,
                                                         float* __restrict__ partials, int y0) {
  const int nb = gridDim.x, b = blockIdx.x;
  const int y = blockIdx.y + y0;  // y0 > 0: the tail after a fused KMV pass summed updates < y0
  const int64_t base = (int64_t)b * kBlock * kMfSumsPerThread + threadIdx.x;
  __shared__ float lds[kWavesPerBlock * (1 + 2 * D)];
  if (y == a.n_steps + 1) {
    float v[1 + 2 * D] = {};
#pragma unroll 4
    for (int j = 0; j < kMfSumsPerThread; ++j) {
      const int64_t i = base + (int64_t)j * kBlock;
      if (i < a.N) {
        v[0] += 1.f;
#pragma unroll
        for (int k = 0; k < 2 * D; ++k) v[1 + k] += z0[i * a.ld_z0 + k];
      }
    }
    block_reduce_to_slab(v, 1 + 2 * D, lds, partials, b, nb);
    return;
  }
  float acc[D] = {};
  const uint32_t s = (uint32_t)y;
#pragma unroll 2
  for (int j = 0; j < kMfSumsPerThread; ++j) {
    const int64_t i = base + (int64_t)j * kBlock;
    if (i < a.N) {
      const uint64_t gid = (uint64_t)(a.poff + i);
      float xi[D];
      gen_normals<D, EXPLICIT>(a, (uint32_t)gid, (uint32_t)(gid >> 32), s, i, xi);
#pragma unroll
      for (int k = 0; k < D; ++k) acc[k] += xi[k];
    }
  }
  block_reduce_to_slab(acc, D, lds, partials + (int64_t)(1 + 2 * D + y * D) * nb, b, nb);
}

// One lane per coordinate (the mean recursion is coordinate-wise): sums (all-reduced) -> xbar
// [n+1, D] fp32 (the mean BEFORE update s) and optionally xsum [n+2, 1+D] fp64 = [count, count*xbar_s]
// (the per-update exchange's record, s = 0..n+1). h_s are the particles' own fp32 step sizes.
__global__ void mf_path_kernel(int D, int n_steps, float dt, float tau0, float gamma, float ns,
                               const double* __restrict__ sums, float* __restrict__ xbar,
                               double* __restrict__ xsum) {
  const int k = threadIdx.x;
  const double cnt = sums[0];
  if (xsum && k == 0)
    for (int s = 0; s <= n_steps + 1; ++s) xsum[(int64_t)s * (1 + D)] = cnt;
  if (k >= D) return;
  const double inv = cnt > 0 ? 1.0 / cnt : 0.0;
  double xb = sums[1 + k] * inv, vb = sums[1 + D + k] * inv;
  for (int s = 0; s <= n_steps; ++s) {
    xbar[(int64_t)s * D + k] = (float)xb;
    if (xsum) xsum[(int64_t)s * (1 + D) + 1 + k] = cnt * xb;
    const float hf = (s == 0) ? tau0 : ((s == n_steps) ? dt - tau0 : dt);
    const double h = (double)hf, sh = (double)(sqrtf(hf) * ns);
    vb = vb - gamma * h * vb + sh * (sums[1 + 2 * D + (int64_t)s * D + k] * inv);
    xb = xb + h * vb;
  }
  if (xsum) xsum[(int64_t)(n_steps + 1) * (1 + D) + 1 + k] = cnt * xb;
}

static int mf_sums_grid(int64_t N) { return (int)((N + (int64_t)kBlock * kMfSumsPerThread - 1) / ((int64_t)kBlock * kMfSumsPerThread)); }

extern "C" int64_t pdeinv_mf_sums_len(const pdeinv_sde_desc* d) {
  if (!d || d->dim < 1 || d->dim > PDEINV_MAX_DIM || d->n_steps < 1) return 0;
  return mf_sums_len(d->dim, d->n_steps);
}

extern "C" size_t pdeinv_mf_sums_workspace_bytes(const pdeinv_sde_desc* d) {
  if (!d || d->dim < 1 || d->dim > PDEINV_MAX_DIM || d->n_steps < 1 || d->n_particles <= 0) return 0;
  return (size_t)mf_sums_len(d->dim, d->n_steps) * mf_sums_grid(d->n_particles) * sizeof(float);
}

static int mf_sums_launch(const SdeArgs& a, const pdeinv_sde_desc* d, const float* z0, int y0, void* ws,
                          double* sums, hipStream_t st);

extern "C" int pdeinv_mf_sums(const pdeinv_sde_desc* d, const float* z0, void* ws, double* sums, void* stream) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  PDEINV_REQUIRE(d->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC, PDEINV_ERR_INVALID,
                 "mf_sums: potential must be MEANFIELD_QUADRATIC");
  PDEINV_REQUIRE(sums != nullptr, PDEINV_ERR_INVALID, "mf_sums: sums is null");
  const int D = d->dim;
  const int64_t L = mf_sums_len(D, d->n_steps);
  hipStream_t st = (hipStream_t)stream;
  if (a.N == 0) {
    if (hipMemsetAsync(sums, 0, sizeof(double) * L, st) != hipSuccess)
      return fail(PDEINV_ERR_HIP, "mf_sums: hipMemsetAsync failed");
    return PDEINV_OK;
  }
  return mf_sums_launch(a, d, z0, 0, ws, sums, st);
}

// grid.y over y0 .. n_steps + 1; slab-reduces the columns the launch wrote
static int mf_sums_launch(const SdeArgs& a, const pdeinv_sde_desc* d, const float* z0, int y0, void* ws,
                          double* sums, hipStream_t st) {
  PDEINV_REQUIRE(z0 && ws, PDEINV_ERR_INVALID, "mf_sums: null pointer");
  PDEINV_REQUIRE(d->n_steps + 2 <= 65535, PDEINV_ERR_UNSUPPORTED, "mf_sums: n_steps too large");
  PDEINV_REQUIRE(y0 >= 0 && y0 <= d->n_steps + 1, PDEINV_ERR_INVALID, "mf_sums: bad first update");
  const int D = d->dim;
  const int64_t L = mf_sums_len(D, d->n_steps);
  const int nb = mf_sums_grid(a.N);
  const dim3 g(nb, d->n_steps + 2 - y0);
  float* p = (float*)ws;
  switch (D) {
#define CASE(DD)                                                                                         \
  case DD:                                                                                               \
    if (a.noise) hipLaunchKernelGGL((mf_sums_kernel<DD, true>), g, dim3(kBlock), 0, st, a, z0, p, y0);   \
    else hipLaunchKernelGGL((mf_sums_kernel<DD, false>), g, dim3(kBlock), 0, st, a, z0, p, y0);          \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(10) CASE(12) CASE(16)
#undef CASE
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "mf_sums: dim must be one of 1-8, 10, 12, 16");
  }
  int rc = check_launch("mf_sums_kernel");
  if (rc) return rc;
  if (y0 == 0) {
    launch_slab_reduce(p, nb, (int)L, sums, st);
  } else {  // [count, x0, v0] and the updates y0 .. n_steps
    const int64_t c0 = 1 + 2 * D + (int64_t)y0 * D;
    launch_slab_reduce(p, nb, 1 + 2 * D, sums, st);
    if (L > c0) launch_slab_reduce(p + c0 * nb, nb, (int)(L - c0), sums + c0, st);
  }
  return check_launch("slab_reduce_kernel");
}

int pdeinv::mf_sums_tail(const pdeinv_sde_desc* d, const float* z0, int y0, void* ws, double* sums, hipStream_t st) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  PDEINV_REQUIRE(d->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC, PDEINV_ERR_INVALID,
                 "mf_sums: potential must be MEANFIELD_QUADRATIC");
  PDEINV_REQUIRE(a.N > 0 && sums, PDEINV_ERR_INVALID, "mf_sums tail: empty ensemble or null sums");
  return mf_sums_launch(a, d, z0, y0, ws, sums, st);
}

int pdeinv::mf_noise_of(const pdeinv_sde_desc* d, int dim, int64_t n_particles, MfNoise& out) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  PDEINV_REQUIRE(d->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC, PDEINV_ERR_INVALID,
                 "fused mean-path sums: the next simulate must be MEANFIELD_QUADRATIC");
  PDEINV_REQUIRE(d->dim == dim && d->n_particles == n_particles, PDEINV_ERR_INVALID,
                 "fused mean-path sums: the next simulate's dim / n_particles must be the KMV pass's");
  PDEINV_REQUIRE(d->d_noise == nullptr, PDEINV_ERR_UNSUPPORTED,
                 "fused mean-path sums: Philox noise only (the explicit-noise mode runs pdeinv_mf_sums)");
  out = MfNoise{a.k0, a.k1, a.ctr_off, a.poff};
  return PDEINV_OK;
}

extern "C" int pdeinv_mf_mean_path(const pdeinv_sde_desc* d, const double* sums, float* xbar, double* xsum,
                                   void* stream) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  PDEINV_REQUIRE(d->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC, PDEINV_ERR_INVALID,
                 "mf_mean_path: potential must be MEANFIELD_QUADRATIC");
  PDEINV_REQUIRE(d->d_shift_u == nullptr, PDEINV_ERR_INVALID,
                 "mf_mean_path: the shared tau0 is drawn from the stream (shift_u unsupported)");
  PDEINV_REQUIRE(sums && xbar, PDEINV_ERR_INVALID, "mf_mean_path: null pointer");
  hipLaunchKernelGGL(mf_path_kernel, dim3(1), dim3(kWave), 0, (hipStream_t)stream, d->dim, d->n_steps, a.dt,
                     shared_tau0_host(a, d), a.gamma, a.ns, sums, xbar, xsum);
  return check_launch("mf_path_kernel");
}

extern "C" int pdeinv_sde_tau0(const pdeinv_sde_desc* d, float* out, void* stream) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  if (a.N == 0) return PDEINV_OK;
  PDEINV_REQUIRE(out != nullptr, PDEINV_ERR_INVALID, "sde_tau0: out is null");
  hipLaunchKernelGGL(tau0_kernel, dim3(sim_grid(a.N)), dim3(kBlock), 0, (hipStream_t)stream, a, out);
  return check_launch("tau0_kernel");
}

// ---- McKean–Vlasov simulate + the next simulate's mean-path sums ------------------------------
// pdeinv_sde_simulate (fused McKean–Vlasov path) that also returns pdeinv_mf_sums(next, z0_next): the noise
// sums are drawn inside the simulator (sde_simulate_kernel NXT, the store-bound kernel's idle VALU), the
// [count, sum x0, sum v0] head by the z0 pass of pdeinv_mf_sums. The next simulate differs from this one in
// its Philox counter only (same key, particles, dim, n_steps); equal to pdeinv_mf_sums up to the fp32
// partial-sum order.
static size_t mf_next_slab_bytes(const pdeinv_sde_desc* d) {
  return ((size_t)(d->n_steps + 1) * d->dim * sim_grid(d->n_particles) * sizeof(float) + 255) & ~(size_t)255;
}

extern "C" size_t pdeinv_sde_simulate_mf_next_workspace_bytes(const pdeinv_sde_desc* d) {
  if (!d || d->dim < 1 || d->dim > 8 || d->n_particles <= 0 || d->n_steps < 1) return 0;
  return mf_next_slab_bytes(d) + pdeinv_mf_sums_workspace_bytes(d);
}

template <int D>
static void launch_sim_mf_next(const SdeArgs& a, const MfNext& nx, const float* z0, float* traj, float* tau,
                               float* last, hipStream_t st) {
  hipLaunchKernelGGL((sde_simulate_kernel<D, PDEINV_POT_MEANFIELD_QUADRATIC, false, kStoreStaged, 1, false,
                                          1, false, true>),
                     dim3(sim_grid(a.N)), dim3(kBlock), 0, st, a, z0, traj, tau, last, nullptr, GmmResFused{}, nx);
}

extern "C" int pdeinv_sde_simulate_mf_next(const pdeinv_sde_desc* d, const float* z0, float* traj, float* tau,
                                           float* last, const pdeinv_sde_desc* next, const float* z0_next, void* ws,
                                           double* sums_next, void* stream) {
  SdeArgs a;
  int rc = build_args(d, a);
  if (rc) return rc;
  PDEINV_REQUIRE(next != nullptr && sums_next != nullptr, PDEINV_ERR_INVALID, "sde_mf_next: null next / sums");
  PDEINV_REQUIRE(d->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC &&
                     next->potential.kind == PDEINV_POT_MEANFIELD_QUADRATIC,
                 PDEINV_ERR_INVALID, "sde_mf_next: both simulates must be MEANFIELD_QUADRATIC");
  PDEINV_REQUIRE(d->d_meanfield != nullptr, PDEINV_ERR_INVALID,
                 "sde_mf_next: McKean–Vlasov needs d_meanfield (pdeinv_mf_mean_path)");
  PDEINV_REQUIRE(d->d_shift_u == nullptr, PDEINV_ERR_INVALID,
                 "sde_mf_next: McKean–Vlasov draws its shared tau0 from the stream (shift_u unsupported)");
  PDEINV_REQUIRE(d->d_noise == nullptr && next->d_noise == nullptr, PDEINV_ERR_UNSUPPORTED,
                 "sde_mf_next: Philox noise only (the explicit-noise mode runs pdeinv_mf_sums)");
  PDEINV_REQUIRE(next->dim == d->dim && next->n_particles == d->n_particles &&
                     next->particle_offset == d->particle_offset && next->seed == d->seed &&
                     next->n_steps == d->n_steps,
                 PDEINV_ERR_INVALID, "sde_mf_next: the next simulate must differ in its counter offset only");
  const int D = d->dim;
  PDEINV_REQUIRE(D % 2 == 0 && D <= 8 && d->n_steps + 1 <= 128, PDEINV_ERR_UNSUPPORTED,
                 "sde_mf_next: even dim <= 8 and n_steps + 1 <= 128");
  a.xbar = d->d_meanfield;
  a.tau0_mf = shared_tau0_host(a, d);
  hipStream_t st = (hipStream_t)stream;
  if (a.N == 0) {
    if (hipMemsetAsync(sums_next, 0, sizeof(double) * mf_sums_len(D, d->n_steps), st) != hipSuccess)
      return fail(PDEINV_ERR_HIP, "sde_mf_next: hipMemsetAsync failed");
    return PDEINV_OK;
  }
  PDEINV_REQUIRE(z0 && z0_next && ws, PDEINV_ERR_INVALID, "sde_mf_next: null pointer");
  PDEINV_REQUIRE(aligned(traj, 16) && aligned(last, 16) && aligned(tau, 4), PDEINV_ERR_INVALID,
                 "sde_mf_next: traj/last must be 16-byte aligned");
  MfNext nx{};
  nx.partials = (float*)ws;
  nx.ctr_off = next->counter_offset;
  nx.np1 = d->n_steps + 1;
  switch (D) {
    case 2: launch_sim_mf_next<2>(a, nx, z0, traj, tau, last, st); break;
    case 4: launch_sim_mf_next<4>(a, nx, z0, traj, tau, last, st); break;
    case 6: launch_sim_mf_next<6>(a, nx, z0, traj, tau, last, st); break;
    default: launch_sim_mf_next<8>(a, nx, z0, traj, tau, last, st); break;
  }
  rc = check_launch("sde_simulate_kernel<MEANFIELD, next sums>");
  if (rc) return rc;
  launch_slab_reduce(nx.partials, sim_grid(a.N), nx.np1 * D, sums_next + 1 + 2 * D, st);
  rc = check_launch("slab_reduce_kernel");
  if (rc) return rc;
  return mf_sums_tail(next, z0_next, d->n_steps + 1, (char*)ws + mf_next_slab_bytes(d), sums_next, st);
}

