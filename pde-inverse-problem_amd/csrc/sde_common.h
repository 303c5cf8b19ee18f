// sde_common.h — the simulator pieces shared by sde.hip (the simulator family) and sde_kmv.hip (the
// McKean–Vlasov simulate fused with the KMV residual's stamp sums): the kernel argument block, the drift and
// noise helpers, the store helpers and the host-side descriptor checks.
#pragma once
#include <math.h>
#include <stddef.h>
#include <stdlib.h>

#include <cmath>

#include "common.h"

namespace pdeinv {

struct SdeArgs {
  int64_t N, poff, ld_z0;
  int32_t n_steps, random_shift, K, has_center;
  int32_t remap;  // 1 (default): XCD-contiguous block order (xcd_block); PDEINV_SIM_REMAP=0 disables
  float dt, gamma, ns, neg_half_inv_s2_log2e, inv_s2, l2s;
  uint32_t k0, k1, ctr_off;
  const float* noise;
  const float* shift_u;
  // MEANFIELD_QUADRATIC (fused multi-step path): xbar [n_steps+1, d], the ensemble mean of the
  // positions before each update (pdeinv_mf_mean_path), and the shared clock tau0 of the ensemble
  const float* xbar;
  float tau0_mf;
  // QUADRATIC: A (d*d) then c (d). GMM (packed on the host at compile-time offsets):
  // GMM: [kMaxGmmK*d raw mu | kMaxGmmK constants c_k = -|mu_k|^2 log2e / (2 s^2)]
  float params[2 * 16 * PDEINV_MAX_DIM + 16];
};

constexpr int kMaxGmmK = 16;

// d standard normals for update s of particle (plo, phi) — stream layout of include/pdeinv.h.
// EXPLICIT (the explicit-noise parity mode) is a compile-time choice: a global load left on the
// Philox path of the step loop makes the compiler wait vmcnt(0) at the join, and on gfx950 vmcnt
// also counts the previous steps' trajectory stores — every step would wait for them to retire.
template <int D, bool EXPLICIT = false>
__device__ __forceinline__ void gen_normals(const SdeArgs& a, uint32_t plo, uint32_t phi,
                                            uint32_t s, int64_t i, float* xi) {
  if constexpr (EXPLICIT) {
    const float* src = a.noise + ((int64_t)s * a.N + i) * D;
#pragma unroll
    for (int k = 0; k < D; ++k) xi[k] = src[k];
    return;
  }
  stream_normals<D>(a.k0, a.k1, a.ctr_off + s, plo, phi, xi);
}

// grad U(q) = A (q - c) = A q - b, b = A c packed on the host (KOU: A = tilde_F, c = 0,
// …_OU.py:130-138): the FMA chain starts at -b, so a centre costs no per-step instruction.
typedef const __attribute__((address_space(4))) float kfloat;
typedef const __attribute__((address_space(4))) char kchar;
// SdeArgs::params in the kernel-argument segment (sde_simulate_kernel's first argument, offset 0), made
// opaque per use: held across the step loop, d^2 + d uniform floats beyond ~32 overflow the scalar
// register file and the spills come back as v_readlane on every update (d = 8: 46-66 per update).
__device__ __forceinline__ kfloat* kernarg_params() {
  kfloat* p = (kfloat*)((kchar*)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(SdeArgs, params));
  asm volatile("" : "+s"(p));
  return p;
}

// McKean–Vlasov drift with the mean path precomputed: grad U(q) = A (q - xbar_s), the same
// operation order as the per-update exchange (mf_step_kernel) and the C oracle (y = q - xbar, then
// A y). xbar_s is wave-uniform (scalar loads from a small device array, one row per update).
// A is read from the kernel-argument segment with scalar loads at every update (kernarg_params): held
// across the step loop, its d^2 SGPRs (64 at d = 8) overflowed the scalar file and the spills came back
// as 46 v_readlane per update (C4 step loop 208 -> 162 VALU instructions per update).
// xbar_s through the constant address space: a scalar load (lgkmcnt). As a global load it was a vector load whose
// vmcnt wait, on gfx950, also waited for every trajectory store of the previous update still in flight.
template <int D>
__device__ __forceinline__ void grad_meanfield(const SdeArgs&, const float* q, const float* xbp, float* g) {
  kfloat* A = kernarg_params();
  kfloat* xb = (kfloat*)xbp;
  float y[D];
#pragma unroll
  for (int c = 0; c < D; ++c) y[c] = q[c] - xb[c];
#pragma unroll
  for (int r = 0; r < D; ++r) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) acc = fmaf(A[r * D + c], y[c], acc);
    g[r] = acc;
  }
}

// Dispatch order -> particle block: the hardware hands consecutive workgroups to the 8 XCDs in
// turn (b -> XCD b % 8); this map gives XCD x the contiguous block range [x*nb/8, (x+1)*nb/8), so
// each XCD's L2 sees one contiguous stretch of every trajectory slab instead of every 8th 8 KiB
// piece. Measured on the C2 launch, same buffers A/B in one process: 1.53 -> 1.46 ms and
// 1.26 -> 1.20 ms (4-5 %, every allocation; tools/sim_alloc.py, profiles/r01_sim_remap_ab.log).
// Results are unchanged: a particle's numbers depend only on its global id, and the moment
// partial slots are indexed by the mapped block. (Not used by mf_step_kernel: there the C4 bench
// measured 6.8 ms without vs 7.5 ms with it, across processes.)
__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8, l = b / 8;
  return x < r ? x * (q + 1) + l : r * (q + 1) + (x - r) * q + l;
}

// Store modes for the per-step trajectory rows (M = 2d floats per particle):
//  kStoreNT     — each lane stores its own row (M/4 dwordx4, nontemporal): one store
//                 instruction covers 64 rows but only 16 of every 4*M bytes;
//  kStorePlain  — the same with default-policy stores;
//  kStoreStaged — the wave's 64 rows go through a 64*M*4-byte LDS slot so that every store
//                 instruction writes 1 KiB contiguous (whole lines), nontemporal.
enum { kStoreNT = 0, kStorePlain = 1, kStoreStaged = 2 };

template <int D, int STORE>
__device__ __forceinline__ void store_row(float* dst, const float* z) {
  constexpr int M = 2 * D;
  if constexpr (M % 4 == 0) {
#pragma unroll
    for (int k = 0; k < M; k += 4) {
      if constexpr (STORE == kStorePlain)
        *reinterpret_cast<f32x4*>(dst + k) = f32x4{z[k], z[k + 1], z[k + 2], z[k + 3]};
      else
        __builtin_nontemporal_store(f32x4{z[k], z[k + 1], z[k + 2], z[k + 3]},
                                    reinterpret_cast<f32x4*>(dst + k));
    }
  } else {
#pragma unroll
    for (int k = 0; k < M; k += 2)
      __builtin_nontemporal_store(f32x2{z[k], z[k + 1]}, reinterpret_cast<f32x2*>(dst + k));
  }
}

__device__ __forceinline__ float tau_value(float tau0, int s, float dt) {
#pragma clang fp contract(off)
  return tau0 + (float)s * dt;  // tau_0 + arange(n)*dt, two roundings (sampling_utils.py:48)
}

// McKean–Vlasov: the NEXT simulate's mean-path noise sums (the sum_i xi_{i,s} part of pdeinv_mf_sums) drawn
// inside this simulate (NXT). The sums depend on the particle ids and the next simulate's Philox counter only,
// so this store-bound kernel can draw them with its idle VALU while it streams the trajectory, and the KMV
// pass that follows reads at full rate. A wave owns its 64 particles x np1 updates of the next simulate and
// draws one (particle, update) pair per lane and step: lane l takes pairs q = l np1 + s (s = 0..np1-1, the
// simulator's own steps), q -> (update q / 64, particle q % 64). A lane's np1 consecutive pairs span at most
// three updates (np1 <= 128), so it keeps three running sums; after the last step the block combines them in
// a fixed order (per update: waves, then the 1-3 lanes that drew it) into one slab column per update.
struct MfNext {
  float* partials;   // [(np1 * D) columns][gridDim.x]: column s * D + k
  uint32_t ctr_off;  // the next simulate's Philox counter offset (same key and particle ids)
  int32_t np1;       // updates per simulate (n_steps + 1), <= 128
};

__host__ __device__ inline int64_t mf_sums_len(int D, int n_steps) { return 1 + 2 * D + (int64_t)(n_steps + 1) * D; }

static inline bool aligned(const void* p, size_t a) { return p == nullptr || ((uintptr_t)p % a) == 0; }

static inline int build_args(const pdeinv_sde_desc* d, SdeArgs& a) {
  PDEINV_REQUIRE(d != nullptr, PDEINV_ERR_INVALID, "sde: null descriptor");
  PDEINV_REQUIRE(d->dim >= 1 && d->dim <= PDEINV_MAX_DIM, PDEINV_ERR_UNSUPPORTED,
                 "sde: dim must be in [1, 16]");
  PDEINV_REQUIRE(d->n_steps >= 1, PDEINV_ERR_INVALID, "sde: n_steps must be >= 1");
  PDEINV_REQUIRE(d->n_particles >= 0, PDEINV_ERR_INVALID, "sde: n_particles must be >= 0");
  PDEINV_REQUIRE(d->particle_offset >= 0, PDEINV_ERR_INVALID, "sde: particle_offset must be >= 0");
  PDEINV_REQUIRE(std::isfinite(d->dt) && d->dt > 0.f, PDEINV_ERR_INVALID, "sde: dt must be > 0");
  PDEINV_REQUIRE(std::isfinite(d->gamma) && std::isfinite(d->noise_scale), PDEINV_ERR_INVALID,
                 "sde: gamma / noise_scale must be finite");
  const int D = d->dim;
  a = SdeArgs{};
  a.N = d->n_particles;
  a.poff = d->particle_offset;
  a.ld_z0 = d->ld_z0 ? d->ld_z0 : 2 * D;
  PDEINV_REQUIRE(a.ld_z0 >= 2 * D, PDEINV_ERR_INVALID, "sde: ld_z0 < 2*dim");
  a.n_steps = d->n_steps;
  a.random_shift = d->random_shift ? 1 : 0;
  a.dt = d->dt;
  a.gamma = d->gamma;
  a.ns = d->noise_scale;
  a.k0 = (uint32_t)d->seed;
  a.k1 = (uint32_t)(d->seed >> 32);
  a.ctr_off = d->counter_offset;
  a.noise = d->d_noise;
  a.shift_u = d->d_shift_u;
  {
    const char* r = ab_env("PDEINV_SIM_REMAP");  // A/B switch for tools/sim_alloc.py
    a.remap = r ? atoi(r) : 1;
  }
  const pdeinv_potential& p = d->potential;
  int n_params = 0;
  switch (p.kind) {
    case PDEINV_POT_QUADRATIC:
    case PDEINV_POT_MEANFIELD_QUADRATIC:
      a.has_center = (p.kind == PDEINV_POT_QUADRATIC && p.has_center) ? 1 : 0;
      n_params = D * D + (a.has_center ? D : 0);
      break;
    case PDEINV_POT_GMM:
      PDEINV_REQUIRE(p.n_centers >= 1 && p.n_centers <= kMaxGmmK &&
                         p.n_centers * D <= PDEINV_MAX_PARAMS,
                     PDEINV_ERR_UNSUPPORTED, "sde: GMM needs 1 <= n_centers <= 16");
      PDEINV_REQUIRE(std::isfinite(p.sigma) && p.sigma > 0.f, PDEINV_ERR_INVALID,
                     "sde: GMM sigma must be > 0");
      PDEINV_REQUIRE(p.params != nullptr, PDEINV_ERR_INVALID, "sde: potential params are null");
      a.K = p.n_centers;
      a.inv_s2 = 1.0f / (p.sigma * p.sigma);
      a.neg_half_inv_s2_log2e = -0.5f * a.inv_s2 * 1.4426950408889634f;
      a.l2s = (float)(1.4426950408889634 / ((double)p.sigma * (double)p.sigma));
      {
        const double sc = 1.4426950408889634 / ((double)p.sigma * (double)p.sigma);
        const int K = p.n_centers;
        for (int k = 0; k < K; ++k) {
          double n2 = 0;
          for (int i = 0; i < D; ++i) {
            const double m = p.params[k * D + i];
            a.params[k * D + i] = (float)m;
            n2 += m * m;
          }
          a.params[kMaxGmmK * D + k] = (float)(-0.5 * n2 * sc);
        }
      }
      n_params = 0;  // packed above
      break;
    case PDEINV_POT_NONE:
      n_params = 0;  // quadratic with A = 0
      break;
    default:
      return fail(PDEINV_ERR_UNSUPPORTED, "sde: unknown potential kind");
  }
  if (n_params) {
    PDEINV_REQUIRE(p.params != nullptr, PDEINV_ERR_INVALID, "sde: potential params are null");
    for (int k = 0; k < D * D; ++k) a.params[k] = p.params[k];
    if (a.has_center) {  // b = A c in fp64, rounded once (grad_quadratic)
      for (int r = 0; r < D; ++r) {
        double b = 0;
        for (int c = 0; c < D; ++c) b += (double)p.params[r * D + c] * (double)p.params[D * D + c];
        a.params[D * D + r] = (float)b;
      }
    }
  }
  return PDEINV_OK;
}

// The interacting ensemble shares one clock: tau0 from global id UINT64_MAX (include/pdeinv.h).
// Computed on the host with the same Philox so that every rank and every step agrees.
static inline float shared_tau0_host(const SdeArgs& a, const pdeinv_sde_desc* d) {
  if (!a.random_shift) return 0.f;
  uint32_t c0 = 0xFFFFFFFFu, c1 = 0xFFFFFFFFu, c2 = a.ctr_off, c3 = 0x80000000u;
  uint32_t k0 = a.k0, k1 = a.k1;
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)kM0 * c0, p1 = (uint64_t)kM1 * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += kW0;
    k1 += kW1;
  }
  const float u = (float)(c0 >> 8) * 0x1p-24f;
  (void)d;
  return u * a.dt;
}

}  // namespace pdeinv
