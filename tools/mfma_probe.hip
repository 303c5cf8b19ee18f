// MFMA issue-rate probe (tools only): v_mfma_f32_32x32x2_f32 chains at 1 / 2 waves per SIMD, with and
// without per-step operand traffic, to find the ceiling the MLP row GEMMs can reach.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o tools/_bin/mfma_probe && tools/_bin/mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// NACC independent accumulators; MODE 0: operands from registers; 1: B from LDS (ds_read_b128 per 16
// steps, as rgemm); 2: + A loaded from global per 16 steps (dwordx4 x4, as rgemm's plane loads)
template <int NACC, int MODE>
__global__ __launch_bounds__(512, 1) void probe(int iters, const float* __restrict__ g, float* out) {
  __shared__ f32x4 lds[128 * 65];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 128 * 65; i += 512) lds[i] = f32x4{1.f, 1.f, 1.f, 1.f} * (float)(i & 7) * 1e-3f;
  __syncthreads();
  f32x16 acc[NACC];
  for (int q = 0; q < NACC; ++q) acc[q] = f32x16{};
  float a = lane * 1e-3f, b = 1.f;
  float bt[16], at[16];
  for (int s = 0; s < 16; ++s) { bt[s] = b + s; at[s] = a - s; }
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE >= 1) {
      const f32x4* p = lds + ((lane & 31) * 65 + (it & 15) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { const f32x4 v = p[j]; bt[4*j] = v[0]; bt[4*j+1] = v[1]; bt[4*j+2] = v[2]; bt[4*j+3] = v[3]; }
    }
    if constexpr (MODE >= 10) {  // MODE - 10 independent VALU FMAs per MFMA (the layer-1 prologue's mix)
      constexpr int NV = MODE - 10;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = at[j] * 1.0001f;
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int q = 0; q < NACC; ++q) {
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(at[s], bt[s], acc[q], 0, 0, 0);
#pragma unroll
          for (int j = 0; j < NV; ++j) v[j & 7] = fmaf(v[j & 7], 0.999f, bt[(s + j) & 15]);
        }
#pragma unroll
      for (int j = 0; j < 8; ++j) at[j] += v[j] * 1e-30f;
      continue;
    }
    if constexpr (MODE == 3 || MODE == 4) {  // prefetched one iteration ahead (register double buffer), NP planes
      constexpr int NP = MODE == 3 ? 1 : 3;
      float nx[NP][16];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        const f32x4* p = reinterpret_cast<const f32x4*>(g + (size_t)pl * (4 << 20) + (size_t)((blockIdx.x * 512 + threadIdx.x + it * 7) & 0xFFFF) * 64 + (it & 3) * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) { const f32x4 v = p[j]; nx[pl][4*j] = v[0]; nx[pl][4*j+1] = v[1]; nx[pl][4*j+2] = v[2]; nx[pl][4*j+3] = v[3]; }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(at[s] + (q % NP), bt[s], acc[q], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 16; ++s) { at[s] = nx[0][s]; if (NP > 1) bt[s] = nx[NP - 1][s] + nx[1][s]; }
      continue;
    }
    if constexpr (MODE == 2) {
      const f32x4* p = reinterpret_cast<const f32x4*>(g + (size_t)((blockIdx.x * 512 + threadIdx.x) & 0xFFFF) * 64 + (it & 3) * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) { const f32x4 v = p[j]; at[4*j] = v[0]; at[4*j+1] = v[1]; at[4*j+2] = v[2]; at[4*j+3] = v[3]; }
    }
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(at[s], bt[s], acc[q], 0, 0, 0);
  }
  float t = 0.f;
  for (int q = 0; q < NACC; ++q) t += acc[q][lane & 15];
  out[blockIdx.x * 512 + threadIdx.x] = t;
}

template <int NACC, int MODE>
void run(const char* name, int waves_per_block, const float* g, float* out) {
  const int iters = 4096, blocks = 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<NACC, MODE>), dim3(blocks), dim3(64 * waves_per_block), 0, 0, 16, g, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<NACC, MODE>), dim3(blocks), dim3(64 * waves_per_block), 0, 0, iters, g, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 2 * 16 * NACC * (double)iters * blocks * waves_per_block;
  printf("%-34s waves/CU %d: %7.1f TFLOP/s (%.3f of 157.3)\n", name, waves_per_block, flops / ms / 1e9, flops / ms / 1e9 / 157.3);
}

int main() {
  float *g, *out;
  hipMalloc(&g, 64ull << 20);
  hipMemset(g, 0, 64ull << 20);
  hipMalloc(&out, 256 * 512 * 4);
  for (int w : {4, 8}) {
    run<6, 0>("regs, 6 acc", w, g, out);
    run<4, 0>("regs, 4 acc", w, g, out);
    run<12, 0>("regs, 12 acc", w, g, out);
    run<6, 1>("+ B ds_read_b128 / 16 steps, 6 acc", w, g, out);
    run<6, 2>("+ A dwordx4 x4 / 16 steps, 6 acc", w, g, out);
    run<6, 3>("A dwordx4 x4 prefetched, 6 acc", w, g, out);
    run<6, 4>("3 planes dwordx4 x12 prefetched, 6 acc", w, g, out);
    run<6, 12>("+ 2 VALU per MFMA, 6 acc", w, g, out);
    run<6, 14>("+ 4 VALU per MFMA, 6 acc", w, g, out);
    run<6, 16>("+ 6 VALU per MFMA, 6 acc", w, g, out);
    run<6, 18>("+ 8 VALU per MFMA, 6 acc", w, g, out);
  }
  return 0;
}
