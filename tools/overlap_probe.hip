// Store/VALU overlap probe for the simulator's step loop (not part of the library).
// Each wave owns 64 consecutive rows of 32 B and, per step, runs WORK x 8 independent FMAs
// (stand-in for Philox + Box–Muller + EM), stages its rows through LDS and writes its 2 KiB piece
// of slab s (+ 256 B of tau) — the C2 byte pattern (n = 100, N = 2^21). Occupancy is limited with
// dynamic LDS (blocks per CU = 160 KiB / lds). Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int WORK, int TAU, int STAGE = 1, int NT = 1>
__global__ __launch_bounds__(256) void probe(f4* traj, float* tau, long N, int n, float* sink) {
  extern __shared__ f4 dyn[];
  __shared__ f4 stage[256 * 2];
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const long wave_row0 = i - lane;
  f4* slot = stage + (threadIdx.x - lane) * 2;
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = (float)(i + k) * 1e-7f;
  for (int s = 0; s < n; ++s) {
#pragma unroll
    for (int w = 0; w < WORK; ++w) {
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] = fmaf(a[k], 0.999f, 1e-3f);
    }
    f4 v0, v1;
    if (STAGE) {
      slot[lane * 2] = f4{a[0], a[1], a[2], a[3]};
      slot[lane * 2 + 1] = f4{a[4], a[5], a[6], a[7]};
      __builtin_amdgcn_wave_barrier();
      v0 = slot[lane];
      v1 = slot[64 + lane];
    } else {  // already in store order (the sim_like bound)
      v0 = f4{a[0], a[1], a[2], a[3]};
      v1 = f4{a[4], a[5], a[6], a[7]};
    }
    f4* dst = traj + (wave_row0 + (long)s * N) * 2;
    if (NT) {
      __builtin_nontemporal_store(v0, dst + lane);
      __builtin_nontemporal_store(v1, dst + 64 + lane);
    } else {
      dst[lane] = v0;
      dst[64 + lane] = v1;
    }
    if (TAU == 1) __builtin_nontemporal_store(a[0], tau + (long)s * N + i);
    // TAU == 2: wave w of the block writes the whole block's 1 KiB tau row of every step s = w mod 4
    if (TAU == 2 && (s & 3) == (threadIdx.x >> 6))
      __builtin_nontemporal_store(f4{a[1], a[2], a[3], a[4]},
                                  reinterpret_cast<f4*>(tau + (long)s * N + (long)blockIdx.x * 256) + lane);
    __builtin_amdgcn_wave_barrier();
  }
  if (a[0] == 12345.f) sink[0] = dyn[0][0];
}

__global__ __launch_bounds__(256) void sim_like(f4* traj, long N, int n, float scale) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const long wave_row0 = i - lane;
  f4* base = traj + wave_row0 * 2;
  float v = (float)i * scale;
  for (int s = 0; s < n; ++s) {
    f4* dst = base + (long)s * N * 2;
    __builtin_nontemporal_store(f4{v, v + 1, v + 2, v + 3}, dst + lane);
    __builtin_nontemporal_store(f4{v + 4, v + 5, v + 6, v + 7}, dst + 64 + lane);
    v += 1.f;
  }
}

template <int WORK>
__global__ __launch_bounds__(256) void compute_only(long N, int n, float* sink) {
  extern __shared__ f4 dyn[];
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = (float)(i + k) * 1e-7f;
  for (int s = 0; s < n; ++s) {
#pragma unroll
    for (int w = 0; w < WORK; ++w) {
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] = fmaf(a[k], 0.999f, 1e-3f);
    }
  }
  float t = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) t += a[k];
  if (t == 12345.f) sink[0] = dyn[0][0];
}

template <class F>
static float timeit(F f) {
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  for (int w = 0; w < 3; ++w) f();
  (void)hipEventRecord(s);
  for (int r = 0; r < 10; ++r) f();
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms;
  (void)hipEventElapsedTime(&ms, s, e);
  return ms / 10;
}

template <int WORK, int TAUM, int STAGE, int NT>
static void row(f4* traj, float* tau, float* sink, long N, int n) {
  const size_t bytes = (size_t)N * n * (TAUM ? 36 : 32);
  (void)hipFuncSetAttribute((const void*)probe<WORK, TAUM, STAGE, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  for (int bpc : {5, 0}) {
    const size_t lds = bpc ? (160 * 1024) / bpc - 8 * 1024 - 64 : 0;
    const float ms = timeit([&] { probe<WORK, TAUM, STAGE, NT><<<N / 256, 256, lds>>>(traj, tau, N, n, sink); });
    printf("TAU=%d WORK=%3d STAGE=%d NT=%d blocks/CU=%d  %6.3f ms  %7.1f GB/s\n", TAUM, WORK, STAGE, NT, bpc, ms,
           bytes / (ms / 1e3) / 1e9);
  }
}

int main(int argc, char** argv) {
  const long N = 1L << 21;
  const int n = 100;
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  f4* traj;
  float *tau = nullptr, *sink;
  if (hipMalloc(&traj, (size_t)N * n * 32) != hipSuccess) return 1;
  printf("traj %p\n", (void*)traj);
  if (mode != 1 && hipMalloc(&tau, (size_t)N * n * 4) != hipSuccess) return 1;
  if (hipMalloc(&sink, 64) != hipSuccess) return 1;
  if (mode == 4) {  // DPM ramp: time consecutive batches of 25 launches for ~4 s
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int b = 0; b < 120; ++b) {
      (void)hipEventRecord(e0);
      for (int r = 0; r < 25; ++r) sim_like<<<N / 256, 256>>>(traj, N, n, 1.0f);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (b % 6 == 0 || b < 6) printf("batch %3d  %6.3f ms/launch  %7.1f GB/s\n", b, ms / 25, N * n * 32.0 / (ms / 25 / 1e3) / 1e9);
    }
    return 0;
  }
  if (mode == 3) {
    for (float sc : {1.0f, 1e-7f, 0.0f}) {
      const float ms = timeit([&] { sim_like<<<N / 256, 256>>>(traj, N, n, sc); });
      printf("sim_like scale %g %6.3f ms %7.1f GB/s\n", sc, ms, N * n * 32.0 / (ms / 1e3) / 1e9);
    }
    return 0;
  }
  if (mode == 1 || mode == 2) {  // plain launches, no attribute, no dynamic LDS
    const float ms = timeit([&] { probe<0, 0, 0, 1><<<N / 256, 256>>>(traj, tau, N, n, sink); });
    printf("mode %d probe<0,0,0,1> plain launch %6.3f ms %7.1f GB/s\n", mode, ms, N * n * 32.0 / (ms / 1e3) / 1e9);
    return 0;
  }
  row<0, 0, 0, 1>(traj, tau, sink, N, n);
  row<0, 0, 1, 1>(traj, tau, sink, N, n);
  row<0, 0, 1, 0>(traj, tau, sink, N, n);
  row<0, 1, 1, 0>(traj, tau, sink, N, n);
  row<16, 1, 1, 0>(traj, tau, sink, N, n);
  return 0;
}
