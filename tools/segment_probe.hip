// segment_probe.hip — does the simulator's store rate depend on how long its waves live? The C2 trajectory shape
// (n = 100 slabs of N x 32 B, time-major), written by waves that each own 64 rows for S consecutive slabs, the
// 100 / S segments as separate launches (S = 100: the simulator's one launch; smaller S: shorter-lived waves, the
// next segment's waves re-reading nothing). Not part of the library; tools/store_pattern.hip holds the other shapes.
// Build: hipcc -O3 --offload-arch=gfx950 tools/segment_probe.hip -o tools/_bin/segment_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void seg(f4* traj, long N, int s0, int S) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  f4* base = traj + (i - lane) * 2;
  float v = (float)i;
  for (int s = s0; s < s0 + S; ++s) {
    f4* dst = base + (long)s * N * 2;
    __builtin_nontemporal_store(f4{v, v + 1, v + 2, v + 3}, dst + lane);
    __builtin_nontemporal_store(f4{v + 4, v + 5, v + 6, v + 7}, dst + 64 + lane);
    v += 1.f;
  }
}

// S slabs per wave, but the grid walks the particles in R rounds of N / R rows per launch group: a block's rows
// are contiguous and the resident blocks write a narrower window of each slab
__global__ __launch_bounds__(256) void seg_rows(f4* traj, long N, long row0, int S) {
  const long i = row0 + (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  f4* base = traj + (i - lane) * 2;
  float v = (float)i;
  for (int s = 0; s < S; ++s) {
    f4* dst = base + (long)s * N * 2;
    __builtin_nontemporal_store(f4{v, v + 1, v + 2, v + 3}, dst + lane);
    __builtin_nontemporal_store(f4{v + 4, v + 5, v + 6, v + 7}, dst + 64 + lane);
    v += 1.f;
  }
}

__global__ __launch_bounds__(256) void oneshot(f4* p) {
  f4* q = p + (long)blockIdx.x * 1024;
#pragma unroll
  for (int k = 0; k < 4; ++k) q[(long)k * 256 + threadIdx.x] = f4{1.f, 2.f, 3.f, (float)k};
}

template <class F>
static float timeit(F f) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int w = 0; w < 3; ++w) f();
  hipEventRecord(s);
  for (int r = 0; r < 10; ++r) f();
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms / 10;
}

int main() {
  const long N = 1L << 21;
  const int n = 100;
  const size_t bytes = (size_t)N * n * 32;
  f4* traj;
  if (hipMalloc(&traj, bytes) != hipSuccess) return 1;
  auto rep = [&](const char* name, int a, float ms) {
    printf("%-28s %4d %7.3f ms  %7.1f GB/s\n", name, a, ms, bytes / (ms / 1e3) / 1e9);
  };
  for (int rnd = 0; rnd < 2; ++rnd) {
    for (int S : {100, 50, 25, 20, 10, 5, 2, 1})
      rep("slab segments of S", S, timeit([&] {
            for (int s0 = 0; s0 < n; s0 += S) seg<<<N / 256, 256>>>(traj, N, s0, S);
          }));
    for (int R : {2, 4, 8, 16, 32})
      rep("row rounds R (S = 100)", R, timeit([&] {
            for (int r = 0; r < R; ++r) seg_rows<<<N / R / 256, 256>>>(traj, N, r * (N / R), n);
          }));
    rep("oneshot lane-major VPT=4", 4, timeit([&] { oneshot<<<bytes / 16 / 1024, 256>>>(traj); }));
    rep("hipMemsetD32Async", 0, timeit([&] { (void)hipMemsetD32Async((hipDeviceptr_t)traj, 0x3f800000, bytes / 4, 0); }));
  }
  return 0;
}
