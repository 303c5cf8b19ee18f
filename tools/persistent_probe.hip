// persistent_probe.hip — the C2 trajectory shape (n = 100 slabs of N x 32 B) written by a resident-only grid whose
// waves each own G groups of 64 rows and walk the steps outermost (for s: for g: store the group's 2 KiB of slab s),
// so every wave of the GPU stays within a step of the others and the concurrent writes cover one slab. Group-major
// rows (group g of wave w = rows (g * n_waves + w) * 64: at inner index g the waves write one contiguous window) or
// wave-major ((w * G + g) * 64). Compared with the simulator's one-wave-per-64-rows launch (tools/segment_probe.hip).
// Not part of the library. Build: hipcc -O3 --offload-arch=gfx950 tools/persistent_probe.hip -o tools/_bin/persistent_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int G, bool GROUP_MAJOR>
__global__ __launch_bounds__(256) void persist(f4* traj, long N, int n) {
  const int lane = threadIdx.x & 63;
  const long w = ((long)blockIdx.x * 256 + threadIdx.x) >> 6;
  const long nw = (long)gridDim.x * 4;
  float v = (float)lane;
  for (int s = 0; s < n; ++s) {
    f4* slab = traj + (long)s * N * 2;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const long row0 = (GROUP_MAJOR ? (g * nw + w) : (w * G + g)) * 64;
      f4* dst = slab + row0 * 2;
      __builtin_nontemporal_store(f4{v, v + 1, v + 2, (float)g}, dst + lane);
      __builtin_nontemporal_store(f4{v + 4, v + 5, v + 6, (float)s}, dst + 64 + lane);
    }
    v += 1.f;
  }
}

__global__ __launch_bounds__(256) void seg1(f4* traj, long N, int s0) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  f4* dst = traj + (i - lane) * 2 + (long)s0 * N * 2;
  const float v = (float)i;
  __builtin_nontemporal_store(f4{v, v + 1, v + 2, v + 3}, dst + lane);
  __builtin_nontemporal_store(f4{v + 4, v + 5, v + 6, v + 7}, dst + 64 + lane);
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
  auto rep = [&](const char* name, float ms) { printf("%-40s %7.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms / 1e3) / 1e9); };
  const long groups = N / 64;  // 32768
  for (int rnd = 0; rnd < 2; ++rnd) {
#define RUN(G, GM)                                                                                           \
    {                                                                                                        \
      const int blocks = (int)(groups / G / 4);                                                              \
      char nm[64];                                                                                           \
      snprintf(nm, sizeof nm, "persist G=%d %s (%d waves)", G, GM ? "group-major" : "wave-major", blocks * 4); \
      rep(nm, timeit([&] { persist<G, GM><<<blocks, 256>>>(traj, N, n); }));                                 \
    }
    RUN(4, true) RUN(8, true) RUN(16, true) RUN(32, true) RUN(8, false) RUN(16, false)
    rep("one slab per launch (100 launches)", timeit([&] { for (int s = 0; s < n; ++s) seg1<<<N / 256, 256>>>(traj, N, s); }));
  }
  return 0;
}
