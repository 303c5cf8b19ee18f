// Store-pattern calibration for the simulator's trajectory writes (not part of the library).
// Writes the C2 trajectory shape (n = 100 slabs of N x 32 B, time-major) with no arithmetic, in
// the simulator's wave-staged form, for several block sizes and store policies; plus a flat
// contiguous fill of the same bytes for reference. Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));

// every wave owns 64 consecutive rows of 32 B; per step it writes its 2 KiB piece of slab s
template <int B, int POL>
__global__ __launch_bounds__(B) void sim_like(f4* traj, long N, int n) {
  const long i = (long)blockIdx.x * B + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const long wave_row0 = i - lane;
  f4* base = traj + wave_row0 * 2;  // 2 f4 per row
  float v = (float)i;
  for (int s = 0; s < n; ++s) {
    f4* dst = base + (long)s * N * 2;
    const f4 a = f4{v, v + 1, v + 2, v + 3}, b = f4{v + 4, v + 5, v + 6, v + 7};
    if (POL == 0) {
      __builtin_nontemporal_store(a, dst + lane);
      __builtin_nontemporal_store(b, dst + 64 + lane);
    } else {
      dst[lane] = a;
      dst[64 + lane] = b;
    }
    v += 1.f;
  }
}

// sim_like variants: DATA = 0 same data every step, LDS = 1 allocates (and touches) 8 KiB of LDS
template <int DATA, int LDS>
__global__ __launch_bounds__(256) void sim_like_v(f4* traj, long N, int n) {
  __shared__ f4 stage[LDS ? 512 : 1];
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const long wave_row0 = i - lane;
  f4* base = traj + wave_row0 * 2;
  float v = (float)i;
  if (LDS) stage[threadIdx.x] = f4{v, v, v, v};
  for (int s = 0; s < n; ++s) {
    f4* dst = base + (long)s * N * 2;
    f4 a = f4{v, v + 1, v + 2, v + 3}, b = f4{v + 4, v + 5, v + 6, v + 7};
    if (LDS) a += stage[(threadIdx.x + s) & 255];
    __builtin_nontemporal_store(a, dst + lane);
    __builtin_nontemporal_store(b, dst + 64 + lane);
    if (DATA) v += 1.f;
  }
}

// two particles per lane: the wave owns 128 consecutive rows, 4 KiB per step (4 stores)
template <int B>
__global__ __launch_bounds__(B) void sim_like2(f4* traj, long N, int n) {
  const long w = ((long)blockIdx.x * B + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  f4* base = traj + w * 128 * 2;
  float v = (float)lane;
  for (int s = 0; s < n; ++s) {
    f4* dst = base + (long)s * N * 2;
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(f4{v, v + 1, v + 2, v + (float)k}, dst + k * 64 + lane);
    v += 1.f;
  }
}

// the same bytes, but every wave sweeps a contiguous range of the whole (particle-major) output
template <int B>
__global__ __launch_bounds__(B) void flat(f4* p, long n4) {
  const long per_block = n4 / gridDim.x;
  f4* q = p + (long)blockIdx.x * per_block;
  for (long k = threadIdx.x; k < per_block; k += B) __builtin_nontemporal_store(f4{1.f, 2.f, 3.f, 4.f}, q + k);
}

// one-shot grids (no grid-stride loop), VPT 16-byte vectors per thread:
//   thread-major: thread t writes VPT consecutive vectors (lanes of one instruction 16*VPT B apart)
//   lane-major:   instruction k of the block writes one contiguous 4 KiB run
template <int VPT, bool THREAD_MAJOR>
__global__ __launch_bounds__(256) void oneshot(f4* p) {
  f4* q = p + (long)blockIdx.x * 256 * VPT;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const long off = THREAD_MAJOR ? (long)threadIdx.x * VPT + k : (long)k * 256 + threadIdx.x;
    q[off] = f4{1.f, 2.f, 3.f, (float)k};
  }
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
  printf("traj %p\n", (void*)traj);
  auto rep = [&](const char* name, float ms) { printf("%-34s %7.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms / 1e3) / 1e9); };
  rep("sim_like B=256 nt", timeit([&] { sim_like<256, 0><<<N / 256, 256>>>(traj, N, n); }));
  rep("sim_like B=256 plain", timeit([&] { sim_like<256, 1><<<N / 256, 256>>>(traj, N, n); }));
  rep("sim_like_v const data", timeit([&] { sim_like_v<0, 0><<<N / 256, 256>>>(traj, N, n); }));
  rep("sim_like_v varying data + LDS", timeit([&] { sim_like_v<1, 1><<<N / 256, 256>>>(traj, N, n); }));
  rep("sim_like_v const data + LDS", timeit([&] { sim_like_v<0, 1><<<N / 256, 256>>>(traj, N, n); }));
  rep("sim_like B=256 nt (again)", timeit([&] { sim_like<256, 0><<<N / 256, 256>>>(traj, N, n); }));
  rep("sim_like B=512 nt", timeit([&] { sim_like<512, 0><<<N / 512, 512>>>(traj, N, n); }));
  rep("sim_like B=1024 nt", timeit([&] { sim_like<1024, 0><<<N / 1024, 1024>>>(traj, N, n); }));
  rep("sim_like B=1024 plain", timeit([&] { sim_like<1024, 1><<<N / 1024, 1024>>>(traj, N, n); }));
  rep("sim_like B=64 nt", timeit([&] { sim_like<64, 0><<<N / 64, 64>>>(traj, N, n); }));
  rep("sim_like2 (2 rows/lane) B=256", timeit([&] { sim_like2<256><<<N / 512, 256>>>(traj, N, n); }));
  rep("sim_like2 (2 rows/lane) B=128", timeit([&] { sim_like2<128><<<N / 256, 128>>>(traj, N, n); }));
  const long nv = (long)(bytes / 16);
  rep("oneshot thread-major VPT=4", timeit([&] { oneshot<4, true><<<nv / 1024, 256>>>(traj); }));
  rep("oneshot thread-major VPT=8", timeit([&] { oneshot<8, true><<<nv / 2048, 256>>>(traj); }));
  rep("oneshot lane-major VPT=4", timeit([&] { oneshot<4, false><<<nv / 1024, 256>>>(traj); }));
  rep("oneshot lane-major VPT=16", timeit([&] { oneshot<16, false><<<nv / 4096, 256>>>(traj); }));
  rep("hipMemsetD32Async", timeit([&] { (void)hipMemsetD32Async((hipDeviceptr_t)traj, 0x3f800000, bytes / 4, 0); }));
  for (int g : {1024, 4096, 16384, 65536})
    printf("flat grid %-5d", g), rep("", timeit([&] { flat<256><<<g, 256>>>(traj, (long)(bytes / 16)); }));
  return 0;
}
