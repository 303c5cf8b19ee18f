// slab_pad_probe.hip — does the trajectory's slab stride set the simulator's store rate?
// The C2 trajectory is [n = 100][N = 2^21][32 B]: every update's slab starts exactly 64 MiB after the previous one,
// so the waves of neighbouring updates (a few updates apart at any moment) write addresses that differ by a multiple
// of 64 MiB — the same HBM channel / bank bits, different rows. This probe writes the simulator's store shape (each
// wave 2 KiB of slab s per step, 16-byte chunks, the tau row beside it) with the slab stride padded by P bytes, on
// three separate allocations, and reports TB/s of the 6.7 GB of trajectory bytes. Not part of the library.
// Build: hipcc -O3 --offload-arch=gfx950 tools/slab_pad_probe.hip -o tools/_bin/slab_pad_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void writer(f4* traj, long N, int n, long slab_f4, int work) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const long wave_row0 = i - lane;
  f4* base = traj + wave_row0 * 2;  // 2 f4 per 32-byte row
  float v = (float)i, acc = v;
  for (int s = 0; s < n; ++s) {
    for (int k = 0; k < work; ++k) acc = fmaf(acc, 0.999f, 0.5f);
    f4* dst = base + (long)s * slab_f4;
    const f4 a = f4{acc, v + 1, v + 2, v + 3}, b = f4{v + 4, v + 5, v + 6, acc};
    if (NT) {
      __builtin_nontemporal_store(a, dst + lane);
      __builtin_nontemporal_store(b, dst + 64 + lane);
    } else {
      dst[lane] = a;
      dst[64 + lane] = b;
    }
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
  const long slab = N * 32;  // bytes
  const long pads[] = {0, 256, 2048, 4096 + 256, 65536 + 768, (2L << 20) + 4096, 3 * 1024 * 1024 + 512};
  const int npad = sizeof(pads) / sizeof(pads[0]);
  const size_t bytes = (size_t)(slab + pads[npad - 1]) * n;
  f4* bufs[3];
  for (int a = 0; a < 3; ++a)
    if (hipMalloc(&bufs[a], bytes) != hipSuccess) return 1;
  for (int work : {0, 64}) {
    for (int a = 0; a < 3; ++a) {
      printf("alloc %d work %3d:", a, work);
      for (int p = 0; p < npad; ++p) {
        const long sf4 = (slab + pads[p]) / 16;
        const float ms = timeit([&] { writer<true><<<N / 256, 256>>>(bufs[a], N, n, sf4, work); });
        printf(" pad %ld %.0f", pads[p], (double)slab * n / (ms / 1e3) / 1e9);
      }
      const float msp = timeit([&] { writer<false><<<N / 256, 256>>>(bufs[a], N, n, slab / 16, work); });
      printf(" | plain pad 0 %.0f GB/s\n", (double)slab * n / (msp / 1e3) / 1e9);
    }
  }
  return 0;
}
