// layout_probe.hip — which trajectory write layout holds its rate on ANY physical placement?
// The C2 simulator's time-major stores ran 1.2 ms on some hipMalloc buffers, 1.5 ms on others
// and 1.9-2.1 ms on physically contiguous ones (tools/alloc_probe.cpp), while a memset of the same
// bytes runs 6.2-6.5 TB/s everywhere. Each kernel here writes the C2 trajectory bytes (2^21 rows
// x 32 B x 100 steps) with `work` dependent FMAs between steps (the simulator's update), in:
//   0 time-major   : wave w, step s -> base + s*N*32 + w*2 KiB       (the current layout)
//   1 wave tiles   : wave w, step s -> base + (w*n + s)*2 KiB        ([N/64, n, 64, 2d])
//   2 block tiles  : block b, step s -> base + (b*n + s)*8 KiB + wave*2 KiB
// on hipMalloc and on hipExtMallocWithFlags(Contiguous) buffers. Not part of the library.
// Build: hipcc -O3 --offload-arch=gfx950 tools/layout_probe.hip -o tools/_bin/layout_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f4 __attribute__((ext_vector_type(4)));

// FEAT bits (time-major only): 1 = also store tau [n, N] (4 B per lane per step, nt);
// 2 = stage the rows through LDS as the simulator does (row -> LDS -> 16 B chunks)
template <int LAYOUT, int FEAT = 0>
__global__ __launch_bounds__(256) void writer(f4* traj, long N, int n, int work, float* tau) {
  __shared__ f4 stage[(FEAT & 2) ? 512 : 1];
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long w = i >> 6;  // global wave
  float v = (float)i, acc = v;
  for (int s = 0; s < n; ++s) {
    for (int k = 0; k < work; ++k) acc = fmaf(acc, 0.999f, 0.5f);
    f4* dst;
    if (LAYOUT == 0) dst = traj + ((long)s * N + w * 64) * 2;
    else if (LAYOUT == 1) dst = traj + (w * n + s) * 128;
    else dst = traj + ((long)blockIdx.x * n + s) * 512 + wave * 128;
    f4 a = f4{acc, v + 1, v + 2, v + 3}, b = f4{v + 4, v + 5, v + 6, acc};
    if constexpr ((FEAT & 2) != 0) {
      f4* slot = stage + wave * 128;
      slot[2 * lane] = a;
      slot[2 * lane + 1] = b;
      __builtin_amdgcn_wave_barrier();
      a = slot[lane];
      b = slot[64 + lane];
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_nontemporal_store(a, dst + lane);
    __builtin_nontemporal_store(b, dst + 64 + lane);
    if constexpr ((FEAT & 1) != 0) __builtin_nontemporal_store(acc, tau + (long)s * N + i);
    v += 1.f;
  }
}

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
  } while (0)

int main(int argc, char** argv) {
  const long N = 1 << 21;
  const int n = 100;
  const size_t bytes = (size_t)N * n * 32;
  const int sets = argc > 1 ? atoi(argv[1]) : 2;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int kind = 0; kind < 2; ++kind)
    for (int k = 0; k < sets; ++k) {
      f4* p;
      if (kind == 0) CK(hipMalloc(&p, bytes));
      else if (hipExtMallocWithFlags((void**)&p, bytes, hipDeviceMallocContiguous) != hipSuccess) {
        printf("contiguous alloc failed\n");
        continue;
      }
      float* tau;
      CK(hipMalloc(&tau, (size_t)N * n * 4));
      for (int work : {0, 64, 200}) {
        float ms[8];
        for (int L = 0; L < 8; ++L) {
          // dynamic LDS 24 KiB on variant 7: at most 6 workgroups per CU (the simulator's ~5)
          auto run = [&]() {
            if (L == 0) writer<0><<<N / 256, 256>>>(p, N, n, work, tau);
            if (L == 1) writer<1><<<N / 256, 256>>>(p, N, n, work, tau);
            if (L == 2) writer<2><<<N / 256, 256>>>(p, N, n, work, tau);
            if (L == 3) CK(hipMemsetAsync(p, 0, bytes, nullptr));
            if (L == 4) writer<0, 1><<<N / 256, 256>>>(p, N, n, work, tau);
            if (L == 5) writer<0, 2><<<N / 256, 256>>>(p, N, n, work, tau);
            if (L == 6) writer<0, 3><<<N / 256, 256>>>(p, N, n, work, tau);
            if (L == 7) writer<0, 3><<<N / 256, 256, 24576>>>(p, N, n, work, tau);
          };
          for (int r = 0; r < 3; ++r) run();
          CK(hipEventRecord(e0, nullptr));
          for (int r = 0; r < 10; ++r) run();
          CK(hipEventRecord(e1, nullptr));
          CK(hipEventSynchronize(e1));
          CK(hipEventElapsedTime(&ms[L], e0, e1));
          ms[L] /= 10;
        }
        printf("%-10s set %d work %3d: time-major %.0f | wave-tiles %.0f | block-tiles %.0f | memset %.0f | "
               "tm+tau %.3f ms | tm+lds %.3f ms | tm+tau+lds %.3f ms | +occ6 %.3f ms\n",
               kind ? "contiguous" : "hipMalloc", k, work, bytes / ms[0] / 1e6, bytes / ms[1] / 1e6,
               bytes / ms[2] / 1e6, bytes / ms[3] / 1e6, ms[4], ms[5], ms[6], ms[7]);
        fflush(stdout);
      }
      // not freed: the next set must get different memory
    }
  return 0;
}
