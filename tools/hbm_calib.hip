// Streaming-store / copy calibration for the roofline discussion (not part of the library).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void wr(f4* p, size_t n, float v) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(f4{v, v + 1, v + 2, v + 3}, p + i);
}
__global__ void wr_plain(f4* p, size_t n, float v) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = f4{v, v, v, v};
}
__global__ void cp(const f4* a, f4* b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
int main() {
  size_t bytes = 7616000000ull, n = bytes / 16;
  f4 *p, *q;
  hipMalloc(&p, bytes); hipMalloc(&q, bytes);
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  for (int g : {2048, 8192, 65536}) {
    for (int k = 0; k < 3; ++k) {
      float ms;
      hipEventRecord(s); for (int r = 0; r < 5; ++r) wr<<<g, 256>>>(p, n, r); hipEventRecord(e); hipEventSynchronize(e);
      hipEventElapsedTime(&ms, s, e); if (k == 2) printf("grid %6d nt-store  %.1f GB/s\n", g, 5 * bytes / (ms / 1e3) / 1e9);
      hipEventRecord(s); for (int r = 0; r < 5; ++r) wr_plain<<<g, 256>>>(p, n, r); hipEventRecord(e); hipEventSynchronize(e);
      hipEventElapsedTime(&ms, s, e); if (k == 2) printf("grid %6d store     %.1f GB/s\n", g, 5 * bytes / (ms / 1e3) / 1e9);
      hipEventRecord(s); for (int r = 0; r < 5; ++r) cp<<<g, 256>>>(p, q, n / 2); hipEventRecord(e); hipEventSynchronize(e);
      hipEventElapsedTime(&ms, s, e); if (k == 2) printf("grid %6d copy      %.1f GB/s (r+w)\n", g, 5 * bytes / (ms / 1e3) / 1e9);
    }
  }
  return 0;
}
