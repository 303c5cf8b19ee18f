// 4 x 4 transpose across the four 16-lane groups of a wave with v_permlane32_swap + v_permlane16_swap:
// register i of lane group g holds X[g][i] -> afterwards register i of group g holds X[i][g].
// Build: hipcc --offload-arch=gfx950 -O3 tools/transpose4_probe.hip -o tools/transpose4_probe.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ __forceinline__ void swap32(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__global__ void k(float* o) {
  const int l = threadIdx.x, g = l >> 4, p = l & 15;
  float r[4];
  for (int i = 0; i < 4; ++i) r[i] = 1000.f * g + 100.f * i + p;
  swap32(r[0], r[2]);
  swap32(r[1], r[3]);
  swap16(r[0], r[1]);
  swap16(r[2], r[3]);
  for (int i = 0; i < 4; ++i) o[l * 4 + i] = r[i];
}
int main() {
  float* d;
  (void)hipMalloc(&d, 256 * sizeof(float));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[256];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int g = l >> 4, p = l & 15;
      const float want = 1000.f * i + 100.f * g + p;  // X[i][g]
      if (h[l * 4 + i] != want) ++bad;
    }
  printf("transpose4 (swap32 r0/r2, r1/r3; swap16 r0/r1, r2/r3): %s (%d mismatches)\n", bad ? "NO" : "yes", bad);
  if (bad)
    for (int l = 0; l < 64; l += 16) printf("lane %d: %g %g %g %g\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  return 0;
}
