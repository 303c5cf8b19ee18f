// v_mfma_f32_4x4x1_16b_f32 on gfx950: operand / result lane map (exact small integers) and issue rate
// against v_mfma_f32_16x16x4_f32. Build: hipcc --offload-arch=gfx950 -O3 tools/mfma4_probe.hip -o /tmp/mfma4
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(float* out) {
  const int l = threadIdx.x;
  const float a = (float)(l + 1), b = (float)(100 * (l + 1));
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int v = 0; v < 4; ++v) out[l * 4 + v] = c[v];
}

template <int KIND, int NC>
__global__ void rate_kernel(float* out, int iters) {
  const int l = threadIdx.x & 63;
  float a = (float)l * 1e-3f, b = 1e-3f;
  f32x4 c[NC];
#pragma unroll
  for (int q = 0; q < NC; ++q) c[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int q = 0; q < NC; ++q)
      c[q] = KIND ? __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[q], 0, 0, 0) : __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[q], 0, 0, 0);
  }
  f32x4 s = c[0];
#pragma unroll
  for (int q = 1; q < NC; ++q) s += c[q];
  if (s[0] == 12345.f) out[0] = s[1];
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 4 * sizeof(float));
  hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, d);
  float h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // hypothesis: lane 4b + j, register i = A[lane 4b + i] * B[lane 4b + j]
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int v = 0; v < 4; ++v) {
      const int b = l / 4, j = l % 4;
      const float want = (float)(4 * b + v + 1) * (float)(100 * (4 * b + j + 1));
      if (h[l * 4 + v] != want) ++bad;
    }
  printf("layout hypothesis D[lane 4b+j][reg i] = A[4b+i] * B[4b+j]: %s (%d mismatches)\n", bad ? "NO" : "yes", bad);
  if (bad) {
    for (int l = 0; l < 8; ++l) printf("lane %d: %g %g %g %g\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000, blocks = 256 * 4;
  for (int v = 0; v < 6; ++v) {
    const int kind = v & 1, nc = v < 2 ? 8 : (v < 4 ? 16 : 4);
    float ms = 0.f;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (kind) {
        if (nc == 8) hipLaunchKernelGGL((rate_kernel<1, 8>), dim3(blocks), dim3(64), 0, 0, d, iters);
        else if (nc == 16) hipLaunchKernelGGL((rate_kernel<1, 16>), dim3(blocks), dim3(64), 0, 0, d, iters);
        else hipLaunchKernelGGL((rate_kernel<1, 4>), dim3(blocks), dim3(64), 0, 0, d, iters);
      } else {
        if (nc == 8) hipLaunchKernelGGL((rate_kernel<0, 8>), dim3(blocks), dim3(64), 0, 0, d, iters);
        else if (nc == 16) hipLaunchKernelGGL((rate_kernel<0, 16>), dim3(blocks), dim3(64), 0, 0, d, iters);
        else hipLaunchKernelGGL((rate_kernel<0, 4>), dim3(blocks), dim3(64), 0, 0, d, iters);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    const double macs = (double)blocks * iters * nc * (kind ? 1024 : 256);
    printf("%s %2d chains: %.3f ms, %.1f TFLOP/s (one wave per SIMD)\n", kind ? "16x16x4f32" : "4x4x1f32  ", nc, ms,
           2 * macs / ms / 1e9);
  }
  return 0;
}
