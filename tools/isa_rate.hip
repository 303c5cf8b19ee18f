// Issue cost of the simulator step's instruction mix on one MI355X (SIMD cycles per wave64
// instruction): 8 independent chains per lane, 4 waves per SIMD on every CU, timed with hip events;
// cycles = time * clock * SIMDs / (waves * instructions). The clock is read from the device.
//   hipcc -O3 --offload-arch=gfx950 tools/isa_rate.hip -o tools/isa_rate && tools/isa_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 4096, kChains = 8;

__global__ void k_mad_u64(uint32_t* out, uint32_t seed) {
  uint32_t x[kChains];
  for (int c = 0; c < kChains; ++c) x[c] = seed + threadIdx.x * 7 + c;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      const uint64_t p = (uint64_t)0xD2511F53u * x[c];
      x[c] = (uint32_t)(p >> 32) ^ (uint32_t)p;  // v_mad_u64_u32 + one xor
    }
  }
  uint32_t s = 0;
  for (int c = 0; c < kChains; ++c) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma(float* out, float seed) {
  float x[kChains];
  for (int c = 0; c < kChains; ++c) x[c] = seed + threadIdx.x + c;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = fmaf(x[c], 0.999f, 0.001f);
  }
  float s = 0;
  for (int c = 0; c < kChains; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// v_pk_fma_f32: two fp32 FMAs per lane per instruction (the C3 kernel's centre-pair math)
__global__ void k_pk_fma(float* out, float seed) {
  f32x2 x[kChains];
  for (int c = 0; c < kChains; ++c) x[c] = f32x2{seed + threadIdx.x + c, seed - threadIdx.x - c};
  const f32x2 m = {0.999f, 0.998f}, a = {0.001f, 0.002f};
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = x[c] * m + a;
  }
  float s = 0;
  for (int c = 0; c < kChains; ++c) s += x[c][0] + x[c][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_xor(uint32_t* out, uint32_t seed) {
  uint32_t x[kChains];
  for (int c = 0; c < kChains; ++c) x[c] = seed + threadIdx.x * 7 + c;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = __builtin_amdgcn_bitop3_b32(x[c], 0x9E3779B9u, x[(c + 1) % kChains], 0x96);
  }
  uint32_t s = 0;
  for (int c = 0; c < kChains; ++c) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_log(float* out, float seed) {
  float x[kChains];
  for (int c = 0; c < kChains; ++c) x[c] = 1.5f + 1e-6f * (threadIdx.x + c) + seed;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = __builtin_amdgcn_logf(x[c]) + 1.5f;
  }
  float s = 0;
  for (int c = 0; c < kChains; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const int cus = p.multiProcessorCount, simds = cus * 4;
  const int blocks = cus * 4, threads = 256;  // 16 waves / CU = 4 per SIMD
  void* buf;
  hipMalloc(&buf, (size_t)blocks * threads * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double waves = (double)blocks * threads / 64;
  auto run = [&](const char* name, auto launch, double insts_per_iter, double flop_per_lane_inst = 0) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double t = ms / 5 * 1e-3;
    const double cyc = t * clk_khz * 1e3 * simds / (waves * kIters * kChains * insts_per_iter);
    printf("%-40s %.3f ms  %.2f SIMD cycles per wave-instruction (clock %d MHz)", name, ms / 5, cyc, clk_khz / 1000);
    if (flop_per_lane_inst > 0)  // chip-wide fp32 rate at the measured issue cost
      printf("  %.1f TFLOP/s", waves * 64 * kIters * kChains * insts_per_iter * flop_per_lane_inst / t / 1e12);
    printf("\n");
  };
  run("v_mad_u64_u32 (+ v_xor)", [&] { hipLaunchKernelGGL(k_mad_u64, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)buf, 1u); }, 1.0);
  run("v_fma_f32", [&] { hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, (float*)buf, 1.f); }, 1.0, 2.0);
  run("v_pk_fma_f32", [&] { hipLaunchKernelGGL(k_pk_fma, dim3(blocks), dim3(threads), 0, 0, (float*)buf, 1.f); }, 1.0, 4.0);
  run("v_bitop3_b32", [&] { hipLaunchKernelGGL(k_xor, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)buf, 1u); }, 1.0);
  run("v_log_f32 (+ v_add)", [&] { hipLaunchKernelGGL(k_log, dim3(blocks), dim3(threads), 0, 0, (float*)buf, 0.f); }, 1.0);
  hipFree(buf);
  return 0;
}
