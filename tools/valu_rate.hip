// VALU issue cost per wave64 instruction on one MI355X, for the opcodes of the C3 step loop (fused simulate + GMM
// residual, sde.hip): every CU runs W waves per SIMD (argv[1], default 3 = C3's occupancy), each wave 8
// independent chains of one opcode (inline asm, so the opcode is exactly the one named). Two clocks:
//   real    = s_memtime ticks (shader clock) of the loop, read by every wave: cycles per instruction per SIMD =
//             ticks / (instructions per wave x W) — the clock the chip actually ran under this load;
//   nominal = HIP-event wall time x 2.4 GHz (the clock the 157.3 TFLOP/s fp32 peak is quoted at).
// The loop is unrolled 8 x 8 (64 instructions of the opcode per loop branch). Prints one JSON line per opcode; run
// under rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE (tools/r05_valu_pmc.sh) for the SIMD cycles
// per instruction in the SQ's own accounting, which tools/c3_valu_model.py prices the C3 step loop with.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o tools/_bin/valu_rate && tools/_bin/valu_rate 3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kIters = 2048, kChains = 8;
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define BODY_F(ASM)                                                                  \
  float x[kChains];                                                                  \
  for (int c = 0; c < kChains; ++c) x[c] = 1.1f + 1e-6f * (threadIdx.x + c) + seed; \
  const float k1 = 0.999f, k2 = 0.001f;                                              \
  const uint64_t t0 = __builtin_amdgcn_s_memtime();                                  \
  _Pragma("unroll 8") for (int it = 0; it < kIters; ++it) {                          \
    _Pragma("unroll") for (int c = 0; c < kChains; ++c) asm volatile(ASM : "+v"(x[c]) : "v"(k1), "v"(k2)); \
  }                                                                                  \
  const uint64_t t1 = __builtin_amdgcn_s_memtime();                                  \
  float s = 0;                                                                       \
  for (int c = 0; c < kChains; ++c) s += x[c];                                       \
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                    \
  if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;

#define BODY_P(ASM)                                                                  \
  f32x2 x[kChains];                                                                  \
  for (int c = 0; c < kChains; ++c) x[c] = f32x2{1.1f + seed + c, 0.9f - 1e-6f * threadIdx.x}; \
  const f32x2 k1 = {0.999f, 0.998f}, k2 = {0.001f, 0.002f};                          \
  const uint64_t t0 = __builtin_amdgcn_s_memtime();                                  \
  _Pragma("unroll 8") for (int it = 0; it < kIters; ++it) {                          \
    _Pragma("unroll") for (int c = 0; c < kChains; ++c) asm volatile(ASM : "+v"(x[c]) : "v"(k1), "v"(k2)); \
  }                                                                                  \
  const uint64_t t1 = __builtin_amdgcn_s_memtime();                                  \
  float s = 0;                                                                       \
  for (int c = 0; c < kChains; ++c) s += x[c][0] + x[c][1];                          \
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                    \
  if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;

#define KF(NAME, ASM) \
  __global__ void NAME(float* out, uint64_t* ticks, float seed) { BODY_F(ASM) }
#define KP(NAME, ASM) \
  __global__ void NAME(float* out, uint64_t* ticks, float seed) { BODY_P(ASM) }

KF(k_fma, "v_fma_f32 %0, %0, %1, %2")
KF(k_add, "v_add_f32 %0, %0, %1")
KF(k_mul, "v_mul_f32 %0, %0, %1")
KF(k_max, "v_max_f32 %0, %0, %1")
KF(k_mov, "v_mov_b32 %0, %1")
KF(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KF(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KF(k_exp, "v_exp_f32 %0, %0")
KF(k_log, "v_log_f32 %0, %0")
KF(k_sin, "v_sin_f32 %0, %0")
KF(k_rcp, "v_rcp_f32 %0, %0")
KF(k_sqrt, "v_sqrt_f32 %0, %0")
KP(k_pk_fma, "v_pk_fma_f32 %0, %0, %1, %2")
KP(k_pk_mul, "v_pk_mul_f32 %0, %0, %1")
KP(k_pk_add, "v_pk_add_f32 %0, %0, %1")
KP(k_mov_b64, "v_mov_b64 %0, %1")
KP(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %1")

// a transcendental beside other VALU work: chain 0 v_exp_f32, chains 1..7 v_pk_fma_f32 (the C3 loop issues one
// transcendental per ~15 other VALU instructions) — prices the exp when it is not the only thing issuing
__global__ void k_mix_exp_pk(float* out, uint64_t* ticks, float seed) {
  f32x2 x[kChains];
  for (int c = 0; c < kChains; ++c) x[c] = f32x2{1.1f + seed + c, 0.9f - 1e-6f * threadIdx.x};
  const f32x2 k1 = {0.999f, 0.998f}, k2 = {0.001f, 0.002f};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int it = 0; it < kIters; ++it) {
    asm volatile("v_exp_f32 %0, %0" : "+v"(x[0][0]));
#pragma unroll
    for (int c = 1; c < kChains; ++c) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(k1), "v"(k2));
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int c = 0; c < kChains; ++c) s += x[c][0] + x[c][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

__global__ void k_mad_u64(float* out, uint64_t* ticks, float seed) {
  uint64_t x[kChains];
  for (int c = 0; c < kChains; ++c) x[c] = 0x12345u + threadIdx.x * 7 + c + (uint32_t)seed;
  const uint32_t m = 0xD2511F53u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      uint64_t r;
      asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %3" : "=v"(r) : "v"(m), "v"((uint32_t)x[c]), "v"(x[c])
                   : "s100", "s101");
      x[c] = r;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t s = 0;
  for (int c = 0; c < kChains; ++c) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(uint32_t)s;
  if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 3;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount, simds = cus * 4;
  const int threads = 256, blocks = cus * W;  // 4 waves per block, one per SIMD: W waves per SIMD
  const double waves = (double)blocks * threads / 64;
  float* buf;
  uint64_t* tk;
  hipMalloc(&buf, (size_t)blocks * threads * 4);
  hipMalloc(&tk, (size_t)blocks * 4 * 8);
  uint64_t* h = (uint64_t*)malloc((size_t)blocks * 4 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  // dynamic LDS per block sized so that exactly W blocks fit on a CU (160 KiB / W): the dispatcher cannot stack more
  // on some CUs than on others, so every SIMD runs W waves for the whole launch
  const size_t lds = (size_t)(160 * 1024 / W) - 1024;
  auto run = [&](const char* name, void (*k)(float*, uint64_t*, float)) {
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), lds, 0, buf, tk, 1.f);
    hipDeviceSynchronize();
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), lds, 0, buf, tk, 1.f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(h, tk, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
    double mt = 0;
    for (int i = 0; i < blocks * 4; ++i) mt += (double)h[i];
    mt /= blocks * 4;
    const double insts = (double)kIters * kChains;
    const double real = mt / (insts * W);  // shader cycles per wave-instruction per SIMD
    const double t = ms / reps * 1e-3;
    const double nominal = t * 2.4e9 * simds / (waves * insts);
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"real_cycles\": %.3f, \"nominal_cycles\": %.3f, "
           "\"clock_ghz\": %.3f}\n", name, W, real, nominal, mt / t * 1e-9 * (t > 0 ? 1.0 : 0.0));
  };
  run("v_fma_f32", k_fma);
  run("v_add_f32", k_add);
  run("v_mul_f32", k_mul);
  run("v_max_f32", k_max);
  run("v_mov_b32", k_mov);
  run("v_bitop3_b32", k_bitop3);
  run("v_and_or_b32", k_and_or);
  run("v_exp_f32", k_exp);
  run("v_log_f32", k_log);
  run("v_sin_f32", k_sin);
  run("v_rcp_f32", k_rcp);
  run("v_sqrt_f32", k_sqrt);
  run("v_pk_fma_f32", k_pk_fma);
  run("v_pk_mul_f32", k_pk_mul);
  run("v_pk_add_f32", k_pk_add);
  run("v_mov_b64", k_mov_b64);
  run("v_lshl_add_u64", k_lshl_add_u64);
  run("v_mad_u64_u32", k_mad_u64);
  run("mix: v_exp_f32 + 7 v_pk_fma_f32", k_mix_exp_pk);
  hipFree(buf);
  hipFree(tk);
  free(h);
  return 0;
}
