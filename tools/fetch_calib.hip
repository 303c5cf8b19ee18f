// fetch_calib.hip — what FETCH_SIZE reports for coalesced streaming reads of 4, 8 and 16 bytes per lane (gfx950).
// MI355X_MICROARCH.md: for 16-B-per-lane reads FETCH_SIZE is exactly half the bytes (128-B requests tallied at 64 B)
// and "other access widths are uncalibrated". The C5 plane loads are 4 B per lane (mlp_fused.hip ldo / wgrad2), so the
// per-kernel traffic of tools/c5_traffic.py (FETCH_SIZE x 2 + WRITE_SIZE) needs this calibration. Each kernel reads
// the same 1 GiB once (a grid-stride sum into one float per thread, written out so nothing is dead).
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/_bin/fetch_calib
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/_bin/fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename T>
__global__ __launch_bounds__(256) void read_width(const T* __restrict__ p, long n, float* __restrict__ out) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const T v = p[i];
    if constexpr (sizeof(T) == 4) s += v;
    else if constexpr (sizeof(T) == 8) s += v[0] + v[1];
    else s += v[0] + v[1] + v[2] + v[3];
  }
  out[(long)blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  const size_t bytes = 1ul << 30;
  float* buf;
  float* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4096 * 256 * sizeof(float)) != hipSuccess) return 1;
  if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
  for (int rep = 0; rep < 2; ++rep) {
    read_width<float><<<4096, 256>>>(buf, (long)(bytes / 4), out);
    read_width<f2><<<4096, 256>>>(reinterpret_cast<const f2*>(buf), (long)(bytes / 8), out);
    read_width<f4><<<4096, 256>>>(reinterpret_cast<const f4*>(buf), (long)(bytes / 16), out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("read 1 GiB at 4, 8, 16 B per lane, twice each\n");
  return 0;
}
