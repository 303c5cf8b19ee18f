// alloc_probe.cpp — is the C2 simulator's launch time a property of the output buffer's
// physical placement? Times pdeinv_sde_simulate (d=4 KOU, 2^21 particles, n=100, fused moments)
// on several output-buffer sets made by hipMalloc and by hipExtMallocWithFlags(Contiguous),
// with and without the tau output, plus hipMemsetAsync of the same trajectory bytes.
// Build: hipcc -O2 --offload-arch=gfx950 tools/alloc_probe.cpp -Iinclude
//        -Lpde-inverse-problem_amd/_build -lpdeinv -Wl,-rpath,$PWD/pde-inverse-problem_amd/_build
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "pdeinv.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static const int d = 4, n = 100;
static int64_t N = 1 << 21;

struct Set {
  float *traj, *tau, *last;
  const char* how;
};

static bool alloc(void** p, size_t bytes, int kind) {
  if (kind == 0) return hipMalloc(p, bytes) == hipSuccess;
  return hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess;
}

int main(int argc, char** argv) {
  const int per_kind = argc > 1 ? atoi(argv[1]) : 3;
  if (argc > 2) N += atoll(argv[2]);  // N = 2^21 + extra rows: breaks the power-of-two step stride
  printf("N = %lld particles, step stride %lld B\n", (long long)N, (long long)N * 2 * d * 4);
  const size_t traj_b = (size_t)n * N * 2 * d * 4, tau_b = (size_t)n * N * 4, last_b = (size_t)N * 2 * d * 4;
  float* z0;
  CK(hipMalloc(&z0, last_b));
  std::vector<float> h(N * 2 * d);
  srand(1);
  for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
  CK(hipMemcpy(z0, h.data(), last_b, hipMemcpyHostToDevice));
  float F[16] = {2, 0.3f, 0.1f, 0, 0.3f, 1.5f, 0.2f, 0.1f, 0.1f, 0.2f, 1.8f, 0.3f, 0, 0.1f, 0.3f, 1.2f};
  pdeinv_sde_desc desc;
  memset(&desc, 0, sizeof desc);
  desc.n_particles = N;
  desc.dim = d;
  desc.n_steps = n;
  desc.dt = 0.02f;
  desc.gamma = 1.f;
  desc.noise_scale = 1.41421356f;
  desc.random_shift = 1;
  desc.seed = 1;
  desc.potential.kind = PDEINV_POT_QUADRATIC;
  desc.potential.params = F;
  void* ws;
  CK(hipMalloc(&ws, pdeinv_sde_workspace_bytes(&desc)));
  double* mom;
  CK(hipMalloc(&mom, 3 * pdeinv_moment_len(2 * d) * sizeof(double)));

  std::vector<Set> sets;
  for (int kind = 0; kind < 2; ++kind)
    for (int k = 0; k < per_kind; ++k) {
      Set s{nullptr, nullptr, nullptr, kind ? "contiguous" : "hipMalloc"};
      if (!alloc((void**)&s.traj, traj_b, kind) || !alloc((void**)&s.tau, tau_b, kind) ||
          !alloc((void**)&s.last, last_b, kind)) {
        printf("%s alloc %d failed\n", s.how, k);
        (void)hipGetLastError();
        continue;
      }
      sets.push_back(s);
    }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double byt = (double)N * (8 * d + n * (8 * d + 4) + 8 * d);
  for (int rnd = 0; rnd < 2; ++rnd)
    for (size_t k = 0; k < sets.size(); ++k) {
      Set& s = sets[k];
      float ms[3];
      for (int v = 0; v < 3; ++v) {
        for (int w = 0; w < 3; ++w)
          if (pdeinv_sde_simulate(&desc, z0, s.traj, s.tau, s.last, ws, mom, nullptr)) {
            printf("err %s\n", pdeinv_last_error());
            return 1;
          }
        CK(hipEventRecord(e0, nullptr));
        for (int r = 0; r < 20; ++r) {
          if (v == 0) pdeinv_sde_simulate(&desc, z0, s.traj, s.tau, s.last, ws, mom, nullptr);
          if (v == 1) pdeinv_sde_simulate(&desc, z0, s.traj, nullptr, s.last, ws, mom, nullptr);
          if (v == 2) CK(hipMemsetAsync(s.traj, 0, traj_b, nullptr));
        }
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[v], e0, e1));
        ms[v] /= 20;
      }
      printf("round %d set %zu %-10s traj %p: sim %.4f ms (%.0f GB/s) | sim-no-tau %.4f ms | memset %.0f GB/s\n",
             rnd, k, s.how, (void*)s.traj, ms[0], byt / ms[0] / 1e6, ms[1], traj_b / ms[2] / 1e6);
      fflush(stdout);
    }
  return 0;
}
