/* Host AddressSanitizer / UBSan driver for the CPU oracle (the optional
 * -fsanitize=address host build). TEST INFRASTRUCTURE ONLY: it compiles pdeinv_oracle.c into one
 * executable with -fsanitize=address,undefined (oracle/Makefile target `asan`) and runs every oracle
 * entry point on small ragged inputs — partial Philox blocks (d = 3, 5), N = 0, 1 and 37, explicit
 * noise, the interacting McKean–Vlasov system, strided rows — plus the Random123 Philox4x32-10 KATs
 * (SURVEY.md §8(c) P7). Any out-of-bounds access or UB aborts with a sanitizer report; the exit code
 * is the number of failed checks. Run by tests/test_oracle.py::test_oracle_under_asan. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]);
int oracle_sde_simulate(int64_t N, int64_t particle_offset, int d, int n_steps, float dt, float gamma,
                        float noise_scale, int random_shift, uint64_t seed, uint32_t counter_offset, int kind,
                        int K, float sigma, const float* params, int has_center, const float* noise,
                        const float* shift_u, const float* z0, int64_t ld_z0, float* traj, float* tau, float* last);
void oracle_moments(const float* z, int64_t n, int m, int64_t ld, double* out);
void oracle_gaussian_sample(int64_t n, int m, uint64_t seed, uint32_t counter_offset, int64_t row_offset,
                            const float* mean, const float* cov_half, float* out);
void oracle_philox_fill(uint64_t seed, uint32_t ctr_z, uint32_t ctr_w, int64_t n_blocks, uint32_t* out);

static int fails = 0;
#define CHECK(c)                                             \
  do {                                                       \
    if (!(c)) {                                              \
      fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
      ++fails;                                               \
    }                                                        \
  } while (0)

static float* alloc_f(size_t n) {  /* exact-size heap blocks: ASan sees any overrun */
  float* p = (float*)malloc(sizeof(float) * (n ? n : 1));
  for (size_t i = 0; i < n; ++i) p[i] = (float)((i * 2654435761u) % 1000) / 500.0f - 1.0f;
  return p;
}

int main(void) {
  /* P7: Random123 known answers */
  const uint32_t kat[3][10] = {
      {0, 0, 0, 0, 0, 0, 0x6627e8d5u, 0xe169c58du, 0xbc57ac4cu, 0x9b00dbd8u},
      {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x408f276du, 0x41c83b0eu,
       0xa20bc7c6u, 0x6d5451fdu},
      {0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u, 0xa4093822u, 0x299f31d0u, 0xd16cfe09u, 0x94fdccebu,
       0x5001e420u, 0x24126ea1u}};
  for (int t = 0; t < 3; ++t) {
    uint32_t out[4];
    oracle_philox4x32_10(kat[t], kat[t] + 4, out);
    CHECK(memcmp(out, kat[t] + 6, sizeof(out)) == 0);
  }
  /* the simulator on ragged shapes, every potential kind (0 quadratic, 1 GMM, 2 mean field) */
  const int dims[] = {1, 3, 4, 5, 8};
  const int64_t Ns[] = {0, 1, 37};
  for (int di = 0; di < 5; ++di)
    for (int ni = 0; ni < 3; ++ni)
      for (int kind = 0; kind < 3; ++kind)
        for (int explicit_noise = 0; explicit_noise < 2; ++explicit_noise) {
          const int d = dims[di], n = 7, K = 3;
          const int64_t N = Ns[ni], ld = 2 * d + 3; /* strided z0 rows */
          float* z0 = alloc_f((size_t)N * ld);
          float* params = alloc_f(kind == 1 ? (size_t)K * d : (size_t)d * d + d);
          float* noise = explicit_noise ? alloc_f((size_t)(n + 1) * N * d) : NULL;
          float* u = explicit_noise ? alloc_f(kind == 2 ? 1 : (size_t)N) : NULL;
          if (u) for (int64_t i = 0; i < (kind == 2 ? 1 : N); ++i) u[i] = 0.5f * (u[i] + 1.0f);
          float* traj = alloc_f((size_t)n * N * 2 * d);
          float* tau = alloc_f((size_t)n * N);
          float* last = alloc_f((size_t)N * 2 * d);
          const int rc = oracle_sde_simulate(N, 5, d, n, 0.02f, 0.7f, sqrtf(2.0f), 1, 0x1234ull, 3u, kind, K, 1.0f,
                                             params, kind != 1, noise, u, z0, ld, traj, tau, last);
          CHECK(rc == 0);
          for (int64_t i = 0; i < (int64_t)n * N * 2 * d; ++i) CHECK(isfinite(traj[i]));
          double mom[1 + 16 + 16 * 17 / 2];
          oracle_moments(traj, (int64_t)n * N, 2 * d, 0, mom);
          CHECK(mom[0] == (double)(n * N));
          free(z0); free(params); free(noise); free(u); free(traj); free(tau); free(last);
        }
  /* Gaussian sampler with m not a multiple of 4 (partial Philox blocks), Philox fill */
  for (int m = 1; m <= 9; ++m) {
    float* mean = alloc_f((size_t)m);
    float* ch = alloc_f((size_t)m * m);
    float* out = alloc_f((size_t)11 * m);
    oracle_gaussian_sample(11, m, 99, 1, 1000, mean, ch, out);
    for (int i = 0; i < 11 * m; ++i) CHECK(isfinite(out[i]));
    free(mean); free(ch); free(out);
  }
  uint32_t* bits = (uint32_t*)malloc(sizeof(uint32_t) * 4 * 13);
  oracle_philox_fill(7, 1, 2, 13, bits);
  free(bits);
  CHECK(oracle_sde_simulate(4, 0, 0, 3, 0.1f, 1.f, 1.f, 0, 1, 0, 0, 0, 1.f, NULL, 1, NULL, NULL, NULL, 0, NULL,
                            NULL, NULL) == -1); /* d = 0 rejected before any access */
  printf("asan driver: %d failed checks\n", fails);
  return fails;
}
