// optim.hip — fused optimizer step for the trainer (core/trainer.py:85-86 of the reference:
// optax.chain(add_decayed_weights(wd), adam(lr, b1, b2, eps)) then optax.apply_updates).
// One pass over the flat parameter vector instead of ~10 elementwise launches per leaf.
#include <math.h>

#include "common.h"

namespace pdeinv {

// g' = g + wd p;  mu = b1 mu + (1 - b1) g';  nu = b2 nu + (1 - b2) g'^2;
// p -= lr * (mu / c1) / (sqrt(nu / c2) + eps),  c1 = 1 - b1^t, c2 = 1 - b2^t  (optax scale_by_adam)
__global__ void adam_update_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ mu,
                                   float* __restrict__ nu, int64_t n, float lr, float b1, float b2, float eps,
                                   float wd, float inv_c1, float inv_c2) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const float pv = p[i];
    const float gv = fmaf(wd, pv, g[i]);
    const float m = fmaf(b1, mu[i], (1.f - b1) * gv);
    const float v = fmaf(b2, nu[i], (1.f - b2) * gv * gv);
    mu[i] = m;
    nu[i] = v;
    p[i] = pv - lr * (m * inv_c1) / (sqrtf(v * inv_c2) + eps);
  }
}

}  // namespace pdeinv

using namespace pdeinv;

extern "C" int pdeinv_adam_update(float* params, const float* grad, float* mu, float* nu, int64_t n, float lr,
                                  float b1, float b2, float eps, float weight_decay, int32_t count, void* stream) {
  PDEINV_REQUIRE(n >= 0 && count >= 1, PDEINV_ERR_INVALID, "adam_update: n < 0 or count < 1");
  if (n == 0) return PDEINV_OK;
  PDEINV_REQUIRE(params && grad && mu && nu, PDEINV_ERR_INVALID, "adam_update: null pointer");
  const double c1 = 1.0 - pow((double)b1, (double)count), c2 = 1.0 - pow((double)b2, (double)count);
  const int64_t blocks = grid_for(n) < 2048 ? grid_for(n) : 2048;
  hipLaunchKernelGGL(adam_update_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, params, grad,
                     mu, nu, n, lr, b1, b2, eps, weight_decay, (float)(1.0 / c1), (float)(1.0 / c2));
  return check_launch("adam_update_kernel");
}
