// adam.hip -- fused multi-tensor Adam step for the Gaussian parameter groups on gfx950.
//
// Replaces the optimizer step of the reference's training loop (gc_trainer.py:281,298 ->
// torch.optim.Adam over the six splatfacto groups configured at gc_config.py:58-87: means,
// scales, quats, opacities, features_dc, features_rest; eps 1e-15; per-group learning rate,
// means decaying exponentially).  torch's foreach Adam streams the 59 floats per Gaussian
// through ~6 separate passes (lerp, mul, addcmul, sqrt, div, add, addcdiv); here ONE launch
// covers every group: each thread reads p, g, m, v (16 B) and writes p, m, v (12 B) per
// element, with 16-byte vector accesses -- the HBM floor of the update.
//
// Arithmetic follows torch's foreach implementation operation by operation:
//   m = lerp(m, g, 1 - beta1)                (weight < 0.5: m + w * (g - m))
//   v = v * beta2 + (1 - beta2) * g * g
//   p = p - step_size * m / (sqrt(v) / bias_correction2_sqrt + eps)
// with step_size = lr / (1 - beta1^t) and bias_correction2_sqrt = sqrt(1 - beta2^t) computed
// on the host in double (as torch does for non-capturable Adam).
#include "adam_math.h"

namespace gs {
namespace {

constexpr int MAX_SEGS = 8;
constexpr int ADAM_TPB = 256;
constexpr int ADAM_VEC = 4;  // elements per thread per iteration (one 16-byte vector)
typedef float f4 __attribute__((ext_vector_type(4)));

struct AdamTable {
  float *p[MAX_SEGS];
  const float *g[MAX_SEGS];
  float *m[MAX_SEGS];
  float *v[MAX_SEGS];
  long long n[MAX_SEGS];
  long long block0[MAX_SEGS + 1];  // first block of each segment (prefix over segments)
  float step_size[MAX_SEGS];
  float bc2_sqrt[MAX_SEGS];
  int nseg;
};


__global__ __launch_bounds__(ADAM_TPB) void adam_kernel(AdamTable t, float beta1, float beta2,
                                                        float eps) {
  int s = 0;
  while (s + 1 < t.nseg && (long long)blockIdx.x >= t.block0[s + 1]) ++s;
  const long long base = ((long long)blockIdx.x - t.block0[s]) * ADAM_TPB * ADAM_VEC;
  const long long i = base + (long long)threadIdx.x * ADAM_VEC;
  const long long n = t.n[s];
  if (i >= n) return;
  const float w1 = 1.f - beta1, w2 = 1.f - beta2;
  const float ss = t.step_size[s], bc2s = t.bc2_sqrt[s];
  float *p = t.p[s];
  const float *g = t.g[s];
  float *m = t.m[s];
  float *v = t.v[s];
  const bool vec = i + ADAM_VEC <= n && ((((uintptr_t)(p + i)) | ((uintptr_t)(g + i)) |
                                          ((uintptr_t)(m + i)) | ((uintptr_t)(v + i))) &
                                         15) == 0;
  if (vec) {
    f4 P = *reinterpret_cast<f4 *>(p + i);
    const f4 G = *reinterpret_cast<const f4 *>(g + i);
    f4 M = *reinterpret_cast<f4 *>(m + i);
    f4 V = *reinterpret_cast<f4 *>(v + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float pk = P[k], mk = M[k], vk = V[k];
      adam_elem(pk, G[k], mk, vk, w1, beta2, w2, ss, bc2s, eps);
      P[k] = pk;
      M[k] = mk;
      V[k] = vk;
    }
    *reinterpret_cast<f4 *>(p + i) = P;
    *reinterpret_cast<f4 *>(m + i) = M;
    *reinterpret_cast<f4 *>(v + i) = V;
  } else {
    for (long long k = i; k < n && k < i + ADAM_VEC; ++k) {
      float pk = p[k], mk = m[k], vk = v[k];
      adam_elem(pk, g[k], mk, vk, w1, beta2, w2, ss, bc2s, eps);
      p[k] = pk;
      m[k] = mk;
      v[k] = vk;
    }
  }
}

}  // namespace
}  // namespace gs

using namespace gs;

extern "C" int gsplat_adam_step(int num_tensors, float *const *params, const float *const *grads,
                                float *const *exp_avgs, float *const *exp_avg_sqs,
                                const int64_t *numels, const float *lrs, int step, float beta1,
                                float beta2, float eps, void *stream) {
  if (num_tensors < 0 || num_tensors > MAX_SEGS || step < 1 || !(beta1 > 0.5f && beta1 < 1.f) ||
      !(beta2 >= 0.f && beta2 < 1.f)) {
    // beta1 > 0.5 keeps torch's lerp weight 1 - beta1 below 0.5, i.e. in its
    // "self + w (end - self)" branch; every Adam configuration here uses beta1 = 0.9.
    set_error("adam_step: bad args (tensors=%d step=%d beta1=%g beta2=%g)", num_tensors, step,
              (double)beta1, (double)beta2);
    return 1;
  }
  AdamTable t = {};
  t.nseg = num_tensors;
  long long blocks = 0;
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  for (int s = 0; s < num_tensors; ++s) {
    if (numels[s] < 0) {
      set_error("adam_step: negative numel");
      return 1;
    }
    t.p[s] = params[s];
    t.g[s] = grads[s];
    t.m[s] = exp_avgs[s];
    t.v[s] = exp_avg_sqs[s];
    t.n[s] = numels[s];
    t.block0[s] = blocks;
    blocks += (numels[s] + ADAM_TPB * ADAM_VEC - 1) / (ADAM_TPB * ADAM_VEC);
    t.step_size[s] = (float)(lrs[s] / bc1);
    t.bc2_sqrt[s] = (float)sqrt(bc2);
  }
  t.block0[num_tensors] = blocks;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(ADAM_TPB), 0, (hipStream_t)stream,
                     t, beta1, beta2, eps);
  return check_launch("adam_step");
}
