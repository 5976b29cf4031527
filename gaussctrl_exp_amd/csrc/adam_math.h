// adam_math.h -- one torch.optim.Adam element update (foreach, non-capturable semantics),
// shared by adam.hip (the multi-tensor step) and preprocess.hip (the step fused into the
// training render's backward).  Every multiply-add is an explicit fmaf and no other a*b+c
// pattern occurs, so the rounding is the same under any -ffp-contract setting.
#pragma once

#include "common.h"

namespace gs {
namespace {

__device__ __forceinline__ void adam_elem(float &p, float g, float &m, float &v, float w1,
                                          float beta2, float w2, float ss, float bc2s,
                                          float eps) {
  m = fmaf(w1, g - m, m);  // torch lerp, weight < 0.5 branch
  v = fmaf(w2 * g, g, v * beta2);
  const float denom = sqrtf(v) / bc2s + eps;
  p = fmaf(-ss, m / denom, p);
}

}  // namespace
}  // namespace gs
