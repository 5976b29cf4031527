// common.h -- shared device helpers for the gfx950 rasterizer kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gsplat_mi355x.h"

#define GS_BLOCK 16           // tile edge (gsplat config.h BLOCK_X = BLOCK_Y = 16)
#define GS_TILE_PIX 256       // pixels per tile
#define GS_WAVE 64            // CDNA wavefront

namespace gs {

// Error reporting for the C ABI (thread-local message, int status).
void set_error(const char *fmt, ...);
// Records the first failing HIP runtime call of the current C-ABI call; check_launch()
// reports it (or any pending launch error) and resets the record.
void note(hipError_t e, const char *what);
int check_launch(const char *what);

static inline unsigned int cdiv(long long a, long long b) { return (unsigned int)((a + b - 1) / b); }

// Saturating float->int truncation, NaN -> 0: the semantics of v_cvt_i32_f32 (and of
// CUDA's cvt.rzi.s32.f32 that gsplat was compiled to).  Spelled out so the oracle's
// restatement matches it bit for bit.
__device__ __forceinline__ int f2i_sat(float x) {
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Order LDS traffic between the lanes of ONE wave (no workgroup barrier needed when a
// wave owns its LDS region).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Full-wave sum with DPP row ops; result valid in lane 63.
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false));
  return v;
}

// Full-wave sum broadcast as a wave-uniform (SGPR) value.
__device__ __forceinline__ float wave_sum(float v) {
  float r = wave_sum_to_lane63(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, r), 63));
}

__device__ __forceinline__ int wave_max_int(int v) {
  for (int off = 32; off >= 1; off >>= 1) {
    int o = __shfl_xor(v, off, 64);
    v = v > o ? v : o;
  }
  return v;
}

}  // namespace gs
