// sh_math.h -- real spherical-harmonics basis (degrees 0-4) and the LDS row staging shared by
// sh.hip (gsplat compute_sh_forward / backward) and preprocess.hip (the fused caller glue).
// Restates gsplat 0.1.2.1 sh.cuh.  The arithmetic carries its own
// `fp contract(on)` pragma (a*b+c fused within one expression, never across statements), so
// it rounds the same in the -ffp-contract=off translation
// units (preprocess.hip) as in the default ones (sh.hip).
#pragma once

#include "common.h"

namespace gs {
namespace {

constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f,
                SH_C2_2 = 0.31539156525252005f, SH_C2_3 = -1.0925484305920792f,
                SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f, SH_C3_1 = 2.890611442640554f,
                SH_C3_2 = -0.4570457994644658f, SH_C3_3 = 0.3731763325901154f,
                SH_C3_4 = -0.4570457994644658f, SH_C3_5 = 1.445305721320277f,
                SH_C3_6 = -0.5900435899266435f;
constexpr float SH_C4_0 = 2.5033429417967046f, SH_C4_1 = -1.7701307697799304f,
                SH_C4_2 = 0.9461746957575601f, SH_C4_3 = -0.6690465435572892f,
                SH_C4_4 = 0.10578554691520431f, SH_C4_5 = -0.6690465435572892f,
                SH_C4_6 = 0.47308734787878004f, SH_C4_7 = -1.7701307697799304f,
                SH_C4_8 = 0.6258357354491761f;

__host__ __device__ __forceinline__ int num_bases(int degree) {
  return degree <= 0 ? 1 : degree == 1 ? 4 : degree == 2 ? 9 : degree == 3 ? 16 : 25;
}

// Basis values in sh_coeffs_to_color's consumption order (same expressions as the oracle).
__device__ __forceinline__ int sh_basis(int degree, float dx, float dy, float dz, float *b) {
#pragma clang fp contract(on)
  b[0] = SH_C0;
  if (degree < 1) return 1;
  float norm = sqrtf(dx * dx + dy * dy + dz * dz);
  float x = dx / norm, y = dy / norm, z = dz / norm;
  float xx = x * x, xy = x * y, xz = x * z, yy = y * y, yz = y * z, zz = z * z;
  b[1] = -SH_C1 * y;
  b[2] = SH_C1 * z;
  b[3] = -SH_C1 * x;
  if (degree < 2) return 4;
  b[4] = SH_C2_0 * xy;
  b[5] = SH_C2_1 * yz;
  b[6] = SH_C2_2 * (2.f * zz - xx - yy);
  b[7] = SH_C2_3 * xz;
  b[8] = SH_C2_4 * (xx - yy);
  if (degree < 3) return 9;
  b[9] = SH_C3_0 * y * (3.f * xx - yy);
  b[10] = SH_C3_1 * xy * z;
  b[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
  b[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
  b[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
  b[14] = SH_C3_5 * z * (xx - yy);
  b[15] = SH_C3_6 * x * (xx - 3.f * yy);
  if (degree < 4) return 16;
  b[16] = SH_C4_0 * xy * (xx - yy);
  b[17] = SH_C4_1 * yz * (3.f * xx - yy);
  b[18] = SH_C4_2 * xy * (7.f * zz - 1.f);
  b[19] = SH_C4_3 * yz * (7.f * zz - 3.f);
  b[20] = SH_C4_4 * (zz * (35.f * zz - 30.f) + 3.f);
  b[21] = SH_C4_5 * xz * (7.f * zz - 3.f);
  b[22] = SH_C4_6 * (xx - yy) * (7.f * zz - 1.f);
  b[23] = SH_C4_7 * xz * (xx - 3.f * yy);
  b[24] = SH_C4_8 * (xx * (xx - 3.f * yy) - yy * (3.f * xx - yy));
  return 25;
}

// 256 Gaussians per workgroup (49 KiB of LDS at degree 3); 128 at degree 4.
__host__ __device__ constexpr int sh_threads(int K) { return K > 16 ? 128 : 256; }

// LDS row pitch: each thread reads/writes its own row, so an even pitch (48 floats at
// degree 3) puts a wave's 64 rows on 4 of the 64 banks (16-way conflicts); an odd pitch
// spreads them over all banks.
__host__ __device__ constexpr int sh_row_pitch(int K) { return (K * 3) | 1; }
template <int ROW, int ROWP>
__device__ __forceinline__ int sh_lds_index(int k) {
  const int r = k / ROW;
  return r * ROWP + (k - r * ROW);
}

// Copies cnt rows of ROW floats (src, contiguous) into LDS rows of pitch ROWP with 16-byte
// coalesced loads when src is 16-byte aligned; a full block issues all of a thread's loads
// before its first LDS write.
template <int ROW, int ROWP, int THREADS>
__device__ __forceinline__ void stage_rows(const float *__restrict__ src, int cnt, float *smem) {
  const int total = cnt * ROW;
  if ((((uintptr_t)src) & 15) == 0) {
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    if (cnt == THREADS && (THREADS * ROW) % 4 == 0) {
      constexpr int NV = THREADS * ROW / 4;
      constexpr int PER = (NV + THREADS - 1) / THREADS;
      float4 v[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int k = u * THREADS + threadIdx.x;
        if (NV % THREADS == 0 || k < NV) v[u] = s4[k];
      }
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int k = u * THREADS + threadIdx.x;
        if (NV % THREADS == 0 || k < NV) {
          smem[sh_lds_index<ROW, ROWP>(4 * k)] = v[u].x;
          smem[sh_lds_index<ROW, ROWP>(4 * k + 1)] = v[u].y;
          smem[sh_lds_index<ROW, ROWP>(4 * k + 2)] = v[u].z;
          smem[sh_lds_index<ROW, ROWP>(4 * k + 3)] = v[u].w;
        }
      }
      return;
    }
    const int nv = total >> 2;
    for (int k = threadIdx.x; k < nv; k += THREADS) {
      const float4 v = s4[k];
      const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) smem[sh_lds_index<ROW, ROWP>(4 * k + u)] = e[u];
    }
    for (int k = (nv << 2) + threadIdx.x; k < total; k += THREADS)
      smem[sh_lds_index<ROW, ROWP>(k)] = src[k];
  } else {
    for (int k = threadIdx.x; k < total; k += THREADS) smem[sh_lds_index<ROW, ROWP>(k)] = src[k];
  }
}

// stage_rows split in two so that a kernel can do other work while the slab is in flight:
// issue() starts a full, aligned block's 16-byte loads into registers; land() writes them to
// LDS (or stages a partial / unaligned block with stage_rows).  Sync after land().
template <int ROW, int ROWP, int THREADS>
struct RowStager {
  static constexpr int NV = THREADS * ROW / 4;
  static constexpr int PER = (NV + THREADS - 1) / THREADS;
  float4 v[PER];
  bool fast;
  __device__ __forceinline__ void issue(const float *__restrict__ src, int cnt) {
    fast = cnt == THREADS && (THREADS * ROW) % 4 == 0 && (((uintptr_t)src) & 15) == 0;
    if (!fast) return;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int k = u * THREADS + threadIdx.x;
      if (NV % THREADS == 0 || k < NV) v[u] = s4[k];
    }
  }
  __device__ __forceinline__ void land(const float *__restrict__ src, int cnt, float *smem) {
    if (!fast) {
      stage_rows<ROW, ROWP, THREADS>(src, cnt, smem);
      return;
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int k = u * THREADS + threadIdx.x;
      if (NV % THREADS == 0 || k < NV) {
        smem[sh_lds_index<ROW, ROWP>(4 * k)] = v[u].x;
        smem[sh_lds_index<ROW, ROWP>(4 * k + 1)] = v[u].y;
        smem[sh_lds_index<ROW, ROWP>(4 * k + 2)] = v[u].z;
        smem[sh_lds_index<ROW, ROWP>(4 * k + 3)] = v[u].w;
      }
    }
  }
};

// Writes columns [C0, C0 + WIDTH) of cnt LDS rows (pitch ROWP) to dst (row r's WIDTH values
// at dst[r * WIDTH]), with 16-byte coalesced stores when dst is 16-byte aligned.
template <int WIDTH, int C0, int ROWP, int THREADS>
__device__ __forceinline__ void store_cols(const float *smem, int cnt, float *__restrict__ dst) {
  const int total = cnt * WIDTH;
  auto at = [&](int k) {
    const int r = k / WIDTH;
    return smem[r * ROWP + C0 + (k - r * WIDTH)];
  };
  if ((((uintptr_t)dst) & 15) == 0) {
    const int nv = total >> 2;
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    for (int k = threadIdx.x; k < nv; k += THREADS) {
      float4 v;
      v.x = at(4 * k);
      v.y = at(4 * k + 1);
      v.z = at(4 * k + 2);
      v.w = at(4 * k + 3);
      d4[k] = v;
    }
    for (int k = (nv << 2) + threadIdx.x; k < total; k += THREADS) dst[k] = at(k);
  } else {
    for (int k = threadIdx.x; k < total; k += THREADS) dst[k] = at(k);
  }
}

// Writes the block's cnt staged coefficient rows (LDS, pitch sh_row_pitch) to dst [cnt * K * 3].
template <int K>
__device__ __forceinline__ void store_rows(const float *smem, int cnt, float *dst) {
  store_cols<K * 3, 0, sh_row_pitch(K), sh_threads(K)>(smem, cnt, dst);
}

// One colour channel from the first nb bases b[] of a coefficient row, summed band by band as
// gsplat's sh_coeffs_to_color does; co(k) returns basis k's coefficient of this channel.
template <int K, typename Co>
__device__ __forceinline__ float sh_channel(const float *b, int nb, Co co) {
#pragma clang fp contract(on)
  float acc = b[0] * co(0);
#pragma unroll
  for (int band = 1; band <= 4; ++band) {
    if ((band + 1) * (band + 1) > nb || (band + 1) * (band + 1) > K) break;
    float s = 0.f;
#pragma unroll
    for (int k = band * band; k < (band + 1) * (band + 1); ++k) s += b[k] * co(k);
    acc += s;
  }
  return acc;
}

}  // namespace
}  // namespace gs
