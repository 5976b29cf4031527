// raster.hip -- per-tile front-to-back alpha blending (forward) and its reverse-order
// backward, for gfx950.
//
// Replaces gsplat 0.1.2.1 _C.rasterize_forward / _C.rasterize_backward (forward.cu /
// backward.cu; semantics SURVEY.md Appendix A9/A10), reached from
// /root/reference/gaussctrl/gc_model.py:208-220 (RGB + alpha) and :225-236 (depth).
//
// MI355X mapping (the path is per-pixel serial compositing: no MFMA):
//  * One wave64 owns one 16x16 tile; each lane owns 4 pixels of a column (rows
//    r, r+4, r+8, r+12).  No workgroup barrier is ever needed: a wave stages its own
//    tile's Gaussians in its own LDS slice, 64 at a time (one Gaussian per lane, loaded
//    coalesced from the sorted id list), then every lane reads each staged Gaussian as an
//    LDS broadcast and applies it to its 4 pixels -- one LDS read per 4 pixel-evaluations.
//  * Early termination is per wave (__all over 256 pixels) and is tested after every
//    Gaussian, not per 256-Gaussian batch as in gsplat.
//  * Backward: the per-pixel contributions to one Gaussian are summed in registers over the
//    lane's 4 pixels, then across the wave with DPP row operations (6 VALU ops per value,
//    no LDS), and one lane issues the 9 float atomics of the (tile, Gaussian) pair.  Waves
//    with no valid pixel for a Gaussian skip the reduction entirely.
//  * 4 tiles (4 independent waves) per 256-thread workgroup.
//  * C != 3 (gsplat nd_rasterize): one pixel per lane, 4 waves per tile, register
//    accumulators sized by a compile-time channel bound.
#include "common.h"

namespace gs {
namespace {

constexpr int WPB = 4;             // tiles (waves) per workgroup
constexpr int PXL = 4;             // pixels per lane
constexpr float ALPHA_MIN = 1.f / 255.f;

struct __attribute__((aligned(16))) GFwd {
  float x, y, a, b;
  float c, o, r, g;
  float bl, p0, p1, p2;
};

struct __attribute__((aligned(16))) GBwd {
  float x, y, a, b;
  float c, o, r, g;
  float bl;
  int id;
  float p0, p1;
};

__global__ __launch_bounds__(64 * WPB) void raster_fwd3_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, float *__restrict__ out_img,
    float *__restrict__ final_Ts, int *__restrict__ final_idx) {
  __shared__ GFwd lds[WPB][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = blockIdx.x * WPB + wave;
  if (tile >= tbx * tby) return;  // wave-uniform
  const int tx = tile % tbx, ty = tile / tbx;
  const int j = tx * GS_BLOCK + (lane & 15);
  const int i0 = ty * GS_BLOCK + (lane >> 4);
  const float px = (float)j;
  float py[PXL], T[PXL], cr[PXL], cg[PXL], cb[PXL];
  int cur[PXL];
  bool done[PXL];
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + 4 * k;
    py[k] = (float)i;
    T[k] = 1.f;
    cr[k] = cg[k] = cb[k] = 0.f;
    cur[k] = 0;
    done[k] = !(i < H && j < W);
  }
  const int2 range = bins[tile];
  GFwd *slot = lds[wave];
  for (int b = range.x; b < range.y; b += 64) {
    if (__all(done[0] && done[1] && done[2] && done[3])) break;
    const int idx = b + lane;
    if (idx < range.y) {
      const int g = gids[idx];
      const float2 xy = xys[g];
      GFwd s;
      s.x = xy.x;
      s.y = xy.y;
      s.a = conics[3 * g];
      s.b = conics[3 * g + 1];
      s.c = conics[3 * g + 2];
      s.o = opacity[g];
      s.r = colors[3 * g];
      s.g = colors[3 * g + 1];
      s.bl = colors[3 * g + 2];
      slot[lane] = s;
    }
    wave_lds_sync();
    const int n = min(64, range.y - b);
    for (int t = 0; t < n; ++t) {
      const GFwd G = slot[t];
      bool all_done = true;
#pragma unroll
      for (int k = 0; k < PXL; ++k) {
        if (!done[k]) {
          const float dx = G.x - px, dy = G.y - py[k];
          const float sigma = 0.5f * (G.a * dx * dx + G.c * dy * dy) + G.b * dx * dy;
          const float alpha = fminf(0.999f, G.o * __expf(-sigma));
          if (sigma >= 0.f && alpha >= ALPHA_MIN) {
            const float nT = T[k] * (1.f - alpha);
            if (nT <= 1e-4f) {
              done[k] = true;
            } else {
              const float vis = alpha * T[k];
              cr[k] += G.r * vis;
              cg[k] += G.g * vis;
              cb[k] += G.bl * vis;
              T[k] = nT;
              cur[k] = b + t;
            }
          }
        }
        all_done = all_done && done[k];
      }
      if (__all(all_done)) break;
    }
    wave_lds_sync();
  }
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + 4 * k;
    if (i < H && j < W) {
      const int pix = i * W + j;
      final_Ts[pix] = T[k];
      final_idx[pix] = cur[k];
      out_img[3 * pix] = cr[k] + T[k] * bg0;
      out_img[3 * pix + 1] = cg[k] + T[k] * bg1;
      out_img[3 * pix + 2] = cb[k] + T[k] * bg2;
    }
  }
}

__global__ __launch_bounds__(64 * WPB) void raster_bwd3_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, const float *__restrict__ final_Ts,
    const int *__restrict__ final_idx, const float *__restrict__ v_out,
    const float *__restrict__ v_out_alpha, float alpha_max, float *__restrict__ v_xy,
    float *__restrict__ v_conic, float *__restrict__ v_rgb, float *__restrict__ v_opacity) {
  __shared__ GBwd lds[WPB][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = blockIdx.x * WPB + wave;
  if (tile >= tbx * tby) return;
  const int tx = tile % tbx, ty = tile / tbx;
  const int j = tx * GS_BLOCK + (lane & 15);
  const int i0 = ty * GS_BLOCK + (lane >> 4);
  const float px = (float)j;
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
  float py[PXL], T[PXL], Tf[PXL], vr[PXL], vg[PXL], vb[PXL], va[PXL], bgdot[PXL];
  float br[PXL], bgr[PXL], bb[PXL];
  int binf[PXL];
  int maxbin = -1;
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + 4 * k;
    py[k] = (float)i;
    br[k] = bgr[k] = bb[k] = 0.f;
    if (i < H && j < W) {
      const int pix = i * W + j;
      Tf[k] = final_Ts[pix];
      binf[k] = final_idx[pix];
      vr[k] = v_out[3 * pix];
      vg[k] = v_out[3 * pix + 1];
      vb[k] = v_out[3 * pix + 2];
      va[k] = v_out_alpha[pix];
    } else {
      Tf[k] = 0.f;
      binf[k] = -1;
      vr[k] = vg[k] = vb[k] = va[k] = 0.f;
    }
    T[k] = Tf[k];
    bgdot[k] = bg0 * vr[k] + bg1 * vg[k] + bg2 * vb[k];
    maxbin = max(maxbin, binf[k]);
  }
  maxbin = wave_max_int(maxbin);
  const int2 range = bins[tile];
  const int last = min(maxbin, range.y - 1);
  GBwd *slot = lds[wave];
  for (int b = last; b >= range.x; b -= 64) {
    const int idx = b - lane;
    if (idx >= range.x) {
      const int g = gids[idx];
      const float2 xy = xys[g];
      GBwd s;
      s.x = xy.x;
      s.y = xy.y;
      s.a = conics[3 * g];
      s.b = conics[3 * g + 1];
      s.c = conics[3 * g + 2];
      s.o = opacity[g];
      s.r = colors[3 * g];
      s.g = colors[3 * g + 1];
      s.bl = colors[3 * g + 2];
      s.id = g;
      slot[lane] = s;
    }
    wave_lds_sync();
    const int n = min(64, b - range.x + 1);
    for (int t = 0; t < n; ++t) {
      const int k_idx = b - t;
      const GBwd G = slot[t];
      float s_x = 0.f, s_y = 0.f, s_a = 0.f, s_b = 0.f, s_c = 0.f, s_r = 0.f, s_g = 0.f,
            s_bl = 0.f, s_o = 0.f;
      bool anyv = false;
#pragma unroll
      for (int k = 0; k < PXL; ++k) {
        const float dx = G.x - px, dy = G.y - py[k];
        const float sigma = 0.5f * (G.a * dx * dx + G.c * dy * dy) + G.b * dx * dy;
        const float vis = __expf(-sigma);
        const float alpha = fminf(alpha_max, G.o * vis);
        const bool valid = k_idx <= binf[k] && sigma >= 0.f && alpha >= ALPHA_MIN;
        if (valid) {
          anyv = true;
          const float ra = __builtin_amdgcn_rcpf(1.f - alpha);
          T[k] *= ra;
          const float fac = alpha * T[k];
          s_r += fac * vr[k];
          s_g += fac * vg[k];
          s_bl += fac * vb[k];
          float v_alpha = (G.r * T[k] - br[k] * ra) * vr[k] + (G.g * T[k] - bgr[k] * ra) * vg[k] +
                          (G.bl * T[k] - bb[k] * ra) * vb[k];
          v_alpha += Tf[k] * ra * va[k];
          v_alpha += -Tf[k] * ra * bgdot[k];
          br[k] += G.r * fac;
          bgr[k] += G.g * fac;
          bb[k] += G.bl * fac;
          const float v_sigma = -G.o * vis * v_alpha;
          s_a += 0.5f * v_sigma * dx * dx;
          s_b += 0.5f * v_sigma * dx * dy;
          s_c += 0.5f * v_sigma * dy * dy;
          s_x += v_sigma * (G.a * dx + G.b * dy);
          s_y += v_sigma * (G.b * dx + G.c * dy);
          s_o += vis * v_alpha;
        }
      }
      if (__any(anyv)) {
        s_x = wave_sum(s_x);
        s_y = wave_sum(s_y);
        s_a = wave_sum(s_a);
        s_b = wave_sum(s_b);
        s_c = wave_sum(s_c);
        s_r = wave_sum(s_r);
        s_g = wave_sum(s_g);
        s_bl = wave_sum(s_bl);
        s_o = wave_sum(s_o);
        if (lane == 0) {
          const int g = G.id;
          atomicAdd(v_xy + 2 * g, s_x);
          atomicAdd(v_xy + 2 * g + 1, s_y);
          atomicAdd(v_conic + 3 * g, s_a);
          atomicAdd(v_conic + 3 * g + 1, s_b);
          atomicAdd(v_conic + 3 * g + 2, s_c);
          atomicAdd(v_rgb + 3 * g, s_r);
          atomicAdd(v_rgb + 3 * g + 1, s_g);
          atomicAdd(v_rgb + 3 * g + 2, s_bl);
          atomicAdd(v_opacity + g, s_o);
        }
      }
    }
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------- N-channel variants
// One pixel per thread, 256 threads per tile, Gaussians staged 256 at a time in LDS
// (colors read through L2: channel count is a runtime value up to CMAX).

struct __attribute__((aligned(16))) GN {
  float x, y, a, b;
  float c, o;
  int id;
  float p;
};

template <int CMAX>
__global__ __launch_bounds__(256) void raster_fwdn_kernel(
    int tbx, int tby, int H, int W, int C, const int *__restrict__ gids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys,
    const float *__restrict__ conics, const float *__restrict__ colors,
    const float *__restrict__ opacity, const float *__restrict__ background,
    float *__restrict__ out_img, float *__restrict__ final_Ts, int *__restrict__ final_idx) {
  __shared__ GN lds[256];
  const int tile = blockIdx.x;
  const int tx = tile % tbx, ty = tile / tbx;
  const int j = tx * GS_BLOCK + (threadIdx.x & 15);
  const int i = ty * GS_BLOCK + (threadIdx.x >> 4);
  const bool inside = i < H && j < W;
  const float px = (float)j, py = (float)i;
  float acc[CMAX];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) acc[c] = 0.f;
  float T = 1.f;
  int cur = 0;
  bool done = !inside;
  const int2 range = bins[tile];
  for (int b = range.x; b < range.y; b += 256) {
    if (__syncthreads_count(done) >= 256) break;
    const int idx = b + threadIdx.x;
    if (idx < range.y) {
      const int g = gids[idx];
      const float2 xy = xys[g];
      GN s;
      s.x = xy.x;
      s.y = xy.y;
      s.a = conics[3 * g];
      s.b = conics[3 * g + 1];
      s.c = conics[3 * g + 2];
      s.o = opacity[g];
      s.id = g;
      lds[threadIdx.x] = s;
    }
    __syncthreads();
    const int n = min(256, range.y - b);
    for (int t = 0; t < n && !done; ++t) {
      const GN G = lds[t];
      const float dx = G.x - px, dy = G.y - py;
      const float sigma = 0.5f * (G.a * dx * dx + G.c * dy * dy) + G.b * dx * dy;
      const float alpha = fminf(0.999f, G.o * __expf(-sigma));
      if (sigma < 0.f || alpha < ALPHA_MIN) continue;
      const float nT = T * (1.f - alpha);
      if (nT <= 1e-4f) {
        done = true;
        break;
      }
      const float vis = alpha * T;
      const float *col = colors + (size_t)C * G.id;
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) acc[c] += col[c] * vis;
      T = nT;
      cur = b + t;
    }
  }
  if (inside) {
    const int pix = i * W + j;
    final_Ts[pix] = T;
    final_idx[pix] = cur;
#pragma unroll
    for (int c = 0; c < CMAX; ++c)
      if (c < C) out_img[(size_t)C * pix + c] = acc[c] + T * background[c];
  }
}

template <int CMAX>
__global__ __launch_bounds__(256) void raster_bwdn_kernel(
    int tbx, int tby, int H, int W, int C, const int *__restrict__ gids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys,
    const float *__restrict__ conics, const float *__restrict__ colors,
    const float *__restrict__ opacity, const float *__restrict__ background,
    const float *__restrict__ final_Ts, const int *__restrict__ final_idx,
    const float *__restrict__ v_out, const float *__restrict__ v_out_alpha, float alpha_max,
    float *__restrict__ v_xy, float *__restrict__ v_conic, float *__restrict__ v_colors,
    float *__restrict__ v_opacity) {
  __shared__ GN lds[256];
  const int tile = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int tx = tile % tbx, ty = tile / tbx;
  const int j = tx * GS_BLOCK + (threadIdx.x & 15);
  const int i = ty * GS_BLOCK + (threadIdx.x >> 4);
  const bool inside = i < H && j < W;
  const float px = (float)j, py = (float)i;
  const int pix = inside ? i * W + j : 0;
  const float Tf = inside ? final_Ts[pix] : 0.f;
  float T = Tf;
  const int binf = inside ? final_idx[pix] : -1;
  const float va = inside ? v_out_alpha[pix] : 0.f;
  float vo[CMAX], buf[CMAX];
  float bgdot = 0.f;
#pragma unroll
  for (int c = 0; c < CMAX; ++c) {
    vo[c] = (inside && c < C) ? v_out[(size_t)C * pix + c] : 0.f;
    buf[c] = 0.f;
    if (c < C) bgdot += background[c] * vo[c];
  }
  __shared__ int smax;
  if (threadIdx.x == 0) smax = -1;
  __syncthreads();
  atomicMax(&smax, binf);
  __syncthreads();
  const int2 range = bins[tile];
  const int last = min(smax, range.y - 1);
  for (int b = last; b >= range.x; b -= 256) {
    __syncthreads();
    const int idx = b - (int)threadIdx.x;
    if (idx >= range.x) {
      const int g = gids[idx];
      const float2 xy = xys[g];
      GN s;
      s.x = xy.x;
      s.y = xy.y;
      s.a = conics[3 * g];
      s.b = conics[3 * g + 1];
      s.c = conics[3 * g + 2];
      s.o = opacity[g];
      s.id = g;
      lds[threadIdx.x] = s;
    }
    __syncthreads();
    const int n = min(256, b - range.x + 1);
    for (int t = 0; t < n; ++t) {
      const int k_idx = b - t;
      const GN G = lds[t];
      const float dx = G.x - px, dy = G.y - py;
      const float sigma = 0.5f * (G.a * dx * dx + G.c * dy * dy) + G.b * dx * dy;
      const float vis = __expf(-sigma);
      const float alpha = fminf(alpha_max, G.o * vis);
      const bool valid = k_idx <= binf && sigma >= 0.f && alpha >= ALPHA_MIN;
      if (!__any(valid)) continue;
      float s_col[CMAX];
      float s_x = 0.f, s_y = 0.f, s_a = 0.f, s_b = 0.f, s_c = 0.f, s_o = 0.f;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) s_col[c] = 0.f;
      const float *col = colors + (size_t)C * G.id;
      if (valid) {
        const float ra = __builtin_amdgcn_rcpf(1.f - alpha);
        T *= ra;
        const float fac = alpha * T;
        float v_alpha = 0.f;
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) {
            s_col[c] = fac * vo[c];
            v_alpha += (col[c] * T - buf[c] * ra) * vo[c];
            buf[c] += col[c] * fac;
          }
        v_alpha += Tf * ra * va;
        v_alpha += -Tf * ra * bgdot;
        const float v_sigma = -G.o * vis * v_alpha;
        s_a = 0.5f * v_sigma * dx * dx;
        s_b = 0.5f * v_sigma * dx * dy;
        s_c = 0.5f * v_sigma * dy * dy;
        s_x = v_sigma * (G.a * dx + G.b * dy);
        s_y = v_sigma * (G.b * dx + G.c * dy);
        s_o = vis * v_alpha;
      }
      s_x = wave_sum(s_x);
      s_y = wave_sum(s_y);
      s_a = wave_sum(s_a);
      s_b = wave_sum(s_b);
      s_c = wave_sum(s_c);
      s_o = wave_sum(s_o);
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) s_col[c] = wave_sum(s_col[c]);
      if (lane == 0) {
        const int g = G.id;
        atomicAdd(v_xy + 2 * g, s_x);
        atomicAdd(v_xy + 2 * g + 1, s_y);
        atomicAdd(v_conic + 3 * g, s_a);
        atomicAdd(v_conic + 3 * g + 1, s_b);
        atomicAdd(v_conic + 3 * g + 2, s_c);
        atomicAdd(v_opacity + g, s_o);
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) atomicAdd(v_colors + (size_t)C * g + c, s_col[c]);
      }
    }
  }
}

}  // namespace
}  // namespace gs

using namespace gs;

#define ND_DISPATCH(KERNEL, ...)                                                          \
  do {                                                                                    \
    if (channels <= 4)                                                                    \
      hipLaunchKernelGGL(KERNEL<4>, dim3(T), dim3(256), 0, st, __VA_ARGS__);              \
    else if (channels <= 8)                                                               \
      hipLaunchKernelGGL(KERNEL<8>, dim3(T), dim3(256), 0, st, __VA_ARGS__);              \
    else if (channels <= 16)                                                              \
      hipLaunchKernelGGL(KERNEL<16>, dim3(T), dim3(256), 0, st, __VA_ARGS__);             \
    else if (channels <= 32)                                                              \
      hipLaunchKernelGGL(KERNEL<32>, dim3(T), dim3(256), 0, st, __VA_ARGS__);             \
    else                                                                                  \
      hipLaunchKernelGGL(KERNEL<64>, dim3(T), dim3(256), 0, st, __VA_ARGS__);             \
  } while (0)

extern "C" int gsplat_rasterize_forward(int tile_bounds_x, int tile_bounds_y, int img_height,
                                        int img_width, int channels,
                                        const int32_t *gaussian_ids_sorted,
                                        const int32_t *tile_bins, const float *xys,
                                        const float *conics, const float *colors,
                                        const float *opacity, const float *background,
                                        float *out_img, float *final_Ts, int32_t *final_idx,
                                        void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0 || img_height <= 0 || img_width <= 0 ||
      channels < 1 || channels > 64 ||
      (long long)tile_bounds_x * GS_BLOCK < img_width ||
      (long long)tile_bounds_y * GS_BLOCK < img_height) {
    set_error("rasterize_forward: bad sizes (tiles=%dx%d H=%d W=%d C=%d)", tile_bounds_x,
              tile_bounds_y, img_height, img_width, channels);
    return 1;
  }
  const int T = tile_bounds_x * tile_bounds_y;
  if (channels == 3) {
    hipLaunchKernelGGL(raster_fwd3_kernel, dim3(cdiv(T, WPB)), dim3(64 * WPB), 0, st,
                       tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,
                       (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,
                       background, out_img, final_Ts, final_idx);
  } else {
    ND_DISPATCH(raster_fwdn_kernel, tile_bounds_x, tile_bounds_y, img_height, img_width,
                channels, gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys,
                conics, colors, opacity, background, out_img, final_Ts, final_idx);
  }
  return check_launch("rasterize_forward");
}

extern "C" int gsplat_rasterize_backward(int tile_bounds_x, int tile_bounds_y, int img_height,
                                         int img_width, int channels, int num_points,
                                         const int32_t *gaussian_ids_sorted,
                                         const int32_t *tile_bins, const float *xys,
                                         const float *conics, const float *colors,
                                         const float *opacity, const float *background,
                                         const float *final_Ts, const int32_t *final_idx,
                                         const float *v_output, const float *v_output_alpha,
                                         float alpha_max, float *v_xy, float *v_conic,
                                         float *v_colors, float *v_opacity, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0 || img_height <= 0 || img_width <= 0 ||
      channels < 1 || channels > 64 || num_points < 0 ||
      (long long)tile_bounds_x * GS_BLOCK < img_width ||
      (long long)tile_bounds_y * GS_BLOCK < img_height) {
    set_error("rasterize_backward: bad sizes (tiles=%dx%d H=%d W=%d C=%d N=%d)", tile_bounds_x,
              tile_bounds_y, img_height, img_width, channels, num_points);
    return 1;
  }
  if (num_points > 0) {
    note(hipMemsetAsync(v_xy, 0, (size_t)num_points * 2 * sizeof(float), st), "hipMemsetAsync");
    note(hipMemsetAsync(v_conic, 0, (size_t)num_points * 3 * sizeof(float), st), "hipMemsetAsync");
    note(hipMemsetAsync(v_colors, 0, (size_t)num_points * channels * sizeof(float), st), "hipMemsetAsync");
    note(hipMemsetAsync(v_opacity, 0, (size_t)num_points * sizeof(float), st), "hipMemsetAsync");
  }
  const int T = tile_bounds_x * tile_bounds_y;
  if (channels == 3) {
    hipLaunchKernelGGL(raster_bwd3_kernel, dim3(cdiv(T, WPB)), dim3(64 * WPB), 0, st,
                       tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,
                       (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,
                       background, final_Ts, final_idx, v_output, v_output_alpha, alpha_max,
                       v_xy, v_conic, v_colors, v_opacity);
  } else {
    ND_DISPATCH(raster_bwdn_kernel, tile_bounds_x, tile_bounds_y, img_height, img_width,
                channels, gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys,
                conics, colors, opacity, background, final_Ts, final_idx, v_output,
                v_output_alpha, alpha_max, v_xy, v_conic, v_colors, v_opacity);
  }
  return check_launch("rasterize_backward");
}
