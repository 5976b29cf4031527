// loss.hip -- fused splatfacto photometric loss for gfx950:
//     loss = (1 - lambda) * mean|gt - pred| + lambda * (1 - SSIM(gt, pred))
// with pytorch_msssim's SSIM (11x11 Gaussian window, sigma 1.5, 'valid' filtering, data range
// 1, K = (0.01, 0.03), mean over channels and positions), as nerfstudio 1.0 splatfacto's
// get_loss_dict computes it on every training step (the reference reaches it
// through gc_pipeline.py:477-478).  The torch restatement it must match is
// gaussctrl_exp_amd/train.py ssim() / splatfacto_loss().
//
// MI355X design (stencil work, HBM/LDS-bound; no MFMA):
//  * Forward: one 256-thread workgroup per 16x16 block of SSIM outputs (block origin (bx, by)).
//    Per channel it stages the 26x26 input patches of gt and pred in LDS, runs the separable
//    filter horizontally (5 moments: x, y, x^2, y^2, xy) then vertically, and evaluates the
//    SSIM map m and its partial derivatives with respect to the filtered pred statistics
//    (mu_y, E[y^2], E[xy]); those three maps are written for the backward.  The same
//    workgroup sums |gt - pred| over its 16x16 input block (the blocks tile the image) and
//    the SSIM values of its outputs; per-block partial sums are reduced by one tiny kernel
//    into the loss scalar (deterministic, no host sync).
//  * Backward: one workgroup per 16x16 block of input pixels correlates the three derivative
//    maps (26x26 halo patch in LDS, separable) back to input resolution and adds the L1 sign
//    term; the upstream gradient is read from device memory (no host sync).
#include "common.h"

namespace gs {
namespace {

constexpr int WIN = 11;
constexpr int TB = 16;              // block edge
constexpr int PATCH = TB + WIN - 1;  // 26
constexpr float K1 = 0.01f, K2 = 0.03f;

struct Win {
  float w[WIN];
};

__device__ __forceinline__ float block_sum(float v, float *red) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

// partials[block] = {sum |gt - pred| over the block's input pixels (all channels),
//                    sum of SSIM map values over the block's valid outputs (all channels)}
__global__ __launch_bounds__(256) void l1_ssim_fwd_kernel(int H, int W, int C,
                                                          const float *__restrict__ pred,
                                                          const float *__restrict__ gt, Win win,
                                                          float *__restrict__ partials,
                                                          float *__restrict__ dmaps) {
  __shared__ float sx[PATCH][PATCH + 1], sy[PATCH][PATCH + 1];
  __shared__ float hm[5][PATCH][TB + 1];
  __shared__ float red[4];
  const int Ho = H - WIN + 1, Wo = W - WIN + 1;
  const int nbx = (W + TB - 1) / TB;
  const int bx = (blockIdx.x % nbx) * TB, by = (blockIdx.x / nbx) * TB;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const float c1 = K1 * K1, c2 = K2 * K2;
  float l1 = 0.f, ssum = 0.f;
  const size_t plane = (size_t)Ho * Wo;
  for (int c = 0; c < C; ++c) {
    for (int k = threadIdx.x; k < PATCH * PATCH; k += 256) {
      const int r = k / PATCH, q = k % PATCH;
      const int i = by + r, j = bx + q;
      float xv = 0.f, yv = 0.f;
      if (i < H && j < W) {
        xv = gt[((size_t)i * W + j) * C + c];
        yv = pred[((size_t)i * W + j) * C + c];
      }
      sx[r][q] = xv;
      sy[r][q] = yv;
    }
    __syncthreads();
    {  // L1 over this block's own input pixels
      const int i = by + ty, j = bx + tx;
      if (i < H && j < W) l1 += fabsf(sx[ty][tx] - sy[ty][tx]);
    }
    // horizontal pass: rows 0..25, output columns 0..15
    for (int k = threadIdx.x; k < PATCH * TB; k += 256) {
      const int r = k / TB, q = k % TB;
      float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f, m4 = 0.f;
#pragma unroll
      for (int t = 0; t < WIN; ++t) {
        const float w = win.w[t], xv = sx[r][q + t], yv = sy[r][q + t];
        m0 += w * xv;
        m1 += w * yv;
        m2 += w * xv * xv;
        m3 += w * yv * yv;
        m4 += w * xv * yv;
      }
      hm[0][r][q] = m0;
      hm[1][r][q] = m1;
      hm[2][r][q] = m2;
      hm[3][r][q] = m3;
      hm[4][r][q] = m4;
    }
    __syncthreads();
    {
      const int oi = by + ty, oj = bx + tx;
      if (oi < Ho && oj < Wo) {
        float mu1 = 0.f, mu2 = 0.f, exx = 0.f, eyy = 0.f, exy = 0.f;
#pragma unroll
        for (int t = 0; t < WIN; ++t) {
          const float w = win.w[t];
          mu1 += w * hm[0][ty + t][tx];
          mu2 += w * hm[1][ty + t][tx];
          exx += w * hm[2][ty + t][tx];
          eyy += w * hm[3][ty + t][tx];
          exy += w * hm[4][ty + t][tx];
        }
        const float s11 = exx - mu1 * mu1, s22 = eyy - mu2 * mu2, s12 = exy - mu1 * mu2;
        const float A = 2.f * mu1 * mu2 + c1, B = mu1 * mu1 + mu2 * mu2 + c1;
        const float Cn = 2.f * s12 + c2, D = s11 + s22 + c2;
        const float l = A / B, cs = Cn / D;
        ssum += l * cs;
        // d m / d mu2, d m / d E[y^2], d m / d E[xy]  (mu1, E[x^2] belong to gt: constant)
        const float dl = (2.f * mu1 * B - 2.f * mu2 * A) / (B * B);
        const float dcs = (-2.f * mu1 * D + 2.f * mu2 * Cn) / (D * D);
        const size_t o = (size_t)oi * Wo + oj;
        dmaps[(size_t)(0 * C + c) * plane + o] = dl * cs + l * dcs;
        dmaps[(size_t)(1 * C + c) * plane + o] = -l * Cn / (D * D);
        dmaps[(size_t)(2 * C + c) * plane + o] = 2.f * l / D;
      }
    }
    __syncthreads();
  }
  l1 = block_sum(l1, red);
  ssum = block_sum(ssum, red);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = l1;
    partials[2 * blockIdx.x + 1] = ssum;
  }
}

// loss = (1 - lambda) * L1 / (C H W) + lambda * (1 - SSIM_sum / (C Ho Wo)); one workgroup,
// double accumulation in a fixed order (deterministic).
__global__ __launch_bounds__(256) void l1_ssim_finalize_kernel(int nblocks, const float *partials,
                                                               double inv_l1, double inv_ssim,
                                                               float lambda, float *loss) {
  __shared__ double ra[256], rb[256];
  double a = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < nblocks; k += 256) {
    a += partials[2 * k];
    b += partials[2 * k + 1];
  }
  ra[threadIdx.x] = a;
  rb[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      ra[threadIdx.x] += ra[threadIdx.x + s];
      rb[threadIdx.x] += rb[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    loss[0] = (float)((1.0 - lambda) * ra[0] * inv_l1 + lambda * (1.0 - rb[0] * inv_ssim));
}

__global__ __launch_bounds__(256) void l1_ssim_bwd_kernel(
    int H, int W, int C, const float *__restrict__ pred, const float *__restrict__ gt, Win win,
    const float *__restrict__ dmaps, const float *__restrict__ grad_out, float ssim_scale,
    float l1_scale, float *__restrict__ v_pred) {
  __shared__ float sd[3][PATCH][PATCH + 1];
  __shared__ float hd[3][PATCH][TB + 1];
  const int Ho = H - WIN + 1, Wo = W - WIN + 1;
  const int nbx = (W + TB - 1) / TB;
  const int bx = (blockIdx.x % nbx) * TB, by = (blockIdx.x / nbx) * TB;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const float g = grad_out[0];
  const float gs = g * ssim_scale, gl = g * l1_scale;
  const size_t plane = (size_t)Ho * Wo;
  // input q receives from outputs p = q - t, t in [0, 10]: patch rows/cols start at b - 10
  const int oy0 = by - (WIN - 1), ox0 = bx - (WIN - 1);
  for (int c = 0; c < C; ++c) {
    for (int k = threadIdx.x; k < PATCH * PATCH; k += 256) {
      const int r = k / PATCH, q = k % PATCH;
      const int oi = oy0 + r, oj = ox0 + q;
      const bool ok = oi >= 0 && oj >= 0 && oi < Ho && oj < Wo;
      const size_t o = ok ? (size_t)oi * Wo + oj : 0;
#pragma unroll
      for (int m = 0; m < 3; ++m) sd[m][r][q] = ok ? dmaps[(size_t)(m * C + c) * plane + o] : 0.f;
    }
    __syncthreads();
    // horizontal: input column q gathers output columns q - t -> patch column (q + 10 - t)
    for (int k = threadIdx.x; k < PATCH * TB; k += 256) {
      const int r = k / TB, q = k % TB;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int t = 0; t < WIN; ++t) {
        const float w = win.w[t];
        a0 += w * sd[0][r][q + WIN - 1 - t];
        a1 += w * sd[1][r][q + WIN - 1 - t];
        a2 += w * sd[2][r][q + WIN - 1 - t];
      }
      hd[0][r][q] = a0;
      hd[1][r][q] = a1;
      hd[2][r][q] = a2;
    }
    __syncthreads();
    const int i = by + ty, j = bx + tx;
    if (i < H && j < W) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int t = 0; t < WIN; ++t) {
        const float w = win.w[t];
        s0 += w * hd[0][ty + WIN - 1 - t][tx];
        s1 += w * hd[1][ty + WIN - 1 - t][tx];
        s2 += w * hd[2][ty + WIN - 1 - t][tx];
      }
      const size_t e = ((size_t)i * W + j) * C + c;
      const float xv = gt[e], yv = pred[e];
      const float d = yv - xv;
      const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      v_pred[e] = gs * (s0 + 2.f * yv * s1 + xv * s2) + gl * sgn;
    }
    __syncthreads();
  }
}

}  // namespace
}  // namespace gs

using namespace gs;

extern "C" int gsplat_l1_ssim_num_blocks(int img_height, int img_width) {
  if (img_height <= 0 || img_width <= 0) return 0;
  return (int)(cdiv(img_width, TB) * cdiv(img_height, TB));
}

static bool l1_ssim_args_ok(int H, int W, int C, const char *what) {
  if (H < WIN || W < WIN || C < 1 || C > 64) {
    set_error("%s: need H, W >= %d and 1 <= C <= 64 (H=%d W=%d C=%d)", what, WIN, H, W, C);
    return false;
  }
  return true;
}

static Win load_win(const float *window) {
  Win w;
  for (int t = 0; t < WIN; ++t) w.w[t] = window[t];
  return w;
}

extern "C" int gsplat_l1_ssim_forward(int img_height, int img_width, int channels,
                                      const float *pred, const float *gt, const float *window11,
                                      float ssim_lambda, float *partials, float *dmaps,
                                      float *loss, void *stream) {
  if (!l1_ssim_args_ok(img_height, img_width, channels, "l1_ssim_forward")) return 1;
  hipStream_t st = (hipStream_t)stream;
  const int nb = gsplat_l1_ssim_num_blocks(img_height, img_width);
  const Win w = load_win(window11);
  hipLaunchKernelGGL(l1_ssim_fwd_kernel, dim3(nb), dim3(256), 0, st, img_height, img_width,
                     channels, pred, gt, w, partials, dmaps);
  const double n1 = (double)channels * img_height * img_width;
  const double n2 = (double)channels * (img_height - WIN + 1) * (img_width - WIN + 1);
  hipLaunchKernelGGL(l1_ssim_finalize_kernel, dim3(1), dim3(256), 0, st, nb, partials,
                     1.0 / n1, 1.0 / n2, ssim_lambda, loss);
  return check_launch("l1_ssim_forward");
}

extern "C" int gsplat_l1_ssim_backward(int img_height, int img_width, int channels,
                                       const float *pred, const float *gt, const float *window11,
                                       float ssim_lambda, const float *dmaps,
                                       const float *grad_loss, float *v_pred, void *stream) {
  if (!l1_ssim_args_ok(img_height, img_width, channels, "l1_ssim_backward")) return 1;
  hipStream_t st = (hipStream_t)stream;
  const int nb = gsplat_l1_ssim_num_blocks(img_height, img_width);
  const Win w = load_win(window11);
  const double n1 = (double)channels * img_height * img_width;
  const double n2 = (double)channels * (img_height - WIN + 1) * (img_width - WIN + 1);
  hipLaunchKernelGGL(l1_ssim_bwd_kernel, dim3(nb), dim3(256), 0, st, img_height, img_width,
                     channels, pred, gt, w, dmaps, grad_loss, (float)(-ssim_lambda / n2),
                     (float)((1.0 - ssim_lambda) / n1), v_pred);
  return check_launch("l1_ssim_backward");
}
