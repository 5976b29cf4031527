// loss.hip -- fused splatfacto photometric loss for gfx950:
//     loss = (1 - lambda) * mean|gt - pred| + lambda * (1 - SSIM(gt, pred))
// with pytorch_msssim's SSIM (11x11 Gaussian window, sigma 1.5, 'valid' filtering, data range
// 1, K = (0.01, 0.03), mean over channels and positions), as nerfstudio 1.0 splatfacto's
// get_loss_dict computes it on every training step (the reference reaches it
// through gc_pipeline.py:477-478).  The torch restatement it must match is
// gaussctrl_exp_amd/train.py ssim() / splatfacto_loss().
//
// MI355X design (stencil work, HBM/LDS-bound; no MFMA):
//  * Forward: one 256-thread workgroup per 32x16 block of SSIM outputs (block origin (bx, by)).
//    Per channel it stages the 42x26 input patches of gt and pred in LDS, runs the separable
//    filter horizontally (5 moments: x, y, x^2, y^2, xy) then vertically, and evaluates the
//    SSIM map m and its partial derivatives with respect to the filtered pred statistics
//    (mu_y, E[y^2], E[xy]); those three maps are written for the backward.  The same
//    workgroup sums |gt - pred| over its 32x16 input block (the blocks tile the image) and
//    the SSIM values of its outputs; per-block partial sums are reduced by one tiny kernel
//    into the loss scalar (deterministic, no host sync).
//  * Backward: one workgroup per 32x16 block of input pixels correlates the three derivative
//    maps (42x26 halo patch in LDS, separable) back to input resolution and adds the L1 sign
//    term; the upstream gradient is read from device memory (no host sync).
#include "common.h"

namespace gs {
namespace {

constexpr int WIN = 11;
constexpr int TW = 32, TH = 16;      // block: 32 columns x 16 rows
constexpr int PW = TW + WIN - 1;     // 42-column halo patch
constexpr int PH = TH + WIN - 1;     // 26-row halo patch
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

// LDS layout rule (MI355X_MICROARCH.md §LDS): ds_read_b32 / ds_write_b32 bank by dword
// address mod 32 within each 32-lane half-wave.  Every pass below maps a half-wave to 32
// consecutive columns of ONE row, so all its LDS accesses are conflict-free; thread t works
// on column t % 32 and rows 2 (t / 32) and 2 (t / 32) + 1 of its block.

// partials[block] = {sum |gt - pred| over the block's input pixels (all channels),
//                    sum of SSIM map values over the block's valid outputs (all channels)}
// The caller's image clamp (gc_model.py:222: torch.clamp(rgb, max=1.0)) folded into the loss:
// CLAMP kernels read min(pred, 1) (NaN stays NaN, as torch.clamp) and mask the gradient where
// torch's clamp backward does (pass where pred <= 1).
template <bool CLAMP>
__device__ __forceinline__ float clamp_pred(float x) {
  return CLAMP ? (x > 1.f ? 1.f : x) : x;
}
template <bool CLAMP>
__device__ __forceinline__ float clamp_mask(float x) {
  return CLAMP ? (x <= 1.f ? 1.f : 0.f) : 1.f;
}

template <bool CLAMP>
__global__ __launch_bounds__(256) void l1_ssim_fwd_kernel(int H, int W, int C,
                                                          const float *__restrict__ pred,
                                                          const float *__restrict__ gt, Win win,
                                                          float *__restrict__ partials,
                                                          float *__restrict__ dmaps) {
  __shared__ float sx[PH * PW], sy[PH * PW];
  __shared__ float hm[5][PH][TW];
  __shared__ float red[4];
  const int Ho = H - WIN + 1, Wo = W - WIN + 1;
  const int nbx = (W + TW - 1) / TW;
  const int bx = (blockIdx.x % nbx) * TW, by = (blockIdx.x / nbx) * TH;
  const int tx = threadIdx.x & 31, ty = (threadIdx.x >> 5) * 2;
  const float c1 = K1 * K1, c2 = K2 * K2;
  float l1 = 0.f, ssum = 0.f;
  const size_t plane = (size_t)Ho * Wo;
  // the patch is staged with the next channel's values prefetched into registers while the
  // current channel is filtered (SLOTS = ceil(26 * 42 / 256) elements per thread)
  constexpr int SLOTS = (PH * PW + 255) / 256;
  float px[SLOTS], py[SLOTS];
  auto fetch = [&](int c) {
#pragma unroll
    for (int u = 0; u < SLOTS; ++u) {
      const int k = threadIdx.x + 256 * u;
      const int r = k / PW, q = k - r * PW;
      const int i = by + r, j = bx + q;
      px[u] = py[u] = 0.f;
      if (k < PH * PW && i < H && j < W) {
        px[u] = gt[((size_t)i * W + j) * C + c];
        py[u] = clamp_pred<CLAMP>(pred[((size_t)i * W + j) * C + c]);
      }
    }
  };
  fetch(0);
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int u = 0; u < SLOTS; ++u) {
      const int k = threadIdx.x + 256 * u;
      if (k < PH * PW) {
        sx[k] = px[u];
        sy[k] = py[u];
      }
    }
    if (c + 1 < C) fetch(c + 1);
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {  // L1 over this block's own input pixels
      const int i = by + ty + rr, j = bx + tx;
      if (i < H && j < W) l1 += fabsf(sx[(ty + rr) * PW + tx] - sy[(ty + rr) * PW + tx]);
    }
    // horizontal pass: patch rows 0..25, output columns 0..31 (one row per half-wave)
    for (int k = threadIdx.x; k < PH * TW; k += 256) {
      const int r = k >> 5, q = k & 31;
      float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f, m4 = 0.f;
#pragma unroll
      for (int t = 0; t < WIN; ++t) {
        const float w = win.w[t], xv = sx[r * PW + q + t], yv = sy[r * PW + q + t];
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
    // vertical pass: output rows ty and ty + 1 share 10 of their 11 taps (12 rows loaded)
    float a[2][5];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int m = 0; m < 5; ++m) a[rr][m] = 0.f;
#pragma unroll
    for (int u = 0; u <= WIN; ++u) {
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        const float h = hm[m][ty + u][tx];
        if (u < WIN) a[0][m] += win.w[u] * h;
        if (u >= 1) a[1][m] += win.w[u - 1] * h;
      }
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int oi = by + ty + rr, oj = bx + tx;
      if (oi < Ho && oj < Wo) {
        const float mu1 = a[rr][0], mu2 = a[rr][1], exx = a[rr][2], eyy = a[rr][3],
                    exy = a[rr][4];
        const float s11 = exx - mu1 * mu1, s22 = eyy - mu2 * mu2, s12 = exy - mu1 * mu2;
        const float A = 2.f * mu1 * mu2 + c1, B = mu1 * mu1 + mu2 * mu2 + c1;
        const float Cn = 2.f * s12 + c2, D = s11 + s22 + c2;
        const float rB = 1.f / B, rD = 1.f / D;  // two divisions; the rest are products
        const float l = A * rB, cs = Cn * rD;
        ssum += l * cs;
        // d m / d mu2, d m / d E[y^2], d m / d E[xy]  (mu1, E[x^2] belong to gt: constant)
        const float dl = (2.f * mu1 * B - 2.f * mu2 * A) * (rB * rB);
        const float dcs = (-2.f * mu1 * D + 2.f * mu2 * Cn) * (rD * rD);
        const size_t o = (size_t)oi * Wo + oj;
        dmaps[(size_t)(0 * C + c) * plane + o] = dl * cs + l * dcs;
        dmaps[(size_t)(1 * C + c) * plane + o] = -l * cs * rD;
        dmaps[(size_t)(2 * C + c) * plane + o] = 2.f * l * rD;
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

// ssim_lambda == 0: plain L1 (the SSIM term has weight zero) -- one streaming pass.
// partials[2 b] = sum |gt - pred| over this block's grid-stride share, partials[2 b + 1] = 0.
template <bool CLAMP>
__global__ __launch_bounds__(256) void l1_only_fwd_kernel(long long n, const float *__restrict__ pred,
                                                          const float *__restrict__ gt,
                                                          float *__restrict__ partials) {
  __shared__ float red[4];
  float acc = 0.f;
  long long i0 = 0;
  if ((((uintptr_t)pred | (uintptr_t)gt) & 15) == 0) {  // 16-B vectors, then the tail
    const long long n4 = n >> 2;
    const float4 *p4 = reinterpret_cast<const float4 *>(pred);
    const float4 *g4 = reinterpret_cast<const float4 *>(gt);
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4;
         i += (long long)gridDim.x * 256) {
      const float4 p = p4[i], g = g4[i];
      acc += fabsf(g.x - clamp_pred<CLAMP>(p.x)) + fabsf(g.y - clamp_pred<CLAMP>(p.y)) +
             fabsf(g.z - clamp_pred<CLAMP>(p.z)) + fabsf(g.w - clamp_pred<CLAMP>(p.w));
    }
    i0 = n4 << 2;
  }
  for (long long i = i0 + (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    acc += fabsf(gt[i] - clamp_pred<CLAMP>(pred[i]));
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = acc;
    partials[2 * blockIdx.x + 1] = 0.f;
  }
}

template <bool CLAMP>
__global__ __launch_bounds__(256) void l1_only_bwd_kernel(long long n, const float *__restrict__ pred,
                                                          const float *__restrict__ gt,
                                                          const float *__restrict__ grad_out,
                                                          float l1_scale,
                                                          float *__restrict__ v_pred) {
  const float gl = grad_out[0] * l1_scale;
  auto g1 = [&](float p, float g) {
    const float d = clamp_pred<CLAMP>(p) - g;
    return gl * (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) * clamp_mask<CLAMP>(p);
  };
  long long i0 = 0;
  if ((((uintptr_t)pred | (uintptr_t)gt | (uintptr_t)v_pred) & 15) == 0) {  // 16-B vectors
    const long long n4 = n >> 2;
    const float4 *p4 = reinterpret_cast<const float4 *>(pred);
    const float4 *g4 = reinterpret_cast<const float4 *>(gt);
    float4 *v4 = reinterpret_cast<float4 *>(v_pred);
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4;
         i += (long long)gridDim.x * 256) {
      const float4 p = p4[i], g = g4[i];
      v4[i] = make_float4(g1(p.x, g.x), g1(p.y, g.y), g1(p.z, g.z), g1(p.w, g.w));
    }
    i0 = n4 << 2;
  }
  for (long long i = i0 + (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    v_pred[i] = g1(pred[i], gt[i]);
}

// loss = (1 - lambda) * L1 / (C H W) + lambda * (1 - SSIM_sum / (C Ho Wo)); one workgroup,
// double accumulation in a fixed order (deterministic).
__global__ __launch_bounds__(1024) void l1_ssim_finalize_kernel(int nblocks, const float *partials,
                                                                double inv_l1, double inv_ssim,
                                                                float lambda, float *loss) {
  // (1,024 threads, every load of a round issued before the first add: a loop waiting for each
  // load in turn is a chain of L2 latencies)
  constexpr int NT = 1024, U = 4;
  __shared__ double ra[NT], rb[NT];
  double a = 0.0, b = 0.0;
  for (int base = 0; base < nblocks; base += NT * U) {
    float2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = base + u * NT + threadIdx.x;
      v[u] = k < nblocks ? reinterpret_cast<const float2 *>(partials)[k] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a += v[u].x;
      b += v[u].y;
    }
  }
  ra[threadIdx.x] = a;
  rb[threadIdx.x] = b;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      ra[threadIdx.x] += ra[threadIdx.x + s];
      rb[threadIdx.x] += rb[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    loss[0] = (float)((1.0 - lambda) * ra[0] * inv_l1 + lambda * (1.0 - rb[0] * inv_ssim));
}

template <bool CLAMP>
__global__ __launch_bounds__(256) void l1_ssim_bwd_kernel(
    int H, int W, int C, const float *__restrict__ pred, const float *__restrict__ gt, Win win,
    const float *__restrict__ dmaps, const float *__restrict__ grad_out, float ssim_scale,
    float l1_scale, float *__restrict__ v_pred) {
  __shared__ float sd[3][PH * PW];
  __shared__ float hd[3][PH][TW];
  const int Ho = H - WIN + 1, Wo = W - WIN + 1;
  const int nbx = (W + TW - 1) / TW;
  const int bx = (blockIdx.x % nbx) * TW, by = (blockIdx.x / nbx) * TH;
  const int tx = threadIdx.x & 31, ty = (threadIdx.x >> 5) * 2;
  const float g = grad_out[0];
  const float gs = g * ssim_scale, gl = g * l1_scale;
  const size_t plane = (size_t)Ho * Wo;
  // input q receives from outputs p = q - t, t in [0, 10]: patch rows/cols start at b - 10
  const int oy0 = by - (WIN - 1), ox0 = bx - (WIN - 1);
  constexpr int SLOTS = (PH * PW + 255) / 256;
  float pd[3][SLOTS];
  auto fetch = [&](int c) {
#pragma unroll
    for (int u = 0; u < SLOTS; ++u) {
      const int k = threadIdx.x + 256 * u;
      const int r = k / PW, q = k - r * PW;
      const int oi = oy0 + r, oj = ox0 + q;
      const bool ok = k < PH * PW && oi >= 0 && oj >= 0 && oi < Ho && oj < Wo;
      const size_t o = ok ? (size_t)oi * Wo + oj : 0;
#pragma unroll
      for (int m = 0; m < 3; ++m) pd[m][u] = ok ? dmaps[(size_t)(m * C + c) * plane + o] : 0.f;
    }
  };
  fetch(0);
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int u = 0; u < SLOTS; ++u) {
      const int k = threadIdx.x + 256 * u;
      if (k < PH * PW) {
#pragma unroll
        for (int m = 0; m < 3; ++m) sd[m][k] = pd[m][u];
      }
    }
    if (c + 1 < C) fetch(c + 1);
    __syncthreads();
    // horizontal: input column q gathers output columns q - t -> patch column (q + 10 - t)
    for (int k = threadIdx.x; k < PH * TW; k += 256) {
      const int r = k >> 5, q = k & 31;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int t = 0; t < WIN; ++t) {
        const float w = win.w[t];
        const int e = r * PW + q + WIN - 1 - t;
        a0 += w * sd[0][e];
        a1 += w * sd[1][e];
        a2 += w * sd[2][e];
      }
      hd[0][r][q] = a0;
      hd[1][r][q] = a1;
      hd[2][r][q] = a2;
    }
    __syncthreads();
    // vertical: input row ty gathers patch rows ty + 10 - t (t ascending = u descending);
    // rows ty and ty + 1 share 10 of their 11 taps
    float s[2][3];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int m = 0; m < 3; ++m) s[rr][m] = 0.f;
#pragma unroll
    for (int u = WIN; u >= 0; --u) {
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const float h = hd[m][ty + u][tx];
        if (u < WIN) s[0][m] += win.w[WIN - 1 - u] * h;
        if (u >= 1) s[1][m] += win.w[WIN - u] * h;
      }
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int i = by + ty + rr, j = bx + tx;
      if (i < H && j < W) {
        const size_t e = ((size_t)i * W + j) * C + c;
        const float p = pred[e];
        const float xv = gt[e], yv = clamp_pred<CLAMP>(p);
        const float d = yv - xv;
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        v_pred[e] = (gs * (s[rr][0] + 2.f * yv * s[rr][1] + xv * s[rr][2]) + gl * sgn) *
                    clamp_mask<CLAMP>(p);
      }
    }
    __syncthreads();
  }
}

}  // namespace


}  // namespace gs

using namespace gs;

extern "C" int gsplat_l1_ssim_num_blocks(int img_height, int img_width) {
  if (img_height <= 0 || img_width <= 0) return 0;
  return (int)(cdiv(img_width, TW) * cdiv(img_height, TH));
}

static bool l1_ssim_args_ok(int H, int W, int C, const char *what, float lambda = 1.f) {
  const int min_hw = lambda == 0.f ? 1 : WIN;  // the L1-only path has no SSIM window
  if (H < min_hw || W < min_hw || C < 1 || C > 64) {
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
                                      float ssim_lambda, int clamp_pred, float *partials,
                                      float *dmaps, float *loss, void *stream) {
  if (!l1_ssim_args_ok(img_height, img_width, channels, "l1_ssim_forward", ssim_lambda)) return 1;
  hipStream_t st = (hipStream_t)stream;
  const int nb = gsplat_l1_ssim_num_blocks(img_height, img_width);
  if (ssim_lambda == 0.f) {  // L1 only: no SSIM statistics, dmaps untouched
    if (clamp_pred)
      hipLaunchKernelGGL(l1_only_fwd_kernel<true>, dim3(nb), dim3(256), 0, st,
                         (long long)img_height * img_width * channels, pred, gt, partials);
    else
      hipLaunchKernelGGL(l1_only_fwd_kernel<false>, dim3(nb), dim3(256), 0, st,
                         (long long)img_height * img_width * channels, pred, gt, partials);
  } else {
    const Win w = load_win(window11);
    if (clamp_pred)
      hipLaunchKernelGGL(l1_ssim_fwd_kernel<true>, dim3(nb), dim3(256), 0, st, img_height,
                         img_width, channels, pred, gt, w, partials, dmaps);
    else
      hipLaunchKernelGGL(l1_ssim_fwd_kernel<false>, dim3(nb), dim3(256), 0, st, img_height,
                         img_width, channels, pred, gt, w, partials, dmaps);
  }
  const double n1 = (double)channels * img_height * img_width;
  const double n2 = (double)channels * (img_height - WIN + 1) * (img_width - WIN + 1);
  hipLaunchKernelGGL(l1_ssim_finalize_kernel, dim3(1), dim3(1024), 0, st, nb, partials,
                     1.0 / n1, 1.0 / n2, ssim_lambda, loss);
  return check_launch("l1_ssim_forward");
}

extern "C" int gsplat_l1_ssim_backward(int img_height, int img_width, int channels,
                                       const float *pred, const float *gt, const float *window11,
                                       float ssim_lambda, int clamp_pred, const float *dmaps,
                                       const float *grad_loss, float *v_pred, void *stream) {
  if (!l1_ssim_args_ok(img_height, img_width, channels, "l1_ssim_backward", ssim_lambda)) return 1;
  hipStream_t st = (hipStream_t)stream;
  const int nb = gsplat_l1_ssim_num_blocks(img_height, img_width);
  const double n1 = (double)channels * img_height * img_width;
  const double n2 = (double)channels * (img_height - WIN + 1) * (img_width - WIN + 1);
  if (ssim_lambda == 0.f) {
    if (clamp_pred)
      hipLaunchKernelGGL(l1_only_bwd_kernel<true>, dim3(nb), dim3(256), 0, st, (long long)n1, pred,
                         gt, grad_loss, (float)(1.0 / n1), v_pred);
    else
      hipLaunchKernelGGL(l1_only_bwd_kernel<false>, dim3(nb), dim3(256), 0, st, (long long)n1,
                         pred, gt, grad_loss, (float)(1.0 / n1), v_pred);
    return check_launch("l1_ssim_backward");
  }
  const Win w = load_win(window11);
  if (clamp_pred)
    hipLaunchKernelGGL(l1_ssim_bwd_kernel<true>, dim3(nb), dim3(256), 0, st, img_height,
                       img_width, channels, pred, gt, w, dmaps, grad_loss,
                       (float)(-ssim_lambda / n2), (float)((1.0 - ssim_lambda) / n1), v_pred);
  else
    hipLaunchKernelGGL(l1_ssim_bwd_kernel<false>, dim3(nb), dim3(256), 0, st, img_height,
                       img_width, channels, pred, gt, w, dmaps, grad_loss,
                       (float)(-ssim_lambda / n2), (float)((1.0 - ssim_lambda) / n1), v_pred);
  return check_launch("l1_ssim_backward");
}
