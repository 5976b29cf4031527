// sh.hip -- spherical-harmonics colour evaluation (forward / backward) for gfx950.
//
// Replaces gsplat 0.1.2.1 _C.compute_sh_forward/backward (sh.cuh), called from
// /root/reference/gaussctrl/gc_model.py:200.  The coefficient block is [N, K, 3] fp32
// (K = num_sh_bases(degree), 192 B per Gaussian at degree 3): the largest per-Gaussian
// stream of the whole path.  A lane-per-Gaussian load of it would stride 192 B per lane,
// so each 256-thread workgroup instead stages its 256 Gaussians' coefficient block through
// LDS with 16-byte, fully coalesced loads (forward) / stores (backward); the per-Gaussian
// arithmetic then reads its own row from LDS.
#include "sh_math.h"
#include "adam_math.h"
#include "exchange_layout.h"

namespace gs {
namespace {

// The block's coefficient slab [256*K*3] is staged through LDS (stage_rows: 16-byte loads
// when the slab start is 16-byte aligned, else dword loads).
template <int K>
__global__ __launch_bounds__(256) void sh_fwd_kernel(int n, int degrees_to_use,
                                                     const float *__restrict__ viewdirs,
                                                     const float *__restrict__ coeffs,
                                                     float *__restrict__ colors) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int ROW = K * 3;
  constexpr int ROWP = sh_row_pitch(K);
  constexpr int SH_THREADS = sh_threads(K);
  const long long g0 = (long long)blockIdx.x * SH_THREADS;
  const int cnt = (int)min((long long)SH_THREADS, (long long)n - g0);
  stage_rows<ROW, ROWP, SH_THREADS>(coeffs + g0 * ROW, cnt, smem);
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= cnt) return;
  const long long g = g0 + t;
  float b[25];
  int nb = sh_basis(degrees_to_use, viewdirs[3 * g], viewdirs[3 * g + 1], viewdirs[3 * g + 2],
                    b);
  const float *co = smem + t * ROWP;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    colors[3 * g + c] = sh_channel<K>(b, nb, [&](int k) { return co[k * 3 + c]; });
}

// SPLIT: the gradient goes to v_coeffs = v_dc [N,3] (basis 0) and v_rest [N,K-1,3] -- the
// caller's cat(features_dc[:, None], features_rest) undone (sh.py bypasses that cat in the
// autograd graph, so the parameters receive contiguous gradients and need no layout copies).
template <int K, bool SPLIT = false>
__global__ __launch_bounds__(256) void sh_bwd_kernel(int n, int degrees_to_use,
                                                             const float *__restrict__ viewdirs,
                                                             const float *__restrict__ v_colors,
                                                             float *__restrict__ v_coeffs,
                                                             float *__restrict__ v_rest = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int ROW = K * 3;
  constexpr int ROWP = sh_row_pitch(K);
  constexpr int SH_THREADS = sh_threads(K);
  const long long g0 = (long long)blockIdx.x * SH_THREADS;
  const int cnt = (int)min((long long)SH_THREADS, (long long)n - g0);
  const int t = threadIdx.x;
  if (t < cnt) {
    const long long g = g0 + t;
    float b[25];
    int nb = sh_basis(degrees_to_use, viewdirs[3 * g], viewdirs[3 * g + 1],
                      viewdirs[3 * g + 2], b);
    float vc0 = v_colors[3 * g], vc1 = v_colors[3 * g + 1], vc2 = v_colors[3 * g + 2];
    float *row = smem + t * ROWP;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float bk = k < nb ? b[k] : 0.f;
      row[k * 3 + 0] = bk * vc0;
      row[k * 3 + 1] = bk * vc1;
      row[k * 3 + 2] = bk * vc2;
    }
  }
  __syncthreads();
  if constexpr (SPLIT) {
    store_cols<3, 0, ROWP, SH_THREADS>(smem, cnt, v_coeffs + g0 * 3);
    if constexpr (K > 1) store_cols<ROW - 3, 3, ROWP, SH_THREADS>(smem, cnt, v_rest + g0 * (ROW - 3));
  } else {
    store_rows<K>(smem, cnt, v_coeffs + g0 * ROW);
  }
}

// Multi-view SH backward for data-parallel training: the coefficient
// gradient of one view is the rank-1 product Y(dir) (x) v_colors, and the direction is the
// (replicated) mean minus that view's camera centre, so the ranks exchange only v_colors
// (12 B per Gaussian) plus their camera centre, and every rank evaluates
//   v_coeffs[i] = sum_r Y(means[i] - campos_r) (x) v_colors_r[i]
// itself -- in view order, so every rank produces bit-identical gradients.
// views[r * view_stride + 3 i + c] = v_colors of view r; views[r * view_stride + 3 n + c] =
// camera centre of view r.
// SPLIT: the coefficient gradient goes to two tensors, v_coeffs = v_dc [N,3] (basis 0) and
// v_rest [N,K-1,3] (bases 1..K-1) -- splatfacto's features_dc / features_rest parameters,
// which the fused training path (preprocess.hip) keeps separate.
template <int K, bool SPLIT = false>
__global__ __launch_bounds__(256) void sh_bwd_views_kernel(int n, int degrees_to_use,
                                                           int num_views,
                                                           const float *__restrict__ means,
                                                           const float *__restrict__ views,
                                                           long long view_stride,
                                                           float *__restrict__ v_coeffs,
                                                           float *__restrict__ v_rest = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int ROW = K * 3;
  constexpr int ROWP = sh_row_pitch(K);
  constexpr int SH_THREADS = sh_threads(K);
  const long long g0 = (long long)blockIdx.x * SH_THREADS;
  const int cnt = (int)min((long long)SH_THREADS, (long long)n - g0);
  const int t = threadIdx.x;
  if (t < cnt) {
    const long long g = g0 + t;
    const float mx = means[3 * g], my = means[3 * g + 1], mz = means[3 * g + 2];
    float acc[ROW];
#pragma unroll
    for (int k = 0; k < ROW; ++k) acc[k] = 0.f;
    // software-pipelined over views: view r+1's colour gradient and camera centre are in
    // flight while view r's basis and outer product are computed
    const float *cam = views + 3LL * n;  // uniform addresses: scalar loads
    float c0 = cam[0], c1 = cam[1], c2 = cam[2];
    float vc0 = views[3 * g], vc1 = views[3 * g + 1], vc2 = views[3 * g + 2];
    for (int r = 0; r < num_views; ++r) {
      const float dx = mx - c0, dy = my - c1, dz = mz - c2;
      const float u0 = vc0, u1 = vc1, u2 = vc2;
      if (r + 1 < num_views) {
        const float *view = views + (r + 1) * view_stride;
        c0 = view[3LL * n];
        c1 = view[3LL * n + 1];
        c2 = view[3LL * n + 2];
        vc0 = view[3 * g];
        vc1 = view[3 * g + 1];
        vc2 = view[3 * g + 2];
      }
      float b[25];
      const int nb = sh_basis(degrees_to_use, dx, dy, dz, b);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float bk = k < nb ? b[k] : 0.f;
        acc[k * 3 + 0] += bk * u0;
        acc[k * 3 + 1] += bk * u1;
        acc[k * 3 + 2] += bk * u2;
      }
    }
    float *row = smem + t * ROWP;
#pragma unroll
    for (int k = 0; k < ROW; ++k) row[k] = acc[k];
  }
  __syncthreads();
  if constexpr (SPLIT) {
    store_cols<3, 0, ROWP, SH_THREADS>(smem, cnt, v_coeffs + g0 * 3);
    if constexpr (K > 1) store_cols<ROW - 3, 3, ROWP, SH_THREADS>(smem, cnt, v_rest + g0 * (ROW - 3));
  } else {
    store_rows<K>(smem, cnt, v_coeffs + g0 * ROW);
  }
}

// sh_bwd_views_kernel<K, true> over a table of dense and sparse view records
// (exchange_layout.h): the sum runs in table order, skipping a sparse record's absent
// Gaussians -- exactly zero colour gradients, whose products would add +-0 to an accumulator
// that is never -0 -- so sparse and dense records of the same views give the same bits.
// Software-pipelined two views deep: view r + 2's mask word, prefix and camera centre (dense:
// its colour gradient) are loaded while view r + 1's row is resolved and its colour gradient
// loaded, while view r's basis and outer product are computed.
struct XsAhead {  // a view's first-stage loads
  unsigned long long m;
  uint32_t pre;
  float c[3], u[3];
};
__device__ __forceinline__ void xs_load_a(const ViewTable &tab, int r, long long n, long long g,
                                          long long W, XsAhead &a) {
  const float *p = tab.rec[r];
  if (tab.cap[r] < 0) {
    a.c[0] = p[3 * n];
    a.c[1] = p[3 * n + 1];
    a.c[2] = p[3 * n + 2];
    a.u[0] = p[3 * g];
    a.u[1] = p[3 * g + 1];
    a.u[2] = p[3 * g + 2];
    a.m = ~0ull;
    a.pre = 0u;
  } else {
    a.c[0] = p[0];
    a.c[1] = p[1];
    a.c[2] = p[2];
    a.m = reinterpret_cast<const unsigned long long *>(p + XS_HDR)[g >> 6];
    a.pre = reinterpret_cast<const uint32_t *>(p + XS_HDR + 2 * W)[g >> 6];
  }
}
// second stage: the row of a sparse view and its colour gradient (0 when absent)
__device__ __forceinline__ bool xs_resolve(const ViewTable &tab, int r, long long n, long long g,
                                           XsAhead &a) {
  if (tab.cap[r] < 0) return true;
  const int b = (int)(g & 63);
  const bool has = (a.m >> b) & 1ull;
  const long long pos = (long long)a.pre + __popcll(a.m & ((1ull << b) - 1ull));
  a.u[0] = a.u[1] = a.u[2] = 0.f;
  if (has && pos < tab.cap[r]) {
    const float *vals = tab.rec[r] + xs_values_at(n);
    a.u[0] = vals[3 * pos];
    a.u[1] = vals[3 * pos + 1];
    a.u[2] = vals[3 * pos + 2];
    return true;
  }
  return false;
}
// The Adam step of the two SH-feature groups fused into the multi-view table kernel (N > 1
// training step, TrainStep): the summed coefficient gradient never leaves the workgroup -- each
// parameter element is updated from its LDS gradient row with adam_math.h's element update (the
// arithmetic of gsplat_adam_step), so the 2 x 192 B per Gaussian of gradient write + re-read
// of the unfused table kernel + multi-tensor Adam disappear.  Group 0 = features_dc [N,3],
// group 1 = features_rest [N,K-1,3]; ss / bc2s as the host computes them for gsplat_adam_step.
struct ShAdam {
  float *p[2], *m[2], *v[2];
  float ss[2], bc2s;
  float beta1, beta2, eps;
};

// Columns [C0, C0 + WIDTH) of the block's cnt LDS gradient rows (pitch ROWP) applied to the
// contiguous parameter slab p/m/v[base : base + cnt * WIDTH] (one group): 16-B accesses when
// the three slabs are 16-B aligned, else dwords -- every element through adam_elem either way.
template <int WIDTH, int C0, int ROWP, int THREADS>
__device__ __forceinline__ void adam_cols(const float *smem, int cnt, const ShAdam &o, int grp,
                                          long long base) {
  const int total = cnt * WIDTH;
  const float w1 = 1.f - o.beta1, w2 = 1.f - o.beta2;
  const float ss = o.ss[grp], bc2s = o.bc2s;
  float *__restrict__ P = o.p[grp] + base;
  float *__restrict__ M = o.m[grp] + base;
  float *__restrict__ V = o.v[grp] + base;
  auto at = [&](int k) {
    const int r = k / WIDTH;
    return smem[r * ROWP + C0 + (k - r * WIDTH)];
  };
  const bool vec = ((((uintptr_t)P) | ((uintptr_t)M) | ((uintptr_t)V)) & 15) == 0;
  int k0 = 0;
  if (vec) {
    const int nv = total >> 2;
    float4 *P4 = reinterpret_cast<float4 *>(P), *M4 = reinterpret_cast<float4 *>(M),
           *V4 = reinterpret_cast<float4 *>(V);
    for (int k = threadIdx.x; k < nv; k += THREADS) {
      float4 pv = P4[k], mv = M4[k], vv = V4[k];
      adam_elem(pv.x, at(4 * k), mv.x, vv.x, w1, o.beta2, w2, ss, bc2s, o.eps);
      adam_elem(pv.y, at(4 * k + 1), mv.y, vv.y, w1, o.beta2, w2, ss, bc2s, o.eps);
      adam_elem(pv.z, at(4 * k + 2), mv.z, vv.z, w1, o.beta2, w2, ss, bc2s, o.eps);
      adam_elem(pv.w, at(4 * k + 3), mv.w, vv.w, w1, o.beta2, w2, ss, bc2s, o.eps);
      P4[k] = pv;
      M4[k] = mv;
      V4[k] = vv;
    }
    k0 = nv << 2;
  }
  for (int k = k0 + threadIdx.x; k < total; k += THREADS) {
    float pv = P[k], mv = M[k], vv = V[k];
    adam_elem(pv, at(k), mv, vv, w1, o.beta2, w2, ss, bc2s, o.eps);
    P[k] = pv;
    M[k] = mv;
    V[k] = vv;
  }
}

template <int K, bool ADAM = false>
__global__ __launch_bounds__(256) void sh_bwd_table_kernel(int n, int degrees_to_use,
                                                           int num_views,
                                                           const float *__restrict__ means,
                                                           const ViewTable tab,
                                                           float *__restrict__ v_dc,
                                                           float *__restrict__ v_rest,
                                                           const ShAdam adam = {}) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int ROW = K * 3;
  constexpr int ROWP = sh_row_pitch(K);
  constexpr int SH_THREADS = sh_threads(K);
  const long long g0 = (long long)blockIdx.x * SH_THREADS;
  const int cnt = (int)min((long long)SH_THREADS, (long long)n - g0);
  const int t = threadIdx.x;
  if (t < cnt) {
    const long long g = g0 + t;
    const long long W = xs_words(n);
    const float mx = means[3 * g], my = means[3 * g + 1], mz = means[3 * g + 2];
    float acc[ROW];
#pragma unroll
    for (int k = 0; k < ROW; ++k) acc[k] = 0.f;
    XsAhead b, a;  // b: view r + 1 (resolved), a: view r + 2 (first stage)
    xs_load_a(tab, 0, n, g, W, b);
    bool hb = xs_resolve(tab, 0, n, g, b);
    if (num_views > 1) xs_load_a(tab, 1, n, g, W, a);
    for (int r = 0; r < num_views; ++r) {
      const float c0 = b.c[0], c1 = b.c[1], c2 = b.c[2];
      const float u0 = b.u[0], u1 = b.u[1], u2 = b.u[2];
      const bool has = hb;
      if (r + 1 < num_views) {
        b = a;
        hb = xs_resolve(tab, r + 1, n, g, b);
        if (r + 2 < num_views) xs_load_a(tab, r + 2, n, g, W, a);
      }
      if (!has) continue;
      float bs[25];
      const int nb = sh_basis(degrees_to_use, mx - c0, my - c1, mz - c2, bs);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float bk = k < nb ? bs[k] : 0.f;
        acc[k * 3 + 0] += bk * u0;
        acc[k * 3 + 1] += bk * u1;
        acc[k * 3 + 2] += bk * u2;
      }
    }
    float *rowp = smem + t * ROWP;
#pragma unroll
    for (int k = 0; k < ROW; ++k) rowp[k] = acc[k];
  }
  __syncthreads();
  if constexpr (ADAM) {
    adam_cols<3, 0, ROWP, SH_THREADS>(smem, cnt, adam, 0, g0 * 3);
    if constexpr (K > 1) adam_cols<ROW - 3, 3, ROWP, SH_THREADS>(smem, cnt, adam, 1, g0 * (ROW - 3));
  } else {
    store_cols<3, 0, ROWP, SH_THREADS>(smem, cnt, v_dc + g0 * 3);
    if constexpr (K > 1)
      store_cols<ROW - 3, 3, ROWP, SH_THREADS>(smem, cnt, v_rest + g0 * (ROW - 3));
  }
}

}  // namespace
}  // namespace gs

using namespace gs;

#define SH_DISPATCH(KERNEL, ...)                                                         \
  switch (K) {                                                                           \
    case 1: hipLaunchKernelGGL(KERNEL<1>, grid, block, smem, st, __VA_ARGS__); break;    \
    case 4: hipLaunchKernelGGL(KERNEL<4>, grid, block, smem, st, __VA_ARGS__); break;    \
    case 9: hipLaunchKernelGGL(KERNEL<9>, grid, block, smem, st, __VA_ARGS__); break;    \
    case 16: hipLaunchKernelGGL(KERNEL<16>, grid, block, smem, st, __VA_ARGS__); break;  \
    default: hipLaunchKernelGGL(KERNEL<25>, grid, block, smem, st, __VA_ARGS__); break;  \
  }

extern "C" int gsplat_compute_sh_forward(int num_points, int degree, int degrees_to_use,
                                         const float *viewdirs, const float *coeffs,
                                         float *colors, void *stream) {
  if (num_points < 0 || degree < 0 || degree > 4 || degrees_to_use < 0 ||
      degrees_to_use > degree) {
    set_error("compute_sh_forward: bad args (N=%d degree=%d degrees_to_use=%d)", num_points,
              degree, degrees_to_use);
    return 1;
  }
  if (num_points == 0) return 0;
  const int K = num_bases(degree);
  const int thr = sh_threads(K);
  dim3 grid(cdiv(num_points, thr)), block(thr);
  size_t smem = (size_t)thr * sh_row_pitch(K) * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  SH_DISPATCH(sh_fwd_kernel, num_points, degrees_to_use, viewdirs, coeffs, colors);
  return check_launch("compute_sh_forward");
}

extern "C" int gsplat_compute_sh_backward(int num_points, int degree, int degrees_to_use,
                                          const float *viewdirs, const float *v_colors,
                                          float *v_coeffs, void *stream) {
  if (num_points < 0 || degree < 0 || degree > 4 || degrees_to_use < 0 ||
      degrees_to_use > degree) {
    set_error("compute_sh_backward: bad args (N=%d degree=%d degrees_to_use=%d)", num_points,
              degree, degrees_to_use);
    return 1;
  }
  if (num_points == 0) return 0;
  const int K = num_bases(degree);
  const int thr = sh_threads(K);
  dim3 grid(cdiv(num_points, thr)), block(thr);
  size_t smem = (size_t)thr * sh_row_pitch(K) * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  SH_DISPATCH(sh_bwd_kernel, num_points, degrees_to_use, viewdirs, v_colors, v_coeffs);
  return check_launch("compute_sh_backward");
}

extern "C" int gsplat_compute_sh_backward_views(int num_points, int degree, int degrees_to_use,
                                                int num_views, const float *means3d,
                                                const float *views, long long view_stride,
                                                float *v_coeffs, void *stream) {
  if (num_points < 0 || degree < 0 || degree > 4 || degrees_to_use < 0 ||
      degrees_to_use > degree || num_views < 1 || view_stride < 3LL * num_points + 3) {
    set_error("compute_sh_backward_views: bad args (N=%d degree=%d degrees_to_use=%d views=%d "
              "stride=%lld)", num_points, degree, degrees_to_use, num_views, view_stride);
    return 1;
  }
  if (num_points == 0) return 0;
  const int K = num_bases(degree);
  const int thr = sh_threads(K);
  dim3 grid(cdiv(num_points, thr)), block(thr);
  size_t smem = (size_t)thr * sh_row_pitch(K) * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  SH_DISPATCH(sh_bwd_views_kernel, num_points, degrees_to_use, num_views, means3d, views,
              view_stride, v_coeffs);
  return check_launch("compute_sh_backward_views");
}

extern "C" int gsplat_compute_sh_backward_views_split(int num_points, int degree,
                                                      int degrees_to_use, int num_views,
                                                      const float *means3d, const float *views,
                                                      long long view_stride, float *v_dc,
                                                      float *v_rest, void *stream) {
  if (num_points < 0 || degree < 0 || degree > 4 || degrees_to_use < 0 ||
      degrees_to_use > degree || num_views < 1 || view_stride < 3LL * num_points + 3 ||
      (num_points > 0 && (!v_dc || (degree > 0 && !v_rest)))) {
    set_error("compute_sh_backward_views_split: bad args (N=%d degree=%d degrees_to_use=%d "
              "views=%d stride=%lld)", num_points, degree, degrees_to_use, num_views, view_stride);
    return 1;
  }
  if (num_points == 0) return 0;
  const int K = num_bases(degree);
  const int thr = sh_threads(K);
  dim3 grid(cdiv(num_points, thr)), block(thr);
  size_t smem = (size_t)thr * sh_row_pitch(K) * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
#define SPLIT_CASE(KK)                                                                    \
  case KK:                                                                                \
    hipLaunchKernelGGL((sh_bwd_views_kernel<KK, true>), grid, block, smem, st, num_points, \
                       degrees_to_use, num_views, means3d, views, view_stride, v_dc, v_rest); \
    break;
    SPLIT_CASE(1)
    SPLIT_CASE(4)
    SPLIT_CASE(9)
    SPLIT_CASE(16)
    SPLIT_CASE(25)
#undef SPLIT_CASE
  }
  return check_launch("compute_sh_backward_views_split");
}

extern "C" int gsplat_compute_sh_backward_split(int num_points, int degree, int degrees_to_use,
                                                const float *viewdirs, const float *v_colors,
                                                float *v_dc, float *v_rest, void *stream) {
  if (num_points < 0 || degree < 0 || degree > 4 || degrees_to_use < 0 ||
      degrees_to_use > degree || (num_points > 0 && (!v_dc || (degree > 0 && !v_rest)))) {
    set_error("compute_sh_backward_split: bad args (N=%d degree=%d degrees_to_use=%d)",
              num_points, degree, degrees_to_use);
    return 1;
  }
  if (num_points == 0) return 0;
  const int K = num_bases(degree);
  const int thr = sh_threads(K);
  dim3 grid(cdiv(num_points, thr)), block(thr);
  size_t smem = (size_t)thr * sh_row_pitch(K) * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
#define SPLIT_CASE(KK)                                                                     \
  case KK:                                                                                 \
    hipLaunchKernelGGL((sh_bwd_kernel<KK, true>), grid, block, smem, st, num_points,        \
                       degrees_to_use, viewdirs, v_colors, v_dc, v_rest);                   \
    break;
    SPLIT_CASE(1)
    SPLIT_CASE(4)
    SPLIT_CASE(9)
    SPLIT_CASE(16)
    SPLIT_CASE(25)
#undef SPLIT_CASE
  }
  return check_launch("compute_sh_backward_split");
}

extern "C" int gsplat_compute_sh_backward_view_table(int num_points, int degree,
                                                     int degrees_to_use, int num_views,
                                                     const float *means3d,
                                                     const float *const *records,
                                                     const long long *capacities, float *v_dc,
                                                     float *v_rest, void *stream) {
  if (num_points < 0 || degree < 0 || degree > 4 || degrees_to_use < 0 ||
      degrees_to_use > degree || num_views < 1 || num_views > XS_MAX_VIEWS || !records ||
      !capacities || (num_points > 0 && (!means3d || !v_dc || (degree > 0 && !v_rest)))) {
    set_error("compute_sh_backward_view_table: bad args (N=%d degree=%d degrees_to_use=%d "
              "views=%d, at most %d)", num_points, degree, degrees_to_use, num_views,
              XS_MAX_VIEWS);
    return 1;
  }
  ViewTable tab{};
  for (int r = 0; r < num_views; ++r) {
    if (!records[r] || capacities[r] > num_points) {
      set_error("compute_sh_backward_view_table: record %d is NULL or its capacity %lld exceeds "
                "N=%d", r, capacities[r], num_points);
      return 1;
    }
    tab.rec[r] = records[r];
    tab.cap[r] = capacities[r];
  }
  if (num_points == 0) return 0;
  const int K = num_bases(degree);
  const int thr = sh_threads(K);
  dim3 grid(cdiv(num_points, thr)), block(thr);
  size_t smem = (size_t)thr * sh_row_pitch(K) * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  SH_DISPATCH(sh_bwd_table_kernel, num_points, degrees_to_use, num_views, means3d, tab, v_dc,
              v_rest);
  return check_launch("compute_sh_backward_view_table");
}

extern "C" int gsplat_compute_sh_backward_view_table_adam(
    int num_points, int degree, int degrees_to_use, int num_views, const float *means3d,
    const float *const *records, const long long *capacities, float *features_dc,
    float *features_rest, float *exp_avg_dc, float *exp_avg_sq_dc, float *exp_avg_rest,
    float *exp_avg_sq_rest, float lr_dc, float lr_rest, int step, float beta1, float beta2,
    float eps, void *stream) {
  if (num_points < 0 || degree < 0 || degree > 4 || degrees_to_use < 0 ||
      degrees_to_use > degree || num_views < 1 || num_views > XS_MAX_VIEWS || !records ||
      !capacities || step < 1 || !(beta1 > 0.5f && beta1 < 1.f) || !(beta2 >= 0.f && beta2 < 1.f) ||
      (num_points > 0 && (!means3d || !features_dc || !exp_avg_dc || !exp_avg_sq_dc ||
                          (degree > 0 && (!features_rest || !exp_avg_rest || !exp_avg_sq_rest))))) {
    set_error("compute_sh_backward_view_table_adam: bad args (N=%d degree=%d degrees_to_use=%d "
              "views=%d, at most %d, step=%d beta1=%g beta2=%g)", num_points, degree,
              degrees_to_use, num_views, XS_MAX_VIEWS, step, (double)beta1, (double)beta2);
    return 1;
  }
  ViewTable tab{};
  for (int r = 0; r < num_views; ++r) {
    if (!records[r] || capacities[r] > num_points) {
      set_error("compute_sh_backward_view_table_adam: record %d is NULL or its capacity %lld "
                "exceeds N=%d", r, capacities[r], num_points);
      return 1;
    }
    tab.rec[r] = records[r];
    tab.cap[r] = capacities[r];
  }
  if (num_points == 0) return 0;
  // torch non-capturable Adam: bias corrections in double on the host (as gsplat_adam_step)
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  ShAdam o{};
  o.p[0] = features_dc;
  o.m[0] = exp_avg_dc;
  o.v[0] = exp_avg_sq_dc;
  o.p[1] = features_rest;
  o.m[1] = exp_avg_rest;
  o.v[1] = exp_avg_sq_rest;
  o.ss[0] = (float)(lr_dc / bc1);
  o.ss[1] = (float)(lr_rest / bc1);
  o.bc2s = (float)sqrt(bc2);
  o.beta1 = beta1;
  o.beta2 = beta2;
  o.eps = eps;
  const int K = num_bases(degree);
  const int thr = sh_threads(K);
  dim3 grid(cdiv(num_points, thr)), block(thr);
  size_t smem = (size_t)thr * sh_row_pitch(K) * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
#define ADAM_CASE(KK)                                                                        \
  case KK:                                                                                   \
    hipLaunchKernelGGL((sh_bwd_table_kernel<KK, true>), grid, block, smem, st, num_points,    \
                       degrees_to_use, num_views, means3d, tab, nullptr, nullptr, o);        \
    break;
    ADAM_CASE(1)
    ADAM_CASE(4)
    ADAM_CASE(9)
    ADAM_CASE(16)
    ADAM_CASE(25)
#undef ADAM_CASE
  }
  return check_launch("compute_sh_backward_view_table_adam");
}
