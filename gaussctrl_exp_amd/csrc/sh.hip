// sh.hip -- spherical-harmonics colour evaluation (forward / backward) for gfx950.
//
// Replaces gsplat 0.1.2.1 _C.compute_sh_forward/backward (sh.cuh), called from
// /root/reference/gaussctrl/gc_model.py:200.  The coefficient block is [N, K, 3] fp32
// (K = num_sh_bases(degree), 192 B per Gaussian at degree 3): the largest per-Gaussian
// stream of the whole path.  A lane-per-Gaussian load of it would stride 192 B per lane,
// so each 256-thread workgroup instead stages its 256 Gaussians' coefficient block through
// LDS with 16-byte, fully coalesced loads (forward) / stores (backward); the per-Gaussian
// arithmetic then reads its own row from LDS.
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

// Writes the block's cnt staged rows (LDS, pitch sh_row_pitch) to dst [cnt * K * 3] with
// 16-byte coalesced stores when dst is 16-byte aligned.
template <int K>
__device__ __forceinline__ void store_rows(const float *smem, int cnt, float *dst) {
  constexpr int ROW = K * 3;
  constexpr int ROWP = sh_row_pitch(K);
  constexpr int SH_THREADS = sh_threads(K);
  const int total = cnt * ROW;
  if ((((uintptr_t)dst) & 15) == 0) {
    const int nv = total >> 2;
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    for (int k = threadIdx.x; k < nv; k += SH_THREADS) {
      float4 v;
      v.x = smem[sh_lds_index<ROW, ROWP>(4 * k)];
      v.y = smem[sh_lds_index<ROW, ROWP>(4 * k + 1)];
      v.z = smem[sh_lds_index<ROW, ROWP>(4 * k + 2)];
      v.w = smem[sh_lds_index<ROW, ROWP>(4 * k + 3)];
      d4[k] = v;
    }
    for (int k = (nv << 2) + threadIdx.x; k < total; k += SH_THREADS)
      dst[k] = smem[sh_lds_index<ROW, ROWP>(k)];
  } else {
    for (int k = threadIdx.x; k < total; k += SH_THREADS)
      dst[k] = smem[sh_lds_index<ROW, ROWP>(k)];
  }
}

// Coefficient rows are K*3 floats; the block's slab [256*K*3] is copied with 16-byte
// vector loads when the slab start is 16-byte aligned, else with dword loads.
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
  const int total = cnt * ROW;
  const float *src = coeffs + g0 * ROW;
  if (ROW % 4 == 0 && cnt == SH_THREADS && (((uintptr_t)src) & 15) == 0) {
    // full block: all of this thread's ROW/4 16-byte loads are issued before any LDS write
    constexpr int PER = ROW % 4 == 0 ? ROW / 4 : 1;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    float4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) v[u] = s4[u * SH_THREADS + threadIdx.x];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int k = 4 * (u * SH_THREADS + threadIdx.x);
      smem[sh_lds_index<ROW, ROWP>(k)] = v[u].x;
      smem[sh_lds_index<ROW, ROWP>(k + 1)] = v[u].y;
      smem[sh_lds_index<ROW, ROWP>(k + 2)] = v[u].z;
      smem[sh_lds_index<ROW, ROWP>(k + 3)] = v[u].w;
    }
  } else if ((((uintptr_t)src) & 15) == 0) {
    const int nv = total >> 2;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    for (int k = threadIdx.x; k < nv; k += SH_THREADS) {
      const float4 v = s4[k];
      const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) smem[sh_lds_index<ROW, ROWP>(4 * k + u)] = e[u];
    }
    for (int k = (nv << 2) + threadIdx.x; k < total; k += SH_THREADS)
      smem[sh_lds_index<ROW, ROWP>(k)] = src[k];
  } else {
    for (int k = threadIdx.x; k < total; k += SH_THREADS)
      smem[sh_lds_index<ROW, ROWP>(k)] = src[k];
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= cnt) return;
  const long long g = g0 + t;
  float b[25];
  int nb = sh_basis(degrees_to_use, viewdirs[3 * g], viewdirs[3 * g + 1], viewdirs[3 * g + 2],
                    b);
  const float *co = smem + t * ROWP;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float acc = b[0] * co[c];
#pragma unroll
    for (int band = 1; band <= 4; ++band) {
      if ((band + 1) * (band + 1) > nb || (band + 1) * (band + 1) > K) break;
      float s = 0.f;
#pragma unroll
      for (int k = band * band; k < (band + 1) * (band + 1); ++k) s += b[k] * co[k * 3 + c];
      acc += s;
    }
    colors[3 * g + c] = acc;
  }
}

template <int K>
__global__ __launch_bounds__(256) void sh_bwd_kernel(int n, int degrees_to_use,
                                                             const float *__restrict__ viewdirs,
                                                             const float *__restrict__ v_colors,
                                                             float *__restrict__ v_coeffs) {
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
  store_rows<K>(smem, cnt, v_coeffs + g0 * ROW);
}

// Multi-view SH backward for data-parallel training: the coefficient
// gradient of one view is the rank-1 product Y(dir) (x) v_colors, and the direction is the
// (replicated) mean minus that view's camera centre, so the ranks exchange only v_colors
// (12 B per Gaussian) plus their camera centre, and every rank evaluates
//   v_coeffs[i] = sum_r Y(means[i] - campos_r) (x) v_colors_r[i]
// itself -- in view order, so every rank produces bit-identical gradients.
// views[r * view_stride + 3 i + c] = v_colors of view r; views[r * view_stride + 3 n + c] =
// camera centre of view r.
template <int K>
__global__ __launch_bounds__(256) void sh_bwd_views_kernel(int n, int degrees_to_use,
                                                           int num_views,
                                                           const float *__restrict__ means,
                                                           const float *__restrict__ views,
                                                           long long view_stride,
                                                           float *__restrict__ v_coeffs) {
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
  store_rows<K>(smem, cnt, v_coeffs + g0 * ROW);
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
