// project.hip -- 3D->2D Gaussian projection, forward and backward, for gfx950.
//
// Replaces gsplat 0.1.2.1 _C.project_gaussians_forward/backward (called from
// /root/reference/gaussctrl/gc_model.py:174-188).  One lane per Gaussian; the per-Gaussian
// work is ~300 VALU ops against 40 B in / 56 B out, so the kernel is HBM-bound and the
// launch is sized for >> 256 CUs at the 100k-5M Gaussians of interest.
//
// BUILT WITH -ffp-contract=off: radii, tile bounding boxes and num_tiles_hit must agree
// bit for bit with the CPU restatement (oracle/gsplat_oracle.c), so every fp32 operation
// here has the same operands and order as there (no FMA contraction, correctly rounded
// '/' and sqrtf -- hipcc's default -fhip-fp32-correctly-rounded-divide-sqrt).
#include "project_math.h"

namespace gs {
namespace {

__global__ __launch_bounds__(256) void project_fwd_kernel(
    int n, const float *__restrict__ means, const float *__restrict__ scales,
    const float *__restrict__ quats, const float *__restrict__ viewmat,
    const float *__restrict__ projmat, ProjParams pp, float *__restrict__ cov3d,
    float *__restrict__ xys, float *__restrict__ depths, int *__restrict__ radii,
    float *__restrict__ conics, int *__restrict__ num_tiles_hit, BinKeys bin) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Cam cam;
  load_cam(cam, viewmat, projmat);
  // Culled Gaussians keep zeros in every output gsplat zero-initialises; the outputs are
  // written unconditionally here so the caller may pass uninitialised memory.
  ProjOut o;
  project_one(cam, pp, means[3 * i], means[3 * i + 1], means[3 * i + 2], scales[3 * i],
              scales[3 * i + 1], scales[3 * i + 2], quats[4 * i], quats[4 * i + 1],
              quats[4 * i + 2], quats[4 * i + 3], o);
#pragma unroll
  for (int k = 0; k < 6; ++k) cov3d[6 * i + k] = o.cov[k];
  conics[3 * i] = o.con[0];
  conics[3 * i + 1] = o.con[1];
  conics[3 * i + 2] = o.con[2];
  xys[2 * i] = o.xy[0];
  xys[2 * i + 1] = o.xy[1];
  depths[i] = o.depth;
  radii[i] = o.radius;
  num_tiles_hit[i] = o.tiles;
  if (bin.keys) {  // the binning's depth-sort inputs (binning.hip depth_keys_kernel's outputs)
    const bool vis = o.radius > 0;
    bin.keys[i] = vis ? __float_as_uint(o.depth) : 0xFFFFFFFFu;
    bin.vals[i] = (uint32_t)i;
    const int c = vis ? o.tiles : 0;
    uint4 q = {c > 0 ? (uint32_t)c : 0u, 0u, 0u, 0u};
    if (c > 0) {
      int x0, x1, y0, y1;
      tile_bbox(o.xy[0], o.xy[1], (float)o.radius, pp.tbx, pp.tby, x0, x1, y0, y1);
      q.y = (uint32_t)x0 | ((uint32_t)y0 << 16);
      q.z = (uint32_t)x1 | ((uint32_t)y1 << 16);
    }
    bin.rec[i] = q;
  }
}

__global__ __launch_bounds__(256) void project_bwd_kernel(
    int n, const float *__restrict__ means, const float *__restrict__ scales,
    const float *__restrict__ quats, const float *__restrict__ viewmat,
    const float *__restrict__ projmat, ProjParams pp, const float *__restrict__ cov3d,
    const int *__restrict__ radii, const float *__restrict__ conics,
    const float *__restrict__ v_xy, const float *__restrict__ v_depth,
    const float *__restrict__ v_conic, float *__restrict__ v_cov2d_out,
    float *__restrict__ v_cov3d_out, float *__restrict__ v_mean_out,
    float *__restrict__ v_scale_out, float *__restrict__ v_quat_out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ProjGrad g = {};
  if (radii[i] > 0) {
    Cam cam;
    load_cam(cam, viewmat, projmat);
    const float cv[6] = {cov3d[6 * i], cov3d[6 * i + 1], cov3d[6 * i + 2],
                         cov3d[6 * i + 3], cov3d[6 * i + 4], cov3d[6 * i + 5]};
    project_backward_one(cam, pp, means[3 * i], means[3 * i + 1], means[3 * i + 2],
                         scales[3 * i], scales[3 * i + 1], scales[3 * i + 2], quats[4 * i],
                         quats[4 * i + 1], quats[4 * i + 2], quats[4 * i + 3], cv,
                         conics[3 * i], conics[3 * i + 1], conics[3 * i + 2], v_xy[2 * i],
                         v_xy[2 * i + 1], v_depth ? v_depth[i] : 0.f, v_conic[3 * i],
                         v_conic[3 * i + 1], v_conic[3 * i + 2], g);
  }
  if (v_cov2d_out) {  // intermediate gradients: optional (the autograd wrapper drops them)
#pragma unroll
    for (int k = 0; k < 3; ++k) v_cov2d_out[3 * i + k] = g.vc2[k];
  }
  if (v_cov3d_out) {
#pragma unroll
    for (int k = 0; k < 6; ++k) v_cov3d_out[6 * i + k] = g.vc3[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) v_mean_out[3 * i + k] = g.vmean[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) v_scale_out[3 * i + k] = g.vscale[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) v_quat_out[4 * i + k] = g.vquat[k];
}

__global__ __launch_bounds__(256) void cov2d_bounds_kernel(int n, const float *__restrict__ cov2d,
                                                           float *__restrict__ conics,
                                                           float *__restrict__ radii) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = cov2d[3 * i], b = cov2d[3 * i + 1], c = cov2d[3 * i + 2];
  float det = a * c - b * b;
  float o0 = 0.f, o1 = 0.f, o2 = 0.f, r = 0.f;
  if (det != 0.f) {
    float inv_det = 1.f / det;
    o0 = c * inv_det;
    o1 = -b * inv_det;
    o2 = a * inv_det;
    float bb = 0.5f * (a + c);
    float v1 = bb + sqrtf(fmaxf(0.1f, bb * bb - det));
    float v2 = bb - sqrtf(fmaxf(0.1f, bb * bb - det));
    r = ceilf(3.f * sqrtf(fmaxf(v1, v2)));
  }
  conics[3 * i] = o0;
  conics[3 * i + 1] = o1;
  conics[3 * i + 2] = o2;
  radii[i] = r;
}

}  // namespace
}  // namespace gs

using namespace gs;

static int project_forward_impl(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, int tile_bounds_x, int tile_bounds_y,
    float clip_thresh, float *cov3d, float *xys, float *depths, int32_t *radii,
    float *conics, int32_t *num_tiles_hit, void *workspace1, size_t workspace1_bytes,
    void *stream, const char *who) {
  if (num_points < 0 || img_height <= 0 || img_width <= 0 || tile_bounds_x <= 0 ||
      tile_bounds_y <= 0) {
    set_error("%s: bad sizes (N=%d H=%d W=%d tiles=%dx%d)", who, num_points, img_height,
              img_width, tile_bounds_x, tile_bounds_y);
    return 1;
  }
  BinKeys bin = {nullptr, nullptr, nullptr, 0};
  if (workspace1) {
    bin = bin_keys_view(workspace1, num_points);
    if (workspace1_bytes < bin.bytes) {
      set_error("%s: workspace %zu < %zu bytes (gsplat_bin_count_workspace_size)", who,
                workspace1_bytes, bin.bytes);
      return 1;
    }
  }
  if (num_points == 0) return 0;
  const ProjParams pp = make_proj_params(fx, fy, cx, cy, glob_scale, clip_thresh, img_height,
                                         img_width, tile_bounds_x, tile_bounds_y);
  hipLaunchKernelGGL(project_fwd_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0,
                     (hipStream_t)stream, num_points, means3d, scales, quats, viewmat, projmat,
                     pp, cov3d, xys, depths, radii, conics, num_tiles_hit, bin);
  return check_launch(who);
}

extern "C" int gsplat_project_gaussians_forward(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, int tile_bounds_x, int tile_bounds_y,
    float clip_thresh, float *cov3d, float *xys, float *depths, int32_t *radii,
    float *conics, int32_t *num_tiles_hit, void *stream) {
  return project_forward_impl(num_points, means3d, scales, glob_scale, quats, viewmat, projmat,
                              fx, fy, cx, cy, img_height, img_width, tile_bounds_x,
                              tile_bounds_y, clip_thresh, cov3d, xys, depths, radii, conics,
                              num_tiles_hit, nullptr, 0, stream, "project_gaussians_forward");
}

extern "C" int gsplat_project_gaussians_forward_binned(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, int tile_bounds_x, int tile_bounds_y,
    float clip_thresh, float *cov3d, float *xys, float *depths, int32_t *radii,
    float *conics, int32_t *num_tiles_hit, void *workspace1, size_t workspace1_bytes,
    void *stream) {
  if (!workspace1) {
    set_error("project_gaussians_forward_binned: no workspace");
    return 1;
  }
  return project_forward_impl(num_points, means3d, scales, glob_scale, quats, viewmat, projmat,
                              fx, fy, cx, cy, img_height, img_width, tile_bounds_x,
                              tile_bounds_y, clip_thresh, cov3d, xys, depths, radii, conics,
                              num_tiles_hit, workspace1, workspace1_bytes, stream,
                              "project_gaussians_forward_binned");
}

extern "C" int gsplat_project_gaussians_backward(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, const float *cov3d,
    const int32_t *radii, const float *conics, const float *v_xy, const float *v_depth,
    const float *v_conic, float *v_cov2d, float *v_cov3d, float *v_mean3d, float *v_scale,
    float *v_quat, void *stream) {
  if (num_points < 0 || img_height <= 0 || img_width <= 0) {
    set_error("project_gaussians_backward: bad sizes");
    return 1;
  }
  if (num_points == 0) return 0;
  const ProjParams pp = make_proj_params(fx, fy, cx, cy, glob_scale, 0.f, img_height, img_width,
                                         1, 1);
  hipLaunchKernelGGL(project_bwd_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0,
                     (hipStream_t)stream, num_points, means3d, scales, quats, viewmat, projmat,
                     pp, cov3d, radii, conics, v_xy, v_depth, v_conic, v_cov2d, v_cov3d,
                     v_mean3d, v_scale, v_quat);
  return check_launch("project_gaussians_backward");
}

extern "C" int gsplat_compute_cov2d_bounds(int num_points, const float *covs2d, float *conics,
                                           float *radii, void *stream) {
  if (num_points < 0) {
    set_error("compute_cov2d_bounds: bad size");
    return 1;
  }
  if (num_points == 0) return 0;
  hipLaunchKernelGGL(cov2d_bounds_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0,
                     (hipStream_t)stream, num_points, covs2d, conics, radii);
  return check_launch("compute_cov2d_bounds");
}
