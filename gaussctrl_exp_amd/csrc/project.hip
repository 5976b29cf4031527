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
#include "common.h"

namespace gs {
namespace {

struct M3 {
  float m[9];  // row-major
};

__device__ __forceinline__ M3 mul(const M3 &a, const M3 &b) {
  M3 t;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      t.m[r * 3 + c] = a.m[r * 3 + 0] * b.m[0 * 3 + c] + a.m[r * 3 + 1] * b.m[1 * 3 + c] +
                       a.m[r * 3 + 2] * b.m[2 * 3 + c];
  return t;
}

__device__ __forceinline__ M3 transpose(const M3 &a) {
  M3 t;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) t.m[c * 3 + r] = a.m[r * 3 + c];
  return t;
}

__device__ __forceinline__ M3 quat_to_rotmat(float q0, float q1, float q2, float q3) {
  float s = 1.f / sqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
  float w = q0 * s, x = q1 * s, y = q2 * s, z = q3 * s;
  M3 R;
  R.m[0] = 1.f - 2.f * (y * y + z * z);
  R.m[1] = 2.f * (x * y - w * z);
  R.m[2] = 2.f * (x * z + w * y);
  R.m[3] = 2.f * (x * y + w * z);
  R.m[4] = 1.f - 2.f * (x * x + z * z);
  R.m[5] = 2.f * (y * z - w * x);
  R.m[6] = 2.f * (x * z - w * y);
  R.m[7] = 2.f * (y * z + w * x);
  R.m[8] = 1.f - 2.f * (x * x + y * y);
  return R;
}

__device__ __forceinline__ M3 diag3(float a, float b, float c) {
  M3 S;
#pragma unroll
  for (int k = 0; k < 9; ++k) S.m[k] = 0.f;
  S.m[0] = a;
  S.m[4] = b;
  S.m[8] = c;
  return S;
}

struct Cam {
  float vm[12];  // viewmat rows 0..2
  float pm[16];  // projmat
};

__device__ __forceinline__ void load_cam(Cam &c, const float *__restrict__ viewmat,
                                         const float *__restrict__ projmat) {
#pragma unroll
  for (int k = 0; k < 12; ++k) c.vm[k] = viewmat[k];
#pragma unroll
  for (int k = 0; k < 16; ++k) c.pm[k] = projmat[k];
}

// gsplat tile bbox (helpers.cuh get_tile_bbox / get_bbox)
__device__ __forceinline__ void tile_bbox(float x, float y, float radius, int tbx, int tby,
                                          int &x0, int &x1, int &y0, int &y1) {
  float cx = x / (float)GS_BLOCK, cy = y / (float)GS_BLOCK;
  float rx = radius / (float)GS_BLOCK, ry = radius / (float)GS_BLOCK;
  int a;
  a = f2i_sat(cx - rx); a = a < 0 ? 0 : a; x0 = a < tbx ? a : tbx;
  a = f2i_sat(cx + rx + 1.f); a = a < 0 ? 0 : a; x1 = a < tbx ? a : tbx;
  a = f2i_sat(cy - ry); a = a < 0 ? 0 : a; y0 = a < tby ? a : tby;
  a = f2i_sat(cy + ry + 1.f); a = a < 0 ? 0 : a; y1 = a < tby ? a : tby;
}

__global__ __launch_bounds__(256) void project_fwd_kernel(
    int n, const float *__restrict__ means, const float *__restrict__ scales, float glob_scale,
    const float *__restrict__ quats, const float *__restrict__ viewmat,
    const float *__restrict__ projmat, float fx, float fy, float cx, float cy, int H, int W,
    int tbx, int tby, float tan_fovx, float tan_fovy, float clip_thresh,
    float *__restrict__ cov3d, float *__restrict__ xys, float *__restrict__ depths,
    int *__restrict__ radii, float *__restrict__ conics, int *__restrict__ num_tiles_hit) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Cam cam;
  load_cam(cam, viewmat, projmat);
  const float *vm = cam.vm;
  float p0 = means[3 * i], p1 = means[3 * i + 1], p2 = means[3 * i + 2];

  // Culled Gaussians keep zeros in every output gsplat zero-initialises; the outputs
  // are written unconditionally here so the caller may pass uninitialised memory.
  float o_cov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float o_con[3] = {0.f, 0.f, 0.f};
  float o_xy[2] = {0.f, 0.f};
  float o_depth = 0.f;
  int o_radius = 0, o_tiles = 0;

  float pz = vm[8] * p0 + vm[9] * p1 + vm[10] * p2 + vm[11];
  if (pz > clip_thresh) {
    // scale_rot_to_cov3d
    M3 R = quat_to_rotmat(quats[4 * i], quats[4 * i + 1], quats[4 * i + 2], quats[4 * i + 3]);
    M3 S = diag3(glob_scale * scales[3 * i], glob_scale * scales[3 * i + 1],
                 glob_scale * scales[3 * i + 2]);
    M3 M = mul(R, S);
    M3 V = mul(M, transpose(M));
    o_cov[0] = V.m[0];
    o_cov[1] = V.m[3];
    o_cov[2] = V.m[6];
    o_cov[3] = V.m[4];
    o_cov[4] = V.m[7];
    o_cov[5] = V.m[8];
    // project_cov3d_ewa
    float tx = vm[0] * p0 + vm[1] * p1 + vm[2] * p2 + vm[3];
    float ty = vm[4] * p0 + vm[5] * p1 + vm[6] * p2 + vm[7];
    float tz = vm[8] * p0 + vm[9] * p1 + vm[10] * p2 + vm[11];
    float lim_x = 1.3f * tan_fovx, lim_y = 1.3f * tan_fovy;
    tx = tz * fminf(lim_x, fmaxf(-lim_x, tx / tz));
    ty = tz * fminf(lim_y, fmaxf(-lim_y, ty / tz));
    float rz = 1.f / tz;
    float rz2 = rz * rz;
    M3 J = {{fx * rz, 0.f, -fx * tx * rz2, 0.f, fy * rz, -fy * ty * rz2, 0.f, 0.f, 0.f}};
    M3 Wm = {{vm[0], vm[1], vm[2], vm[4], vm[5], vm[6], vm[8], vm[9], vm[10]}};
    M3 Vs = {{o_cov[0], o_cov[1], o_cov[2], o_cov[1], o_cov[3], o_cov[4], o_cov[2], o_cov[4],
              o_cov[5]}};
    M3 T = mul(J, Wm);
    M3 C = mul(mul(T, Vs), transpose(T));
    float c00 = C.m[0] + 0.3f, c01 = C.m[3], c11 = C.m[4] + 0.3f;
    // compute_cov2d_bounds
    float det = c00 * c11 - c01 * c01;
    if (det != 0.f) {
      float inv_det = 1.f / det;
      o_con[0] = c11 * inv_det;
      o_con[1] = -c01 * inv_det;
      o_con[2] = c00 * inv_det;
      float b = 0.5f * (c00 + c11);
      float v1 = b + sqrtf(fmaxf(0.1f, b * b - det));
      float v2 = b - sqrtf(fmaxf(0.1f, b * b - det));
      float radius = ceilf(3.f * sqrtf(fmaxf(v1, v2)));
      // project_pix
      const float *P = cam.pm;
      float hx = P[0] * p0 + P[1] * p1 + P[2] * p2 + P[3];
      float hy = P[4] * p0 + P[5] * p1 + P[6] * p2 + P[7];
      float hw = P[12] * p0 + P[13] * p1 + P[14] * p2 + P[15];
      float rw = 1.f / (hw + 1e-6f);
      float nx = hx * rw, ny = hy * rw;
      float x = 0.5f * (float)W * nx + cx - 0.5f;
      float y = 0.5f * (float)H * ny + cy - 0.5f;
      int x0, x1, y0, y1;
      tile_bbox(x, y, radius, tbx, tby, x0, x1, y0, y1);
      int area = (x1 - x0) * (y1 - y0);
      if (area > 0) {
        o_tiles = area;
        o_depth = pz;
        o_radius = f2i_sat(radius);
        o_xy[0] = x;
        o_xy[1] = y;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) cov3d[6 * i + k] = o_cov[k];
  conics[3 * i] = o_con[0];
  conics[3 * i + 1] = o_con[1];
  conics[3 * i + 2] = o_con[2];
  xys[2 * i] = o_xy[0];
  xys[2 * i + 1] = o_xy[1];
  depths[i] = o_depth;
  radii[i] = o_radius;
  num_tiles_hit[i] = o_tiles;
}

__global__ __launch_bounds__(256) void project_bwd_kernel(
    int n, const float *__restrict__ means, const float *__restrict__ scales, float glob_scale,
    const float *__restrict__ quats, const float *__restrict__ viewmat,
    const float *__restrict__ projmat, float fx, float fy, int H, int W,
    const float *__restrict__ cov3d, const int *__restrict__ radii,
    const float *__restrict__ conics, const float *__restrict__ v_xy,
    const float *__restrict__ v_depth, const float *__restrict__ v_conic,
    float *__restrict__ v_cov2d_out, float *__restrict__ v_cov3d_out,
    float *__restrict__ v_mean_out, float *__restrict__ v_scale_out,
    float *__restrict__ v_quat_out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float vc2[3] = {0.f, 0.f, 0.f};
  float vc3[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float vmean[3] = {0.f, 0.f, 0.f};
  float vscale[3] = {0.f, 0.f, 0.f};
  float vquat[4] = {0.f, 0.f, 0.f, 0.f};
  if (radii[i] > 0) {
    Cam cam;
    load_cam(cam, viewmat, projmat);
    const float *vm = cam.vm;
    const float *P = cam.pm;
    float p0 = means[3 * i], p1 = means[3 * i + 1], p2 = means[3 * i + 2];
    // project_pix_vjp (w-derivative dropped)
    {
      float hw = P[12] * p0 + P[13] * p1 + P[14] * p2 + P[15];
      float rw = 1.f / (hw + 1e-6f);
      float vnx = 0.5f * (float)W * v_xy[2 * i];
      float vny = 0.5f * (float)H * v_xy[2 * i + 1];
      float vpx = vnx * rw, vpy = vny * rw, vpz = 0.f;
      vmean[0] = P[0] * vpx + P[4] * vpy + P[8] * vpz;
      vmean[1] = P[1] * vpx + P[5] * vpy + P[9] * vpz;
      vmean[2] = P[2] * vpx + P[6] * vpy + P[10] * vpz;
    }
    float vz = v_depth ? v_depth[i] : 0.f;
    vmean[0] += vm[8] * vz;
    vmean[1] += vm[9] * vz;
    vmean[2] += vm[10] * vz;
    // cov2d_to_conic_vjp
    {
      float a = conics[3 * i], b = conics[3 * i + 1], c = conics[3 * i + 2];
      float ga = v_conic[3 * i], gb = v_conic[3 * i + 1], gc = v_conic[3 * i + 2];
      float xg00 = a * ga + b * gb, xg01 = a * gb + b * gc;
      float xg10 = b * ga + c * gb, xg11 = b * gb + c * gc;
      float s00 = xg00 * a + xg01 * b, s01 = xg00 * b + xg01 * c;
      float s10 = xg10 * a + xg11 * b, s11 = xg10 * b + xg11 * c;
      vc2[0] = -s00;
      vc2[1] = -s10 + -s01;
      vc2[2] = -s11;
    }
    // project_cov3d_ewa_vjp (no fov clamp)
    {
      M3 Wm = {{vm[0], vm[1], vm[2], vm[4], vm[5], vm[6], vm[8], vm[9], vm[10]}};
      float tx = vm[0] * p0 + vm[1] * p1 + vm[2] * p2 + vm[3];
      float ty = vm[4] * p0 + vm[5] * p1 + vm[6] * p2 + vm[7];
      float tz = vm[8] * p0 + vm[9] * p1 + vm[10] * p2 + vm[11];
      float rz = 1.f / tz;
      float rz2 = rz * rz;
      float rz3 = rz2 * rz;
      M3 J = {{fx * rz, 0.f, -fx * tx * rz2, 0.f, fy * rz, -fy * ty * rz2, 0.f, 0.f, 0.f}};
      const float *cv = cov3d + 6 * i;
      M3 V = {{cv[0], cv[1], cv[2], cv[1], cv[3], cv[4], cv[2], cv[4], cv[5]}};
      M3 G = {{vc2[0], 0.5f * vc2[1], 0.f, 0.5f * vc2[1], vc2[2], 0.f, 0.f, 0.f, 0.f}};
      M3 T = mul(J, Wm);
      M3 Tt = transpose(T);
      M3 vV = mul(mul(Tt, G), T);
      M3 vT1 = mul(mul(G, T), transpose(V));
      M3 vT2 = mul(mul(transpose(G), T), V);
      M3 vT;
#pragma unroll
      for (int k = 0; k < 9; ++k) vT.m[k] = vT1.m[k] + vT2.m[k];
      vc3[0] = vV.m[0];
      vc3[1] = vV.m[3] + vV.m[1];
      vc3[2] = vV.m[6] + vV.m[2];
      vc3[3] = vV.m[4];
      vc3[4] = vV.m[7] + vV.m[5];
      vc3[5] = vV.m[8];
      M3 vJ = mul(vT, transpose(Wm));
      float vJ20 = vJ.m[2], vJ21 = vJ.m[5], vJ00 = vJ.m[0], vJ11 = vJ.m[4];
      float vt0 = -fx * rz2 * vJ20;
      float vt1 = -fy * rz2 * vJ21;
      float vt2 = -fx * rz2 * vJ00 + 2.f * fx * tx * rz3 * vJ20 - fy * rz2 * vJ11 +
                  2.f * fy * ty * rz3 * vJ21;
      vmean[0] += vt0 * Wm.m[0] + vt1 * Wm.m[3] + vt2 * Wm.m[6];
      vmean[1] += vt0 * Wm.m[1] + vt1 * Wm.m[4] + vt2 * Wm.m[7];
      vmean[2] += vt0 * Wm.m[2] + vt1 * Wm.m[5] + vt2 * Wm.m[8];
    }
    // scale_rot_to_cov3d_vjp + quat_to_rotmat_vjp
    {
      float q0 = quats[4 * i], q1 = quats[4 * i + 1], q2 = quats[4 * i + 2], q3 = quats[4 * i + 3];
      M3 vV = {{vc3[0], 0.5f * vc3[1], 0.5f * vc3[2], 0.5f * vc3[1], vc3[3], 0.5f * vc3[4],
                0.5f * vc3[2], 0.5f * vc3[4], vc3[5]}};
      M3 R = quat_to_rotmat(q0, q1, q2, q3);
      M3 S = diag3(glob_scale * scales[3 * i], glob_scale * scales[3 * i + 1],
                   glob_scale * scales[3 * i + 2]);
      M3 M = mul(R, S);
      M3 vM = mul(vV, M);
#pragma unroll
      for (int k = 0; k < 9; ++k) vM.m[k] = 2.f * vM.m[k];
#pragma unroll
      for (int c = 0; c < 3; ++c)
        vscale[c] = (R.m[0 * 3 + c] * vM.m[0 * 3 + c] + R.m[1 * 3 + c] * vM.m[1 * 3 + c] +
                     R.m[2 * 3 + c] * vM.m[2 * 3 + c]) *
                    glob_scale;
      M3 vRm = mul(vM, S);
      const float *vR = vRm.m;
      float s = 1.f / sqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
      float w = q0 * s, x = q1 * s, y = q2 * s, z = q3 * s;
#define GR(c, r) vR[(r) * 3 + (c)]
      vquat[0] = 2.f * (x * (GR(1, 2) - GR(2, 1)) + y * (GR(2, 0) - GR(0, 2)) +
                        z * (GR(0, 1) - GR(1, 0)));
      vquat[1] = 2.f * (-2.f * x * (GR(1, 1) + GR(2, 2)) + y * (GR(0, 1) + GR(1, 0)) +
                        z * (GR(0, 2) + GR(2, 0)) + w * (GR(1, 2) - GR(2, 1)));
      vquat[2] = 2.f * (x * (GR(0, 1) + GR(1, 0)) - 2.f * y * (GR(0, 0) + GR(2, 2)) +
                        z * (GR(1, 2) + GR(2, 1)) + w * (GR(2, 0) - GR(0, 2)));
      vquat[3] = 2.f * (x * (GR(0, 2) + GR(2, 0)) + y * (GR(1, 2) + GR(2, 1)) -
                        2.f * z * (GR(0, 0) + GR(1, 1)) + w * (GR(0, 1) - GR(1, 0)));
#undef GR
    }
  }
  if (v_cov2d_out) {  // intermediate gradients: optional (the autograd wrapper drops them)
#pragma unroll
    for (int k = 0; k < 3; ++k) v_cov2d_out[3 * i + k] = vc2[k];
  }
  if (v_cov3d_out) {
#pragma unroll
    for (int k = 0; k < 6; ++k) v_cov3d_out[6 * i + k] = vc3[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) v_mean_out[3 * i + k] = vmean[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) v_scale_out[3 * i + k] = vscale[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) v_quat_out[4 * i + k] = vquat[k];
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

extern "C" int gsplat_project_gaussians_forward(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, int tile_bounds_x, int tile_bounds_y,
    float clip_thresh, float *cov3d, float *xys, float *depths, int32_t *radii,
    float *conics, int32_t *num_tiles_hit, void *stream) {
  if (num_points < 0 || img_height <= 0 || img_width <= 0 || tile_bounds_x <= 0 ||
      tile_bounds_y <= 0) {
    set_error("project_gaussians_forward: bad sizes (N=%d H=%d W=%d tiles=%dx%d)", num_points,
              img_height, img_width, tile_bounds_x, tile_bounds_y);
    return 1;
  }
  if (num_points == 0) return 0;
  // gsplat computes tan_fov = 0.5 * img_size / f with a double literal.
  float tan_fovx = (float)(0.5 * (double)img_width / (double)fx);
  float tan_fovy = (float)(0.5 * (double)img_height / (double)fy);
  hipLaunchKernelGGL(project_fwd_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0,
                     (hipStream_t)stream, num_points, means3d, scales, glob_scale, quats, viewmat,
                     projmat, fx, fy, cx, cy, img_height, img_width, tile_bounds_x, tile_bounds_y,
                     tan_fovx, tan_fovy, clip_thresh, cov3d, xys, depths, radii, conics,
                     num_tiles_hit);
  return check_launch("project_gaussians_forward");
}

extern "C" int gsplat_project_gaussians_backward(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, const float *cov3d,
    const int32_t *radii, const float *conics, const float *v_xy, const float *v_depth,
    const float *v_conic, float *v_cov2d, float *v_cov3d, float *v_mean3d, float *v_scale,
    float *v_quat, void *stream) {
  (void)cx;
  (void)cy;
  if (num_points < 0 || img_height <= 0 || img_width <= 0) {
    set_error("project_gaussians_backward: bad sizes");
    return 1;
  }
  if (num_points == 0) return 0;
  hipLaunchKernelGGL(project_bwd_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0,
                     (hipStream_t)stream, num_points, means3d, scales, glob_scale, quats, viewmat,
                     projmat, fx, fy, img_height, img_width, cov3d, radii, conics, v_xy, v_depth,
                     v_conic, v_cov2d, v_cov3d, v_mean3d, v_scale, v_quat);
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
