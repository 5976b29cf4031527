// project_math.h -- per-Gaussian projection arithmetic shared by project.hip (the gsplat
// project_gaussians kernels) and preprocess.hip (the fused caller-glue kernels).
//
// Restates gsplat 0.1.2.1 helpers.cuh / forward.cu project_gaussians_forward_kernel and
// backward.cu project_gaussians_backward_kernel.  Every
// translation unit that includes this header is built with -ffp-contract=off, so the
// operation order below is the oracle's (oracle/gsplat_oracle.c) bit for bit, and the fused
// and unfused paths produce identical projections from identical activated inputs.
#pragma once

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

// Camera-side constants of one projection call.
struct ProjParams {
  float fx, fy, cx, cy, glob_scale, tan_fovx, tan_fovy, clip_thresh;
  int H, W, tbx, tby;
  int quirks;  // GSPLAT_QUIRK_* bits (common.h), from gsplat_set_quirks at launch
};

// gsplat computes tan_fov = 0.5 * img_size / f with a double literal.
static inline ProjParams make_proj_params(float fx, float fy, float cx, float cy,
                                          float glob_scale, float clip_thresh, int H, int W,
                                          int tbx, int tby) {
  ProjParams pp;
  pp.fx = fx;
  pp.fy = fy;
  pp.cx = cx;
  pp.cy = cy;
  pp.glob_scale = glob_scale;
  pp.tan_fovx = (float)(0.5 * (double)W / (double)fx);
  pp.tan_fovy = (float)(0.5 * (double)H / (double)fy);
  pp.clip_thresh = clip_thresh;
  pp.quirks = g_quirks;
  pp.H = H;
  pp.W = W;
  pp.tbx = tbx;
  pp.tby = tby;
  return pp;
}

// scale_rot_to_cov3d: upper triangle [xx, xy, xz, yy, yz, zz] of R S S^T R^T.
__device__ __forceinline__ void cov3d_one(float glob_scale, float s0, float s1, float s2,
                                          float q0, float q1, float q2, float q3, float cov[6]) {
  M3 R = quat_to_rotmat(q0, q1, q2, q3);
  M3 S = diag3(glob_scale * s0, glob_scale * s1, glob_scale * s2);
  M3 M = mul(R, S);
  M3 V = mul(M, transpose(M));
  cov[0] = V.m[0];
  cov[1] = V.m[3];
  cov[2] = V.m[6];
  cov[3] = V.m[4];
  cov[4] = V.m[7];
  cov[5] = V.m[8];
}

// One Gaussian's forward projection outputs.  Culled Gaussians keep zeros in every output
// gsplat zero-initialises (cov3d / conics follow gsplat's write order).
struct ProjOut {
  float cov[6], con[3], xy[2], depth;
  int radius, tiles;
};

// gsplat project_gaussians_forward_kernel for one Gaussian: mean p, scale s, quaternion q.
__device__ __forceinline__ void project_one(const Cam &cam, const ProjParams &pp, float p0,
                                            float p1, float p2, float s0, float s1, float s2,
                                            float q0, float q1, float q2, float q3, ProjOut &o) {
  const float *vm = cam.vm;
#pragma unroll
  for (int k = 0; k < 6; ++k) o.cov[k] = 0.f;
  o.con[0] = o.con[1] = o.con[2] = 0.f;
  o.xy[0] = o.xy[1] = 0.f;
  o.depth = 0.f;
  o.radius = 0;
  o.tiles = 0;
  const float fx = pp.fx, fy = pp.fy;

  float pz = vm[8] * p0 + vm[9] * p1 + vm[10] * p2 + vm[11];
  if (!(pz > pp.clip_thresh)) return;
  cov3d_one(pp.glob_scale, s0, s1, s2, q0, q1, q2, q3, o.cov);
  // project_cov3d_ewa
  float tx = vm[0] * p0 + vm[1] * p1 + vm[2] * p2 + vm[3];
  float ty = vm[4] * p0 + vm[5] * p1 + vm[6] * p2 + vm[7];
  float tz = vm[8] * p0 + vm[9] * p1 + vm[10] * p2 + vm[11];
  float lim_x = 1.3f * pp.tan_fovx, lim_y = 1.3f * pp.tan_fovy;
  tx = tz * fminf(lim_x, fmaxf(-lim_x, tx / tz));
  ty = tz * fminf(lim_y, fmaxf(-lim_y, ty / tz));
  float rz = 1.f / tz;
  float rz2 = rz * rz;
  M3 J = {{fx * rz, 0.f, -fx * tx * rz2, 0.f, fy * rz, -fy * ty * rz2, 0.f, 0.f, 0.f}};
  M3 Wm = {{vm[0], vm[1], vm[2], vm[4], vm[5], vm[6], vm[8], vm[9], vm[10]}};
  M3 Vs = {{o.cov[0], o.cov[1], o.cov[2], o.cov[1], o.cov[3], o.cov[4], o.cov[2], o.cov[4],
            o.cov[5]}};
  M3 T = mul(J, Wm);
  M3 C = mul(mul(T, Vs), transpose(T));
  float c00 = C.m[0] + 0.3f, c01 = C.m[3], c11 = C.m[4] + 0.3f;
  // compute_cov2d_bounds
  float det = c00 * c11 - c01 * c01;
  if (det == 0.f) return;
  float inv_det = 1.f / det;
  o.con[0] = c11 * inv_det;
  o.con[1] = -c01 * inv_det;
  o.con[2] = c00 * inv_det;
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
  float x = 0.5f * (float)pp.W * nx + pp.cx - 0.5f;
  float y = 0.5f * (float)pp.H * ny + pp.cy - 0.5f;
  int x0, x1, y0, y1;
  tile_bbox(x, y, radius, pp.tbx, pp.tby, x0, x1, y0, y1);
  int area = (x1 - x0) * (y1 - y0);
  if (area > 0) {
    o.tiles = area;
    o.depth = pz;
    o.radius = f2i_sat(radius);
    o.xy[0] = x;
    o.xy[1] = y;
  }
}

// One Gaussian's projection gradients (gsplat project_gaussians_backward_kernel).
struct ProjGrad {
  float vc2[3], vc3[6], vmean[3], vscale[3], vquat[4];
};

// For radii > 0 only (the callers write zeros otherwise).  cv = the forward's cov3d,
// (a, b, c) the forward's conic, (vx, vy) / vz / (ga, gb, gc) the upstream xy / depth / conic
// gradients.
__device__ __forceinline__ void project_backward_one(const Cam &cam, const ProjParams &pp,
                                                     float p0, float p1, float p2, float s0,
                                                     float s1, float s2, float q0, float q1,
                                                     float q2, float q3, const float cv[6],
                                                     float a, float b, float c, float vx,
                                                     float vy, float vz, float ga, float gb,
                                                     float gc, ProjGrad &g) {
  const float *vm = cam.vm;
  const float *P = cam.pm;
  const float fx = pp.fx, fy = pp.fy, glob_scale = pp.glob_scale;
  // project_pix_vjp (w-derivative dropped)
  {
    float hw = P[12] * p0 + P[13] * p1 + P[14] * p2 + P[15];
    float rw = 1.f / (hw + 1e-6f);
    float vnx = 0.5f * (float)pp.W * vx;
    float vny = 0.5f * (float)pp.H * vy;
    float vpx = vnx * rw, vpy = vny * rw, vpz = 0.f;
    g.vmean[0] = P[0] * vpx + P[4] * vpy + P[8] * vpz;
    g.vmean[1] = P[1] * vpx + P[5] * vpy + P[9] * vpz;
    g.vmean[2] = P[2] * vpx + P[6] * vpy + P[10] * vpz;
  }
  g.vmean[0] += vm[8] * vz;
  g.vmean[1] += vm[9] * vz;
  g.vmean[2] += vm[10] * vz;
  // cov2d_to_conic_vjp: G = [[ga, gb], [gb, gc]] holds the gradient of each symmetric entry;
  // without the conic-half convention the upstream gb is d/d(conic.y) of both entries at once
  if (!(pp.quirks & GSPLAT_QUIRK_CONIC_HALF)) gb = 0.5f * gb;
  {
    float xg00 = a * ga + b * gb, xg01 = a * gb + b * gc;
    float xg10 = b * ga + c * gb, xg11 = b * gb + c * gc;
    float s00 = xg00 * a + xg01 * b, s01 = xg00 * b + xg01 * c;
    float s10 = xg10 * a + xg11 * b, s11 = xg10 * b + xg11 * c;
    g.vc2[0] = -s00;
    g.vc2[1] = -s10 + -s01;
    g.vc2[2] = -s11;
  }
  // project_cov3d_ewa_vjp (gsplat: no fov clamp; without that quirk, the
  // Jacobian of the clamped forward: t_x = t_z clamp(t_x / t_z) passes d/dt_x inside the
  // clamp and +-lim * d/dt_z outside)
  {
    M3 Wm = {{vm[0], vm[1], vm[2], vm[4], vm[5], vm[6], vm[8], vm[9], vm[10]}};
    float tx = vm[0] * p0 + vm[1] * p1 + vm[2] * p2 + vm[3];
    float ty = vm[4] * p0 + vm[5] * p1 + vm[6] * p2 + vm[7];
    float tz = vm[8] * p0 + vm[9] * p1 + vm[10] * p2 + vm[11];
    const bool clamped = !(pp.quirks & GSPLAT_QUIRK_EWA_UNCLAMPED);
    float limx = 1.3f * pp.tan_fovx, limy = 1.3f * pp.tan_fovy, sx = 0.f, sy = 0.f;
    if (clamped) {
      const float ux = tx / tz, uy = ty / tz;
      sx = ux < -limx ? -limx : (ux > limx ? limx : 0.f);  // 0: inside the clamp
      sy = uy < -limy ? -limy : (uy > limy ? limy : 0.f);
      tx = tz * fminf(limx, fmaxf(-limx, ux));
      ty = tz * fminf(limy, fmaxf(-limy, uy));
    }
    float rz = 1.f / tz;
    float rz2 = rz * rz;
    float rz3 = rz2 * rz;
    M3 J = {{fx * rz, 0.f, -fx * tx * rz2, 0.f, fy * rz, -fy * ty * rz2, 0.f, 0.f, 0.f}};
    M3 V = {{cv[0], cv[1], cv[2], cv[1], cv[3], cv[4], cv[2], cv[4], cv[5]}};
    M3 G = {{g.vc2[0], 0.5f * g.vc2[1], 0.f, 0.5f * g.vc2[1], g.vc2[2], 0.f, 0.f, 0.f, 0.f}};
    M3 T = mul(J, Wm);
    M3 Tt = transpose(T);
    M3 vV = mul(mul(Tt, G), T);
    M3 vT1 = mul(mul(G, T), transpose(V));
    M3 vT2 = mul(mul(transpose(G), T), V);
    M3 vT;
#pragma unroll
    for (int k = 0; k < 9; ++k) vT.m[k] = vT1.m[k] + vT2.m[k];
    g.vc3[0] = vV.m[0];
    g.vc3[1] = vV.m[3] + vV.m[1];
    g.vc3[2] = vV.m[6] + vV.m[2];
    g.vc3[3] = vV.m[4];
    g.vc3[4] = vV.m[7] + vV.m[5];
    g.vc3[5] = vV.m[8];
    M3 vJ = mul(vT, transpose(Wm));
    float vJ20 = vJ.m[2], vJ21 = vJ.m[5], vJ00 = vJ.m[0], vJ11 = vJ.m[4];
    float vt0 = -fx * rz2 * vJ20;
    float vt1 = -fy * rz2 * vJ21;
    float vt2 = -fx * rz2 * vJ00 + 2.f * fx * tx * rz3 * vJ20 - fy * rz2 * vJ11 +
                2.f * fy * ty * rz3 * vJ21;
    if (clamped) {
      if (sx != 0.f) { vt2 += sx * vt0; vt0 = 0.f; }
      if (sy != 0.f) { vt2 += sy * vt1; vt1 = 0.f; }
    }
    g.vmean[0] += vt0 * Wm.m[0] + vt1 * Wm.m[3] + vt2 * Wm.m[6];
    g.vmean[1] += vt0 * Wm.m[1] + vt1 * Wm.m[4] + vt2 * Wm.m[7];
    g.vmean[2] += vt0 * Wm.m[2] + vt1 * Wm.m[5] + vt2 * Wm.m[8];
  }
  // scale_rot_to_cov3d_vjp + quat_to_rotmat_vjp
  {
    const float *vc3 = g.vc3;
    M3 vV = {{vc3[0], 0.5f * vc3[1], 0.5f * vc3[2], 0.5f * vc3[1], vc3[3], 0.5f * vc3[4],
              0.5f * vc3[2], 0.5f * vc3[4], vc3[5]}};
    M3 R = quat_to_rotmat(q0, q1, q2, q3);
    M3 S = diag3(glob_scale * s0, glob_scale * s1, glob_scale * s2);
    M3 M = mul(R, S);
    M3 vM = mul(vV, M);
#pragma unroll
    for (int k = 0; k < 9; ++k) vM.m[k] = 2.f * vM.m[k];
#pragma unroll
    for (int cc = 0; cc < 3; ++cc)
      g.vscale[cc] = (R.m[0 * 3 + cc] * vM.m[0 * 3 + cc] + R.m[1 * 3 + cc] * vM.m[1 * 3 + cc] +
                      R.m[2 * 3 + cc] * vM.m[2 * 3 + cc]) *
                     glob_scale;
    M3 vRm = mul(vM, S);
    const float *vR = vRm.m;
    float s = 1.f / sqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
    float w = q0 * s, x = q1 * s, y = q2 * s, z = q3 * s;
#define GR(c, r) vR[(r) * 3 + (c)]
    g.vquat[0] = 2.f * (x * (GR(1, 2) - GR(2, 1)) + y * (GR(2, 0) - GR(0, 2)) +
                        z * (GR(0, 1) - GR(1, 0)));
    g.vquat[1] = 2.f * (-2.f * x * (GR(1, 1) + GR(2, 2)) + y * (GR(0, 1) + GR(1, 0)) +
                        z * (GR(0, 2) + GR(2, 0)) + w * (GR(1, 2) - GR(2, 1)));
    g.vquat[2] = 2.f * (x * (GR(0, 1) + GR(1, 0)) - 2.f * y * (GR(0, 0) + GR(2, 2)) +
                        z * (GR(1, 2) + GR(2, 1)) + w * (GR(2, 0) - GR(0, 2)));
    g.vquat[3] = 2.f * (x * (GR(0, 2) + GR(2, 0)) + y * (GR(1, 2) + GR(2, 1)) -
                        2.f * z * (GR(0, 0) + GR(1, 1)) + w * (GR(0, 1) - GR(1, 0)));
#undef GR
  }
}

}  // namespace
}  // namespace gs
