// torch_ops.cpp -- the schema-typed torch operator layer over the C ABI (SURVEY.md §8b "Native
// ABI"): TORCH_LIBRARY(gsplat_mi355x) ops for the gsplat 0.1.2.1 primitives, each a thin
// wrapper that checks device / dtype / shape through the dispatcher's tensors, allocates its
// outputs with the caching allocator, and calls the extern "C" launcher of
// libgsplat_mi355x.so on the current HIP stream.  Meta (fake) kernels give every op its output
// shapes without running it, so graphs that call the ops trace under torch.compile.
//
//   op               C-ABI entry (include/gsplat_mi355x.h)     replaces (gsplat 0.1.2.1)
//   project_fwd      gsplat_project_gaussians_forward          _C.project_gaussians_forward
//   project_bwd      gsplat_project_gaussians_backward         _C.project_gaussians_backward
//   sh_fwd / sh_bwd  gsplat_compute_sh_forward / _backward     _C.compute_sh_forward / _backward
//   map_intersects   gsplat_map_gaussian_to_intersects         _C.map_gaussian_to_intersects
//   sort_pairs       gsplat_sort_isect_pairs                   torch.sort in bin_and_sort_gaussians
//   tile_bins        gsplat_get_tile_bin_edges                 _C.get_tile_bin_edges
//   raster_fwd       gsplat_rasterize_forward                  _C.rasterize_forward / nd_...
//   raster_bwd       gsplat_rasterize_backward                 _C.rasterize_backward / nd_...
// (the reference's call sites: gc_model.py:174-236 through gsplat's autograd wrappers)
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <ATen/ATen.h>

#include "../../include/gsplat_mi355x.h"

// The op namespace: gsplat_mi355x, or gsplat_mi355x_hooks for the copy linked against the test
// library (Makefile: libgsplat_torch_ops_hooks.so; gaussctrl_exp_amd/ops.py under _lib.hooks()).
#ifndef GSPLAT_OPS_NS
#define GSPLAT_OPS_NS gsplat_mi355x
#endif
#define GS_TORCH_LIBRARY(ns, m) TORCH_LIBRARY(ns, m)
#define GS_TORCH_LIBRARY_IMPL(ns, k, m) TORCH_LIBRARY_IMPL(ns, k, m)

namespace {

using at::Tensor;

void *stream_of(const Tensor &t) {
  return (void *)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check(int rc, const char *what) {
  TORCH_CHECK(rc == 0, "gsplat_mi355x::", what, ": ", gsplat_last_error());
}

// Every op runs its launcher on the device of its first tensor argument (a device guard makes it
// current) and requires all its tensors there.
thread_local c10::Device g_op_device = c10::Device(c10::kCPU);
void need(const Tensor &t, const char *name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), "gsplat_mi355x: ", name, " must be a ROCm device tensor");
  TORCH_CHECK(g_op_device.is_cpu() || t.device() == g_op_device, "gsplat_mi355x: ", name,
              " is on ", t.device(), ", the op's other tensors on ", g_op_device);
  TORCH_CHECK(t.scalar_type() == dt, "gsplat_mi355x: ", name, " must be ", dt, ", got ",
              t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), "gsplat_mi355x: ", name, " must be contiguous");
}

void need_rows(const Tensor &t, const char *name, int64_t n, int64_t cols) {
  TORCH_CHECK(t.numel() == n * cols, "gsplat_mi355x: ", name, " must hold ", n, " x ", cols,
              " values, got shape ", t.sizes());
}

struct OpDevice {  // the op's device: guard + same-device checks in need()
  c10::OptionalDeviceGuard guard;
  explicit OpDevice(const Tensor &first) {
    TORCH_CHECK(first.is_cuda(), "gsplat_mi355x: expected ROCm device tensors (no CPU path)");
    guard.reset_device(first.device());
    g_op_device = first.device();
  }
  ~OpDevice() { g_op_device = c10::Device(c10::kCPU); }
};

int sh_bases(int64_t degree) {
  TORCH_CHECK(degree >= 0 && degree <= 4, "gsplat_mi355x: SH degree must be in [0, 4]");
  return (int)((degree + 1) * (degree + 1));
}

at::TensorOptions f32(const Tensor &like) { return like.options().dtype(at::kFloat); }
at::TensorOptions i32(const Tensor &like) { return like.options().dtype(at::kInt); }

// ---------------------------------------------------------------- projection
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> project_fwd(
    const Tensor &means3d, const Tensor &scales, double glob_scale, const Tensor &quats,
    const Tensor &viewmat, const Tensor &projmat, double fx, double fy, double cx, double cy,
    int64_t img_height, int64_t img_width, int64_t tile_bounds_x, int64_t tile_bounds_y,
    double clip_thresh) {
  const int64_t n = means3d.size(0);
  OpDevice od(means3d);
  need(means3d, "means3d", at::kFloat);
  need(scales, "scales", at::kFloat);
  need(quats, "quats", at::kFloat);
  need(viewmat, "viewmat", at::kFloat);
  need(projmat, "projmat", at::kFloat);
  need_rows(means3d, "means3d", n, 3);
  need_rows(scales, "scales", n, 3);
  need_rows(quats, "quats", n, 4);
  TORCH_CHECK(viewmat.numel() >= 12 && projmat.numel() == 16,
              "gsplat_mi355x: viewmat needs >= 12 values, projmat 16");
  Tensor xys = at::empty({n, 2}, f32(means3d)), depths = at::empty({n}, f32(means3d));
  Tensor radii = at::empty({n}, i32(means3d)), conics = at::empty({n, 3}, f32(means3d));
  Tensor nth = at::empty({n}, i32(means3d)), cov3d = at::empty({n, 6}, f32(means3d));
  check(gsplat_project_gaussians_forward(
            (int)n, means3d.data_ptr<float>(), scales.data_ptr<float>(), (float)glob_scale,
            quats.data_ptr<float>(), viewmat.data_ptr<float>(), projmat.data_ptr<float>(),
            (float)fx, (float)fy, (float)cx, (float)cy, (int)img_height, (int)img_width,
            (int)tile_bounds_x, (int)tile_bounds_y, (float)clip_thresh, cov3d.data_ptr<float>(),
            xys.data_ptr<float>(), depths.data_ptr<float>(), radii.data_ptr<int32_t>(),
            conics.data_ptr<float>(), nth.data_ptr<int32_t>(), stream_of(means3d)),
        "project_fwd");
  return {xys, depths, radii, conics, nth, cov3d};
}

std::tuple<Tensor, Tensor, Tensor> project_bwd(
    const Tensor &means3d, const Tensor &scales, double glob_scale, const Tensor &quats,
    const Tensor &viewmat, const Tensor &projmat, double fx, double fy, double cx, double cy,
    int64_t img_height, int64_t img_width, const Tensor &cov3d, const Tensor &radii,
    const Tensor &conics, const Tensor &v_xy, const c10::optional<Tensor> &v_depth,
    const Tensor &v_conic) {
  const int64_t n = means3d.size(0);
  OpDevice od(means3d);
  need(means3d, "means3d", at::kFloat);
  need(scales, "scales", at::kFloat);
  need(quats, "quats", at::kFloat);
  need(viewmat, "viewmat", at::kFloat);
  need(projmat, "projmat", at::kFloat);
  need(cov3d, "cov3d", at::kFloat);
  need(radii, "radii", at::kInt);
  need(conics, "conics", at::kFloat);
  need(v_xy, "v_xy", at::kFloat);
  need(v_conic, "v_conic", at::kFloat);
  need_rows(means3d, "means3d", n, 3);
  need_rows(scales, "scales", n, 3);
  need_rows(quats, "quats", n, 4);
  need_rows(cov3d, "cov3d", n, 6);
  need_rows(radii, "radii", n, 1);
  need_rows(conics, "conics", n, 3);
  TORCH_CHECK(viewmat.numel() >= 12 && projmat.numel() == 16,
              "gsplat_mi355x: viewmat needs >= 12 values, projmat 16");
  need_rows(v_xy, "v_xy", n, 2);
  need_rows(v_conic, "v_conic", n, 3);
  const float *vd = nullptr;
  if (v_depth.has_value()) {
    need(*v_depth, "v_depth", at::kFloat);
    need_rows(*v_depth, "v_depth", n, 1);
    vd = v_depth->data_ptr<float>();
  }
  Tensor vm = at::empty({n, 3}, f32(means3d)), vs = at::empty({n, 3}, f32(means3d));
  Tensor vq = at::empty({n, 4}, f32(means3d));
  check(gsplat_project_gaussians_backward(
            (int)n, means3d.data_ptr<float>(), scales.data_ptr<float>(), (float)glob_scale,
            quats.data_ptr<float>(), viewmat.data_ptr<float>(), projmat.data_ptr<float>(),
            (float)fx, (float)fy, (float)cx, (float)cy, (int)img_height, (int)img_width,
            cov3d.data_ptr<float>(), radii.data_ptr<int32_t>(), conics.data_ptr<float>(),
            v_xy.data_ptr<float>(), vd, v_conic.data_ptr<float>(), nullptr, nullptr,
            vm.data_ptr<float>(), vs.data_ptr<float>(), vq.data_ptr<float>(), stream_of(means3d)),
        "project_bwd");
  return {vm, vs, vq};
}

// ---------------------------------------------------------------- spherical harmonics
Tensor sh_fwd(int64_t degree, int64_t degrees_to_use, const Tensor &viewdirs,
              const Tensor &coeffs) {
  const int64_t n = viewdirs.size(0);
  OpDevice od(viewdirs);
  const int K = sh_bases(degree);
  need(viewdirs, "viewdirs", at::kFloat);
  need(coeffs, "coeffs", at::kFloat);
  need_rows(viewdirs, "viewdirs", n, 3);
  need_rows(coeffs, "coeffs", n, 3 * K);
  Tensor colors = at::empty({n, 3}, f32(viewdirs));
  check(gsplat_compute_sh_forward((int)n, (int)degree, (int)degrees_to_use,
                                  viewdirs.data_ptr<float>(), coeffs.data_ptr<float>(),
                                  colors.data_ptr<float>(), stream_of(viewdirs)),
        "sh_fwd");
  return colors;
}

Tensor sh_bwd(int64_t degree, int64_t degrees_to_use, const Tensor &viewdirs,
              const Tensor &v_colors) {
  const int64_t n = viewdirs.size(0);
  OpDevice od(viewdirs);
  const int K = sh_bases(degree);
  need(viewdirs, "viewdirs", at::kFloat);
  need(v_colors, "v_colors", at::kFloat);
  need_rows(viewdirs, "viewdirs", n, 3);
  need_rows(v_colors, "v_colors", n, 3);
  Tensor v_coeffs = at::empty({n, K, 3}, f32(viewdirs));
  check(gsplat_compute_sh_backward((int)n, (int)degree, (int)degrees_to_use,
                                   viewdirs.data_ptr<float>(), v_colors.data_ptr<float>(),
                                   v_coeffs.data_ptr<float>(), stream_of(viewdirs)),
        "sh_bwd");
  return v_coeffs;
}

// ---------------------------------------------------------------- gsplat-layout binning
std::tuple<Tensor, Tensor> map_intersects(const Tensor &xys, const Tensor &depths,
                                          const Tensor &radii, const Tensor &cum_tiles_hit,
                                          int64_t tile_bounds_x, int64_t tile_bounds_y,
                                          int64_t num_intersects) {
  const int64_t n = xys.size(0);
  OpDevice od(xys);
  need(xys, "xys", at::kFloat);
  need(depths, "depths", at::kFloat);
  need(radii, "radii", at::kInt);
  need(cum_tiles_hit, "cum_tiles_hit", at::kInt);
  need_rows(xys, "xys", n, 2);
  need_rows(depths, "depths", n, 1);
  need_rows(radii, "radii", n, 1);
  need_rows(cum_tiles_hit, "cum_tiles_hit", n, 1);
  TORCH_CHECK(num_intersects >= 0, "gsplat_mi355x: num_intersects must be >= 0");
  // zero-filled like gsplat's torch.zeros outputs: slots past cum_tiles_hit[-1] stay 0
  Tensor isect = at::zeros({num_intersects}, xys.options().dtype(at::kLong));
  Tensor gid = at::zeros({num_intersects}, i32(xys));
  if (n > 0 && num_intersects > 0)
    check(gsplat_map_gaussian_to_intersects(
              (int)n, xys.data_ptr<float>(), depths.data_ptr<float>(), radii.data_ptr<int32_t>(),
              cum_tiles_hit.data_ptr<int32_t>(), (int)tile_bounds_x, (int)tile_bounds_y,
              isect.data_ptr<int64_t>(), gid.data_ptr<int32_t>(), stream_of(xys)),
          "map_intersects");
  return {isect, gid};
}

std::tuple<Tensor, Tensor> sort_pairs(const Tensor &keys, const Tensor &vals, int64_t key_bits) {
  OpDevice od(keys);
  need(keys, "keys", at::kLong);
  need(vals, "vals", at::kInt);
  const int64_t m = keys.numel();
  TORCH_CHECK(vals.numel() == m, "gsplat_mi355x: keys and vals differ in length");
  Tensor ko = at::empty_like(keys), vo = at::empty_like(vals);
  if (m > 0) {
    Tensor ws = at::empty({(int64_t)gsplat_sort_isect_pairs_workspace_size(m)},
                          keys.options().dtype(at::kByte));
    check(gsplat_sort_isect_pairs(m, (int)key_bits, keys.data_ptr<int64_t>(),
                                  vals.data_ptr<int32_t>(), ko.data_ptr<int64_t>(),
                                  vo.data_ptr<int32_t>(), ws.data_ptr(), (size_t)ws.numel(),
                                  stream_of(keys)),
          "sort_pairs");
  }
  return {ko, vo};
}

Tensor tile_bins(const Tensor &isect_ids_sorted, int64_t num_rows) {
  OpDevice od(isect_ids_sorted);
  need(isect_ids_sorted, "isect_ids_sorted", at::kLong);
  Tensor bins = at::empty({num_rows, 2}, i32(isect_ids_sorted));
  check(gsplat_get_tile_bin_edges(isect_ids_sorted.numel(), isect_ids_sorted.data_ptr<int64_t>(),
                                  bins.data_ptr<int32_t>(), num_rows, stream_of(isect_ids_sorted)),
        "tile_bins");
  return bins;
}

// ---------------------------------------------------------------- rasterization
void check_raster_inputs(const Tensor &gids, const Tensor &bins, const Tensor &xys,
                         const Tensor &conics, const Tensor &colors, const Tensor &opacity,
                         const Tensor &background, int64_t tbx, int64_t tby) {
  need(gids, "gaussian_ids_sorted", at::kInt);
  need(bins, "tile_bins", at::kInt);
  need(xys, "xys", at::kFloat);
  need(conics, "conics", at::kFloat);
  need(colors, "colors", at::kFloat);
  need(opacity, "opacity", at::kFloat);
  need(background, "background", at::kFloat);
  const int64_t n = xys.size(0);
  TORCH_CHECK(colors.dim() == 2 && colors.size(0) == n, "gsplat_mi355x: colors must be [N, C]");
  need_rows(conics, "conics", n, 3);
  need_rows(opacity, "opacity", n, 1);
  TORCH_CHECK(background.numel() == colors.size(1), "gsplat_mi355x: background must be [C]");
  TORCH_CHECK(bins.numel() >= tbx * tby * 2, "gsplat_mi355x: tile_bins must be [tiles, 2]");
}

std::tuple<Tensor, Tensor, Tensor> raster_fwd(int64_t tbx, int64_t tby, int64_t H, int64_t W,
                                              const Tensor &gids, const Tensor &bins,
                                              const Tensor &xys, const Tensor &conics,
                                              const Tensor &colors, const Tensor &opacity,
                                              const Tensor &background) {
  OpDevice od(xys);
  check_raster_inputs(gids, bins, xys, conics, colors, opacity, background, tbx, tby);
  const int64_t C = colors.size(1);
  Tensor out = at::empty({H, W, C}, f32(xys)), fT = at::empty({H, W}, f32(xys));
  Tensor fi = at::empty({H, W}, i32(xys));
  check(gsplat_rasterize_forward((int)tbx, (int)tby, (int)H, (int)W, (int)C,
                                 gids.data_ptr<int32_t>(), bins.data_ptr<int32_t>(),
                                 xys.data_ptr<float>(), conics.data_ptr<float>(),
                                 colors.data_ptr<float>(), opacity.data_ptr<float>(),
                                 background.data_ptr<float>(), out.data_ptr<float>(),
                                 fT.data_ptr<float>(), fi.data_ptr<int32_t>(), stream_of(xys)),
        "raster_fwd");
  return {out, fT, fi};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> raster_bwd(
    int64_t tbx, int64_t tby, int64_t H, int64_t W, const Tensor &gids, const Tensor &bins,
    const Tensor &xys, const Tensor &conics, const Tensor &colors, const Tensor &opacity,
    const Tensor &background, const Tensor &final_Ts, const Tensor &final_idx,
    const Tensor &v_output, const c10::optional<Tensor> &v_output_alpha, double alpha_max) {
  OpDevice od(xys);
  check_raster_inputs(gids, bins, xys, conics, colors, opacity, background, tbx, tby);
  need(final_Ts, "final_Ts", at::kFloat);
  need(final_idx, "final_idx", at::kInt);
  need(v_output, "v_output", at::kFloat);
  const int64_t n = xys.size(0), C = colors.size(1);
  need_rows(final_Ts, "final_Ts", H * W, 1);
  need_rows(final_idx, "final_idx", H * W, 1);
  need_rows(v_output, "v_output", H * W, C);
  const float *va = nullptr;
  if (v_output_alpha.has_value()) {
    need(*v_output_alpha, "v_output_alpha", at::kFloat);
    need_rows(*v_output_alpha, "v_output_alpha", H * W, 1);
    va = v_output_alpha->data_ptr<float>();
  }
  Tensor v_xy = at::empty({n, 2}, f32(xys)), v_conic = at::empty({n, 3}, f32(xys));
  Tensor v_colors = at::empty({n, C}, f32(xys)), v_opac = at::empty({n, 1}, f32(xys));
  Tensor ws = at::empty({(int64_t)gsplat_rasterize_backward_workspace_size((int)n, (int)C)},
                        xys.options().dtype(at::kByte));
  check(gsplat_rasterize_backward((int)tbx, (int)tby, (int)H, (int)W, (int)C, (int)n,
                                  gids.data_ptr<int32_t>(), bins.data_ptr<int32_t>(),
                                  xys.data_ptr<float>(), conics.data_ptr<float>(),
                                  colors.data_ptr<float>(), opacity.data_ptr<float>(),
                                  background.data_ptr<float>(), final_Ts.data_ptr<float>(),
                                  final_idx.data_ptr<int32_t>(), v_output.data_ptr<float>(), va,
                                  (float)alpha_max, v_xy.data_ptr<float>(),
                                  v_conic.data_ptr<float>(), v_colors.data_ptr<float>(),
                                  v_opac.data_ptr<float>(), ws.numel() ? ws.data_ptr() : nullptr,
                                  (size_t)ws.numel(), stream_of(xys)),
        "raster_bwd");
  return {v_xy, v_conic, v_colors, v_opac};
}

// ---------------------------------------------------------------- Meta (shape-only) kernels
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> project_fwd_meta(
    const Tensor &means3d, const Tensor &, double, const Tensor &, const Tensor &,
    const Tensor &, double, double, double, double, int64_t, int64_t, int64_t, int64_t, double) {
  const int64_t n = means3d.size(0);
  auto o = means3d.options();
  return {at::empty({n, 2}, o.dtype(at::kFloat)), at::empty({n}, o.dtype(at::kFloat)),
          at::empty({n}, o.dtype(at::kInt)),      at::empty({n, 3}, o.dtype(at::kFloat)),
          at::empty({n}, o.dtype(at::kInt)),      at::empty({n, 6}, o.dtype(at::kFloat))};
}
std::tuple<Tensor, Tensor, Tensor> project_bwd_meta(
    const Tensor &means3d, const Tensor &, double, const Tensor &, const Tensor &,
    const Tensor &, double, double, double, double, int64_t, int64_t, const Tensor &,
    const Tensor &, const Tensor &, const Tensor &, const c10::optional<Tensor> &,
    const Tensor &) {
  const int64_t n = means3d.size(0);
  auto o = means3d.options().dtype(at::kFloat);
  return {at::empty({n, 3}, o), at::empty({n, 3}, o), at::empty({n, 4}, o)};
}
Tensor sh_fwd_meta(int64_t, int64_t, const Tensor &viewdirs, const Tensor &) {
  return at::empty({viewdirs.size(0), 3}, viewdirs.options().dtype(at::kFloat));
}
Tensor sh_bwd_meta(int64_t degree, int64_t, const Tensor &viewdirs, const Tensor &) {
  return at::empty({viewdirs.size(0), sh_bases(degree), 3}, viewdirs.options().dtype(at::kFloat));
}
std::tuple<Tensor, Tensor> map_intersects_meta(const Tensor &xys, const Tensor &, const Tensor &,
                                               const Tensor &, int64_t, int64_t, int64_t m) {
  return {at::empty({m}, xys.options().dtype(at::kLong)),
          at::empty({m}, xys.options().dtype(at::kInt))};
}
std::tuple<Tensor, Tensor> sort_pairs_meta(const Tensor &keys, const Tensor &vals, int64_t) {
  return {at::empty_like(keys), at::empty_like(vals)};
}
Tensor tile_bins_meta(const Tensor &isect, int64_t num_rows) {
  return at::empty({num_rows, 2}, isect.options().dtype(at::kInt));
}
std::tuple<Tensor, Tensor, Tensor> raster_fwd_meta(int64_t, int64_t, int64_t H, int64_t W,
                                                   const Tensor &, const Tensor &,
                                                   const Tensor &xys, const Tensor &,
                                                   const Tensor &colors, const Tensor &,
                                                   const Tensor &) {
  auto o = xys.options();
  return {at::empty({H, W, colors.size(1)}, o.dtype(at::kFloat)),
          at::empty({H, W}, o.dtype(at::kFloat)), at::empty({H, W}, o.dtype(at::kInt))};
}
std::tuple<Tensor, Tensor, Tensor, Tensor> raster_bwd_meta(
    int64_t, int64_t, int64_t, int64_t, const Tensor &, const Tensor &, const Tensor &xys,
    const Tensor &, const Tensor &colors, const Tensor &, const Tensor &, const Tensor &,
    const Tensor &, const Tensor &, const c10::optional<Tensor> &, double) {
  const int64_t n = xys.size(0);
  auto o = xys.options().dtype(at::kFloat);
  return {at::empty({n, 2}, o), at::empty({n, 3}, o), at::empty({n, colors.size(1)}, o),
          at::empty({n, 1}, o)};
}

}  // namespace

GS_TORCH_LIBRARY(GSPLAT_OPS_NS, m) {
  m.def("project_fwd(Tensor means3d, Tensor scales, float glob_scale, Tensor quats, "
        "Tensor viewmat, Tensor projmat, float fx, float fy, float cx, float cy, int img_height, "
        "int img_width, int tile_bounds_x, int tile_bounds_y, float clip_thresh) -> "
        "(Tensor xys, Tensor depths, Tensor radii, Tensor conics, Tensor num_tiles_hit, "
        "Tensor cov3d)");
  m.def("project_bwd(Tensor means3d, Tensor scales, float glob_scale, Tensor quats, "
        "Tensor viewmat, Tensor projmat, float fx, float fy, float cx, float cy, int img_height, "
        "int img_width, Tensor cov3d, Tensor radii, Tensor conics, Tensor v_xy, "
        "Tensor? v_depth, Tensor v_conic) -> (Tensor v_mean3d, Tensor v_scale, Tensor v_quat)");
  m.def("sh_fwd(int degree, int degrees_to_use, Tensor viewdirs, Tensor coeffs) -> Tensor");
  m.def("sh_bwd(int degree, int degrees_to_use, Tensor viewdirs, Tensor v_colors) -> Tensor");
  m.def("map_intersects(Tensor xys, Tensor depths, Tensor radii, Tensor cum_tiles_hit, "
        "int tile_bounds_x, int tile_bounds_y, int num_intersects) -> "
        "(Tensor isect_ids, Tensor gaussian_ids)");
  m.def("sort_pairs(Tensor keys, Tensor vals, int key_bits) -> (Tensor, Tensor)");
  m.def("tile_bins(Tensor isect_ids_sorted, int num_rows) -> Tensor");
  m.def("raster_fwd(int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, "
        "Tensor gaussian_ids_sorted, Tensor tile_bins, Tensor xys, Tensor conics, "
        "Tensor colors, Tensor opacity, Tensor background) -> "
        "(Tensor out_img, Tensor final_Ts, Tensor final_idx)");
  m.def("raster_bwd(int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, "
        "Tensor gaussian_ids_sorted, Tensor tile_bins, Tensor xys, Tensor conics, "
        "Tensor colors, Tensor opacity, Tensor background, Tensor final_Ts, Tensor final_idx, "
        "Tensor v_output, Tensor? v_output_alpha, float alpha_max) -> "
        "(Tensor v_xy, Tensor v_conic, Tensor v_colors, Tensor v_opacity)");
}

GS_TORCH_LIBRARY_IMPL(GSPLAT_OPS_NS, CUDA, m) {  // the ROCm device dispatch key
  m.impl("project_fwd", &project_fwd);
  m.impl("project_bwd", &project_bwd);
  m.impl("sh_fwd", &sh_fwd);
  m.impl("sh_bwd", &sh_bwd);
  m.impl("map_intersects", &map_intersects);
  m.impl("sort_pairs", &sort_pairs);
  m.impl("tile_bins", &tile_bins);
  m.impl("raster_fwd", &raster_fwd);
  m.impl("raster_bwd", &raster_bwd);
}

GS_TORCH_LIBRARY_IMPL(GSPLAT_OPS_NS, Meta, m) {
  m.impl("project_fwd", &project_fwd_meta);
  m.impl("project_bwd", &project_bwd_meta);
  m.impl("sh_fwd", &sh_fwd_meta);
  m.impl("sh_bwd", &sh_bwd_meta);
  m.impl("map_intersects", &map_intersects_meta);
  m.impl("sort_pairs", &sort_pairs_meta);
  m.impl("tile_bins", &tile_bins_meta);
  m.impl("raster_fwd", &raster_fwd_meta);
  m.impl("raster_bwd", &raster_bwd_meta);
}
