/*
 * gsplat_mi355x.h -- C ABI of the MI355X (gfx950) 3D Gaussian splatting rasterizer.
 *
 * Drop-in boundary: these entry points are what gsplat 0.1.2.1's Python autograd
 * wrappers bind through `gsplat._C` (un-vendored dependency pinned at
 * /root/reference/README.md:58, called from /root/reference/gaussctrl/gc_model.py:174-236).
 * One entry point per `_C` function, with the same argument meaning; plain pointers,
 * sizes and a hipStream_t passed as void*.  All tensor pointers are DEVICE pointers to
 * contiguous row-major storage (float32 unless named *_i32 / int).  No entry point
 * allocates, frees or synchronises: scratch comes from a caller-provided workspace whose
 * size is reported by the matching *_workspace_size() query, so every call is
 * hipGraph-capturable.
 *
 * Return value: 0 on success, non-zero on error (gsplat_last_error() describes it);
 * argument errors are reported before anything is launched.
 *
 * Reference interfaces replaced (gsplat 0.1.2.1, [ext] = not vendored in the reference):
 *   gsplat_project_gaussians_forward   <- _C.project_gaussians_forward  (gc_model.py:174-188)
 *   gsplat_project_gaussians_backward  <- _C.project_gaussians_backward (autograd of :174)
 *   gsplat_compute_sh_forward          <- _C.compute_sh_forward         (gc_model.py:200)
 *   gsplat_compute_sh_backward         <- _C.compute_sh_backward        (autograd of :200)
 *   gsplat_compute_cov2d_bounds        <- _C.compute_cov2d_bounds       (gsplat.utils)
 *   gsplat_map_gaussian_to_intersects  <- _C.map_gaussian_to_intersects (gsplat.utils)
 *   gsplat_sort_isect_pairs            <- torch.sort + torch.gather in utils.bin_and_sort_gaussians
 *   gsplat_get_tile_bin_edges          <- _C.get_tile_bin_edges         (gsplat.utils)
 *   gsplat_bin_count / gsplat_bin_emit <- the cumsum/map/sort/bin sequence inside
 *                                         rasterize.py _RasterizeGaussians.forward
 *                                         (gc_model.py:208-220, :225-236), fused
 *   gsplat_rasterize_forward           <- _C.rasterize_forward / _C.nd_rasterize_forward
 *   gsplat_rasterize_backward          <- _C.rasterize_backward / _C.nd_rasterize_backward
 *   gsplat_fused_preprocess_forward /  <- gc_model.py:158-215's activations + project_gaussians
 *   gsplat_fused_preprocess_backward      + spherical_harmonics (fused training render)
 */
#ifndef GSPLAT_MI355X_H
#define GSPLAT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 16: gsplat_exchange_sparse_plan needs a send buffer of 4 + 4W floats (its popcounts are staged
 * in the values area); the binning's phase-2 workspace layout follows the tile sort.
 * 17: gsplat_compute_sh_backward_view_table_adam; the region binning (test hooks) is gone. */
#define GSPLAT_MI355X_ABI_VERSION 17

int gsplat_abi_version(void);
const char *gsplat_last_error(void);

/* ---- gsplat 0.1.2.1 behaviours recalled but unverified (SURVEY.md Appendix A [VERIFY]) -
 * One process-wide mask, read at each launch (default GSPLAT_QUIRKS_ALL = gsplat as recalled;
 * the Python layer sets it from the GSPLAT_MI355X_QUIRKS environment variable).
 *   ALPHA_099      A10: the rasterize backward clamps alpha at 0.99 (forward 0.999).  The
 *                  callers pass that clamp as alpha_max; the bit records the choice.
 *   CONIC_HALF     A7/A9: v_conic.y = 1/2 v_sigma dx dy, paired with a conic VJP taking it as
 *                  the gradient of each symmetric entry; off: v_conic.y = d loss / d conic.y.
 *                  Gradients of means/scales/quats are identical either way.
 *   EWA_UNCLAMPED  A6: the EWA VJP recomputes t without the 1.3 tan_fov clamp; off: the
 *                  derivative of the clamped forward.
 * Replaces no gsplat entry point: gsplat has these behaviours hard-coded in
 * gsplat/cuda/csrc/{backward.cu, helpers.cuh}. */
#define GSPLAT_QUIRK_ALPHA_099 1
#define GSPLAT_QUIRK_CONIC_HALF 2
#define GSPLAT_QUIRK_EWA_UNCLAMPED 4
#define GSPLAT_QUIRKS_ALL 7
int gsplat_set_quirks(int mask);
int gsplat_get_quirks(void);

/* ---- deterministic backward (debugging) -------------------------------
 * on != 0: the C = 3 rasterize backward entries (gsplat_rasterize_backward,
 * _backward_chunked, _backward_records) add every wave's per-Gaussian totals as exact
 * integers (each total truncated to a multiple of 2^-80 and added as three 40-bit limbs into
 * 64-bit accumulators) instead of fp32 atomics, then convert: gradients are bit-identical from
 * run to run at any gradient magnitude.  Slower (integer atomics, an extra pass over N); the
 * accumulators are one library-owned buffer per device, allocated on first use, and calls on
 * different streams or threads are serialised on it (debug mode only).  Replaces no gsplat
 * entry point (gsplat's backward.cu atomics are order-nondeterministic). */
int gsplat_set_deterministic(int on);
int gsplat_get_deterministic(void);

/* ---- projection (forward.cu / backward.cu project_gaussians_*) ----------------------
 * means3d [N,3], scales [N,3], quats [N,4] (w,x,y,z), viewmat >= 12 floats (row-major
 * [3,4] or [4,4]; first 12 read), projmat [4,4].  Outputs are fully written (culled
 * Gaussians get zeros, except conics/cov3d which follow gsplat's write order). */
int gsplat_project_gaussians_forward(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, int tile_bounds_x, int tile_bounds_y,
    float clip_thresh, float *cov3d, float *xys, float *depths, int32_t *radii,
    float *conics, int32_t *num_tiles_hit, void *stream);

/* gsplat_project_gaussians_forward that also writes the binning's depth-sort inputs (depth
 * keys, ids, per-Gaussian tile records) into a gsplat_bin_count workspace (>=
 * gsplat_bin_count_workspace_size(num_points) bytes), so the rasterize call that follows bins
 * with gsplat_bin_count_keyed instead of re-reading xys/depths/radii/num_tiles_hit
 * (the drop-in project_gaussians does this; no gsplat counterpart). */
int gsplat_project_gaussians_forward_binned(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, int tile_bounds_x, int tile_bounds_y,
    float clip_thresh, float *cov3d, float *xys, float *depths, int32_t *radii,
    float *conics, int32_t *num_tiles_hit, void *workspace1, size_t workspace1_bytes,
    void *stream);

/* Outputs v_cov2d [N,3], v_cov3d [N,6], v_mean3d [N,3], v_scale [N,3], v_quat [N,4] are
 * fully written (zeros where radii <= 0); v_cov2d / v_cov3d (gsplat's intermediate
 * gradients, which its autograd wrapper discards) may be NULL.  v_depth may be NULL (an all-zero depth gradient,
 * which is what the gsplat autograd wrapper passes when nothing consumed depths). */
int gsplat_project_gaussians_backward(
    int num_points, const float *means3d, const float *scales, float glob_scale,
    const float *quats, const float *viewmat, const float *projmat, float fx, float fy,
    float cx, float cy, int img_height, int img_width, const float *cov3d,
    const int32_t *radii, const float *conics, const float *v_xy, const float *v_depth,
    const float *v_conic, float *v_cov2d, float *v_cov3d, float *v_mean3d, float *v_scale,
    float *v_quat, void *stream);

/* ---- spherical harmonics (sh.cuh) ----------------------------------------------------
 * coeffs [N, num_sh_bases(degree), 3]; colors [N,3]; v_coeffs fully written. */
int gsplat_compute_sh_forward(int num_points, int degree, int degrees_to_use,
                              const float *viewdirs, const float *coeffs, float *colors,
                              void *stream);
int gsplat_compute_sh_backward(int num_points, int degree, int degrees_to_use,
                               const float *viewdirs, const float *v_colors, float *v_coeffs,
                               void *stream);

/* gsplat_compute_sh_backward with the coefficient gradient split into v_dc [N,3] (basis 0)
 * and v_rest [N, K-1, 3] (may be NULL when degree == 0): the gradients of the caller's
 * cat(features_dc[:, None], features_rest) inputs, so the drop-in spherical_harmonics can
 * hand splatfacto's parameters contiguous gradients (no cat backward, no layout copies). */
int gsplat_compute_sh_backward_split(int num_points, int degree, int degrees_to_use,
                                     const float *viewdirs, const float *v_colors, float *v_dc,
                                     float *v_rest, void *stream);

/* Data-parallel extension (no gsplat counterpart): the sum over num_views
 * cameras of the SH coefficient gradient, v_coeffs[i] = sum_r Y(means3d[i] - campos_r) (x)
 * v_colors_r[i], summed in view order (bit-identical on every rank).  views holds one
 * record per view, view_stride (>= 3 N + 3) floats apart: v_colors_r [N,3] followed by
 * campos_r [3] -- exactly what an all-gather of each rank's [v_colors | campos] produces.
 * v_coeffs [N, num_sh_bases(degree), 3] fully written. */
int gsplat_compute_sh_backward_views(int num_points, int degree, int degrees_to_use,
                                     int num_views, const float *means3d, const float *views,
                                     long long view_stride, float *v_coeffs, void *stream);

/* Split-output variant for the fused training path: v_dc [N,3] gets basis 0, v_rest
 * [N, num_sh_bases(degree) - 1, 3] the rest (may be NULL when degree == 0) -- splatfacto's
 * separate features_dc / features_rest gradients, without a combined tensor. */
int gsplat_compute_sh_backward_views_split(int num_points, int degree, int degrees_to_use,
                                           int num_views, const float *means3d,
                                           const float *views, long long view_stride,
                                           float *v_dc, float *v_rest, void *stream);
/* gsplat_compute_sh_backward_views_split over a table of records (HOST arrays of num_views <=
 * 64 device pointers and capacities): capacities[r] < 0 -> records[r] is a dense record
 * (v_colors [3N] | camera centre | pad), else a sparse one of that capacity
 * (gsplat_exchange_pack_sparse).  Sums in table order; sparse and dense records of the same
 * views give bit-identical results. */
int gsplat_compute_sh_backward_view_table(int num_points, int degree, int degrees_to_use,
                                          int num_views, const float *means3d,
                                          const float *const *records,
                                          const long long *capacities, float *v_dc,
                                          float *v_rest, void *stream);
/* gsplat_compute_sh_backward_view_table with the Adam step of the two SH-feature groups fused
 * in (the N > 1 training step; replaces the table kernel + gsplat_adam_step over features_dc /
 * features_rest at gc_trainer.py:281): the summed gradient is applied in place to features_dc
 * [N,3] / features_rest [N, num_sh_bases(degree) - 1, 3] and their exp_avg / exp_avg_sq
 * moments, with gsplat_adam_step's element arithmetic and bias corrections (lr_dc / lr_rest,
 * step >= 1, beta1 in (0.5, 1)) -- bit-identical to the two calls.  No gradient is written. */
int gsplat_compute_sh_backward_view_table_adam(
    int num_points, int degree, int degrees_to_use, int num_views, const float *means3d,
    const float *const *records, const long long *capacities, float *features_dc,
    float *features_rest, float *exp_avg_dc, float *exp_avg_sq_dc, float *exp_avg_rest,
    float *exp_avg_sq_rest, float lr_dc, float lr_rest, int step, float beta1, float beta2,
    float eps, void *stream);

/* covs2d [N,3] -> conics [N,3], radii [N] (float).  det == 0 rows get zeros. */
int gsplat_compute_cov2d_bounds(int num_points, const float *covs2d, float *conics,
                                float *radii, void *stream);

/* ---- gsplat-layout binning (utils.py) -------------------------------------------------
 * isect_ids [I] int64 = (tile_id << 32) | float_bits(depth), gaussian_ids [I] int32,
 * written at cum_tiles_hit[i-1] for Gaussian i (cum_tiles_hit = inclusive cumsum). */
int gsplat_map_gaussian_to_intersects(int num_points, const float *xys, const float *depths,
                                      const int32_t *radii, const int32_t *cum_tiles_hit,
                                      int tile_bounds_x, int tile_bounds_y, int64_t *isect_ids,
                                      int32_t *gaussian_ids, void *stream);

/* Stable LSD radix sort of (isect_ids, gaussian_ids) pairs by key bits [0, key_bits).
 * Keys must be non-negative.  Outputs may not alias inputs. */
size_t gsplat_sort_isect_pairs_workspace_size(int64_t num_items);
int gsplat_sort_isect_pairs(int64_t num_items, int key_bits, const int64_t *keys_in,
                            const int32_t *vals_in, int64_t *keys_out, int32_t *vals_out,
                            void *workspace, size_t workspace_bytes, void *stream);

/* tile_bins [num_rows,2] int32: zero-filled here, then [first,last+1) per tile id. Tile
 * ids >= num_rows are dropped (gsplat 0.1.x sizes the table by num_intersects). */
int gsplat_get_tile_bin_edges(int64_t num_intersects, const int64_t *isect_ids_sorted,
                              int32_t *tile_bins, int64_t num_rows, void *stream);

/* ---- fused binning for rasterize (cumsum -> map -> sort -> bins) ------------------------
 * Phase 1 (gsplat_bin_count) orders the visible Gaussians (radii > 0) front to back
 * (stable on the depth bits, ties by Gaussian id) and writes d_counts[0] = visible count,
 * d_counts[1] = total intersections I (device int32[2]).  The caller reads d_counts -- the
 * one host sync, like gsplat's cum_tiles_hit[-1].item() -- sizes gaussian_ids_sorted from I,
 * and calls gsplat_bin_emit with BOTH workspaces (phase 1's must be left untouched in
 * between).  Phase 2 (the tile sort: the depth-ordered intersections emitted as (tile, id)
 * pairs -- or, from 2^24 of them, generated inside the first pass -- and sorted stably by tile;
 * small scenes: tile buckets with per-tile sorts) writes gaussian_ids_sorted [I] and tile_bins
 * [tbx*tby, 2]; the order is identical to a stable sort of gsplat's 64-bit isect_ids. */
size_t gsplat_bin_count_workspace_size(int num_points);
/* Phase-2 workspace for the binning scheme in use (it depends on N and the tile grid; the
 * small-scene tile buckets also on I). */
size_t gsplat_bin_emit_workspace_size_for(int num_points, int64_t num_intersects,
                                          int tile_bounds_x, int tile_bounds_y);
int gsplat_bin_count(int num_points, const float *xys, const float *depths,
                     const int32_t *radii, const int32_t *num_tiles_hit, int tile_bounds_x,
                     int tile_bounds_y, int32_t *d_counts, void *workspace1,
                     size_t workspace1_bytes, void *stream);
/* gsplat_bin_count for a workspace whose depth-sort inputs (depth keys, ids, per-Gaussian
 * binning records) gsplat_fused_preprocess_forward_binned already wrote: the same outputs
 * without reading xys/depths/radii/num_tiles_hit again. */
int gsplat_bin_count_keyed(int num_points, int tile_bounds_x, int tile_bounds_y,
                           int32_t *d_counts, void *workspace1, size_t workspace1_bytes,
                           void *stream);
/* gsplat_bin_count_keyed with the depth-key range carried across calls (d_counts: int32[4],
 * [2] and [3] zeroed by the caller): depth-sort passes over key bits `assume_const` covers --
 * bits an earlier call found constant over the visible depths, e.g. the shared exponent byte --
 * are not launched.  Afterwards d_counts[2] = 1 if this call's visible depth keys do vary in an
 * assumed-constant bit (the order, and every binning output after it, is then wrong: re-bin
 * with assume_const = 0), d_counts[3] = the key bits that vary (the next call's assumption is
 * its complement).  assume_const = 0: gsplat_bin_count_keyed's results. */
int gsplat_bin_count_keyed_ex(int num_points, int tile_bounds_x, int tile_bounds_y,
                              int32_t *d_counts, void *workspace1, size_t workspace1_bytes,
                              uint32_t assume_const, void *stream);
int gsplat_bin_emit(int num_points, int64_t num_intersects, int tile_bounds_x,
                    int tile_bounds_y, int32_t *gaussian_ids_sorted, int32_t *tile_bins,
                    const void *workspace1, size_t workspace1_bytes, void *workspace2,
                    size_t workspace2_bytes, void *stream);
/* Phase 2 split around the host's read of I, so that the GPU is not idle while the host
 * waits for it: gsplat_bin_emit_prelaunch, issued right after phase 1 with buffers sized for
 * `capacity` intersections (e.g. the last call's I plus a margin), launches the part of
 * phase 2 that needs only phase 1's results (the emission into capacity slots, the table
 * cleared; I > capacity emits nothing and leaves the table all-zero).  Then, with the host's I:
 *   I <= capacity: gsplat_bin_emit_finish(..., I, capacity, ...) with the SAME buffers, stream
 *                  and capacity (the workspace layout follows capacity);
 *   I >  capacity: gsplat_bin_emit (or a new prelaunch + finish) into buffers sized for I.
 * gaussian_ids_sorted needs capacity slots; workspace2 gsplat_bin_emit_workspace_size_for(N,
 * capacity, ...) bytes.  Results are identical to gsplat_bin_emit's. */
int gsplat_bin_emit_prelaunch(int num_points, int64_t capacity, int tile_bounds_x,
                              int tile_bounds_y, int32_t *tile_bins, const void *workspace1,
                              size_t workspace1_bytes, void *workspace2, size_t workspace2_bytes,
                              void *stream);
int gsplat_bin_emit_finish(int num_points, int64_t num_intersects, int64_t capacity,
                           int tile_bounds_x, int tile_bounds_y, int32_t *gaussian_ids_sorted,
                           int32_t *tile_bins, const void *workspace1, size_t workspace1_bytes,
                           void *workspace2, size_t workspace2_bytes, void *stream);
/* The whole of phase 2 before the host knows I: the emission and tile sort launched for
 * `capacity` intersections, sorting the device-side I -- so the blend can be launched right
 * behind it and the host reads I (d_counts[1]) only afterwards, while the GPU works.
 * I <= capacity: gaussian_ids_sorted[0, I) and tile_bins are gsplat_bin_emit's exactly.
 * I > capacity: nothing is placed and tile_bins is left all-zero (a blend behind it renders the
 * background and touches no id); the caller re-bins into buffers sized for I (gsplat_bin_emit
 * from the same workspace1).  Buffers as for gsplat_bin_emit_prelaunch.  Returns 2 (nothing
 * launched) when the binning scheme for (num_points, tiles) needs I on the host -- the
 * small-scene tile buckets: use prelaunch + finish there.
 * Replaces, like gsplat_bin_emit, gsplat 0.1.2.1 rasterize.py's map / sort / bin edges. */
/* gsplat_bin_count_keyed_ex + gsplat_bin_emit_speculative in one call (I published to
 * d_counts[1] from the device).  Same outputs and overflow / range-violation semantics as the
 * two calls; the small-scene tile buckets also run capacity-launched here (each bucket kernel
 * returns at once on an overflow, the table cleared).  d_counts int32[4] as
 * gsplat_bin_count_keyed_ex's. */
int gsplat_bin_speculative(int num_points, int64_t capacity, int tile_bounds_x, int tile_bounds_y,
                           int32_t *d_counts, void *workspace1, size_t workspace1_bytes,
                           uint32_t assume_const, int32_t *gaussian_ids_sorted, int32_t *tile_bins,
                           void *workspace2, size_t workspace2_bytes, void *stream);
int gsplat_bin_emit_speculative(int num_points, int64_t capacity, int tile_bounds_x,
                                int tile_bounds_y, int32_t *gaussian_ids_sorted,
                                int32_t *tile_bins, const void *workspace1,
                                size_t workspace1_bytes, void *workspace2, size_t workspace2_bytes,
                                void *stream);

/* ---- rasterization (forward.cu rasterize_forward, backward.cu rasterize_backward) -----
 * colors [N,C], opacity [N] (or [N,1]), background [C]; out_img [H,W,C], final_Ts [H,W],
 * final_idx [H,W] int32.  C == 3 takes the specialised kernel; 1 <= C <= 64 otherwise. */
int gsplat_rasterize_forward(int tile_bounds_x, int tile_bounds_y, int img_height,
                             int img_width, int channels, const int32_t *gaussian_ids_sorted,
                             const int32_t *tile_bins, const float *xys, const float *conics,
                             const float *colors, const float *opacity,
                             const float *background, float *out_img, float *final_Ts,
                             int32_t *final_idx, void *stream);

/* Fused RGB+depth eval forward (no gsplat counterpart): out_img [H,W,3],
 * final_Ts, final_idx exactly as gsplat_rasterize_forward with C = 3, plus out_depth [H,W] =
 * sum of depth * alpha * T -- channel 0 of a second forward with colours = depths and a zero
 * background (gc_model.py:225-236), from the same binning and traversal.  depths [N]. */
int gsplat_rasterize_forward_rgbd(int tile_bounds_x, int tile_bounds_y, int img_height,
                                  int img_width, const int32_t *gaussian_ids_sorted,
                                  const int32_t *tile_bins, const float *xys,
                                  const float *conics, const float *colors,
                                  const float *depths, const float *opacity,
                                  const float *background, float *out_img, float *out_depth,
                                  float *final_Ts, int32_t *final_idx, void *stream);

/* v_output [H,W,C], v_output_alpha [H,W] (may be NULL: an all-zero alpha gradient); gradients v_xy [N,2], v_conic [N,3],
 * v_colors [N,C], v_opacity [N] are fully written.  alpha_max is the backward alpha clamp
 * (gsplat 0.1.x uses 0.99f).  workspace holds the per-Gaussian gradient
 * records the kernel accumulates into (gsplat_rasterize_backward_workspace_size bytes;
 * may be 0 / NULL when that size is 0). */
/* List-split backward (C = 3; no gsplat counterpart).  gsplat's backward walks each tile's
 * whole depth-sorted list from the back, one block per tile; with few tiles (small images) or
 * a few very long lists (real scenes) the longest tiles' waves bound the launch while the rest
 * of the GPU idles.  The chunked backward cuts every tile's walk (list positions up to the
 * last one any of its pixels composites, from final_idx) into parts of `chunk` (a multiple of
 * 64) positions and runs each part as its own waves, the long tiles' parts dispatched first.
 * A part's waves first re-walk the positions behind it computing only transmittance and the
 * colour behind, with the very operations of the full walk, so every wave's per-Gaussian totals
 * are bit-identical to the unsplit walk's (gradients: within fp32 atomic-order rounding, and
 * bit-identical in the deterministic mode).  gsplat_rasterize_chunk_size picks `chunk` (0 = do
 * not split) for a frame; gsplat_rasterize_split_bytes sizes the plan buffer the backward
 * fills at its start (per-tile walk lengths and the (tile, part) dispatch list).
 * chunk <= 0 makes the entry the plain gsplat_rasterize_backward (C = 3). */
int gsplat_rasterize_chunk_size(int tile_bounds_x, int tile_bounds_y, int64_t num_intersects);
size_t gsplat_rasterize_split_bytes(int tile_bounds_x, int tile_bounds_y, int64_t num_intersects,
                                    int chunk);
int gsplat_rasterize_backward_chunked(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, int num_points,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *v_output,
    const float *v_output_alpha, float alpha_max, float *v_xy, float *v_conic, float *v_colors,
    float *v_opacity, int64_t num_intersects, int chunk, void *plan, size_t plan_bytes,
    void *workspace, size_t workspace_bytes, void *stream);
/* The RGB forward (C = 3) that also clears `clear_bytes` (a multiple of 16) at `clear`: the
 * fused training render hands it the per-Gaussian gradient records, which the blend kernel
 * zeroes with the memory bandwidth its VALU-bound loop leaves idle (instead of the preprocess
 * kernel spending ~18 us on it).  With clear_radii != NULL the buffer is 64-B records and
 * record g is cleared only when clear_radii[g] > 0 (the backward touches no other).  With
 * chunk > 0 (gsplat_rasterize_chunk_size) and a plan buffer of gsplat_rasterize_split_bytes, the
 * blend's waves also fill the plan's walk table (each wave's largest final index), so the list-
 * split backward given that plan and plan_filled = 1 skips the kernel that derives it from
 * final_idx.  Below 3,584 tiles the plan also carries the list-split forward (parts of chunk
 * positions blended in their own waves and combined in list order): final_idx equals
 * gsplat_rasterize_forward's bit for bit, final_T and the image within fp32 rounding of the
 * regrouped transmittance product.  chunk < 0: that split forward alone with parts of -chunk
 * positions (a render with no backward: no walk table), plan of
 * gsplat_rasterize_split_bytes(.., -chunk).  chunk == 0: no plan (may be NULL); outputs equal
 * gsplat_rasterize_forward's. */
int gsplat_rasterize_forward_clearing(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    float *out_img, float *final_Ts, int32_t *final_idx, void *clear, size_t clear_bytes,
    const int32_t *clear_radii, int64_t num_intersects, int chunk, void *plan,
    size_t plan_bytes, void *stream);
#ifdef GSPLAT_TEST_HOOKS
/* Test library only: force the list-split chunk (> 0, rounded up to 64), disable it (< 0) or
 * restore the automatic choice (0). */
int gsplat_debug_set_chunk(int chunk);
#endif

size_t gsplat_rasterize_backward_workspace_size(int num_points, int channels);
int gsplat_rasterize_backward(int tile_bounds_x, int tile_bounds_y, int img_height,
                              int img_width, int channels, int num_points,
                              const int32_t *gaussian_ids_sorted, const int32_t *tile_bins,
                              const float *xys, const float *conics, const float *colors,
                              const float *opacity, const float *background,
                              const float *final_Ts, const int32_t *final_idx,
                              const float *v_output, const float *v_output_alpha,
                              float alpha_max, float *v_xy, float *v_conic, float *v_colors,
                              float *v_opacity, void *workspace, size_t workspace_bytes,
                              void *stream);

/* ---- fused training render (no gsplat counterpart; SURVEY.md §8a a1-a3, a10 + caller) ----
 * The reference caller's per-Gaussian glue (gc_model.py:158-215: exp(scales), quats/|quats|,
 * cat(features_dc, features_rest), viewdirs, SH -> clamp(rgb + 0.5, min 0) or sigmoid(dc),
 * sigmoid(opacities)) evaluated inside the projection + SH kernel, and its chain rule inside
 * the backward.  Raw splatfacto parameters in: means3d [N,3], log_scales [N,3], quats [N,4]
 * (unnormalised), opacity_logits [N], features_dc [N,3], features_rest [N, sh_bases-1, 3]
 * (NULL when sh_bases == 1), campos [3] (DEVICE; the camera centre, c2w[:3,3]).
 * Forward writes xys, depths, radii, conics, num_tiles_hit (as gsplat_project_gaussians_forward
 * on the activated inputs), colors [N,3] (clamped SH colour; a colour the clamp raised from
 * below zero is stored as -0.0f so the backward knows it) and opacity [N] (sigmoid).  With
 * grad_records != NULL (gsplat_grad_records_bytes) it zeroes the record of every visible
 * Gaussian (radii > 0) for gsplat_rasterize_backward_records (the fused render passes NULL
 * and lets gsplat_rasterize_forward_clearing clear them instead).  scales_out [N,3] / quats_out [N,4]
 * (optional, testing) receive the activated scales and normalised quaternions.
 * Backward reads the records and writes v_means3d [N,3], v_log_scales [N,3], v_quats [N,4],
 * v_opacity_logits [N] and either v_features_dc [N,3] + v_features_rest [N, sh_bases-1, 3],
 * or -- v_colors != NULL, sh_bases > 1, data-parallel view exchange -- the gradient of the SH
 * colour v_colors [N,3] instead of the two feature gradients (sum them with
 * gsplat_compute_sh_backward_views_split).  Every output is fully written. */
int gsplat_fused_preprocess_forward(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *opacity_logits,
    const float *features_dc, const float *features_rest, const float *viewmat,
    const float *projmat, const float *campos, float fx, float fy, float cx, float cy,
    int img_height, int img_width, int tile_bounds_x, int tile_bounds_y, float clip_thresh,
    float *xys, float *depths, int32_t *radii, float *conics, int32_t *num_tiles_hit,
    float *colors, float *opacity, void *grad_records, float *scales_out, float *quats_out,
    void *stream);
/* The forward above (no records, no debug outputs) that also writes the binning's depth-sort
 * inputs into a gsplat_bin_count workspace (gsplat_bin_count_workspace_size(num_points)
 * bytes), from the projection's registers; follow it with gsplat_bin_count_keyed on that
 * workspace.  Saves the binning's depth-key pass over xys/depths/radii/num_tiles_hit. */
int gsplat_fused_preprocess_forward_binned(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *opacity_logits,
    const float *features_dc, const float *features_rest, const float *viewmat,
    const float *projmat, const float *campos, float fx, float fy, float cx, float cy,
    int img_height, int img_width, int tile_bounds_x, int tile_bounds_y, float clip_thresh,
    float *xys, float *depths, int32_t *radii, float *conics, int32_t *num_tiles_hit,
    float *colors, float *opacity, void *bin_workspace, size_t bin_workspace_bytes,
    void *stream);
/* gsplat_fused_preprocess_forward_binned in two parts for two streams: part 1 = the
 * activations, projection, opacity and the binning's inputs (colors may be NULL); part 2 = the
 * SH colours alone (reads means3d, features_dc, features_rest, campos; writes colors; every
 * projection output and the workspace may be NULL).  Outputs equal the one-kernel forward's
 * bit for bit.  The fused render issues part 2 on a second stream, where the colours' loads
 * (12 K + 24 B per Gaussian) overlap the binning's latency-bound sort passes, joining before
 * the blend.  (Same reference rows as the forward above: gc_model.py:172-215.) */
int gsplat_fused_preprocess_forward_part(
    int part, int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *opacity_logits,
    const float *features_dc, const float *features_rest, const float *viewmat,
    const float *projmat, const float *campos, float fx, float fy, float cx, float cy,
    int img_height, int img_width, int tile_bounds_x, int tile_bounds_y, float clip_thresh,
    float *xys, float *depths, int32_t *radii, float *conics, int32_t *num_tiles_hit,
    float *colors, float *opacity, void *bin_workspace, size_t bin_workspace_bytes,
    void *stream);
int gsplat_fused_preprocess_backward(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *viewmat, const float *projmat,
    const float *campos, float fx, float fy, float cx, float cy, int img_height, int img_width,
    const int32_t *radii, const float *conics, const float *colors, const float *opacity,
    const void *grad_records, float *v_means3d, float *v_log_scales, float *v_quats,
    float *v_opacity_logits, float *v_features_dc, float *v_features_rest, float *v_colors,
    void *stream);

/* The data-parallel view exchange's send record (no gsplat counterpart), packed
 * straight from the raster backward's gradient records: send [3N + 4] = the SH-output colour
 * gradient v_colors [N,3] exactly as gsplat_fused_preprocess_backward writes it (zero for
 * radii <= 0), then the camera centre campos [3], then 0.  Ready right after the raster
 * backward, so the all-gather overlaps the rest of the backward. */
int gsplat_exchange_pack_colors(int num_points, const void *grad_records, size_t records_bytes,
                                const int32_t *radii, const float *colors, const float *campos,
                                float *send, void *stream);

/* The sparse view record (no gsplat counterpart): only the visible Gaussians'
 * colour gradients travel, after a visibility bitmap and its prefix -- 12 B per visible
 * Gaussian + 0.19 B per Gaussian instead of 12 B per Gaussian (c4 garden, 55 % visible: 6.8
 * B).  Layout in floats, W = ceil(N/64): [0,3) camera centre, [3] visible count (uint32
 * bits), [4, 4+2W) uint64 masks (bit b of word w <=> radii[64w+b] > 0), [4+2W, 4+3W) uint32
 * exclusive prefix of their popcounts, [4+3W, 4+3W+3C) the visible Gaussians' v_colors in
 * index order, C >= the count (the capacity the ranks agreed on).
 * gsplat_exchange_sparse_floats: the record's length in floats for capacity C (-1: bad args).
 * gsplat_exchange_sparse_plan: writes the count, masks and prefix from radii (the forward,
 * once radii exist), into send's first 4 + 3W floats; send must hold 4 + 4W floats (the
 * popcounts are staged in the values area, which pack overwrites).
 * gsplat_exchange_pack_sparse: after the raster backward, the camera centre and the values
 * (as gsplat_exchange_pack_colors computes them) into a planned send of >= that length. */
long long gsplat_exchange_sparse_floats(int num_points, long long capacity);
int gsplat_exchange_sparse_plan(int num_points, const int32_t *radii, float *send, void *stream);
int gsplat_exchange_pack_sparse(int num_points, const void *grad_records, size_t records_bytes,
                                const int32_t *radii, const float *colors, const float *campos,
                                float *send, long long capacity, void *stream);
/* gsplat_fused_preprocess_backward in the view-exchange mode (v_colors written, sh_bases > 1)
 * for a rank that renders several views per step: the four geometry gradients are ADDED to
 * v_means3d, v_log_scales, v_quats, v_opacity_logits (the earlier views' sum); v_colors is
 * this view's. */
int gsplat_fused_preprocess_backward_accumulate(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *viewmat, const float *projmat,
    const float *campos, float fx, float fy, float cx, float cy, int img_height, int img_width,
    const int32_t *radii, const float *conics, const float *colors, const float *opacity,
    const void *grad_records, float *v_means3d, float *v_log_scales, float *v_quats,
    float *v_opacity_logits, float *v_colors, void *stream);

/* Single-GPU training step: gsplat_fused_preprocess_backward with the Adam step of the six
 * parameter groups fused in (torch.optim.Adam foreach semantics, exactly gsplat_adam_step's
 * arithmetic).  The gradients stay in registers; means3d, log_scales, quats, opacity_logits,
 * features_dc, features_rest are updated IN PLACE, together with their exp_avgs /
 * exp_avg_sqs (HOST arrays of 6 device pointers, group order as listed); lrs: HOST array of
 * the 6 learning rates; step >= 1 after increment; 0.5 < beta1 < 1.  Every Gaussian is
 * updated (culled ones with a zero gradient, as torch does). */
int gsplat_fused_preprocess_backward_adam(
    int num_points, int sh_bases, int degrees_to_use, float *means3d, float *log_scales,
    float *quats, float *opacity_logits, float *features_dc, float *features_rest,
    const float *viewmat, const float *projmat, const float *campos, float fx, float fy,
    float cx, float cy, int img_height, int img_width, const int32_t *radii, const float *conics,
    const float *colors, const float *opacity, const void *grad_records, float *const *exp_avgs,
    float *const *exp_avg_sqs, const float *lrs, int step, float beta1, float beta2, float eps,
    void *stream);

/* Per-Gaussian gradient records (64 B each) the fused path's rasterize backward accumulates
 * into, as pixel moments over every pixel the Gaussian is composited at (d = xy - pixel,
 * w = vis * v_alpha): floats 0 sum dx w, 1 sum dy w, 2 sum dx^2 w, 3 sum dx dy w, 4 sum dy^2 w,
 * 5-7 v_colors, 8 sum w (= v_opacity), 9-15 unused; gsplat's gradients follow per Gaussian as
 * v_xy = -o (a Sx + b Sy, b Sx + c Sy), v_conic = -o/2 (Sxx, Sxy, Syy) (conic = (a, b, c),
 * o = opacity; v_conic.y doubled without GSPLAT_QUIRK_CONIC_HALF).  gsplat_rasterize_backward_records is gsplat_rasterize_backward (C = 3, default
 * variant, list-split when chunk > 0 as in the _chunked entry; plan_filled = 1: the plan's walk
 * table came from gsplat_rasterize_forward_clearing with the same plan) without the zero fill and
 * without the split into v_xy / v_conic / v_colors / v_opacity -- the records must be zeroed
 * by the caller (gsplat_fused_preprocess_forward does it for the visible Gaussians, the
 * only ones the kernel touches) and are read
 * by gsplat_fused_preprocess_backward. */
size_t gsplat_grad_records_bytes(int num_points);
int gsplat_rasterize_backward_records(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, int num_points,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *v_output,
    const float *v_output_alpha, float alpha_max, int64_t num_intersects, int chunk,
    void *plan, size_t plan_bytes, int plan_filled, void *records, size_t records_bytes,
    void *stream);
/* The training step's L1 photometric loss folded into the blend (no gsplat counterpart: the
 * loss of gc_pipeline.py:477-478 with splatfacto's ssim_lambda = 0, on gc_model.py:222's
 * clamped image when clamp_pred).  The forward is gsplat_rasterize_forward_clearing plus
 * loss[0] = mean over the H x W x 3 image of |clamp(out_img) - gt| (gt [H,W,3]; per-wave
 * partials, one float per wave, gsplat_rasterize_l1_partials_bytes; summed in double); the
 * backward is
 * gsplat_rasterize_backward_records whose upstream image gradient is not read but formed per
 * pixel from (pred = that forward's out_img, gt, grad_loss [1] device scalar): grad_loss/(3HW)
 * * sign(clamp(pred) - gt) * (pred <= 1 when clamp_pred) -- gsplat_l1_ssim_backward's
 * lambda = 0 arithmetic, so the records equal the unfused step's bit for bit.  No alpha
 * gradient. */
size_t gsplat_rasterize_l1_partials_bytes(int tile_bounds_x, int tile_bounds_y);
int gsplat_rasterize_forward_clearing_l1(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    float *out_img, float *final_Ts, int32_t *final_idx, void *clear, size_t clear_bytes,
    const int32_t *clear_radii, int64_t num_intersects, int chunk, void *plan, size_t plan_bytes,
    const float *gt, int clamp_pred, float *partials, size_t partials_bytes, float *loss,
    void *stream);
int gsplat_rasterize_backward_records_l1(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, int num_points,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *pred, const float *gt,
    int clamp_pred, const float *grad_loss, float alpha_max, int64_t num_intersects, int chunk,
    void *plan, size_t plan_bytes, int plan_filled, void *records, size_t records_bytes,
    void *stream);
/* The records -> gsplat's four rasterize gradients (v_xy [N,2], v_conic [N,3] in gsplat's
 * convention (GSPLAT_QUIRK_CONIC_HALF), v_colors [N,3], v_opacity [N]) -- the tail of
 * gsplat_rasterize_backward, for a caller that cleared the records in the forward blend
 * (gsplat_rasterize_forward_clearing) and accumulated them with
 * gsplat_rasterize_backward_records (the drop-in rasterize_gaussians does). */
int gsplat_grad_records_split(int num_points, const void *records, size_t records_bytes,
                              const float *conics, const float *opacity, float *v_xy,
                              float *v_conic, float *v_colors, float *v_opacity, void *stream);

/* ---- test hooks (not part of the gsplat surface) ------------------------------------------
 * Exported only by the test library libgsplat_mi355x_hooks.so (the same sources built with
 * -DGSPLAT_TEST_HOOKS: identical kernels, plus these switches, which select the non-default
 * paths the parity tests cover and the profiling tools' wave log); the shipped
 * libgsplat_mi355x.so runs the shipped configuration only.  (gaussctrl_exp_amd/_lib.py
 * hooks() runs a test against the test library.) */
#ifdef GSPLAT_TEST_HOOKS
/* Measurement hook (not part of the gsplat surface): fwd_pxl must be 1 (the forward's 8x8
 * blocks); bwd_pxl selects the C = 3 backward's geometry: 0 = by frame size (shipped: blocks
 * below 3,584 tiles, strips above), 1 = 8x8 blocks, one pixel per lane, two Gaussians per
 * iteration, 2 = 16x8 strips, two pixels per lane; bwd_flags bits 20-27 = K: the block -> tile
 * order of the blend kernels, chunks of K block slots dealt round-robin over the 8 XCDs (0: the
 * shipped K = 8, 255: plain dispatch order); bits 28-29: the forward's staging pipeline (0: by
 * frame size, shipped -- on below 3,584 tiles; 1 off; 2 on); bit 30: the forward's keep bits
 * off (the list-split backward culls for itself).  Every variant meets the same
 * parity bar (none changes the arithmetic).  Process-wide; (1, 0, 0) is the shipped
 * configuration. */
int gsplat_debug_set_raster_variant(int fwd_pxl, int bwd_pxl, int bwd_flags);
/* 1 while the shipped raster variants are selected (the record-based entries need them). */
int gsplat_debug_raster_variant_is_default(void);

/* Binning dispatch switches (not part of the gsplat surface; every setting gives the identical
 * output, tests cover each).  Each returns the previous setting; -1 (or, for the scheme, -2)
 * only queries.
 * gsplat_debug_depth_key_range: depth-sort passes whose digit is the same for every kept key
 *   (from the keys' AND / OR, found during the first pass) only copy -- from 2^22 keys (1,
 *   shipped), always (2) -- or rank as any pass (0).
 * gsplat_debug_binning_scheme: -1 by size (shipped: tile buckets + per-tile LDS sorts for
 *   scenes of <= 131,072 Gaussians on frames up to 16,447 tiles, else the depth sort + stable
 *   tile sort), 0 depth sort + tile sort, 1 tile buckets.
 *   Must not change between a gsplat_bin_count and its gsplat_bin_emit.
 * gsplat_debug_tile_sort_gen: the tile sort's first pass is generated from the depth-ordered
 *   allotments instead of emitted and re-read from capacities of min_i intersections (shipped
 *   2^24); < 0 only queries.  Must not change between a workspace-size query and its use.
 * gsplat_debug_emit_counts: gsplat_bin_speculative's tile sort takes its first digit counts
 *   from the emission (1, shipped) or from a count launch over the emitted pairs (0). */
int gsplat_debug_depth_key_range(int on);
int gsplat_debug_binning_scheme(int scheme);
long long gsplat_debug_tile_sort_gen(long long min_i);
int gsplat_debug_emit_counts(int on);
/* Profiling hook: the backward blend kernels record per wave {start, end (s_memrealtime,
 * 100 MHz), HW_ID, XCC_ID, work slot} as [waves][5] uint64 into the device buffer (NULL
 * disables); the buffer needs 5 entries per launched wave. */
int gsplat_debug_wave_log(void *buffer);
#endif  /* GSPLAT_TEST_HOOKS */
/* Measurement hook (shipped: bench.py's lane_occupancy): lane-slot accounting of the shipped blend kernels (separate counting instantiations,
 * the shipped code is unchanged).  buffer = device u64[6], accumulated by every later forward
 * (clearing) and record backward launch until called again with NULL:
 * [0] backward lane slots (wave iterations x 128 pixel slots), [1] slots whose pixel is live for
 * the Gaussian (in the image, idx <= final_idx), [2] valid pairs (sigma >= 0, alpha >= 1/255);
 * [3..5] the same for the forward (wave iterations x 2 Gaussians x 64 pixels; live = not yet
 * terminated). */
int gsplat_debug_pair_count(void *buffer);

/* ---- training-step photometric loss -------------------------------------
 * nerfstudio 1.0 splatfacto get_loss_dict's main loss, which the reference's training step
 * computes on every iteration (gc_pipeline.py:477-478):
 *     loss = (1 - lambda) * mean|gt - pred| + lambda * (1 - SSIM(gt, pred))
 * with pytorch_msssim's SSIM (11x11 Gaussian window, 'valid' filtering, data range 1,
 * K = (0.01, 0.03)).  pred / gt: [H, W, C] fp32 (the caller's rgb and gt images, H, W >= 11);
 * window11: HOST pointer to the 11 normalised window weights.  Forward writes partials
 * [2 * gsplat_l1_ssim_num_blocks(H, W)] (scratch), dmaps [3 * C * (H-10) * (W-10)] (kept for
 * the backward) and the loss scalar (device).  Backward reads the upstream gradient scalar
 * from device memory (no host sync) and writes v_pred [H, W, C] (gt gets no gradient).
 * clamp_pred != 0 folds the caller's torch.clamp(rgb, max=1.0) (gc_model.py:222) in: the loss
 * of min(pred, 1), with the gradient masked where pred > 1 (torch's clamp backward). */
int gsplat_l1_ssim_num_blocks(int img_height, int img_width);
int gsplat_l1_ssim_forward(int img_height, int img_width, int channels, const float *pred,
                           const float *gt, const float *window11, float ssim_lambda,
                           int clamp_pred, float *partials, float *dmaps, float *loss,
                           void *stream);
int gsplat_l1_ssim_backward(int img_height, int img_width, int channels, const float *pred,
                            const float *gt, const float *window11, float ssim_lambda,
                            int clamp_pred, const float *dmaps, const float *grad_loss,
                            float *v_pred, void *stream);

/* ---- optimizer step -----------------------------------------------------
 * One torch.optim.Adam step (non-capturable foreach semantics, no weight decay / amsgrad) over
 * up to 8 parameter tensors in ONE launch, as the reference's trainer takes it for the six
 * splatfacto groups (gc_trainer.py:281,298; gc_config.py:58-87).  params / grads / exp_avgs /
 * exp_avg_sqs: HOST arrays of device pointers (fp32, contiguous); numels, lrs: HOST arrays;
 * step: the step number after increment (>= 1); beta1 must lie in (0.5, 1) (torch's lerp
 * formula changes below).  Updates params, exp_avgs, exp_avg_sqs in place. */
int gsplat_adam_step(int num_tensors, float *const *params, const float *const *grads,
                     float *const *exp_avgs, float *const *exp_avg_sqs, const int64_t *numels,
                     const float *lrs, int step, float beta1, float beta2, float eps,
                     void *stream);

#ifdef __cplusplus
}
#endif

#endif /* GSPLAT_MI355X_H */
