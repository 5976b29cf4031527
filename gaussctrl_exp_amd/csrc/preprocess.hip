// preprocess.hip -- the reference caller's per-Gaussian glue fused into the projection and
// SH kernels: the fused training render (no gsplat counterpart; SURVEY.md §8a rows a1-a3,
// a10 plus their caller).
//
// GaussCtrlModel.get_outputs (/root/reference/gaussctrl/gc_model.py:158-215) prepares
// gsplat's inputs with ~10 torch ops per step -- cat(features_dc, features_rest) (:172),
// exp(scales) (:177), quats / |quats| (:178), viewdirs = normalise(means - campos)
// (:197-198), SH -> clamp(rgb + 0.5, min=0) (:200-201) or sigmoid(dc) (:203),
// sigmoid(opacities) (:215) -- and autograd runs their backwards and copies the SH-feature
// gradients out of cat's strided views.  At 1M Gaussians that glue cost more device time
// than the projection, SH and raster-forward kernels together.  The fused path evaluates all
// of it per Gaussian, in registers:
//  * fused_fwd_kernel: raw parameters -> activations (torch's formulas) -> gsplat projection
//    (project_math.h: the same arithmetic as project.hip) -> SH colour straight from the two
//    feature tensors (features_rest staged through LDS with 16-byte loads) -> clamp; writes
//    exactly what binning and rasterization consume, and zeroes the Gaussian's
//    rasterize-backward gradient record when it is visible (no separate memset).
//  * fused_bwd_kernel: gradient record -> projection VJP (project_math.h) -> chain rule
//    through the activations with torch's own backward formulas (exp' = result, sigmoid' =
//    (1 - y) y, the division and vector-norm backwards of the quaternion normalisation, the
//    clamp mask) -> the six raw-parameter gradients, the SH-feature ones written straight
//    into their own contiguous tensors (LDS-staged 16-byte stores).
// Built with -ffp-contract=off (projection bit-identical to project.hip given the same
// activated inputs); the SH helpers carry their own contract pragma (sh_math.h).
#include "adam_math.h"
#include "project_math.h"
#include "sh_math.h"
#include "exchange_layout.h"

namespace gs {
namespace {

constexpr int RECF = 16;  // floats per gradient record (raster.hip REC)

// clamp(x, min=0) that keeps the clamp's backward mask in the sign bit: x < 0 -> -0.0f,
// otherwise x (NaN stays NaN, as torch.clamp).  A -0 colour leaves every rasterizer sum
// unchanged, and the backward passes the gradient exactly where torch's clamp_min backward
// does (x >= 0): non-negative value with a clear sign bit.
__device__ __forceinline__ float clamp0_signed(float x) { return x < 0.f ? -0.f : x; }
__device__ __forceinline__ bool clamp0_passes(float stored) {
  return stored >= 0.f && !__builtin_signbit(stored);
}

// torch.sigmoid on ROCm: 1 / (1 + exp(-x)) in fp32.
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }

struct FusedFwdArgs {
  int n, degrees_to_use;
  const float *means, *log_scales, *quats, *opacity_logits, *features_dc, *features_rest;
  const float *viewmat, *projmat, *campos;
  float *xys, *depths;
  int *radii;
  float *conics;
  int *num_tiles_hit;
  float *colors, *opacity;
  float *records;                // NULL: no backward planned
  float *scales_out, *quats_out;  // debug (activated inputs), NULL normally
  BinKeys bin;                    // bin.keys != NULL: also write the binning's sort inputs
};

struct FusedBwdArgs {
  int n, degrees_to_use;
  const float *means, *log_scales, *quats, *viewmat, *projmat, *campos;
  const int *radii;
  const float *conics, *colors, *opacity, *records;
  float *v_means, *v_log_scales, *v_quats, *v_opacity_logits, *v_dc, *v_rest;
  float *v_colors;  // non-NULL: write the SH-output gradient here instead of v_dc / v_rest
  int accumulate;   // add the four geometry gradients to the outputs' values (v_colors mode)
};

// Adam fused into the backward (single-GPU training step): the six parameter tensors are
// updated in place from the gradients in registers, which are never written to memory.
// Group order = splatfacto's (means, scales, quats, opacities, features_dc, features_rest).
struct FusedAdamArgs {
  float *p[6], *m[6], *v[6];
  float ss[6], bc2s[6];  // lr / (1 - beta1^t), sqrt(1 - beta2^t) (host, double -> float)
  float beta1, beta2, eps;
};

// The caller's activations (gc_model.py:177-178): exp(scales), quats / |quats|.
__device__ __forceinline__ void activate(const float *__restrict__ ls, const float *__restrict__ q,
                                         long long g, float s[3], float qr[4], float qn[4],
                                         float &norm) {
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = expf(ls[3 * g + k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) qr[k] = q[4 * g + k];
  // torch's vector-norm reduction order for a 4-vector (measured bit-identical on MI355X:
  // tests/test_gpu_fused.py records it), so qn equals the caller's quats / |quats| exactly
  norm = sqrtf((qr[0] * qr[0] + qr[1] * qr[1]) + (qr[2] * qr[2] + qr[3] * qr[3]));
#pragma unroll
  for (int k = 0; k < 4; ++k) qn[k] = qr[k] / norm;
}

// activate() on values already in registers
__device__ __forceinline__ void activate_vals(const float ls[3], const float q[4], float s[3],
                                              float qr[4], float qn[4], float &norm) {
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = expf(ls[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) qr[k] = q[k];
  norm = sqrtf((qr[0] * qr[0] + qr[1] * qr[1]) + (qr[2] * qr[2] + qr[3] * qr[3]));
#pragma unroll
  for (int k = 0; k < 4; ++k) qn[k] = qr[k] / norm;
}

// SH basis along the caller's view direction: viewdirs = (means - campos) / |means - campos|
// (gc_model.py:197-198), which gsplat renormalises in-kernel (sh.cuh).
__device__ __forceinline__ int view_basis(int degrees_to_use, float p0, float p1, float p2,
                                          const float *__restrict__ campos, float *b) {
  typedef __attribute__((address_space(4))) const float cfloat;  // uniform: scalar loads
  cfloat *cp = (cfloat *)campos;
  float dx = p0 - cp[0], dy = p1 - cp[1], dz = p2 - cp[2];
  // torch's reduction order for the norm of a 3-vector (measured bit-identical on MI355X)
  const float dn = sqrtf((dx * dx + dz * dz) + dy * dy);
  dx = dx / dn;
  dy = dy / dn;
  dz = dz / dn;
  return sh_basis(degrees_to_use, dx, dy, dz, b);
}

// Camera matrices through the constant address space: uniform scalar loads (lgkmcnt), which
// leave the vector-memory counter to the per-Gaussian loads and the features_rest slab.
__device__ __forceinline__ void load_cam_scalar(Cam &c, const float *viewmat,
                                                const float *projmat) {
  typedef __attribute__((address_space(4))) const float cfloat;
  cfloat *vm = (cfloat *)viewmat;
  cfloat *pm = (cfloat *)projmat;
#pragma unroll
  for (int k = 0; k < 12; ++k) c.vm[k] = vm[k];
#pragma unroll
  for (int k = 0; k < 16; ++k) c.pm[k] = pm[k];
}

// One block's forward.  FULL (every block but a partial last one, slab 16-B aligned): no branch
// between this Gaussian's own loads, the slab's loads and the projection, so the projection
// waits only for its own inputs (vmcnt counts in issue order and a branch in between makes the
// compiler drain the counter) while the features_rest slab stays in flight; the slab lands in
// LDS after the projection.  Otherwise: guarded loads and stage_rows.
// PART: 0 the whole forward; 1 the projection part (activations, projection, opacity, the
// binning's inputs) without the SH colours; 2 the SH colours alone (gsplat_fused_preprocess_
// forward_part: the two parts on two streams, the colours' 216 B per Gaussian overlapping the
// binning's latency-bound sort passes).  Each part's outputs are the whole forward's, bit for bit
// (the same code; a part only leaves out the other's loads and stores).
template <int K, bool FULL, int PART = 0>
__device__ __forceinline__ void fused_fwd_body(const FusedFwdArgs &a, const ProjParams &pp,
                                               float *smem, long long g0, int cnt) {
  constexpr int RROW = (K - 1) * 3;  // features_rest floats per Gaussian
  constexpr int RP = RROW | 1;       // odd LDS pitch: conflict-free per-thread rows
  constexpr int THR = sh_threads(K);
  constexpr int NV = THR * RROW / 4;  // the full slab's float4s
  constexpr int PER = (NV + THR - 1) / THR;
  const int t = threadIdx.x;
  const bool live = FULL || t < cnt;
  const long long g = g0 + (live ? t : 0);
  constexpr bool PROJ = PART != 2, COLOURS = PART != 1;
  Cam cam;
  if constexpr (PROJ) load_cam_scalar(cam, a.viewmat, a.projmat);
  float p0, p1, p2, dc[3] = {0.f, 0.f, 0.f}, lsv[3] = {0.f, 0.f, 0.f},
                    qv[4] = {0.f, 0.f, 0.f, 0.f}, ologit = 0.f;
  p0 = a.means[3 * g];
  p1 = a.means[3 * g + 1];
  p2 = a.means[3 * g + 2];
  if constexpr (PROJ) {
#pragma unroll
    for (int k = 0; k < 3; ++k) lsv[k] = a.log_scales[3 * g + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) qv[k] = a.quats[4 * g + k];
    ologit = a.opacity_logits[g];
  }
  if constexpr (COLOURS) {
#pragma unroll
    for (int c = 0; c < 3; ++c) dc[c] = a.features_dc[3 * g + c];
  }
  const float *rest_src = K > 1 ? a.features_rest + g0 * RROW : nullptr;
  float4 slab[FULL && K > 1 && COLOURS ? PER : 1];
  if constexpr (FULL && K > 1 && COLOURS) {
    const float4 *s4 = reinterpret_cast<const float4 *>(rest_src);
#pragma unroll
    for (int u = 0; u < PER; ++u) slab[u] = s4[min(u * THR + t, NV - 1)];  // clamped: no branch
  }
  if (PROJ && live) {
    float s[3], qr[4], qn[4], norm;
    activate_vals(lsv, qv, s, qr, qn, norm);
    ProjOut o;
    project_one(cam, pp, p0, p1, p2, s[0], s[1], s[2], qn[0], qn[1], qn[2], qn[3], o);
    a.xys[2 * g] = o.xy[0];
    a.xys[2 * g + 1] = o.xy[1];
    a.depths[g] = o.depth;
    a.radii[g] = o.radius;
    a.conics[3 * g] = o.con[0];
    a.conics[3 * g + 1] = o.con[1];
    a.conics[3 * g + 2] = o.con[2];
    a.num_tiles_hit[g] = o.tiles;
    if (a.bin.keys) {  // binning.hip depth_keys_kernel's outputs, from the registers
      const bool vis = o.radius > 0;
      a.bin.keys[g] = vis ? __float_as_uint(o.depth) : 0xFFFFFFFFu;
      a.bin.vals[g] = (uint32_t)g;
      const int c = vis ? o.tiles : 0;
      uint4 q = {c > 0 ? (uint32_t)c : 0u, 0u, 0u, 0u};
      if (c > 0) {
        int x0, x1, y0, y1;
        tile_bbox(o.xy[0], o.xy[1], (float)o.radius, pp.tbx, pp.tby, x0, x1, y0, y1);
        q.y = (uint32_t)x0 | ((uint32_t)y0 << 16);
        q.z = (uint32_t)x1 | ((uint32_t)y1 << 16);
      }
      a.bin.rec[g] = q;
    }
    if (a.records && o.radius > 0) {  // only visible Gaussians receive raster atomics
      // the whole 64-B record (one full line: no partial-line read-modify-write)
      float4 *r = reinterpret_cast<float4 *>(a.records + g * RECF);
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      r[0] = z;
      r[1] = z;
      r[2] = z;
      r[3] = z;
    }
    a.opacity[g] = sigmoidf(ologit);  // gc_model.py:215
    if (a.scales_out) {
#pragma unroll
      for (int k = 0; k < 3; ++k) a.scales_out[3 * g + k] = s[k];
    }
    if (a.quats_out) {
#pragma unroll
      for (int k = 0; k < 4; ++k) a.quats_out[4 * g + k] = qn[k];
    }
  }
  if constexpr (!COLOURS) {
    return;
  } else if constexpr (K == 1) {  // sh_degree 0: sigmoid(features_dc) (gc_model.py:203)
    if (live) {
#pragma unroll
      for (int c = 0; c < 3; ++c) a.colors[3 * g + c] = sigmoidf(dc[c]);
    }
  } else {
    if constexpr (FULL) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int k = u * THR + t;
        if (NV % THR == 0 || k < NV) {
          smem[sh_lds_index<RROW, RP>(4 * k)] = slab[u].x;
          smem[sh_lds_index<RROW, RP>(4 * k + 1)] = slab[u].y;
          smem[sh_lds_index<RROW, RP>(4 * k + 2)] = slab[u].z;
          smem[sh_lds_index<RROW, RP>(4 * k + 3)] = slab[u].w;
        }
      }
    } else {
      stage_rows<RROW, RP, THR>(rest_src, cnt, smem);
    }
    __syncthreads();
    if (live) {
      float b[25];
      const int nb = view_basis(a.degrees_to_use, p0, p1, p2, a.campos, b);
      const float *row = smem + t * RP;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v =
            sh_channel<K>(b, nb, [&](int k) { return k == 0 ? dc[c] : row[(k - 1) * 3 + c]; });
        a.colors[3 * g + c] = clamp0_signed(v + 0.5f);  // gc_model.py:201
      }
    }
  }
}

template <int K>
__global__ __launch_bounds__(sh_threads(K)) void fused_fwd_kernel(FusedFwdArgs a, ProjParams pp) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int THR = sh_threads(K);
  const long long g0 = (long long)blockIdx.x * THR;
  const int cnt = (int)min((long long)THR, (long long)a.n - g0);
  const bool aligned =
      K == 1 || ((((uintptr_t)(a.features_rest + g0 * (K - 1) * 3)) & 15) == 0 &&
                 (THR * (K - 1) * 3) % 4 == 0);
  if (cnt == THR && aligned)
    fused_fwd_body<K, true>(a, pp, smem, g0, cnt);
  else
    fused_fwd_body<K, false>(a, pp, smem, g0, cnt);
}

// the two parts of fused_fwd_kernel (PART 1 / 2 of fused_fwd_body)
template <int K>
__global__ __launch_bounds__(sh_threads(K)) void fused_fwd_proj_kernel(FusedFwdArgs a,
                                                                       ProjParams pp) {
  constexpr int THR = sh_threads(K);
  const long long g0 = (long long)blockIdx.x * THR;
  const int cnt = (int)min((long long)THR, (long long)a.n - g0);
  if (cnt == THR)
    fused_fwd_body<K, true, 1>(a, pp, nullptr, g0, cnt);
  else
    fused_fwd_body<K, false, 1>(a, pp, nullptr, g0, cnt);
}

template <int K>
__global__ __launch_bounds__(sh_threads(K)) void fused_fwd_sh_kernel(FusedFwdArgs a,
                                                                     ProjParams pp) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int THR = sh_threads(K);
  const long long g0 = (long long)blockIdx.x * THR;
  const int cnt = (int)min((long long)THR, (long long)a.n - g0);
  const bool aligned =
      K == 1 || ((((uintptr_t)(a.features_rest + g0 * (K - 1) * 3)) & 15) == 0 &&
                 (THR * (K - 1) * 3) % 4 == 0);
  if (cnt == THR && aligned)
    fused_fwd_body<K, true, 2>(a, pp, smem, g0, cnt);
  else
    fused_fwd_body<K, false, 2>(a, pp, smem, g0, cnt);
}

template <int K, bool ADAM = false>
__global__ __launch_bounds__(sh_threads(K)) void fused_bwd_kernel(FusedBwdArgs a, ProjParams pp,
                                                                  FusedAdamArgs o = {}) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int RROW = (K - 1) * 3;
  constexpr int RP = RROW | 1;
  constexpr int THR = sh_threads(K);
  const long long g0 = (long long)blockIdx.x * THR;
  const int cnt = (int)min((long long)THR, (long long)a.n - g0);
  const bool rest_out = K > 1 && a.v_colors == nullptr;
  const int t = threadIdx.x;
  if (t < cnt) {
    const long long g = g0 + t;
    float vmean[3] = {0.f, 0.f, 0.f}, vls[3] = {0.f, 0.f, 0.f}, vq[4] = {0.f, 0.f, 0.f, 0.f};
    float vlogit = 0.f, vc[3] = {0.f, 0.f, 0.f};
    const bool vis = a.radii[g] > 0;
    const float p0 = a.means[3 * g], p1 = a.means[3 * g + 1], p2 = a.means[3 * g + 2];
    if (vis) {
      const float4 *rec = reinterpret_cast<const float4 *>(a.records + g * RECF);
      const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2];
      const float rv[9] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x};
      const float ca = a.conics[3 * g], cb = a.conics[3 * g + 1], cc = a.conics[3 * g + 2];
      const float y = a.opacity[g];
      // raster gradients from the record's moments (common.h record_grads)
      const RasterGrads rg =
          record_grads(rv, ca, cb, cc, y, !(pp.quirks & GSPLAT_QUIRK_CONIC_HALF));
      float s[3], qr[4], qn[4], norm;
      activate(a.log_scales, a.quats, g, s, qr, qn, norm);
      Cam cam;
      load_cam(cam, a.viewmat, a.projmat);
      float cv[6];
      cov3d_one(pp.glob_scale, s[0], s[1], s[2], qn[0], qn[1], qn[2], qn[3], cv);
      ProjGrad pg;
      project_backward_one(cam, pp, p0, p1, p2, s[0], s[1], s[2], qn[0], qn[1], qn[2], qn[3],
                           cv, ca, cb, cc, rg.vxy[0], rg.vxy[1], 0.f, rg.vconic[0], rg.vconic[1],
                           rg.vconic[2], pg);
#pragma unroll
      for (int k = 0; k < 3; ++k) vmean[k] = pg.vmean[k];
      // exp backward: grad * result
#pragma unroll
      for (int k = 0; k < 3; ++k) vls[k] = pg.vscale[k] * s[k];
      // quats / norm: div backward (grad / other; -grad * ((self / other) / other), summed
      // over the broadcast dim) + linalg_vector_norm backward (self * (grad / norm))
      float gn = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) gn += -pg.vquat[k] * ((qr[k] / norm) / norm);
#pragma unroll
      for (int k = 0; k < 4; ++k) vq[k] = pg.vquat[k] / norm + qr[k] * (gn / norm);
      // sigmoid backward: grad * (1 - y) * y
      vlogit = rg.vopacity * (1.f - y) * y;
      const float *vrgb = rg.vrgb;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float col = a.colors[3 * g + c];
        vc[c] = K == 1 ? vrgb[c] * (1.f - col) * col : (clamp0_passes(col) ? vrgb[c] : 0.f);
      }
    }
    float vdc[3] = {vc[0], vc[1], vc[2]};  // K == 1: sigmoid backward already applied
    float b[25];
    b[0] = 0.f;
    int nb = 0;  // culled: every coefficient gradient is 0
    if constexpr (K > 1) {
      if (!a.v_colors) {
        if (vis) nb = view_basis(a.degrees_to_use, p0, p1, p2, a.campos, b);
        // gsplat compute_sh_backward: v_coeffs[k][c] = basis_k * v_rgb[c] for k < nb, else 0
#pragma unroll
        for (int c = 0; c < 3; ++c) vdc[c] = b[0] * vc[c];
      }
    }
    if constexpr (ADAM) {
      const float w1 = 1.f - o.beta1, w2 = 1.f - o.beta2;
      auto upd = [&](int grp, long long idx, float gv) {
        float pv = o.p[grp][idx], mv = o.m[grp][idx], vv = o.v[grp][idx];
        adam_elem(pv, gv, mv, vv, w1, o.beta2, w2, o.ss[grp], o.bc2s[grp], o.eps);
        o.p[grp][idx] = pv;
        o.m[grp][idx] = mv;
        o.v[grp][idx] = vv;
      };
      // a group's W floats of this Gaussian as one vector access per array (p, m, v): 12-B
      // rows as dwordx3, the quaternion's 16-B row as dwordx4 when the three arrays are
      // 16-B aligned -- a third of the per-element dword accesses
      struct __attribute__((aligned(4))) F3 { float x[3]; };
      struct __attribute__((aligned(16))) F4 { float x[4]; };
      auto upd3 = [&](int grp, const float gv[3]) {
        F3 pv = reinterpret_cast<const F3 *>(o.p[grp])[g];
        F3 mv = reinterpret_cast<const F3 *>(o.m[grp])[g];
        F3 vv = reinterpret_cast<const F3 *>(o.v[grp])[g];
#pragma unroll
        for (int k = 0; k < 3; ++k)
          adam_elem(pv.x[k], gv[k], mv.x[k], vv.x[k], w1, o.beta2, w2, o.ss[grp], o.bc2s[grp],
                    o.eps);
        reinterpret_cast<F3 *>(o.p[grp])[g] = pv;
        reinterpret_cast<F3 *>(o.m[grp])[g] = mv;
        reinterpret_cast<F3 *>(o.v[grp])[g] = vv;
      };
      upd3(0, vmean);
      upd3(1, vls);
      if (((((uintptr_t)o.p[2]) | ((uintptr_t)o.m[2]) | ((uintptr_t)o.v[2])) & 15) == 0) {
        F4 pv = reinterpret_cast<const F4 *>(o.p[2])[g];
        F4 mv = reinterpret_cast<const F4 *>(o.m[2])[g];
        F4 vv = reinterpret_cast<const F4 *>(o.v[2])[g];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          adam_elem(pv.x[k], vq[k], mv.x[k], vv.x[k], w1, o.beta2, w2, o.ss[2], o.bc2s[2], o.eps);
        reinterpret_cast<F4 *>(o.p[2])[g] = pv;
        reinterpret_cast<F4 *>(o.m[2])[g] = mv;
        reinterpret_cast<F4 *>(o.v[2])[g] = vv;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) upd(2, 4 * g + k, vq[k]);
      }
      upd(3, g, vlogit);
      upd3(4, vdc);
    } else {
      if (a.accumulate) {  // a further view of this rank's step (exchange multi-view mode)
#pragma unroll
        for (int k = 0; k < 3; ++k) vmean[k] += a.v_means[3 * g + k];
#pragma unroll
        for (int k = 0; k < 3; ++k) vls[k] += a.v_log_scales[3 * g + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) vq[k] += a.v_quats[4 * g + k];
        vlogit += a.v_opacity_logits[g];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) a.v_means[3 * g + k] = vmean[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) a.v_log_scales[3 * g + k] = vls[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) a.v_quats[4 * g + k] = vq[k];
      a.v_opacity_logits[g] = vlogit;
      if (K == 1 || !a.v_colors) {
#pragma unroll
        for (int c = 0; c < 3; ++c) a.v_dc[3 * g + c] = vdc[c];
      }
    }
    if constexpr (K > 1) {
      if (a.v_colors) {  // data-parallel view exchange sums the SH gradient later
#pragma unroll
        for (int c = 0; c < 3; ++c) a.v_colors[3 * g + c] = vc[c];
      } else {
      float *row = smem + t * RP;
#pragma unroll
      for (int k = 1; k < K; ++k) {
        const float bk = k < nb ? b[k] : 0.f;
        row[(k - 1) * 3 + 0] = bk * vc[0];
        row[(k - 1) * 3 + 1] = bk * vc[1];
        row[(k - 1) * 3 + 2] = bk * vc[2];
      }
      }
    }
  }
  if constexpr (K > 1) {
    if (rest_out) {
      __syncthreads();
      if constexpr (ADAM) {  // features_rest: coalesced slab update from the LDS gradient rows
        const int total = cnt * RROW;
        const long long off = g0 * RROW;
        const float w1 = 1.f - o.beta1, w2 = 1.f - o.beta2;
        float *P = o.p[5] + off, *M = o.m[5] + off, *V = o.v[5] + off;
        auto grad_at = [&](int k) {
          const int r = k / RROW;
          return smem[r * RP + (k - r * RROW)];
        };
        int k0 = 0;
        if (((((uintptr_t)P) | ((uintptr_t)M) | ((uintptr_t)V)) & 15) == 0) {
          // 16-byte vectors: the slab of a block starts 16-byte aligned (256 x 180 B)
          typedef float f4 __attribute__((ext_vector_type(4)));
          const int nv = total >> 2;
          for (int q = threadIdx.x; q < nv; q += THR) {
            f4 pv = reinterpret_cast<f4 *>(P)[q], mv = reinterpret_cast<f4 *>(M)[q],
               vv = reinterpret_cast<f4 *>(V)[q];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float pj = pv[j], mj = mv[j], vj = vv[j];
              adam_elem(pj, grad_at(4 * q + j), mj, vj, w1, o.beta2, w2, o.ss[5], o.bc2s[5],
                        o.eps);
              pv[j] = pj;
              mv[j] = mj;
              vv[j] = vj;
            }
            reinterpret_cast<f4 *>(P)[q] = pv;
            reinterpret_cast<f4 *>(M)[q] = mv;
            reinterpret_cast<f4 *>(V)[q] = vv;
          }
          k0 = nv << 2;
        }
        for (int k = k0 + threadIdx.x; k < total; k += THR) {
          float pv = P[k], mv = M[k], vv = V[k];
          adam_elem(pv, grad_at(k), mv, vv, w1, o.beta2, w2, o.ss[5], o.bc2s[5], o.eps);
          P[k] = pv;
          M[k] = mv;
          V[k] = vv;
        }
      } else {
        store_cols<RROW, 0, RP, THR>(smem, cnt, a.v_rest + g0 * RROW);
      }
    }
  }
}

bool valid_bases(int K) { return K == 1 || K == 4 || K == 9 || K == 16 || K == 25; }
int degree_of(int K) { return K == 1 ? 0 : K == 4 ? 1 : K == 9 ? 2 : K == 16 ? 3 : 4; }

}  // namespace
}  // namespace gs

using namespace gs;

#define FUSED_DISPATCH(KERNEL, ARGS)                                                       \
  switch (K) {                                                                            \
    case 1: hipLaunchKernelGGL(KERNEL<1>, grid, dim3(thr), smem, st, ARGS, pp); break;    \
    case 4: hipLaunchKernelGGL(KERNEL<4>, grid, dim3(thr), smem, st, ARGS, pp); break;    \
    case 9: hipLaunchKernelGGL(KERNEL<9>, grid, dim3(thr), smem, st, ARGS, pp); break;    \
    case 16: hipLaunchKernelGGL(KERNEL<16>, grid, dim3(thr), smem, st, ARGS, pp); break;  \
    default: hipLaunchKernelGGL(KERNEL<25>, grid, dim3(thr), smem, st, ARGS, pp); break;  \
  }

static int fused_forward_impl(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *opacity_logits,
    const float *features_dc, const float *features_rest, const float *viewmat,
    const float *projmat, const float *campos, float fx, float fy, float cx, float cy,
    int img_height, int img_width, int tile_bounds_x, int tile_bounds_y, float clip_thresh,
    float *xys, float *depths, int32_t *radii, float *conics, int32_t *num_tiles_hit,
    float *colors, float *opacity, void *grad_records, float *scales_out, float *quats_out,
    void *bin_workspace, size_t bin_workspace_bytes, void *stream, int part = 0) {
  const int K = sh_bases;
  if (num_points < 0 || !valid_bases(K) || degrees_to_use < 0 || degrees_to_use > degree_of(K) ||
      img_height <= 0 || img_width <= 0 || tile_bounds_x <= 0 || tile_bounds_y <= 0 ||
      (num_points > 0 && K > 1 && (!features_rest || !campos))) {
    set_error("fused_preprocess_forward: bad args (N=%d sh_bases=%d degrees_to_use=%d H=%d W=%d "
              "tiles=%dx%d)", num_points, sh_bases, degrees_to_use, img_height, img_width,
              tile_bounds_x, tile_bounds_y);
    return 1;
  }
  if (num_points == 0) return 0;
  FusedFwdArgs args{num_points, degrees_to_use, means3d, log_scales, quats, opacity_logits,
                    features_dc, features_rest, viewmat, projmat, campos, xys, depths, radii,
                    conics, num_tiles_hit, colors, opacity, (float *)grad_records, scales_out,
                    quats_out, BinKeys{nullptr, nullptr, nullptr, 0}};
  if (bin_workspace) {
    args.bin = bin_keys_view(bin_workspace, num_points);
    if (bin_workspace_bytes < args.bin.bytes || tile_bounds_x > 65535 || tile_bounds_y > 65535) {
      set_error("fused_preprocess_forward_binned: binning workspace %zu < %zu bytes (or tiles "
                "%dx%d)", bin_workspace_bytes, args.bin.bytes, tile_bounds_x, tile_bounds_y);
      return 1;
    }
  }
  const ProjParams pp = make_proj_params(fx, fy, cx, cy, 1.f, clip_thresh, img_height,
                                         img_width, tile_bounds_x, tile_bounds_y);
  const int thr = sh_threads(K);
  const dim3 grid(cdiv(num_points, thr));
  const size_t smem = K > 1 ? (size_t)thr * (((K - 1) * 3) | 1) * sizeof(float) : 0;
  hipStream_t st = (hipStream_t)stream;
  if (part == 1) {
    const size_t smem = 0;  // (no features_rest slab)
    FUSED_DISPATCH(fused_fwd_proj_kernel, args);
  } else if (part == 2) {
    FUSED_DISPATCH(fused_fwd_sh_kernel, args);
  } else {
    FUSED_DISPATCH(fused_fwd_kernel, args);
  }
  return check_launch("fused_preprocess_forward");
}

extern "C" int gsplat_fused_preprocess_forward(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *opacity_logits,
    const float *features_dc, const float *features_rest, const float *viewmat,
    const float *projmat, const float *campos, float fx, float fy, float cx, float cy,
    int img_height, int img_width, int tile_bounds_x, int tile_bounds_y, float clip_thresh,
    float *xys, float *depths, int32_t *radii, float *conics, int32_t *num_tiles_hit,
    float *colors, float *opacity, void *grad_records, float *scales_out, float *quats_out,
    void *stream) {
  return fused_forward_impl(num_points, sh_bases, degrees_to_use, means3d, log_scales, quats,
                            opacity_logits, features_dc, features_rest, viewmat, projmat, campos,
                            fx, fy, cx, cy, img_height, img_width, tile_bounds_x, tile_bounds_y,
                            clip_thresh, xys, depths, radii, conics, num_tiles_hit, colors,
                            opacity, grad_records, scales_out, quats_out, nullptr, 0, stream);
}

extern "C" int gsplat_fused_preprocess_forward_binned(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *opacity_logits,
    const float *features_dc, const float *features_rest, const float *viewmat,
    const float *projmat, const float *campos, float fx, float fy, float cx, float cy,
    int img_height, int img_width, int tile_bounds_x, int tile_bounds_y, float clip_thresh,
    float *xys, float *depths, int32_t *radii, float *conics, int32_t *num_tiles_hit,
    float *colors, float *opacity, void *bin_workspace, size_t bin_workspace_bytes,
    void *stream) {
  if (!bin_workspace) {
    set_error("fused_preprocess_forward_binned: no binning workspace");
    return 1;
  }
  return fused_forward_impl(num_points, sh_bases, degrees_to_use, means3d, log_scales, quats,
                            opacity_logits, features_dc, features_rest, viewmat, projmat, campos,
                            fx, fy, cx, cy, img_height, img_width, tile_bounds_x, tile_bounds_y,
                            clip_thresh, xys, depths, radii, conics, num_tiles_hit, colors,
                            opacity, nullptr, nullptr, nullptr, bin_workspace,
                            bin_workspace_bytes, stream);
}

extern "C" int gsplat_fused_preprocess_forward_part(
    int part, int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *opacity_logits,
    const float *features_dc, const float *features_rest, const float *viewmat,
    const float *projmat, const float *campos, float fx, float fy, float cx, float cy,
    int img_height, int img_width, int tile_bounds_x, int tile_bounds_y, float clip_thresh,
    float *xys, float *depths, int32_t *radii, float *conics, int32_t *num_tiles_hit,
    float *colors, float *opacity, void *bin_workspace, size_t bin_workspace_bytes,
    void *stream) {
  if (part != 1 && part != 2) {
    set_error("fused_preprocess_forward_part: part %d (1 = projection, 2 = colours)", part);
    return 1;
  }
  if (part == 1 && !bin_workspace) {
    set_error("fused_preprocess_forward_part: no binning workspace");
    return 1;
  }
  if (num_points > 0 && (part == 2 ? !colors || !means3d || !features_dc
                                   : !xys || !depths || !radii || !conics || !num_tiles_hit ||
                                         !opacity || !means3d || !log_scales || !quats ||
                                         !opacity_logits || !viewmat || !projmat)) {
    set_error("fused_preprocess_forward_part: missing tensors for part %d", part);
    return 1;
  }
  return fused_forward_impl(num_points, sh_bases, degrees_to_use, means3d, log_scales, quats,
                            opacity_logits, features_dc, features_rest, viewmat, projmat, campos,
                            fx, fy, cx, cy, img_height, img_width, tile_bounds_x, tile_bounds_y,
                            clip_thresh, xys, depths, radii, conics, num_tiles_hit, colors,
                            opacity, nullptr, nullptr, nullptr, part == 1 ? bin_workspace : nullptr,
                            bin_workspace_bytes, stream, part);
}

static int fused_backward_impl(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *viewmat, const float *projmat,
    const float *campos, float fx, float fy, float cx, float cy, int img_height, int img_width,
    const int32_t *radii, const float *conics, const float *colors, const float *opacity,
    const void *grad_records, float *v_means3d, float *v_log_scales, float *v_quats,
    float *v_opacity_logits, float *v_features_dc, float *v_features_rest, float *v_colors,
    int accumulate, void *stream) {
  const int K = sh_bases;
  if (num_points < 0 || !valid_bases(K) || degrees_to_use < 0 || degrees_to_use > degree_of(K) ||
      img_height <= 0 || img_width <= 0 ||
      (num_points > 0 && (!grad_records || (K > 1 && !campos) ||
                          (K > 1 && !v_colors && !v_features_rest)))) {
    set_error("fused_preprocess_backward: bad args (N=%d sh_bases=%d degrees_to_use=%d H=%d W=%d)",
              num_points, sh_bases, degrees_to_use, img_height, img_width);
    return 1;
  }
  if (num_points == 0) return 0;
  // 0.5: the shipped packed backward accumulates 2 v_conic (raster.hip split_grads_kernel)
  FusedBwdArgs args{num_points, degrees_to_use, means3d, log_scales, quats, viewmat, projmat,
                    campos, radii, conics, colors, opacity, (const float *)grad_records,
                    v_means3d, v_log_scales, v_quats, v_opacity_logits, v_features_dc,
                    v_features_rest, K > 1 ? v_colors : nullptr, accumulate};
  const ProjParams pp = make_proj_params(fx, fy, cx, cy, 1.f, 0.f, img_height, img_width, 1, 1);
  const int thr = sh_threads(K);
  const dim3 grid(cdiv(num_points, thr));
  const size_t smem = (K > 1 && !args.v_colors) ? (size_t)thr * (((K - 1) * 3) | 1) * sizeof(float)
                                                : 0;
  hipStream_t st = (hipStream_t)stream;
  FUSED_DISPATCH(fused_bwd_kernel, args);
  return check_launch("fused_preprocess_backward");
}

extern "C" int gsplat_fused_preprocess_backward(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *viewmat, const float *projmat,
    const float *campos, float fx, float fy, float cx, float cy, int img_height, int img_width,
    const int32_t *radii, const float *conics, const float *colors, const float *opacity,
    const void *grad_records, float *v_means3d, float *v_log_scales, float *v_quats,
    float *v_opacity_logits, float *v_features_dc, float *v_features_rest, float *v_colors,
    void *stream) {
  return fused_backward_impl(num_points, sh_bases, degrees_to_use, means3d, log_scales, quats,
                             viewmat, projmat, campos, fx, fy, cx, cy, img_height, img_width,
                             radii, conics, colors, opacity, grad_records, v_means3d,
                             v_log_scales, v_quats, v_opacity_logits, v_features_dc,
                             v_features_rest, v_colors, 0, stream);
}

extern "C" int gsplat_fused_preprocess_backward_accumulate(
    int num_points, int sh_bases, int degrees_to_use, const float *means3d,
    const float *log_scales, const float *quats, const float *viewmat, const float *projmat,
    const float *campos, float fx, float fy, float cx, float cy, int img_height, int img_width,
    const int32_t *radii, const float *conics, const float *colors, const float *opacity,
    const void *grad_records, float *v_means3d, float *v_log_scales, float *v_quats,
    float *v_opacity_logits, float *v_colors, void *stream) {
  if (sh_bases <= 1 || (num_points > 0 && (!v_colors || !v_means3d || !v_log_scales ||
                                           !v_quats || !v_opacity_logits))) {
    set_error("fused_preprocess_backward_accumulate: needs sh_bases > 1 and v_colors (the view "
              "exchange), N=%d sh_bases=%d", num_points, sh_bases);
    return 1;
  }
  return fused_backward_impl(num_points, sh_bases, degrees_to_use, means3d, log_scales, quats,
                             viewmat, projmat, campos, fx, fy, cx, cy, img_height, img_width,
                             radii, conics, colors, opacity, grad_records, v_means3d,
                             v_log_scales, v_quats, v_opacity_logits, nullptr, nullptr, v_colors,
                             1, stream);
}

// The data-parallel view exchange's record (exchange.ShViewExchange), straight from the raster
// backward's gradient records: send[0, 3N) = the SH-output colour gradient exactly as
// fused_bwd_kernel<K > 1> writes v_colors (record colour sums through the clamp mask kept in
// the colours' sign bit; zero for culled Gaussians), send[3N, 3N + 3) = the camera centre,
// send[3N + 3] = 0.  It exists as soon as the raster backward is done, so its all-gather
// overlaps fused_bwd_kernel and the geometry all-reduce instead of following them.
__global__ __launch_bounds__(256) void exchange_pack_kernel(int n, const float *__restrict__ rec,
                                                            const int *__restrict__ radii,
                                                            const float *__restrict__ colors,
                                                            const float *__restrict__ campos,
                                                            float *__restrict__ send) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (g < 3 && blockIdx.x == 0) send[3LL * n + g] = campos[g];
  if (g == 3) send[3LL * n + 3] = 0.f;
  if (g >= n) return;
  float v[3] = {0.f, 0.f, 0.f};
  if (radii[g] > 0) {
    const float4 r1 = reinterpret_cast<const float4 *>(rec + g * RECF)[1];
    const float rgb[3] = {r1.y, r1.z, r1.w};  // REC_R, REC_G, REC_B (record_grads' vrgb)
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = clamp0_passes(colors[3 * g + c]) ? rgb[c] : 0.f;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) send[3 * g + c] = v[c];
}

extern "C" int gsplat_exchange_pack_colors(int num_points, const void *grad_records,
                                           size_t records_bytes, const int32_t *radii,
                                           const float *colors, const float *campos, float *send,
                                           void *stream) {
  if (num_points < 0 || (size_t)num_points * RECF * sizeof(float) > records_bytes ||
      !campos || !send || (num_points > 0 && (!grad_records || !radii || !colors))) {
    set_error("exchange_pack_colors: bad args (N=%d records %zu bytes)", num_points,
              records_bytes);
    return 1;
  }
  hipLaunchKernelGGL(exchange_pack_kernel, dim3(cdiv(num_points + 4, 256)), dim3(256), 0,
                     (hipStream_t)stream, num_points, (const float *)grad_records, radii, colors,
                     campos, send);
  return check_launch("exchange_pack_colors");
}

// The sparse view record (exchange_layout.h), for views that see a fraction of the scene
// (c4 garden: 55 % visible): the masks, their prefix and the count depend only on radii, so
// gsplat_exchange_sparse_plan runs in the forward and the count's all-gather (the ranks
// agree on the capacity) completes long before the backward packs the values.
// xs_mask_kernel: one wave per 64 Gaussians -- the ballot is the mask word, its popcount goes
// to a scratch word in the (not yet written) values area, which xs_scan_kernel scans into the
// prefix slots.  (Round 5 first scanned the prefix slots in place: a workgroup summing the
// words before its chunk then raced the earlier workgroups rewriting theirs -- wrong prefixes
// and a wrong total, seen as garbage capacities from the third step of a gloo rehearsal.)
__global__ __launch_bounds__(256) void xs_mask_kernel(int n, const int *__restrict__ radii,
                                                      float *__restrict__ send) {
  const long long W = xs_words(n);
  const long long w = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (w >= W) return;  // (uniform per wave)
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  const unsigned long long m = __ballot(g < n && radii[g] > 0);
  if ((threadIdx.x & 63) == 0) {
    reinterpret_cast<unsigned long long *>(send + XS_HDR)[w] = m;
    reinterpret_cast<uint32_t *>(send + XS_HDR + 3 * W)[w] = (uint32_t)__popcll(m);
  }
}

__device__ __forceinline__ uint32_t xs_wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// The exclusive scan of the W per-word counts (the scratch words) into the prefix slots,
// XS_CHUNK words per workgroup: each workgroup first sums the counts of every word before its
// chunk (L2-resident; the last one of a 5M-Gaussian record reads ~78K words), then scans its
// chunk; the last workgroup writes the total into the header.
constexpr int XS_CHUNK = 4096;
__global__ __launch_bounds__(1024) void xs_scan_kernel(long long W, float *__restrict__ send) {
  constexpr int PER = XS_CHUNK / 1024;
  uint32_t *c = reinterpret_cast<uint32_t *>(send + XS_HDR + 2 * W);           // prefix slots
  const uint32_t *cnt = reinterpret_cast<const uint32_t *>(send + XS_HDR + 3 * W);  // counts
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t base_s;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long c0 = (long long)blockIdx.x * XS_CHUNK;
  uint32_t before = 0;
  for (long long k = threadIdx.x; k < c0; k += 1024) before += cnt[k];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) before += __shfl_xor(before, o, 64);
  if (threadIdx.x == 0) base_s = 0;
  __syncthreads();
  if (lane == 0) atomicAdd(&base_s, before);
  const long long s0 = c0 + (long long)threadIdx.x * PER;
  uint32_t v[PER], tot = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    v[k] = s0 + k < W ? cnt[s0 + k] : 0u;
    tot += v[k];
  }
  const uint32_t inc = xs_wave_incl_scan(tot);
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();  // (also: every wave has read its counts and added to base_s)
  uint32_t wpre = 0, all = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t x = wsum[j];
    wpre += j < wv ? x : 0u;
    all += x;
  }
  uint32_t run = base_s + wpre + inc - tot;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (s0 + k < W) c[s0 + k] = run;
    run += v[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
    reinterpret_cast<uint32_t *>(send)[3] = base_s + all;
}

// The values: each visible Gaussian's colour gradient (as exchange_pack_kernel computes it) at
// its row; the camera centre into the header.
__global__ __launch_bounds__(256) void xs_pack_kernel(int n, const float *__restrict__ rec,
                                                      const int *__restrict__ radii,
                                                      const float *__restrict__ colors,
                                                      const float *__restrict__ campos,
                                                      float *__restrict__ send, long long cap) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < 3) send[threadIdx.x] = campos[threadIdx.x];
  if (g >= n || radii[g] <= 0) return;
  const long long W = xs_words(n);
  const unsigned long long m = reinterpret_cast<const unsigned long long *>(send + XS_HDR)[g >> 6];
  const long long pos = (long long)reinterpret_cast<const uint32_t *>(send + XS_HDR + 2 * W)[g >> 6] +
                        __popcll(m & ((1ull << (g & 63)) - 1ull));
  if (pos >= cap) return;
  const float4 r1 = reinterpret_cast<const float4 *>(rec + g * RECF)[1];
  const float rgb[3] = {r1.y, r1.z, r1.w};
  float *vals = send + xs_values_at(n);
#pragma unroll
  for (int c = 0; c < 3; ++c) vals[3 * pos + c] = clamp0_passes(colors[3 * g + c]) ? rgb[c] : 0.f;
}

extern "C" long long gsplat_exchange_sparse_floats(int num_points, long long capacity) {
  if (num_points < 0 || capacity < 0 || capacity > num_points) return -1;
  return xs_values_at(num_points) + 3 * capacity;
}

extern "C" int gsplat_exchange_sparse_plan(int num_points, const int32_t *radii, float *send,
                                           void *stream) {
  if (num_points < 0 || !send || (num_points > 0 && !radii)) {
    set_error("exchange_sparse_plan: bad args (N=%d)", num_points);
    return 1;
  }
  hipStream_t st = (hipStream_t)stream;
  const long long W = xs_words(num_points);
  if (W > 0)
    hipLaunchKernelGGL(xs_mask_kernel, dim3((unsigned)cdiv(W * 64, 256)), dim3(256), 0, st,
                       num_points, radii, send);
  hipLaunchKernelGGL(xs_scan_kernel, dim3((unsigned)max(1LL, (W + XS_CHUNK - 1) / XS_CHUNK)),
                     dim3(1024), 0, st, W, send);
  return check_launch("exchange_sparse_plan");
}

extern "C" int gsplat_exchange_pack_sparse(int num_points, const void *grad_records,
                                           size_t records_bytes, const int32_t *radii,
                                           const float *colors, const float *campos,
                                           float *send, long long capacity, void *stream) {
  if (num_points < 0 || (size_t)num_points * RECF * sizeof(float) > records_bytes ||
      !campos || !send || capacity < 0 || capacity > num_points ||
      (num_points > 0 && (!grad_records || !radii || !colors))) {
    set_error("exchange_pack_sparse: bad args (N=%d records %zu bytes capacity %lld)",
              num_points, records_bytes, capacity);
    return 1;
  }
  hipLaunchKernelGGL(xs_pack_kernel, dim3(cdiv(num_points + 3, 256)), dim3(256), 0,
                     (hipStream_t)stream, num_points, (const float *)grad_records, radii, colors,
                     campos, send, capacity);
  return check_launch("exchange_pack_sparse");
}

extern "C" int gsplat_fused_preprocess_backward_adam(
    int num_points, int sh_bases, int degrees_to_use, float *means3d, float *log_scales,
    float *quats, float *opacity_logits, float *features_dc, float *features_rest,
    const float *viewmat, const float *projmat, const float *campos, float fx, float fy,
    float cx, float cy, int img_height, int img_width, const int32_t *radii, const float *conics,
    const float *colors, const float *opacity, const void *grad_records, float *const *exp_avgs,
    float *const *exp_avg_sqs, const float *lrs, int step, float beta1, float beta2, float eps,
    void *stream) {
  const int K = sh_bases;
  if (num_points < 0 || !valid_bases(K) || degrees_to_use < 0 || degrees_to_use > degree_of(K) ||
      img_height <= 0 || img_width <= 0 || step < 1 || !(beta1 > 0.5f && beta1 < 1.f) ||
      !(beta2 >= 0.f && beta2 < 1.f) || !exp_avgs || !exp_avg_sqs || !lrs ||
      (num_points > 0 && (!grad_records || (K > 1 && (!campos || !features_rest))))) {
    set_error("fused_preprocess_backward_adam: bad args (N=%d sh_bases=%d degrees_to_use=%d "
              "step=%d)", num_points, sh_bases, degrees_to_use, step);
    return 1;
  }
  if (num_points == 0) return 0;
  FusedBwdArgs args{num_points, degrees_to_use, means3d, log_scales, quats, viewmat, projmat,
                    campos, radii, conics, colors, opacity, (const float *)grad_records,
                    nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  FusedAdamArgs o{};
  float *params[6] = {means3d, log_scales, quats, opacity_logits, features_dc, features_rest};
  // torch non-capturable Adam: bias corrections in double on the host (as gsplat_adam_step)
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  for (int k = 0; k < 6; ++k) {
    o.p[k] = params[k];
    o.m[k] = exp_avgs[k];
    o.v[k] = exp_avg_sqs[k];
    o.ss[k] = (float)(lrs[k] / bc1);
    o.bc2s[k] = (float)sqrt(bc2);
  }
  o.beta1 = beta1;
  o.beta2 = beta2;
  o.eps = eps;
  const ProjParams pp = make_proj_params(fx, fy, cx, cy, 1.f, 0.f, img_height, img_width, 1, 1);
  const int thr = sh_threads(K);
  const dim3 grid(cdiv(num_points, thr));
  const size_t smem = K > 1 ? (size_t)thr * (((K - 1) * 3) | 1) * sizeof(float) : 0;
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
#define ADAM_CASE(KK)                                                                      \
  case KK:                                                                                 \
    hipLaunchKernelGGL((fused_bwd_kernel<KK, true>), grid, dim3(thr), smem, st, args, pp, o); \
    break;
    ADAM_CASE(1)
    ADAM_CASE(4)
    ADAM_CASE(9)
    ADAM_CASE(16)
    ADAM_CASE(25)
#undef ADAM_CASE
  }
  return check_launch("fused_preprocess_backward_adam");
}

