// raster.hip -- per-tile front-to-back alpha blending (forward) and its reverse-order
// backward, for gfx950.
//
// Replaces gsplat 0.1.2.1 _C.rasterize_forward / _C.rasterize_backward (forward.cu /
// backward.cu; semantics SURVEY.md Appendix A9/A10), reached from
// /root/reference/gaussctrl/gc_model.py:208-220 (RGB + alpha) and :225-236 (depth).
//
// MI355X mapping (per-pixel serial compositing: VALU-issue bound, no MFMA):
//  * A 16x16 tile is split into independent wave rectangles (wave_rect): the forward uses
//    four 8x8 blocks, the backward two 16x8 strips with two pixels per lane.  Each wave
//    stages its own copy of the tile's sorted Gaussians in its own LDS slice, 64 at a time
//    (one Gaussian per lane, coalesced id loads; colour loaded only if kept), so a wave
//    whose pixels have all terminated leaves early and no workgroup barrier is executed.
//    (One wave per tile would serialise a 2.8k-Gaussian tile on one wave.)
//  * While staging, each lane culls its Gaussian against the wave's rectangle with the
//    exact minimum of sigma over the rectangle (touches_rect) and the survivors are
//    compacted in order with a ballot + mbcnt prefix, so the per-pixel loop only visits
//    Gaussians that can pass gsplat's alpha >= 1/255 test somewhere in the rectangle.  The
//    cull keeps a rounding margin, so results are unchanged bit for bit.
//  * Forward (raster_fwd3u_kernel): two staged Gaussians per iteration -- their sigma /
//    exp / alpha are independent; the blend is applied in list order, branch-free.
//  * Backward (shipped: raster_bwd3p_kernel<1>, 16x8 strips, 2 pixels per lane): the lane's
//    two pixels are a float2 pair blended branch-free; per Gaussian the lane folds them into
//    9 partial sums (sigma-gradient moments, colour and opacity terms), the wave
//    reduce-scatters the 9 sums (common.h reduce_rec: permlane32/16 swaps + 3 DPP steps) so
//    that 9 lanes each hold one total, and ONE 9-lane atomic instruction adds them to the
//    Gaussian's 64-byte gradient record; a split kernel then writes gsplat's
//    v_xy / v_conic / v_colors / v_opacity tensors.
//  * Every variant evaluates sigma and exp(-sigma) through the same helpers (gs_sigma*,
//    gs_vis*), so forward and backward take identical per-pixel decisions.
//  * C != 3 (gsplat nd_rasterize): one pixel per lane, 4 waves per tile, register
//    accumulators sized by a compile-time channel bound.
#include "common.h"

#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <type_traits>

namespace gs {
namespace {

constexpr float ALPHA_MIN = 1.f / 255.f;
// The backward's record atomics use 32-bit element offsets (id * REC + slot < 2^31).
constexpr int MAX_BWD_POINTS = 1 << 27;
constexpr int REC = 16;  // floats per gradient record: x y a b c r g b o + pad = 64 B
constexpr int SPLIT_WAVES = 4;  // walk-table entries per tile (list-split plan; split_work_kernel)

// Deterministic backward (gsplat_set_deterministic): every wave's per-Gaussian totals
// (reduce18 / reduce_rec: a fixed reduction order, so run-independent) are added as exact
// integers instead of fp32 atomics.  A total v is quantised to X = trunc(v * 2^80), split into
// three signed 40-bit limbs (v ~ l0 2^-80 + l1 2^-40 + l2), and each limb is added to a 64-bit
// integer accumulator; integer addition is associative, so the sums -- and every gradient
// downstream -- are bit-identical from run to run whatever order the waves finish in, and
// det_finish_kernel converts them into the usual float records.  The resolution (2^-80 ~ 8e-25)
// is relative to nothing: a mean-reduced loss's 1e-9 wave totals keep ~50 significant bits
// (a fixed 2^-32 step lost them).  |v| is clamped below 2^40; a limb sum stays below
// 2^63 for up to 2^22 totals per Gaussian and field (an 8x8 block per total: 2^28 pixels).
constexpr int DET_LIMBS = 3;
__device__ __forceinline__ void det_add(unsigned long long *acc, float v) {
  const uint32_t u = __float_as_uint(v);
  int e = (int)((u >> 23) & 0xff);
  if (e == 0) return;                 // zero or denormal (< 2^-126: below the resolution)
  if (e > 126 + 40) e = 126 + 40;     // |v| < 2^40 (inf / NaN saturate)
  const unsigned long long m = (u & 0x7fffffu) | 0x800000u;  // v = m 2^(e - 150)
  const int sh = e - 70;                                      // X = v 2^80 = m 2^(e - 70)
  unsigned __int128 X;
  if (sh >= 0) X = (unsigned __int128)m << sh;
  else X = sh > -64 ? (unsigned __int128)(m >> -sh) : 0;
  constexpr unsigned long long M40 = (1ull << 40) - 1;
  long long l0 = (long long)((unsigned long long)X & M40);
  long long l1 = (long long)((unsigned long long)(X >> 40) & M40);
  long long l2 = (long long)(unsigned long long)(X >> 80);
  if (u >> 31) {
    l0 = -l0;
    l1 = -l1;
    l2 = -l2;
  }
  atomicAdd(acc, (unsigned long long)l0);
  atomicAdd(acc + 1, (unsigned long long)l1);
  atomicAdd(acc + 2, (unsigned long long)l2);
}
__global__ __launch_bounds__(256) void det_finish_kernel(int n,
                                                         const unsigned long long *__restrict__ det,
                                                         float *__restrict__ rec) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= n) return;
#pragma unroll
  for (int k = 0; k < REC_FIELDS; ++k) {
    const unsigned long long *a = det + ((size_t)g * REC_FIELDS + k) * DET_LIMBS;
    const double v = ((double)(long long)a[2] + (double)(long long)a[1] * 0x1p-40) +
                     (double)(long long)a[0] * 0x1p-80;
    rec[(size_t)g * REC + k] = (float)v;
  }
}
bool g_det = false;
// The deterministic accumulators (debug mode only): one buffer per device, allocated on first
// use and grown as needed.  A use (DetLease) holds a process-wide lock from the clear to the
// enqueue of det_finish_kernel, and the next use -- on any stream or thread -- waits for the
// event recorded after the previous one's finish before clearing, so two backwards in flight
// never share the accumulators.  Growing synchronises the device first (no queued kernel still
// reads the old buffer).
constexpr int DET_MAX_DEVICES = 64;
struct DetState {
  unsigned long long *buf = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;
};
std::mutex g_det_mu;
DetState g_det_dev[DET_MAX_DEVICES];
struct DetLease {
  std::unique_lock<std::mutex> lock;
  DetState *s = nullptr;
  unsigned long long *buf = nullptr;
  hipStream_t st = nullptr;
  DetLease(int n, hipStream_t stream) : lock(g_det_mu), st(stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= DET_MAX_DEVICES) {
      set_error("deterministic backward: no usable device");
      return;
    }
    s = &g_det_dev[dev];
    const size_t need = (size_t)n * REC_FIELDS * DET_LIMBS * sizeof(unsigned long long);
    if (!s->done) note(hipEventCreateWithFlags(&s->done, hipEventDisableTiming), "hipEventCreate");
    else note(hipStreamWaitEvent(st, s->done, 0), "hipStreamWaitEvent");
    if (need > s->cap) {
      if (s->buf) {
        note(hipDeviceSynchronize(), "hipDeviceSynchronize");
        note(hipFree(s->buf), "hipFree");
      }
      s->buf = nullptr;
      s->cap = 0;
      if (hipMalloc(&s->buf, need) == hipSuccess) s->cap = need;
      else s->buf = nullptr;
    }
    if (s->buf) note(hipMemsetAsync(s->buf, 0, need, st), "hipMemsetAsync");
    buf = s->buf;
  }
  // call after det_finish_kernel has been enqueued on st
  void finish() {
    if (s && s->done) note(hipEventRecord(s->done, st), "hipEventRecord");
  }
};
constexpr int FWD_PXL = 1;  // forward: 8x8 blocks, two Gaussians per iteration (4 waves/tile)
// backward geometry (gsplat_debug_set_raster_variant's bwd_pxl): 1 = 8x8 blocks, one pixel per
// lane, two Gaussians per iteration (raster_bwd8_kernel); 2 = 16x8 strips, two pixels per lane
// (raster_bwd3p_kernel); 0 = by frame size, see bwd_geometry()
constexpr int BWD_PXL = 0;  // 0: by frame size (bwd_geometry)
// Tuning / ablation knobs (gsplat_debug_set_raster_variant); defaults are the shipped ones.
int g_fwd_pxl = FWD_PXL, g_bwd_pxl = BWD_PXL, g_bwd_flags = 0;
// forward staging pipelined one batch ahead (the PF instantiation, see RawG): -1 by frame
// size (below 3,584 tiles, where the longest waves bound the launch), 0 off, 1 on
// (gsplat_debug_set_raster_variant flags bits 28-29: 0 auto, 1 off, 2 on).  (The same pipeline
// in the 8x8 backward measured no gain: c3 0.132 -> 0.134 ms, c2 0.123 -> 0.125 ms; its
// EAGER staging already overlaps the data loads, and its blend per batch is longer.)
int g_pf_mode = -1;
// the forward's culls handed to the list-split backward (KeepSrc); debug flag bit 30 turns it off
bool g_keep_bits = true;
static bool pipelined_staging(int tbx, int tby) {
  return g_pf_mode < 0 ? (long long)tbx * tby < 3584 : g_pf_mode > 0;
}

struct __attribute__((aligned(16))) GStage {
  float x, y, ha, b;  // mean, 0.5*conic.a, conic.b
  float hc, o, r, g;  // 0.5*conic.c, opacity, colour
  float bl;
  int idx;  // position in the tile's sorted list
  int id;   // Gaussian id
  float d;  // depth (fused RGB+depth forward only)
  // (round 4: the order {mean, conic | hc, o, idx, id | colour, d}, which lets the backward
  // issue all three row reads at the top of an iteration, measured slower in the forward --
  // 0.145 -> 0.149 ms at the headline, backward unchanged -- and was not kept)
};

typedef float f2 __attribute__((ext_vector_type(2)));

// Staged record t of a wave's LDS slice.  The slice's base is made wave-uniform where it is
// taken (readfirstlane of the wave index), so a blend iteration forms the address in SALU and
// one v_mov instead of a 64-bit vector multiply-add (v_mad_u64_u32) per read.
__device__ __forceinline__ GStage stage_at(const GStage *stage, int t) { return stage[t]; }

// sigma = 0.5 (a dx^2 + c dy^2) + b dx dy, evaluated as fma(fma(c/2, dy, b dx), dy, a/2 dx^2)
// with explicit fmas.  EVERY blend kernel below (scalar or packed, forward or backward) uses
// exactly this rounding, so the backward re-derives the forward's per-pixel decisions
// (sigma >= 0, alpha >= 1/255) bit for bit.  hA = (ha*dx)*dx and bdx = b*dx are per
// (Gaussian, lane): a lane's pixels share one column.
__device__ __forceinline__ float gs_sigma(float hc, float bdx, float hA, float dy) {
  return fmaf(fmaf(hc, dy, bdx), dy, hA);
}
// exp(-sigma) with the hardware exp2 (gsplat: __expf).
constexpr float NEG_LOG2E = -0x1.715476p+0f;
__device__ __forceinline__ float gs_vis(float sigma) {
  return __builtin_amdgcn_exp2f(sigma * NEG_LOG2E);
}

__device__ __forceinline__ f2 vfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
template <typename V>
__device__ __forceinline__ V gs_sigma2v(float hc, float bdx, float hA, V dy) {
  return vfma(vfma(V(hc), dy, V(bdx)), dy, V(hA));
}
template <typename V>
__device__ __forceinline__ V gs_vis2v(V sigma) {
  const V e = sigma * NEG_LOG2E;
  return V{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
}

// Exactness-preserving cull of one Gaussian against the wave's pixel-centre rectangle
// [rx0,rx1] x [ry0,ry1].  With d = xy - p ranging over the box [dx0,dx1] x [dy0,dy1],
// sigma(p) = 0.5 q(d), q = a dx^2 + 2 b dx dy + c dy^2, is convex for a positive-definite
// conic, so its minimum over the box is 0 when the mean lies inside, else the smallest of the
// four edge minima (each a clamped 1-D minimisation).  The Gaussian is dropped only when that
// minimum, lowered by a rounding margin proportional to the magnitude of q's terms plus an
// absolute 1e-3, still makes o * exp(-sigma) < 1/255 -- i.e. when gsplat's per-pixel test
// rejects it at every pixel of the rectangle.  A Gaussian with o < 1/255 is never composited
// (alpha <= o).  Non-positive-definite conics and NaNs are kept.  Compared with an isotropic
// (smallest-eigenvalue) bound this removes ~42 % of the per-wave iterations at the headline
// size: elongated Gaussians no longer count as touching rectangles they only pass near.
__device__ __forceinline__ float q_edge(float e, float lo, float hi, float diag_e, float diag_f,
                                        float b, float &mag) {
  // min over f in [lo, hi] of diag_e e^2 + 2 b e f + diag_f f^2 (diag_f > 0)
  const float f = fminf(fmaxf(-b * e / diag_f, lo), hi);
  const float t0 = diag_e * e * e, t1 = 2.f * b * e * f, t2 = diag_f * f * f;
  mag = t0 + fabsf(t1) + t2;
  return t0 + t1 + t2;
}
__device__ __forceinline__ bool touches_rect(float gx, float gy, float a, float b, float c,
                                             float o, float rx0, float rx1, float ry0,
                                             float ry1) {
  if (!(o >= ALPHA_MIN)) return false;
  if (!(a > 0.f) || !(a * c - b * b > 0.f)) return true;  // not positive definite (or NaN)
  const float dx0 = gx - rx1, dx1 = gx - rx0, dy0 = gy - ry1, dy1 = gy - ry0;
  if (dx0 <= 0.f && dx1 >= 0.f && dy0 <= 0.f && dy1 >= 0.f) return true;  // mean inside
  float m0, m1, m2, m3;
  const float q0 = q_edge(dx0, dy0, dy1, a, c, b, m0), q1 = q_edge(dx1, dy0, dy1, a, c, b, m1);
  const float q2 = q_edge(dy0, dx0, dx1, c, a, b, m2), q3 = q_edge(dy1, dx0, dx1, c, a, b, m3);
  float q = q0, m = m0;
  if (q1 < q) { q = q1; m = m1; }
  if (q2 < q) { q = q2; m = m2; }
  if (q3 < q) { q = q3; m = m3; }
  const float sigma_lb = 0.5f * (q - 1e-5f * m) - 1e-3f;
  return !(sigma_lb > __logf(255.f * o));
}

// The same cull as touches_rect, branch-free for the staging loops: every lane evaluates all
// of it (the wave executes the union of the branches anyway), the clamped minimiser of each
// edge uses the hardware reciprocal instead of an IEEE division (~10 instructions each), and
// log(255 o) the hardware log2 (255 o >= 1 for every Gaussian that is not dropped, so no
// denormal scaling).  Still exactness-preserving: a perturbed minimiser f' gives
// q(f') >= q(f*) only by diag_f (f' - f*)^2, a relative 2^-44 for an ulp-level error of f,
// and the log error is ~1e-7 -- both far inside the rounding margin (1e-5 |terms| + 1e-3)
// the bound already subtracts.  Non-positive-definite conics and NaNs are kept.
__device__ __forceinline__ float q_edge_r(float e, float lo, float hi, float diag_e, float rdiag_f,
                                          float diag_f, float b, float &mag) {
  const float f = fminf(fmaxf(-b * e * rdiag_f, lo), hi);
  const float t0 = diag_e * e * e, t1 = 2.f * b * e * f, t2 = diag_f * f * f;
  mag = t0 + fabsf(t1) + t2;
  return t0 + t1 + t2;
}
__device__ __forceinline__ bool touches_rect_bf(float gx, float gy, float a, float b, float c,
                                                float o, float rx0, float rx1, float ry0,
                                                float ry1) {
  const float dx0 = gx - rx1, dx1 = gx - rx0, dy0 = gy - ry1, dy1 = gy - ry0;
  const float ra = __builtin_amdgcn_rcpf(a), rc = __builtin_amdgcn_rcpf(c);
  float m0, m1, m2, m3;
  const float q0 = q_edge_r(dx0, dy0, dy1, a, rc, c, b, m0);
  const float q1 = q_edge_r(dx1, dy0, dy1, a, rc, c, b, m1);
  const float q2 = q_edge_r(dy0, dx0, dx1, c, ra, a, b, m2);
  const float q3 = q_edge_r(dy1, dx0, dx1, c, ra, a, b, m3);
  float q = q0, m = m0;
  if (q1 < q) { q = q1; m = m1; }
  if (q2 < q) { q = q2; m = m2; }
  if (q3 < q) { q = q3; m = m3; }
  const float sigma_lb = 0.5f * (q - 1e-5f * m) - 1e-3f;
  const bool far = sigma_lb > __builtin_amdgcn_logf(255.f * o) * 0x1.62e430p-1f;  // ln 2
  const bool pd = a > 0.f && a * c - b * b > 0.f;  // false for NaN
  const bool inside = dx0 <= 0.f && dx1 >= 0.f && dy0 <= 0.f && dy1 >= 0.f;
  return o >= ALPHA_MIN && (!pd || inside || !far);
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Stage this lane's Gaussian (list position idx) if it can touch the wave's rectangle.
// Returns keep; fills s.  EAGER: after the id, every load of the Gaussian -- mean, conic, opacity
// AND colour -- is issued at once, so staging costs two dependent memory round trips (id,
// then the rest) instead of four (id, opacity, conic + mean, then the colour of the kept
// ones); the empty asm makes the colour a use before the keep branch, so the compiler cannot
// sink its load into that branch.
//
// EAGER = false (the forward kernels): the branchy cull and the colour loaded only for kept
// Gaussians -- the forward's 8x8 blocks keep few of the staged ones, and the eager form's
// extra live registers cost it an occupancy level (62 -> 66 VGPRs: 0.132 -> 0.137 ms at the
// headline), while the backward gains (0.316 -> 0.313 ms).
template <bool EAGER = false>
__device__ __forceinline__ bool stage_gaussian(int idx, const int *__restrict__ gids,
                                               const float2 *__restrict__ xys,
                                               const float *__restrict__ conics,
                                               const float *__restrict__ colors,
                                               const float *__restrict__ opacity, float rx0,
                                               float rx1, float ry0, float ry1, GStage &s) {
  const int g = gids[idx];
  const float2 xy = xys[g];
  const float a = conics[3 * g], b = conics[3 * g + 1], c = conics[3 * g + 2];
  const float o = opacity[g];
  if constexpr (!EAGER) {
    const bool keep = touches_rect(xy.x, xy.y, a, b, c, o, rx0, rx1, ry0, ry1);
    if (keep) {
      s.x = xy.x;
      s.y = xy.y;
      s.ha = 0.5f * a;
      s.b = b;
      s.hc = 0.5f * c;
      s.o = o;
      s.r = colors[3 * g];
      s.g = colors[3 * g + 1];
      s.bl = colors[3 * g + 2];
      s.idx = idx;
      s.id = g;
    }
    return keep;
  }
  float cr = colors[3 * g], cg = colors[3 * g + 1], cb = colors[3 * g + 2];
  const bool keep = touches_rect_bf(xy.x, xy.y, a, b, c, o, rx0, rx1, ry0, ry1);
  asm volatile("" : "+v"(cr), "+v"(cg), "+v"(cb));
  if (keep) {
    s.x = xy.x;
    s.y = xy.y;
    s.ha = 0.5f * a;
    s.b = b;
    s.hc = 0.5f * c;
    s.o = o;
    s.r = cr;
    s.g = cg;
    s.bl = cb;
    s.idx = idx;
    s.id = g;
  }
  return keep;
}

// Software-pipelined staging (the PF forward, frames below 3,584 tiles): a batch's data is
// loaded (RawG, all of it, whatever the cull decides) one batch ahead and its ids two batches
// ahead, so a wave walking a long list overlaps both dependent memory round trips of the next
// batch with the blending of this one instead of waiting for them every 64 positions.  Worth it
// where the longest waves bound the launch (small frames: c3 bear forward 0.124 -> 0.094 ms);
// on full frames the 12 extra VGPRs (one occupancy level) and the loads of culled Gaussians'
// colours cost more (headline forward 0.125 -> 0.144 ms).
struct RawG {
  float2 xy;
  float a, b, c, o, r, g, bl;
};
__device__ __forceinline__ RawG raw_load(int g, const float2 *__restrict__ xys,
                                         const float *__restrict__ conics,
                                         const float *__restrict__ colors,
                                         const float *__restrict__ opacity) {
  RawG q;
  q.xy = xys[g];
  q.a = conics[3 * g];
  q.b = conics[3 * g + 1];
  q.c = conics[3 * g + 2];
  q.o = opacity[g];
  q.r = colors[3 * g];
  q.g = colors[3 * g + 1];
  q.bl = colors[3 * g + 2];
  return q;
}
// stage_gaussian's cull and fill on prefetched data (BF: the branch-free cull of the backward)
template <bool BF>
__device__ __forceinline__ bool stage_raw(const RawG &q, bool live, int idx, int g, float rx0,
                                          float rx1, float ry0, float ry1, GStage &s) {
  const bool keep =
      live && (BF ? touches_rect_bf(q.xy.x, q.xy.y, q.a, q.b, q.c, q.o, rx0, rx1, ry0, ry1)
                  : touches_rect(q.xy.x, q.xy.y, q.a, q.b, q.c, q.o, rx0, rx1, ry0, ry1));
  if (keep) {
    s.x = q.xy.x;
    s.y = q.xy.y;
    s.ha = 0.5f * q.a;
    s.b = q.b;
    s.hc = 0.5f * q.c;
    s.o = q.o;
    s.r = q.r;
    s.g = q.g;
    s.bl = q.bl;
    s.idx = idx;
    s.id = g;
  }
  return keep;
}
// The pipeline state: ids of batch k+1 (loaded) and k+2 (in flight), data of batch k+1 (in
// flight).
struct StagePipe {
  int g_next, g_after;
  RawG r_next;
};

// ---- keep bits: the forward's culls handed to the backward --------------------------------
// Every forward wave (one 8x8 block of a tile) records the ballot of its cull per 64-position
// batch: word k of block slot wt of tile t (positions range.x + 64 k .. + 63, bit m for
// range.x + 64 k + m) lives at kbits[wt * kbw + (range.x >> 6) + t + k] -- collision-free
// between tiles (a tile's last word index is below the next tile's first), kbw = I / 64 + T + 2
// words per block slot.  Words are written for the batches the wave staged, which include the
// one holding its pixels' largest final index (tile_last), so a backward wave reads a block's
// words only up to that batch.  The cull is exactness-preserving (touches_rect), so the union
// of a strip's two blocks' bits holds every Gaussian with a valid pair in the strip, and a
// Gaussian added by the union is invalid at every pixel it was not kept for: the backward's
// per-pixel sums are bit-identical to the ones its own cull gives.
//
// What it buys the backward: it visits only kept positions, 64 per staging round (the headline
// keeps ~1 in 6 positions per strip), instead of staging and culling every position of its walk
// 64 at a time -- a wave's staging round trips drop ~5x and the cull's VALU work is gone.
struct KeepSrc {
  const unsigned long long *w0, *w1;  // the two blocks' words of this tile (w1 may alias w0)
  int kmax0, kmax1;                   // last valid word index per block (-1: none)
  int x;                              // range.x (word 0's first position)
};
__device__ __forceinline__ KeepSrc keep_src(const unsigned long long *__restrict__ kbits,
                                            long long kbw, const int *__restrict__ tile_last,
                                            int tile, int2 range, int wt0, int wt1) {
  KeepSrc S;
  const long long base = (long long)(range.x >> 6) + tile;
  S.w0 = kbits + wt0 * kbw + base;
  S.w1 = kbits + wt1 * kbw + base;
  const int l0 = tile_last[SPLIT_WAVES * tile + wt0], l1 = tile_last[SPLIT_WAVES * tile + wt1];
  S.kmax0 = l0 >= range.x ? (l0 - range.x) >> 6 : -1;
  S.kmax1 = l1 >= range.x ? (l1 - range.x) >> 6 : -1;
  S.x = range.x;
  return S;
}
// The kept positions tp - m (m = 0..63) as bit m (descending positions), positions below
// `bottom` cleared.
__device__ __forceinline__ unsigned long long keep_word_desc(const KeepSrc &S, int tp,
                                                             int bottom) {
  const int lo = tp - 63;
  const int rel = lo - S.x;
  const int k0 = rel >> 6, s = rel & 63;  // (arithmetic shift: floor)
  unsigned long long a0 = 0, a1 = 0;
  if (k0 >= 0 && k0 <= S.kmax0) a0 = S.w0[k0];
  if (k0 >= 0 && k0 <= S.kmax1) a0 |= S.w1[k0];
  if (k0 + 1 >= 0 && k0 + 1 <= S.kmax0) a1 = S.w0[k0 + 1];
  if (k0 + 1 >= 0 && k0 + 1 <= S.kmax1) a1 |= S.w1[k0 + 1];
  unsigned long long asc = s ? (a0 >> s) | (a1 << (64 - s)) : a0;  // bit j: position lo + j
  const int cut = bottom - lo;
  if (cut > 0) asc = cut >= 64 ? 0ull : asc & (~0ull << cut);
  return __builtin_bitreverse64(asc);
}
// Bit index of the n-th (0-based) lowest set bit of w (n < popcount(w)).
__device__ __forceinline__ int select_set_bit(unsigned long long w, int n) {
  uint32_t x = (uint32_t)w;
  int pos = 0, c = __popc(x);
  if (n >= c) {
    n -= c;
    x = (uint32_t)(w >> 32);
    pos = 32;
  }
#pragma unroll
  for (int width = 16; width >= 1; width >>= 1) {
    c = __popc(x & ((1u << width) - 1u));
    if (n >= c) {
      n -= c;
      x >>= width;
      pos += width;
    }
  }
  return pos;
}
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = __lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}
// Walk the kept positions from `top` down to `bottom` (inclusive), 64 per round: each lane
// finds its round slot's position (the owning batch by a binary search over the batches'
// prefix counts, then the bit within the batch word), `stage_one(pos, s)` fills its GStage,
// the round's records land in stage[0 .. n) in descending position order and `blend(n)` runs
// over them.  Windows of 64 batches (4,096 positions) per mask load.
// GS_STAGE_AHEAD: the next round's positions are found and their ids loaded before this round
// is blended, so a round's staging waits for one dependent load (the records) instead of two
// (ids, then records).  stage_one(pos, id, s) fills the record of position pos, id = gids[pos].
#ifndef GS_STAGE_AHEAD
#define GS_STAGE_AHEAD 1
#endif
// put(slot, s): where slot `slot`'s record goes (s == nullptr: the slot is past the round's
// count); walk_kept stores GStage records at stage[slot].
template <typename StageF, typename BlendF, typename PutF>
__device__ __forceinline__ void walk_kept_put(const KeepSrc &S, int top, int bottom,
                                              int2 *ahead, const int *__restrict__ gids,
                                              StageF &&stage_one, BlendF &&blend, PutF &&put) {
  const int lane = __lane_id();
  for (int wtop = top; wtop >= bottom; wtop -= 4096) {
    const int tp = wtop - 64 * lane;
    const unsigned long long dw = tp >= bottom ? keep_word_desc(S, tp, bottom) : 0ull;
    const int cnt = __popcll(dw);
    const int incl = wave_incl_scan(cnt);
    const int excl = incl - cnt;
    const int total = __builtin_amdgcn_readlane(incl, 63);
    // the position of this lane's slot of the round starting at r (-1 past the window's total)
    auto pos_of = [&](int r) -> int {
      const int j = r + lane;
      int l = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const int c = l + step;
        if (__shfl(excl, c, 64) <= j) l = c;
      }
      const unsigned long long w = __shfl(dw, l, 64);
      const int m = select_set_bit(w, j - __shfl(excl, l, 64));
      return j < total ? wtop - 64 * l - m : -1;
    };
    if (total <= 0) continue;
#if GS_STAGE_AHEAD
    {
      const int p0 = pos_of(0);
      ahead[lane] = make_int2(p0, p0 >= 0 ? gids[p0] : 0);
    }
#endif
    for (int r = 0; r < total; r += 64) {
#if GS_STAGE_AHEAD
      // (position, id) of this lane's slot, found and loaded during the previous round; kept in
      // LDS across the blend (no VGPRs held through it).  The next round's id load goes out with
      // this round's record loads: both latencies overlap, the records' wait covers it.
      const int2 cur = ahead[lane];
      int2 nxt = make_int2(-1, 0);
      if (r + 64 < total) {
        nxt.x = pos_of(r + 64);
        if (nxt.x >= 0) nxt.y = gids[nxt.x];
      }
      if (cur.x >= 0) {
        GStage s;
        stage_one(cur.x, cur.y, s);
        put(lane, &s);
      } else {
        put(lane, (const GStage *)nullptr);
      }
      ahead[lane] = nxt;
#else
      const int pcur = pos_of(r);
      GStage s;
      if (pcur >= 0) {
        stage_one(pcur, gids[pcur], s);
        put(lane, &s);
      } else {
        put(lane, (const GStage *)nullptr);
      }
#endif
      wave_lds_sync();
      blend(min(64, total - r));
      wave_lds_sync();
    }
  }
}
template <typename StageF, typename BlendF>
__device__ __forceinline__ void walk_kept(const KeepSrc &S, int top, int bottom, GStage *stage,
                                          int2 *ahead, const int *__restrict__ gids,
                                          StageF &&stage_one, BlendF &&blend) {
  walk_kept_put(S, top, bottom, ahead, gids, stage_one, blend,
                [&](int l, const GStage *s) {
                  if (s) stage[l] = *s;
                });
}

// stage_gaussian<true> without the cull (the forward's keep bits already decided it)
__device__ __forceinline__ void stage_kept(int idx, int g, const float2 *__restrict__ xys,
                                           const float *__restrict__ conics,
                                           const float *__restrict__ colors,
                                           const float *__restrict__ opacity, GStage &s) {
  const float2 xy = xys[g];
  s.x = xy.x;
  s.y = xy.y;
  s.ha = 0.5f * conics[3 * g];
  s.b = conics[3 * g + 1];
  s.hc = 0.5f * conics[3 * g + 2];
  s.o = opacity[g];
  s.r = colors[3 * g];
  s.g = colors[3 * g + 1];
  s.bl = colors[3 * g + 2];
  s.idx = idx;
  s.id = g;
}

// A workgroup of 4 waves covers 4 / (waves per tile) tiles.  A wave owns a COLS-wide
// rectangle of its tile: lanes map to (column lane % COLS, row lane / COLS), and each lane
// holds PXL pixels spaced 64 / COLS rows apart.  COLS = 16 gives full-width strips, COLS = 8
// gives more compact blocks (fewer Gaussians touch an 8x8 block than a 16x4 strip).
struct WaveRect {
  bool live;
  int tile, j, i0;
  float rx0, rx1, ry0, ry1;
};
// Debug hook (gsplat_debug_wave_log): when set, the backward blend kernels record per wave
// {start, end (s_memrealtime, 100 MHz), HW_ID, XCC_ID, work slot} into [waves][WAVE_LOG_F] u64.
// Attribution build (-DGS_BWD_ATTR, tools/bwd_attr.sh; never the shipped library): the strip
// backward also sums s_memtime cycles per wave -- [5] its blend rounds, [6] their reduce_rec +
// record-atomic tails, [7] the walk before its first round, [8] rounds << 32 | iterations,
// [9] tail iterations, [10] its whole life -- so a wave's time splits into staging (life - blend
// - prologue), blend math (blend - tail) and tail; the end times give the launch's imbalance.
#ifdef GS_BWD_ATTR
#define GS_ATTR 1
#define WAVE_LOG_F 11
#else
#define GS_ATTR 0
#define WAVE_LOG_F 5
#endif
__device__ unsigned long long *g_wave_log = nullptr;
struct WaveLog {
  unsigned long long t0;
  __device__ __forceinline__ WaveLog() : t0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ __forceinline__ void done(int slot, const unsigned long long *attr = nullptr) const {
#ifndef GSPLAT_TEST_HOOKS
    return;  // (the shipped library has no wave log: gsplat_debug_wave_log is a test hook)
#endif
    unsigned long long *log = g_wave_log;
    if (GS_ATTR && !attr) return;  // (attribution build: only the strip backward logs)
    if (log && (threadIdx.x & 63) == 0) {
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
      const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
      unsigned long long *e = log + (size_t)WAVE_LOG_F * w;
      e[0] = t0;
      e[1] = t1;
      e[2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      e[3] = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
      e[4] = (unsigned)slot;
#if GS_ATTR
      for (int k = 0; k < 6; ++k) e[5 + k] = attr ? attr[k] : 0ull;
#endif
    }
  }
};

// Debug hook (gsplat_debug_pair_count): lane-slot accounting of the shipped blend kernels,
// counted by separate <..., CNT = true> instantiations (the shipped code is unchanged).  Per
// kernel three u64 sums: lane slots issued (wave iterations x pixel slots a wave iteration
// spans), pairs whose pixel is still live for the Gaussian (inside the image and, in the
// backward, idx <= final_idx; in the forward, not yet terminated), and pairs that are
// composited (valid: sigma >= 0 and alpha >= 1/255 as well).  [0..2] backward, [3..5] forward.
__device__ unsigned long long *g_pair_count = nullptr;
static bool g_pair_count_on = false;
__device__ __forceinline__ void pair_count_flush(int base, unsigned slots, unsigned live,
                                                 unsigned valid) {
  // slots is wave-uniform (counted once per wave); live/valid are per-lane
  unsigned long long l = live, v = valid;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    l += __shfl_xor(l, o);
    v += __shfl_xor(v, o);
  }
  unsigned long long *c = g_pair_count;
  if (c && (threadIdx.x & 63) == 0) {
    atomicAdd(c + base, (unsigned long long)slots);
    atomicAdd(c + base + 1, l);
    atomicAdd(c + base + 2, v);
  }
}

// XCD-aware block order (gsplat_debug_set_raster_variant flag 1024): the dispatcher deals
// workgroups to the 8 XCDs round-robin, so consecutive blocks -- neighbouring tiles, which
// stage largely the same Gaussians -- land on different L2s.  With the remap each XCD takes a
// contiguous run of blocks (bijective for any grid size).
// g_xcd_remap: 0 off, -1 contiguous runs (flag 1024), K > 0 chunked: the grid is cut into
// chunks of K consecutive block slots and chunk c goes to XCD c % 8, so a chunk's neighbouring
// tiles share one L2 while a heavy image region is still dealt over all eight XCDs (bijective:
// the tail past the last whole round of 8K blocks keeps its slots).  Shipped: K = 8 (8 tiles
// of the forward, 16 of the backward per chunk; tools/exp_xcd.py, same-process medians vs
// dispatch order: headline fwd 0.123 -> 0.118 / bwd 0.331 -> 0.319 ms, garden c4 fwd 0.195 ->
// 0.151 / bwd 0.393 -> 0.400, c5 0.254 -> 0.248 / 0.746 -> 0.740, bear c3 unchanged).
// Flags bits 20-27 (gsplat_debug_set_raster_variant): 0 the default, 255 dispatch order,
// else K; flag 1024 contiguous runs.
constexpr int XCD_CHUNK = 8;
__device__ int g_xcd_remap = XCD_CHUNK;
__device__ __forceinline__ int block_slot() {
  const int b = blockIdx.x;
  const int K = g_xcd_remap;
  if (!K) return b;
  const int n = gridDim.x;
  if (K > 0) {
    const int full = n - n % (8 * K);
    if (b >= full) return b;
    const int x = b & 7, k = b >> 3;
    return ((k / K) * 8 + x) * K + k % K;
  }
  const int q = n >> 3, r = n & 7, x = b & 7, k = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// Work slot of this wave: block slot * (tiles per workgroup) + wave / (waves per tile).
template <int PXL, int COLS>
__device__ __forceinline__ int wave_slot() {
  constexpr int WPT = (GS_BLOCK / COLS) * (GS_BLOCK / ((64 / COLS) * PXL));
  return block_slot() * (4 / WPT) + (threadIdx.x >> 6) / WPT;
}
template <int PXL, int COLS>
__device__ __forceinline__ WaveRect wave_rect(int tbx, int tby, int H, int W, int tile = -1,
                                              int wt_item = -1) {
  constexpr int LROWS = 64 / COLS;      // rows per lane pass
  constexpr int WROWS = LROWS * PXL;    // rows per wave
  constexpr int WX = GS_BLOCK / COLS, WY = GS_BLOCK / WROWS;
  constexpr int WPT = WX * WY;          // waves per tile
  static_assert(WPT >= 1 && WPT <= 4 && 4 % WPT == 0, "wave footprint must tile 16x16");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  WaveRect r;
  if (tile >= 0) {
    r.tile = tile;
  } else {
    const int slot = wave_slot<PXL, COLS>();
    r.tile = slot;
  }
  const int wt = wt_item >= 0 ? wt_item : wave % WPT;
  const int tx = r.tile % tbx, ty = r.tile / tbx;
  const int c0 = tx * GS_BLOCK + (wt % WX) * COLS, r0 = ty * GS_BLOCK + (wt / WX) * WROWS;
  r.live = r.tile < tbx * tby && c0 < W && r0 < H;
  r.j = c0 + lane % COLS;
  r.i0 = r0 + lane / COLS;
  r.rx0 = (float)c0;
  r.rx1 = (float)min(c0 + COLS - 1, W - 1);
  r.ry0 = (float)r0;
  r.ry1 = (float)min(r0 + WROWS - 1, H - 1);
  return r;
}
template <int PXL, int COLS>
constexpr int tiles_per_block() {
  return 4 / ((GS_BLOCK / COLS) * (GS_BLOCK / ((64 / COLS) * PXL)));
}

// ---- the fused L1 loss (gsplat_rasterize_forward_clearing_l1 / _backward_records_l1) ----
// The training step's photometric loss mean |clamp(pred, max=1) - gt| (gc_model.py:222's clamp,
// splatfacto's L1 with ssim_lambda = 0) folded into the blend kernels: the forward's waves sum
// |clamp(pred) - gt| over their pixels into per-wave partials (the loss is their double sum,
// loss.hip's finalize), and the backward forms each pixel's upstream gradient itself instead
// of reading v_out -- exactly loss.hip l1_only_bwd_kernel's arithmetic, so the gradients equal
// the unfused step's bit for bit: gl = grad_loss * (1/n), v = gl * sign(clamp(p) - g) * mask,
// mask = (p <= 1) (torch's clamp backward; clamp keeps a NaN, the mask drops it).
struct L1Grad {
  const float *pred, *gt, *grad_loss;  // pred: the forward's raw image; null: read v_out
  float scale;                         // 1 / (3 H W)
  int clamp;
};
__device__ __forceinline__ float l1_clampv(float x, int clamp) { return clamp && x > 1.f ? 1.f : x; }
__device__ __forceinline__ float l1_grad1(float gl, float p, float g, int clamp) {
  const float d = l1_clampv(p, clamp) - g;
  const float m = clamp ? (p <= 1.f ? 1.f : 0.f) : 1.f;
  return gl * (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) * m;
}
// pixel pix's upstream colour gradient: v_out's, or the fused L1 loss's
__device__ __forceinline__ void upstream_rgb(const L1Grad &l1, const float *__restrict__ v_out,
                                             int pix, float &r, float &g, float &b) {
  if (l1.pred) {
    const float gl = l1.grad_loss[0] * l1.scale;
    r = l1_grad1(gl, l1.pred[3 * pix], l1.gt[3 * pix], l1.clamp);
    g = l1_grad1(gl, l1.pred[3 * pix + 1], l1.gt[3 * pix + 1], l1.clamp);
    b = l1_grad1(gl, l1.pred[3 * pix + 2], l1.gt[3 * pix + 2], l1.clamp);
  } else {
    r = v_out[3 * pix];
    g = v_out[3 * pix + 1];
    b = v_out[3 * pix + 2];
  }
}

// ---------------------------------------------------------------- forward, C = 3
// Two staged Gaussians per iteration (PXL pixels per lane, branch-free): both Gaussians'
// sigma / exp / alpha are independent and evaluated together; only the transmittance
// update is applied in list order, so every pixel sees exactly the scalar kernel's
// sequence of operations.
//
// DEPTH (fused RGB+depth eval render): each staged Gaussian also carries its
// depth, accumulated with the same weight as the colour channels into out_depth -- exactly
// channel 0 of a second render with colours = depth and a zero background (gc_model.py:
// 225-238), without the second binning and traversal.
template <int PXL, int COLS, bool DEPTH = false, bool CNT = false, bool PF = false>
__global__ __launch_bounds__(256) void raster_fwd3u_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, float *__restrict__ out_img,
    float *__restrict__ final_Ts, int *__restrict__ final_idx,
    const float *__restrict__ depths = nullptr, float *__restrict__ out_depth = nullptr,
    float4 *__restrict__ zero = nullptr,
    long long zero_n = 0, const int *__restrict__ zero_radii = nullptr,
    int *__restrict__ tile_last = nullptr, unsigned long long *__restrict__ kbits = nullptr,
    long long kbw = 0, const float *__restrict__ l1_gt = nullptr,
    float *__restrict__ l1_part = nullptr, int l1_clamp = 0) {
  // Side job: clear a buffer (the fused path's gradient records) with the memory bandwidth the
  // VALU-bound blend leaves idle -- a grid-stride sweep of coalesced 16-B stores, issued by each
  // wave as it finishes (issued first, the blend's first load wait would also wait for them:
  // gfx9's vmcnt counts stores).
  auto clear_side_job = [&]() {
    for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < zero_n;
         k += (long long)gridDim.x * 256)
      if (!zero_radii || zero_radii[k >> 2] > 0)  // 64-B records of visible Gaussians only
        zero[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  };
  const WaveLog wlog;
  const WaveRect R = wave_rect<PXL, COLS>(tbx, tby, H, W);
  // tile_last (the list-split plan's walk table, see split_work_kernel): per wave of a tile,
  // the largest final index of its pixels (-1: none in the image)
  constexpr int WPT = (GS_BLOCK / COLS) * (GS_BLOCK / ((64 / COLS) * PXL));
  static_assert(WPT == SPLIT_WAVES, "one walk-table entry per wave of a tile");
  const int wt = (threadIdx.x >> 6) % WPT;
  // the fused L1 loss's per-wave partial l1_part[w] (gsplat_rasterize_forward_clearing_l1)
  const long long l1_w = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (!R.live) {  // wave-uniform
    if (tile_last && R.tile < tbx * tby && (threadIdx.x & 63) == 0)
      tile_last[WPT * R.tile + wt] = -1;
    if (l1_part && (threadIdx.x & 63) == 0) l1_part[l1_w] = 0.f;
    clear_side_job();
    return;
  }
  __shared__ GStage lds[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = R.tile, j = R.j, i0 = R.i0;
  const float px = (float)j;
  const float rx0 = R.rx0, rx1 = R.rx1, ry0 = R.ry0, ry1 = R.ry1;
  constexpr int LROWS = 64 / COLS;
  float py[PXL], T[PXL], cr[PXL], cg[PXL], cb[PXL], cd[PXL];
  int cur[PXL];
  bool done[PXL];
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + LROWS * k;
    py[k] = (float)i;
    T[k] = 1.f;
    cr[k] = cg[k] = cb[k] = cd[k] = 0.f;
    cur[k] = 0;
    done[k] = !(i < H && j < W);
  }
  const int2 range = bins[tile];
  GStage *stage = lds[__builtin_amdgcn_readfirstlane(wave)];  // (uniform: SGPR address arithmetic)
  unsigned c_slots = 0, c_live = 0, c_valid = 0;  // (CNT only)
  StagePipe pipe{};  // (PF: see RawG)
  if (PF && range.x < range.y) {
    pipe.g_next = gids[min(range.x + lane, range.y - 1)];
    pipe.r_next = raw_load(pipe.g_next, xys, conics, colors, opacity);
    pipe.g_after = gids[min(range.x + 64 + lane, range.y - 1)];
  }
  // the backward's keep bits (see KeepSrc): one word per staged batch, each stored when the
  // next batch's loads go out (vmcnt counts stores too, so a store issued before the blend
  // would hold the blend's first wait; issued with loads that are waited for anyway it is free)
  const long long kb_base = wt * kbw + (long long)(range.x >> 6) + tile;
  long long kb_at = -1;
  unsigned long long kb_word = 0;
  for (int b = range.x; b < range.y; b += 64) {
    bool all_done = true;
#pragma unroll
    for (int k = 0; k < PXL; ++k) all_done = all_done && done[k];
    if (__all(all_done)) break;
    if (kbits && kb_at >= 0 && lane == 0) kbits[kb_at] = kb_word;
    const int idx = b + lane;
    GStage s;
    bool keep;
    if constexpr (PF) {
      const int g = pipe.g_next;
      const RawG q = pipe.r_next;
      // the next batch's data and the one after's ids (clamped into the list: unused past it)
      pipe.g_next = pipe.g_after;
      pipe.r_next = raw_load(pipe.g_next, xys, conics, colors, opacity);
      pipe.g_after = gids[min(b + 128 + lane, range.y - 1)];
      keep = stage_raw<false>(q, idx < range.y, idx, g, rx0, rx1, ry0, ry1, s);
    } else {
      keep = idx < range.y &&
             stage_gaussian(idx, gids, xys, conics, colors, opacity, rx0, rx1, ry0, ry1, s);
    }
    if (DEPTH && keep) s.d = depths[s.id];
    const unsigned long long kmask = __ballot(keep);
    const int n = __popcll(kmask);
    if (keep) stage[lanes_below(kmask)] = s;
    kb_at = kb_base + ((b - range.x) >> 6);  // (stored with the next batch's loads, see above)
    kb_word = kmask;
    wave_lds_sync();
    for (int t = 0; t < n; t += 2) {
      GStage G[2];
      G[0] = stage_at(stage, t);
      G[1] = stage_at(stage, min(t + 1, 63));
      const bool live1 = t + 1 < n;
      if (!live1) G[1].r = G[1].g = G[1].bl = G[1].d = 0.f;  // stale slot: keep 0 * x finite
      if constexpr (CNT) c_slots += 2 * PXL * 64;
      float sg[2][PXL], al[2][PXL];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float dx = G[u].x - px;
        const float hA = G[u].ha * dx * dx, bdx = G[u].b * dx;
#pragma unroll
        for (int k = 0; k < PXL; ++k) {
          sg[u][k] = gs_sigma(G[u].hc, bdx, hA, G[u].y - py[k]);
          al[u][k] = fminf(0.999f, G[u].o * gs_vis(sg[u][k]));
        }
      }
      bool fin = true;
#pragma unroll
      for (int k = 0; k < PXL; ++k) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bool v = !done[k] && (u == 0 || live1) && sg[u][k] >= 0.f &&
                         al[u][k] >= ALPHA_MIN;
          if constexpr (CNT) {
            c_live += (!done[k] && (u == 0 || live1)) ? 1u : 0u;
            c_valid += v ? 1u : 0u;
          }
          const float nT = T[k] * (1.f - al[u][k]);
          const bool term = v && nT <= 1e-4f, comp = v && !term;
          done[k] = done[k] || term;
          const float w = comp ? al[u][k] * T[k] : 0.f;
          cr[k] += G[u].r * w;
          cg[k] += G[u].g * w;
          cb[k] += G[u].bl * w;
          if (DEPTH) cd[k] += G[u].d * w;
          T[k] = comp ? nT : T[k];
          cur[k] = comp ? G[u].idx : cur[k];
        }
        fin = fin && done[k];
      }
      if (__all(fin)) break;
    }
    wave_lds_sync();
  }
  if (kbits && kb_at >= 0 && lane == 0) kbits[kb_at] = kb_word;
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + LROWS * k;
    if (i < H && j < W) {
      const int pix = i * W + j;
      final_Ts[pix] = T[k];
      final_idx[pix] = cur[k];
      out_img[3 * pix] = cr[k] + T[k] * bg0;
      out_img[3 * pix + 1] = cg[k] + T[k] * bg1;
      out_img[3 * pix + 2] = cb[k] + T[k] * bg2;
      if (DEPTH) out_depth[pix] = cd[k] + T[k] * 0.f;  // the depth render's zero background
    }
  }
  if (l1_part) {  // sum |clamp(pred) - gt| over the wave's pixels (fixed order: deterministic)
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < PXL; ++k) {
      const int i = i0 + LROWS * k;
      if (i < H && j < W) {
        const int pix = i * W + j;
        acc += fabsf(l1_gt[3 * pix] - l1_clampv(cr[k] + T[k] * bg0, l1_clamp)) +
               fabsf(l1_gt[3 * pix + 1] - l1_clampv(cg[k] + T[k] * bg1, l1_clamp)) +
               fabsf(l1_gt[3 * pix + 2] - l1_clampv(cb[k] + T[k] * bg2, l1_clamp));
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) l1_part[l1_w] = acc;
  }
  if (tile_last) {
    int m = -1;
#pragma unroll
    for (int k = 0; k < PXL; ++k)
      if (i0 + LROWS * k < H && j < W) m = max(m, cur[k]);
    m = wave_max_int(m);
    if (lane == 0) tile_last[WPT * tile + wt] = m;
  }
  if constexpr (CNT) pair_count_flush(3, c_slots, c_live, c_valid);
  wlog.done(tile);
  clear_side_job();
}

// ---------------------------------------------------------------- backward, C = 3
// Packed backward: 2*NP pixels per lane as float2 pairs, branch-free (an invalid pixel gets
// alpha = vis = 0: T, the colour buffer and every partial sum are unchanged exactly).
// Per pixel the colour buffer enters v_alpha only through q - sum_c buf_c * v_c (q: the
// background / alpha-output term below), carried as that one running value Qs (each Gaussian
// behind subtracts fac * (colour . v_out) with one fma), and the
// sigma gradient as moments V = sum v_sigma, Vy = sum v_sigma dy, Vyy = sum v_sigma dy^2
// (dx is constant along the lane's column), from which
//   v_conic = 0.5 (dx^2 V, dx Vy, Vyy),  v_xy = (a dx V + b Vy, b dx V + c Vy).
//
// SPLIT (list-split backward, see split_plan_kernel): the work slots are (tile, part) items
// instead of tiles.  Part j covers list positions [range.x + j chunk, range.x + (j + 1) chunk);
// its waves first walk the positions behind the part (pre_walk: T recovered and the colour
// behind accumulated with exactly the operations of the full walk, no gradient) and then
// blend the part itself -- per pixel the same arithmetic in the same order as the unsplit
// walk, so the per-wave totals (and the deterministic mode's sums) are unchanged, while a
// long list's parts run as separate, earlier-dispatched waves.
#define BWD3P_PARAMS                                                                         \
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins, \
    const float2 *__restrict__ xys, const float *__restrict__ conics,                            \
    const float *__restrict__ colors, const float *__restrict__ opacity,                         \
    const float *__restrict__ background, const float *__restrict__ final_Ts,                    \
    const int *__restrict__ final_idx, const float *__restrict__ v_out,                          \
    const float *__restrict__ v_out_alpha, float alpha_max, float *__restrict__ rec, int chunk,  \
    const int2 *__restrict__ items, const int *__restrict__ n_items,                             \
    unsigned long long *__restrict__ det, const unsigned long long *__restrict__ kbits,          \
    long long kbw, const int *__restrict__ tile_last, L1Grad l1
#define BWD3P_ARGS                                                                           \
  tbx, tby, H, W, gids, bins, xys, conics, colors, opacity, background, final_Ts, final_idx,  \
      v_out, v_out_alpha, alpha_max, rec, chunk, items, n_items, det, kbits, kbw, tile_last, l1
// One work item of the strip backward: tile `ctile` (-1: the wave's own slot), list part `part`
// (SPLIT), strip `wt` of the tile (-1: by the wave's index in its workgroup).
template <int NP, bool ATOMICS, int COLS, bool SPLIT, typename PV, bool DET, bool CNT, bool KB>
__device__ __forceinline__ void bwd3p_item(BWD3P_PARAMS, int ctile, int part, int wt_item) {
  constexpr int PXL = 2 * NP;
  constexpr int LROWS = 64 / COLS;
  const WaveLog wlog;
  const unsigned long long at_t0 = GS_ATTR ? __builtin_amdgcn_s_memtime() : 0ull;
  const WaveRect R = wave_rect<PXL, COLS>(tbx, tby, H, W, ctile, wt_item);
  if (!R.live) return;  // wave-uniform
  __shared__ GStage lds[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = R.tile, j = R.j, i0 = R.i0;
  const float px = (float)j;
  const float rx0 = R.rx0, rx1 = R.rx1, ry0 = R.ry0, ry1 = R.ry1;
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
  PV py[NP], T[NP], vr[NP], vg[NP], vb[NP], Qs[NP];
  int binf[PXL];
  int maxbin = -1;
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + LROWS * k, p = k >> 1;
    float Tf = 0.f, r = 0.f, g = 0.f, bl = 0.f, a = 0.f;
    int bf = -1;
    if (i < H && j < W) {
      const int pix = i * W + j;
      Tf = final_Ts[pix];
      bf = final_idx[pix];
      upstream_rgb(l1, v_out, pix, r, g, bl);
      a = v_out_alpha ? v_out_alpha[pix] : 0.f;
    }
    // v_alpha's background/alpha terms: Tf/(1-alpha) * (v_alpha_out - bg . v_out)
    const float qk = Tf * (a - (bg0 * r + bg1 * g + bg2 * bl));
    if (k & 1) {
      py[p].y = (float)i; T[p].y = Tf; vr[p].y = r; vg[p].y = g; vb[p].y = bl; Qs[p].y = qk;
    } else {
      py[p].x = (float)i; T[p].x = Tf; vr[p].x = r; vg[p].x = g; vb[p].x = bl; Qs[p].x = qk;
    }
    binf[k] = bf;
    maxbin = max(maxbin, bf);
  }
  const int2 range = bins[tile];
  int lo = range.x, hi = range.y;
  if (SPLIT) {
    lo = range.x + part * chunk;
    hi = (int)min((long long)lo + chunk, (long long)range.y);  // (no int overflow)
  }
  maxbin = wave_max_int(maxbin);
  const int slot = reduce_rec_slot(REC_SX, REC_SY, REC_SXX, REC_SXY, REC_SYY, REC_R, REC_G, REC_B,
                                   REC_S0);
  // canonical once, so fminf needs no per-iteration canonicalisation of the bound
  const float amax = __builtin_canonicalizef(alpha_max);
  GStage *stage = lds[__builtin_amdgcn_readfirstlane(wave)];  // (uniform: SGPR address arithmetic)
  __shared__ int2 ahead_lds[4][64];  // (KB: walk_kept's next-round ids)
  int2 *ahead = ahead_lds[__builtin_amdgcn_readfirstlane(wave)];
  // KB: the kept positions from the forward's keep bits (the strip's two 8x8 blocks)
  KeepSrc S{};
  if constexpr (KB) {
    // the strip's row half: blocks 2 wt, 2 wt + 1
    const int wt = wt_item >= 0 ? wt_item : (threadIdx.x >> 6) & 1;
    S = keep_src(kbits, kbw, tile_last, tile, range, 2 * wt, 2 * wt + 1);
  }
  auto stage1 = [&](int idx, int g, GStage &s) {
    stage_kept(idx, g, xys, conics, colors, opacity, s);
  };
  auto pre_blend = [&](int n) {
    for (int t = 0; t < n; ++t) {
        const GStage G = stage_at(stage, t);
        const float dx = G.x - px;
        const float hA = G.ha * dx * dx, bdx = G.b * dx;
#pragma unroll
        for (int p = 0; p < NP; ++p) {  // (the main loop's T / Qs operations, nothing else)
          const PV dy = G.y - py[p];
          const PV sig = gs_sigma2v<PV>(G.hc, bdx, hA, dy);
          const PV vis = gs_vis2v<PV>(sig);
          const PV ov = G.o * vis;
          const PV al = {fminf(amax, ov.x), fminf(amax, ov.y)};
          const bool v0 = G.idx <= binf[2 * p] && sig.x >= 0.f && al.x >= ALPHA_MIN;
          const bool v1 = G.idx <= binf[2 * p + 1] && sig.y >= 0.f && al.y >= ALPHA_MIN;
          const PV am = {v0 ? al.x : 0.f, v1 ? al.y : 0.f};
          const PV om = 1.f - am;
          const PV ra = {__builtin_amdgcn_rcpf(om.x), __builtin_amdgcn_rcpf(om.y)};
          T[p] = T[p] * ra;
          const PV fac = am * T[p];
          const PV gv = vfma(PV(G.r), vr[p], vfma(PV(G.g), vg[p], G.bl * vb[p]));
          Qs[p] = vfma(-fac, gv, Qs[p]);
        }
    }
  };
  if (SPLIT) {  // the positions behind this part: T and the colour behind only
    if constexpr (KB) {
      walk_kept(S, min(maxbin, range.y - 1), hi, stage, ahead, gids, stage1, pre_blend);
    } else {
      for (int b = min(maxbin, range.y - 1); b >= hi; b -= 64) {
        const int idx = b - lane;
        GStage s;
        const bool keep = idx >= hi && stage_gaussian<true>(idx, gids, xys, conics, colors,
                                                            opacity, rx0, rx1, ry0, ry1, s);
        const unsigned long long kmask = __ballot(keep);
        if (keep) stage[lanes_below(kmask)] = s;
        const int n = __popcll(kmask);
        wave_lds_sync();
        pre_blend(n);
        wave_lds_sync();
      }
    }
  }
  const int last = min(maxbin, hi - 1);
  unsigned c_slots = 0, c_live = 0, c_valid = 0;  // (CNT only)
  // (GS_ATTR: [0] blend, [1] tail, [2] prologue cycles, [3] rounds << 32 | iterations,
  //  [4] tail iterations, [5] life; cycles by s_memtime)
  unsigned long long at[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
  auto main_blend = [&](int n) {
    constexpr int U = 1;  // (two per iteration measured slower: register pressure)
    unsigned long long at_b0 = 0;
    if constexpr (GS_ATTR) {
      at_b0 = __builtin_amdgcn_s_memtime();
      if (at[3] == 0) at[2] = at_b0 - at_t0;  // (the prologue: kernel start to first round)
      at[3] += (1ull << 32) + (unsigned long long)n;
    }
    for (int t = 0; t < n; t += U) {
      float rsum[U][7];  // sa, my, myy, r, g, b and dx: reduce_rec's inputs
      bool anyv[U];
      int gid[U];
      unsigned long long anyw[U];
      if constexpr (CNT) c_slots += U * PXL * 64;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        GStage G = stage_at(stage, min(t + u, 63));
        const bool live = t + u < n;
        if (!live) G.r = G.g = G.bl = G.o = 0.f;  // stale slot: keep T / Qs finite
        gid[u] = G.id;
        // read with the rest of the staged record at the top of the iteration: left to the
        // compiler, the id's LDS read sank to the atomic at the end -- a second LDS round trip
        asm volatile("" : "+v"(gid[u]));
        const float dx = G.x - px;
        const float hA = G.ha * dx * dx, bdx = G.b * dx;
        // per-lane sums as scalar dot products over the pixel pair (two scalar fmas cost what
        // one packed fma does on gfx950, and need no packed horizontal add afterwards); the
        // -o factor of the sigma gradient is applied once to the sums, not per pixel
        float sr = 0.f, sg = 0.f, sb = 0.f, sa = 0.f, my = 0.f, myy = 0.f;
        bool any = false;
        unsigned long long anym = 0;  // wave mask of lanes with a valid pair (SGPR)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const PV dy = G.y - py[p];
          const PV sig = gs_sigma2v<PV>(G.hc, bdx, hA, dy);
          const PV vis = gs_vis2v<PV>(sig);
          const PV ov = G.o * vis;
          const PV al = {fminf(amax, ov.x), fminf(amax, ov.y)};
          const bool v0 = live && G.idx <= binf[2 * p] && sig.x >= 0.f && al.x >= ALPHA_MIN;
          const bool v1 =
              live && G.idx <= binf[2 * p + 1] && sig.y >= 0.f && al.y >= ALPHA_MIN;
          any = any || v0 || v1;
          anym |= __builtin_amdgcn_ballot_w64(v0 || v1);
          if constexpr (CNT) {
            c_live += (live && G.idx <= binf[2 * p] ? 1u : 0u) +
                      (live && G.idx <= binf[2 * p + 1] ? 1u : 0u);
            c_valid += (v0 ? 1u : 0u) + (v1 ? 1u : 0u);
          }
          const PV am = {v0 ? al.x : 0.f, v1 ? al.y : 0.f};
          const PV vm = {v0 ? vis.x : 0.f, v1 ? vis.y : 0.f};
          const PV om = 1.f - am;
          const PV ra = {__builtin_amdgcn_rcpf(om.x), __builtin_amdgcn_rcpf(om.y)};
          T[p] = T[p] * ra;
          const PV fac = am * T[p];
          // (the first pair's terms start the sums: no 0 + x kept for signed zeros)
          sr = fmaf(fac.y, vr[p].y, p ? fmaf(fac.x, vr[p].x, sr) : fac.x * vr[p].x);
          sg = fmaf(fac.y, vg[p].y, p ? fmaf(fac.x, vg[p].x, sg) : fac.x * vg[p].x);
          sb = fmaf(fac.y, vb[p].y, p ? fmaf(fac.x, vb[p].x, sb) : fac.x * vb[p].x);
          const PV gv = vfma(
              PV(G.r), vr[p], vfma(PV(G.g), vg[p], G.bl * vb[p]));
          const PV v_alpha = vfma(gv, T[p], ra * Qs[p]);
          Qs[p] = vfma(-fac, gv, Qs[p]);
          const PV vva = vm * v_alpha;
          const PV vdy = vva * dy;
          sa = p ? sa + (vva.x + vva.y) : vva.x + vva.y;
          my = fmaf(vva.y, dy.y, p ? fmaf(vva.x, dy.x, my) : vva.x * dy.x);
          myy = fmaf(vdy.y, dy.y, p ? fmaf(vdy.x, dy.x, myy) : vdy.x * dy.x);
        }
        anyv[u] = any;
        anyw[u] = anym;
        // the record moments (common.h record_grads): the six lane sums and dx, which is
        // constant along the lane's column -- reduce_rec forms sx, sxx, sxy from column sums
        rsum[u][0] = sa; rsum[u][1] = my; rsum[u][2] = myy;
        rsum[u][3] = sr; rsum[u][4] = sg; rsum[u][5] = sb; rsum[u][6] = dx;
      }
      unsigned long long any_all = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) any_all |= anyw[u];
      if (any_all) {  // (an SGPR test, no VGPR round trip)
        unsigned long long at_t = 0;
        if constexpr (GS_ATTR) at_t = __builtin_amdgcn_s_memtime();
        float v[U];
#ifdef GS_ABLATE_NO_REDUCE  // attribution build (tools/attr_bwd.sh): a lane-local sum instead
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float s = rsum[u][0];
#pragma unroll
          for (int k = 1; k < 7; ++k) s += rsum[u][k];
          v[u] = s;
        }
#else
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] = reduce_rec(rsum[u][0], rsum[u][1], rsum[u][2], rsum[u][3], rsum[u][4],
                            rsum[u][5], rsum[u][6]);
#endif
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if constexpr (DET) {  // deterministic mode: exact integer sums of the wave totals
            if (__any(anyv[u]) && slot >= 0)
              det_add(det + ((size_t)gid[u] * REC_FIELDS + slot) * DET_LIMBS, v[u]);
          } else if constexpr (ATOMICS) {
#ifdef GS_ABLATE_NO_ATOMIC  // attribution build (tools/attr_bwd.sh): the total consumed, no add
            asm volatile("" ::"v"(v[u]), "v"(gid[u]));
#else
            // 32-bit element offset (the entry points reject N >= 2^27): the atomic takes the
            // SGPR base + a VGPR offset, no 64-bit address arithmetic per iteration
            if (anyw[u] && slot >= 0)
              atomicAdd(rec + (uint32_t)(gid[u] * REC + slot), v[u]);
#endif
          } else {
            asm volatile("" ::"v"(v[u]));
          }
        }
        if constexpr (GS_ATTR) {
          at[1] += __builtin_amdgcn_s_memtime() - at_t;
          at[4] += 1;
        }
      }
    }
    if constexpr (GS_ATTR) at[0] += __builtin_amdgcn_s_memtime() - at_b0;
  };
  if constexpr (KB) {
    walk_kept(S, last, lo, stage, ahead, gids, stage1, main_blend);
  } else {
    for (int b = last; b >= lo; b -= 64) {
      const int idx = b - lane;
      GStage s;
      const bool keep = idx >= lo && stage_gaussian<true>(idx, gids, xys, conics, colors, opacity,
                                                          rx0, rx1, ry0, ry1, s);
      const unsigned long long kmask = __ballot(keep);
      if (keep) stage[lanes_below(kmask)] = s;
      const int n = __popcll(kmask);
      wave_lds_sync();
      main_blend(n);
      wave_lds_sync();
    }
  }
  if constexpr (CNT) pair_count_flush(0, c_slots, c_live, c_valid);
  if constexpr (GS_ATTR) {
    at[5] = __builtin_amdgcn_s_memtime() - at_t0;
    if (at[3] == 0) at[2] = at[5];
  }
  wlog.done(tile, GS_ATTR ? at : nullptr);
}

template <int NP, bool ATOMICS, int COLS, bool SPLIT = false, typename PV = f2,
          bool DET = false, bool CNT = false, bool KB = false>
__global__ __launch_bounds__(256) void raster_bwd3p_kernel(BWD3P_PARAMS) {
  int ctile = -1, part = 0;
  if (SPLIT) {
    const int slot = wave_slot<2 * NP, COLS>();
    if (slot >= *n_items) return;  // wave-uniform: past the last item
    const int2 it = items[slot];
    ctile = it.x;
    part = it.y;
  }
  bwd3p_item<NP, ATOMICS, COLS, SPLIT, PV, DET, CNT, KB>(BWD3P_ARGS, ctile, part, -1);
}

// ---------------------------------------------------------------- block backward (shipped)
// The forward's geometry: a wave owns an 8x8 block of its tile (4 waves per tile, one pixel
// per lane) and walks the block's culled list back to front two staged Gaussians per
// iteration.  Against the 16x8 strips with two pixels per lane:
//  * the exact rectangle cull against an 8x8 block keeps fewer Gaussians, so more of the
//    lane slots an iteration spends are valid pixel-Gaussian pairs (forward: 52 % vs 40 %);
//  * twice as many waves of half the length: the part of the kernel in which fewer waves than
//    wave slots remain (the tail) shrinks;
//  * the two Gaussians' sigma / exp / alpha / cull tests are independent instruction chains;
//    only the transmittance and colour-behind updates run in list order;
//  * per pixel the lane forms the record moments (w, dx w, dy w, dx^2 w, dx dy w, dy^2 w and
//    alpha T v_out: record_grads() in common.h) with five products, and ONE 18-value
//    reduce-scatter (reduce18) sums both Gaussians' nine moments, whose totals one atomic
//    instruction (18 lanes, two records) adds to the records.
// Per pixel the arithmetic is gsplat's backward (T recovered by dividing by 1 - alpha with the
// hardware reciprocal, v_alpha from the colour behind); the per-pixel decisions (sigma >= 0,
// alpha >= 1/255, idx <= final_idx) are the forward's bit for bit (gs_sigma / gs_vis).
//
// SPLIT: list-split items as raster_bwd3p_kernel (the four waves of a workgroup take the four
// 8x8 blocks of one (tile, part) item, with the same pre-walk).  DET: integer accumulation
// (det_add).  CNT: lane-slot accounting (gsplat_debug_pair_count).
template <bool SPLIT = false, bool DET = false, bool CNT = false, bool KB = false>
__global__ __launch_bounds__(256) void raster_bwd8_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, const float *__restrict__ final_Ts,
    const int *__restrict__ final_idx, const float *__restrict__ v_out,
    const float *__restrict__ v_out_alpha, float alpha_max, float *__restrict__ rec,
    int chunk = 0, const int2 *__restrict__ items = nullptr,
    const int *__restrict__ n_items = nullptr, unsigned long long *__restrict__ det = nullptr,
    const unsigned long long *__restrict__ kbits = nullptr, long long kbw = 0,
    const int *__restrict__ tile_last = nullptr, L1Grad l1 = {}) {
  int ctile = -1, part = 0;
  if (SPLIT) {
    const int slot = wave_slot<1, 8>();
    if (slot >= *n_items) return;  // wave-uniform: past the last item
    const int2 it = items[slot];
    ctile = it.x;
    part = it.y;
  }
  const WaveLog wlog;
  const WaveRect R = wave_rect<1, 8>(tbx, tby, H, W, ctile);
  if (!R.live) return;  // wave-uniform
  __shared__ GStage lds[4][64];
  const int wave = threadIdx.x >> 6;
  const int tile = R.tile, j = R.j, i = R.i0;
  const float px = (float)j, py = (float)i;
  float T = 0.f, vr = 0.f, vg = 0.f, vb = 0.f, Qs = 0.f;  // Qs: as raster_bwd3p_kernel's
  int bf = -1;
  const bool inside = i < H && j < W;
  if (inside) {
    const int pix = i * W + j;
    T = final_Ts[pix];
    bf = final_idx[pix];
    upstream_rgb(l1, v_out, pix, vr, vg, vb);
    const float a = v_out_alpha ? v_out_alpha[pix] : 0.f;
    // v_alpha's background / alpha-output terms: T_final / (1 - alpha) * (v_alpha_out - bg . v)
    Qs = T * (a - (background[0] * vr + background[1] * vg + background[2] * vb));
  }
  const int2 range = bins[tile];
  int lo = range.x, hi = range.y;
  if (SPLIT) {
    lo = range.x + part * chunk;
    hi = (int)min((long long)lo + chunk, (long long)range.y);  // (no int overflow)
  }
  const int maxbin = wave_max_int(bf);
  // reduce18 lane roles, learned once: value k = slot (Gaussian slot / 9, field slot % 9)
  const int slot = reduce18_slot();
  const bool for0 = slot >= 0 && slot < 9, for1 = slot >= 9;
  const int field = slot >= 9 ? slot - 9 : slot;
  const float amax = __builtin_canonicalizef(alpha_max);
  GStage *stage = lds[__builtin_amdgcn_readfirstlane(wave)];  // (uniform: SGPR address arithmetic)
  auto put = [&](int q, const GStage *sp) {
    if (sp) stage[q] = *sp;
  };
  __shared__ int2 ahead_lds[4][64];  // (KB: walk_kept's next-round ids)
  int2 *ahead = ahead_lds[__builtin_amdgcn_readfirstlane(wave)];
  // this batch's staged Gaussian (b: the batch top, bottom: the lowest position staged)
  auto stage_next = [&](int b, int bottom, GStage &s) {
    const int idx = b - (int)(threadIdx.x & 63);
    return idx >= bottom && stage_gaussian<true>(idx, gids, xys, conics, colors, opacity, R.rx0,
                                                 R.rx1, R.ry0, R.ry1, s);
  };
  // KB: the kept positions from the forward's keep bits (this wave's own 8x8 block)
  KeepSrc S{};
  if constexpr (KB) {
    const int wt = (threadIdx.x >> 6) & 3;
    S = keep_src(kbits, kbw, tile_last, tile, range, wt, wt);
    S.kmax1 = -1;  // one block
  }
  auto stage1 = [&](int idx, int g, GStage &s) {
    stage_kept(idx, g, xys, conics, colors, opacity, s);
  };
  auto pre_blend = [&](int n) {
    for (int t = 0; t < n; ++t) {  // (the main loop's T / Qs operations, nothing else)
      const GStage G = stage_at(stage, t);
      const float dx = G.x - px, dy = G.y - py;
      const float sg = gs_sigma(G.hc, G.b * dx, G.ha * dx * dx, dy);
      const float al = fminf(amax, G.o * gs_vis(sg));
      const bool v = G.idx <= bf && sg >= 0.f && al >= ALPHA_MIN;
      const float am = v ? al : 0.f;
      T = T * __builtin_amdgcn_rcpf(1.f - am);
      const float fac = am * T;
      Qs = fmaf(-fac, fmaf(G.r, vr, fmaf(G.g, vg, G.bl * vb)), Qs);
    }
  };
  if (SPLIT) {  // the positions behind this part: T and the colour behind only
    if constexpr (KB) {
      walk_kept_put(S, min(maxbin, range.y - 1), hi, ahead, gids, stage1, pre_blend, put);
    } else {
      for (int b = min(maxbin, range.y - 1); b >= hi; b -= 64) {
        GStage s;
        const bool keep = stage_next(b, hi, s);
        const unsigned long long kmask = __ballot(keep);
        const int n = __popcll(kmask);
        if (keep) put(lanes_below(kmask), &s);
        if ((n & 1) && (threadIdx.x & 63) == 0) put(n, nullptr);
        wave_lds_sync();
        pre_blend(n);
        wave_lds_sync();
      }
    }
  }
  const int last = min(maxbin, hi - 1);
  unsigned c_slots = 0, c_live = 0, c_valid = 0;  // (CNT only)
  auto main_blend = [&](int n) {
    for (int t = 0; t < n; t += 2) {
      GStage G0 = stage_at(stage, t), G1 = stage_at(stage, min(t + 1, 63));
      const bool live1 = t + 1 < n;
      if (!live1) G1.r = G1.g = G1.bl = G1.o = 0.f;  // stale slot: alpha 0, finite terms
      int gid0 = G0.id, gid1 = G1.id;
      asm volatile("" : "+v"(gid0), "+v"(gid1));  // read with the records, not at the atomic
      // the two Gaussians' per-pixel terms (independent)
      const float dx0 = G0.x - px, dy0 = G0.y - py, dx1 = G1.x - px, dy1 = G1.y - py;
      const float sg0 = gs_sigma(G0.hc, G0.b * dx0, G0.ha * dx0 * dx0, dy0);
      const float sg1 = gs_sigma(G1.hc, G1.b * dx1, G1.ha * dx1 * dx1, dy1);
      const float vis0 = gs_vis(sg0), vis1 = gs_vis(sg1);
      const float al0 = fminf(amax, G0.o * vis0), al1 = fminf(amax, G1.o * vis1);
      const bool v0 = G0.idx <= bf && sg0 >= 0.f && al0 >= ALPHA_MIN;
      const bool v1 = live1 && G1.idx <= bf && sg1 >= 0.f && al1 >= ALPHA_MIN;
      const unsigned long long any0 = __builtin_amdgcn_ballot_w64(v0),
                               any1 = __builtin_amdgcn_ballot_w64(v1);
      if constexpr (CNT) {
        c_slots += 2 * 64;
        c_live += (G0.idx <= bf ? 1u : 0u) + (live1 && G1.idx <= bf ? 1u : 0u);
        c_valid += (v0 ? 1u : 0u) + (v1 ? 1u : 0u);
      }
      // list order (back to front): G0 then G1 -- T and the colour behind are sequential
      const float am0 = v0 ? al0 : 0.f, am1 = v1 ? al1 : 0.f;
      const float ra0 = __builtin_amdgcn_rcpf(1.f - am0);
      T = T * ra0;
      const float fac0 = am0 * T;
      const float gv0 = fmaf(G0.r, vr, fmaf(G0.g, vg, G0.bl * vb));
      const float va0 = fmaf(gv0, T, ra0 * Qs);
      Qs = fmaf(-fac0, gv0, Qs);
      const float ra1 = __builtin_amdgcn_rcpf(1.f - am1);
      T = T * ra1;
      const float fac1 = am1 * T;
      const float gv1 = fmaf(G1.r, vr, fmaf(G1.g, vg, G1.bl * vb));
      const float va1 = fmaf(gv1, T, ra1 * Qs);
      Qs = fmaf(-fac1, gv1, Qs);
      if (any0 | any1) {  // (an SGPR test)
        const float w0 = (v0 ? vis0 : 0.f) * va0, w1 = (v1 ? vis1 : 0.f) * va1;
        const float sx0 = dx0 * w0, sy0 = dy0 * w0, sx1 = dx1 * w1, sy1 = dy1 * w1;
        const float m[18] = {sx0, sy0, dx0 * sx0, dy0 * sx0, dy0 * sy0,
                             fac0 * vr, fac0 * vg, fac0 * vb, w0,
                             sx1, sy1, dx1 * sx1, dy1 * sx1, dy1 * sy1,
                             fac1 * vr, fac1 * vg, fac1 * vb, w1};
        const float v = reduce18(m);
        const bool act = (for0 && any0) || (for1 && any1);
        const int g = for1 ? gid1 : gid0;
        if constexpr (DET) {
          if (act) det_add(det + ((size_t)g * REC_FIELDS + field) * DET_LIMBS, v);
        } else {
          // 32-bit element offset (the entry points reject N >= 2^27)
          if (act) atomicAdd(rec + (uint32_t)(g * REC + field), v);
        }
      }
    }
  };
  if constexpr (KB) {
    walk_kept_put(S, last, lo, ahead, gids, stage1, main_blend, put);
  } else {
    for (int b = last; b >= lo; b -= 64) {
      GStage s;
      const bool keep = stage_next(b, lo, s);
      const unsigned long long kmask = __ballot(keep);
      const int n = __popcll(kmask);
      if (keep) put(lanes_below(kmask), &s);
      if ((n & 1) && (threadIdx.x & 63) == 0) put(n, nullptr);
      wave_lds_sync();
      main_blend(n);
      wave_lds_sync();
    }
  }
  if constexpr (CNT) pair_count_flush(0, c_slots, c_live, c_valid);
  wlog.done(tile);
}

// ---- list-split plan of the backward (SPLIT kernels) -------------------------------------
// The walk table: per tile, 4 entries (one per wave of its pixels) holding the largest final
// index of those pixels (-1 when none lies in the image).  The forward fills it as its waves
// finish (raster_fwd3u_kernel's tile_last) when given the plan; otherwise split_work_kernel
// (one workgroup per tile, from final_idx) does.  The tile's backward walk covers list positions
// range.x .. min(max of the 4, range.y - 1): none when that max lies before range.x (no pixel
// composited anything: final_idx 0 outside the list).
__global__ __launch_bounds__(256) void split_work_kernel(int tbx, int tby, int H, int W,
                                                         const int *__restrict__ final_idx,
                                                         int *__restrict__ work) {
  const int t = blockIdx.x;
  const int i = (t / tbx) * GS_BLOCK + (threadIdx.x >> 4), j = (t % tbx) * GS_BLOCK + (threadIdx.x & 15);
  int m = -1;
  if (i < H && j < W) m = final_idx[i * W + j];
  m = wave_max_int(m);
  if ((threadIdx.x & 63) == 0) work[SPLIT_WAVES * t + (threadIdx.x >> 6)] = m;
}
__device__ __forceinline__ int split_walk_length(const int *__restrict__ work, int2 r, int t) {
  const int *w = work + SPLIT_WAVES * t;
  const int m = max(max(w[0], w[1]), max(w[2], w[3]));
  return m < r.x ? 0 : min(m, r.y - 1) - r.x + 1;
}

// split_plan_kernel (one workgroup): the backward's work items, longest first.  A tile with
// walk length L (split_work_kernel) becomes one item when L <= chunk, else ceil(L / chunk) parts
// (part k: positions [k chunk, (k + 1) chunk) of the walk).  An item's cost is its own positions
// plus SPLIT_PREWALK_COST times the positions behind it it re-walks; items are dispatched in
// decreasing cost (quarter-octave buckets), which is the longest-processing-time-first schedule
// that bounds a launch's tail by its longest item rather than by where the longest tiles sit.
// items[s] = (tile, part) of work slot s, *n_items the count.  (Order within a bucket follows
// LDS atomics; every item is independent, so the order changes timing only.)
constexpr float SPLIT_PREWALK_COST = 0.35f;
__device__ __forceinline__ int split_cost_bucket(int L, int k, int chunk, bool split) {
  const int own = split ? min(chunk, L - k * chunk) : L;
  const int behind = split ? max(0, L - (k + 1) * chunk) : 0;
  const unsigned c = 1u + (unsigned)(own + SPLIT_PREWALK_COST * (float)behind);
  const int oct = 31 - __clz(c);
  const int q = oct >= 2 ? (int)((c >> (oct - 2)) & 3u) : 0;
  return 63 - min(63, 4 * oct + q);  // bucket 0: the costliest
}

__device__ __forceinline__ void split_plan_body(int T, int chunk, const int2 *__restrict__ bins,
                                                const int *__restrict__ work,
                                                int2 *__restrict__ items,
                                                int *__restrict__ n_items, int *hist, int *cur) {
  const int tid = threadIdx.x;
  if (tid < 64) hist[tid] = 0;
  __syncthreads();
  for (int t = tid; t < T; t += 1024) {
    const int L = split_walk_length(work, bins[t], t);
    if (L <= 0) continue;
    const bool split = L > chunk;
    const int m = split ? (L + chunk - 1) / chunk : 1;
    for (int k = 0; k < m; ++k) atomicAdd(&hist[split_cost_bucket(L, k, chunk, split)], 1);
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the 64 bucket counts (one wave)
    const int h = hist[tid];
    int x = h;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d, 64);
      if (tid >= d) x += y;
    }
    cur[tid] = x - h;
    if (tid == 63) *n_items = x;
  }
  __syncthreads();
  for (int t = tid; t < T; t += 1024) {
    const int L = split_walk_length(work, bins[t], t);
    if (L <= 0) continue;
    const bool split = L > chunk;
    const int m = split ? (L + chunk - 1) / chunk : 1;
    for (int k = 0; k < m; ++k)
      items[atomicAdd(&cur[split_cost_bucket(L, k, chunk, split)], 1)] = make_int2(t, k);
  }
}
__global__ __launch_bounds__(1024) void split_plan_kernel(int T, int chunk,
                                                          const int2 *__restrict__ bins,
                                                          const int *__restrict__ work,
                                                          int2 *__restrict__ items,
                                                          int *__restrict__ n_items) {
  __shared__ int hist[64], cur[64];
  split_plan_body(T, chunk, bins, work, items, n_items, hist, cur);
}

// One launch behind a plan-filling or loss-computing blend (forward_clearing_impl): workgroup
// 0 sums the fused L1 loss's per-wave partials (loss = inv_n * the double sum, every load of a
// round in flight before the adds), workgroup 1 orders the list-split plan from the walk table
// the blend just filled -- two one-workgroup jobs that were a launch each (the plan at the
// start of the backward: ~7 us of the headline step apiece).  Either may be absent (part or
// items null); the grid is then one workgroup.
__global__ __launch_bounds__(1024) void post_forward_kernel(int n_part, const float *__restrict__ part,
                                                            double inv_n, float *__restrict__ loss,
                                                            int T, int chunk,
                                                            const int2 *__restrict__ bins,
                                                            const int *__restrict__ work,
                                                            int2 *__restrict__ items,
                                                            int *__restrict__ n_items) {
  __shared__ double red[1024];
  __shared__ int hist[64], cur[64];
  const bool loss_job = part && (blockIdx.x == 0 || !items);
  if (!loss_job) {
    split_plan_body(T, chunk, bins, work, items, n_items, hist, cur);
    return;
  }
  constexpr int U = 16;
  double a = 0.0;
  for (int base = 0; base < n_part; base += 1024 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = base + u * 1024 + threadIdx.x;
      v[u] = k < n_part ? part[k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) a += (double)v[u];
  }
  red[threadIdx.x] = a;
  __syncthreads();
  for (int st = 512; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = (float)(red[0] * inv_n);
}

// Gradient records (moments, common.h record_grads) -> gsplat's v_xy [N,2], v_conic [N,3],
// v_colors [N,3], v_opacity [N].  A Gaussian no pixel was composited at has an all-zero
// record and gets exact +0 gradients (gsplat's untouched zero-initialised sums), whatever
// its conic holds.
static inline bool conic_y_full() { return !(g_quirks & GSPLAT_QUIRK_CONIC_HALF); }

__global__ __launch_bounds__(256) void split_grads_kernel(int n, const float4 *__restrict__ rec,
                                                          const float *__restrict__ conics,
                                                          const float *__restrict__ opacity,
                                                          bool cy_full, float *__restrict__ v_xy,
                                                          float *__restrict__ v_conic,
                                                          float *__restrict__ v_rgb,
                                                          float *__restrict__ v_opacity) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= n) return;
  const float4 r0 = rec[(size_t)g * (REC / 4)], r1 = rec[(size_t)g * (REC / 4) + 1],
               r2 = rec[(size_t)g * (REC / 4) + 2];
  const float r[9] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x};
  bool touched = false;
#pragma unroll
  for (int k = 0; k < 9; ++k) touched = touched || r[k] != 0.f;
  RasterGrads d{};
  if (touched)
    d = record_grads(r, conics[3 * g], conics[3 * g + 1], conics[3 * g + 2], opacity[g], cy_full);
  v_xy[2 * g] = d.vxy[0];
  v_xy[2 * g + 1] = d.vxy[1];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    v_conic[3 * g + k] = d.vconic[k];
    v_rgb[3 * g + k] = d.vrgb[k];
  }
  v_opacity[g] = d.vopacity;
}

// ---------------------------------------------------------------- N-channel variants
// One pixel per thread, 256 threads per tile, Gaussians staged 256 at a time in LDS
// (colors read through L2: channel count is a runtime value up to CMAX).

struct __attribute__((aligned(16))) GN {
  float x, y, a, b;
  float c, o;
  int id;
  float p;
};

template <int CMAX>
__global__ __launch_bounds__(256) void raster_fwdn_kernel(
    int tbx, int tby, int H, int W, int C, const int *__restrict__ gids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys,
    const float *__restrict__ conics, const float *__restrict__ colors,
    const float *__restrict__ opacity, const float *__restrict__ background,
    float *__restrict__ out_img, float *__restrict__ final_Ts, int *__restrict__ final_idx) {
  __shared__ GN lds[256];
  const int tile = blockIdx.x;
  const int tx = tile % tbx, ty = tile / tbx;
  const int j = tx * GS_BLOCK + (threadIdx.x & 15);
  const int i = ty * GS_BLOCK + (threadIdx.x >> 4);
  const bool inside = i < H && j < W;
  const float px = (float)j, py = (float)i;
  float acc[CMAX];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) acc[c] = 0.f;
  float T = 1.f;
  int cur = 0;
  bool done = !inside;
  const int2 range = bins[tile];
  for (int b = range.x; b < range.y; b += 256) {
    if (__syncthreads_count(done) >= 256) break;
    const int idx = b + threadIdx.x;
    if (idx < range.y) {
      const int g = gids[idx];
      const float2 xy = xys[g];
      GN s;
      s.x = xy.x;
      s.y = xy.y;
      s.a = conics[3 * g];
      s.b = conics[3 * g + 1];
      s.c = conics[3 * g + 2];
      s.o = opacity[g];
      s.id = g;
      lds[threadIdx.x] = s;
    }
    __syncthreads();
    const int n = min(256, range.y - b);
    for (int t = 0; t < n && !done; ++t) {
      const GN G = lds[t];
      const float dx = G.x - px, dy = G.y - py;
      const float sigma = 0.5f * (G.a * dx * dx + G.c * dy * dy) + G.b * dx * dy;
      const float alpha = fminf(0.999f, G.o * __expf(-sigma));
      if (sigma < 0.f || alpha < ALPHA_MIN) continue;
      const float nT = T * (1.f - alpha);
      if (nT <= 1e-4f) {
        done = true;
        break;
      }
      const float vis = alpha * T;
      const float *col = colors + (size_t)C * G.id;
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) acc[c] += col[c] * vis;
      T = nT;
      cur = b + t;
    }
  }
  if (inside) {
    const int pix = i * W + j;
    final_Ts[pix] = T;
    final_idx[pix] = cur;
#pragma unroll
    for (int c = 0; c < CMAX; ++c)
      if (c < C) out_img[(size_t)C * pix + c] = acc[c] + T * background[c];
  }
}

template <int CMAX>
__global__ __launch_bounds__(256) void raster_bwdn_kernel(
    int tbx, int tby, int H, int W, int C, const int *__restrict__ gids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys,
    const float *__restrict__ conics, const float *__restrict__ colors,
    const float *__restrict__ opacity, const float *__restrict__ background,
    const float *__restrict__ final_Ts, const int *__restrict__ final_idx,
    const float *__restrict__ v_out, const float *__restrict__ v_out_alpha, float alpha_max,
    float conic_b_scale, float *__restrict__ v_xy, float *__restrict__ v_conic,
    float *__restrict__ v_colors, float *__restrict__ v_opacity) {
  // conic_b_scale: gsplat's v_conic.y = 1/2 v_sigma dx dy under GSPLAT_QUIRK_CONIC_HALF,
  // d loss / d conic.y = v_sigma dx dy without it (what record_grads() gives the C = 3 path)
  __shared__ GN lds[256];
  const int tile = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int tx = tile % tbx, ty = tile / tbx;
  const int j = tx * GS_BLOCK + (threadIdx.x & 15);
  const int i = ty * GS_BLOCK + (threadIdx.x >> 4);
  const bool inside = i < H && j < W;
  const float px = (float)j, py = (float)i;
  const int pix = inside ? i * W + j : 0;
  const float Tf = inside ? final_Ts[pix] : 0.f;
  float T = Tf;
  const int binf = inside ? final_idx[pix] : -1;
  const float va = inside && v_out_alpha ? v_out_alpha[pix] : 0.f;
  float vo[CMAX], buf[CMAX];
  float bgdot = 0.f;
#pragma unroll
  for (int c = 0; c < CMAX; ++c) {
    vo[c] = (inside && c < C) ? v_out[(size_t)C * pix + c] : 0.f;
    buf[c] = 0.f;
    if (c < C) bgdot += background[c] * vo[c];
  }
  __shared__ int smax;
  if (threadIdx.x == 0) smax = -1;
  __syncthreads();
  atomicMax(&smax, binf);
  __syncthreads();
  const int2 range = bins[tile];
  const int last = min(smax, range.y - 1);
  for (int b = last; b >= range.x; b -= 256) {
    __syncthreads();
    const int idx = b - (int)threadIdx.x;
    if (idx >= range.x) {
      const int g = gids[idx];
      const float2 xy = xys[g];
      GN s;
      s.x = xy.x;
      s.y = xy.y;
      s.a = conics[3 * g];
      s.b = conics[3 * g + 1];
      s.c = conics[3 * g + 2];
      s.o = opacity[g];
      s.id = g;
      lds[threadIdx.x] = s;
    }
    __syncthreads();
    const int n = min(256, b - range.x + 1);
    for (int t = 0; t < n; ++t) {
      const int k_idx = b - t;
      const GN G = lds[t];
      const float dx = G.x - px, dy = G.y - py;
      const float sigma = 0.5f * (G.a * dx * dx + G.c * dy * dy) + G.b * dx * dy;
      const float vis = __expf(-sigma);
      const float alpha = fminf(alpha_max, G.o * vis);
      const bool valid = k_idx <= binf && sigma >= 0.f && alpha >= ALPHA_MIN;
      if (!__any(valid)) continue;
      float s_col[CMAX];
      float s_x = 0.f, s_y = 0.f, s_a = 0.f, s_b = 0.f, s_c = 0.f, s_o = 0.f;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) s_col[c] = 0.f;
      const float *col = colors + (size_t)C * G.id;
      if (valid) {
        const float ra = __builtin_amdgcn_rcpf(1.f - alpha);
        T *= ra;
        const float fac = alpha * T;
        float v_alpha = 0.f;
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) {
            s_col[c] = fac * vo[c];
            v_alpha += (col[c] * T - buf[c] * ra) * vo[c];
            buf[c] += col[c] * fac;
          }
        v_alpha += Tf * ra * va;
        v_alpha += -Tf * ra * bgdot;
        const float v_sigma = -G.o * vis * v_alpha;
        s_a = 0.5f * v_sigma * dx * dx;
        s_b = conic_b_scale * v_sigma * dx * dy;
        s_c = 0.5f * v_sigma * dy * dy;
        s_x = v_sigma * (G.a * dx + G.b * dy);
        s_y = v_sigma * (G.b * dx + G.c * dy);
        s_o = vis * v_alpha;
      }
      s_x = wave_sum(s_x);
      s_y = wave_sum(s_y);
      s_a = wave_sum(s_a);
      s_b = wave_sum(s_b);
      s_c = wave_sum(s_c);
      s_o = wave_sum(s_o);
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) s_col[c] = wave_sum(s_col[c]);
      if (lane == 0) {
        const int g = G.id;
        atomicAdd(v_xy + 2 * g, s_x);
        atomicAdd(v_xy + 2 * g + 1, s_y);
        atomicAdd(v_conic + 3 * g, s_a);
        atomicAdd(v_conic + 3 * g + 1, s_b);
        atomicAdd(v_conic + 3 * g + 2, s_c);
        atomicAdd(v_opacity + g, s_o);
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) atomicAdd(v_colors + (size_t)C * g + c, s_col[c]);
      }
    }
  }
}

}  // namespace
}  // namespace gs

using namespace gs;

#define ND_DISPATCH(KERNEL, ...)                                                          \
  do {                                                                                    \
    if (channels <= 4)                                                                    \
      hipLaunchKernelGGL(KERNEL<4>, dim3(T), dim3(256), 0, st, __VA_ARGS__);              \
    else if (channels <= 8)                                                               \
      hipLaunchKernelGGL(KERNEL<8>, dim3(T), dim3(256), 0, st, __VA_ARGS__);              \
    else if (channels <= 16)                                                              \
      hipLaunchKernelGGL(KERNEL<16>, dim3(T), dim3(256), 0, st, __VA_ARGS__);             \
    else if (channels <= 32)                                                              \
      hipLaunchKernelGGL(KERNEL<32>, dim3(T), dim3(256), 0, st, __VA_ARGS__);             \
    else                                                                                  \
      hipLaunchKernelGGL(KERNEL<64>, dim3(T), dim3(256), 0, st, __VA_ARGS__);             \
  } while (0)

// ---- list-split backward ------------------------------------------------------------------
// Plan workspace (gsplat_rasterize_split_bytes): the walk table work[4 T] int (filled by the
// forward or split_work_kernel), items[T + ceil(I/chunk)] int2 and n_items int (filled by
// split_plan_kernel at the start of the backward).
int g_chunk_override = 0;  // gsplat_debug_set_chunk: 0 auto, > 0 forced, < 0 off
constexpr double SPLIT_MEANS = 0.6;
constexpr long long SPLIT_MAX_TILES = 12288;
struct SplitWs {
  int *work;
  int2 *items;
  int *n_items;
  long long items_bound;
  unsigned long long *kbits;  // the forward's keep bits (KeepSrc), SPLIT_WAVES x kbw words
  long long kbw;
  size_t bytes;
};
static SplitWs carve_split_ws(void *base, long long T, long long I, int chunk) {
  SplitWs w{};
  w.items_bound = T + (I + chunk - 1) / chunk;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return (char *)base + o;
  };
  w.work = (int *)take((size_t)T * SPLIT_WAVES * sizeof(int));
  w.items = (int2 *)take((size_t)w.items_bound * sizeof(int2));
  w.n_items = (int *)take(sizeof(int));
  w.kbw = I / 64 + T + 2;
  w.kbits = (unsigned long long *)take((size_t)SPLIT_WAVES * w.kbw * sizeof(unsigned long long));
  w.bytes = off;
  return w;
}
static bool default_variants() {
  // (the staging pipeline bits change the schedule only)
  return g_fwd_pxl == FWD_PXL && g_bwd_pxl == BWD_PXL && (g_bwd_flags & ~(7 << 28)) == 0;
}

// Which list-split plans carry keep bits: the forward that fills a plan notes whether it also
// wrote the keep bits (g_keep_bits at that time), and the backward on that plan walks them only
// then -- a switch flipped between the two calls (debug flag bit 30) cannot make the backward
// read words no forward wrote.  Keyed by the plan's address, which the next
// forward on that buffer overwrites.
// The same note records whether the forward also ordered the plan (post_forward_kernel), so
// the backward skips its split_plan_kernel.
static std::mutex g_plan_kb_mu;
static std::unordered_map<const void *, int> g_plan_kb;  // bit 0 keep bits, bit 1 plan ordered
static void plan_kbits_note(const void *plan, bool written, bool planned = false) {
  std::lock_guard<std::mutex> lk(g_plan_kb_mu);
  if (g_plan_kb.size() > 4096) g_plan_kb.clear();  // (stale entries of freed plans)
  g_plan_kb[plan] = (written ? 1 : 0) | (planned ? 2 : 0);
}
static int plan_note(const void *plan) {
  std::lock_guard<std::mutex> lk(g_plan_kb_mu);
  const auto it = g_plan_kb.find(plan);
  return it != g_plan_kb.end() ? it->second : 0;
}
static bool plan_kbits_written(const void *plan) { return plan_note(plan) & 1; }
static bool plan_ordered(const void *plan) { return plan_note(plan) & 2; }

extern "C" int gsplat_rasterize_chunk_size(int tile_bounds_x, int tile_bounds_y,
                                           int64_t num_intersects) {
  if (g_chunk_override < 0 || num_intersects <= 0 || tile_bounds_x <= 0 || tile_bounds_y <= 0)
    return 0;
  if (g_chunk_override > 0) return (g_chunk_override + 63) / 64 * 64;
  // Parts of about SPLIT_MEANS mean list lengths, longest items first (split_plan_kernel).
  // From SPLIT_MAX_TILES tiles up the frame alone fills the chip many times over and the
  // cost-ordered dispatch loses more L2 locality than it saves in tail (c5 2048^2, 16,384
  // tiles: 0.646 ms unsplit vs 0.657; headline 0.302 -> 0.276, c3 bear 0.162 -> 0.132, c4
  // garden 0.351 -> 0.334 at 0.6 means; profiles/r03_split_sweep.txt).
  const long long T = (long long)tile_bounds_x * tile_bounds_y;
  if (T >= SPLIT_MAX_TILES) return 0;
  const long long c = (long long)(SPLIT_MEANS * (double)num_intersects / (double)T);
  return (int)std::min<long long>(1 << 20, std::max<long long>(256, (c + 63) / 64 * 64));
}

extern "C" size_t gsplat_rasterize_split_bytes(int tile_bounds_x, int tile_bounds_y,
                                               int64_t num_intersects, int chunk) {
  if (chunk <= 0 || chunk % 64 || tile_bounds_x <= 0 || tile_bounds_y <= 0 || num_intersects < 0)
    return 0;
  return carve_split_ws(nullptr, (long long)tile_bounds_x * tile_bounds_y, num_intersects, chunk)
      .bytes;
}

#ifdef GSPLAT_TEST_HOOKS  // the test library only
extern "C" int gsplat_debug_set_chunk(int chunk) {
  g_chunk_override = chunk;
  return 0;
}
#endif

static bool bad_frame(int tbx, int tby, int H, int W) {
  return tbx <= 0 || tby <= 0 || H <= 0 || W <= 0 || (long long)tbx * GS_BLOCK < W ||
         (long long)tby * GS_BLOCK < H;
}

// The shipped C = 3 forward: 8x8 blocks, two Gaussians per iteration (CNT: the lane-slot
// counting instantiation, same arithmetic), optional record clear.
template <bool DEPTH>
static void launch_fwd(hipStream_t st, int tbx, int tby, int H, int W, const int32_t *gids,
                       const int32_t *bins, const float *xys, const float *conics,
                       const float *colors, const float *opacity, const float *background,
                       float *out_img, float *final_Ts, int32_t *final_idx, const float *depths,
                       float *out_depth, float4 *zero, long long zn, const int32_t *zero_radii,
                       int *tile_last = nullptr, unsigned long long *kbits = nullptr,
                       long long kbw = 0, const float *l1_gt = nullptr, float *l1_part = nullptr,
                       int l1_clamp = 0) {
  const unsigned grid = cdiv((long long)tbx * tby, (tiles_per_block<1, 8>()));
#define FWDK(CNT, PF)                                                                      \
  hipLaunchKernelGGL((raster_fwd3u_kernel<1, 8, DEPTH, CNT, PF>), dim3(grid), dim3(256), 0, st, \
                     tbx, tby, H, W, gids, (const int2 *)bins, (const float2 *)xys, conics,     \
                     colors, opacity, background, out_img, final_Ts, final_idx, depths,         \
                     out_depth, zero, zn, zero_radii, tile_last, kbits, kbw, l1_gt, l1_part,    \
                     l1_clamp)
  const bool pf = pipelined_staging(tbx, tby);
  if (!DEPTH && g_pair_count_on) {
    if (pf) FWDK(true, true); else FWDK(true, false);
  } else {
    if (pf) FWDK(false, true); else FWDK(false, false);
  }
#undef FWDK
}

extern "C" int gsplat_rasterize_forward(int tile_bounds_x, int tile_bounds_y, int img_height,
                                        int img_width, int channels,
                                        const int32_t *gaussian_ids_sorted,
                                        const int32_t *tile_bins, const float *xys,
                                        const float *conics, const float *colors,
                                        const float *opacity, const float *background,
                                        float *out_img, float *final_Ts, int32_t *final_idx,
                                        void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (bad_frame(tile_bounds_x, tile_bounds_y, img_height, img_width) || channels < 1 ||
      channels > 64) {
    set_error("rasterize_forward: bad sizes (tiles=%dx%d H=%d W=%d C=%d)", tile_bounds_x,
              tile_bounds_y, img_height, img_width, channels);
    return 1;
  }
  const int T = tile_bounds_x * tile_bounds_y;
  if (channels == 3) {
    launch_fwd<false>(st, tile_bounds_x, tile_bounds_y, img_height, img_width,
                      gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity, background,
                      out_img, final_Ts, final_idx, nullptr, nullptr, nullptr, 0, nullptr);
  } else {
    ND_DISPATCH(raster_fwdn_kernel, tile_bounds_x, tile_bounds_y, img_height, img_width,
                channels, gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys,
                conics, colors, opacity, background, out_img, final_Ts, final_idx);
  }
  return check_launch("rasterize_forward");
}

extern "C" int gsplat_rasterize_forward_rgbd(int tile_bounds_x, int tile_bounds_y,
                                             int img_height, int img_width,
                                             const int32_t *gaussian_ids_sorted,
                                             const int32_t *tile_bins, const float *xys,
                                             const float *conics, const float *colors,
                                             const float *depths, const float *opacity,
                                             const float *background, float *out_img,
                                             float *out_depth, float *final_Ts,
                                             int32_t *final_idx, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (bad_frame(tile_bounds_x, tile_bounds_y, img_height, img_width) || !depths || !out_depth) {
    set_error("rasterize_forward_rgbd: bad sizes or NULL depth buffers (tiles=%dx%d H=%d W=%d)",
              tile_bounds_x, tile_bounds_y, img_height, img_width);
    return 1;
  }
  launch_fwd<true>(st, tile_bounds_x, tile_bounds_y, img_height, img_width,
                   gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity, background,
                   out_img, final_Ts, final_idx, depths, out_depth, nullptr, 0, nullptr);
  return check_launch("rasterize_forward_rgbd");
}

#ifdef GSPLAT_TEST_HOOKS  // the test library only
// Measurement knob: bwd_pxl picks the backward geometry (BWD_PXL above); bits 20-27 of flags
// the XCD chunk of the blend kernels' block order (0 the default K = 8, 255 dispatch order).
extern "C" int gsplat_debug_set_raster_variant(int fwd_pxl, int bwd_pxl, int bwd_flags) {
  if (fwd_pxl != 1 || bwd_pxl < 0 || bwd_pxl > 2 || (bwd_flags & ~(0x7ff << 20)) ||
      ((bwd_flags >> 28) & 3) == 3) {
    set_error("debug_set_raster_variant: fwd_pxl must be 1, bwd_pxl 0 (by frame size), 1 (8x8 "
              "blocks) or 2 (16x8 strips), flags only the XCD chunk "
              "(bits 20-27), the staging pipeline (bits 28-29: 0 auto, 1 off, 2 on) and bit "
              "30 (the forward's keep bits off)");
    return 1;
  }
  g_fwd_pxl = fwd_pxl;
  g_bwd_pxl = bwd_pxl;
  g_bwd_flags = bwd_flags;
  g_keep_bits = !(bwd_flags & (1 << 30));
  const int pfm = (bwd_flags >> 28) & 3;
  g_pf_mode = pfm == 0 ? -1 : pfm == 1 ? 0 : 1;
  const int chunk = (bwd_flags >> 20) & 0xff;
  const int remap = chunk == 0xff ? 0 : chunk ? chunk : XCD_CHUNK;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_xcd_remap), &remap, sizeof(int)) != hipSuccess) {
    set_error("debug_set_raster_variant: hipMemcpyToSymbol failed");
    return 1;
  }
  return 0;
}

extern "C" int gsplat_debug_raster_variant_is_default(void) { return default_variants() ? 1 : 0; }
#endif

extern "C" int gsplat_set_deterministic(int on) {
  g_det = on != 0;
  return 0;
}
extern "C" int gsplat_get_deterministic(void) { return g_det ? 1 : 0; }

#ifdef GSPLAT_TEST_HOOKS  // the test library only (tools/wave_timeline.py, tools/bwd_attr.py)
extern "C" int gsplat_debug_wave_log(void *buffer) {
  unsigned long long *p = (unsigned long long *)buffer;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_wave_log), &p, sizeof(p)) != hipSuccess) {
    set_error("debug_wave_log: hipMemcpyToSymbol failed");
    return 1;
  }
  return 0;
}
#endif

extern "C" int gsplat_debug_pair_count(void *buffer) {
  unsigned long long *p = (unsigned long long *)buffer;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_pair_count), &p, sizeof(p)) != hipSuccess) {
    set_error("debug_pair_count: hipMemcpyToSymbol failed");
    return 1;
  }
  g_pair_count_on = p != nullptr;
  return 0;
}

// Backward geometry of a frame: the 8x8 blocks (4 waves per tile) for frames with few tiles,
// where the strips' 2 waves per tile leave SIMDs idle (512^2, c3 bear: 0.231 -> 0.160 ms
// without the list split); the 16x8 strips from 3,584 tiles up, where the chip is full and
// their reduce-scatter per 128 pixels (against one per 64) is cheaper per pixel-Gaussian pair
// (headline 0.296 vs 0.308 ms, c4 0.364 vs 0.367, c5 0.692 vs 0.806; profiles/r03_bwd_geometry.txt).
static int bwd_geometry(int tbx, int tby) {
  if (g_bwd_pxl) return g_bwd_pxl;
  return (long long)tbx * tby < 3584 ? 1 : 2;
}

// The C = 3 backward into the records `rec` (which the caller cleared), with the list split
// when w != NULL, the integer accumulators when det != NULL (then det_finish_kernel writes the
// records), the lane-slot counting instantiation when the pair-count hook is on.
static void launch_bwd(hipStream_t st, int tbx, int tby, int H, int W, int n,
                       const int32_t *gids, const int32_t *bins, const float *xys,
                       const float *conics, const float *colors, const float *opacity,
                       const float *background, const float *final_Ts, const int32_t *final_idx,
                       const float *v_output, const float *v_output_alpha, float alpha_max,
                       float *rec, int chunk, const SplitWs *w, unsigned long long *det,
                       bool work_ready = false, bool kbits_ready = false, L1Grad l1 = {},
                       bool plan_ready = false) {
  const long long slots = w ? w->items_bound : (long long)tbx * tby;
  const int2 *its = w ? w->items : nullptr;
  const int *ni = w ? w->n_items : nullptr;
  if (w) {
    const int T = tbx * tby;
    if (!work_ready)  // (the forward did not fill the walk table)
      hipLaunchKernelGGL(split_work_kernel, dim3(T), dim3(256), 0, st, tbx, tby, H, W, final_idx,
                         w->work);
    if (!(work_ready && plan_ready))  // (the forward's post_forward_kernel ordered it)
      hipLaunchKernelGGL(split_plan_kernel, dim3(1), dim3(1024), 0, st, T, chunk,
                         (const int2 *)bins, (const int *)w->work, w->items, w->n_items);
  }
  const bool cnt = g_pair_count_on && !det;
  // the forward's keep bits: only when the forward that filled this plan also wrote them
  // (plan_kbits_written: whatever g_keep_bits says now -- ADVICE r3)
  const bool kb = w && work_ready && kbits_ready;
  const unsigned long long *kbits = kb ? w->kbits : nullptr;
  const long long kbw = kb ? w->kbw : 0;
  const int *tl = kb ? w->work : nullptr;
  if (bwd_geometry(tbx, tby) == 1) {
    const unsigned grid = cdiv(slots, (tiles_per_block<1, 8>()));
#define BWD8(CH, DET, CNT, KB)                                                             \
  hipLaunchKernelGGL((raster_bwd8_kernel<CH, DET, CNT, KB>), dim3(grid), dim3(256), 0, st, tbx,  \
                     tby, H, W, gids, (const int2 *)bins, (const float2 *)xys, conics, colors,  \
                     opacity, background, final_Ts, final_idx, v_output, v_output_alpha,        \
                     alpha_max, rec, chunk, its, ni, det, kbits, kbw, tl, l1)
    if (w && kb) {
      if (det) BWD8(true, true, false, true); else if (cnt) BWD8(true, false, true, true);
      else BWD8(true, false, false, true);
    } else if (w) {
      if (det) BWD8(true, true, false, false); else if (cnt) BWD8(true, false, true, false);
      else BWD8(true, false, false, false);
    } else {
      if (det) BWD8(false, true, false, false); else if (cnt) BWD8(false, false, true, false);
      else BWD8(false, false, false, false);
    }

#undef BWD8
  } else {
    const unsigned grid = cdiv(slots, (tiles_per_block<2, 16>()));
#define BWDS(CH, DET, CNT, KB)                                                             \
  hipLaunchKernelGGL((raster_bwd3p_kernel<1, true, 16, CH, f2, DET, CNT, KB>), dim3(grid),       \
                     dim3(256), 0, st, tbx, tby, H, W, gids, (const int2 *)bins,                \
                     (const float2 *)xys, conics, colors, opacity, background, final_Ts,        \
                     final_idx, v_output, v_output_alpha, alpha_max, rec, chunk, its, ni, det,  \
                     kbits, kbw, tl, l1)
    if (w && kb) {
      if (det) BWDS(true, true, false, true); else if (cnt) BWDS(true, false, true, true);
      else BWDS(true, false, false, true);
    } else if (w) {
      if (det) BWDS(true, true, false, false); else if (cnt) BWDS(true, false, true, false);
      else BWDS(true, false, false, false);
    } else {
      if (det) BWDS(false, true, false, false); else if (cnt) BWDS(false, false, true, false);
      else BWDS(false, false, false, false);
    }
#undef BWDS
  }
  if (det)
    hipLaunchKernelGGL(det_finish_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, n, det, rec);
}

// Validates, leases the deterministic accumulators if on, and runs launch_bwd.
static int backward_into_records(const char *who, hipStream_t st, int tbx, int tby, int H,
                                 int W, int n, const int32_t *gids, const int32_t *bins,
                                 const float *xys, const float *conics, const float *colors,
                                 const float *opacity, const float *background,
                                 const float *final_Ts, const int32_t *final_idx,
                                 const float *v_output, const float *v_output_alpha,
                                 float alpha_max, float *rec, int64_t num_intersects, int chunk,
                                 void *plan, size_t plan_bytes, bool work_ready = false,
                                 bool kbits_ready = false, L1Grad l1 = {},
                                 bool plan_ready = false) {
  SplitWs w{};
  if (chunk > 0) {
    w = carve_split_ws(plan, (long long)tbx * tby, num_intersects, chunk);
    if (!plan || plan_bytes < w.bytes) {
      set_error("%s: split plan buffer %zu < %zu bytes", who, plan_bytes, w.bytes);
      return 1;
    }
  }
  if (g_det) {
    DetLease lease(n, st);
    if (!lease.buf) return check_launch(who);
    launch_bwd(st, tbx, tby, H, W, n, gids, bins, xys, conics, colors, opacity, background,
               final_Ts, final_idx, v_output, v_output_alpha, alpha_max, rec, chunk,
               chunk > 0 ? &w : nullptr, lease.buf, work_ready, kbits_ready, l1, plan_ready);
    lease.finish();
  } else {
    launch_bwd(st, tbx, tby, H, W, n, gids, bins, xys, conics, colors, opacity, background,
               final_Ts, final_idx, v_output, v_output_alpha, alpha_max, rec, chunk,
               chunk > 0 ? &w : nullptr, nullptr, work_ready, kbits_ready, l1, plan_ready);
  }
  return 0;
}

static void launch_split(hipStream_t st, int n, const float *rec, const float *conics,
                         const float *opacity, float *v_xy, float *v_conic, float *v_colors,
                         float *v_opacity) {
  hipLaunchKernelGGL(split_grads_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, n,
                     (const float4 *)rec, conics, opacity, conic_y_full(), v_xy, v_conic,
                     v_colors, v_opacity);
}

extern "C" size_t gsplat_rasterize_backward_workspace_size(int num_points, int channels) {
  return channels == 3 && num_points > 0 ? (size_t)num_points * REC * sizeof(float) : 0;
}

extern "C" int gsplat_rasterize_backward(int tile_bounds_x, int tile_bounds_y, int img_height,
                                         int img_width, int channels, int num_points,
                                         const int32_t *gaussian_ids_sorted,
                                         const int32_t *tile_bins, const float *xys,
                                         const float *conics, const float *colors,
                                         const float *opacity, const float *background,
                                         const float *final_Ts, const int32_t *final_idx,
                                         const float *v_output, const float *v_output_alpha,
                                         float alpha_max, float *v_xy, float *v_conic,
                                         float *v_colors, float *v_opacity, void *workspace,
                                         size_t workspace_bytes, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (bad_frame(tile_bounds_x, tile_bounds_y, img_height, img_width) || channels < 1 ||
      channels > 64 || num_points < 0 || num_points >= MAX_BWD_POINTS) {
    set_error("rasterize_backward: bad sizes (tiles=%dx%d H=%d W=%d C=%d N=%d)", tile_bounds_x,
              tile_bounds_y, img_height, img_width, channels, num_points);
    return 1;
  }
  const int T = tile_bounds_x * tile_bounds_y;
  if (channels == 3) {
    const size_t need = gsplat_rasterize_backward_workspace_size(num_points, channels);
    if (workspace_bytes < need || (need && !workspace)) {
      set_error("rasterize_backward: workspace %zu < %zu bytes", workspace_bytes, need);
      return 1;
    }
    if (num_points == 0) return check_launch("rasterize_backward");
    float *rec = (float *)workspace;
    note(hipMemsetAsync(rec, 0, need, st), "hipMemsetAsync");
    if (backward_into_records("rasterize_backward", st, tile_bounds_x, tile_bounds_y,
                              img_height, img_width, num_points, gaussian_ids_sorted, tile_bins,
                              xys, conics, colors, opacity, background, final_Ts, final_idx,
                              v_output, v_output_alpha, alpha_max, rec, 0, 0, nullptr, 0))
      return 1;
    launch_split(st, num_points, rec, conics, opacity, v_xy, v_conic, v_colors, v_opacity);
  } else {
    if (num_points > 0) {
      note(hipMemsetAsync(v_xy, 0, (size_t)num_points * 2 * sizeof(float), st), "hipMemsetAsync");
      note(hipMemsetAsync(v_conic, 0, (size_t)num_points * 3 * sizeof(float), st),
           "hipMemsetAsync");
      note(hipMemsetAsync(v_colors, 0, (size_t)num_points * channels * sizeof(float), st),
           "hipMemsetAsync");
      note(hipMemsetAsync(v_opacity, 0, (size_t)num_points * sizeof(float), st),
           "hipMemsetAsync");
    }
    ND_DISPATCH(raster_bwdn_kernel, tile_bounds_x, tile_bounds_y, img_height, img_width,
                channels, gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys,
                conics, colors, opacity, background, final_Ts, final_idx, v_output,
                v_output_alpha, alpha_max, conic_y_full() ? 1.f : 0.5f, v_xy, v_conic, v_colors,
                v_opacity);
  }
  return check_launch("rasterize_backward");
}

static int forward_clearing_impl(
    const char *who, int tile_bounds_x, int tile_bounds_y, int img_height, int img_width,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    float *out_img, float *final_Ts, int32_t *final_idx, void *clear, size_t clear_bytes,
    const int32_t *clear_radii, int64_t num_intersects, int chunk, void *plan, size_t plan_bytes,
    const float *l1_gt, float *l1_part, int l1_clamp, float *l1_loss, void *stream) {
  if (bad_frame(tile_bounds_x, tile_bounds_y, img_height, img_width) || clear_bytes % 16 ||
      (clear_bytes && !clear) || (clear_radii && clear_bytes % 64) || chunk < 0 ||
      (chunk > 0 && (chunk % 64 || num_intersects < 0))) {
    set_error("%s: bad sizes (tiles=%dx%d H=%d W=%d clear=%zu chunk=%d)", who, tile_bounds_x,
              tile_bounds_y, img_height, img_width, clear_bytes, chunk);
    return 1;
  }
  int *tile_last = nullptr;  // the list-split plan's walk table, filled by the blend's waves
  unsigned long long *kbits = nullptr;  // and the backward's keep bits (KeepSrc)
  long long kbw = 0;
  if (chunk > 0) {
    const SplitWs w =
        carve_split_ws(plan, (long long)tile_bounds_x * tile_bounds_y, num_intersects, chunk);
    if (!plan || plan_bytes < w.bytes) {
      set_error("%s: split plan buffer %zu < %zu bytes", who, plan_bytes, w.bytes);
      return 1;
    }
    tile_last = w.work;
    if (g_keep_bits) {
      kbits = w.kbits;
      kbw = w.kbw;
    }
    plan_kbits_note(plan, kbits != nullptr, true);
  }
  launch_fwd<false>((hipStream_t)stream, tile_bounds_x, tile_bounds_y, img_height, img_width,
                    gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity, background,
                    out_img, final_Ts, final_idx, nullptr, nullptr, (float4 *)clear,
                    (long long)(clear_bytes / 16), clear_radii, tile_last, kbits, kbw, l1_gt,
                    l1_part, l1_clamp);
  // the loss of the partials and the list-split plan, one launch (post_forward_kernel)
  const bool plan_job = chunk > 0, loss_job = l1_part != nullptr;
  if (plan_job || loss_job) {
    const long long T = (long long)tile_bounds_x * tile_bounds_y;
    SplitWs w{};
    if (plan_job) w = carve_split_ws(plan, T, num_intersects, chunk);
    const int n_part = loss_job ? (int)(gsplat_rasterize_l1_partials_bytes(tile_bounds_x,
                                                                          tile_bounds_y) / 4)
                                : 0;
    hipLaunchKernelGGL(post_forward_kernel, dim3((plan_job ? 1 : 0) + (loss_job ? 1 : 0)),
                       dim3(1024), 0, (hipStream_t)stream, n_part, l1_part,
                       1.0 / (3.0 * img_height * img_width), l1_loss, (int)T, chunk,
                       (const int2 *)tile_bins, (const int *)w.work, plan_job ? w.items : nullptr,
                       w.n_items);
  }
  return check_launch(who);
}

// The RGB forward that also clears the gradient records of the Gaussians the backward will
// accumulate into (all records, or those with radii > 0 when clear_radii is given).
extern "C" int gsplat_rasterize_forward_clearing(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    float *out_img, float *final_Ts, int32_t *final_idx, void *clear, size_t clear_bytes,
    const int32_t *clear_radii, int64_t num_intersects, int chunk, void *plan, size_t plan_bytes,
    void *stream) {
  return forward_clearing_impl("rasterize_forward_clearing", tile_bounds_x, tile_bounds_y,
                               img_height, img_width, gaussian_ids_sorted, tile_bins, xys, conics,
                               colors, opacity, background, out_img, final_Ts, final_idx, clear,
                               clear_bytes, clear_radii, num_intersects, chunk, plan, plan_bytes,
                               nullptr, nullptr, 0, nullptr, stream);
}

// The per-wave L1 partials of gsplat_rasterize_forward_clearing_l1 (one float per wave).
extern "C" size_t gsplat_rasterize_l1_partials_bytes(int tile_bounds_x, int tile_bounds_y) {
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0) return 0;
  const long long grid = cdiv((long long)tile_bounds_x * tile_bounds_y, (tiles_per_block<1, 8>()));
  return (size_t)grid * 4 * sizeof(float);
}

extern "C" int gsplat_rasterize_forward_clearing_l1(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    float *out_img, float *final_Ts, int32_t *final_idx, void *clear, size_t clear_bytes,
    const int32_t *clear_radii, int64_t num_intersects, int chunk, void *plan, size_t plan_bytes,
    const float *gt, int clamp_pred, float *partials, size_t partials_bytes, float *loss,
    void *stream) {
  const char *who = "rasterize_forward_clearing_l1";
  const size_t need = gsplat_rasterize_l1_partials_bytes(tile_bounds_x, tile_bounds_y);
  if (!gt || !partials || !loss || partials_bytes < need) {
    set_error("%s: NULL gt / partials / loss or partials %zu < %zu bytes", who, partials_bytes,
              need);
    return 1;
  }
  if (forward_clearing_impl(who, tile_bounds_x, tile_bounds_y, img_height, img_width,
                            gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity,
                            background, out_img, final_Ts, final_idx, clear, clear_bytes,
                            clear_radii, num_intersects, chunk, plan, plan_bytes, gt, partials,
                            clamp_pred ? 1 : 0, loss, stream))
    return 1;
  return check_launch(who);
}

extern "C" int gsplat_rasterize_backward_chunked(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, int num_points,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *v_output,
    const float *v_output_alpha, float alpha_max, float *v_xy, float *v_conic, float *v_colors,
    float *v_opacity, int64_t num_intersects, int chunk, void *plan, size_t plan_bytes,
    void *workspace, size_t workspace_bytes, void *stream) {
  if (chunk <= 0)
    return gsplat_rasterize_backward(tile_bounds_x, tile_bounds_y, img_height, img_width, 3,
                                     num_points, gaussian_ids_sorted, tile_bins, xys, conics,
                                     colors, opacity, background, final_Ts, final_idx, v_output,
                                     v_output_alpha, alpha_max, v_xy, v_conic, v_colors,
                                     v_opacity, workspace, workspace_bytes, stream);
  hipStream_t st = (hipStream_t)stream;
  const size_t need = gsplat_rasterize_backward_workspace_size(num_points, 3);
  if (bad_frame(tile_bounds_x, tile_bounds_y, img_height, img_width) || num_points < 0 ||
      num_points >= MAX_BWD_POINTS || chunk % 64 || num_intersects < 0 ||
      workspace_bytes < need || (need && !workspace)) {
    set_error("rasterize_backward_chunked: bad sizes (tiles=%dx%d H=%d W=%d N=%d chunk=%d) or "
              "workspace %zu < %zu bytes", tile_bounds_x, tile_bounds_y, img_height, img_width,
              num_points, chunk, workspace_bytes, need);
    return 1;
  }
  if (num_points == 0) return check_launch("rasterize_backward_chunked");
  float *rec = (float *)workspace;
  note(hipMemsetAsync(rec, 0, need, st), "hipMemsetAsync");
  if (backward_into_records("rasterize_backward_chunked", st, tile_bounds_x, tile_bounds_y,
                            img_height, img_width, num_points, gaussian_ids_sorted, tile_bins, xys,
                            conics, colors, opacity, background, final_Ts, final_idx, v_output,
                            v_output_alpha, alpha_max, rec, num_intersects, chunk, plan,
                            plan_bytes))
    return 1;
  launch_split(st, num_points, rec, conics, opacity, v_xy, v_conic, v_colors, v_opacity);
  return check_launch("rasterize_backward_chunked");
}

extern "C" int gsplat_grad_records_split(int num_points, const void *records,
                                         size_t records_bytes, const float *conics,
                                         const float *opacity, float *v_xy, float *v_conic,
                                         float *v_colors, float *v_opacity, void *stream) {
  const size_t need = num_points > 0 ? (size_t)num_points * REC * sizeof(float) : 0;
  if (num_points < 0 || records_bytes < need ||
      (need && (!records || !conics || !opacity))) {
    set_error("grad_records_split: records %zu < %zu bytes or NULL conics/opacity (N=%d)",
              records_bytes, need, num_points);
    return 1;
  }
  if (num_points == 0) return 0;
  launch_split((hipStream_t)stream, num_points, (const float *)records, conics, opacity, v_xy,
               v_conic, v_colors, v_opacity);
  return check_launch("grad_records_split");
}

extern "C" size_t gsplat_grad_records_bytes(int num_points) {
  return num_points > 0 ? (size_t)num_points * REC * sizeof(float) : 0;
}

static int backward_records_impl(
    const char *who, int tile_bounds_x, int tile_bounds_y, int img_height, int img_width,
    int num_points, const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *v_output,
    const float *v_output_alpha, float alpha_max, int64_t num_intersects, int chunk,
    void *plan, size_t plan_bytes, int plan_filled, void *records, size_t records_bytes,
    L1Grad l1, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  const size_t need = gsplat_grad_records_bytes(num_points);
  if (bad_frame(tile_bounds_x, tile_bounds_y, img_height, img_width) || num_points < 0 ||
      num_points >= MAX_BWD_POINTS || num_intersects < 0 || (chunk > 0 && chunk % 64) ||
      records_bytes < need || (need && !records) || (!v_output && !l1.pred)) {
    set_error("%s: bad sizes (tiles=%dx%d H=%d W=%d N=%d chunk=%d records %zu < %zu bytes) or "
              "no upstream gradient", who, tile_bounds_x, tile_bounds_y, img_height, img_width,
              num_points, chunk, records_bytes, need);
    return 1;
  }
  if (num_points == 0 || num_intersects == 0) return check_launch(who);
  // deterministic mode: the records' clear by the forward is superseded by det_finish_kernel
  if (backward_into_records(who, st, tile_bounds_x, tile_bounds_y, img_height, img_width,
                            num_points, gaussian_ids_sorted, tile_bins, xys, conics, colors,
                            opacity, background, final_Ts, final_idx, v_output, v_output_alpha,
                            alpha_max, (float *)records, num_intersects, chunk, plan, plan_bytes,
                            plan_filled != 0, plan_filled != 0 && plan_kbits_written(plan), l1,
                            plan_filled != 0 && plan_ordered(plan)))
    return 1;
  return check_launch(who);
}

extern "C" int gsplat_rasterize_backward_records(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, int num_points,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *v_output,
    const float *v_output_alpha, float alpha_max, int64_t num_intersects, int chunk,
    void *plan, size_t plan_bytes, int plan_filled, void *records, size_t records_bytes,
    void *stream) {
  return backward_records_impl("rasterize_backward_records", tile_bounds_x, tile_bounds_y,
                               img_height, img_width, num_points, gaussian_ids_sorted, tile_bins,
                               xys, conics, colors, opacity, background, final_Ts, final_idx,
                               v_output, v_output_alpha, alpha_max, num_intersects, chunk, plan,
                               plan_bytes, plan_filled, records, records_bytes, L1Grad{}, stream);
}

extern "C" int gsplat_rasterize_backward_records_l1(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, int num_points,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *pred, const float *gt,
    int clamp_pred, const float *grad_loss, float alpha_max, int64_t num_intersects, int chunk,
    void *plan, size_t plan_bytes, int plan_filled, void *records, size_t records_bytes,
    void *stream) {
  if (!pred || !gt || !grad_loss) {
    set_error("rasterize_backward_records_l1: NULL pred / gt / grad_loss");
    return 1;
  }
  const L1Grad l1{pred, gt, grad_loss, (float)(1.0 / (3.0 * img_height * img_width)),
                  clamp_pred ? 1 : 0};
  return backward_records_impl("rasterize_backward_records_l1", tile_bounds_x, tile_bounds_y,
                               img_height, img_width, num_points, gaussian_ids_sorted, tile_bins,
                               xys, conics, colors, opacity, background, final_Ts, final_idx,
                               nullptr, nullptr, alpha_max, num_intersects, chunk, plan,
                               plan_bytes, plan_filled, records, records_bytes, l1, stream);
}
