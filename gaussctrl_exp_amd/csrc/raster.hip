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
//    reduce-scatters the 9 sums (common.h reduce9: permlane32/16 swaps + 3 DPP steps) so
//    that 9 lanes each hold one total, and ONE 9-lane atomic instruction adds them to the
//    Gaussian's 64-byte gradient record; a split kernel then writes gsplat's
//    v_xy / v_conic / v_colors / v_opacity tensors.
//  * Every variant evaluates sigma and exp(-sigma) through the same helpers (gs_sigma*,
//    gs_vis*), so forward and backward take identical per-pixel decisions.
//  * C != 3 (gsplat nd_rasterize): one pixel per lane, 4 waves per tile, register
//    accumulators sized by a compile-time channel bound.
#include "common.h"

#include <algorithm>
#include <type_traits>

namespace gs {
namespace {

constexpr float ALPHA_MIN = 1.f / 255.f;
// The backward's record atomics use 32-bit element offsets (id * REC + slot < 2^31).
constexpr int MAX_BWD_POINTS = 1 << 27;
constexpr int REC = 16;  // floats per gradient record: x y a b c r g b o + pad = 64 B

// Deterministic backward (gsplat_set_deterministic): every wave's nine per-Gaussian totals
// (reduce9: a fixed reduction order, so run-independent) are added as 64-bit fixed-point
// integers (2^-32 units) instead of fp32 atomics.  Integer addition is associative, so the
// sums -- and every gradient downstream -- are bit-identical from run to run whatever order
// the waves finish in; det_finish_kernel converts them into the usual float records.  The
// quantisation error (<= 2^-33 per wave total) is far below the fp32 atomics' own.
constexpr int DET_REC = 9;
constexpr float DET_SCALE = 4294967296.f;  // 2^32
__device__ __forceinline__ unsigned long long det_quantize(float v) {
  const float s = fminf(fmaxf(v * DET_SCALE, -9.2e18f), 9.2e18f);  // |v| < 2^31
  return (unsigned long long)__float2ll_rn(s);
}
__global__ __launch_bounds__(256) void det_finish_kernel(int n,
                                                         const unsigned long long *__restrict__ det,
                                                         float *__restrict__ rec) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= n) return;
#pragma unroll
  for (int k = 0; k < DET_REC; ++k)
    rec[(size_t)g * REC + k] =
        (float)((double)(long long)det[(size_t)g * DET_REC + k] * (1.0 / 4294967296.0));
}
bool g_det = false;
unsigned long long *g_det_buf = nullptr;
size_t g_det_cap = 0;
// The deterministic accumulators (debug mode only: allocated on first use, grown as needed,
// then cleared on the call's stream).
unsigned long long *det_buffer(int n, hipStream_t st) {
  const size_t need = (size_t)n * DET_REC * sizeof(unsigned long long);
  if (need > g_det_cap) {
    if (g_det_buf) note(hipFree(g_det_buf), "hipFree");
    g_det_buf = nullptr;
    note(hipMalloc(&g_det_buf, need), "hipMalloc");
    g_det_cap = g_det_buf ? need : 0;
  }
  if (g_det_buf) note(hipMemsetAsync(g_det_buf, 0, need, st), "hipMemsetAsync");
  return g_det_buf;
}
constexpr int FWD_PXL = 1;  // forward: 8x8 blocks, two Gaussians per iteration (4 waves/tile)
constexpr int BWD_PXL = 2;  // packed backward, 16x8 strips (2 waves per tile)
// Tuning / ablation knobs (gsplat_debug_set_raster_variant); defaults are the shipped ones.
int g_fwd_pxl = FWD_PXL, g_bwd_pxl = BWD_PXL, g_bwd_flags = 0;

struct __attribute__((aligned(16))) GStage {
  float x, y, ha, b;  // mean, 0.5*conic.a, conic.b
  float hc, o, r, g;  // 0.5*conic.c, opacity, colour
  float bl;
  int idx;  // position in the tile's sorted list
  int id;   // Gaussian id
  float d;  // depth (fused RGB+depth forward only)
};

typedef float f2 __attribute__((ext_vector_type(2)));

// sigma = 0.5 (a dx^2 + c dy^2) + b dx dy, evaluated as fma(fma(c/2, dy, b dx), dy, a/2 dx^2)
// with explicit fmas.  EVERY blend kernel below (scalar or packed, forward or backward) uses
// exactly this rounding, so the backward re-derives the forward's per-pixel decisions
// (sigma >= 0, alpha >= 1/255) bit for bit.  hA = (ha*dx)*dx and bdx = b*dx are per
// (Gaussian, lane): a lane's pixels share one column.
__device__ __forceinline__ float gs_sigma(float hc, float bdx, float hA, float dy) {
  return fmaf(fmaf(hc, dy, bdx), dy, hA);
}
__device__ __forceinline__ f2 gs_sigma2(float hc, float bdx, float hA, f2 dy) {
  return __builtin_elementwise_fma(__builtin_elementwise_fma((f2)hc, dy, (f2)bdx), dy, (f2)hA);
}
// exp(-sigma) with the hardware exp2 (gsplat: __expf).
constexpr float NEG_LOG2E = -0x1.715476p+0f;
__device__ __forceinline__ float gs_vis(float sigma) {
  return __builtin_amdgcn_exp2f(sigma * NEG_LOG2E);
}
__device__ __forceinline__ f2 gs_vis2(f2 sigma) {
  const f2 e = sigma * NEG_LOG2E;
  return (f2){__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
}

// A pixel pair as two scalars (s2) or one packed register pair (f2): the same arithmetic,
// rounding and decisions either way; s2 compiles to scalar v_fma/v_mul (gfx950 issues packed
// fp32 ops no faster than two scalar ones), f2 to v_pk_*.
struct s2 {
  float x, y;
  __device__ __forceinline__ s2() {}
  __device__ __forceinline__ s2(float v) : x(v), y(v) {}
  __device__ __forceinline__ s2(float a, float b) : x(a), y(b) {}
};
__device__ __forceinline__ s2 operator+(s2 a, s2 b) { return s2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ s2 operator-(s2 a, s2 b) { return s2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ s2 operator*(s2 a, s2 b) { return s2(a.x * b.x, a.y * b.y); }
__device__ __forceinline__ s2 operator+(float a, s2 b) { return s2(a) + b; }
__device__ __forceinline__ s2 operator-(float a, s2 b) { return s2(a) - b; }
__device__ __forceinline__ s2 operator*(float a, s2 b) { return s2(a) * b; }
__device__ __forceinline__ s2 operator*(s2 a, float b) { return a * s2(b); }
__device__ __forceinline__ s2 &operator+=(s2 &a, s2 b) { a = a + b; return a; }
__device__ __forceinline__ s2 vfma(s2 a, s2 b, s2 c) {
  return s2(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y));
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
// {start, end (s_memrealtime, 100 MHz), HW_ID, XCC_ID, work slot} into [waves][5] u64.
__device__ unsigned long long *g_wave_log = nullptr;
struct WaveLog {
  unsigned long long t0;
  __device__ __forceinline__ WaveLog() : t0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ __forceinline__ void done(int slot) const {
    unsigned long long *log = g_wave_log;
    if (log && (threadIdx.x & 63) == 0) {
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
      const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
      log[5 * w + 0] = t0;
      log[5 * w + 1] = t1;
      log[5 * w + 2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      log[5 * w + 3] = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
      log[5 * w + 4] = (unsigned)slot;
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
// Tile swizzle of the work slots (gsplat_debug_set_tile_swizzle): slots run through bands of
// GH tile rows in groups of GW x GH tiles (row-major inside a group), so the XCD chunks above
// hold 2-D neighbourhoods instead of runs along one tile row.  Bijective over [0, T): a band's
// last group is narrower when GW does not divide tbx, rows below the last full band keep
// their slot order.  GW = GH = 1: the plain row-major order.
__device__ int g_tile_gw = 1, g_tile_gh = 1;
__device__ __forceinline__ int swizzle_tile(int s, int tbx, int tby) {
  const int gw = g_tile_gw, gh = g_tile_gh;
  if (gw * gh == 1) return s;
  const int band_slots = gh * tbx, nbands = tby / gh;
  const int band = s / band_slots;
  if (band >= nbands) return s;
  const int w = s - band * band_slots, gsz = gw * gh, nfull = tbx / gw;
  int tx, ty;
  if (w < nfull * gsz) {
    const int cg = w / gsz, r = w - cg * gsz;
    tx = cg * gw + r % gw;
    ty = r / gw;
  } else {
    const int rw = tbx - nfull * gw, r = w - nfull * gsz;
    tx = nfull * gw + r % rw;
    ty = r / rw;
  }
  return (band * gh + ty) * tbx + tx;
}

template <int PXL, int COLS>
__device__ __forceinline__ WaveRect wave_rect(int tbx, int tby, int H, int W, int tile = -1) {
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
    r.tile = slot < tbx * tby ? swizzle_tile(slot, tbx, tby) : slot;
  }
  const int wt = wave % WPT;
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

// ---------------------------------------------------------------- forward, C = 3
// Scalar variant: PXL pixels per lane (rows i0 + 4k of one column).
template <int PXL>
__global__ __launch_bounds__(256) void raster_fwd3_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, float *__restrict__ out_img,
    float *__restrict__ final_Ts, int *__restrict__ final_idx) {
  constexpr int WPT = 4 / PXL;    // waves per tile
  constexpr int TPBLK = 4 / WPT;  // tiles per workgroup
  constexpr int ROWS = 4 * PXL;   // rows per strip
  __shared__ GStage lds[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = blockIdx.x * TPBLK + wave / WPT;
  const int strip = wave % WPT;
  if (tile >= tbx * tby) return;  // wave-uniform
  const int tx = tile % tbx, ty = tile / tbx;
  const int r0 = ty * GS_BLOCK + strip * ROWS;
  if (r0 >= H) return;  // strip entirely below the image
  const int j = tx * GS_BLOCK + (lane & 15);
  const int i0 = r0 + (lane >> 4);
  const float px = (float)j;
  const float rx0 = (float)(tx * GS_BLOCK), rx1 = (float)min(tx * GS_BLOCK + 15, W - 1);
  const float ry0 = (float)r0, ry1 = (float)min(r0 + ROWS - 1, H - 1);
  float py[PXL], T[PXL], cr[PXL], cg[PXL], cb[PXL];
  int cur[PXL];
  bool done[PXL];
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + 4 * k;
    py[k] = (float)i;
    T[k] = 1.f;
    cr[k] = cg[k] = cb[k] = 0.f;
    cur[k] = 0;
    done[k] = !(i < H && j < W);
  }
  const int2 range = bins[tile];
  GStage *stage = lds[wave];
  for (int b = range.x; b < range.y; b += 64) {
    bool all_done = true;
#pragma unroll
    for (int k = 0; k < PXL; ++k) all_done = all_done && done[k];
    if (__all(all_done)) break;
    const int idx = b + lane;
    GStage s;
    const bool keep = idx < range.y &&
                      stage_gaussian(idx, gids, xys, conics, colors, opacity, rx0, rx1, ry0,
                                     ry1, s);
    const unsigned long long kmask = __ballot(keep);
    if (keep) stage[lanes_below(kmask)] = s;
    const int n = __popcll(kmask);
    wave_lds_sync();
    for (int t = 0; t < n; ++t) {
      const GStage G = stage[t];
      const float dx = G.x - px;
      const float hA = G.ha * dx * dx, bdx = G.b * dx;
      bool fin = true;
#pragma unroll
      for (int k = 0; k < PXL; ++k) {
        if (!done[k]) {
          const float sigma = gs_sigma(G.hc, bdx, hA, G.y - py[k]);
          const float alpha = fminf(0.999f, G.o * gs_vis(sigma));
          if (sigma >= 0.f && alpha >= ALPHA_MIN) {
            const float nT = T[k] * (1.f - alpha);
            if (nT <= 1e-4f) {
              done[k] = true;
            } else {
              const float vis = alpha * T[k];
              cr[k] += G.r * vis;
              cg[k] += G.g * vis;
              cb[k] += G.bl * vis;
              T[k] = nT;
              cur[k] = G.idx;
            }
          }
        }
        fin = fin && done[k];
      }
      if (__all(fin)) break;
    }
    wave_lds_sync();
  }
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + 4 * k;
    if (i < H && j < W) {
      const int pix = i * W + j;
      final_Ts[pix] = T[k];
      final_idx[pix] = cur[k];
      out_img[3 * pix] = cr[k] + T[k] * bg0;
      out_img[3 * pix + 1] = cg[k] + T[k] * bg1;
      out_img[3 * pix + 2] = cb[k] + T[k] * bg2;
    }
  }
}

// Two staged Gaussians per iteration (PXL pixels per lane, branch-free): both Gaussians'
// sigma / exp / alpha are independent and evaluated together; only the transmittance
// update is applied in list order, so every pixel sees exactly the scalar kernel's
// sequence of operations.
//
// DEPTH (fused RGB+depth eval render): each staged Gaussian also carries its
// depth, accumulated with the same weight as the colour channels into out_depth -- exactly
// channel 0 of a second render with colours = depth and a zero background (gc_model.py:
// 225-238), without the second binning and traversal.
//
// CKPT (list-split backward, see chunk_plan_kernel): for a tile whose list is longer than
// `chunk`, each pixel's state (T, accumulated colour) is recorded after every `chunk` list
// positions and at the end, so the backward can start each chunk from it.
template <int PXL, int COLS, bool DEPTH = false, bool CKPT = false, bool CNT = false>
__global__ __launch_bounds__(256) void raster_fwd3u_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, float *__restrict__ out_img,
    float *__restrict__ final_Ts, int *__restrict__ final_idx,
    const float *__restrict__ depths = nullptr, float *__restrict__ out_depth = nullptr,
    int chunk = 0, const int *__restrict__ ckpt_off = nullptr,
    float4 *__restrict__ ckpt = nullptr, float4 *__restrict__ zero = nullptr,
    long long zero_n = 0, const int *__restrict__ zero_radii = nullptr) {
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
  if (!R.live) {  // wave-uniform
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
  GStage *stage = lds[wave];
  unsigned c_slots = 0, c_live = 0, c_valid = 0;  // (CNT only)
  // checkpoints (CKPT): m states per chunked tile, state k after list position
  // range.x + (k + 1) * chunk (k = m - 1: the final state)
  int m = 0, nextk = 0;
  if (CKPT) {
    const int len = range.y - range.x;
    if (len > chunk) m = (len + chunk - 1) / chunk;
  }
  auto write_ckpt = [&](int kk) {  // (addresses recomputed here: fewer live registers)
    const size_t base = ((size_t)ckpt_off[tile] + kk) * (GS_BLOCK * GS_BLOCK);
    const int ly0 = i0 - (tile / tbx) * GS_BLOCK, lx = j - (tile % tbx) * GS_BLOCK;
#pragma unroll
    for (int k = 0; k < PXL; ++k)
      if (i0 + LROWS * k < H && j < W)
        ckpt[base + (ly0 + LROWS * k) * GS_BLOCK + lx] = make_float4(T[k], cr[k], cg[k], cb[k]);
  };
  for (int b = range.x; b < range.y; b += 64) {
    if (CKPT && m) {
      if (nextk < m - 1 && b - range.x == (nextk + 1) * chunk) write_ckpt(nextk++);
    }
    bool all_done = true;
#pragma unroll
    for (int k = 0; k < PXL; ++k) all_done = all_done && done[k];
    if (__all(all_done)) break;
    const int idx = b + lane;
    GStage s;
    const bool keep = idx < range.y &&
                      stage_gaussian(idx, gids, xys, conics, colors, opacity, rx0, rx1, ry0,
                                     ry1, s);
    if (DEPTH && keep) s.d = depths[s.id];
    const unsigned long long kmask = __ballot(keep);
    if (keep) stage[lanes_below(kmask)] = s;
    const int n = __popcll(kmask);
    wave_lds_sync();
    for (int t = 0; t < n; t += 2) {
      GStage G[2];
      G[0] = stage[t];
      G[1] = stage[min(t + 1, 63)];
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
  if (CKPT) {  // boundaries after an early exit, and the final state
    for (int kk = nextk; kk < m; ++kk) write_ckpt(kk);
  }
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
  if constexpr (CNT) pair_count_flush(3, c_slots, c_live, c_valid);
  wlog.done(tile);
  clear_side_job();
}

// Packed variant: 2*NP pixels per lane held as NP float2 pairs and blended branch-free
// with v_pk_{fma,mul,add}_f32 (two fp32 lanes per VALU op).  A pixel that is not composited
// this step gets alpha 0, which leaves T and the colour sums exactly unchanged.
template <int NP>
__global__ __launch_bounds__(256) void raster_fwd3p_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, float *__restrict__ out_img,
    float *__restrict__ final_Ts, int *__restrict__ final_idx) {
  constexpr int PXL = 2 * NP;
  constexpr int WPT = 4 / PXL;
  constexpr int TPBLK = 4 / WPT;
  constexpr int ROWS = 4 * PXL;
  __shared__ GStage lds[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = blockIdx.x * TPBLK + wave / WPT;
  const int strip = wave % WPT;
  if (tile >= tbx * tby) return;
  const int tx = tile % tbx, ty = tile / tbx;
  const int r0 = ty * GS_BLOCK + strip * ROWS;
  if (r0 >= H) return;
  const int j = tx * GS_BLOCK + (lane & 15);
  const int i0 = r0 + (lane >> 4);
  const float px = (float)j;
  const float rx0 = (float)(tx * GS_BLOCK), rx1 = (float)min(tx * GS_BLOCK + 15, W - 1);
  const float ry0 = (float)r0, ry1 = (float)min(r0 + ROWS - 1, H - 1);
  f2 py[NP], T[NP], cr[NP], cg[NP], cb[NP];
  int cur[PXL];
  bool done[PXL];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int ia = i0 + 8 * p, ib = ia + 4;
    py[p] = (f2){(float)ia, (float)ib};
    T[p] = (f2)1.f;
    cr[p] = cg[p] = cb[p] = (f2)0.f;
    cur[2 * p] = cur[2 * p + 1] = 0;
    done[2 * p] = !(ia < H && j < W);
    done[2 * p + 1] = !(ib < H && j < W);
  }
  const int2 range = bins[tile];
  GStage *stage = lds[wave];
  for (int b = range.x; b < range.y; b += 64) {
    bool all_done = true;
#pragma unroll
    for (int k = 0; k < PXL; ++k) all_done = all_done && done[k];
    if (__all(all_done)) break;
    const int idx = b + lane;
    GStage s;
    const bool keep = idx < range.y &&
                      stage_gaussian(idx, gids, xys, conics, colors, opacity, rx0, rx1, ry0,
                                     ry1, s);
    const unsigned long long kmask = __ballot(keep);
    if (keep) stage[lanes_below(kmask)] = s;
    const int n = __popcll(kmask);
    wave_lds_sync();
    for (int t = 0; t < n; ++t) {
      const GStage G = stage[t];
      const float dx = G.x - px;
      const float hA = G.ha * dx * dx, bdx = G.b * dx;
      bool fin = true;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const f2 sg = gs_sigma2(G.hc, bdx, hA, G.y - py[p]);
        const f2 ov = G.o * gs_vis2(sg);
        const f2 al = {fminf(0.999f, ov.x), fminf(0.999f, ov.y)};
        const f2 nT = T[p] * (1.f - al);
        const bool v0 = !done[2 * p] && sg.x >= 0.f && al.x >= ALPHA_MIN;
        const bool v1 = !done[2 * p + 1] && sg.y >= 0.f && al.y >= ALPHA_MIN;
        const bool t0 = v0 && nT.x <= 1e-4f, t1 = v1 && nT.y <= 1e-4f;
        const bool c0 = v0 && !t0, c1 = v1 && !t1;
        done[2 * p] = done[2 * p] || t0;
        done[2 * p + 1] = done[2 * p + 1] || t1;
        const f2 w = (f2){c0 ? al.x : 0.f, c1 ? al.y : 0.f} * T[p];
        cr[p] = __builtin_elementwise_fma((f2)G.r, w, cr[p]);
        cg[p] = __builtin_elementwise_fma((f2)G.g, w, cg[p]);
        cb[p] = __builtin_elementwise_fma((f2)G.bl, w, cb[p]);
        T[p] = (f2){c0 ? nT.x : T[p].x, c1 ? nT.y : T[p].y};
        cur[2 * p] = c0 ? G.idx : cur[2 * p];
        cur[2 * p + 1] = c1 ? G.idx : cur[2 * p + 1];
        fin = fin && done[2 * p] && done[2 * p + 1];
      }
      if (__all(fin)) break;
    }
    wave_lds_sync();
  }
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + 4 * k;
    const int p = k >> 1;
    const float Tk = (k & 1) ? T[p].y : T[p].x;
    if (i < H && j < W) {
      const int pix = i * W + j;
      final_Ts[pix] = Tk;
      final_idx[pix] = cur[k];
      out_img[3 * pix] = ((k & 1) ? cr[p].y : cr[p].x) + Tk * bg0;
      out_img[3 * pix + 1] = ((k & 1) ? cg[p].y : cg[p].x) + Tk * bg1;
      out_img[3 * pix + 2] = ((k & 1) ? cb[p].y : cb[p].x) + Tk * bg2;
    }
  }
}

// ---------------------------------------------------------------- backward, C = 3
// Record fields: 0 v_x, 1 v_y, 2..4 v_conic (a, b, c) * CONIC_SCALE^-1, 5..7 v_rgb,
// 8 v_opacity.  The scalar kernel stores v_conic itself (scale 1); the packed kernel stores
// 2*v_conic (the 0.5 is applied once in split_grads_kernel, exact).
template <int PXL, bool ATOMICS>
__global__ __launch_bounds__(256) void raster_bwd3_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, const float *__restrict__ final_Ts,
    const int *__restrict__ final_idx, const float *__restrict__ v_out,
    const float *__restrict__ v_out_alpha, float alpha_max, float *__restrict__ rec) {
  constexpr int WPT = 4 / PXL;
  constexpr int TPBLK = 4 / WPT;
  constexpr int ROWS = 4 * PXL;
  __shared__ GStage lds[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = blockIdx.x * TPBLK + wave / WPT;
  const int strip = wave % WPT;
  if (tile >= tbx * tby) return;
  const int tx = tile % tbx, ty = tile / tbx;
  const int r0 = ty * GS_BLOCK + strip * ROWS;
  if (r0 >= H) return;
  const int j = tx * GS_BLOCK + (lane & 15);
  const int i0 = r0 + (lane >> 4);
  const float px = (float)j;
  const float rx0 = (float)(tx * GS_BLOCK), rx1 = (float)min(tx * GS_BLOCK + 15, W - 1);
  const float ry0 = (float)r0, ry1 = (float)min(r0 + ROWS - 1, H - 1);
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
  float py[PXL], T[PXL], Tf[PXL], vr[PXL], vg[PXL], vb[PXL], va[PXL], bgdot[PXL];
  float br[PXL], bgr[PXL], bb[PXL];
  int binf[PXL];
  int maxbin = -1;
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + 4 * k;
    py[k] = (float)i;
    br[k] = bgr[k] = bb[k] = 0.f;
    if (i < H && j < W) {
      const int pix = i * W + j;
      Tf[k] = final_Ts[pix];
      binf[k] = final_idx[pix];
      vr[k] = v_out[3 * pix];
      vg[k] = v_out[3 * pix + 1];
      vb[k] = v_out[3 * pix + 2];
      va[k] = v_out_alpha ? v_out_alpha[pix] : 0.f;
    } else {
      Tf[k] = 0.f;
      binf[k] = -1;
      vr[k] = vg[k] = vb[k] = va[k] = 0.f;
    }
    T[k] = Tf[k];
    bgdot[k] = bg0 * vr[k] + bg1 * vg[k] + bg2 * vb[k];
    maxbin = max(maxbin, binf[k]);
  }
  maxbin = wave_max_int(maxbin);
  const int slot = reduce9_slot();  // record field this lane adds (reduce9), or -1
  const int2 range = bins[tile];
  const int last = min(maxbin, range.y - 1);
  GStage *stage = lds[wave];
  for (int b = last; b >= range.x; b -= 64) {
    const int idx = b - lane;
    GStage s;
    const bool keep = idx >= range.x &&
                      stage_gaussian(idx, gids, xys, conics, colors, opacity, rx0, rx1, ry0,
                                     ry1, s);
    const unsigned long long kmask = __ballot(keep);
    if (keep) stage[lanes_below(kmask)] = s;
    const int n = __popcll(kmask);
    wave_lds_sync();
    for (int t = 0; t < n; ++t) {
      const GStage G = stage[t];
      const float dx = G.x - px;
      const float hA = G.ha * dx * dx, bdx = G.b * dx;
      const float a2 = 2.f * G.ha, c2 = 2.f * G.hc;
      float s_x = 0.f, s_y = 0.f, s_a = 0.f, s_b = 0.f, s_c = 0.f, s_r = 0.f, s_g = 0.f,
            s_bl = 0.f, s_o = 0.f;
      bool anyv = false;
#pragma unroll
      for (int k = 0; k < PXL; ++k) {
        const float dy = G.y - py[k];
        const float sigma = gs_sigma(G.hc, bdx, hA, dy);
        const float vis = gs_vis(sigma);
        const float alpha = fminf(alpha_max, G.o * vis);
        const bool valid = G.idx <= binf[k] && sigma >= 0.f && alpha >= ALPHA_MIN;
        if (valid) {
          anyv = true;
          const float ra = __builtin_amdgcn_rcpf(1.f - alpha);
          T[k] *= ra;
          const float fac = alpha * T[k];
          s_r += fac * vr[k];
          s_g += fac * vg[k];
          s_bl += fac * vb[k];
          float v_alpha = (G.r * T[k] - br[k] * ra) * vr[k] + (G.g * T[k] - bgr[k] * ra) * vg[k] +
                          (G.bl * T[k] - bb[k] * ra) * vb[k];
          v_alpha += Tf[k] * ra * va[k];
          v_alpha += -Tf[k] * ra * bgdot[k];
          br[k] += G.r * fac;
          bgr[k] += G.g * fac;
          bb[k] += G.bl * fac;
          const float v_sigma = -G.o * vis * v_alpha;
          s_a += 0.5f * v_sigma * dx * dx;
          s_b += 0.5f * v_sigma * dx * dy;
          s_c += 0.5f * v_sigma * dy * dy;
          s_x += v_sigma * (a2 * dx + G.b * dy);
          s_y += v_sigma * (G.b * dx + c2 * dy);
          s_o += vis * v_alpha;
        }
      }
      if (__any(anyv)) {
        const float parts[9] = {s_x, s_y, s_a, s_b, s_c, s_r, s_g, s_bl, s_o};
        const float v = reduce9(parts);
        if constexpr (ATOMICS) {
          if (slot >= 0) atomicAdd(rec + (size_t)G.id * REC + slot, v);
        } else {
          asm volatile("" ::"v"(v));  // ablation build: keep the reduction, drop the atomic
        }
      }
    }
    wave_lds_sync();
  }
}

// Packed backward: 2*NP pixels per lane as float2 pairs, branch-free (an invalid pixel gets
// alpha = vis = 0: T, the colour buffer and every partial sum are unchanged exactly).
// Per pixel the colour buffer is carried as one dot product Sb = sum_c buf_c * v_c, and the
// sigma gradient as moments V = sum v_sigma, Vy = sum v_sigma dy, Vyy = sum v_sigma dy^2
// (dx is constant along the lane's column), from which
//   v_conic = 0.5 (dx^2 V, dx Vy, Vyy),  v_xy = (a dx V + b Vy, b dx V + c Vy).
//
// CHUNKED (list-split backward): the work slots are (tile, chunk) items of chunk_plan_kernel's
// table instead of tiles.  Chunk j of a tile covers list positions
// [range.x + j * chunk, range.x + (j + 1) * chunk) and starts from the forward's checkpoint
// after its last position: T = checkpoint T, and the colour behind it, Sb = (C_final - C_j) . v,
// instead of T_final and 0 -- so long lists and small images (few tiles) still fill the GPU.
template <int NP, bool ATOMICS, int COLS, bool CHUNKED = false, typename PV = f2,
          bool DET = false, bool CNT = false>
__global__ __launch_bounds__(256) void raster_bwd3p_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, const float *__restrict__ final_Ts,
    const int *__restrict__ final_idx, const float *__restrict__ v_out,
    const float *__restrict__ v_out_alpha, float alpha_max, float *__restrict__ rec,
    bool stage_only, int chunk = 0, const int *__restrict__ item_off = nullptr,
    const int *__restrict__ item_tile = nullptr, const int *__restrict__ ckpt_off = nullptr,
    const float4 *__restrict__ ckpt = nullptr, unsigned long long *__restrict__ det = nullptr) {
  constexpr int PXL = 2 * NP;
  constexpr int LROWS = 64 / COLS;
  int ctile = -1, cj = 0;
  if (CHUNKED) {
    const int slot = wave_slot<PXL, COLS>();
    if (slot >= item_off[tbx * tby]) return;  // wave-uniform: past the last item
    ctile = item_tile[slot];
    cj = slot - item_off[ctile];
  }
  const WaveLog wlog;
  const WaveRect R = wave_rect<PXL, COLS>(tbx, tby, H, W, ctile);
  if (!R.live) return;  // wave-uniform
  __shared__ GStage lds[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = R.tile, j = R.j, i0 = R.i0;
  const float px = (float)j;
  const float rx0 = R.rx0, rx1 = R.rx1, ry0 = R.ry0, ry1 = R.ry1;
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
  PV py[NP], T[NP], vr[NP], vg[NP], vb[NP], q[NP], Sb[NP];
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
      r = v_out[3 * pix];
      g = v_out[3 * pix + 1];
      bl = v_out[3 * pix + 2];
      a = v_out_alpha ? v_out_alpha[pix] : 0.f;
    }
    // v_alpha's background/alpha terms: Tf/(1-alpha) * (v_alpha_out - bg . v_out)
    const float qk = Tf * (a - (bg0 * r + bg1 * g + bg2 * bl));
    if (k & 1) {
      py[p].y = (float)i; T[p].y = Tf; vr[p].y = r; vg[p].y = g; vb[p].y = bl; q[p].y = qk;
    } else {
      py[p].x = (float)i; T[p].x = Tf; vr[p].x = r; vg[p].x = g; vb[p].x = bl; q[p].x = qk;
    }
    Sb[p] = PV(0.f);
    binf[k] = bf;
    maxbin = max(maxbin, bf);
  }
  const int2 range = bins[tile];
  int lo = range.x, hi = range.y;
  if (CHUNKED) {
    const int len = range.y - range.x;
    const int m = len > chunk ? (len + chunk - 1) / chunk : 1;
    if (m > 1) {
      lo = range.x + cj * chunk;
      hi = min(lo + chunk, range.y);
      if (cj < m - 1) {  // start from the checkpoint after this chunk
        const size_t cb = (size_t)ckpt_off[tile] * (GS_BLOCK * GS_BLOCK);
        const int oy = (tile / tbx) * GS_BLOCK, ox = (tile % tbx) * GS_BLOCK;
#pragma unroll
        for (int k = 0; k < PXL; ++k) {
          const int i = i0 + LROWS * k, p = k >> 1;
          if (i < H && j < W) {
            const int lpix = (i - oy) * GS_BLOCK + (j - ox);
            const float4 cj4 = ckpt[cb + (size_t)cj * (GS_BLOCK * GS_BLOCK) + lpix];
            const float4 cf4 = ckpt[cb + (size_t)(m - 1) * (GS_BLOCK * GS_BLOCK) + lpix];
            const float vr_ = (k & 1) ? vr[p].y : vr[p].x, vg_ = (k & 1) ? vg[p].y : vg[p].x,
                        vb_ = (k & 1) ? vb[p].y : vb[p].x;
            const float sb = (cf4.y - cj4.y) * vr_ + (cf4.z - cj4.z) * vg_ + (cf4.w - cj4.w) * vb_;
            if (k & 1) { T[p].y = cj4.x; Sb[p].y = sb; } else { T[p].x = cj4.x; Sb[p].x = sb; }
          }
        }
      }
    }
  }
  maxbin = wave_max_int(maxbin);
  const int slot = reduce9_slot();
  // canonical once, so fminf needs no per-iteration canonicalisation of the bound
  const float amax = __builtin_canonicalizef(alpha_max);
  const int last = min(maxbin, hi - 1);
  GStage *stage = lds[wave];
  unsigned c_slots = 0, c_live = 0, c_valid = 0;  // (CNT only)
  for (int b = last; b >= lo; b -= 64) {
    const int idx = b - lane;
    GStage s;
    const bool keep = idx >= lo &&
                      stage_gaussian<true>(idx, gids, xys, conics, colors, opacity, rx0, rx1, ry0,
                                     ry1, s);
    const unsigned long long kmask = __ballot(keep);
    if (keep) stage[lanes_below(kmask)] = s;
    const int n = __popcll(kmask);
    wave_lds_sync();
    constexpr int U = 1;  // (two per iteration measured slower: register pressure)
    for (int t = 0; t < (stage_only ? 0 : n); t += U) {
      float parts[U][9];
      bool anyv[U];
      int gid[U];
      unsigned long long anyw[U];
      if constexpr (CNT) c_slots += U * PXL * 64;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        GStage G = stage[min(t + u, 63)];
        const bool live = t + u < n;
        if (!live) G.r = G.g = G.bl = G.o = 0.f;  // stale slot: keep T / Sb finite
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
          const PV v_alpha = vfma(gv, T[p], ra * (q[p] - Sb[p]));
          Sb[p] = vfma(fac, gv, Sb[p]);
          const PV vva = vm * v_alpha;
          const PV vdy = vva * dy;
          sa = p ? sa + (vva.x + vva.y) : vva.x + vva.y;
          my = fmaf(vva.y, dy.y, p ? fmaf(vva.x, dy.x, my) : vva.x * dy.x);
          myy = fmaf(vdy.y, dy.y, p ? fmaf(vdy.x, dy.x, myy) : vdy.x * dy.x);
        }
        anyv[u] = any;
        anyw[u] = anym;
        const float Vs = -G.o * sa, Vys = -G.o * my;
        const float dxV = dx * Vs;
        parts[u][0] = fmaf(2.f * G.ha, dxV, G.b * Vys);  // v_x
        parts[u][1] = fmaf(G.b, dxV, 2.f * G.hc * Vys);  // v_y
        parts[u][2] = dx * dxV;                          // 2 v_conic.a
        parts[u][3] = dx * Vys;                          // 2 v_conic.b
        parts[u][4] = -G.o * myy;                        // 2 v_conic.c
        parts[u][5] = sr;
        parts[u][6] = sg;
        parts[u][7] = sb;
        parts[u][8] = sa;
      }
      unsigned long long any_all = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) any_all |= anyw[u];
      if (any_all) {  // (an SGPR test, no VGPR round trip)
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = reduce9(parts[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if constexpr (DET) {  // deterministic mode: exact integer sums of the wave totals
            if (__any(anyv[u]) && slot >= 0)
              atomicAdd(det + (size_t)gid[u] * DET_REC + slot, det_quantize(v[u]));
          } else if constexpr (ATOMICS) {
            // 32-bit element offset (the entry points reject N >= 2^27): the atomic takes the
            // SGPR base + a VGPR offset, no 64-bit address arithmetic per iteration
            if (anyw[u] && slot >= 0)
              atomicAdd(rec + (uint32_t)(gid[u] * REC + slot), v[u]);
          } else {
            asm volatile("" ::"v"(v[u]));
          }
        }
      }
    }
    wave_lds_sync();
  }
  if constexpr (CNT) pair_count_flush(0, c_slots, c_live, c_valid);
  wlog.done(tile);
}

// ---------------------------------------------------------------- tile-wave backward
// One wave per 16x16 tile.  Lane l holds column l & 15 and rows rg, rg+4 | rg+8, rg+12
// (rg = l >> 4) as two float2 pixel pairs: pair 0 lies in the tile's top 16x8 half, pair 1 in
// the bottom half.  Each staged Gaussian carries two cull bits (top / bottom half, each also
// limited to that half's last contributing list position), and the blend of a pair runs only
// when its half is touched (a wave-uniform branch).  The per-Gaussian fixed cost -- LDS read,
// the nine partial sums, the reduce-scatter and the atomic -- is paid once per tile instead of
// once per 16x8 strip, while the per-pixel work keeps the 16x8 cull (measured on the headline
// scene: 191.5 staged Gaussians per tile against 293.2 strip iterations).
//
// Per pixel the blend drops two products and two selects of raster_bwd3p_kernel: for a
// Gaussian with o <= alpha_max the alpha clamp cannot bind (vis <= 1 wherever sigma >= 0), so
// alpha = o * vis and vis * v_alpha = (alpha * v_alpha) / o.  The lanes accumulate
// alpha * v_alpha and its dy moments; the factors -o and 1/o are applied once per Gaussian
// before the reduction.  A Gaussian with o > alpha_max takes the clamped form.
struct __attribute__((aligned(16))) GStageB {
  float x, y, ha, b;   // mean, 0.5*conic.a, conic.b
  float hc, o, r, g;   // 0.5*conic.c, opacity, colour
  float bl;
  int idx;             // position in the tile's sorted list
  int id;              // Gaussian id
  int halves;          // bit 0: touches the top 16x8 half, bit 1: the bottom half
};

template <bool CHUNKED = false, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(5, 8))) void
raster_bwd4_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, const float *__restrict__ final_Ts,
    const int *__restrict__ final_idx, const float *__restrict__ v_out,
    const float *__restrict__ v_out_alpha, float alpha_max, float *__restrict__ rec,
    int chunk = 0, const int *__restrict__ item_off = nullptr,
    const int *__restrict__ item_tile = nullptr, const int *__restrict__ ckpt_off = nullptr,
    const float4 *__restrict__ ckpt = nullptr, const int *__restrict__ order = nullptr,
    int *__restrict__ queue = nullptr) {
  constexpr int PXL = 4, LROWS = 4;
  const WaveLog wlog;
  __shared__ GStageB lds[WPB][64];
  const int nslots = CHUNKED ? item_off[tbx * tby] : tbx * tby;
  // one work slot (tile, or list-split item) per wave; with a queue, waves are persistent and
  // take further slots from it (first slots dealt in launch order, then queue + #waves)
  int tile = -1;
  auto run = [&](const int wslot) {
  int ctile = wslot, cj = 0;
  if (!CHUNKED && order && wslot < tbx * tby) ctile = order[wslot];
  if (CHUNKED) {
    ctile = item_tile[wslot];
    cj = wslot - item_off[ctile];
  }
  const WaveRect R = wave_rect<PXL, 16>(tbx, tby, H, W, ctile);
  if (!R.live) return;  // wave-uniform
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  tile = R.tile;
  const int j = R.j, i0 = R.i0;
  const float px = (float)j;
  // the two halves' pixel-centre rectangles (the bottom one may lie below the image)
  const float rx0 = R.rx0, rx1 = R.rx1;
  const float ty0 = R.ry0, ty1 = fminf(R.ry0 + 7.f, R.ry1);
  const float by0 = R.ry0 + 8.f, by1 = R.ry1;
  const bool bottom_live = by0 <= by1;
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
  f2 py[2], T[2], vr[2], vg[2], vb[2], q[2], Sb[2];
  int binf[PXL];
  int mb0 = -1, mb1 = -1;
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int i = i0 + LROWS * k, p = k >> 1;
    float Tf = 0.f, r = 0.f, g = 0.f, bl = 0.f, a = 0.f;
    int bf = -1;
    if (i < H && j < W) {
      const int pix = i * W + j;
      Tf = final_Ts[pix];
      bf = final_idx[pix];
      r = v_out[3 * pix];
      g = v_out[3 * pix + 1];
      bl = v_out[3 * pix + 2];
      a = v_out_alpha ? v_out_alpha[pix] : 0.f;
    }
    const float qk = Tf * (a - (bg0 * r + bg1 * g + bg2 * bl));
    if (k & 1) {
      py[p].y = (float)i; T[p].y = Tf; vr[p].y = r; vg[p].y = g; vb[p].y = bl; q[p].y = qk;
    } else {
      py[p].x = (float)i; T[p].x = Tf; vr[p].x = r; vg[p].x = g; vb[p].x = bl; q[p].x = qk;
    }
    Sb[p] = (f2)0.f;
    binf[k] = bf;
    if (p == 0) mb0 = max(mb0, bf); else mb1 = max(mb1, bf);
  }
  const int2 range = bins[tile];
  int lo = range.x, hi = range.y;
  if (CHUNKED) {
    const int len = range.y - range.x;
    const int m = len > chunk ? (len + chunk - 1) / chunk : 1;
    if (m > 1) {
      lo = range.x + cj * chunk;
      hi = min(lo + chunk, range.y);
      if (cj < m - 1) {  // start from the checkpoint after this chunk
        const size_t cb = (size_t)ckpt_off[tile] * (GS_BLOCK * GS_BLOCK);
        const int oy = (tile / tbx) * GS_BLOCK, ox = (tile % tbx) * GS_BLOCK;
#pragma unroll
        for (int k = 0; k < PXL; ++k) {
          const int i = i0 + LROWS * k, p = k >> 1;
          if (i < H && j < W) {
            const int lpix = (i - oy) * GS_BLOCK + (j - ox);
            const float4 cj4 = ckpt[cb + (size_t)cj * (GS_BLOCK * GS_BLOCK) + lpix];
            const float4 cf4 = ckpt[cb + (size_t)(m - 1) * (GS_BLOCK * GS_BLOCK) + lpix];
            const float vr_ = (k & 1) ? vr[p].y : vr[p].x, vg_ = (k & 1) ? vg[p].y : vg[p].x,
                        vb_ = (k & 1) ? vb[p].y : vb[p].x;
            const float sb = (cf4.y - cj4.y) * vr_ + (cf4.z - cj4.z) * vg_ + (cf4.w - cj4.w) * vb_;
            if (k & 1) { T[p].y = cj4.x; Sb[p].y = sb; } else { T[p].x = cj4.x; Sb[p].x = sb; }
          }
        }
      }
    }
  }
  mb0 = min(wave_max_int(mb0), hi - 1);
  mb1 = min(wave_max_int(mb1), hi - 1);
  const int slot = reduce9_slot();
  const int last = max(mb0, mb1);
  GStageB *stage = lds[wave];
  for (int b = last; b >= lo; b -= 64) {
    const int idx = b - lane;
    int halves = 0;
    GStageB s;
    if (idx >= lo) {
      const int g = gids[idx];
      const float2 xy = xys[g];
      const float a = conics[3 * g], bb = conics[3 * g + 1], c = conics[3 * g + 2];
      const float o = opacity[g];
      if (idx <= mb0 && touches_rect(xy.x, xy.y, a, bb, c, o, rx0, rx1, ty0, ty1)) halves = 1;
      if (bottom_live && idx <= mb1 &&
          touches_rect(xy.x, xy.y, a, bb, c, o, rx0, rx1, by0, by1))
        halves |= 2;
      if (halves) {
        s.x = xy.x;
        s.y = xy.y;
        s.ha = 0.5f * a;
        s.b = bb;
        s.hc = 0.5f * c;
        s.o = o;
        s.r = colors[3 * g];
        s.g = colors[3 * g + 1];
        s.bl = colors[3 * g + 2];
        s.idx = idx;
        s.id = g;
        s.halves = halves | (o <= alpha_max ? 0 : 4);
      }
    }
    const unsigned long long kmask = __ballot(halves != 0);
    if (halves) stage[lanes_below(kmask)] = s;
    const int n = __popcll(kmask);
    wave_lds_sync();
    for (int t = 0; t < n; ++t) {
      const GStageB G = stage[t];
      // bits 0/1: halves touched; bit 2: o > alpha_max (the clamped form)
      const int hv = __builtin_amdgcn_readfirstlane(G.halves);
      const float dx = G.x - px;
      const float hA = G.ha * dx * dx, bdx = G.b * dx;
      f2 sr = 0.f, sg = 0.f, sb = 0.f, sa = 0.f, Vy = 0.f, Vyy = 0.f;
      bool any = false;
      // one pixel pair: sa accumulates o * vis * v_alpha (the unclamped alpha times v_alpha)
      auto pair = [&](auto clamped, int p, int k0) {
        constexpr bool CL = decltype(clamped)::value;
        const f2 dy = G.y - py[p];
        const f2 sig = gs_sigma2v<f2>(G.hc, bdx, hA, dy);
        const f2 vis = gs_vis2v<f2>(sig);
        const f2 ov = G.o * vis;
        f2 al = ov;
        if constexpr (CL) al = (f2){fminf(alpha_max, ov.x), fminf(alpha_max, ov.y)};
        const bool v0 = G.idx <= binf[k0] && sig.x >= 0.f && al.x >= ALPHA_MIN;
        const bool v1 = G.idx <= binf[k0 + 1] && sig.y >= 0.f && al.y >= ALPHA_MIN;
        any = any || v0 || v1;
        const f2 am = {v0 ? al.x : 0.f, v1 ? al.y : 0.f};
        f2 ovm = am;
        if constexpr (CL) ovm = (f2){v0 ? ov.x : 0.f, v1 ? ov.y : 0.f};
        const f2 om = 1.f - am;
        const f2 ra = {__builtin_amdgcn_rcpf(om.x), __builtin_amdgcn_rcpf(om.y)};
        T[p] = T[p] * ra;
        const f2 fac = am * T[p];
        sr = vfma(fac, vr[p], sr);
        sg = vfma(fac, vg[p], sg);
        sb = vfma(fac, vb[p], sb);
        const f2 gv = vfma((f2)G.r, vr[p], vfma((f2)G.g, vg[p], G.bl * vb[p]));
        const f2 v_alpha = vfma(gv, T[p], ra * (q[p] - Sb[p]));
        Sb[p] = vfma(fac, gv, Sb[p]);
        const f2 va = ovm * v_alpha;
        sa += va;
        const f2 vady = va * dy;
        Vy += vady;
        Vyy = vfma(vady, dy, Vyy);
      };
      using F = std::integral_constant<bool, false>;
      using Tr = std::integral_constant<bool, true>;
      if (hv & 4) {
        if (hv & 1) pair(Tr{}, 0, 0);
        if (hv & 2) pair(Tr{}, 1, 2);
      } else {
        if (hv & 1) pair(F{}, 0, 0);
        if (hv & 2) pair(F{}, 1, 2);
      }
      if (__any(any)) {
        const float Sa = sa.x + sa.y;
        const float Vs = -Sa, Vys = -(Vy.x + Vy.y);
        const float dxV = dx * Vs;
        float parts[9];
        parts[0] = fmaf(2.f * G.ha, dxV, G.b * Vys);  // v_x
        parts[1] = fmaf(G.b, dxV, 2.f * G.hc * Vys);  // v_y
        parts[2] = dx * dxV;                          // 2 v_conic.a
        parts[3] = dx * Vys;                          // 2 v_conic.b
        parts[4] = -(Vyy.x + Vyy.y);                  // 2 v_conic.c
        parts[5] = sr.x + sr.y;
        parts[6] = sg.x + sg.y;
        parts[7] = sb.x + sb.y;
        parts[8] = Sa * __builtin_amdgcn_rcpf(G.o);  // v_opacity = sum vis * v_alpha
        const float v = reduce9(parts);
        if (slot >= 0) atomicAdd(rec + (size_t)G.id * REC + slot, v);
      }
    }
    wave_lds_sync();
  }
  };
  const int nw = gridDim.x * WPB;
  for (int wslot = block_slot() * WPB + (threadIdx.x >> 6); wslot < nslots;) {
    run(wslot);
    if (!queue) break;
    int v = 0;
    if ((threadIdx.x & 63) == 0) v = atomicAdd(queue, 1);
    wslot = nw + __builtin_amdgcn_readfirstlane(v);
  }
  wlog.done(tile);
}

// ---------------------------------------------------------------- grouped backward
// Row-local reduce-scatter of nine values over each 16-lane DPP row (row_ror:8,
// row_half_mirror, quad perms): afterwards nine lanes of every row each hold the row sum of
// one value (reduce9_row_slot() says which) -- four independent reductions per instruction.
__device__ __forceinline__ float reduce9_row(const float (&v)[9]) {
  const int lane = __lane_id();
  const bool h8 = lane & 8, h4 = lane & 4, h2 = lane & 2, h1 = lane & 1;
  const float a0 = dpp_pair_sum<0x128>(v[0], v[5], h8), a1 = dpp_pair_sum<0x128>(v[1], v[6], h8),
              a2 = dpp_pair_sum<0x128>(v[2], v[7], h8), a3 = dpp_pair_sum<0x128>(v[3], v[8], h8),
              a4 = dpp_pair_sum<0x128>(v[4], 0.f, h8);
  const float b0 = dpp_pair_sum<0x141>(a0, a2, h4), b1 = dpp_pair_sum<0x141>(a1, a3, h4),
              b2 = dpp_pair_sum<0x141>(a4, 0.f, h4);
  const float c0 = dpp_pair_sum<0x4E>(b0, b1, h2), c1 = dpp_pair_sum<0x4E>(b2, 0.f, h2);
  return dpp_pair_sum<0xB1>(c0, c1, h1);
}
__device__ __forceinline__ int reduce9_row_slot() {
  float p[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) p[k] = (__lane_id() & 15) == 0 ? (float)(k + 1) : 0.f;
  return (int)reduce9_row(p) - 1;
}
__device__ __forceinline__ int row_max_int(int v) {  // max over the lane's 16-lane row
  for (int off = 8; off >= 1; off >>= 1) {
    const int o = __shfl_xor(v, off, 64);
    v = v > o ? v : o;
  }
  return v;
}

// Backward with sub-wave lists (gsplat_debug_set_raster_variant flag 2048): the wave's 16x8
// strip is split into four 8x4 rectangles, one per 16-lane row (two vertically adjacent
// pixels per lane), and each row walks its own culled list of the staged Gaussians -- a
// Gaussian is visited only by the rows whose rectangle it can touch (exact min-sigma cull per
// rectangle, and idx <= the rectangle's largest final_idx), so a wave iteration carries up to
// four different Gaussians.  Per iteration each row reduce-scatters its nine partial sums
// with row-local DPP and one atomic instruction adds all four rows' records.
template <bool CHUNKED = false>
__global__ __launch_bounds__(256) void raster_bwd3g_kernel(
    int tbx, int tby, int H, int W, const int *__restrict__ gids, const int2 *__restrict__ bins,
    const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opacity,
    const float *__restrict__ background, const float *__restrict__ final_Ts,
    const int *__restrict__ final_idx, const float *__restrict__ v_out,
    const float *__restrict__ v_out_alpha, float alpha_max, float *__restrict__ rec,
    int chunk = 0, const int *__restrict__ item_off = nullptr,
    const int *__restrict__ item_tile = nullptr, const int *__restrict__ ckpt_off = nullptr,
    const float4 *__restrict__ ckpt = nullptr) {
  constexpr int PXL = 2, COLS = 16;
  typedef f2 PV;
  int ctile = -1, cj = 0;
  if (CHUNKED) {
    const int slot = wave_slot<PXL, COLS>();
    if (slot >= item_off[tbx * tby]) return;  // wave-uniform: past the last item
    ctile = item_tile[slot];
    cj = slot - item_off[ctile];
  }
  const WaveRect R = wave_rect<PXL, COLS>(tbx, tby, H, W, ctile);
  if (!R.live) return;  // wave-uniform
  __shared__ GStage lds[4][64];
  __shared__ unsigned char lists[4][4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 4, m = lane & 15;
  const int tile = R.tile;
  const int c0 = (int)R.rx0, r0 = (int)R.ry0;
  const int j = c0 + (grp & 1) * 8 + (m & 7);
  const int i0 = r0 + (grp >> 1) * 4 + (m >> 3) * 2;
  const float px = (float)j;
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
  PV py, T, vr, vg, vb, q, Sb;
  int binf[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = i0 + k;
    float Tf = 0.f, r = 0.f, g = 0.f, bl = 0.f, a = 0.f;
    int bf = -1;
    if (i < H && j < W) {
      const int pix = i * W + j;
      Tf = final_Ts[pix];
      bf = final_idx[pix];
      r = v_out[3 * pix];
      g = v_out[3 * pix + 1];
      bl = v_out[3 * pix + 2];
      a = v_out_alpha ? v_out_alpha[pix] : 0.f;
    }
    const float qk = Tf * (a - (bg0 * r + bg1 * g + bg2 * bl));
    if (k) {
      py.y = (float)i; T.y = Tf; vr.y = r; vg.y = g; vb.y = bl; q.y = qk;
    } else {
      py.x = (float)i; T.x = Tf; vr.x = r; vg.x = g; vb.x = bl; q.x = qk;
    }
    binf[k] = bf;
  }
  Sb = PV(0.f);
  const int2 range = bins[tile];
  int lo = range.x, hi = range.y;
  if (CHUNKED) {
    const int len = range.y - range.x;
    const int nch = len > chunk ? (len + chunk - 1) / chunk : 1;
    if (nch > 1) {
      lo = range.x + cj * chunk;
      hi = min(lo + chunk, range.y);
      if (cj < nch - 1) {  // start from the checkpoint after this chunk
        const size_t cb = (size_t)ckpt_off[tile] * (GS_BLOCK * GS_BLOCK);
        const int oy = (tile / tbx) * GS_BLOCK, ox = (tile % tbx) * GS_BLOCK;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int i = i0 + k;
          if (i < H && j < W) {
            const int lpix = (i - oy) * GS_BLOCK + (j - ox);
            const float4 cj4 = ckpt[cb + (size_t)cj * (GS_BLOCK * GS_BLOCK) + lpix];
            const float4 cf4 = ckpt[cb + (size_t)(nch - 1) * (GS_BLOCK * GS_BLOCK) + lpix];
            const float vr_ = k ? vr.y : vr.x, vg_ = k ? vg.y : vg.x, vb_ = k ? vb.y : vb.x;
            const float sb = (cf4.y - cj4.y) * vr_ + (cf4.z - cj4.z) * vg_ + (cf4.w - cj4.w) * vb_;
            if (k) { T.y = cj4.x; Sb.y = sb; } else { T.x = cj4.x; Sb.x = sb; }
          }
        }
      }
    }
  }
  // per-row (8x4 rectangle) largest final_idx, and the rectangles (wave-uniform)
  const int rmax = row_max_int(max(binf[0], binf[1]));
  int gmax[4];
  float gx0[4], gx1[4], gy0[4], gy1[4];
  bool gok[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    gmax[g] = __builtin_amdgcn_readlane(rmax, 16 * g);
    const int sx0 = c0 + (g & 1) * 8, sy0 = r0 + (g >> 1) * 4;
    gok[g] = sx0 < W && sy0 < H && gmax[g] >= 0;
    gx0[g] = (float)sx0;
    gx1[g] = (float)min(sx0 + 7, W - 1);
    gy0[g] = (float)sy0;
    gy1[g] = (float)min(sy0 + 3, H - 1);
  }
  const int maxbin = max(max(gmax[0], gmax[1]), max(gmax[2], gmax[3]));
  const int slot = reduce9_row_slot();
  const int last = min(maxbin, hi - 1);
  GStage *stage = lds[wave];
  for (int b = last; b >= lo; b -= 64) {
    const int idx = b - lane;
    GStage s;
    bool kg[4] = {false, false, false, false};
    if (idx >= lo) {
      const int gid = gids[idx];
      const float2 xy = xys[gid];
      const float a = conics[3 * gid], bb = conics[3 * gid + 1], c = conics[3 * gid + 2];
      const float o = opacity[gid];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        kg[g] = gok[g] && idx <= gmax[g] &&
                touches_rect(xy.x, xy.y, a, bb, c, o, gx0[g], gx1[g], gy0[g], gy1[g]);
      if (kg[0] || kg[1] || kg[2] || kg[3]) {
        s.x = xy.x;
        s.y = xy.y;
        s.ha = 0.5f * a;
        s.b = bb;
        s.hc = 0.5f * c;
        s.o = o;
        s.r = colors[3 * gid];
        s.g = colors[3 * gid + 1];
        s.bl = colors[3 * gid + 2];
        s.idx = idx;
        s.id = gid;
      }
    }
    const bool keep = kg[0] || kg[1] || kg[2] || kg[3];
    const unsigned long long kmask = __ballot(keep);
    const int my_slot = (int)lanes_below(kmask);
    if (keep) stage[my_slot] = s;
    int ng[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const unsigned long long gm = __ballot(kg[g]);
      ng[g] = __popcll(gm);
      if (kg[g]) lists[wave][g][lanes_below(gm)] = (unsigned char)my_slot;
    }
    wave_lds_sync();
    const int nmax = max(max(ng[0], ng[1]), max(ng[2], ng[3]));
    const int myn = grp == 0 ? ng[0] : grp == 1 ? ng[1] : grp == 2 ? ng[2] : ng[3];
    for (int t = 0; t < nmax; ++t) {
      const bool live = t < myn;
      GStage G = stage[lists[wave][grp][live ? t : 0] & 63];
      if (!live) G.r = G.g = G.bl = G.o = 0.f;  // keep T / Sb finite; no contribution
      const float dx = G.x - px;
      const float hA = G.ha * dx * dx, bdx = G.b * dx;
      const PV dy = G.y - py;
      const PV sig = gs_sigma2v<PV>(G.hc, bdx, hA, dy);
      const PV vis = gs_vis2v<PV>(sig);
      const PV ov = G.o * vis;
      const PV al = {fminf(alpha_max, ov.x), fminf(alpha_max, ov.y)};
      const bool v0 = live && G.idx <= binf[0] && sig.x >= 0.f && al.x >= ALPHA_MIN;
      const bool v1 = live && G.idx <= binf[1] && sig.y >= 0.f && al.y >= ALPHA_MIN;
      const PV am = {v0 ? al.x : 0.f, v1 ? al.y : 0.f};
      const PV vm = {v0 ? vis.x : 0.f, v1 ? vis.y : 0.f};
      const PV om = 1.f - am;
      const PV ra = {__builtin_amdgcn_rcpf(om.x), __builtin_amdgcn_rcpf(om.y)};
      T = T * ra;
      const PV fac = am * T;
      const PV gv = vfma(PV(G.r), vr, vfma(PV(G.g), vg, G.bl * vb));
      const PV v_alpha = vfma(gv, T, ra * (q - Sb));
      Sb = vfma(fac, gv, Sb);
      const unsigned long long amask = __ballot(v0 || v1);
      if (amask) {
        const PV vva = vm * v_alpha;
        const PV vs = vva * (-G.o);
        const PV vsdy = vs * dy;
        const float Vs = vs.x + vs.y, Vys = vsdy.x + vsdy.y;
        const float dxV = dx * Vs;
        float parts[9];
        parts[0] = fmaf(2.f * G.ha, dxV, G.b * Vys);  // v_x
        parts[1] = fmaf(G.b, dxV, 2.f * G.hc * Vys);  // v_y
        parts[2] = dx * dxV;                          // 2 v_conic.a
        parts[3] = dx * Vys;                          // 2 v_conic.b
        const PV vsdy2 = vsdy * dy;
        parts[4] = vsdy2.x + vsdy2.y;                 // 2 v_conic.c
        const PV fr = fac * vr, fg = fac * vg, fb = fac * vb;
        parts[5] = fr.x + fr.y;
        parts[6] = fg.x + fg.y;
        parts[7] = fb.x + fb.y;
        parts[8] = vva.x + vva.y;
        const float v = reduce9_row(parts);
        const bool row_any = ((amask >> (16 * grp)) & 0xFFFFull) != 0;
        if (row_any && slot >= 0) atomicAdd(rec + (size_t)G.id * REC + slot, v);
      }
    }
    wave_lds_sync();
  }
}

// Tile processing order (one workgroup): tiles by decreasing list length, ties by tile id.
// The backward deals consecutive work slots to CUs round-robin, so each SIMD receives one tile
// from every cost tier and the per-SIMD sums even out (longest-processing-time-first dealing).
// Keys (log2-spaced length bucket, tile) are sorted by an LDS bitonic sort; frames with more
// than 16,384 tiles keep the identity order.
constexpr int ORDER_MAX = 16384;
__global__ __launch_bounds__(1024) void tile_order_kernel(int T, const int2 *__restrict__ bins,
                                                          int *__restrict__ order) {
  __shared__ uint32_t key[ORDER_MAX];
  const int tid = threadIdx.x;
  if (T > ORDER_MAX) {
    for (int t = tid; t < T; t += 1024) order[t] = t;
    return;
  }
  int n = 1;
  while (n < T) n <<= 1;
  for (int t = tid; t < n; t += 1024) {
    uint32_t k = 0xFFFFFFFFu;  // padding sorts last
    if (t < T) {
      const int2 r = bins[t];
      const int len = max(r.y - r.x, 0);
      const uint32_t b = min(1023u, (uint32_t)(log2f((float)len + 1.f) * 64.f));
      k = ((1023u - b) << 18) | (uint32_t)t;  // descending length, ascending tile
    }
    key[t] = k;
  }
  __syncthreads();
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < (n >> 1); i += 1024) {
        const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint32_t a = key[lo], b = key[hi];
        if ((a > b) == up) {
          key[lo] = b;
          key[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int t = tid; t < T; t += 1024) order[t] = (int)(key[t] & 0x3FFFFu);
}

// List-split plan (one workgroup): per tile, the number of backward items (chunks of the
// depth-sorted list, 1 for a tile no longer than `chunk`, 0 for an empty one) and of forward
// checkpoints (as many as chunks for a split tile, else 0); exclusive scans of both give
// item_off[T + 1] / ckpt_off[T + 1], and item_tile[] maps each item back to its tile.
__global__ __launch_bounds__(1024) void chunk_plan_kernel(int T, const int2 *__restrict__ bins,
                                                          int chunk, int *__restrict__ item_off,
                                                          int *__restrict__ ckpt_off,
                                                          int *__restrict__ item_tile) {
  __shared__ int sa[1024], sc[1024];
  const int tid = threadIdx.x;
  const int per = (T + 1023) / 1024;
  const int t0 = min(T, tid * per), t1 = min(T, t0 + per);
  auto items = [&](int t, int &mi, int &mc) {
    const int2 r = bins[t];
    const int len = r.y - r.x;
    mi = len <= 0 ? 0 : (len > chunk ? (len + chunk - 1) / chunk : 1);
    mc = len > chunk ? mi : 0;
  };
  int a = 0, c = 0;
  for (int t = t0; t < t1; ++t) {
    int mi, mc;
    items(t, mi, mc);
    a += mi;
    c += mc;
  }
  sa[tid] = a;
  sc[tid] = c;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
    const int va = tid >= d ? sa[tid - d] : 0, vc = tid >= d ? sc[tid - d] : 0;
    __syncthreads();
    sa[tid] += va;
    sc[tid] += vc;
    __syncthreads();
  }
  int ra = sa[tid] - a, rc = sc[tid] - c;
  for (int t = t0; t < t1; ++t) {
    int mi, mc;
    items(t, mi, mc);
    item_off[t] = ra;
    ckpt_off[t] = rc;
    for (int k = 0; k < mi; ++k) item_tile[ra + k] = t;
    ra += mi;
    rc += mc;
  }
  if (tid == 1023) {
    item_off[T] = sa[1023];
    ckpt_off[T] = sc[1023];
  }
}

// Gradient records -> gsplat's v_xy [N,2], v_conic [N,3], v_colors [N,3], v_opacity [N].
// Scale of a record's conic.y sum into gsplat's v_conic.y: the records hold the gradient of
// each conic entry in gsplat's halved convention times 1/s; without the CONIC_HALF quirk
// v_conic.y is d loss / d conic.y, twice that.
static inline float conic_y_scale(float s) {
  return (g_quirks & GSPLAT_QUIRK_CONIC_HALF) ? s : 2.f * s;
}

__global__ __launch_bounds__(256) void split_grads_kernel(int n, const float4 *__restrict__ rec,
                                                          float conic_scale, float conic_scale_b,
                                                          float *__restrict__ v_xy,
                                                          float *__restrict__ v_conic,
                                                          float *__restrict__ v_rgb,
                                                          float *__restrict__ v_opacity) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= n) return;
  const float4 r0 = rec[(size_t)g * (REC / 4)], r1 = rec[(size_t)g * (REC / 4) + 1],
               r2 = rec[(size_t)g * (REC / 4) + 2];
  v_xy[2 * g] = r0.x;
  v_xy[2 * g + 1] = r0.y;
  v_conic[3 * g] = conic_scale * r0.z;
  v_conic[3 * g + 1] = conic_scale_b * r0.w;
  v_conic[3 * g + 2] = conic_scale * r1.x;
  v_rgb[3 * g] = r1.y;
  v_rgb[3 * g + 1] = r1.z;
  v_rgb[3 * g + 2] = r1.w;
  v_opacity[g] = r2.x;
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
    float *__restrict__ v_xy, float *__restrict__ v_conic, float *__restrict__ v_colors,
    float *__restrict__ v_opacity) {
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
        s_b = 0.5f * v_sigma * dx * dy;
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

// ---- list-split backward (checkpointed forward) ----------------------------------------
// Workspace layout (gsplat_rasterize_checkpoint_bytes): item_off[T+1], ckpt_off[T+1],
// item_tile[T + ceil(I/chunk)], 16-B aligned float4 ckpt[(2 ceil(I/chunk) + 1) * 256].
int g_chunk_override = 0;  // gsplat_debug_set_chunk: 0 auto, > 0 forced, < 0 off
struct ChunkWs {
  int *item_off, *ckpt_off, *item_tile;
  float4 *ckpt;
  long long items_bound, ckpt_bound;
  size_t bytes;
};
static ChunkWs carve_chunk_ws(void *base, long long T, long long I, int chunk) {
  ChunkWs w{};
  const long long per = (I + chunk - 1) / chunk;
  w.items_bound = T + per;
  w.ckpt_bound = 2 * per + 1;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return (char *)base + o;
  };
  w.item_off = (int *)take((size_t)(T + 1) * sizeof(int));
  w.ckpt_off = (int *)take((size_t)(T + 1) * sizeof(int));
  w.item_tile = (int *)take((size_t)w.items_bound * sizeof(int));
  w.ckpt = (float4 *)take((size_t)w.ckpt_bound * GS_BLOCK * GS_BLOCK * sizeof(float4));
  w.bytes = off;
  return w;
}
static bool default_variants() {  // (flag 4096, the tile-wave backward, keeps the layout)
  return g_fwd_pxl == FWD_PXL && g_bwd_pxl == BWD_PXL && (g_bwd_flags & ~4096) == 0;
}

extern "C" int gsplat_rasterize_chunk_size(int tile_bounds_x, int tile_bounds_y,
                                           int64_t num_intersects) {
  if (g_chunk_override < 0 || !default_variants() || num_intersects <= 0) return 0;
  if (g_chunk_override > 0) return (g_chunk_override + 63) / 64 * 64;
  // Split only frames with too few tiles to occupy the chip: the backward runs 2 waves per
  // tile and ~7 fit per SIMD (7,168 on 256 CUs), so below ~3,584 tiles (e.g. 512x512 =
  // 1,024) CUs sit idle and splitting lists into 256-position chunks pays (bear c3: backward
  // 0.269 -> 0.195 ms).  At 1080x1080 (4,624 tiles) the tile count already fills the chip
  // and splitting measured 12-30 % slower (pixels saturate early, so the front chunk keeps
  // the critical path while checkpoints cost traffic) -- see DESIGN.md.
  const long long T = (long long)tile_bounds_x * tile_bounds_y;
  return T < 3584 ? 256 : 0;
}

extern "C" size_t gsplat_rasterize_checkpoint_bytes(int tile_bounds_x, int tile_bounds_y,
                                                    int64_t num_intersects, int chunk) {
  if (chunk <= 0 || chunk % 64 || tile_bounds_x <= 0 || tile_bounds_y <= 0 || num_intersects < 0)
    return 0;
  return carve_chunk_ws(nullptr, (long long)tile_bounds_x * tile_bounds_y, num_intersects, chunk)
      .bytes;
}

extern "C" int gsplat_debug_set_chunk(int chunk) {
  g_chunk_override = chunk;
  return 0;
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
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0 || img_height <= 0 || img_width <= 0 ||
      channels < 1 || channels > 64 ||
      (long long)tile_bounds_x * GS_BLOCK < img_width ||
      (long long)tile_bounds_y * GS_BLOCK < img_height) {
    set_error("rasterize_forward: bad sizes (tiles=%dx%d H=%d W=%d C=%d)", tile_bounds_x,
              tile_bounds_y, img_height, img_width, channels);
    return 1;
  }
  const int T = tile_bounds_x * tile_bounds_y;
  if (channels == 3) {
#define FWD3(P)                                                                            \
  hipLaunchKernelGGL(raster_fwd3_kernel<P>, dim3(cdiv(T, P)), dim3(256), 0, st, tile_bounds_x, \
                     tile_bounds_y, img_height, img_width, gaussian_ids_sorted,                \
                     (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,    \
                     background, out_img, final_Ts, final_idx)
#define FWD3P(NP)                                                                          \
  hipLaunchKernelGGL(raster_fwd3p_kernel<NP>, dim3(cdiv(T, 2 * NP)), dim3(256), 0, st,          \
                     tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,  \
                     (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,     \
                     background, out_img, final_Ts, final_idx)
#define FWD3U(P, C)                                                                        \
  hipLaunchKernelGGL((raster_fwd3u_kernel<P, C>), dim3(cdiv(T, (tiles_per_block<P, C>()))),    \
                     dim3(256), 0, st, tile_bounds_x, tile_bounds_y, img_height, img_width,     \
                     gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys, conics, \
                     colors, opacity, background, out_img, final_Ts, final_idx)
    // flags: 4 scalar one-Gaussian-per-iteration kernel, 8 packed float2 kernel, 16 full-width
    // (16-column) rectangles; default: two Gaussians per iteration on 8-column rectangles.
    const bool scalar = g_bwd_flags & 4, packed = g_bwd_flags & 8, wide = g_bwd_flags & 16;
    if (g_fwd_pxl == 4) {
      if (scalar) FWD3(4); else if (packed) FWD3P(2); else FWD3U(4, 16);
    } else if (g_fwd_pxl == 2) {
      if (scalar) FWD3(2); else if (packed) FWD3P(1); else if (wide) FWD3U(2, 16); else FWD3U(2, 8);
    } else {
      if (scalar) FWD3(1); else if (wide) FWD3U(1, 16);
      else FWD3U(1, 8);
    }
#undef FWD3U
#undef FWD3
#undef FWD3P
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
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0 || img_height <= 0 || img_width <= 0 ||
      (long long)tile_bounds_x * GS_BLOCK < img_width ||
      (long long)tile_bounds_y * GS_BLOCK < img_height || !depths || !out_depth) {
    set_error("rasterize_forward_rgbd: bad sizes or NULL depth buffers (tiles=%dx%d H=%d W=%d)",
              tile_bounds_x, tile_bounds_y, img_height, img_width);
    return 1;
  }
  const int T = tile_bounds_x * tile_bounds_y;
  hipLaunchKernelGGL((raster_fwd3u_kernel<1, 8, true>), dim3(cdiv(T, (tiles_per_block<1, 8>()))),
                     dim3(256), 0, st, tile_bounds_x, tile_bounds_y, img_height, img_width,
                     gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys, conics,
                     colors, opacity, background, out_img, final_Ts, final_idx, depths,
                     out_depth);
  return check_launch("rasterize_forward_rgbd");
}

extern "C" int gsplat_debug_set_raster_variant(int fwd_pxl, int bwd_pxl, int bwd_flags) {
  auto ok = [](int p) { return p == 1 || p == 2 || p == 4; };
  if (!ok(fwd_pxl) || !ok(bwd_pxl)) {
    set_error("debug_set_raster_variant: pixels per lane must be 1, 2 or 4");
    return 1;
  }
  g_fwd_pxl = fwd_pxl;
  g_bwd_pxl = bwd_pxl;
  g_bwd_flags = bwd_flags & ~(1024 | (0xff << 20));
  const int chunk = (bwd_flags >> 20) & 0xff;
  const int remap = (bwd_flags & 1024) ? -1 : chunk == 0xff ? 0 : chunk ? chunk : XCD_CHUNK;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_xcd_remap), &remap, sizeof(int)) != hipSuccess) {
    set_error("debug_set_raster_variant: hipMemcpyToSymbol failed");
    return 1;
  }
  return 0;
}

extern "C" int gsplat_debug_set_tile_swizzle(int gw, int gh) {
  if (gw < 1 || gh < 1 || gw > 64 || gh > 64) {
    set_error("debug_set_tile_swizzle: group sides must be in 1..64");
    return 1;
  }
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_tile_gw), &gw, sizeof(int)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_tile_gh), &gh, sizeof(int)) != hipSuccess) {
    set_error("debug_set_tile_swizzle: hipMemcpyToSymbol failed");
    return 1;
  }
  return 0;
}

extern "C" int gsplat_debug_raster_variant_is_default(void) { return default_variants() ? 1 : 0; }

extern "C" int gsplat_set_deterministic(int on) {
  g_det = on != 0;
  return 0;
}
extern "C" int gsplat_get_deterministic(void) { return g_det ? 1 : 0; }

extern "C" int gsplat_debug_wave_log(void *buffer) {
  unsigned long long *p = (unsigned long long *)buffer;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_wave_log), &p, sizeof(p)) != hipSuccess) {
    set_error("debug_wave_log: hipMemcpyToSymbol failed");
    return 1;
  }
  return 0;
}

extern "C" int gsplat_debug_pair_count(void *buffer) {
  unsigned long long *p = (unsigned long long *)buffer;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_pair_count), &p, sizeof(p)) != hipSuccess) {
    set_error("debug_pair_count: hipMemcpyToSymbol failed");
    return 1;
  }
  g_pair_count_on = p != nullptr;
  return 0;
}

// The shipped 16x8-strip backward in deterministic mode (integer accumulators in det).
static void launch_bwd_det(hipStream_t st, int tbx, int tby, int H, int W, const int32_t *gids,
                           const int32_t *bins, const float *xys, const float *conics,
                           const float *colors, const float *opacity, const float *background,
                           const float *final_Ts, const int32_t *final_idx,
                           const float *v_output, const float *v_output_alpha, float alpha_max,
                           float *rec, unsigned long long *det) {
  hipLaunchKernelGGL((raster_bwd3p_kernel<1, true, 16, false, f2, true>),
                     dim3(cdiv((long long)tbx * tby, (tiles_per_block<2, 16>()))), dim3(256), 0,
                     st, tbx, tby, H, W, gids, (const int2 *)bins, (const float2 *)xys, conics,
                     colors, opacity, background, final_Ts, final_idx, v_output, v_output_alpha,
                     alpha_max, rec, false, 0, nullptr, nullptr, nullptr, nullptr, det);
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
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0 || img_height <= 0 || img_width <= 0 ||
      channels < 1 || channels > 64 || num_points < 0 || num_points >= MAX_BWD_POINTS ||
      (long long)tile_bounds_x * GS_BLOCK < img_width ||
      (long long)tile_bounds_y * GS_BLOCK < img_height) {
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
#define BWD3(P, A)                                                                         \
  hipLaunchKernelGGL((raster_bwd3_kernel<P, A>), dim3(cdiv(T, P)), dim3(256), 0, st,          \
                     tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,  \
                     (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,     \
                     background, final_Ts, final_idx, v_output, v_output_alpha, alpha_max, rec)
#define BWD3P(NP, A, C)                                                                    \
  hipLaunchKernelGGL((raster_bwd3p_kernel<NP, A, C>),                                       \
                     dim3(cdiv(T, (tiles_per_block<2 * NP, C>()))), dim3(256), 0, st,         \
                     tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,  \
                     (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,     \
                     background, final_Ts, final_idx, v_output, v_output_alpha, alpha_max, rec, \
                     (g_bwd_flags & 64) != 0)
    const bool atomics = !(g_bwd_flags & 1);
    const bool packed = g_bwd_pxl >= 2 && !(g_bwd_flags & 2);
    const bool narrow = g_bwd_flags & 32;  // 8-column wave rectangles
    if (g_det) {
      if (!default_variants() || (g_bwd_flags & 4096)) {
        set_error("rasterize_backward: deterministic mode needs the default raster variant");
        return 1;
      }
      unsigned long long *det = det_buffer(num_points, st);
      if (!det) return check_launch("rasterize_backward");
      launch_bwd_det(st, tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,
                     tile_bins, xys, conics, colors, opacity, background, final_Ts, final_idx,
                     v_output, v_output_alpha, alpha_max, rec, det);
      hipLaunchKernelGGL(det_finish_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0, st,
                         num_points, det, rec);
    } else if (packed) {
      if (g_bwd_pxl == 4) {
        if (atomics) BWD3P(2, true, 16); else BWD3P(2, false, 16);  // 16x16: one wave
      } else {
        if (narrow) { if (atomics) BWD3P(1, true, 8); else BWD3P(1, false, 8); }
        else if (atomics && (g_bwd_flags & 2048)) {  // sub-wave lists (8x4 rectangles per row)
          hipLaunchKernelGGL((raster_bwd3g_kernel<false>),
                             dim3(cdiv(T, (tiles_per_block<2, 16>()))), dim3(256), 0, st,
                             tile_bounds_x, tile_bounds_y, img_height, img_width,
                             gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys,
                             conics, colors, opacity, background, final_Ts, final_idx, v_output,
                             v_output_alpha, alpha_max, rec);
        }
        else if (atomics && (g_bwd_flags & 512)) {  // ablation: scalar pixel pairs
          hipLaunchKernelGGL((raster_bwd3p_kernel<1, true, 16, false, s2>),
                             dim3(cdiv(T, (tiles_per_block<2, 16>()))), dim3(256), 0, st,
                             tile_bounds_x, tile_bounds_y, img_height, img_width,
                             gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys,
                             conics, colors, opacity, background, final_Ts, final_idx, v_output,
                             v_output_alpha, alpha_max, rec, (g_bwd_flags & 64) != 0);
        } else if (atomics && (g_bwd_flags & 4096)) {  // ablation: one wave per tile
          if (g_bwd_flags & 8192)
            hipLaunchKernelGGL((raster_bwd4_kernel<false, 1>), dim3(T), dim3(64), 0, st,
                               tile_bounds_x, tile_bounds_y, img_height, img_width,
                               gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys,
                               conics, colors, opacity, background, final_Ts, final_idx, v_output,
                               v_output_alpha, alpha_max, rec);
          else {
            const int *ord = nullptr;
            if (g_bwd_flags & 16384) {
              static int *buf = nullptr;
              static int cap = 0;
              if (cap < T) {
                if (buf) (void)hipFree(buf);
                note(hipMalloc(&buf, (size_t)T * sizeof(int)), "hipMalloc");
                cap = T;
              }
              hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, st, T,
                                 (const int2 *)tile_bins, buf);
              ord = buf;
            }
            int *queue = nullptr;
            unsigned grid = cdiv(T, 4);
            const int pw = (g_bwd_flags >> 15) & 7;  // persistent waves per SIMD (0: off)
            if (pw && (unsigned)(256 * pw) < grid) {
              static int *qbuf = nullptr;
              if (!qbuf) note(hipMalloc(&qbuf, sizeof(int)), "hipMalloc");
              note(hipMemsetAsync(qbuf, 0, sizeof(int), st), "hipMemsetAsync");
              queue = qbuf;
              grid = 256 * pw;
            }
            hipLaunchKernelGGL((raster_bwd4_kernel<false>), dim3(grid), dim3(256), 0, st,
                               tile_bounds_x, tile_bounds_y, img_height, img_width,
                               gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys,
                               conics, colors, opacity, background, final_Ts, final_idx, v_output,
                               v_output_alpha, alpha_max, rec, 0, nullptr, nullptr, nullptr,
                               nullptr, ord, queue);
          }
        } else { if (atomics) BWD3P(1, true, 16); else BWD3P(1, false, 16); }  // 16x8 strips
      }
    } else if (g_bwd_pxl == 4) { if (atomics) BWD3(4, true); else BWD3(4, false); }
    else if (g_bwd_pxl == 1) { if (atomics) BWD3(1, true); else BWD3(1, false); }
    else { if (atomics) BWD3(2, true); else BWD3(2, false); }
#undef BWD3
#undef BWD3P
    hipLaunchKernelGGL(split_grads_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0, st,
                       num_points, (const float4 *)rec, packed ? 0.5f : 1.f,
                       conic_y_scale(packed ? 0.5f : 1.f), v_xy, v_conic, v_colors, v_opacity);
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
                v_output_alpha, alpha_max, v_xy, v_conic, v_colors, v_opacity);
  }
  return check_launch("rasterize_backward");
}

static int rasterize_forward_impl(int tile_bounds_x, int tile_bounds_y, int img_height,
                                  int img_width, const int32_t *gaussian_ids_sorted,
                                  const int32_t *tile_bins, const float *xys, const float *conics,
                                  const float *colors, const float *opacity,
                                  const float *background, float *out_img, float *final_Ts,
                                  int32_t *final_idx, int64_t num_intersects, int chunk,
                                  void *checkpoints, size_t checkpoint_bytes, void *zero,
                                  size_t zero_bytes, const int32_t *zero_radii, void *stream,
                                  const char *who) {
  hipStream_t st = (hipStream_t)stream;
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0 || img_height <= 0 || img_width <= 0 ||
      (long long)tile_bounds_x * GS_BLOCK < img_width ||
      (long long)tile_bounds_y * GS_BLOCK < img_height || (chunk > 0 && chunk % 64) ||
      num_intersects < 0 || zero_bytes % 16 || (zero_bytes && !zero) ||
      (zero_radii && zero_bytes % 64)) {
    set_error("%s: bad sizes (tiles=%dx%d H=%d W=%d chunk=%d zero=%zu)", who, tile_bounds_x,
              tile_bounds_y, img_height, img_width, chunk, zero_bytes);
    return 1;
  }
  const int T = tile_bounds_x * tile_bounds_y;
  const long long zn = (long long)(zero_bytes / 16);
  if (chunk <= 0) {
    if (!default_variants()) {  // debug variants: clear up front, then the variant's launch
      if (zn && hipMemsetAsync(zero, 0, zero_bytes, st) != hipSuccess) {
        set_error("%s: memset failed", who);
        return 1;
      }
      return gsplat_rasterize_forward(tile_bounds_x, tile_bounds_y, img_height, img_width, 3,
                                      gaussian_ids_sorted, tile_bins, xys, conics, colors,
                                      opacity, background, out_img, final_Ts, final_idx, stream);
    }
#define FWDU(CNT)                                                                          \
  hipLaunchKernelGGL((raster_fwd3u_kernel<1, 8, false, false, CNT>),                          \
                     dim3(cdiv(T, (tiles_per_block<1, 8>()))), dim3(256), 0, st, tile_bounds_x, \
                     tile_bounds_y, img_height, img_width, gaussian_ids_sorted,                 \
                     (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,     \
                     background, out_img, final_Ts, final_idx, nullptr, nullptr, 0, nullptr,    \
                     nullptr, (float4 *)zero, zn, zero_radii)
    if (g_pair_count_on) FWDU(true); else FWDU(false);
#undef FWDU
    return check_launch(who);
  }
  const ChunkWs w = carve_chunk_ws(checkpoints, T, num_intersects, chunk);
  if (!checkpoints || checkpoint_bytes < w.bytes || !default_variants()) {
    set_error("%s: checkpoint buffer %zu < %zu bytes (or non-default raster variant)", who,
              checkpoint_bytes, w.bytes);
    return 1;
  }
  hipLaunchKernelGGL(chunk_plan_kernel, dim3(1), dim3(1024), 0, st, T, (const int2 *)tile_bins,
                     chunk, w.item_off, w.ckpt_off, w.item_tile);
#define FWDC(CNT)                                                                          \
  hipLaunchKernelGGL((raster_fwd3u_kernel<1, 8, false, true, CNT>),                           \
                     dim3(cdiv(T, (tiles_per_block<1, 8>()))), dim3(256), 0, st, tile_bounds_x, \
                     tile_bounds_y, img_height, img_width, gaussian_ids_sorted,                 \
                     (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,     \
                     background, out_img, final_Ts, final_idx, nullptr, nullptr, chunk,         \
                     w.ckpt_off, w.ckpt, (float4 *)zero, zn, zero_radii)
  if (g_pair_count_on) FWDC(true); else FWDC(false);
#undef FWDC
  return check_launch(who);
}

extern "C" int gsplat_rasterize_forward_chunked(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    float *out_img, float *final_Ts, int32_t *final_idx, int64_t num_intersects, int chunk,
    void *checkpoints, size_t checkpoint_bytes, void *stream) {
  if (chunk <= 0)
    return gsplat_rasterize_forward(tile_bounds_x, tile_bounds_y, img_height, img_width, 3,
                                    gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity,
                                    background, out_img, final_Ts, final_idx, stream);
  return rasterize_forward_impl(tile_bounds_x, tile_bounds_y, img_height, img_width,
                                gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity,
                                background, out_img, final_Ts, final_idx, num_intersects, chunk,
                                checkpoints, checkpoint_bytes, nullptr, 0, nullptr, stream,
                                "rasterize_forward_chunked");
}

extern "C" int gsplat_rasterize_forward_clearing(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    float *out_img, float *final_Ts, int32_t *final_idx, int64_t num_intersects, int chunk,
    void *checkpoints, size_t checkpoint_bytes, void *clear, size_t clear_bytes,
    const int32_t *clear_radii, void *stream) {
  return rasterize_forward_impl(tile_bounds_x, tile_bounds_y, img_height, img_width,
                                gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity,
                                background, out_img, final_Ts, final_idx, num_intersects, chunk,
                                checkpoints, checkpoint_bytes, clear, clear_bytes, clear_radii,
                                stream, "rasterize_forward_clearing");
}

// List-split backward launch: two waves (16x8 strips) per (tile, chunk) item, or one wave per
// item with the tile-wave kernel (ablation flag 4096).
static void launch_bwd_chunked(hipStream_t st, int tbx, int tby, int H, int W, const int32_t *gids,
                               const int32_t *bins, const float *xys, const float *conics,
                               const float *colors, const float *opacity, const float *background,
                               const float *final_Ts, const int32_t *final_idx,
                               const float *v_output, const float *v_output_alpha,
                               float alpha_max, float *rec, int chunk, const ChunkWs &w,
                               unsigned long long *det = nullptr) {
  if (g_det) {
    hipLaunchKernelGGL((raster_bwd3p_kernel<1, true, 16, true, f2, true>),
                       dim3((unsigned)cdiv(w.items_bound, (long long)(tiles_per_block<2, 16>()))),
                       dim3(256), 0, st, tbx, tby, H, W, gids, (const int2 *)bins,
                       (const float2 *)xys, conics, colors, opacity, background, final_Ts,
                       final_idx, v_output, v_output_alpha, alpha_max, rec, false, chunk,
                       w.item_off, w.item_tile, w.ckpt_off, w.ckpt, det);
    return;
  }
  if (!(g_bwd_flags & 4096)) {
#define BWDC(CNT)                                                                          \
  hipLaunchKernelGGL((raster_bwd3p_kernel<1, true, 16, true, f2, false, CNT>),                \
                     dim3((unsigned)cdiv(w.items_bound, (long long)(tiles_per_block<2, 16>()))),\
                     dim3(256), 0, st, tbx, tby, H, W, gids, (const int2 *)bins,                \
                     (const float2 *)xys, conics, colors, opacity, background, final_Ts,        \
                     final_idx, v_output, v_output_alpha, alpha_max, rec, false, chunk,         \
                     w.item_off, w.item_tile, w.ckpt_off, w.ckpt)
    if (g_pair_count_on) BWDC(true); else BWDC(false);
#undef BWDC
    return;
  }
  hipLaunchKernelGGL((raster_bwd4_kernel<true>), dim3((unsigned)cdiv(w.items_bound, 4LL)),
                     dim3(256), 0, st, tbx, tby, H, W, gids, (const int2 *)bins,
                     (const float2 *)xys, conics, colors, opacity, background, final_Ts,
                     final_idx, v_output, v_output_alpha, alpha_max, rec, chunk, w.item_off,
                     w.item_tile, w.ckpt_off, w.ckpt);
}

extern "C" int gsplat_rasterize_backward_chunked(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, int num_points,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *v_output,
    const float *v_output_alpha, float alpha_max, float *v_xy, float *v_conic, float *v_colors,
    float *v_opacity, int64_t num_intersects, int chunk, const void *checkpoints,
    size_t checkpoint_bytes, void *workspace, size_t workspace_bytes, void *stream) {
  if (chunk <= 0)
    return gsplat_rasterize_backward(tile_bounds_x, tile_bounds_y, img_height, img_width, 3,
                                     num_points, gaussian_ids_sorted, tile_bins, xys, conics,
                                     colors, opacity, background, final_Ts, final_idx, v_output,
                                     v_output_alpha, alpha_max, v_xy, v_conic, v_colors,
                                     v_opacity, workspace, workspace_bytes, stream);
  hipStream_t st = (hipStream_t)stream;
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0 || img_height <= 0 || img_width <= 0 ||
      num_points < 0 || num_points >= MAX_BWD_POINTS ||
      (long long)tile_bounds_x * GS_BLOCK < img_width ||
      (long long)tile_bounds_y * GS_BLOCK < img_height || chunk % 64 || num_intersects < 0) {
    set_error("rasterize_backward_chunked: bad sizes (tiles=%dx%d H=%d W=%d N=%d chunk=%d)",
              tile_bounds_x, tile_bounds_y, img_height, img_width, num_points, chunk);
    return 1;
  }
  const int T = tile_bounds_x * tile_bounds_y;
  const ChunkWs w =
      carve_chunk_ws(const_cast<void *>(checkpoints), T, num_intersects, chunk);
  const size_t need = gsplat_rasterize_backward_workspace_size(num_points, 3);
  if (!checkpoints || checkpoint_bytes < w.bytes || workspace_bytes < need ||
      (need && !workspace) || !default_variants()) {
    set_error("rasterize_backward_chunked: buffers too small (checkpoints %zu < %zu or "
              "workspace %zu < %zu) or non-default raster variant",
              checkpoint_bytes, w.bytes, workspace_bytes, need);
    return 1;
  }
  if (num_points == 0) return check_launch("rasterize_backward_chunked");
  float *rec = (float *)workspace;
  note(hipMemsetAsync(rec, 0, need, st), "hipMemsetAsync");
  unsigned long long *det = g_det ? det_buffer(num_points, st) : nullptr;
  if (g_det && !det) return check_launch("rasterize_backward_chunked");
  launch_bwd_chunked(st, tile_bounds_x, tile_bounds_y, img_height, img_width,
                     gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity, background,
                     final_Ts, final_idx, v_output, v_output_alpha, alpha_max, rec, chunk, w, det);
  if (det)
    hipLaunchKernelGGL(det_finish_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0, st,
                       num_points, det, rec);
  hipLaunchKernelGGL(split_grads_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0, st,
                     num_points, (const float4 *)rec, 0.5f, conic_y_scale(0.5f), v_xy, v_conic,
                     v_colors, v_opacity);
  return check_launch("rasterize_backward_chunked");
}

extern "C" int gsplat_grad_records_split(int num_points, const void *records,
                                         size_t records_bytes, float *v_xy, float *v_conic,
                                         float *v_colors, float *v_opacity, void *stream) {
  const size_t need = num_points > 0 ? (size_t)num_points * REC * sizeof(float) : 0;
  if (num_points < 0 || records_bytes < need || (need && !records)) {
    set_error("grad_records_split: records %zu < %zu bytes (N=%d)", records_bytes, need,
              num_points);
    return 1;
  }
  if (num_points == 0) return 0;
  hipLaunchKernelGGL(split_grads_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0,
                     (hipStream_t)stream, num_points, (const float4 *)records, 0.5f,
                     conic_y_scale(0.5f), v_xy, v_conic, v_colors, v_opacity);
  return check_launch("grad_records_split");
}

extern "C" size_t gsplat_grad_records_bytes(int num_points) {
  return num_points > 0 ? (size_t)num_points * REC * sizeof(float) : 0;
}

extern "C" int gsplat_rasterize_backward_records(
    int tile_bounds_x, int tile_bounds_y, int img_height, int img_width, int num_points,
    const int32_t *gaussian_ids_sorted, const int32_t *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacity, const float *background,
    const float *final_Ts, const int32_t *final_idx, const float *v_output,
    const float *v_output_alpha, float alpha_max, int64_t num_intersects, int chunk,
    const void *checkpoints, size_t checkpoint_bytes, void *records, size_t records_bytes,
    void *stream) {
  hipStream_t st = (hipStream_t)stream;
  const size_t need = gsplat_grad_records_bytes(num_points);
  if (tile_bounds_x <= 0 || tile_bounds_y <= 0 || img_height <= 0 || img_width <= 0 ||
      num_points < 0 || num_points >= MAX_BWD_POINTS ||
      (long long)tile_bounds_x * GS_BLOCK < img_width ||
      (long long)tile_bounds_y * GS_BLOCK < img_height || num_intersects < 0 ||
      (chunk > 0 && chunk % 64) || records_bytes < need || (need && !records)) {
    set_error("rasterize_backward_records: bad sizes (tiles=%dx%d H=%d W=%d N=%d chunk=%d "
              "records %zu < %zu bytes)", tile_bounds_x, tile_bounds_y, img_height, img_width,
              num_points, chunk, records_bytes, need);
    return 1;
  }
  if (!default_variants()) {
    set_error("rasterize_backward_records: needs the default raster variant");
    return 1;
  }
  if (num_points == 0 || num_intersects == 0) return check_launch("rasterize_backward_records");
  const int T = tile_bounds_x * tile_bounds_y;
  float *rec = (float *)records;
  if (g_det && (g_bwd_flags & 4096)) {
    set_error("rasterize_backward_records: deterministic mode needs the strip backward");
    return 1;
  }
  // deterministic mode: the records' clear by the forward is superseded by the integer sums
  unsigned long long *det = g_det ? det_buffer(num_points, st) : nullptr;
  if (g_det && !det) return check_launch("rasterize_backward_records");
  if (chunk > 0) {
    const ChunkWs w = carve_chunk_ws(const_cast<void *>(checkpoints), T, num_intersects, chunk);
    if (!checkpoints || checkpoint_bytes < w.bytes) {
      set_error("rasterize_backward_records: checkpoint buffer %zu < %zu bytes", checkpoint_bytes,
                w.bytes);
      return 1;
    }
    launch_bwd_chunked(st, tile_bounds_x, tile_bounds_y, img_height, img_width,
                       gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity, background,
                       final_Ts, final_idx, v_output, v_output_alpha, alpha_max, rec, chunk, w,
                       det);
  } else if (det) {
    launch_bwd_det(st, tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,
                   tile_bins, xys, conics, colors, opacity, background, final_Ts, final_idx,
                   v_output, v_output_alpha, alpha_max, rec, det);
  } else if (g_bwd_flags & 4096) {
    hipLaunchKernelGGL((raster_bwd4_kernel<false>), dim3(cdiv(T, 4)), dim3(256), 0, st,
                       tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,
                       (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,
                       background, final_Ts, final_idx, v_output, v_output_alpha, alpha_max, rec);
  } else {
#define BWDR(CNT)                                                                          \
  hipLaunchKernelGGL((raster_bwd3p_kernel<1, true, 16, false, f2, false, CNT>),               \
                     dim3(cdiv(T, (tiles_per_block<2, 16>()))), dim3(256), 0, st,              \
                     tile_bounds_x, tile_bounds_y, img_height, img_width, gaussian_ids_sorted,  \
                     (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacity,     \
                     background, final_Ts, final_idx, v_output, v_output_alpha, alpha_max, rec, \
                     false)
    if (g_pair_count_on) BWDR(true); else BWDR(false);
#undef BWDR
  }
  if (det)
    hipLaunchKernelGGL(det_finish_kernel, dim3(cdiv(num_points, 256)), dim3(256), 0, st,
                       num_points, det, rec);
  return check_launch("rasterize_backward_records");
}
