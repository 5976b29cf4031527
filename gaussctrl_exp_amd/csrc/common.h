// common.h -- shared device helpers for the gfx950 rasterizer kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gsplat_mi355x.h"

#define GS_BLOCK 16           // tile edge (gsplat config.h BLOCK_X = BLOCK_Y = 16)
#define GS_TILE_PIX 256       // pixels per tile
#define GS_WAVE 64            // CDNA wavefront

namespace gs {

// Error reporting for the C ABI (thread-local message, int status).
void set_error(const char *fmt, ...);
// Records the first failing HIP runtime call of the current C-ABI call; check_launch()
// reports it (or any pending launch error) and resets the record.
void note(hipError_t e, const char *what);
int check_launch(const char *what);


// gsplat 0.1.2.1 behaviours recalled but unverified (SURVEY.md Appendix A [VERIFY]); each is a
// bit of the process-wide quirk mask (gsplat_set_quirks, default GSPLAT_QUIRKS_ALL):
//   GSPLAT_QUIRK_ALPHA_099       A10: the backward clamps alpha at 0.99 (the forward at 0.999);
//                                off: 0.999 in both.  (Applied by the callers' alpha_max.)
//   GSPLAT_QUIRK_CONIC_HALF      A7/A9: v_conic.y = 1/2 v_sigma dx dy, paired with a conic VJP
//                                that takes it as the gradient of each symmetric off-diagonal;
//                                off: v_conic.y = v_sigma dx dy (d sigma / d conic.y) and the VJP
//                                halves it.  End-to-end gradients are identical either way.
//   GSPLAT_QUIRK_EWA_UNCLAMPED   A6: the EWA VJP recomputes t without the 1.3 tan_fov clamp;
//                                off: the Jacobian of the clamped forward (through the clamp).
extern int g_quirks;

static inline unsigned int cdiv(long long a, long long b) { return (unsigned int)((a + b - 1) / b); }

// Saturating float->int truncation, NaN -> 0: the semantics of v_cvt_i32_f32 (and of
// CUDA's cvt.rzi.s32.f32 that gsplat was compiled to).  Spelled out so the oracle's
// restatement matches it bit for bit.
__device__ __forceinline__ int f2i_sat(float x) {
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Order LDS traffic between the lanes of ONE wave (no workgroup barrier needed when a
// wave owns its LDS region).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Full-wave sum with DPP row ops; result valid in lane 63.
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                     0, __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false));
  return v;
}

// Full-wave sum broadcast as a wave-uniform (SGPR) value.
__device__ __forceinline__ float wave_sum(float v) {
  float r = wave_sum_to_lane63(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, r), 63));
}

// ---- wave64 reduce-scatters ----------------------------------------------------------
// Summing nine per-lane values with nine independent wave_sum()s costs ~9x18 serialised
// DPP slots.  Instead every exchange step halves the number of live slots per lane:
// lanes l / l^32 (v_permlane32_swap), l / l^16 (v_permlane16_swap), l / l^8 (row_ror:8),
// l / 7-l within 8 (row_half_mirror), then a quad sum.  Afterwards each quad of lanes holds
// the full wave sum of ONE of the values (no serial chain).  Which value a lane holds is
// learned once per wave with a probe (reduce_rec_slot, reduce18_slot).

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float,
                            __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF,
                                                        0xF, false));
}

// Pair exchange over lanes l / l^32 (or l^16): one half of the wave keeps x summed with the
// partner's x, the other half keeps y summed with the partner's y.
__device__ __forceinline__ float swap32_sum(float x, float y) {
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                            __builtin_bit_cast(unsigned, y), false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ float swap16_sum(float x, float y) {
  auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x),
                                            __builtin_bit_cast(unsigned, y), false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
// Same through a DPP pairing `ctrl` whose partner lane has the opposite `hi` bit.
template <int CTRL>
__device__ __forceinline__ float dpp_pair_sum(float x, float y, bool hi) {
  const float keep = hi ? y : x, send = hi ? x : y;
  return keep + dpp_f<CTRL>(send);
}

// ---- the record moments' reduce-scatter with the column factor applied mid-ladder --------
// Of the nine record sums of a strip-backward iteration, three are dx times another (sx = dx
// sa, sxx = dx sx, sxy = dx my; dx = G.x - px), and dx is constant along a lane's column
// (lane % 16: the 16-column strips), while the ladder's first two rungs (l^32, l^16) only add
// lanes of one column.  So only the six plain sums (sa, my, myy, r, g, b) take the l^32 rung
// (three swaps, no zero pad); lanes 0-31 then form the three products from their column sums,
// and the l^16 rung carries them beside the colours: 21 VALU ops against 25 for the plain
// ladder over the nine per-lane values (the zero-padded odd value at l^32 and l^16), with the
// products' three multiplies in both (profiles/r06_reduce9_fusion_ab.txt).  The odd slot at
// the l^8 rung is summed in both lanes of the pair (one fused DPP add instead of two selects).
// Afterwards lanes 0-15 hold sa / my / myy totals, 16-31 sx / sxx / sxy, 32-47 r / g / b
// (quads 0, 2, 1 of each sixteen; quad 3 a duplicate), lanes 48-63 products of the colour
// sums (unused).
__device__ __forceinline__ float reduce_rec(float sa, float my, float myy, float r, float g,
                                            float b, float dx) {
  const int lane = __lane_id();
  const float a0 = swap32_sum(sa, r), a1 = swap32_sum(my, g), a2 = swap32_sum(myy, b);
  const float e0 = dx * a0, e1 = dx * e0, e2 = dx * a1;
  const float b0 = swap16_sum(a0, e0), b1 = swap16_sum(a1, e1), b2 = swap16_sum(a2, e2);
  const bool h8 = lane & 8, h4 = lane & 4;
  const float c0 = dpp_pair_sum<0x128>(b0, b1, h8), c1 = b2 + dpp_f<0x128>(b2);
  float d = dpp_pair_sum<0x141>(c0, c1, h4);
  d += dpp_f<0xB1>(d);
  d += dpp_f<0x4E>(d);
  // kept ahead of the caller's atomic branch: sunk into it, the last add lost its DPP fusion
  // (a zeroed move + a DPP move + an add per iteration instead of one v_add_f32_dpp)
  asm volatile("" : "+v"(d));
  return d;
}
// The record field reduce_rec() leaves in this lane (one lane per quad), -1 elsewhere: found
// by reducing a probe (lane 0 holds 1..6, dx = 16 in every lane) and decoding the totals.
__device__ __forceinline__ int reduce_rec_slot(int sx, int sy, int sxx, int sxy, int syy, int r,
                                               int g, int b, int s0) {
  const int lane = __lane_id();
  const bool l0 = lane == 0;
  const float v = reduce_rec(l0 ? 1.f : 0.f, l0 ? 2.f : 0.f, l0 ? 3.f : 0.f, l0 ? 4.f : 0.f,
                             l0 ? 5.f : 0.f, l0 ? 6.f : 0.f, 16.f);
  if ((lane & 3) || (lane & 12) == 12 || lane >= 48) return -1;
  return v == 1.f ? s0 : v == 2.f ? sy : v == 3.f ? syy : v == 4.f ? r : v == 5.f ? g
       : v == 6.f ? b : v == 16.f ? sx : v == 256.f ? sxx : v == 32.f ? sxy : -1;
}

// ---- wave64 reduce-scatter of eighteen values (two Gaussians' nine record moments) -------
// The halving ladder (above) over eighteen values, one rung more: l^32 (18 -> 9: lanes 0-31 keep the
// first nine, 32-63 the second nine), l^16 (9 -> 5), l^8 (5 -> 3), 7-l within eight (3 -> 2),
// l^1 (2 -> 1), and a final sum with l^2.  Each value's total ends in two lanes (l, l^2) of
// one quad: 47 VALU ops for 18 values (two nine-value ladders: 54).
__device__ __forceinline__ float reduce18(const float (&v)[18]) {
  const int lane = __lane_id();
  float a[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) a[k] = swap32_sum(v[k], v[k + 9]);
  float b[5];
#pragma unroll
  for (int k = 0; k < 4; ++k) b[k] = swap16_sum(a[2 * k], a[2 * k + 1]);
  b[4] = swap16_sum(a[8], 0.f);
  const bool h8 = lane & 8, h4 = lane & 4, h1 = lane & 1;
  // the odd slots at l^8 and 7-l are summed in both lanes of their pairs (one fused DPP add
  // each instead of two selects and a zero-padded add); reduce18_slot drops the duplicates
  const float c0 = dpp_pair_sum<0x128>(b[0], b[1], h8), c1 = dpp_pair_sum<0x128>(b[2], b[3], h8),
              c2 = b[4] + dpp_f<0x128>(b[4]);
  const float d0 = dpp_pair_sum<0x141>(c0, c1, h4), d1 = c2 + dpp_f<0x141>(c2);
  float e = dpp_pair_sum<0xB1>(d0, d1, h1);  // quad_perm [1,0,3,2]
  e += dpp_f<0x4E>(e);                        // quad_perm [2,3,0,1]
  asm volatile("" : "+v"(e));  // (kept fused ahead of the caller's atomic branch)
  return e;
}

// Which of the eighteen values reduce18() leaves in this lane: 0..17 for one lane of each
// holding pair (lane bit 1 clear, the lowest such lane), -1 elsewhere (found by a probe,
// like reduce_rec_slot).
__device__ __forceinline__ int reduce18_slot() {
  const int lane = __lane_id();
  float p[18];
#pragma unroll
  for (int k = 0; k < 18; ++k) p[k] = lane == 0 ? (float)(k + 1) : 0.f;
  const int s = (int)reduce18(p) - 1;
  const int cand = (lane & 2) == 0 ? s : -1;
  // a value also left in other lanes (the odd slots' duplicates) is taken from its lowest lane
  int keep = cand;
  for (int k = 0; k < 64; ++k)
    if (k < lane && cand >= 0 && __builtin_amdgcn_readlane(cand, k) == cand) keep = -1;
  return keep;
}

// ---- per-Gaussian gradient records (the C=3 backward's accumulators) -----------------------
// One 64-B record per Gaussian holds the raster gradient as pixel moments, summed over every
// pixel p the Gaussian is composited at (over all tiles), with d = xy - p and
// w_p = vis_p * v_alpha_p (the per-pixel opacity gradient, gsplat backward.cu's vis * v_alpha):
//   0 Sx = sum dx w, 1 Sy = sum dy w, 2 Sxx = sum dx^2 w, 3 Sxy = sum dx dy w,
//   4 Syy = sum dy^2 w, 5..7 v_rgb = sum alpha T v_out, 8 S0 = sum w (= v_opacity).
// Every pixel of a Gaussian shares its conic and opacity o, so gsplat's per-pixel
//   v_sigma = -o w,  v_conic = 1/2 v_sigma (dx^2, dx dy, dy^2),
//   v_xy = v_sigma (a dx + b dy, b dx + c dy)
// sum to the closed forms of record_grads() -- applied once per Gaussian when the record is
// read, instead of per pixel or per wave iteration.
enum { REC_SX = 0, REC_SY, REC_SXX, REC_SXY, REC_SYY, REC_R, REC_G, REC_B, REC_S0, REC_FIELDS };
struct RasterGrads {
  float vxy[2], vconic[3], vrgb[3], vopacity;
};
// conic_y_full: GSPLAT_QUIRK_CONIC_HALF off (v_conic.y = d loss / d conic.y = -o Sxy).
__host__ __device__ __forceinline__ RasterGrads record_grads(const float *r, float ca, float cb,
                                                              float cc, float o,
                                                              bool conic_y_full) {
  RasterGrads g;
  const float no = -o;
  g.vxy[0] = no * (ca * r[REC_SX] + cb * r[REC_SY]);
  g.vxy[1] = no * (cb * r[REC_SX] + cc * r[REC_SY]);
  g.vconic[0] = 0.5f * no * r[REC_SXX];
  g.vconic[1] = (conic_y_full ? 1.f : 0.5f) * no * r[REC_SXY];
  g.vconic[2] = 0.5f * no * r[REC_SYY];
  g.vrgb[0] = r[REC_R];
  g.vrgb[1] = r[REC_G];
  g.vrgb[2] = r[REC_B];
  g.vopacity = r[REC_S0];
  return g;
}

__device__ __forceinline__ int wave_max_int(int v) {
  for (int off = 32; off >= 1; off >>= 1) {
    int o = __shfl_xor(v, off, 64);
    v = v > o ? v : o;
  }
  return v;
}

// The depth-sort inputs inside a gsplat_bin_count workspace (binning.hip): keys [n] (depth
// bits, 0xFFFFFFFF culled), vals [n] (Gaussian ids) and the per-Gaussian binning record
// {tile allotment, x0 | y0 << 16, x1 | y1 << 16, 0} [n].  `bytes` = the workspace size.
struct BinKeys {
  uint32_t *keys, *vals;
  uint4 *rec;
  size_t bytes;
};
BinKeys bin_keys_view(void *workspace1, int n);

}  // namespace gs
