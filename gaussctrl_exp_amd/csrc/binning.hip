// binning.hip -- tile binning for gfx950: device scan, stable LSD radix sort, fused
// depth-ordered intersection emission, tile bin edges, and the gsplat-layout utilities.
//
// Replaces, inside rasterize.py _RasterizeGaussians.forward (gsplat 0.1.2.1, reached from
// /root/reference/gaussctrl/gc_model.py:208-220 and :225-236):
//     cum_tiles_hit = torch.cumsum(num_tiles_hit); I = cum_tiles_hit[-1].item()
//     isect_ids, gaussian_ids = _C.map_gaussian_to_intersects(...)
//     isect_ids_sorted, idx = torch.sort(isect_ids); gaussian_ids_sorted = gather(...)
//     tile_bins = _C.get_tile_bin_edges(I, isect_ids_sorted)
//
// MI355X design (integer work, HBM-bound -- no MFMA):
//   The 64-bit key (tile << 32 | depth_bits) sort of gsplat moves 12 B per intersection
//   through ~6 eight-bit LSD passes.  Sorting by depth first -- N keys of 32 bits, N << I
//   -- and then stably by tile id -- ceil(log2(T+1)) <= 16 bits, two passes over I --
//   yields the identical order (ties by Gaussian id, as a stable sort of gsplat's keys)
//   while moving ~3.5x fewer bytes.  The emission of (tile, id) pairs happens directly in
//   depth order, and tile_bins falls out of the tile-sorted keys.
//
//   Radix pass = per-workgroup digit histogram (LDS atomics) -> device exclusive scan of
//   the [256][nblocks] histogram -> stable scatter whose in-wave rank comes from eight
//   wave64 ballots (a 64-lane match of the 8-bit digit).
#include "common.h"

namespace gs {
namespace {

constexpr int TPB = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = TPB * RS_ITEMS;  // keys per radix workgroup
constexpr int SC_ITEMS = 16;
constexpr int SC_TILE = TPB * SC_ITEMS;  // elements per scan workgroup

// ------------------------------------------------------------------ block scan helpers

// Exclusive scan of one uint per thread across a workgroup of NT threads (NT % 64 == 0).
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t &total,
                                                         uint32_t *lds /*[NT/64]*/) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t o = __shfl_up(inc, off, 64);
    if (lane >= off) inc += o;
  }
  if (lane == 63) lds[wave] = inc;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    uint32_t x = lds[w];
    if (w < wave) wbase += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return wbase + inc - v;
}

__global__ __launch_bounds__(TPB) void scan_reduce_kernel(const uint32_t *__restrict__ in,
                                                          long long m,
                                                          uint32_t *__restrict__ partial) {
  __shared__ uint32_t lds[TPB / 64];
  const long long base = (long long)blockIdx.x * SC_TILE;
  uint32_t s = 0;
#pragma unroll
  for (int r = 0; r < SC_ITEMS; ++r) {
    long long i = base + r * TPB + threadIdx.x;
    if (i < m) s += in[i];
  }
  uint32_t total;
  block_exclusive_scan<TPB>(s, total, lds);
  if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

// Single workgroup: exclusive scan of partial[0..nb) in place; grand total -> *total.
__global__ __launch_bounds__(1024) void scan_partials_kernel(uint32_t *__restrict__ partial,
                                                             int nb, uint32_t *__restrict__ total_out) {
  __shared__ uint32_t lds[16];
  uint32_t running = 0;
  for (int c = 0; c < nb; c += 1024) {
    int i = c + threadIdx.x;
    uint32_t v = i < nb ? partial[i] : 0u;
    uint32_t tot;
    uint32_t ex = block_exclusive_scan<1024>(v, tot, lds);
    if (i < nb) partial[i] = running + ex;
    running += tot;
  }
  if (total_out && threadIdx.x == 0) *total_out = running;
}

// out[i] = partial[block] + exclusive prefix inside the block's tile.  In place is allowed.
__global__ __launch_bounds__(TPB) void scan_downsweep_kernel(const uint32_t *in, long long m,
                                                             const uint32_t *__restrict__ partial,
                                                             uint32_t *out) {
  __shared__ uint32_t lds[TPB / 64];
  const long long base = (long long)blockIdx.x * SC_TILE + (long long)threadIdx.x * SC_ITEMS;
  uint32_t v[SC_ITEMS];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < SC_ITEMS; ++j) {
    long long i = base + j;
    v[j] = i < m ? in[i] : 0u;
    s += v[j];
  }
  uint32_t total;
  uint32_t run = partial[blockIdx.x] + block_exclusive_scan<TPB>(s, total, lds);
#pragma unroll
  for (int j = 0; j < SC_ITEMS; ++j) {
    long long i = base + j;
    if (i < m) out[i] = run;
    run += v[j];
  }
}

struct ScanWs {
  uint32_t *partial;  // cdiv(m, SC_TILE) entries
};

size_t scan_ws_bytes(long long m) { return (size_t)(cdiv(m, SC_TILE) + 1) * sizeof(uint32_t); }

// Exclusive scan of in[0..m) into out (in place allowed); total (device) optional.
void device_exclusive_scan(const uint32_t *in, uint32_t *out, long long m, uint32_t *total,
                           uint32_t *partial, hipStream_t st) {
  if (m <= 0) {
    if (total) note(hipMemsetAsync(total, 0, sizeof(uint32_t), st), "hipMemsetAsync");
    return;
  }
  int nb = (int)cdiv(m, SC_TILE);
  hipLaunchKernelGGL(scan_reduce_kernel, dim3(nb), dim3(TPB), 0, st, in, m, partial);
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, st, partial, nb, total);
  hipLaunchKernelGGL(scan_downsweep_kernel, dim3(nb), dim3(TPB), 0, st, in, m, partial, out);
}

// ------------------------------------------------------------------------ radix sort

template <typename K>
__global__ __launch_bounds__(TPB) void rs_upsweep_kernel(const K *__restrict__ keys, long long n,
                                                         int shift, int nblocks,
                                                         uint32_t *__restrict__ hist) {
  __shared__ uint32_t cnt[4][256];
  const int tid = threadIdx.x, wave = tid >> 6;
#pragma unroll
  for (int w = 0; w < 4; ++w) cnt[w][tid] = 0;
  __syncthreads();
  const long long base = (long long)blockIdx.x * RS_TILE;
#pragma unroll 4
  for (int r = 0; r < RS_ITEMS; ++r) {
    long long i = base + r * TPB + tid;
    if (i < n) {
      uint32_t d = (uint32_t)(keys[i] >> shift) & 255u;
      atomicAdd(&cnt[wave][d], 1u);
    }
  }
  __syncthreads();
  hist[(size_t)tid * nblocks + blockIdx.x] = cnt[0][tid] + cnt[1][tid] + cnt[2][tid] + cnt[3][tid];
}

template <typename K>
__global__ __launch_bounds__(TPB) void rs_downsweep_kernel(
    const K *__restrict__ kin, const uint32_t *__restrict__ vin, K *__restrict__ kout,
    uint32_t *__restrict__ vout, long long n, int shift, int nblocks,
    const uint32_t *__restrict__ hist_scanned) {
  __shared__ uint32_t digit_base[256];
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t woff[4][256];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  digit_base[tid] = hist_scanned[(size_t)tid * nblocks + blockIdx.x];
#pragma unroll
  for (int w = 0; w < 4; ++w) wcnt[w][tid] = 0;
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
  const long long base = (long long)blockIdx.x * RS_TILE;
  for (int r = 0; r < RS_ITEMS; ++r) {
    const long long i = base + r * TPB + tid;
    const bool valid = i < n;
    K key = valid ? kin[i] : (K)0;
    uint32_t val = valid ? vin[i] : 0u;
    const uint32_t d = (uint32_t)(key >> shift) & 255u;
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const unsigned long long m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    if (valid && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    {
      uint32_t s = digit_base[tid];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        uint32_t c = wcnt[w][tid];
        woff[w][tid] = s;
        s += c;
        wcnt[w][tid] = 0;
      }
      digit_base[tid] = s;
    }
    __syncthreads();
    if (valid) {
      const uint32_t pos = woff[wave][d] + rank;
      kout[pos] = key;
      vout[pos] = val;
    }
  }
}

size_t radix_ws_bytes(long long n) {
  long long nb = cdiv(n > 0 ? n : 1, RS_TILE);
  return (size_t)(256 * nb) * sizeof(uint32_t) + scan_ws_bytes(256 * nb);
}

// Stable LSD sort of (keys, vals) by bits [begin_bit, end_bit).  Ping-pongs between
// (ka, va) and (kb, vb); the final pass writes (kout, vout).  Inputs (ka, va) are clobbered
// unless there is exactly one pass.
template <typename K>
int radix_sort_pairs(K *ka, uint32_t *va, K *kb, uint32_t *vb, K *kout, uint32_t *vout,
                     long long n, int begin_bit, int end_bit, void *ws, hipStream_t st) {
  if (n <= 0) return 0;
  const int nb = (int)cdiv(n, RS_TILE);
  uint32_t *hist = (uint32_t *)ws;
  uint32_t *partial = hist + 256 * (size_t)nb;
  int passes = (end_bit - begin_bit + 7) / 8;
  if (passes <= 0) {
    note(hipMemcpyAsync(kout, ka, n * sizeof(K), hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
    note(hipMemcpyAsync(vout, va, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
    return 0;
  }
  K *kin = ka, *kalt = kb;
  uint32_t *vin = va, *valt = vb;
  for (int p = 0; p < passes; ++p) {
    const int shift = begin_bit + 8 * p;
    const bool last = p == passes - 1;
    K *ko = last ? kout : kalt;
    uint32_t *vo = last ? vout : valt;
    hipLaunchKernelGGL(rs_upsweep_kernel<K>, dim3(nb), dim3(TPB), 0, st, kin, n, shift, nb, hist);
    device_exclusive_scan(hist, hist, 256LL * nb, nullptr, partial, st);
    hipLaunchKernelGGL(rs_downsweep_kernel<K>, dim3(nb), dim3(TPB), 0, st, kin, vin, ko, vo, n,
                       shift, nb, hist);
    // next pass reads what this one wrote; its scratch is whatever it did not write
    K *kfree = (kin == ka || kin == kb) ? kin : kalt;
    uint32_t *vfree = (vin == va || vin == vb) ? vin : valt;
    kin = ko;
    vin = vo;
    kalt = kfree;
    valt = vfree;
  }
  return 0;
}

// ------------------------------------------------------------------ fused binning

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

// Depth keys: visible -> float bits of depth (positive floats order as uints), culled ->
// 0xFFFFFFFF (sorted last).  Also counts the visible Gaussians (wave ballot + one atomic).
__global__ __launch_bounds__(TPB) void depth_keys_kernel(int n, const float *__restrict__ depths,
                                                         const int *__restrict__ radii,
                                                         uint32_t *__restrict__ keys,
                                                         uint32_t *__restrict__ vals,
                                                         int *__restrict__ num_visible) {
  int i = blockIdx.x * TPB + threadIdx.x;
  bool vis = false;
  if (i < n) {
    vis = radii[i] > 0;
    keys[i] = vis ? __float_as_uint(depths[i]) : 0xFFFFFFFFu;
    vals[i] = (uint32_t)i;
  }
  unsigned long long b = __ballot(vis);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(num_visible, (int)__popcll(b));
}

__global__ __launch_bounds__(TPB) void gather_counts_kernel(int n, const uint32_t *__restrict__ order,
                                                            const int *__restrict__ radii,
                                                            const int *__restrict__ num_tiles_hit,
                                                            uint32_t *__restrict__ cnt) {
  int p = blockIdx.x * TPB + threadIdx.x;
  if (p >= n) return;
  uint32_t g = order[p];
  int c = radii[g] > 0 ? num_tiles_hit[g] : 0;
  cnt[p] = c > 0 ? (uint32_t)c : 0u;
}

// One lane per depth-ordered Gaussian writes its allotted cnt[p] (tile, id) pairs at
// off[p]; a bbox smaller than the allotment (inconsistent caller inputs) is padded with the
// sentinel tile id T, which sorts past every real tile and is ignored by the bins.
__global__ __launch_bounds__(TPB) void emit_kernel(int n, const uint32_t *__restrict__ order,
                                                   const uint32_t *__restrict__ cnt,
                                                   const uint32_t *__restrict__ off,
                                                   const float *__restrict__ xys,
                                                   const int *__restrict__ radii, int tbx, int tby,
                                                   uint32_t *__restrict__ tkeys,
                                                   uint32_t *__restrict__ tvals) {
  int p = blockIdx.x * TPB + threadIdx.x;
  if (p >= n) return;
  uint32_t c = cnt[p];
  if (c == 0) return;
  uint32_t g = order[p];
  uint32_t o = off[p];
  int x0, x1, y0, y1;
  tile_bbox(xys[2 * g], xys[2 * g + 1], (float)radii[g], tbx, tby, x0, x1, y0, y1);
  uint32_t j = 0;
  for (int y = y0; y < y1 && j < c; ++y)
    for (int x = x0; x < x1 && j < c; ++x, ++j) {
      tkeys[o + j] = (uint32_t)(y * tbx + x);
      tvals[o + j] = g;
    }
  for (; j < c; ++j) {
    tkeys[o + j] = (uint32_t)(tbx * tby);
    tvals[o + j] = g;
  }
}

// tile_bins[t] = [first, last+1) of tile t in the tile-sorted keys (tile_bins pre-zeroed).
template <typename K, int SHIFT>
__global__ __launch_bounds__(TPB) void bin_edges_kernel(long long n, const K *__restrict__ keys,
                                                        int *__restrict__ bins, long long rows) {
  long long k = (long long)blockIdx.x * TPB + threadIdx.x;
  if (k >= n) return;
  long long cur = (long long)(int32_t)(keys[k] >> SHIFT);
  if (k == 0 && cur >= 0 && cur < rows) bins[2 * cur] = 0;
  if (k == n - 1 && cur >= 0 && cur < rows) bins[2 * cur + 1] = (int)n;
  if (k == 0) return;
  long long prev = (long long)(int32_t)(keys[k - 1] >> SHIFT);
  if (prev != cur) {
    if (prev >= 0 && prev < rows) bins[2 * prev + 1] = (int)k;
    if (cur >= 0 && cur < rows) bins[2 * cur] = (int)k;
  }
}

// map_gaussian_to_intersects (gsplat layout: Gaussian-major, bbox row-major).
__global__ __launch_bounds__(TPB) void map_intersects_kernel(
    int n, const float *__restrict__ xys, const float *__restrict__ depths,
    const int *__restrict__ radii, const int *__restrict__ cum_tiles_hit, int tbx, int tby,
    long long *__restrict__ isect_ids, int *__restrict__ gaussian_ids) {
  int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n || radii[i] <= 0) return;
  int x0, x1, y0, y1;
  tile_bbox(xys[2 * i], xys[2 * i + 1], (float)radii[i], tbx, tby, x0, x1, y0, y1);
  int cur = i == 0 ? 0 : cum_tiles_hit[i - 1];
  long long depth_id = (long long)__float_as_int(depths[i]);  // sign-extended like gsplat
  for (int y = y0; y < y1; ++y)
    for (int x = x0; x < x1; ++x) {
      long long tile_id = (long long)(y * tbx + x);
      isect_ids[cur] = (tile_id << 32) | depth_id;
      gaussian_ids[cur] = i;
      ++cur;
    }
}

// ---- workspace layout of the fused binning (phase-1 region first, phase-2 after it) ----
constexpr size_t ALIGN = 256;
inline size_t al(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

struct Phase1 {
  uint32_t *dkeys_a, *dvals_a, *dkeys_b, *dvals_b, *dkeys_s, *order, *cnt, *off, *total;
  void *rs_ws;
  size_t bytes;
};

Phase1 carve_phase1(void *base, int n) {
  Phase1 p;
  char *c = (char *)base;
  size_t o = 0;
  auto take = [&](size_t b) {
    char *r = c + o;
    o += al(b);
    return r;
  };
  size_t nn = (size_t)(n > 0 ? n : 1) * 4;
  p.dkeys_a = (uint32_t *)take(nn);
  p.dvals_a = (uint32_t *)take(nn);
  p.dkeys_b = (uint32_t *)take(nn);
  p.dvals_b = (uint32_t *)take(nn);
  p.dkeys_s = (uint32_t *)take(nn);
  p.order = (uint32_t *)take(nn);
  p.cnt = (uint32_t *)take(nn);
  p.off = (uint32_t *)take(nn);
  p.total = (uint32_t *)take(16);
  size_t rs = radix_ws_bytes(n);
  size_t sc = scan_ws_bytes(n);
  p.rs_ws = take(rs > sc ? rs : sc);
  p.bytes = o;
  return p;
}

struct Phase2 {
  uint32_t *tk_a, *tv_a, *tk_b, *tv_b, *tk_s;
  void *rs_ws;
  size_t bytes;
};

Phase2 carve_phase2(void *base, long long I) {
  Phase2 p;
  char *c = (char *)base;
  size_t o = 0;
  auto take = [&](size_t b) {
    char *r = c + o;
    o += al(b);
    return r;
  };
  size_t ii = (size_t)(I > 0 ? I : 1) * 4;
  p.tk_a = (uint32_t *)take(ii);
  p.tv_a = (uint32_t *)take(ii);
  p.tk_b = (uint32_t *)take(ii);
  p.tv_b = (uint32_t *)take(ii);
  p.tk_s = (uint32_t *)take(ii);
  p.rs_ws = take(radix_ws_bytes(I));
  p.bytes = o;
  return p;
}

int bits_for(long long v) {  // smallest b with (1 << b) > v
  int b = 0;
  while (b < 62 && (1LL << b) <= v) ++b;
  return b;
}

}  // namespace
}  // namespace gs

using namespace gs;

extern "C" size_t gsplat_bin_count_workspace_size(int num_points) {
  return carve_phase1(nullptr, num_points).bytes;
}

extern "C" size_t gsplat_bin_emit_workspace_size(int64_t num_intersects) {
  return carve_phase2(nullptr, num_intersects).bytes;
}

extern "C" int gsplat_bin_count(int num_points, const float *depths, const int32_t *radii,
                                const int32_t *num_tiles_hit, int32_t *d_counts,
                                void *workspace1, size_t workspace1_bytes, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (num_points < 0) {
    set_error("bin_count: bad size");
    return 1;
  }
  Phase1 p = carve_phase1(workspace1, num_points);
  if (workspace1_bytes < p.bytes) {
    set_error("bin_count: workspace %zu < %zu bytes", workspace1_bytes, p.bytes);
    return 1;
  }
  note(hipMemsetAsync(d_counts, 0, 2 * sizeof(int32_t), st), "hipMemsetAsync");
  if (num_points == 0) return check_launch("bin_count");
  const int n = num_points;
  hipLaunchKernelGGL(depth_keys_kernel, dim3(cdiv(n, TPB)), dim3(TPB), 0, st, n, depths, radii,
                     p.dkeys_a, p.dvals_a, d_counts);
  radix_sort_pairs<uint32_t>(p.dkeys_a, p.dvals_a, p.dkeys_b, p.dvals_b, p.dkeys_s, p.order, n, 0,
                             32, p.rs_ws, st);
  hipLaunchKernelGGL(gather_counts_kernel, dim3(cdiv(n, TPB)), dim3(TPB), 0, st, n, p.order,
                     radii, num_tiles_hit, p.cnt);
  device_exclusive_scan(p.cnt, p.off, n, (uint32_t *)(d_counts + 1), (uint32_t *)p.rs_ws, st);
  return check_launch("bin_count");
}

extern "C" int gsplat_bin_emit(int num_points, int64_t num_intersects, const float *xys,
                               const int32_t *radii, int tile_bounds_x, int tile_bounds_y,
                               int32_t *gaussian_ids_sorted, int32_t *tile_bins,
                               const void *workspace1, size_t workspace1_bytes,
                               void *workspace2, size_t workspace2_bytes, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (num_points < 0 || num_intersects < 0 || num_intersects > 0x7FFFFFFFLL ||
      tile_bounds_x <= 0 || tile_bounds_y <= 0) {
    set_error("bin_emit: bad sizes (N=%d I=%lld tiles=%dx%d)", num_points,
              (long long)num_intersects, tile_bounds_x, tile_bounds_y);
    return 1;
  }
  Phase1 p1 = carve_phase1(const_cast<void *>(workspace1), num_points);
  Phase2 p2 = carve_phase2(workspace2, num_intersects);
  if (workspace1_bytes < p1.bytes || workspace2_bytes < p2.bytes) {
    set_error("bin_emit: workspaces %zu/%zu < %zu/%zu bytes", workspace1_bytes,
              workspace2_bytes, p1.bytes, p2.bytes);
    return 1;
  }
  const long long T = (long long)tile_bounds_x * tile_bounds_y;
  note(hipMemsetAsync(tile_bins, 0, (size_t)T * 2 * sizeof(int32_t), st), "hipMemsetAsync");
  if (num_intersects == 0 || num_points == 0) return check_launch("bin_emit");
  const int n = num_points;
  const long long I = num_intersects;
  hipLaunchKernelGGL(emit_kernel, dim3(cdiv(n, TPB)), dim3(TPB), 0, st, n, p1.order, p1.cnt,
                     p1.off, xys, radii, tile_bounds_x, tile_bounds_y, p2.tk_a, p2.tv_a);
  radix_sort_pairs<uint32_t>(p2.tk_a, p2.tv_a, p2.tk_b, p2.tv_b, p2.tk_s,
                             (uint32_t *)gaussian_ids_sorted, I, 0, bits_for(T), p2.rs_ws, st);
  hipLaunchKernelGGL((bin_edges_kernel<uint32_t, 0>), dim3(cdiv(I, TPB)), dim3(TPB), 0, st, I,
                     p2.tk_s, tile_bins, T);
  return check_launch("bin_emit");
}

extern "C" int gsplat_map_gaussian_to_intersects(int num_points, const float *xys,
                                                 const float *depths, const int32_t *radii,
                                                 const int32_t *cum_tiles_hit, int tile_bounds_x,
                                                 int tile_bounds_y, int64_t *isect_ids,
                                                 int32_t *gaussian_ids, void *stream) {
  if (num_points < 0) {
    set_error("map_gaussian_to_intersects: bad size");
    return 1;
  }
  if (num_points == 0) return 0;
  hipLaunchKernelGGL(map_intersects_kernel, dim3(cdiv(num_points, TPB)), dim3(TPB), 0,
                     (hipStream_t)stream, num_points, xys, depths, radii, cum_tiles_hit,
                     tile_bounds_x, tile_bounds_y, (long long *)isect_ids, gaussian_ids);
  return check_launch("map_gaussian_to_intersects");
}

extern "C" size_t gsplat_sort_isect_pairs_workspace_size(int64_t num_items) {
  size_t kk = al((size_t)(num_items > 0 ? num_items : 1) * 8);
  size_t vv = al((size_t)(num_items > 0 ? num_items : 1) * 4);
  return 2 * kk + 2 * vv + radix_ws_bytes(num_items);
}

extern "C" int gsplat_sort_isect_pairs(int64_t num_items, int key_bits, const int64_t *keys_in,
                                       const int32_t *vals_in, int64_t *keys_out,
                                       int32_t *vals_out, void *workspace,
                                       size_t workspace_bytes, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (num_items < 0 || key_bits < 0 || key_bits > 64) {
    set_error("sort_isect_pairs: bad args");
    return 1;
  }
  if (workspace_bytes < gsplat_sort_isect_pairs_workspace_size(num_items)) {
    set_error("sort_isect_pairs: workspace too small");
    return 1;
  }
  if (num_items == 0) return 0;
  size_t kk = al((size_t)num_items * 8), vv = al((size_t)num_items * 4);
  char *c = (char *)workspace;
  uint64_t *ka = (uint64_t *)c, *kb = (uint64_t *)(c + kk);
  uint32_t *va = (uint32_t *)(c + 2 * kk), *vb = (uint32_t *)(c + 2 * kk + vv);
  void *rs = c + 2 * kk + 2 * vv;
  note(hipMemcpyAsync(ka, keys_in, num_items * 8, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
  note(hipMemcpyAsync(va, vals_in, num_items * 4, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
  radix_sort_pairs<uint64_t>(ka, va, kb, vb, (uint64_t *)keys_out, (uint32_t *)vals_out,
                             num_items, 0, key_bits, rs, st);
  return check_launch("sort_isect_pairs");
}

extern "C" int gsplat_get_tile_bin_edges(int64_t num_intersects, const int64_t *isect_ids_sorted,
                                         int32_t *tile_bins, int64_t num_rows, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (num_intersects < 0 || num_rows < 0) {
    set_error("get_tile_bin_edges: bad sizes");
    return 1;
  }
  if (num_rows > 0) note(hipMemsetAsync(tile_bins, 0, (size_t)num_rows * 2 * sizeof(int32_t), st), "hipMemsetAsync");
  if (num_intersects == 0) return check_launch("get_tile_bin_edges");
  hipLaunchKernelGGL((bin_edges_kernel<uint64_t, 32>), dim3(cdiv(num_intersects, TPB)), dim3(TPB),
                     0, st, (long long)num_intersects, (const uint64_t *)isect_ids_sorted,
                     tile_bins, (long long)num_rows);
  return check_launch("get_tile_bin_edges");
}
