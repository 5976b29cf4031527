// binning.hip -- tile binning for gfx950: device scan, stable one-sweep LSD radix sort,
// fused depth-ordered intersection emission, tile bin edges, and the gsplat-layout
// utilities.
//
// Replaces, inside rasterize.py _RasterizeGaussians.forward (gsplat 0.1.2.1, reached from
// /root/reference/gaussctrl/gc_model.py:208-220 and :225-236):
//     cum_tiles_hit = torch.cumsum(num_tiles_hit); I = cum_tiles_hit[-1].item()
//     isect_ids, gaussian_ids = _C.map_gaussian_to_intersects(...)
//     isect_ids_sorted, idx = torch.sort(isect_ids); gaussian_ids_sorted = gather(...)
//     tile_bins = _C.get_tile_bin_edges(I, isect_ids_sorted)
//
// MI355X design (integer work, HBM-bound -- no MFMA):
//   * gsplat sorts I 64-bit keys (tile << 32 | depth_bits).  Sorting the N visible depths
//     first (32-bit keys, N << I) and then the I intersections stably by tile id
//     (ceil(log2(T+1)) <= 16 bits, two passes) gives the identical order -- ties by Gaussian
//     id, as a stable sort of gsplat's keys -- while moving ~3.5x fewer bytes.
//   * Radix sort = one histogram kernel for all digit passes (one read of the keys), then
//     ONE kernel per pass: each workgroup takes a 4096-key tile by ticket, ranks it stably in
//     LDS (wave64 ballot match of the digit, per-wave LDS counters), publishes its digit
//     counts, obtains its global offsets by decoupled look-back over the preceding tiles'
//     tagged status words (agent-scope relaxed atomics, bounded spins), and writes the
//     tile out from LDS in digit order so each digit's run is written by consecutive lanes.
//     Digit width is ceil(bits / passes), so a 13-bit tile key takes two 7-bit passes.
//   * Emission: one wave per 64 depth-ordered Gaussians fills their combined slot range
//     with lanes striding over it (owner found by a 6-step shuffle search), so the
//     (tile, id) stores are coalesced.
#include "common.h"

namespace gs {
namespace {

constexpr int TPB = 256;
// Scan tile of 1,024 entries: the depth-ordered gather of the binning records (one dependent
// load chain per item) runs in 4x as many workgroups as with 4,096 (bin_count_keyed 0.112 ->
// 0.106 ms at the headline, c5 0.285 -> 0.264; profiles/r03_scan_tile_ab.txt).
constexpr int SC_ITEMS = 4;
constexpr int SC_TILE = TPB * SC_ITEMS;  // elements per scan workgroup
// keys per thread of a sort pass (workgroup tile = TPB * items): small sorts use short tiles
// so that more, shorter workgroups run at once (a pass is a chain of latencies per workgroup)
// Keys per thread of a sort pass: 16 (4,096-key tiles) from 4M keys, and for the 32-bit depth
// sort from 448 such tiles, 8 from 256 tiles of 2,048; else 4.  Measured with the XCD-chunked
// tiles (profiles/r06_sort_items_ab.txt): c4's 2M depth keys prefer 16 (binning 0.301 -> 0.291
// ms), the headline's 1M depth keys 8 (-2 to -4 us against 4; 244 tiles of 16 leave CUs idle),
// and c3's tile sort at its 1.9M capacity 4 (0.123 -> 0.126 ms with 16).  (Until round 6: 16
// from 4M keys for all, else 4.)
#ifndef GS_ITEMS16_FROM  // (A/B builds)
#define GS_ITEMS16_FROM (4LL << 20)
#endif
#ifndef GS_ITEMS16_DEPTH_FROM
#define GS_ITEMS16_DEPTH_FROM (448LL * 4096)
#endif
#ifndef GS_ITEMS8_DEPTH_FROM  // (A/B builds)
#define GS_ITEMS8_DEPTH_FROM (256LL * 2048)
#endif
int os_items_for(long long n, int bits) {
  if (n >= (long long)(bits == 32 ? GS_ITEMS16_DEPTH_FROM : GS_ITEMS16_FROM)) return 16;
  return bits == 32 && n >= (long long)(GS_ITEMS8_DEPTH_FROM) ? 8 : 4;
}

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

// The lanes of the wave whose digit d equals this lane's (a ballot match over the digit's
// `width` bits; `valid` lanes only).  Per bit: one sign-extending bit extract (-1 if set), one
// ballot and one three-input bit operation per 32-lane half: peers &= ~(ballot ^ mask).
template <int MAXW>
__device__ __forceinline__ unsigned long long digit_peers(uint32_t d, int width, bool valid) {
  const unsigned long long v = __ballot(valid);
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
  for (int b = 0; b < MAXW; ++b) {
    if (b >= width) break;  // uniform
    const uint32_t mask = (uint32_t)((int32_t)(d << (31 - b)) >> 31);
    const unsigned long long m = __ballot(mask != 0u);
    lo &= ~((uint32_t)m ^ mask);
    hi &= ~((uint32_t)(m >> 32) ^ mask);
  }
  return ((unsigned long long)hi << 32) | lo;
}

// Single workgroup: exclusive scan of partial[0..nb) in place; grand total -> *total.
// (in_place false: only the total, partial[] left as the block sums)
// kfin / assume / vflag: the count phase's depth-key range check for a later emission call
// (gsplat_bin_emit_speculative): vflag = 1 when a digit the sort assumed constant varied.
__global__ __launch_bounds__(1024) void scan_partials_kernel(uint32_t *__restrict__ partial,
                                                             int nb, uint32_t *__restrict__ total_out,
                                                             uint32_t *__restrict__ total_dev = nullptr,
                                                             bool in_place = true,
                                                             const uint32_t *__restrict__ kfin = nullptr,
                                                             uint32_t assume = 0,
                                                             uint32_t *__restrict__ vflag = nullptr,
                                                             uint32_t *__restrict__ out = nullptr) {
  __shared__ uint32_t lds[16];
  uint32_t running = 0;
  for (int c = 0; c < nb; c += 1024) {
    int i = c + threadIdx.x;
    uint32_t v = i < nb ? partial[i] : 0u;
    uint32_t tot;
    uint32_t ex = block_exclusive_scan<1024>(v, tot, lds);
    if (in_place && i < nb) partial[i] = running + ex;
    if (out && i < nb) out[i] = running + ex;  // (out of place: out[nb] = the total, below)
    running += tot;
  }
  if (threadIdx.x == 0) {
    if (total_dev) *total_dev = running;  // device copy (read by the pre-launched emission)
    if (total_out) *total_out = running;
    if (vflag) *vflag = (assume && kfin && ((kfin[0] ^ kfin[1]) & assume)) ? 1u : 0u;
    if (out) out[nb] = running;
  }
}

size_t scan_ws_bytes(long long m) { return (size_t)(cdiv(m, SC_TILE) + 1) * sizeof(uint32_t); }

// ------------------------------------------------------------ one-sweep radix sort

struct SortPlan {
  int passes, width, radix, items;
  long long nblocks;
};

SortPlan sort_plan(long long n, int begin_bit, int end_bit) {
  SortPlan p;
  int bits = end_bit - begin_bit;
  p.passes = bits <= 0 ? 0 : (bits + 7) / 8;
  p.width = p.passes ? (bits + p.passes - 1) / p.passes : 0;
  p.radix = 1 << p.width;
  p.items = os_items_for(n, bits);
  p.nblocks = n > 0 ? cdiv(n, (long long)TPB * p.items) : 0;
  return p;
}

// Workspace: [head: 16 words (1: kept-key count, 2-3: key range)] | tile digit counts
// [radix][nblocks] | row totals | per-tile key ranges
constexpr size_t OS_HEAD_WORDS = 16;

// [head words][one-sweep status: passes x nblocks x radix | reduce-then-scan tile counts
// nblocks x radix + scan scratch]
size_t radix_main_bytes(const SortPlan &p) {
  return (OS_HEAD_WORDS + (size_t)p.nblocks * p.radix + 256) * sizeof(uint32_t);
}

// [head][per-pass state][per-tile key range: nblocks x (and, or)]
size_t radix_ws_bytes(long long n, int begin_bit, int end_bit) {
  const SortPlan p = sort_plan(n, begin_bit, end_bit);
  return radix_main_bytes(p) + (size_t)p.nblocks * 2 * sizeof(uint32_t);
}

// Key range of the compacting depth sort: the AND and OR of all kept keys.  A digit on which
// they agree is the same for every key, so its LSD pass is the identity permutation: its count
// and row-scan kernels return at once and its pass kernel only copies (the launches are issued
// before the range is known).  blk: per-tile (and, or) from pass 0's count (or the key kernel);
// fin: their reduction, by pass 0's row scan.
struct KeyRange {
  uint32_t *blk = nullptr;
  uint32_t *fin = nullptr;
  long long nblk = 0;
  // Passes the host did not launch at all (gsplat_bin_count_keyed_ex): the key bits assumed
  // constant from an earlier call's range; out[0] = 1 if this call's keys vary in any of them
  // (the sort is then wrong and the caller re-bins), out[1] = the bits that vary.
  uint32_t assume = 0;
  int32_t *out = nullptr;
};
__device__ __forceinline__ bool digit_constant(const uint32_t *fin, int shift, int width) {
  return fin && ((((fin[0] ^ fin[1]) >> shift) & ((1u << width) - 1u)) == 0u);
}

// Device-selected ping-pong of the compacting depth sort (KeyRange on): a pass whose digit is
// constant over the kept keys does nothing at all -- its three launches return at once, no copy
// -- so where the data sits before pass q and whether pass q is the last one that moves it
// depend on the key range, which only the device knows.  Pass 0 (the compaction) always moves
// the data: from (ka, va) into (kb, vb), or straight into the output when no later digit varies;
// every later moving pass flips between the two buffers, the last one writes the output.
struct DevIO {
  const uint32_t *fin;       // the key range (AND, OR); null: host-selected buffers
  const void *ka, *kb;       // key ping-pong buffers
  const uint32_t *va, *vb;   // value ping-pong buffers
  void *kout;                // sorted keys (may be null)
  uint32_t *vout;            // sorted values
  int begin, width, passes;
};
__device__ __forceinline__ bool pass_moves(const DevIO &io, int q) {
  return q == 0 || !digit_constant(io.fin, io.begin + q * io.width, io.width);
}
// (ka, va) or (kb, vb): the buffers holding the data before pass q >= 1
__device__ __forceinline__ bool data_in_b(const DevIO &io, int q) {
  int m = 0;
  for (int j = 1; j < q; ++j) m += pass_moves(io, j) ? 1 : 0;
  return (m & 1) == 0;
}
__device__ __forceinline__ bool last_move(const DevIO &io, int q) {
  for (int j = q + 1; j < io.passes; ++j)
    if (pass_moves(io, j)) return false;
  return true;
}
template <typename K>
__device__ __forceinline__ void dev_io(const DevIO &io, int q, const K *&kin, const uint32_t *&vin,
                                       K *&kout, uint32_t *&vout) {
  const bool src_b = q > 0 && data_in_b(io, q);  // pass 0 reads (ka, va)
  kin = (const K *)(src_b ? io.kb : io.ka);
  vin = src_b ? io.vb : io.va;
  if (last_move(io, q)) {
    kout = (K *)io.kout;
    vout = io.vout;
  } else {  // the other buffer
    kout = (K *)(src_b ? io.ka : io.kb);
    vout = (uint32_t *)(src_b ? io.va : io.vb);
  }
}

// The sort tile of workgroup b among G: workgroups are dealt round-robin to the 8 XCDs
// (b % 8), so tile = b makes neighbouring tiles -- whose digit runs share output lines, and
// whose counts share count-matrix lines -- write from different XCDs' L2s.  Each XCD instead
// takes a contiguous range of tiles, in its dispatch order (a bijection on [0, G)): headline
// 1,625 -> 1,650 Mpix/s, c4 1,153 -> 1,161 (profiles/r06_sort_xcd_ab.txt; -DGS_SORT_NO_XCD: the
// round-robin order, for A/B builds).
__device__ __forceinline__ uint32_t sort_tile(uint32_t b, uint32_t G) {
#ifdef GS_SORT_NO_XCD
  (void)G;
  return b;
#else
  const uint32_t x = b & 7u, k = b >> 3, q = G >> 3, r = G & 7u;
  return x * q + min(x, r) + k;
#endif
}

// Reduce-then-scan pass, part 1: the digit histogram of every tile of TPB*ITEMS keys, stored
// digit-major (counts[d * nblocks + tile]) so one exclusive scan yields every tile's global
// offset for every digit.  drop: all-ones keys (culled Gaussians' depth keys) are not counted
// -- the pass drops them (compacting sort); n_dev: the key count is min(n, *n_dev) (the
// compacted length, known on the device only).
template <typename K, int ITEMS>
__global__ __launch_bounds__(TPB) void rts_count_kernel(const K *__restrict__ keys, long long n,
                                                        int shift, int width, long long nblocks,
                                                        uint32_t *__restrict__ counts,
                                                        bool drop = false,
                                                        const uint32_t *__restrict__ n_dev = nullptr,
                                                        KeyRange kr = {}, int pass = 0,
                                                        DevIO io = {}) {
  __shared__ uint32_t h[256];
  __shared__ uint32_t kand, kor;
  const int tid = threadIdx.x;
  if (pass > 0 && digit_constant(kr.fin, shift, width)) return;  // identity pass
  if (io.fin && pass > 0) keys = (const K *)(data_in_b(io, pass) ? io.kb : io.ka);
  const uint32_t tile = sort_tile(blockIdx.x, gridDim.x);
  const long long base = (long long)tile * TPB * ITEMS;
  K k[ITEMS];
  // (the compacted length; above the launch length n: an overflowed capacity launch, which
  // sorts nothing)
  if (n_dev) n = (long long)*n_dev > n ? 0 : (long long)*n_dev;
  const int R = 1 << width;
  const uint32_t dmask = (uint32_t)(R - 1);
  h[tid] = 0;
  if (tid == 0) kand = ~0u, kor = 0u;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const long long i = base + r * TPB + tid;
    k[r] = i < n ? keys[i] : (K)0;
  }
  uint32_t a = ~0u, o = 0u;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r)
    if (base + r * TPB + tid < n && !(drop && k[r] == (K)~(K)0)) {
      atomicAdd(&h[(uint32_t)(k[r] >> shift) & dmask], 1u);
      a &= (uint32_t)k[r];
      o |= (uint32_t)k[r];
    }
  if (pass == 0 && kr.blk) {  // one LDS atomic per wave
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      a &= __shfl_xor(a, off, 64);
      o |= __shfl_xor(o, off, 64);
    }
    if ((tid & 63) == 0) {
      atomicAnd(&kand, a);
      atomicOr(&kor, o);
    }
  }
  __syncthreads();
  if (tid < R) counts[(size_t)tid * nblocks + tile] = h[tid];
  if (pass == 0 && kr.blk && tid == 0) {
    kr.blk[2 * tile] = kand;
    kr.blk[2 * tile + 1] = kor;
  }
}

// Reduce-then-scan pass, part 2: one workgroup per digit scans that digit's row of tile
// counts in place (exclusive) and writes the row total; the pass kernel turns the <= 256 row
// totals into digit bases itself.  (One launch instead of a three-kernel device scan.)
// tsrc: the counts come tile-major from there (tsrc[t * R + d], R = 1 << width: the tile sort's
// first pass as the emission accumulates it, EmitCounts) and the scanned rows go digit-major
// into counts -- the matrix lines each hold one tile's counts of 32 digits, so scanning them in
// place would have 32 workgroups writing words of every line (0.010 vs 0.005 ms at the
// headline); read-only, those lines are shared from L2.
#ifndef GS_RS_NT  // (A/B builds)
#define GS_RS_NT 256
#endif
// row scan: 256 threads x 4 counts per chunk (1,024 x 1 slower by 3 us, 128 x 8 by 2-4 us,
// 64 x 16 by 4-6 us: profiles/r06_rowscan_ab.txt)
constexpr int RS_NT = GS_RS_NT, RS_PER = 1024 / RS_NT;
__global__ __launch_bounds__(RS_NT) void rts_rowscan_kernel(uint32_t *__restrict__ counts,
                                                            long long nblocks,
                                                            uint32_t *__restrict__ rowtot,
                                                            KeyRange kr = {}, int pass = 0,
                                                            int shift = 0, int width = 8,
                                                            const uint32_t *__restrict__ tsrc = nullptr) {
  __shared__ uint32_t lds[RS_NT / 64];
  __shared__ uint32_t kand, kor;
  if (pass > 0 && digit_constant(kr.fin, shift, width)) return;  // identity pass
  if (blockIdx.x == gridDim.x - 1 && pass == 0 && kr.blk) {
    // the extra last workgroup: the key range of the whole sort (off the rows' critical path)
    if (threadIdx.x == 0) kand = ~0u, kor = 0u;
    __syncthreads();
    uint32_t a = ~0u, o = 0u;
    for (long long i = threadIdx.x; i < kr.nblk; i += RS_NT) {
      a &= kr.blk[2 * i];
      o |= kr.blk[2 * i + 1];
    }
    atomicAnd(&kand, a);
    atomicOr(&kor, o);
    __syncthreads();
    if (threadIdx.x == 0) {
      kr.fin[0] = kand;
      kr.fin[1] = kor;
      if (kr.out) {
        kr.out[0] = ((kand ^ kor) & kr.assume) ? 1 : 0;
        kr.out[1] = (int32_t)(kand ^ kor);
      }
    }
    return;
  }
  // chunks of RS_NT x RS_PER counts, each thread RS_PER consecutive ones (all loads of a chunk
  // in flight together), a per-thread scan, then one block scan of the thread totals: a quarter
  // of the waves and barriers of one count per thread of a 1,024-thread workgroup
  uint32_t *row = counts + (size_t)blockIdx.x * nblocks;
  const size_t R = (size_t)1 << width;
  uint32_t running = 0;
  for (long long c0 = 0; c0 < nblocks; c0 += RS_NT * RS_PER) {
    const long long i0 = c0 + (long long)threadIdx.x * RS_PER;
    uint32_t v[RS_PER];
#pragma unroll
    for (int u = 0; u < RS_PER; ++u) {
      const long long i = i0 + u;
      v[u] = i < nblocks ? (tsrc ? tsrc[(size_t)i * R + blockIdx.x] : row[i]) : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int u = 0; u < RS_PER; ++u) {
      const uint32_t x = v[u];
      v[u] = s;
      s += x;
    }
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan<RS_NT>(s, tot, lds);
#pragma unroll
    for (int u = 0; u < RS_PER; ++u)
      if (i0 + u < nblocks) row[i0 + u] = running + ex + v[u];
    running += tot;
  }
  if (threadIdx.x == 0) rowtot[blockIdx.x] = running;
}

template <typename K, int ITEMS>
struct OsSmem {
  // the tile's (key, value) pairs in digit order: 32-bit keys interleaved with their values (one
  // 8-B LDS access per pair) in the small tiles, two arrays otherwise (16 keys per thread: the
  // pairs' extra registers would spill)
  static constexpr bool PAIR = sizeof(K) == 4 && ITEMS <= 8;
  static constexpr int N = TPB * ITEMS;
  __attribute__((aligned(16))) uint32_t raw[PAIR ? 2 * N : N * (sizeof(K) / 4 + 1)];
  uint32_t wcnt[4][256];   // per-wave digit counters, then per-wave digit offsets in the tile
  uint32_t gofs[256];      // global output offset of each digit, minus its tile offset
  uint32_t hscan[256];     // exclusive scan of this pass's digit totals (large tiles)
  uint32_t scan_tmp[4];
  uint32_t tile_n;         // keys this tile writes (all valid ones; fewer when dropping)
  __device__ __forceinline__ void put(uint32_t i, K k, uint32_t v) {
    if constexpr (PAIR) {
      reinterpret_cast<uint2 *>(raw)[i] = make_uint2((uint32_t)k, v);
    } else {
      reinterpret_cast<K *>(raw)[i] = k;
      raw[N * (sizeof(K) / 4) + i] = v;
    }
  }
  __device__ __forceinline__ void get(uint32_t i, K &k, uint32_t &v) const {
    if constexpr (PAIR) {
      const uint2 e = reinterpret_cast<const uint2 *>(raw)[i];
      k = (K)e.x;
      v = e.y;
    } else {
      k = reinterpret_cast<const K *>(raw)[i];
      v = raw[N * (sizeof(K) / 4) + i];
    }
  }
  __device__ __forceinline__ K key(uint32_t i) const {
    if constexpr (PAIR) return (K)raw[2 * i];
    else return reinterpret_cast<const K *>(raw)[i];
  }
};

// Inclusive max-scan over the wave (DPP row shifts, then the row broadcasts; no LDS).
__device__ __forceinline__ int wave_incl_max(int v) {
  constexpr int NONE = -2147483647 - 1;
  v = max(v, __builtin_amdgcn_update_dpp(NONE, v, 0x111, 0xF, 0xF, false));  // row_shr:1
  v = max(v, __builtin_amdgcn_update_dpp(NONE, v, 0x112, 0xF, 0xF, false));  // row_shr:2
  v = max(v, __builtin_amdgcn_update_dpp(NONE, v, 0x114, 0xF, 0xF, false));  // row_shr:4
  v = max(v, __builtin_amdgcn_update_dpp(NONE, v, 0x118, 0xF, 0xF, false));  // row_shr:8
  v = max(v, __builtin_amdgcn_update_dpp(NONE, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = max(v, __builtin_amdgcn_update_dpp(NONE, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}

// The tile sort's first pass generated instead of loaded (GenSrc; intersection counts from
// 2^24, where the emitted pair array would not stay in the 256 MB MALL and writing it and
// reading it back costs more than generating each slot twice): slot s of the depth-ordered
// intersection list belongs to the last depth position p with start[p] <= s (start = the
// exclusive scan of the allotments; a zero allotment shares its start with the next position,
// so the last such p always owns s), and its tile is the (s - start[p])-th of p's box in gsplat's
// row order (the sentinel T past the box, as the emission).  seg[k] = the owner of slot 64 k,
// so a wave finds a round's owners from a window of the 64 positions from seg[k] on.
struct GenSrc {
  const uint32_t *start, *cnt, *order, *seg;
  const uint2 *box;
  int tbx, tby;
  long long n;  // depth positions
};
// Slots s0 + 64 u + lane (u < G; s0 a multiple of 64) of the list of n_slots -> (tile, id);
// every lane of the wave calls it (wave-uniform s0).  The G rounds' loads are issued together,
// level by level (owners' windows, window starts, then the owners' boxes and ids), so a wave
// waits for three load latencies per G rounds instead of per round.  mk: the wave's G x 64 LDS
// ints.
constexpr int GEN_G = 16;
template <int G>
__device__ __forceinline__ void gen_rounds(const GenSrc &g, long long s0, long long n_slots,
                                           int *mk, uint32_t (&key)[G], uint32_t (&val)[G]) {
  const int lane = threadIdx.x & 63;
  const uint32_t T = (uint32_t)(g.tbx * g.tby);
  long long pa[G];
  uint32_t st[G];
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const long long su = s0 + 64 * u;
    pa[u] = su < n_slots ? (long long)g.seg[su >> 6] : 0;
  }
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const long long p = pa[u] + lane;
    st[u] = (s0 + 64 * u < n_slots && p < g.n) ? g.start[p] : 0xFFFFFFFFu;
  }
  // owner = the last window lane q with start[q] <= s: lane 0 owns the round's first slot; a
  // later lane starting inside the round marks its first slot (several with one start: the
  // last of them wins)
  wave_lds_sync();
#pragma unroll
  for (int u = 0; u < G; ++u) mk[u * 64 + lane] = 0;
  wave_lds_sync();
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const uint64_t su = (uint64_t)(s0 + 64 * u);
    if (lane > 0 && (uint64_t)st[u] < su + 64u) atomicMax(&mk[u * 64 + (int)(st[u] - (uint32_t)su)], lane);
  }
  wave_lds_sync();
  long long own[G];
  uint32_t ost[G];
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const long long s = s0 + 64 * u + lane;
    const int q = wave_incl_max(mk[u * 64 + lane]);
    const uint32_t sq = __shfl(st[u], q, 64);
    const uint32_t st63 = __shfl(st[u], 63, 64);
    own[u] = pa[u] + q;
    ost[u] = sq;
    // past the window (only with zero allotments in it): the owner by binary search
    if (q == 63 && s < n_slots && st63 != 0xFFFFFFFFu &&
        (uint64_t)s >= (uint64_t)st63 + (uint64_t)g.cnt[min(pa[u] + 63, g.n - 1)]) {
      long long lo = pa[u] + 63, hi = g.n - 1;  // start[lo] <= s; the last such position
      while (lo < hi) {
        const long long mid = (lo + hi + 1) >> 1;
        if ((uint64_t)g.start[mid] <= (uint64_t)s) lo = mid;
        else hi = mid - 1;
      }
      own[u] = lo;
      ost[u] = g.start[lo];
    }
  }
  uint2 bx[G];
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const bool valid = s0 + 64 * u + lane < n_slots;
    bx[u] = valid ? g.box[own[u]] : make_uint2(0u, 0u);
    val[u] = valid ? g.order[own[u]] : 0u;
  }
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const uint32_t li = (uint32_t)(s0 + 64 * u + lane) - ost[u];
    const int qx0 = (int)(bx[u].x & 0xFFFFu), qy0 = (int)(bx[u].x >> 16);
    const int qx1 = (int)(bx[u].y & 0xFFFFu), qy1 = (int)(bx[u].y >> 16);
    const int qbw = max(qx1 - qx0, 1);
    const int qarea = max(qx1 - qx0, 0) * max(qy1 - qy0, 0);
    key[u] = T;
    if ((int)li < qarea) {  // li / qbw as in the emission (exact below 2^20)
      const int ly = li < (1u << 20)
                         ? (int)(((float)li + 0.5f) * __builtin_amdgcn_rcpf((float)qbw))
                         : (int)li / qbw;
      key[u] = (uint32_t)((qy0 + ly) * g.tbx + qx0 + ((int)li - ly * qbw));
    }
  }
}

// The generated first pass's digit counts (rts_count_kernel's layout): one workgroup per sort
// tile of TPB * ITEMS slots, each wave its ITEMS rounds.
template <int ITEMS>
__global__ __launch_bounds__(TPB) void gen_count_kernel(GenSrc g, long long cap,
                                                        const uint32_t *__restrict__ n_dev,
                                                        int width, long long nblocks,
                                                        uint32_t *__restrict__ counts) {
  __shared__ uint32_t h[256];
  __shared__ int marks[TPB * GEN_G];
  const int tid = threadIdx.x, wave = tid >> 6;
  long long n = cap;
  if (n_dev) n = (long long)*n_dev > cap ? 0 : (long long)*n_dev;
  const int R = 1 << width;
  h[tid] = 0;
  __syncthreads();
  const uint32_t tile = sort_tile(blockIdx.x, gridDim.x);
  const long long sg = (long long)tile * TPB * ITEMS + (long long)wave * (ITEMS * 64);
  constexpr int GG = ITEMS < GEN_G ? ITEMS : GEN_G;
  static_assert(ITEMS % GG == 0, "rounds in groups of GG");
  for (int r = 0; r < ITEMS; r += GG) {
    if (sg + r * 64 >= n) break;  // wave-uniform
    uint32_t k[GG], v[GG];
    gen_rounds<GG>(g, sg + r * 64, n, marks + wave * 64 * GG, k, v);
#pragma unroll
    for (int u = 0; u < GG; ++u)
      if (sg + (r + u) * 64 + (tid & 63) < n) atomicAdd(&h[k[u] & (uint32_t)(R - 1)], 1u);
  }
  __syncthreads();
  if (tid < R) counts[(size_t)tid * nblocks + tile] = h[tid];
}

// Reduce-then-scan pass, part 3: each workgroup ranks its tile of TPB * ITEMS keys stably in
// LDS, takes its digits' global offsets from the row-scanned tile counts plus the digit bases
// (the exclusive scan of the row totals), and writes the tile out in digit order, so each
// digit's run is written by consecutive lanes.
template <typename K, int WIDTH, int ITEMS, bool GEN = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(4, 8))) void os_pass_kernel(
    const K *__restrict__ kin, const uint32_t *__restrict__ vin, K *__restrict__ kout,
    uint32_t *__restrict__ vout, long long n, int shift, int width,
    const uint32_t *__restrict__ rowtot, const uint32_t *__restrict__ offs, long long nblocks,
    bool drop = false, const uint32_t *__restrict__ n_dev = nullptr,
    uint32_t *__restrict__ n_out = nullptr, const uint32_t *__restrict__ kfin = nullptr,
    DevIO io = {}, int q = 0, int *__restrict__ tbins = nullptr, uint32_t tcount = 0,
    GenSrc gen = {}) {
  if (io.fin) {  // device-selected buffers (DevIO): a constant digit moves nothing
    if (q > 0 && digit_constant(io.fin, shift, width)) return;
    const K *ki;
    const uint32_t *vi;
    K *ko;
    uint32_t *vo;
    dev_io<K>(io, q, ki, vi, ko, vo);
    kin = ki;
    vin = vi;
    kout = ko;
    vout = vo;
  }
  // compacting sort: with drop, all-ones keys are left out (pass 0 of the depth sort: culled
  // Gaussians), and block 0 stores the kept count to n_out; later passes sort min(n, *n_dev)
  // keys and the workgroups past them exit at once.
  if (n_dev) {
    n = (long long)*n_dev > n ? 0 : (long long)*n_dev;  // (see rts_count_kernel)
    if ((long long)sort_tile(blockIdx.x, gridDim.x) * TPB * ITEMS >= n) return;  // whole workgroup
  }
  if (digit_constant(kfin, shift, width)) {  // every key has the same digit: a stable copy
    const long long b0 = (long long)sort_tile(blockIdx.x, gridDim.x) * TPB * ITEMS;
    K ck[ITEMS];
    uint32_t cv[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {  // all loads in flight before the first store
      const long long i = min(b0 + r * TPB + threadIdx.x, n - 1);
      if (kout) ck[r] = kin[i];
      cv[r] = vin[i];
    }
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const long long i = b0 + r * TPB + threadIdx.x;
      if (i < n) {
        if (kout) kout[i] = ck[r];
        vout[i] = cv[r];
      }
    }
    return;
  }
  __shared__ OsSmem<K, ITEMS> sm;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int R = 1 << width;
  const uint32_t dmask = (uint32_t)(R - 1);
  const uint32_t t = sort_tile(blockIdx.x, gridDim.x);
  const unsigned long long lt = (1ull << lane) - 1ull;
  K key[ITEMS];
  uint32_t val[ITEMS], rank[ITEMS];
  bool ok[ITEMS];
  // the digit total (and in small tiles this tile's row offset) first: vmcnt retires in issue
  // order, so the scans below wait for them alone
  constexpr bool SMALL = ITEMS <= 8;
  const uint32_t hval = rowtot[min(tid, R - 1)];
  const uint32_t oval = SMALL ? offs[(size_t)min(tid, R - 1) * nblocks + t] : 0u;
  if constexpr (GEN) {  // the generated first pass of the tile sort (gen_rounds)
    // (the marks live in the tile's pair buffer, which is written only after the barriers of
    // the digit-base scan below)
    int *gmarks = reinterpret_cast<int *>(sm.raw);
    constexpr int GG = ITEMS < GEN_G ? ITEMS : GEN_G;
    static_assert(sizeof(sm.raw) >= sizeof(int) * TPB * GG, "marks fit the pair buffer");
    const long long sg = (long long)t * TPB * ITEMS + (long long)wave * (ITEMS * 64);
#pragma unroll
    for (int r = 0; r < ITEMS; r += GG) {
      uint32_t k[GG], v[GG];
      gen_rounds<GG>(gen, sg + r * 64, n, gmarks + wave * 64 * GG, k, v);
#pragma unroll
      for (int u = 0; u < GG; ++u) {
        key[r + u] = (K)k[u];
        val[r + u] = v[u];
      }
    }
  } else {  // (indices clamped into [0, n): no per-element branch, so all 2 x ITEMS loads are
            // in flight together; the validity mask is applied once they are consumed)
    const long long sg = (long long)t * TPB * ITEMS + (long long)wave * (ITEMS * 64);
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const long long i = min(sg + r * 64 + lane, n - 1);
      key[r] = kin[i];
      val[r] = vin[i];
    }
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) sm.wcnt[w][tid] = 0;
  uint32_t hs;  // digit base: exclusive scan of the digit row totals (thread tid: digit tid)
  {
    uint32_t h = tid < R ? hval : 0u, tot;
    hs = block_exclusive_scan<TPB>(h, tot, sm.scan_tmp);  // contains barriers
    if (!SMALL) sm.hscan[tid] = hs;  // (registers are tight with 16 keys per thread)
    if (n_out && blockIdx.x == 0 && tid == 0) *n_out = tot;
  }
  const long long base = (long long)t * TPB * ITEMS;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const bool valid = base + (long long)wave * (ITEMS * 64) + r * 64 + lane < n;
    ok[r] = valid && !(drop && key[r] == (K)~(K)0);
  }
  // Stable rank within the wave: a ballot match finds the lanes sharing this key's digit
  // (peers); the group's lowest lane reserves popc(peers) slots of the wave's LDS counter for
  // that digit with ONE returning LDS atomic and the others read the old value from it
  // (a wave's LDS atomics execute in issue order, so the rounds stay ordered).
  // In groups of four rounds, three sweeps each so the LDS round trips overlap: the matches,
  // then the counter atomics (in round order), then the reads of the leaders' old values.
  constexpr int GRP = ITEMS < 4 ? ITEMS : 4;
#pragma unroll
  for (int r0 = 0; r0 < ITEMS; r0 += GRP) {
    unsigned long long pr[GRP];
    uint32_t old[GRP];
#pragma unroll
    for (int u = 0; u < GRP; ++u)
      pr[u] = digit_peers<WIDTH>((uint32_t)(key[r0 + u] >> shift) & dmask, WIDTH, ok[r0 + u]);
#pragma unroll
    for (int u = 0; u < GRP; ++u) {
      old[u] = 0u;
      if (ok[r0 + u] && (int)__builtin_ctzll(pr[u]) == lane)
        old[u] = atomicAdd(&sm.wcnt[wave][(uint32_t)(key[r0 + u] >> shift) & dmask],
                           (uint32_t)__popcll(pr[u]));
    }
#pragma unroll
    for (int u = 0; u < GRP; ++u) {
      const int leader = ok[r0 + u] ? (int)__builtin_ctzll(pr[u]) : lane;
      rank[r0 + u] = __shfl(old[u], leader, 64) + (uint32_t)__popcll(pr[u] & lt);
    }
  }
  __syncthreads();
  {
    // digit tid's column: the waves' exclusive prefix, then the tile's exclusive digit offset
    // added in place, so a key's tile position is wcnt[wave][digit] + its rank (one LDS read)
    uint32_t cw[4], s = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      cw[w] = s;
      s += sm.wcnt[w][tid];
    }
    uint32_t tot;
    const uint32_t lo = block_exclusive_scan<TPB>(s, tot, sm.scan_tmp);  // (barriers)
#pragma unroll
    for (int w = 0; w < 4; ++w) sm.wcnt[w][tid] = lo + cw[w];
    if (SMALL && tid < R) sm.gofs[tid] = hs + oval - lo;
    if (tid == 0) sm.tile_n = tot;
    __syncthreads();  // every column is read below
    // stable local sort into LDS
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      if (ok[r]) {
        const uint32_t d = (uint32_t)(key[r] >> shift) & dmask;
        sm.put(sm.wcnt[wave][d] + rank[r], key[r], val[r]);
      }
    }
    // large tiles: the row offset's load overlaps the scatter
    if (!SMALL && tid < R)
      sm.gofs[tid] = sm.hscan[tid] + offs[(size_t)tid * nblocks + t] - lo;
  }
  __syncthreads();
  const long long cnt = sm.tile_n;
  {
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const int i = r * TPB + tid;
      if (i < cnt) {
        K k;
        uint32_t v;
        sm.get(i, k, v);
        const uint32_t pos = sm.gofs[(uint32_t)(k >> shift) & dmask] + (uint32_t)i;
        if (kout) kout[pos] = k;  // null: only the values are wanted (compacted depth sort)
        vout[pos] = v;
        // the tile sort's last pass (tbins): the tile table from this tile's runs of equal keys
        // (equal keys sit at consecutive positions): a run's first position -> max(n - pos),
        // its end -> max(pos + 1); over all runs of a tile, the list's first and end
        // (ts_decode_kernel turns n - first back); keys >= tcount (the sentinel) have no row
        if (tbins && (uint32_t)k < tcount) {
          if (i == 0 || sm.key(i - 1) != k) atomicMax(&tbins[2 * (uint32_t)k], (int)(n - pos));
          if (i + 1 == cnt || sm.key(i + 1) != k) atomicMax(&tbins[2 * (uint32_t)k + 1], (int)(pos + 1));
        }
      }
    }
  }
}

// Constant-digit depth passes (gsplat_debug_depth_key_range: 0 off, 1 from 2^22 keys, 2 always,
// the default).  Round 3 copied the data in such a pass (~8 us of range bookkeeping and copy
// against a skipped ranking: a loss below 2^22 keys); with the device-selected buffers (DevIO)
// a constant digit costs its three launches returning at once, and the AND / OR is reduced
// per wave before its LDS atomics.  The headline's visible depths (2.5-5.5) share their top
// byte, so one of its four passes drops out.
int g_key_range = 2;
bool use_key_range(long long n) { return g_key_range == 2 || (g_key_range == 1 && n >= (1LL << 22)); }

uint32_t *rts_tile_counts(void *ws) { return (uint32_t *)ws + OS_HEAD_WORDS; }
// the compacting sort's kept-key count (a head word)
uint32_t *sort_kept_word(void *ws) { return (uint32_t *)ws + 1; }

// Stable LSD sort of (keys, vals) by bits [begin_bit, end_bit).  Ping-pongs between
// (ka, va) and (kb, vb); the last pass writes (kout, vout).  (ka, va) are clobbered when
// there are more than two passes.  ws must hold radix_ws_bytes(n, begin_bit, end_bit).
// first_counts_ready: the caller's key kernel already wrote pass 0's tile digit counts to
// rts_tile_counts(ws).
// drop (first_counts_ready then means counts without the all-ones keys): the first pass leaves
// out all-ones keys, so the sort orders only the kept keys, whose count it stores to
// sort_kept_word(ws) (the sorted output holds that many; kout may be null).
// assume_const / range_out (drop only): gsplat_bin_count_keyed_ex's depth-key range.
// n_dev_all (no drop): the key count on the device, n the launch length (a capacity): every pass
// sorts *n_dev_all keys, none when it exceeds n.  tbins (the tile sort, no KeyRange): the last
// pass also accumulates the tile table of keys < tcount (os_pass_kernel; ts_decode_kernel).
// first_tsrc (with first_counts_ready): pass 0's counts are tile-major there (the emission's,
// EmitCounts, in the kb buffer the pass writes later) -- its row scan reads them from there.
template <typename K>
int radix_sort_pairs(K *ka, uint32_t *va, K *kb, uint32_t *vb, K *kout, uint32_t *vout,
                     long long n, int begin_bit, int end_bit, void *ws, hipStream_t st,
                     bool first_counts_ready = false, bool drop = false,
                     uint32_t assume_const = 0, int32_t *range_out = nullptr,
                     const uint32_t *n_dev_all = nullptr, int *tbins = nullptr,
                     uint32_t tcount = 0, const GenSrc *gen = nullptr,
                     const uint32_t *first_tsrc = nullptr) {
  if (n <= 0) return 0;
  const SortPlan p = sort_plan(n, begin_bit, end_bit);
  if (p.passes == 0) {
    note(hipMemcpyAsync(kout, ka, n * sizeof(K), hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
    note(hipMemcpyAsync(vout, va, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st),
         "hipMemcpyAsync");
    return 0;
  }
  uint32_t *counts = rts_tile_counts(ws);                      // tile digit counts
  uint32_t *rowtot = counts + (size_t)p.nblocks * p.radix;     // their row totals
  uint32_t *kept = sort_kept_word(ws);
  KeyRange kr;
  if (drop && use_key_range(n)) {
    kr.blk = (uint32_t *)((char *)ws + radix_main_bytes(p));
    kr.fin = sort_kept_word(ws) + 1;
    kr.nblk = p.nblocks;
    kr.assume = assume_const;
    kr.out = range_out;
  }
  K *kin = ka, *kalt = kb;
  uint32_t *vin = va, *valt = vb;
  // with the key range, the device picks every pass's buffers (DevIO) and constant digits move
  // nothing (no copy)
  DevIO io{};
  if (kr.fin) io = DevIO{kr.fin, ka, kb, va, vb, kout, vout, begin_bit, p.width, p.passes};
  for (int q = 0; q < p.passes; ++q) {
    // a digit the caller's earlier range says is constant: not launched at all (its three
    // launches cost ~14 us at the headline even when they return at once); the pass-0 range
    // reduction checks the assumption (kr.out)
    const uint32_t qmask = (p.width >= 32 ? ~0u : ((1u << p.width) - 1u)) << (begin_bit + q * p.width);
    if (q > 0 && kr.fin && kr.out && (kr.assume & qmask) == qmask) continue;
    const bool last = q == p.passes - 1;
    K *ko = last ? kout : kalt;
    uint32_t *vo = last ? vout : valt;
    // tile digit counts -> row scans -> offsets
    const int sh = begin_bit + q * p.width;
    const uint32_t *ndev = drop ? (q > 0 ? kept : nullptr) : n_dev_all;
    // first_counts_ready: the key kernel wrote pass 0's counts and key ranges (kr.blk)
    if (q == 0 && gen) {
      if (p.items == 16)
        hipLaunchKernelGGL(gen_count_kernel<16>, dim3((unsigned)p.nblocks), dim3(TPB), 0, st, *gen,
                           n, ndev, p.width, p.nblocks, counts);
      else
        hipLaunchKernelGGL(gen_count_kernel<4>, dim3((unsigned)p.nblocks), dim3(TPB), 0, st, *gen,
                           n, ndev, p.width, p.nblocks, counts);
    } else if (q == 0 && first_counts_ready) {
    } else if (p.items == 16)
      hipLaunchKernelGGL((rts_count_kernel<K, 16>), dim3((unsigned)p.nblocks), dim3(TPB), 0, st,
                         kin, n, sh, p.width, p.nblocks, counts, drop && q == 0, ndev, kr, q, io);
    else if (p.items == 8)
      hipLaunchKernelGGL((rts_count_kernel<K, 8>), dim3((unsigned)p.nblocks), dim3(TPB), 0, st,
                         kin, n, sh, p.width, p.nblocks, counts, drop && q == 0, ndev, kr, q, io);
    else
      hipLaunchKernelGGL((rts_count_kernel<K, 4>), dim3((unsigned)p.nblocks), dim3(TPB), 0, st,
                         kin, n, sh, p.width, p.nblocks, counts, drop && q == 0, ndev, kr, q, io);
    hipLaunchKernelGGL(rts_rowscan_kernel,
                       dim3((unsigned)p.radix + (q == 0 && kr.blk ? 1u : 0u)), dim3(RS_NT), 0,
                       st, counts, p.nblocks, rowtot, kr, q, sh, p.width,
                       q == 0 ? first_tsrc : nullptr);
#define OS_PASS(Wd, It)                                                                     \
  do {                                                                                      \
    if (q == 0 && gen)                                                                      \
      hipLaunchKernelGGL((os_pass_kernel<K, Wd, It, true>), dim3((unsigned)p.nblocks),      \
                         dim3(TPB), 0, st, kin, vin, ko, vo, n, sh, p.width, rowtot, counts, \
                         p.nblocks, false, ndev, nullptr, nullptr, io, q,                   \
                         last ? tbins : nullptr, tcount, *gen);                             \
    else                                                                                    \
      hipLaunchKernelGGL((os_pass_kernel<K, Wd, It>), dim3((unsigned)p.nblocks), dim3(TPB), \
                         0, st, kin, vin, ko, vo, n, sh, p.width, rowtot, counts, p.nblocks, \
                         drop && q == 0, ndev, drop && q == 0 ? kept : nullptr,            \
                         q > 0 && !io.fin ? kr.fin : nullptr, io, q,                        \
                         last ? tbins : nullptr, tcount, GenSrc{});                         \
  } while (0)
#define OS_PASS_W(Wd)                                                                       \
  do {                                                                                      \
    if (p.items == 16) OS_PASS(Wd, 16);                                                     \
    else if (p.items == 8) { if constexpr (Wd == 8) OS_PASS(Wd, 8); }                       \
    else OS_PASS(Wd, 4);                                                                    \
  } while (0)
    switch (p.width) {
      case 1: OS_PASS_W(1); break;
      case 2: OS_PASS_W(2); break;
      case 3: OS_PASS_W(3); break;
      case 4: OS_PASS_W(4); break;
      case 5: OS_PASS_W(5); break;
      case 6: OS_PASS_W(6); break;
      case 7: OS_PASS_W(7); break;
      default: OS_PASS_W(8); break;
    }
#undef OS_PASS_W
#undef OS_PASS
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
// 0xFFFFFFFF (sorted last).  Also writes the Gaussian's binning record, read by coalesced
// loads here so that the depth-ordered passes need ONE gather per Gaussian:
// rec[g] = {tile allotment, x0 | y0 << 16, x1 | y1 << 16, 0} (tile bbox; < 65536 tiles per axis).
// One workgroup per depth-sort tile (TPB * ITEMS keys): with counts != null it also writes the
// tile's histogram of the first sort digit over the visible keys (reduce-then-scan pass 0 of
// the compacting depth sort), saving the sort its first count launch.
template <int ITEMS>
__global__ __launch_bounds__(TPB) void depth_keys_kernel(int n, const float *__restrict__ xys,
                                                         const float *__restrict__ depths,
                                                         const int *__restrict__ radii,
                                                         const int *__restrict__ num_tiles_hit,
                                                         int tbx, int tby,
                                                         uint32_t *__restrict__ keys,
                                                         uint32_t *__restrict__ vals,
                                                         uint4 *__restrict__ rec,
                                                         uint32_t *__restrict__ counts,
                                                         long long nblocks,
                                                         uint32_t *__restrict__ kblk = nullptr) {
  __shared__ uint32_t h[256];
  __shared__ uint32_t kand, kor;
  const int tid = threadIdx.x;
  if (counts) {
    h[tid] = 0;
    if (tid == 0) kand = ~0u, kor = 0u;
    __syncthreads();
  }
  uint32_t ka = ~0u, ko = 0u;  // the visible keys' AND / OR (KeyRange)
  const long long base = (long long)blockIdx.x * TPB * ITEMS;
  // every input of the tile loaded up front (clamped indices, no per-item branch): the loads
  // are in flight together instead of one wait per Gaussian
  int rr[ITEMS], cc[ITEMS];
  float dd[ITEMS];
  float2 xy[ITEMS];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const long long i = min(base + k * TPB + tid, (long long)n - 1);
    rr[k] = radii[i];
    dd[k] = depths[i];
    cc[k] = num_tiles_hit[i];
    xy[k] = reinterpret_cast<const float2 *>(xys)[i];
  }
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const long long i = base + k * TPB + tid;
    if (i >= n) break;
    const int r = rr[k];
    const bool vis = r > 0;
    const uint32_t key = vis ? __float_as_uint(dd[k]) : 0xFFFFFFFFu;
    keys[i] = key;
    vals[i] = (uint32_t)i;
    if (counts && vis) {  // the compacting sort drops culled keys
      atomicAdd(&h[key & 0xFFu], 1u);
      ka &= key;
      ko |= key;
    }
    const int c = vis ? cc[k] : 0;
    uint4 q = {c > 0 ? (uint32_t)c : 0u, 0u, 0u, 0u};
    if (c > 0) {
      int x0, x1, y0, y1;
      tile_bbox(xy[k].x, xy[k].y, (float)r, tbx, tby, x0, x1, y0, y1);
      q.y = (uint32_t)x0 | ((uint32_t)y0 << 16);
      q.z = (uint32_t)x1 | ((uint32_t)y1 << 16);
    }
    rec[i] = q;
  }
  if (counts) {
    if (kblk) {
      atomicAnd(&kand, ka);
      atomicOr(&kor, ko);
    }
    __syncthreads();
    counts[(size_t)tid * nblocks + blockIdx.x] = h[tid];
    if (kblk && tid == 0) {
      kblk[2 * blockIdx.x] = kand;
      kblk[2 * blockIdx.x + 1] = kor;
    }
  }
}

// Depth-ordered allotments and boxes: cnt[p], box[p] from the p-th Gaussian's record (the
// one random gather of the binning).  kept = the compacting depth sort's kept-key count (the
// visible count): order holds only the visible Gaussians and the positions past them get zero
// allotments.  One workgroup per scan tile (SC_TILE entries): it also writes the tile's
// allotment sum, the first step of the device scan of cnt.
__global__ __launch_bounds__(TPB) void gather_counts_kernel(int n, const uint32_t *__restrict__ order,
                                                            const uint32_t *__restrict__ kept,
                                                            const uint4 *__restrict__ rec,
                                                            uint32_t *__restrict__ cnt,
                                                            uint2 *__restrict__ box,
                                                            int *__restrict__ num_visible,
                                                            uint32_t *__restrict__ partial,
                                                            uint32_t *__restrict__ vflag = nullptr,
                                                            uint32_t *__restrict__ zero = nullptr,
                                                            long long zero_words = 0) {
  __shared__ uint32_t lds[TPB / 64];
  // (zero: the emission's first-pass count matrix, EmitCounts -- cleared before the emission)
  for (long long i = (long long)blockIdx.x * TPB + threadIdx.x; zero && i < zero_words;
       i += (long long)gridDim.x * TPB)
    zero[i] = 0u;
  const long long base = (long long)blockIdx.x * SC_TILE;
  uint32_t sum = 0;
  const long long nv = min((long long)n, (long long)*kept);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *num_visible = (int)nv;
    if (vflag) *vflag = 0u;  // (set by scan_partials_kernel when it checks the key range)
  }
  if (base < nv) {  // workgroup-uniform
    // all ids, then all records, with clamped indices and no per-item branch, so each level
    // of the gather has its 16 loads in flight together
    uint32_t ord[SC_ITEMS];
    uint4 q[SC_ITEMS];
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k)
      ord[k] = order[min(base + k * TPB + threadIdx.x, nv - 1)];
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) q[k] = rec[min(ord[k], (uint32_t)n - 1u)];  // (see box_counts)
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) {
      const long long p = base + k * TPB + threadIdx.x;
      if (p < nv) {
        cnt[p] = q[k].x;
        box[p] = make_uint2(q[k].y, q[k].z);
        sum += q[k].x;
      } else if (p < n) {
        cnt[p] = 0u;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) {
      const long long p = base + k * TPB + threadIdx.x;
      if (p < n) cnt[p] = 0u;
    }
  }
  uint32_t total;
  block_exclusive_scan<TPB>(sum, total, lds);
  if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

// The owner of slot j0 + lane of a wave's combined slot range -- the last lane q with
// rel[q] <= j and an allotment (has) -- without a search: every owner starting in the 64-slot
// chunk marks its start offset with j0 + q (LDS max into the wave's 64 marks `mk`, set to -1
// once before the first chunk), and an inclusive max-scan over the chunk's slots, with the
// previous chunk's last owner as carry, gives every slot's owner.  Marks are never cleared: a
// stale mark from an earlier chunk encodes a smaller j0 + q than any owner it could shadow
// (owners start in lane order and their slot ranges do not overlap), so the max is still the
// owner.  (Replaces a 6-step shuffle search: six dependent ds_bpermute round trips per chunk.)
__device__ __forceinline__ int slot_owner(int *mk, uint32_t j0, uint32_t rel, bool has,
                                          int &carry) {
  const int lane = threadIdx.x & 63;
  wave_lds_sync();
  if (has && rel >= j0 && rel < j0 + 64u) atomicMax(&mk[rel - j0], (int)j0 + lane);
  wave_lds_sync();
  const int own = max(wave_incl_max(mk[lane]), carry);
  carry = __builtin_amdgcn_readlane(own, 63);
  return own & 63;
}

// ------------------------------------------------------------------ tile sort (shipped)
// The depth-ordered Gaussians -> gsplat's tile lists by emitting every intersection as a
// (tile, id) pair in depth order and sorting the pairs stably by tile:
//   ts_emit_kernel   one workgroup per 256 depth-ordered Gaussians: their intersection offsets
//                    (the per-1,024-block allotment sums of gather_counts_kernel plus a block
//                    scan -- no separate scan launches), then each wave fills its 64 Gaussians'
//                    combined slot range with lanes striding over it (slot owners from
//                    slot_owner), so the pair stores are coalesced; the tile table is cleared
//                    on the way; workgroup 0 publishes I.
//   radix_sort_pairs the stable LSD sort of the pairs by tile id (ceil(log2(T + 1)) bits: two
//                    passes up to 16,383 tiles), launched at the capacity with the device count
//                    as its length (n_dev_all): no host read of I before it.
//                    Its last pass writes only the ids and accumulates the tile table from
//                    its LDS-sorted runs of equal tile ids (atomicMax of n - first and of end);
//   ts_decode_kernel turns each row back into gsplat's (first, end) -- no sorted keys are
//                    written or re-read.
// Stable sort of depth-ordered pairs by tile = gsplat's order (ties by Gaussian id), bit for
// bit.  Against the region binning of round 5 (removed in round 6; measured on one box: the
// headline 0.22 vs 0.24 ms, c4 garden ~0.30 vs 0.39 ms, profiles/r05_region_binning_sweep.txt)
// the sort's passes are coalesced and balanced by construction, where the region binning's
// per-(depth range, region) workgroups were imbalanced on real scenes.
// partial[]: gather_counts_kernel's per-1,024-Gaussian block sums, scanned here by every
// workgroup (<= a few loads per thread); workgroup 0 publishes their total I to i_dev and
// i_host (the speculative binning; after a count phase that found I already, the same value).
// i_dev > cap (an overflow, or a depth-key digit the sort assumed constant that varied: i_dev =
// ~0): nothing is emitted.
// EmitCounts (the speculative binning, round 6): the tile sort's first digit counts come from
// the emission itself instead of a count launch over the emitted pairs.  A workgroup's slots
// are one contiguous range, so they fall in a few consecutive sort tiles (2^shift slots each):
// the first EC_LT of them are counted in an LDS histogram and added once per (tile, digit) at
// the end, the rest (a very large allotment) straight into the tile-major matrix
// counts[tile * 2^width + digit], which gather_counts_kernel zeroed.
constexpr int EC_LT = 4;
struct EmitCounts {
  uint32_t *counts = nullptr;  // null: the sort counts its first pass itself
  int shift = 0, width = 0;
  long long nblocks = 0;
};
__global__ __launch_bounds__(TPB) void ts_emit_kernel(int n, int nb,
                                                      const uint32_t *__restrict__ order,
                                                      const uint32_t *__restrict__ cnt,
                                                      const uint32_t *__restrict__ partial,
                                                      const uint2 *__restrict__ box, int tbx,
                                                      int tby, uint32_t *__restrict__ tkeys,
                                                      uint32_t *__restrict__ tvals,
                                                      int *__restrict__ tile_bins,
                                                      uint32_t *__restrict__ i_dev,
                                                      int32_t *__restrict__ i_host, uint32_t cap,
                                                      const uint32_t *__restrict__ kfin,
                                                      uint32_t assume,
                                                      uint32_t *__restrict__ gstart = nullptr,
                                                      uint32_t *__restrict__ gseg = nullptr,
                                                      const uint32_t *__restrict__ vflag = nullptr,
                                                      const uint32_t *__restrict__ pscan = nullptr,
                                                      const EmitCounts ec = {}) {
  __shared__ uint32_t lds[TPB / 64];
  __shared__ int marks[TPB];
  __shared__ uint32_t ech[EC_LT * 256];
  for (long long i = (long long)blockIdx.x * TPB + threadIdx.x; i < 2LL * tbx * tby;
       i += (long long)gridDim.x * TPB)
    tile_bins[i] = 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t ecr = 1u << ec.width;  // (the first pass's digits)
  if (ec.counts)
    for (int i = tid; i < EC_LT * (int)ecr; i += TPB) ech[i] = 0u;  // (barriers below)
  const int t = (int)(blockIdx.x / SC_ITEMS), rr = (int)(blockIdx.x % SC_ITEMS);
  const long long b0 = (long long)t * SC_TILE;
  const long long p = b0 + (long long)rr * TPB + tid;
  uint32_t cr[SC_ITEMS];  // this 1,024-block's allotments up to this round (all loads at once)
#pragma unroll
  for (int r = 0; r < SC_ITEMS; ++r) {
    const long long pr = b0 + r * TPB + tid;
    cr[r] = (r <= rr && pr < n) ? cnt[pr] : 0u;
  }
  uint32_t pre = 0, tot = 0;
  if (!pscan) {  // (pscan: the block sums' exclusive scan and total, from many blocks up)
    for (int k = tid; k < nb; k += TPB) {
      const uint32_t v = partial[k];
      tot += v;
      pre += k < t ? v : 0u;
    }
  }
  uint32_t c = 0;
#pragma unroll
  for (int r = 0; r < SC_ITEMS; ++r) {
    if (r < rr) pre += cr[r];
    if (r == rr) c = cr[r];
  }
  uint32_t bpre, btot;
  block_exclusive_scan<TPB>(pre, bpre, lds);  // (only the totals are used)
  if (pscan) {
    bpre += pscan[t];
    btot = pscan[nb];
  } else {
    block_exclusive_scan<TPB>(tot, btot, lds);
  }
  // (vflag: the count phase found the range violated -- a separate count call)
  const bool violated =
      (assume && kfin && (((kfin[0] ^ kfin[1]) & assume) != 0u)) || (vflag && *vflag);
  if (blockIdx.x == 0 && tid == 0) {
    *i_dev = violated ? 0xFFFFFFFFu : btot;
    if (i_host) *i_host = (int32_t)btot;
  }
  if (violated || btot > cap) return;  // workgroup-uniform
  uint32_t rtot;
  const uint32_t start = bpre + block_exclusive_scan<TPB>(c, rtot, lds);
  if (gstart) {  // the generated first pass (GenSrc): start offsets and the 64-slot owners
    if (p < n) {
      gstart[p] = start;
      for (uint32_t k = (start + 63u) >> 6; c && (k << 6) < start + c; ++k) gseg[k] = (uint32_t)p;
    }
    return;
  }
  const long long p0 = p - lane;
  if (p0 >= n) {  // wave-uniform
    if (!ec.counts) return;  // (no barrier below)
  } else {
  const bool in = p < n;
  uint32_t g = 0;
  uint2 bx = make_uint2(0u, 0u);
  if (in && c) {
    g = order[p];
    bx = box[p];
  }
  const uint32_t base = __shfl(start, 0, 64);
  const int last_lane = (int)min(63LL, (long long)n - 1 - p0);
  const uint32_t total = __shfl(start + c, last_lane, 64) - base;
  const uint32_t rel = in ? start - base : total;
  int *mk = marks + (threadIdx.x & ~63);
  mk[lane] = -1;
  int carry = -1;
  for (uint32_t j0 = 0; j0 < total; j0 += 64) {
    const uint32_t j = j0 + lane;
    const int q = slot_owner(mk, j0, rel, c != 0u, carry);
    const uint32_t li = j - __shfl(rel, q, 64);
    const uint32_t q0 = __shfl(bx.x, q, 64), q1 = __shfl(bx.y, q, 64);
    const uint32_t qg = __shfl(g, q, 64);
    const int qx0 = (int)(q0 & 0xFFFFu), qy0 = (int)(q0 >> 16);
    const int qx1 = (int)(q1 & 0xFFFFu), qy1 = (int)(q1 >> 16);
    const int qbw = max(qx1 - qx0, 1);
    const int qarea = max(qx1 - qx0, 0) * max(qy1 - qy0, 0);
    uint32_t tile;
    if ((int)li < qarea) {  // li / qbw (exact below 2^20: the float estimate rounds to the floor)
      const int ly = li < (1u << 20)
                         ? (int)(((float)li + 0.5f) * __builtin_amdgcn_rcpf((float)qbw))
                         : (int)li / qbw;
      tile = (uint32_t)((qy0 + ly) * tbx + qx0 + ((int)li - ly * qbw));
    } else {
      tile = (uint32_t)(tbx * tby);  // an allotment past its box: the sentinel tile
    }
    if (j < total) {
      tkeys[base + j] = tile;
      tvals[base + j] = qg;
      if (ec.counts) {  // the first sort pass's digit count (EmitCounts)
        const uint32_t st = (base + j) >> ec.shift, lt = st - (bpre >> ec.shift);
        const uint32_t d = tile & (ecr - 1u);
        if (lt < (uint32_t)EC_LT) atomicAdd(&ech[lt * ecr + d], 1u);
        else atomicAdd(&ec.counts[(size_t)st * ecr + d], 1u);
      }
    }
  }
  }
  if (ec.counts) {  // every wave of the workgroup reaches this barrier
    __syncthreads();
    const uint32_t ft = bpre >> ec.shift;
    for (int i = tid; i < EC_LT * (int)ecr; i += TPB) {
      const uint32_t v = ech[i];
      const long long st = (long long)ft + (i >> ec.width);
      if (v && st < ec.nblocks) atomicAdd(&ec.counts[(size_t)st * ecr + (i & (ecr - 1u))], v);
    }
  }
}

// The tile table from the last sort pass's run bounds (os_pass_kernel tbins): row t holds
// (max(n - first), max(end)) over the runs of tile t, or (0, 0) when no run (the emission
// cleared it) -> gsplat's (first, end).  n_dev: the device count of a capacity-launched sort
// (above cap the sort did nothing and the table stays cleared).  Replaces writing the sorted
// keys and a pass over them (8 B per intersection).
__global__ __launch_bounds__(TPB) void ts_decode_kernel(long long T, long long cap,
                                                        int *__restrict__ bins,
                                                        const uint32_t *__restrict__ n_dev) {
  long long n = cap;
  if (n_dev) {
    if ((long long)*n_dev > cap) return;
    n = *n_dev;
  }
  const long long t = (long long)blockIdx.x * TPB + threadIdx.x;
  if (t >= T) return;
  const int2 r = reinterpret_cast<int2 *>(bins)[t];
  if (r.y > 0) reinterpret_cast<int2 *>(bins)[t] = make_int2((int)(n - r.x), r.y);
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

// ------------------------------------------------------------------ bucket binning
// The same output as the sorted scheme above (gsplat's order: by tile, then depth bits, then
// Gaussian id) without any device-wide sort:
//   phase 1  bk_totals / bk_finalize: I = sum of tile allotments, visible count (2 launches);
//   phase 2  bk_count: per workgroup of BK_CHUNK Gaussians, an LDS histogram of the tile ids
//              of their intersections (the emit kernel's coalesced expansion) -> M[w][tile];
//            bk_scan: per tile, the exclusive prefix of M over workgroups; the last workgroup
//              scans the tile totals -> tile starts and tile_bins;
//            bk_place: the same expansion again, each intersection's Gaussian id stored at
//              start[tile] + M[w][tile] + (LDS atomic rank) -- grouped by tile, unordered;
//            bk_sort: one workgroup per tile sorts its list by (depth bits, id) with an LDS
//              LSD radix sort (stable wave64 ballot-match ranking, digits whose value never
//              changes inside the tile skipped); longer lists than LDS holds stream through
//              a global ping-pong buffer.  Id ties (equal depth bits) are resolved by sorting
//              the ids first (only when the tile has equal keys).
// Replaces the N-key depth sort (4 passes), the emission and the I-key tile sort (2 passes):
// 4 launches after the host read of I instead of 8, and 2 before it instead of 15.
constexpr int BK_NT = 1024;               // threads of the bucket count / place / scan kernels
constexpr int BK_CHUNK = 4096;            // Gaussians per bucket workgroup
constexpr int BK_MAX_BUCKETS = 16448;     // tiles + 1 (sentinel bucket) held in LDS (~64 KB)

// phase 1: per block, the sum of tile allotments and the number of visible Gaussians
__global__ __launch_bounds__(TPB) void bk_totals_kernel(int n, const uint4 *__restrict__ rec,
                                                        const uint32_t *__restrict__ dkeys,
                                                        uint32_t *__restrict__ partial) {
  __shared__ uint32_t lds[TPB / 64];
  const long long base = (long long)blockIdx.x * SC_TILE;
  uint32_t c = 0, v = 0;
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) {
    const long long i = base + k * TPB + threadIdx.x;
    if (i < n) {
      c += rec[i].x;
      v += dkeys[i] != 0xFFFFFFFFu;
    }
  }
  uint32_t tc, tv;
  block_exclusive_scan<TPB>(c, tc, lds);
  block_exclusive_scan<TPB>(v, tv, lds);
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = tc;
    partial[2 * blockIdx.x + 1] = tv;
  }
}

// One workgroup: d_counts[0] = visible count, d_counts[1] = I (pinned host memory).
__global__ __launch_bounds__(1024) void bk_finalize_kernel(int nb, const uint32_t *__restrict__ partial,
                                                           int *__restrict__ d_counts,
                                                           uint32_t *__restrict__ i_dev) {
  __shared__ uint32_t lds[16];
  uint32_t c = 0, v = 0;
  for (int i = threadIdx.x; i < nb; i += 1024) {
    c += partial[2 * i];
    v += partial[2 * i + 1];
  }
  uint32_t tc, tv;
  block_exclusive_scan<1024>(c, tc, lds);
  block_exclusive_scan<1024>(v, tv, lds);
  if (threadIdx.x == 0) {
    *i_dev = tc;  // device copy (read by the pre-launched placement)
    d_counts[0] = (int)tv;
    __threadfence_system();
    d_counts[1] = (int)tc;  // written last: the host polls this word
  }
}

// The intersections of 64 consecutive Gaussians (one per lane), expanded cooperatively: the
// wave's combined slot range is walked 64 slots at a time and f(tile, gaussian) is called for
// each slot (tile = T for the padding of an allotment larger than its box, as emit_kernel).
template <typename F>
__device__ __forceinline__ void expand_wave(long long p, long long n, const uint4 *__restrict__ rec,
                                            int tbx, int tby, int *marks, F &&f) {
  const int lane = threadIdx.x & 63;
  uint32_t c = 0;
  uint4 q = make_uint4(0u, 0u, 0u, 0u);
  if (p < n) {
    q = rec[p];
    c = q.x;
  }
  // inclusive wave scan of the allotments
  uint32_t inc = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(inc, off, 64);
    if (lane >= off) inc += o;
  }
  const uint32_t total = __shfl(inc, 63, 64);
  const uint32_t rel = inc - c;  // exclusive start of this lane's slots
  const uint32_t g = (uint32_t)p;
  int *mk = marks + (threadIdx.x & ~63);  // (slot owners: slot_owner)
  mk[lane] = -1;
  int carry = -1;
  for (uint32_t j0 = 0; j0 < total; j0 += 64) {
    const uint32_t j = j0 + lane;
    // owner = the last lane o with rel[o] <= j and an allotment (lanes past n start at total)
    const int o = slot_owner(mk, j0, rel, c != 0u, carry);
    const uint32_t li = j - __shfl(rel, o, 64);
    const uint32_t b0 = __shfl(q.y, o, 64), b1 = __shfl(q.z, o, 64);
    const uint32_t og = __shfl(g, o, 64);
    const int qx0 = (int)(b0 & 0xFFFFu), qy0 = (int)(b0 >> 16);
    const int qx1 = (int)(b1 & 0xFFFFu), qy1 = (int)(b1 >> 16);
    const int qbw = max(qx1 - qx0, 1);
    const int qarea = max(qx1 - qx0, 0) * max(qy1 - qy0, 0);
    uint32_t tile;
    if ((int)li < qarea) {
      const int ly = li < (1u << 20)
                         ? (int)(((float)li + 0.5f) * __builtin_amdgcn_rcpf((float)qbw))
                         : (int)li / qbw;
      tile = (uint32_t)((qy0 + ly) * tbx + qx0 + ((int)li - ly * qbw));
    } else {
      tile = (uint32_t)(tbx * tby);
    }
    if (j < total) f(tile, og);
  }
}

__global__ __launch_bounds__(BK_NT) void bk_count_kernel(int n, const uint4 *__restrict__ rec, int tbx,
                                                         int tby, int nbk, uint32_t *__restrict__ M,
                                                         uint32_t *__restrict__ ctr) {
  constexpr int NW = BK_NT / 64;
  __shared__ uint32_t hist[BK_MAX_BUCKETS];
  __shared__ int marks[BK_NT];  // (expand_wave's slot owners)
  for (int i = threadIdx.x; i < nbk; i += BK_NT) hist[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ctr = 0u;  // bk_scan's last-block counter
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long base = (long long)blockIdx.x * BK_CHUNK;
  for (int r = 0; r < BK_CHUNK / (64 * NW); ++r) {
    const long long p0 = base + (long long)(r * NW + wave) * 64;
    if (p0 >= n) break;  // wave-uniform
    expand_wave(p0 + lane, n, rec, tbx, tby, marks,
                [&](uint32_t tile, uint32_t) { atomicAdd(&hist[tile], 1u); });
  }
  __syncthreads();
  uint32_t *col = M + (size_t)blockIdx.x * nbk;
  for (int i = threadIdx.x; i < nbk; i += BK_NT) col[i] = hist[i];
}

// Bucket b = blockIdx.x * 64 + lane; wave v scans workgroup columns [v * cw, (v+1) * cw).
__global__ __launch_bounds__(BK_NT) void bk_scan_kernel(int nbk, int nwg, uint32_t *__restrict__ M,
                                                        uint32_t *__restrict__ tot,
                                                        uint32_t *__restrict__ start,
                                                        uint32_t *__restrict__ ctr, int T,
                                                        int *__restrict__ tile_bins,
                                                        const uint32_t *__restrict__ i_dev = nullptr,
                                                        uint32_t cap = 0) {
  constexpr int NW = BK_NT / 64;
  __shared__ uint32_t seg[NW][64];
  __shared__ uint32_t lds[NW];
  __shared__ bool last;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * 64 + lane;
  const int cw = (nwg + NW - 1) / NW;
  const int w0 = min(wave * cw, nwg), w1 = min(w0 + cw, nwg);
  uint32_t s = 0;
  if (b < nbk) {
    int w = w0;
    for (; w + 8 <= w1; w += 8) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = M[(size_t)(w + u) * nbk + b];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; w < w1; ++w) s += M[(size_t)w * nbk + b];
  }
  seg[wave][lane] = s;
  __syncthreads();
  uint32_t run = 0, total = 0;
#pragma unroll
  for (int v = 0; v < NW; ++v) {
    const uint32_t x = seg[v][lane];
    if (v < wave) run += x;
    total += x;
  }
  if (b < nbk) {
    int w = w0;
    for (; w + 8 <= w1; w += 8) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = M[(size_t)(w + u) * nbk + b];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        M[(size_t)(w + u) * nbk + b] = run;
        run += v[u];
      }
    }
    for (; w < w1; ++w) {
      const uint32_t v = M[(size_t)w * nbk + b];
      M[(size_t)w * nbk + b] = run;
      run += v;
    }
    if (wave == 0) tot[b] = total;
  }
  // the last workgroup to finish scans the bucket totals (one device-scope fence per
  // workgroup: on MI355X it writes back the XCD's L2, far too costly per wave)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(ctr, 1u) == gridDim.x - 1;
    if (last) __threadfence();
  }
  __syncthreads();
  if (!last) return;
  if (i_dev && *i_dev > cap) {  // capacity-launched (EMIT_SPEC) and overflowed: an empty table
    for (int i = threadIdx.x; i < 2 * T; i += BK_NT) tile_bins[i] = 0;
    return;
  }
  uint32_t running = 0;
  for (int c0 = 0; c0 < nbk; c0 += BK_NT) {
    const int i = c0 + threadIdx.x;
    const uint32_t v = i < nbk ? __hip_atomic_load(&tot[i], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                               : 0u;
    uint32_t t;
    const uint32_t ex = running + block_exclusive_scan<BK_NT>(v, t, lds);
    if (i < nbk) {
      start[i] = ex;
      if (i < T) {  // empty tiles stay (0, 0), as gsplat's zero-filled tile_bins
        tile_bins[2 * i] = v ? (int)ex : 0;
        tile_bins[2 * i + 1] = v ? (int)(ex + v) : 0;
      }
    }
    running += t;
  }
}

__global__ __launch_bounds__(BK_NT) void bk_place_kernel(int n, const uint4 *__restrict__ rec, int tbx,
                                                         int tby, int nbk,
                                                         const uint32_t *__restrict__ M,
                                                         const uint32_t *__restrict__ start,
                                                         uint32_t *__restrict__ ids,
                                                         const uint32_t *__restrict__ i_dev = nullptr,
                                                         uint32_t cap = 0) {
  constexpr int NW = BK_NT / 64;
  __shared__ uint32_t cur[BK_MAX_BUCKETS];
  __shared__ int marks[BK_NT];  // (expand_wave's slot owners)
  if (i_dev && *i_dev > cap) return;  // pre-launched: as emit_kernel
  const uint32_t *col = M + (size_t)blockIdx.x * nbk;
  for (int i = threadIdx.x; i < nbk; i += BK_NT) cur[i] = start[i] + col[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long base = (long long)blockIdx.x * BK_CHUNK;
  for (int r = 0; r < BK_CHUNK / (64 * NW); ++r) {
    const long long p0 = base + (long long)(r * NW + wave) * 64;
    if (p0 >= n) break;  // wave-uniform
    expand_wave(p0 + lane, n, rec, tbx, tby, marks, [&](uint32_t tile, uint32_t g) {
      ids[atomicAdd(&cur[tile], 1u)] = g;
    });
  }
}

// ---- per-tile LSD radix sort (bk_sort_kernel) ----
// ITEMS = 0: the MSD kernel's layout (key/val arrays of CAPX entries)
template <int NT, int ITEMS>
struct BsSmem {
  static constexpr int MB = ITEMS ? 2 : 1024;  // MSD buckets (bs_msd_sort; unused by the LSD)
  static constexpr int CAPX = ITEMS ? NT * ITEMS : 4096;
  uint32_t key[CAPX];
  uint32_t val[CAPX];
  uint32_t wcnt[NT / 64][256];
  uint32_t loc_off[256];
  uint32_t base[256];
  uint32_t scan_tmp[NT / 64];
  uint32_t red, red2[3];
  uint32_t mtab[2 * MB];  // MSD bucket counters / cursors and starts
};

// Stable rank, within the workgroup, of this thread's elements r < R (element index
// wave * R * 64 + r * 64 + lane; the first nvalid elements are real) by their 8-bit digit
// dg[r]: dst[r] = chunk-local destination.  Returns, in thread tid < 256, digit tid's count;
// sm.loc_off holds the digits' exclusive scan.
template <int NT, int ITEMS>
__device__ __forceinline__ uint32_t bs_rank(const uint32_t (&dg)[ITEMS], int R, int nvalid,
                                            uint32_t (&dst)[ITEMS], BsSmem<NT, ITEMS> &sm) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int e = tid; e < NW * 256; e += NT) (&sm.wcnt[0][0])[e] = 0;
  __syncthreads();
  uint32_t rank[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    if (r >= R) break;  // wave-uniform
    const int i = wave * R * 64 + r * 64 + lane;
    const bool valid = i < nvalid;
    const uint32_t d = dg[r];
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const unsigned long long m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const int leader = valid ? (int)__builtin_ctzll(peers) : lane;
    uint32_t old = 0;
    if (valid && leader == lane) old = atomicAdd(&sm.wcnt[wave][d], (uint32_t)__popcll(peers));
    old = __shfl(old, leader, 64);
    rank[r] = old + (uint32_t)__popcll(peers & lt);
  }
  __syncthreads();
  uint32_t cnt = 0;
  if (tid < 256) {
    uint32_t sacc = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t c = sm.wcnt[w][tid];
      sm.wcnt[w][tid] = sacc;
      sacc += c;
    }
    cnt = sacc;
  }
  {
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan<NT>(cnt, tot, sm.scan_tmp);
    if (tid < 256) sm.loc_off[tid] = ex;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    if (r >= R) break;
    dst[r] = sm.loc_off[dg[r]] + sm.wcnt[wave][dg[r]] + rank[r];
  }
  return cnt;
}

template <int NT, int ITEMS>
__device__ __forceinline__ uint32_t bs_block_reduce(uint32_t w, bool is_min, BsSmem<NT, ITEMS> &sm) {
  const int tid = threadIdx.x, lane = tid & 63;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint32_t o = __shfl_xor(w, off, 64);
    w = is_min ? min(w, o) : (w | o);
  }
  __syncthreads();
  if (tid == 0) sm.red = is_min ? 0xFFFFFFFFu : 0u;
  __syncthreads();
  if (lane == 0) {
    if (is_min) atomicMin(&sm.red, w); else atomicOr(&sm.red, w);
  }
  __syncthreads();
  return sm.red;
}

// Common case of the per-tile sort: one MSD step into MB buckets by the top bits of key - min
// (unstable LDS scatter), then each element's rank inside its bucket by counting the smaller
// (key, id) pairs there (equal pairs -- a Gaussian padded into the sentinel bucket more than
// once -- ordered by scatter position).  Returns false, having written nothing to global memory,
// when a bucket holds more than BS_MSD_MAXB elements (clustered depths): the LSD path then sorts.
constexpr int BS_MSD_MAXB = 64;
template <int NT, int ITEMS, int SI>
__device__ bool bs_msd_sort(uint32_t s0, uint32_t L, const uint32_t *__restrict__ ids,
                            const uint32_t *__restrict__ dkeys, uint32_t *__restrict__ out,
                            BsSmem<NT, SI> &sm) {
  constexpr int MB = BsSmem<NT, SI>::MB;
  constexpr int LOGMB = MB == 2048 ? 11 : MB == 1024 ? 10 : MB == 512 ? 9 : 8;
  static_assert((1 << LOGMB) == MB, "MSD bucket count must be 256..2048");
  const int tid = threadIdx.x;
  uint32_t k[ITEMS], v[ITEMS], bk[ITEMS], pos[ITEMS];
  uint32_t kmn = 0xFFFFFFFFu, kmx = 0u;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t i = tid + r * NT;
    if (i < L) {
      v[r] = ids[s0 + i];
      k[r] = dkeys[v[r]];
      kmn = min(kmn, k[r]);
      kmx = max(kmx, k[r]);
    }
  }
  uint32_t *hist = sm.mtab, *bstart = sm.mtab + MB;
  for (int e = tid; e < MB; e += NT) hist[e] = 0;
  // min and max in one round: sm.red2 = {min k, min ~k}
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    kmn = min(kmn, (uint32_t)__shfl_xor(kmn, off, 64));
    kmx = max(kmx, (uint32_t)__shfl_xor(kmx, off, 64));
  }
  if (tid == 0) {
    sm.red2[0] = 0xFFFFFFFFu;
    sm.red2[1] = 0u;
  }
  __syncthreads();
  if ((tid & 63) == 0) {
    atomicMin(&sm.red2[0], kmn);
    atomicMax(&sm.red2[1], kmx);
  }
  __syncthreads();
  const uint32_t kmin = sm.red2[0], kmax = sm.red2[1];
  const int bits = 32 - __builtin_clz((kmax - kmin) | 1u);
  const int shift = bits > LOGMB ? bits - LOGMB : 0;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    if (tid + r * NT < L) {
      bk[r] = (k[r] - kmin) >> shift;
      atomicAdd(&hist[bk[r]], 1u);
    }
  }
  __syncthreads();
  constexpr int PER = MB / NT;
  uint32_t c[PER], sum = 0, mx = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    c[j] = hist[tid * PER + j];
    sum += c[j];
    mx = max(mx, c[j]);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, off, 64));
  if (tid == 0) sm.red2[2] = 0u;
  uint32_t tot;
  uint32_t run = block_exclusive_scan<NT>(sum, tot, sm.scan_tmp);  // (barriers)
  if ((tid & 63) == 0) atomicMax(&sm.red2[2], mx);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    bstart[tid * PER + j] = run;
    hist[tid * PER + j] = run;  // scatter cursor
    run += c[j];
  }
  __syncthreads();
  if (sm.red2[2] > (uint32_t)BS_MSD_MAXB) return false;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    if (tid + r * NT < L) {
      pos[r] = atomicAdd(&hist[bk[r]], 1u);
      sm.key[pos[r]] = k[r];
      sm.val[pos[r]] = v[r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    if (tid + r * NT < L) {
      const uint32_t bs = bstart[bk[r]];
      const uint32_t be = bk[r] + 1 < (uint32_t)MB ? bstart[bk[r] + 1] : L;
      uint32_t rank = 0;
      for (uint32_t j = bs; j < be; ++j) {
        const uint32_t kj = sm.key[j], vj = sm.val[j];
        rank += (kj < k[r]) || (kj == k[r] && (vj < v[r] || (vj == v[r] && j < pos[r])));
      }
      out[s0 + bs + rank] = v[r];
    }
  }
  return true;
}

// The per-tile sort's common case (bs_msd_sort) for lists up to NT * ITEMS long; other lists
// (longer, or with a crowded MSD bucket) are flagged in fail[] for bk_sort_kernel.
template <int NT, int ITEMS>
__global__ __launch_bounds__(NT) void bk_msd_kernel(int nbk, const uint32_t *__restrict__ start,
                                                    const uint32_t *__restrict__ tot,
                                                    const uint32_t *__restrict__ ids,
                                                    const uint32_t *__restrict__ dkeys,
                                                    uint32_t *__restrict__ out,
                                                    uint32_t *__restrict__ fail,
                                                    const uint32_t *__restrict__ i_dev = nullptr,
                                                    uint32_t cap = 0) {
  __shared__ BsSmem<NT, 0> sm;
  if (i_dev && *i_dev > cap) return;  // capacity overflow (EMIT_SPEC): nothing was placed
  const int b = blockIdx.x;
  const uint32_t s0 = start[b], L = tot[b];
  bool ok = true;
  if (L == 1) {
    if (threadIdx.x == 0) out[s0] = ids[s0];
  } else if (L > 1) {
    ok = L <= (uint32_t)(NT * ITEMS) &&
         bs_msd_sort<NT, ITEMS>(s0, L, ids, dkeys, out, sm);
  }
  if (threadIdx.x == 0) fail[b] = ok ? 0u : 1u;
}

// Sorts bucket b's list ids[start[b] .. start[b] + tot[b]) by (dkeys[id], id) into out, for
// lists with lo <= length <= hi.  Digits are taken from key - (the list's smallest key), and
// digits that never vary are skipped.  Up to NT * ITEMS elements stay in registers and LDS;
// longer lists stream through (ka, va) / (kb, vb) at the list's offset in chunks of that size.
// Equal keys: sorted by id first (LSD), then by key.
template <int NT, int ITEMS>
__global__ __launch_bounds__(NT) void bk_sort_kernel(int nbk, uint32_t lo, uint32_t hi,
                                                     const uint32_t *__restrict__ start,
                                                     const uint32_t *__restrict__ tot,
                                                     const uint32_t *__restrict__ ids,
                                                     const uint32_t *__restrict__ dkeys,
                                                     uint32_t *__restrict__ out, uint32_t *ka,
                                                     uint32_t *va, uint32_t *kb, uint32_t *vb,
                                                     const uint32_t *__restrict__ fail,
                                                     const uint32_t *__restrict__ i_dev = nullptr,
                                                     uint32_t cap = 0) {
  constexpr int CAP = NT * ITEMS;
  __shared__ BsSmem<NT, ITEMS> sm;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (i_dev && *i_dev > cap) return;  // capacity overflow (EMIT_SPEC)
  if (fail && !fail[b]) return;  // sorted by bk_msd_kernel
  const uint32_t s0 = start[b], L = tot[b];
  if (L < lo || L > hi || L == 0) return;
  if (L == 1) {
    if (tid == 0) out[s0] = ids[s0];
    return;
  }
  if (L <= (uint32_t)CAP) {
    const int R = (int)((L + NT - 1) / NT);  // rows per wave
    uint32_t k[ITEMS], v[ITEMS], dg[ITEMS], dst[ITEMS];
    uint32_t kmn = 0xFFFFFFFFu;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      if (r >= R) break;
      const uint32_t i = wave * R * 64 + r * 64 + lane;
      v[r] = i < L ? ids[s0 + i] : 0u;
      k[r] = i < L ? dkeys[v[r]] : 0xFFFFFFFFu;
      kmn = min(kmn, k[r]);
    }
    const uint32_t kmin = bs_block_reduce(kmn, true, sm);
    uint32_t xv = 0;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      if (r >= R) break;
      if (wave * R * 64 + r * 64 + lane < (int)L) xv |= k[r] - kmin;
    }
    uint32_t keymask = 0, idmask = 0;
    {
      const uint32_t x = bs_block_reduce(xv, false, sm);
      for (int d = 0; d < 4; ++d) keymask |= ((x >> (8 * d)) & 0xFFu) ? 1u << d : 0u;
    }
    for (int phase = 0;; ++phase) {
      // passes: id digits (idmask) then key digits (keymask), least significant first
      for (int q = 0; q < 8; ++q) {
        const bool by_id = q < 4;
        const int d = q & 3;
        if (!(((by_id ? idmask : keymask) >> d) & 1u)) continue;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
          if (r >= R) break;
          dg[r] = ((by_id ? v[r] : k[r] - kmin) >> (8 * d)) & 0xFFu;
        }
        bs_rank<NT, ITEMS>(dg, R, (int)L, dst, sm);
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
          if (r >= R) break;
          if (wave * R * 64 + r * 64 + lane < (int)L) {
            sm.key[dst[r]] = k[r];
            sm.val[dst[r]] = v[r];
          }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
          if (r >= R) break;
          const int i = wave * R * 64 + r * 64 + lane;
          if (i < (int)L) {
            k[r] = sm.key[i];
            v[r] = sm.val[i];
          }
        }
        __syncthreads();
      }
      if (phase == 1) break;
      // in key order now: equal neighbours are id ties, which need the id digits first
      uint32_t tie = 0;
#pragma unroll
      for (int r = 0; r < ITEMS; ++r) {
        if (r >= R) break;
        const int i = wave * R * 64 + r * 64 + lane;
        if (i > 0 && i < (int)L && sm.key[i - 1] == k[r]) tie = 1;
      }
      if (!bs_block_reduce(tie, false, sm)) break;
      uint32_t iv = 0;
#pragma unroll
      for (int r = 0; r < ITEMS; ++r) {
        if (r >= R) break;
        if (wave * R * 64 + r * 64 + lane < (int)L) iv |= v[r];
      }
      const uint32_t ix = bs_block_reduce(iv, false, sm);
      for (int d = 0; d < 4; ++d) idmask |= ((ix >> (8 * d)) & 0xFFu) ? 1u << d : 0u;
    }
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      if (r >= R) break;
      const int i = wave * R * 64 + r * 64 + lane;
      if (i < (int)L) out[s0 + i] = v[r];
    }
    return;
  }
  // long list: chunks of CAP through global memory, id digits always first
  uint32_t kmn = 0xFFFFFFFFu, iv = 0;
  for (uint32_t i = tid; i < L; i += NT) {
    const uint32_t g = ids[s0 + i];
    kmn = min(kmn, dkeys[g]);
    iv |= g;
  }
  const uint32_t kmin = bs_block_reduce(kmn, true, sm);
  uint32_t xv = 0;
  for (uint32_t i = tid; i < L; i += NT) xv |= dkeys[ids[s0 + i]] - kmin;
  const uint32_t x = bs_block_reduce(xv, false, sm);
  const uint32_t ix = bs_block_reduce(iv, false, sm);
  int npass = 0;
  for (int d = 0; d < 4; ++d) npass += (((ix >> (8 * d)) & 0xFFu) != 0) + (((x >> (8 * d)) & 0xFFu) != 0);
  if (npass == 0) {  // one Gaussian repeated (sentinel padding): already in order
    for (uint32_t i = tid; i < L; i += NT) out[s0 + i] = ids[s0 + i];
    return;
  }
  const uint32_t *srck = nullptr, *srcv = ids;  // the first pass gathers the keys
  uint32_t *dk = ka, *dv = va;
  int done = 0;
  for (int q = 0; q < 8; ++q) {
    const bool by_id = q < 4;
    const int d = q & 3, shift = 8 * d;
    if (!(((by_id ? ix : x) >> shift) & 0xFFu)) continue;
    const bool final_pass = ++done == npass;
    // digit histogram of the whole list -> digit bases
    if (tid < 256) sm.base[tid] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < L; i += NT) {
      const uint32_t vv = srcv[s0 + i];
      const uint32_t kk = srck ? srck[s0 + i] : dkeys[vv];
      atomicAdd(&sm.base[((by_id ? vv : kk - kmin) >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    {
      const uint32_t c = tid < 256 ? sm.base[tid] : 0u;
      uint32_t t;
      const uint32_t ex = block_exclusive_scan<NT>(c, t, sm.scan_tmp);
      if (tid < 256) sm.base[tid] = ex;
    }
    __syncthreads();
    for (uint32_t c0 = 0; c0 < L; c0 += CAP) {
      const int nv = (int)min((uint32_t)CAP, L - c0);
      const int R = (nv + NT - 1) / NT;
      uint32_t k[ITEMS], v[ITEMS], dg[ITEMS], dst[ITEMS];
#pragma unroll
      for (int r = 0; r < ITEMS; ++r) {
        if (r >= R) break;
        const int i = wave * R * 64 + r * 64 + lane;
        v[r] = i < nv ? srcv[s0 + c0 + i] : 0u;
        k[r] = i < nv ? (srck ? srck[s0 + c0 + i] : dkeys[v[r]]) : 0u;
        dg[r] = ((by_id ? v[r] : k[r] - kmin) >> shift) & 0xFFu;
      }
      const uint32_t cnt = bs_rank<NT, ITEMS>(dg, R, nv, dst, sm);
#pragma unroll
      for (int r = 0; r < ITEMS; ++r) {
        if (r >= R) break;
        if (wave * R * 64 + r * 64 + lane < nv) {
          const uint32_t pos = sm.base[dg[r]] + dst[r] - sm.loc_off[dg[r]];
          if (final_pass) {
            out[s0 + pos] = v[r];
          } else {
            dk[s0 + pos] = k[r];
            dv[s0 + pos] = v[r];
          }
        }
      }
      __syncthreads();
      if (tid < 256) sm.base[tid] += cnt;  // this chunk's count of digit tid
      __syncthreads();
    }
    srck = dk;
    srcv = dv;
    dk = dk == ka ? kb : ka;
    dv = dv == va ? vb : va;
    __threadfence_block();
    __syncthreads();
  }
}

// ---- workspace layouts of the fused binning (phase 1 and phase 2 are separate buffers) ----
constexpr size_t ALIGN = 256;
inline size_t al(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

struct Carver {
  char *base;
  size_t off = 0;
  explicit Carver(void *b) : base((char *)b) {}
  template <typename T>
  T *take(size_t bytes) {
    T *r = (T *)(base + off);
    off += al(bytes);
    return r;
  }
};

struct Phase1 {
  uint32_t *dkeys_a, *dvals_a, *dkeys_b, *dvals_b, *order, *cnt;
  uint4 *rec;  // per-Gaussian binning record (Gaussian order)
  uint2 *box;  // tile bbox in depth order (gather_counts_kernel)
  uint32_t *dcount;  // I on the device (the capacity-launched sort's bound check)
  void *rs_ws;
  size_t bytes;
};

Phase1 carve_phase1(void *base, int n) {
  Phase1 p;
  Carver c(base);
  size_t nn = (size_t)(n > 0 ? n : 1) * 4;
  p.dkeys_a = c.take<uint32_t>(nn);
  p.dvals_a = c.take<uint32_t>(nn);
  p.dkeys_b = c.take<uint32_t>(nn);
  p.dvals_b = c.take<uint32_t>(nn);
  p.order = c.take<uint32_t>(nn);
  p.cnt = c.take<uint32_t>(nn);
  p.rec = c.take<uint4>(nn * 4);
  p.box = c.take<uint2>(nn * 2);
  p.dcount = c.take<uint32_t>(4 * sizeof(uint32_t));
  size_t rs = radix_ws_bytes(n, 0, 32);
  size_t sc = scan_ws_bytes(n);
  p.rs_ws = c.take<char>(rs > sc ? rs : sc);
  p.bytes = c.off;
  return p;
}

int bits_for(long long v) {  // smallest b with (1 << b) > v
  int b = 0;
  while (b < 62 && (1LL << b) <= v) ++b;
  return b;
}

// bucket scheme, phase 2: M [nwg][nbk], tot/start [nbk], last-block counter, the grouped ids
// and the long-list ping-pong buffers [I] each
struct BkWs {
  uint32_t *M, *tot, *start, *ctr, *fail, *ids, *ka, *va, *kb, *vb;
  int nwg, nbk;
  size_t bytes;
};

BkWs carve_bk(void *base, int n, long long I, long long T) {
  BkWs w;
  Carver c(base);
  w.nwg = (int)cdiv(n > 0 ? n : 1, BK_CHUNK);
  w.nbk = (int)(T + 1);
  const size_t ii = (size_t)(I > 0 ? I : 1) * 4;
  w.M = c.take<uint32_t>((size_t)w.nwg * w.nbk * 4);
  w.tot = c.take<uint32_t>((size_t)w.nbk * 4);
  w.start = c.take<uint32_t>((size_t)w.nbk * 4);
  w.ctr = c.take<uint32_t>(4);
  w.fail = c.take<uint32_t>((size_t)w.nbk * 4);
  w.ids = c.take<uint32_t>(ii);
  w.ka = c.take<uint32_t>(ii);
  w.va = c.take<uint32_t>(ii);
  w.kb = c.take<uint32_t>(ii);
  w.vb = c.take<uint32_t>(ii);
  w.bytes = c.off;
  return w;
}

struct TsWs {
  uint32_t *ka, *va, *kb, *vb;
  uint32_t *gstart, *gseg;  // the generated first pass (cap >= GEN_MIN_I)
  uint32_t *pscan;          // the block sums' scan (many blocks: ts_emit_kernel)
  void *rs;
  size_t bytes;
};
// gen (from GEN_MIN_I intersections): + the start offsets (n) and the 64-slot owners
constexpr long long GEN_MIN_I = 1LL << 24;
constexpr int TS_SCAN_NB = 1024;  // (ts_launch)
long long g_gen_min_i = GEN_MIN_I;  // (gsplat_debug_tile_sort_gen: tests force it lower)
TsWs carve_ts(void *base, long long cap, long long T, int n) {
  TsWs w;
  Carver c(base);
  const size_t ii = (size_t)(cap > 0 ? cap : 1) * sizeof(uint32_t);
  w.ka = c.take<uint32_t>(ii);
  w.va = c.take<uint32_t>(ii);
  w.kb = c.take<uint32_t>(ii);
  w.vb = c.take<uint32_t>(ii);
  // (any sort length up to cap: the short-tile plan below GS_ITEMS16_FROM keys -- the tile
  // sort's keys are never 32 bits -- has more tiles)
  const long long c1 = cap > 0 ? cap : 1,
                  c0 = c1 < (long long)(GS_ITEMS16_FROM) ? c1 : (long long)(GS_ITEMS16_FROM) - 1;
  const size_t r0 = radix_ws_bytes(c0, 0, bits_for(T)), r1 = radix_ws_bytes(c1, 0, bits_for(T));
  w.rs = c.take<char>(r0 > r1 ? r0 : r1);
  w.pscan = c.take<uint32_t>((size_t)(cdiv(n > 0 ? n : 1, SC_TILE) + 1) * 4);
  w.gstart = w.gseg = nullptr;
  if (cap >= g_gen_min_i) {
    w.gstart = c.take<uint32_t>((size_t)(n > 0 ? n : 1) * 4);
    w.gseg = c.take<uint32_t>((size_t)cdiv(cap, 64) * 4 + 4);
  }
  w.bytes = c.off;
  return w;
}

// The tile sort (ts_*) over phase 1's depth-ordered allotments into workspace2 (carve_ts at the
// capacity).  HEAD: the emission (I published to p1.dcount and i_host); TAIL: the
// sort and the tile table over m pairs: with n_dev, *n_dev of them (I on the device; m = cap,
// the launch length), else exactly m = I.
// ec_zeroed: the caller cleared ec_matrix(ws2, cap, T, n) (gather_counts_kernel), so the
// emission counts the sort's first pass (EmitCounts; one call: HEAD and TAIL, m = cap, not the
// generated first pass).
struct EcMatrix {
  uint32_t *counts;
  long long words;
  SortPlan plan;
};
EcMatrix ec_matrix(void *ws2, long long cap, long long T, int n) {
  const TsWs w = carve_ts(ws2, cap, T, n);
  const SortPlan sp = sort_plan(cap, 0, bits_for(T));
  // (in kb: free until the first pass writes it, after its row scan has read the counts;
  // nblocks x radix <= cap / 4 words)
  return EcMatrix{w.kb, sp.nblocks * sp.radix, sp};
}
// (the matrix must fit the kb buffer of cap words: always beyond a few thousand slots)
bool ec_applies(long long cap, long long T) {
  if (!(cap > 0 && cap < g_gen_min_i)) return false;
  const SortPlan sp = sort_plan(cap, 0, bits_for(T));
  return sp.nblocks * sp.radix <= cap;
}

void ts_launch(int n, const Phase1 &p1, void *ws2, int32_t *ids, int32_t *tile_bins, int tbx,
               int tby, long long cap, long long m, int32_t *i_host, uint32_t assume,
               bool head, bool tail, const uint32_t *n_dev, hipStream_t st,
               bool ec_zeroed = false) {
  const long long T = (long long)tbx * tby;
  const TsWs w = carve_ts(ws2, cap, T, n);
  EmitCounts ec{};
  const bool use_ec = ec_zeroed && head && tail && m == cap && !w.gstart;
  if (use_ec) {
    const EcMatrix em = ec_matrix(ws2, cap, T, n);
    ec.counts = em.counts;
    ec.width = em.plan.width;
    ec.shift = em.plan.items == 16 ? 12 : 10;  // (TPB * items slots per sort tile)
    ec.nblocks = em.plan.nblocks;
  }
  const int nb = (int)cdiv(n, SC_TILE);
  // every emission workgroup sums the block sums before it: quadratic in N, so from
  // TS_SCAN_NB blocks (1M Gaussians) one workgroup scans them first (c5: ~95M L2 reads saved)
  const bool scan = nb > TS_SCAN_NB;
  if (head && scan)
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, st,
                       rts_tile_counts(p1.rs_ws), nb, nullptr, nullptr, false, nullptr, 0u,
                       nullptr, w.pscan);
  if (head)
    hipLaunchKernelGGL(ts_emit_kernel, dim3((unsigned)nb * SC_ITEMS), dim3(TPB), 0, st, n, nb,
                       p1.order, p1.cnt, rts_tile_counts(p1.rs_ws), p1.box,
                       tbx, tby, w.ka, w.va, tile_bins, p1.dcount, i_host,
                       (uint32_t)(cap > 0xFFFFFFFELL ? 0xFFFFFFFELL : cap),
                       assume ? sort_kept_word(p1.rs_ws) + 1 : nullptr, assume, w.gstart, w.gseg,
                       p1.dcount + 2, scan ? w.pscan : nullptr, ec);
  if (!tail || m <= 0) return;
  GenSrc g{w.gstart, p1.cnt, p1.order, w.gseg, p1.box, tbx, tby, (long long)n};
  radix_sort_pairs<uint32_t>(w.ka, w.va, w.kb, w.vb, nullptr, (uint32_t *)ids, m, 0, bits_for(T),
                             w.rs, st, use_ec, false, 0u, nullptr, n_dev, tile_bins, (uint32_t)T,
                             w.gstart ? &g : nullptr, use_ec ? ec.counts : nullptr);
  hipLaunchKernelGGL(ts_decode_kernel, dim3(cdiv(T, TPB)), dim3(TPB), 0, st, T, m, tile_bins,
                     n_dev);
}

// Binning scheme (gsplat_debug_binning_scheme): -1 by size (shipped), 0 depth sort + tile sort,
// 1 tile buckets + per-tile sorts.  The buckets need far fewer launches (8 against ~23), which
// wins where every launch is short: small scenes, whose tile lists are short too (c2, 100k
// Gaussians @ 512^2, max list 837: 0.100 vs 0.112 ms).  A long list is sorted by one
// workgroup, so real scenes lose (c3 bear, 300k, max list 7,984: 0.365 vs 0.144 ms; headline
// 1M: 0.287 vs 0.243); the cut is on N, which the count phase must know before I exists.
int g_bin_scheme = -1;
// the emission counts the tile sort's first pass (speculative binning; gsplat_debug_emit_counts;
// -DGS_NO_EMIT_COUNTS: an A/B build with the count launch)
#ifdef GS_NO_EMIT_COUNTS
bool g_emit_counts = false;
#else
bool g_emit_counts = true;
#endif
bool use_bucket(long long n, long long T) {
  if (T + 1 > BK_MAX_BUCKETS) return false;
  return g_bin_scheme < 0 ? n <= (1LL << 17) : g_bin_scheme == 1;
}

}  // namespace

BinKeys bin_keys_view(void *workspace1, int n) {
  const Phase1 p = carve_phase1(workspace1, n);
  return BinKeys{p.dkeys_a, p.dvals_a, p.rec, p.bytes};
}

}  // namespace gs

using namespace gs;

#ifdef GSPLAT_TEST_HOOKS  // the test library only (libgsplat_mi355x_hooks.so, Makefile)
// The tile sort's generated first pass from min_i intersections (capacity; < 0: leave);
// returns the previous threshold.  Set it only between binnings: the workspace layout follows it.
extern "C" long long gsplat_debug_tile_sort_gen(long long min_i) {
  const long long prev = g_gen_min_i;
  if (min_i >= 0) g_gen_min_i = min_i;
  return prev;
}

extern "C" int gsplat_debug_depth_key_range(int on) {
  const int prev = g_key_range;
  if (on >= 0) g_key_range = on > 2 ? 2 : on;
  return prev;
}

// The speculative binning's first tile-sort pass counted by the emission (1, shipped) or by its
// own count launch (0); < 0 leaves it.  Returns the previous setting.
extern "C" int gsplat_debug_emit_counts(int on) {
  const int prev = g_emit_counts ? 1 : 0;
  if (on >= 0) g_emit_counts = on != 0;
  return prev;
}

extern "C" int gsplat_debug_binning_scheme(int scheme) {
  const int prev = g_bin_scheme;
  if (scheme >= -1 && scheme <= 1) g_bin_scheme = scheme;
  return prev;
}
#endif

extern "C" size_t gsplat_bin_emit_workspace_size_for(int num_points, int64_t num_intersects,
                                                     int tile_bounds_x, int tile_bounds_y) {
  const long long T = (long long)tile_bounds_x * tile_bounds_y;
  if (num_points < 0 || num_intersects < 0 || tile_bounds_x <= 0 || tile_bounds_y <= 0) return 0;
  const size_t sorted = carve_ts(nullptr, num_intersects, T, num_points).bytes;
  if (!use_bucket(num_points, T)) return sorted;
  const size_t bk = carve_bk(nullptr, num_points, num_intersects, T).bytes;
  return bk > sorted ? bk : sorted;
}

extern "C" size_t gsplat_bin_count_workspace_size(int num_points) {
  return carve_phase1(nullptr, num_points).bytes;
}

static int bin_count_impl(int num_points, const float *xys, const float *depths,
                          const int32_t *radii, const int32_t *num_tiles_hit, int tile_bounds_x,
                          int tile_bounds_y, int32_t *d_counts, void *workspace1,
                          size_t workspace1_bytes, bool keyed, void *stream,
                          uint32_t assume_const = 0, bool range_out = false,
                          bool no_scan = false, uint32_t *zero = nullptr,
                          long long zero_words = 0) {
  hipStream_t st = (hipStream_t)stream;
  const long long T = (long long)tile_bounds_x * tile_bounds_y;
  if (num_points < 0 || tile_bounds_x <= 0 || tile_bounds_y <= 0 || tile_bounds_x > 65535 ||
      tile_bounds_y > 65535 || T >= (1LL << 31)) {
    set_error("bin_count: bad sizes (N=%d tiles=%dx%d)", num_points, tile_bounds_x,
              tile_bounds_y);
    return 1;
  }
  Phase1 p = carve_phase1(workspace1, num_points);
  if (workspace1_bytes < p.bytes) {
    set_error("bin_count: workspace %zu < %zu bytes", workspace1_bytes, p.bytes);
    return 1;
  }
  if (num_points == 0) {
    note(hipMemsetAsync(d_counts, 0, 2 * sizeof(int32_t), st), "hipMemsetAsync");
    return check_launch("bin_count");
  }
  const int n = num_points;
  if (use_bucket(num_points, T)) {  // buckets: depth keys + records, then I and the visible count
    const SortPlan sp = sort_plan(n, 0, 32);
#define DEPTH_KEYS0(It)                                                                     \
  hipLaunchKernelGGL(depth_keys_kernel<It>, dim3((unsigned)sp.nblocks), dim3(TPB), 0, st, n, xys, \
                     depths, radii, num_tiles_hit, tile_bounds_x, tile_bounds_y, p.dkeys_a,    \
                     p.dvals_a, p.rec, nullptr, sp.nblocks, nullptr)
    if (keyed) {
    } else if (sp.items == 16) DEPTH_KEYS0(16);
    else if (sp.items == 8) DEPTH_KEYS0(8);
    else DEPTH_KEYS0(4);
#undef DEPTH_KEYS0
    const int nb = (int)cdiv(n, SC_TILE);
    uint32_t *partial = (uint32_t *)p.rs_ws;
    hipLaunchKernelGGL(bk_totals_kernel, dim3(nb), dim3(TPB), 0, st, n, p.rec, p.dkeys_a, partial);
    hipLaunchKernelGGL(bk_finalize_kernel, dim3(1), dim3(1024), 0, st, nb, partial, d_counts,
                       p.dcount);
    return check_launch("bin_count");
  }
  // depth keys + records + the sort's pass-0 tile counts.  The depth sort compacts: its first
  // pass drops the culled Gaussians' all-ones keys, so the later passes, the gather and the
  // emission see only the visible ones.  depth_keys_kernel counts pass 0 (visible keys);
  // keyed: the sort counts pass 0 itself
  const SortPlan sp = sort_plan(n, 0, 32);
  const bool pre = !keyed;
  uint32_t *c0 = pre ? rts_tile_counts(p.rs_ws) : nullptr;
#define DEPTH_KEYS(It)                                                                      \
  hipLaunchKernelGGL(depth_keys_kernel<It>, dim3((unsigned)sp.nblocks), dim3(TPB), 0, st, n, xys, \
                     depths, radii, num_tiles_hit, tile_bounds_x, tile_bounds_y, p.dkeys_a,    \
                     p.dvals_a, p.rec, c0, sp.nblocks,                                         \
                     pre && use_key_range(n)                                                  \
                         ? (uint32_t *)((char *)p.rs_ws + radix_main_bytes(sp)) : nullptr)
  if (keyed) {
    // keys, ids and records already written (gsplat_fused_preprocess_forward_binned)
  } else if (sp.items == 16) DEPTH_KEYS(16);
  else if (sp.items == 8) DEPTH_KEYS(8);
  else DEPTH_KEYS(4);
#undef DEPTH_KEYS
  // range_out: d_counts[2..3] are written only when the key range is computed (the caller
  // zeroes them: without a range nothing is assumed and nothing reported)
  if (radix_sort_pairs<uint32_t>(p.dkeys_a, p.dvals_a, p.dkeys_b, p.dvals_b, nullptr, p.order, n,
                                 0, 32, p.rs_ws, st, pre, true,
                                 use_key_range(n) ? assume_const : 0u,
                                 range_out ? d_counts + 2 : nullptr))
    return 1;
  // depth-ordered allotments and boxes (+ per-block allotment sums) -> I
  const int nb = (int)cdiv(n, SC_TILE);
  // the kept count sits in the sort workspace's head, before the tile counts reused below
  const uint32_t *kept = sort_kept_word(p.rs_ws);
  uint32_t *partial = rts_tile_counts(p.rs_ws);  // the sort is done with its tile counts
  hipLaunchKernelGGL(gather_counts_kernel, dim3(nb), dim3(TPB), 0, st, n, p.order, kept, p.rec,
                     p.cnt, p.box, d_counts, partial, p.dcount + 2, zero, zero_words);
  // (the speculative binning: I from ts_emit_kernel)
  if (no_scan) return check_launch("bin_count");
  // I = the sum of the block sums, which stay as they are: the emission (ts_emit_kernel)
  // scans them itself, so a speculative count phase (no_scan) and this one leave the same state
  const uint32_t chk = range_out && use_key_range(n) ? assume_const : 0u;
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, st, partial, nb,
                     (uint32_t *)(d_counts + 1), p.dcount, false, chk ? kept + 1 : nullptr, chk,
                     p.dcount + 2);
  return check_launch("bin_count");
}

extern "C" int gsplat_bin_count(int num_points, const float *xys, const float *depths,
                                const int32_t *radii, const int32_t *num_tiles_hit,
                                int tile_bounds_x, int tile_bounds_y, int32_t *d_counts,
                                void *workspace1, size_t workspace1_bytes, void *stream) {
  return bin_count_impl(num_points, xys, depths, radii, num_tiles_hit, tile_bounds_x,
                        tile_bounds_y, d_counts, workspace1, workspace1_bytes, false, stream);
}

extern "C" int gsplat_bin_count_keyed(int num_points, int tile_bounds_x, int tile_bounds_y,
                                      int32_t *d_counts, void *workspace1,
                                      size_t workspace1_bytes, void *stream) {
  return bin_count_impl(num_points, nullptr, nullptr, nullptr, nullptr, tile_bounds_x,
                        tile_bounds_y, d_counts, workspace1, workspace1_bytes, true, stream);
}

// gsplat_bin_count_keyed plus the depth-key range across calls: depth-sort passes whose digit
// `assume_const` covers are not launched; d_counts[2] = 1 if this call's kept keys vary in an
// assumed-constant bit (the order is then wrong: re-bin), d_counts[3] = the bits that vary --
// both left as the caller set them (zero) when the sort computes no key range.
extern "C" int gsplat_bin_count_keyed_ex(int num_points, int tile_bounds_x, int tile_bounds_y,
                                         int32_t *d_counts, void *workspace1,
                                         size_t workspace1_bytes, uint32_t assume_const,
                                         void *stream) {
  return bin_count_impl(num_points, nullptr, nullptr, nullptr, nullptr, tile_bounds_x,
                        tile_bounds_y, d_counts, workspace1, workspace1_bytes, true, stream,
                        assume_const, true);
}

// The whole binning before the host knows I: the count phase (depth sort with the key-range
// assumption, gather_counts) and the tile sort launched at the capacity (I published from the
// device by ts_emit_kernel).
enum { EMIT_HEAD = 1, EMIT_TAIL = 2, EMIT_ALL = 3, EMIT_SPEC = 4 };
static int bin_emit_impl(int num_points, int64_t num_intersects, int64_t capacity,
                         int tile_bounds_x, int tile_bounds_y, int32_t *gaussian_ids_sorted,
                         int32_t *tile_bins, const void *workspace1, size_t workspace1_bytes,
                         void *workspace2, size_t workspace2_bytes, void *stream, int phase);

extern "C" int gsplat_bin_speculative(int num_points, int64_t capacity, int tile_bounds_x,
                                      int tile_bounds_y, int32_t *d_counts, void *workspace1,
                                      size_t workspace1_bytes, uint32_t assume_const,
                                      int32_t *gaussian_ids_sorted, int32_t *tile_bins,
                                      void *workspace2, size_t workspace2_bytes, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  const long long T = (long long)tile_bounds_x * tile_bounds_y;
  if (num_points <= 0 || capacity <= 0 || capacity > 0x3FFFFFFFLL || tile_bounds_x <= 0 ||
      tile_bounds_y <= 0 || tile_bounds_x > 65535 || tile_bounds_y > 65535 || T >= (1LL << 31)) {
    set_error("bin_speculative: bad sizes (N=%d capacity=%lld tiles=%dx%d)", num_points,
              (long long)capacity, tile_bounds_x, tile_bounds_y);
    return 1;
  }
  if (use_bucket(num_points, T)) {
    // tile buckets: the count phase (I on the device), then every bucket launch at the
    // capacity, each returning at once on an overflow (the table cleared by bk_scan_kernel)
    if (bin_count_impl(num_points, nullptr, nullptr, nullptr, nullptr, tile_bounds_x,
                       tile_bounds_y, d_counts, workspace1, workspace1_bytes, true, stream))
      return 1;
    return bin_emit_impl(num_points, 0, capacity, tile_bounds_x, tile_bounds_y,
                         gaussian_ids_sorted, tile_bins, workspace1, workspace1_bytes,
                         workspace2, workspace2_bytes, stream, EMIT_SPEC);
  }
  Phase1 p1 = carve_phase1(workspace1, num_points);
  const size_t need2 = carve_ts(nullptr, capacity, T, num_points).bytes;
  if (workspace1_bytes < p1.bytes || workspace2_bytes < need2) {
    set_error("bin_speculative: workspaces %zu/%zu < %zu/%zu bytes", workspace1_bytes,
              workspace2_bytes, p1.bytes, need2);
    return 1;
  }
  // the emission counts the tile sort's first pass (EmitCounts): its matrix is cleared by the
  // count phase's gather kernel
  const bool ec = g_emit_counts && ec_applies(capacity, T);
  const EcMatrix em = ec_matrix(workspace2, capacity, T, num_points);
  if (bin_count_impl(num_points, nullptr, nullptr, nullptr, nullptr, tile_bounds_x,
                     tile_bounds_y, d_counts, workspace1, workspace1_bytes, true, stream,
                     assume_const, true, true, ec ? em.counts : nullptr, ec ? em.words : 0))
    return 1;
  const uint32_t assume = use_key_range(num_points) ? assume_const : 0u;
  ts_launch(num_points, p1, workspace2, gaussian_ids_sorted, tile_bins, tile_bounds_x,
            tile_bounds_y, capacity, capacity, d_counts + 1, assume, true, true, p1.dcount, st,
            ec);
  return check_launch("bin_speculative");
}

// The emission in two halves around the host's read of I: HEAD = the launches that need only
// the phase-1 workspace and output buffers of `cap` intersections (sorted scheme: emit_kernel
// unless the generated first pass is chosen; bucket scheme: count, scan and placement), each
// checking the device copy of I against cap; TAIL = the rest (the tile sort / the per-tile
// sorts).  EMIT_ALL = both, with cap = I (gsplat_bin_emit).
// (EMIT_* : declared with gsplat_bin_speculative, above)

static int bin_emit_impl(int num_points, int64_t num_intersects, int64_t capacity,
                         int tile_bounds_x, int tile_bounds_y, int32_t *gaussian_ids_sorted,
                         int32_t *tile_bins, const void *workspace1, size_t workspace1_bytes,
                         void *workspace2, size_t workspace2_bytes, void *stream, int phase) {
  hipStream_t st = (hipStream_t)stream;
  const long long T = (long long)tile_bounds_x * tile_bounds_y;
  if (num_points < 0 || num_intersects < 0 || capacity < num_intersects ||
      capacity > 0x3FFFFFFFLL || tile_bounds_x <= 0 || tile_bounds_y <= 0 ||
      tile_bounds_x > 65535 || tile_bounds_y > 65535 || T >= (1LL << 31)) {
    set_error("bin_emit: bad sizes (N=%d I=%lld capacity=%lld tiles=%dx%d)", num_points,
              (long long)num_intersects, (long long)capacity, tile_bounds_x, tile_bounds_y);
    return 1;
  }
  Phase1 p1 = carve_phase1(const_cast<void *>(workspace1), num_points);
  const long long cap = capacity;
  // HEAD (pre-launched before the host read of I) needs no I-sized buffer; TAIL the rest
  const bool head = phase != EMIT_TAIL;
  const bool tail = phase != EMIT_HEAD;
  const uint32_t *idev = phase == EMIT_HEAD ? p1.dcount : nullptr;  // bound check when pre-launched
  if (use_bucket(num_points, T)) {
    const BkWs w = carve_bk(workspace2, num_points, cap, T);
    if (workspace1_bytes < p1.bytes || workspace2_bytes < w.bytes) {
      set_error("bin_emit: workspaces %zu/%zu < %zu/%zu bytes (phase-2 size from "
                "gsplat_bin_emit_workspace_size_for)", workspace1_bytes, workspace2_bytes,
                p1.bytes, w.bytes);
      return 1;
    }
    if (num_points == 0 || (phase != EMIT_HEAD && phase != EMIT_SPEC && num_intersects == 0)) {
      if (tail)
        note(hipMemsetAsync(tile_bins, 0, (size_t)T * 2 * sizeof(int32_t), st), "hipMemsetAsync");
      return check_launch("bin_emit");
    }
    const int n = num_points;
    // EMIT_SPEC (gsplat_bin_speculative): every launch at the capacity, I read on the device
    const uint32_t *sdev = phase == EMIT_SPEC ? p1.dcount : nullptr;
    if (phase == EMIT_SPEC) idev = p1.dcount;
    if (head) {
      hipLaunchKernelGGL(bk_count_kernel, dim3(w.nwg), dim3(BK_NT), 0, st, n, p1.rec, tile_bounds_x,
                         tile_bounds_y, w.nbk, w.M, w.ctr);
      hipLaunchKernelGGL(bk_scan_kernel, dim3(cdiv(w.nbk, 64)), dim3(BK_NT), 0, st, w.nbk, w.nwg,
                         w.M, w.tot, w.start, w.ctr, (int)T, tile_bins, sdev, (uint32_t)cap);
      hipLaunchKernelGGL(bk_place_kernel, dim3(w.nwg), dim3(BK_NT), 0, st, n, p1.rec,
                         tile_bounds_x, tile_bounds_y, w.nbk, w.M, w.start, w.ids, idev,
                         (uint32_t)cap);
    }
    if (!tail) return check_launch("bin_emit");
    // MSD + bucket ranking for lists up to 4,096 long; then the LSD sort for the others (up to
    // 4,096: 256 threads; longer: 1,024 threads, in LDS up to 14,336, then through the
    // ping-pong buffers)
    hipLaunchKernelGGL((bk_msd_kernel<TPB, 16>), dim3(w.nbk), dim3(TPB), 0, st, w.nbk, w.start,
                       w.tot, w.ids, p1.dkeys_a, (uint32_t *)gaussian_ids_sorted, w.fail, sdev,
                       (uint32_t)cap);
    hipLaunchKernelGGL((bk_sort_kernel<TPB, 16>), dim3(w.nbk), dim3(TPB), 0, st, w.nbk, 0u,
                       (uint32_t)(TPB * 16), w.start, w.tot, w.ids, p1.dkeys_a,
                       (uint32_t *)gaussian_ids_sorted, w.ka, w.va, w.kb, w.vb, w.fail, sdev,
                       (uint32_t)cap);
    hipLaunchKernelGGL((bk_sort_kernel<1024, 14>), dim3(w.nbk), dim3(1024), 0, st, w.nbk,
                       (uint32_t)(TPB * 16 + 1), 0xFFFFFFFFu, w.start, w.tot, w.ids, p1.dkeys_a,
                       (uint32_t *)gaussian_ids_sorted, w.ka, w.va, w.kb, w.vb, w.fail, sdev,
                       (uint32_t)cap);
    return check_launch("bin_emit");
  }
  const size_t need2 = carve_ts(nullptr, cap, T, num_points).bytes;
  if (workspace1_bytes < p1.bytes || workspace2_bytes < need2) {
    set_error("bin_emit: workspaces %zu/%zu < %zu/%zu bytes", workspace1_bytes,
              workspace2_bytes, p1.bytes, need2);
    return 1;
  }
  if (num_points == 0 || (phase != EMIT_HEAD && phase != EMIT_SPEC && num_intersects == 0)) {
    if (tail)
      note(hipMemsetAsync(tile_bins, 0, (size_t)T * 2 * sizeof(int32_t), st), "hipMemsetAsync");
    return check_launch("bin_emit");
  }
  // the tile sort: HEAD = the emission at the capacity (nothing when the device's I exceeds
  // it), TAIL = the sort and table over I (EMIT_SPEC: I on the device, launched at the capacity)
  ts_launch(num_points, p1, workspace2, gaussian_ids_sorted, tile_bins, tile_bounds_x,
            tile_bounds_y, cap, phase == EMIT_SPEC ? cap : num_intersects, nullptr, 0u, head,
            tail, phase == EMIT_SPEC ? p1.dcount : nullptr, st);
  return check_launch("bin_emit");
}

extern "C" int gsplat_bin_emit(int num_points, int64_t num_intersects, int tile_bounds_x,
                               int tile_bounds_y, int32_t *gaussian_ids_sorted,
                               int32_t *tile_bins, const void *workspace1,
                               size_t workspace1_bytes, void *workspace2,
                               size_t workspace2_bytes, void *stream) {
  return bin_emit_impl(num_points, num_intersects, num_intersects, tile_bounds_x, tile_bounds_y,
                       gaussian_ids_sorted, tile_bins, workspace1, workspace1_bytes, workspace2,
                       workspace2_bytes, stream, EMIT_ALL);
}

extern "C" int gsplat_bin_emit_prelaunch(int num_points, int64_t capacity, int tile_bounds_x,
                                         int tile_bounds_y, int32_t *tile_bins,
                                         const void *workspace1, size_t workspace1_bytes,
                                         void *workspace2, size_t workspace2_bytes,
                                         void *stream) {
  return bin_emit_impl(num_points, 0, capacity, tile_bounds_x, tile_bounds_y, nullptr, tile_bins,
                       workspace1, workspace1_bytes, workspace2, workspace2_bytes, stream,
                       EMIT_HEAD);
}

extern "C" int gsplat_bin_emit_finish(int num_points, int64_t num_intersects, int64_t capacity,
                                      int tile_bounds_x, int tile_bounds_y,
                                      int32_t *gaussian_ids_sorted, int32_t *tile_bins,
                                      const void *workspace1, size_t workspace1_bytes,
                                      void *workspace2, size_t workspace2_bytes, void *stream) {
  return bin_emit_impl(num_points, num_intersects, capacity, tile_bounds_x, tile_bounds_y,
                       gaussian_ids_sorted, tile_bins, workspace1, workspace1_bytes, workspace2,
                       workspace2_bytes, stream, EMIT_TAIL);
}

// The tile sort launched at a capacity before the host knows I (the device count decides;
// I > capacity leaves the table cleared and the ids unwritten, and the caller re-bins).  Returns
// 2 without launching anything where the scheme needs I on the host (tile buckets): use
// prelaunch / finish there.
extern "C" int gsplat_bin_emit_speculative(int num_points, int64_t capacity, int tile_bounds_x,
                                           int tile_bounds_y, int32_t *gaussian_ids_sorted,
                                           int32_t *tile_bins, const void *workspace1,
                                           size_t workspace1_bytes, void *workspace2,
                                           size_t workspace2_bytes, void *stream) {
  const long long T = (long long)tile_bounds_x * tile_bounds_y;
  if (num_points > 0 && T > 0 && capacity > 0 &&
      use_bucket(num_points, T))
    return 2;
  if (capacity <= 0) {
    set_error("bin_emit_speculative: capacity must be positive");
    return 1;
  }
  return bin_emit_impl(num_points, 0, capacity, tile_bounds_x, tile_bounds_y,
                       gaussian_ids_sorted, tile_bins, workspace1, workspace1_bytes, workspace2,
                       workspace2_bytes, stream, EMIT_SPEC);
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
  return 2 * kk + 2 * vv + radix_ws_bytes(num_items, 0, 64);
}

extern "C" int gsplat_sort_isect_pairs(int64_t num_items, int key_bits, const int64_t *keys_in,
                                       const int32_t *vals_in, int64_t *keys_out,
                                       int32_t *vals_out, void *workspace,
                                       size_t workspace_bytes, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (num_items < 0 || num_items > 0x3FFFFFFFLL || key_bits < 0 || key_bits > 64) {
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
  if (num_rows > 0)
    note(hipMemsetAsync(tile_bins, 0, (size_t)num_rows * 2 * sizeof(int32_t), st),
         "hipMemsetAsync");
  if (num_intersects == 0) return check_launch("get_tile_bin_edges");
  hipLaunchKernelGGL((bin_edges_kernel<uint64_t, 32>), dim3(cdiv(num_intersects, TPB)), dim3(TPB),
                     0, st, (long long)num_intersects, (const uint64_t *)isect_ids_sorted,
                     tile_bins, (long long)num_rows);
  return check_launch("get_tile_bin_edges");
}
