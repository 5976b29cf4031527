// exchange_layout.h -- the data-parallel view exchange's sparse record.
//
// One rank's view record when only the visible Gaussians' colour gradients travel, in floats
// (the gathered buffer is fp32; integer fields are stored bit for bit), W = ceil(N / 64):
//   [0, 3)                 camera centre
//   [3]                    visible count (uint32 bits)
//   [4, 4 + 2W)            visibility masks: uint64 word w, bit b <=> radii[64 w + b] > 0
//   [4 + 2W, 4 + 3W)       uint32 exclusive prefix of the masks' popcounts
//   [4 + 3W, 4 + 3W + 3C)  v_colors [count, 3] of the visible Gaussians in index order
//                          (C >= count: the capacity all ranks agreed on)
// Gaussian i of the record is present iff its mask bit is set, at row
// prefix[i / 64] + popcount(mask[i / 64] & ((1 << (i % 64)) - 1)).
#pragma once

namespace gs {

constexpr int XS_HDR = 4;
constexpr int XS_MAX_VIEWS = 64;  // records per gsplat_compute_sh_backward_view_table call

__host__ __device__ inline long long xs_words(long long n) { return (n + 63) >> 6; }
__host__ __device__ inline long long xs_values_at(long long n) { return XS_HDR + 3 * xs_words(n); }

// The records of one multi-view SH backward: cap[r] < 0 -> rec[r] is a dense record
// (v_colors [3N] | camera centre [3] | pad), else a sparse record of capacity cap[r].
struct ViewTable {
  const float *rec[XS_MAX_VIEWS];
  long long cap[XS_MAX_VIEWS];
};

}  // namespace gs
