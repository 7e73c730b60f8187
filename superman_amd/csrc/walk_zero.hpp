// walk_zero.hpp — exact-zero row tests shared by the ahead-of-time walks that
// skip (walk_skip.hip: SkipPer's checks; walk_sparse.hip: the chunk end at a
// wave-chunk's first state).  Not part of the segmented walk's hiprtc source.
#pragma once
#include "walk_common.hpp"

namespace sup {

// Zero test of every row, one bit per row: a lane-uniform row holds the same
// value on every lane, so its ballot is 0 or all ones and bit r of it stands
// for lane 0 (rows outside the caller's lane-uniform mask are dropped by the
// caller).  Two scalar ops per row (and, or) beside the compare.
template <int N>
__device__ __forceinline__ uint64_t zero_rows(const double (&x)[N]) {
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const uint64_t b = __builtin_amdgcn_ballot_w64(x[r] == 0.0);
    if (r < 32) lo |= (uint32_t)b & (1u << (r & 31));
    else hi |= (uint32_t)(b >> 32) & (1u << (r & 31));
  }
  return ((uint64_t)hi << 32) | lo;
}

}  // namespace sup
