// walk_dense.hip — dense Ryser / Gray-code walk for gfx950.
//
// Replaces kernel_xshared_coalescing_mshared (reference gpu_exact_dense.cu:329-399;
// fp64-X form revised_perman/gpu_exact_dense.cu:357-427).  Same sum,
//   sum_i (-1)^i prod_j x_j(gray(i)),  x(S) = x0 + sum_{c in S} A[:,c],
// different schedule: wave-uniform Gray walk with X in VGPRs and the flipped
// column in SGPRs (see walk_common.hpp).  Per step and lane: n v_add_f64 +
// (n-1) v_mul_f64 + 1 accumulate = 2n fp64 VALU ops, nothing else on the VALU.
//
// This file is compiled once per N range (SUP_N_LO..SUP_N_HI) so the 64
// template instances build in parallel.
#include "walk_common.hpp"
#include "walk_batch.hpp"
#include "kernels.hpp"

namespace sup {

template <int N>
__global__ __launch_bounds__(kBlock) void walk_dense(WalkParams p) {
  constexpr int NP = pad8(N);
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * NP * 8u;  // engine bit L = walk bit 0

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {
   double keep = 0.0;  // lane j keeps the partial of chunk g*p.group + j
   for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {
    const uint64_t a = (uint64_t)g * p.group + j;
    if (a >= p.chunk_count) break;
    const uint64_t ga = p.chunk_begin + a;
    double x[N];
    chunk_start<N>(x, p, ga, lane);

    double acc = prod4<N>(x);  // t = 0
    uint32_t t = 1;
    // Two steps per trip: odd t flips walk bit 0 (sign -), even t flips
    // walk bit k = ctz(t) (sign +).  neg = 1 when the bit is being cleared.
    for (; t + 1 < T; t += 2) {
      add_col<N>(x, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u));
      acc -= prod4<N>(x);
      const uint32_t u = t + 1;
      const uint32_t k = (uint32_t)__builtin_ctz(u);
      const uint32_t neg = (u >> (k + 1)) & 1u;
      add_col<N>(x, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u));
      acc += prod4<N>(x);
    }
    if (t < T) {
      add_col<N>(x, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u));
      acc -= prod4<N>(x);
    }
    // subset parity = parity(gray(ga)) ^ parity(g(t)) ^ parity(lane); the
    // g(t) part is folded into the alternating signs above.
    if (((uint32_t)ga ^ lane_par) & 1u) acc = -acc;
    const double part = wave_sum(lane_valid ? acc : 0.0);
    keep = (lane == j) ? part : keep;
   }
   // one 64-byte store per group (8 lanes x 8 B), or the fused fold
   chunk_store((uint64_t)g * p.group, (uint32_t)p.group, keep, 0u);
  }
}

// One wave-chunk `ga` of the plain walk: the lane's signed sum (parity of
// the chunk and lane applied), the batched kernel's copy of the
// one-leaf kernel's chunk body (same operations in the same order: the same bits;
// kept apart so the one-leaf kernel's code is untouched).
template <int N>
__device__ __forceinline__ double dense_chunk(const WalkParams& p, uint64_t ga, uint32_t lane, uint32_t lane_par) {
  constexpr int NP = pad8(N);
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * NP * 8u;  // engine bit L = walk bit 0
  double x[N];
  chunk_start<N>(x, p, ga, lane);

  double acc = prod4<N>(x);  // t = 0
  uint32_t t = 1;
  // Two steps per trip: odd t flips walk bit 0 (sign -), even t flips
  // walk bit k = ctz(t) (sign +).  neg = 1 when the bit is being cleared.
  for (; t + 1 < T; t += 2) {
    add_col<N>(x, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u));
    acc -= prod4<N>(x);
    const uint32_t u = t + 1;
    const uint32_t k = (uint32_t)__builtin_ctz(u);
    const uint32_t neg = (u >> (k + 1)) & 1u;
    add_col<N>(x, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u));
    acc += prod4<N>(x);
  }
  if (t < T) {
    add_col<N>(x, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u));
    acc -= prod4<N>(x);
  }
  // subset parity = parity(gray(ga)) ^ parity(g(t)) ^ parity(lane); the
  // g(t) part is folded into the alternating signs above.
  if (((uint32_t)ga ^ lane_par) & 1u) acc = -acc;
  return acc;
}

// A batch of leaves (walk_batch.hpp), as walk_sparse_batch.
template <int N>
__global__ __launch_bounds__(kBlock) void walk_dense_batch(WalkParams p, LeafBatch b) {
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint64_t cmask = (1ull << b.leaf_bits) - 1ull;

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {
    const uint64_t a0 = (uint64_t)g * p.group;
    typedef const __attribute__((address_space(4))) LeafDesc cdesc;
    cdesc* dp = (cdesc*)b.leaves + (a0 >> b.leaf_bits);  // scalar loads: the leaf is wave-uniform
    WalkParams q = p;
    q.cols = dp->cols, q.x0 = dp->x0;
    double keep = 0.0;
    for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {
      const uint64_t a = a0 + j;
      if (a >= p.chunk_count) break;
      const double acc = dense_chunk<N>(q, a & cmask, lane, lane_par);
      const double part = wave_sum(lane_valid ? acc : 0.0);
      keep = (lane == j) ? part : keep;
    }
    const uint64_t a = a0 + lane;
    if (lane < (uint32_t)p.group && a < p.chunk_count) p.chunk_out[a] = keep;
  }
}

template <int N, int HI>
static hipError_t launch_rec(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_dense<N>, dim3(grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_rec<N + 1, HI>(n, p, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_rec(int n, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_dense<N>, kBlock, 0);
  if constexpr (N < HI) return occ_rec<N + 1, HI>(n, blocks_per_cu);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t launch_batch_rec(int n, const WalkParams& p, const LeafBatch& b, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_dense_batch<N>, dim3(grid), dim3(kBlock), 0, s, p, b);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_batch_rec<N + 1, HI>(n, p, b, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_batch_rec(int n, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_dense_batch<N>, kBlock, 0);
  if constexpr (N < HI) return occ_batch_rec<N + 1, HI>(n, blocks_per_cu);
  return hipErrorInvalidValue;
}

#define SUP_CAT2(a, b) a##b
#define SUP_CAT(a, b) SUP_CAT2(a, b)

hipError_t SUP_CAT(launch_dense_, SUP_N_LO)(int n, const WalkParams& p, int grid, hipStream_t s) {
  return launch_rec<SUP_N_LO, SUP_N_HI>(n, p, grid, s);
}
hipError_t SUP_CAT(occupancy_dense_, SUP_N_LO)(int n, int* blocks_per_cu) {
  return occ_rec<SUP_N_LO, SUP_N_HI>(n, blocks_per_cu);
}

hipError_t SUP_CAT(launch_batch_dense_, SUP_N_LO)(int n, const WalkParams& p, const LeafBatch& b, int grid,
                                                 hipStream_t s) {
  return launch_batch_rec<SUP_N_LO, SUP_N_HI>(n, p, b, grid, s);
}
hipError_t SUP_CAT(occupancy_batch_dense_, SUP_N_LO)(int n, int* blocks_per_cu) {
  return occ_batch_rec<SUP_N_LO, SUP_N_HI>(n, blocks_per_cu);
}

}  // namespace sup
