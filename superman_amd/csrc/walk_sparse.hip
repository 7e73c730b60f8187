// walk_sparse.hip — SpaRyser walk for gfx950 (prefix-blocked rows).
//
// Replaces kernel_xshared_coalescing_mshared_sparse (reference
// gpu_exact_sparse.cu:455-552; fp64 form revised_perman/gpu_exact_sparse.cu).
// The reference updates only the CSC rows of the flipped column and keeps the
// product incrementally (prod /= x_old; x += s*v; prod *= x_new, with a
// zero counter).  On gfx950 an fp64 divide is a ~10-instruction sequence, so
// this kernel exploits sparsity structurally instead:
//   * rows are ordered by the first walk column that touches them
//     (host, engine.cpp make_plan), so the rows touched by walk columns
//     0..k are the prefix [0, R_k);
//   * X is kept in 8-row blocks with suffix products U[b] = prod_{rows >= 8b};
//   * a step flipping walk column k updates and re-multiplies only the
//     nblk[k] = ceil(R_k / 8) leading blocks; U[nblk[k]] is still valid.
// With SortOrder/SkipOrder the hot low columns touch few rows, so the average
// step costs a fraction of the dense 2n ops.  Zero rows need no special case:
// a zero x_j simply makes the product 0 (the reference's zero_num logic
// computes the same term).
//
// Chunk end at the first state (round 5): a lane-uniform row that no walk
// column touches keeps its value for the whole wave-chunk (x0 plus the chunk
// bits' columns); when one of those rows (WalkParams::umask, set by the host
// to exactly them for this kernel) is exactly zero, every term of the chunk is
// an exact zero and the chunk's part is +0 without walking it — the segmented
// walk's chunk skip in the ahead-of-time kernel (integer matrices: the -o
// leaves of dwt_59 end ~64 % of their chunks there).  The oracle's mirror and
// the host twin end the same chunks.
#include "walk_common.hpp"
#include "walk_zero.hpp"
#include "walk_batch.hpp"
#include "kernels.hpp"

namespace sup {

template <int N>
__global__ __launch_bounds__(kBlock) void walk_sparse(WalkParams p) {
  constexpr int NP = pad8(N);
  constexpr int NB = Blocks<N>::NB;
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * NP * 8u;
  const int nb0 = nb_of(p, 0);

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {
    double keep = 0.0;
    for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {
      const uint64_t a = (uint64_t)g * p.group + j;
      if (a >= p.chunk_count) break;
      const uint64_t ga = p.chunk_begin + a;
      double x[N];
      chunk_start<N>(x, p, ga, lane);
      if (zero_rows<N>(x) & SUP_KARG(umask)) {  // chunk end: every term an exact zero
        keep = (lane == j) ? 0.0 : keep;
        continue;
      }
      double U[NB + 1];
      suffix_all<N>(x, U);
      double acc = U[0];
      uint32_t t = 1;
      for (; t + 1 < T; t += 2) {
        // re-materialise nb0 in an SGPR every iteration: hoisted "nb0 > B"
        // masks would be spilled to VGPR lanes and cost v_readlane (VALU) per step
        int nbo = nb0;
        asm volatile("" : "+s"(nbo));
        sparse_step<N>(x, U, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u), nbo);
        acc -= U[0];
        const uint32_t u = t + 1;
        const uint32_t k = (uint32_t)__builtin_ctz(u);
        const uint32_t neg = (u >> (k + 1)) & 1u;
        sparse_step<N>(x, U, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u), nb_of(p, k));
        acc += U[0];
      }
      if (t < T) {
        sparse_step<N>(x, U, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u), nb0);
        acc -= U[0];
      }
      if (((uint32_t)ga ^ lane_par) & 1u) acc = -acc;
      const double part = wave_sum(lane_valid ? acc : 0.0);
      keep = (lane == j) ? part : keep;
    }
    chunk_store((uint64_t)g * p.group, (uint32_t)p.group, keep, 0u);
  }
}

// One wave-chunk `ga` of the prefix-blocked walk: the lane's signed sum
// (parity of the chunk and lane applied), the batched kernel's copy of the
// one-leaf kernel's chunk body (same operations in the same order: the same bits;
// kept apart so the one-leaf kernel's code is untouched).
template <int N>
__device__ __forceinline__ double sparse_chunk(const WalkParams& p, uint64_t ga, uint32_t lane, uint32_t lane_par,
                                               uint32_t T, uint32_t offL, int nb0, uint64_t ends) {
  constexpr int NP = pad8(N);
  constexpr int NB = Blocks<N>::NB;
  double x[N];
  chunk_start<N>(x, p, ga, lane);
  if (zero_rows<N>(x) & ends) return 0.0;  // chunk end (see walk_sparse): every lane's part +0
  double U[NB + 1];
  suffix_all<N>(x, U);
  double acc = U[0];
  uint32_t t = 1;
  for (; t + 1 < T; t += 2) {
    // re-materialise nb0 in an SGPR every iteration: hoisted "nb0 > B"
    // masks would be spilled to VGPR lanes and cost v_readlane (VALU) per step
    int nbo = nb0;
    asm volatile("" : "+s"(nbo));
    sparse_step<N>(x, U, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u), nbo);
    acc -= U[0];
    const uint32_t u = t + 1;
    const uint32_t k = (uint32_t)__builtin_ctz(u);
    const uint32_t neg = (u >> (k + 1)) & 1u;
    sparse_step<N>(x, U, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u), nb_of(p, k));
    acc += U[0];
  }
  if (t < T) {
    sparse_step<N>(x, U, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u), nb0);
    acc -= U[0];
  }
  if (((uint32_t)ga ^ lane_par) & 1u) acc = -acc;
  return acc;
}

// A batch of leaves (walk_batch.hpp): chunk a of the launch is chunk
// a mod 2^h of leaf a >> h, with that leaf's tables; a group of chunks never
// spans two leaves (groups are powers of two <= 2^h).
template <int N>
__global__ __launch_bounds__(kBlock) void walk_sparse_batch(WalkParams p, LeafBatch b) {
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * pad8(N) * 8u;
  // a batch holds fewer than 2^32 chunks (run_range_batch): 32-bit indices
  const uint32_t count = (uint32_t)p.chunk_count, group = (uint32_t)p.group;

  for (uint32_t g = next_chunk(p.counter); g * group < count; g = next_chunk(p.counter)) {
    const uint32_t a0 = g * group;
    typedef const __attribute__((address_space(4))) LeafDesc cdesc;
    cdesc* dp = (cdesc*)b.leaves + (a0 >> b.leaf_bits);  // scalar loads: the leaf is wave-uniform
    // only the fields the chunk walk reads (chunk_start: x0, cols, L, m; the step: cols, nblk)
    WalkParams q{};
    q.cols = dp->cols, q.x0 = dp->x0, q.nb_lo = dp->nb_lo, q.nb_hi = dp->nb_hi, q.L = p.L, q.m = p.m;
    const int nb0 = nb_of(q, 0);
    const uint32_t c0 = a0 & ((1u << b.leaf_bits) - 1u);
    double keep = 0.0;
    for (uint32_t j = 0; j < group; ++j) {
      if (a0 + j >= count) break;
      const double acc = sparse_chunk<N>(q, c0 + j, lane, lane_par, T, offL, nb0, dp->ends);
      const double part = wave_sum(lane_valid ? acc : 0.0);
      keep = (lane == j) ? part : keep;
    }
    if (lane < group && a0 + lane < count) p.chunk_out[a0 + lane] = keep;
  }
}

template <int N, int HI>
static hipError_t launch_rec(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_sparse<N>, dim3(grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_rec<N + 1, HI>(n, p, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_rec(int n, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_sparse<N>, kBlock, 0);
  if constexpr (N < HI) return occ_rec<N + 1, HI>(n, blocks_per_cu);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t launch_batch_rec(int n, const WalkParams& p, const LeafBatch& b, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_sparse_batch<N>, dim3(grid), dim3(kBlock), 0, s, p, b);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_batch_rec<N + 1, HI>(n, p, b, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_batch_rec(int n, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_sparse_batch<N>, kBlock, 0);
  if constexpr (N < HI) return occ_batch_rec<N + 1, HI>(n, blocks_per_cu);
  return hipErrorInvalidValue;
}

#define SUP_CAT2(a, b) a##b
#define SUP_CAT(a, b) SUP_CAT2(a, b)

hipError_t SUP_CAT(launch_sparse_, SUP_N_LO)(int n, const WalkParams& p, int grid, hipStream_t s) {
  return launch_rec<SUP_N_LO, SUP_N_HI>(n, p, grid, s);
}
hipError_t SUP_CAT(occupancy_sparse_, SUP_N_LO)(int n, int* blocks_per_cu) {
  return occ_rec<SUP_N_LO, SUP_N_HI>(n, blocks_per_cu);
}

hipError_t SUP_CAT(launch_batch_sparse_, SUP_N_LO)(int n, const WalkParams& p, const LeafBatch& b, int grid,
                                                  hipStream_t s) {
  return launch_batch_rec<SUP_N_LO, SUP_N_HI>(n, p, b, grid, s);
}
hipError_t SUP_CAT(occupancy_batch_sparse_, SUP_N_LO)(int n, int* blocks_per_cu) {
  return occ_batch_rec<SUP_N_LO, SUP_N_HI>(n, blocks_per_cu);
}

}  // namespace sup
