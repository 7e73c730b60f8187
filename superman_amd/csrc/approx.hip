// approx.hip — gfx950 kernels of the randomized permanent estimators
// (reference gpu_approximation_dense.cu:155-371,
// gpu_approximation_sparse.cu:198-453).
//
// One sample per lane, one 64-sample block per wave at a time, blocks taken
// from an atomic queue.  The per-sample code (approx_core.hpp) is integer
// bitset work — popcounts over the row patterns, a Philox draw per step — plus,
// for the scaling estimator, fp64 sums over fp32 factors kept in an HBM
// scratch laid out [index][lane] so a wave's accesses coalesce.  A block's 64
// estimates leave as three pairwise sums (value, square, zero count), written
// by block index: the result depends only on (seed, sample count), never on
// the grid, the device count or which wave took a block.
#include "approx.hpp"
#include "approx_core.hpp"
#include "walk_common.hpp"

namespace sup {

template <int W, int M>
__global__ __launch_bounds__(kBlock) void approx_blocks(ApproxParams p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gl = blockIdx.x * kBlock + threadIdx.x;
  float* dr = p.scratch ? p.scratch + gl : nullptr;
  float* dc = p.scratch ? p.scratch + (size_t)p.n * p.lanes_total + gl : nullptr;
  for (uint32_t b = next_chunk(p.counter); b < p.nblocks; b = next_chunk(p.counter)) {
    const uint64_t sample = (p.block0 + b) * 64u + lane;
    bool zero = false;
    double e;
    if constexpr (M == 0) {
      e = rasmussen_sample<W>(p.rowpat, p.n, p.seed, sample, zero);
    } else {
      e = scaling_sample<W>(p.rowpat, p.colpat, p.n, p.intervals, p.times, p.seed, sample, dr, dc, p.lanes_total,
                            zero);
    }
    const double s = wave_sum(e);
    const double q = wave_sum(e * e);
    const double z = wave_sum(zero ? 1.0 : 0.0);
    if (lane == 0) {
      p.part[b] = s;
      p.part[p.nblocks + b] = q;
      p.part[2 * p.nblocks + b] = z;
    }
  }
}

template <int W>
static hipError_t launch_w(const ApproxParams& p, int grid, hipStream_t s) {
  if (p.method == 0) hipLaunchKernelGGL((approx_blocks<W, 0>), dim3(grid), dim3(kBlock), 0, s, p);
  else hipLaunchKernelGGL((approx_blocks<W, 1>), dim3(grid), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

template <int W>
static hipError_t occ_w(int method, int* b) {
  return method == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(b, approx_blocks<W, 0>, kBlock, 0)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(b, approx_blocks<W, 1>, kBlock, 0);
}

hipError_t launch_approx(int words, const ApproxParams& p, int grid, hipStream_t s) {
  switch (words) {
    case 1: return launch_w<1>(p, grid, s);
    case 2: return launch_w<2>(p, grid, s);
    case 4: return launch_w<4>(p, grid, s);
    case 8: return launch_w<8>(p, grid, s);
    case 16: return launch_w<16>(p, grid, s);
  }
  return hipErrorInvalidValue;
}

hipError_t approx_occupancy(int words, int method, int* blocks_per_cu) {
  switch (words) {
    case 1: return occ_w<1>(method, blocks_per_cu);
    case 2: return occ_w<2>(method, blocks_per_cu);
    case 4: return occ_w<4>(method, blocks_per_cu);
    case 8: return occ_w<8>(method, blocks_per_cu);
    case 16: return occ_w<16>(method, blocks_per_cu);
  }
  return hipErrorInvalidValue;
}

}  // namespace sup
