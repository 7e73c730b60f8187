// approx.hpp — host-visible interface of the estimator kernels (approx.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sup {

// One launch processes sample blocks [block0, block0 + nblocks); block b holds
// samples 64·b .. 64·b + 63 (one per lane of the wave that takes it).
struct ApproxParams {
  const uint64_t* rowpat;  // n x W words: row r's nonzero columns
  const uint64_t* colpat;  // n x W words: column c's nonzero rows
  double* part;            // 3 x nblocks: per-block sum, sum of squares, zero count
  float* scratch;          // scaling only: d_r then d_c, each n x lanes_total floats
  unsigned* counter;       // dynamic block queue (zeroed before the launch)
  uint64_t seed;
  uint64_t block0;
  uint64_t nblocks;
  int n;
  int method;  // 0 Rasmussen, 1 scaling
  int intervals;
  int times;
  uint32_t lanes_total;  // grid x 256 (scratch stride)
  uint32_t pad_;
};

// words: 1, 2, 4, 8 or 16 (n <= 64 * words).
hipError_t launch_approx(int words, const ApproxParams& p, int grid, hipStream_t s);
hipError_t approx_occupancy(int words, int method, int* blocks_per_cu);
// Cooperative form (one wave per sample, factors in LDS; same bits).
hipError_t launch_approx_coop(int words, const ApproxParams& p, int grid, hipStream_t s);
hipError_t approx_coop_occupancy(int words, int method, int n, int* blocks_per_cu);

}  // namespace sup
