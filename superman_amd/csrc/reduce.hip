// reduce.hip — deterministic pairwise reduction of per-wave-chunk partials,
// plus the N-range dispatch of the walk kernels.
//
// The reference sums per-thread partials on the host in thread order after a
// 2-4 MiB D2H copy per launch (gpu_exact_dense.cu:685-693).  Here the
// partials stay in HBM and are folded on the device by 64-way pairwise passes
// (one wave per 64 values, ascending-xor butterfly), so only 8 bytes leave the
// device and the result does not depend on grid size or device count.
#include "kernels.hpp"
#include "walk_common.hpp"

namespace sup {

// One 64-way pass over each of nseg segments of `count` values: group g of
// segment i reads that segment's values [64 g, 64 g + 64) (zero past its
// end), the groups of one 64-way pass over the segment alone.
__global__ __launch_bounds__(kBlock) void pairwise64_pass_seg(const double* __restrict__ in, uint64_t count,
                                                              double* __restrict__ out, uint64_t groups,
                                                              uint64_t nseg) {
  const uint64_t gg = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (gg >= groups * nseg) return;  // wave-uniform
  const uint64_t seg = gg / groups, g = gg - seg * groups;
  const uint64_t i = g * 64u + lane;
  const double v = (i < count) ? in[seg * count + i] : 0.0;
  const double s = wave_sum(v);
  if (lane == 0) out[seg * groups + g] = s;
}

// The reduction kernels run 16 waves per block and issue every load of a wave
// before its first butterfly: a pass is one memory latency, not one per group
// (round 6: config 2's 2^14 partials took 9.8 us in 4-wave blocks that folded
// 16 groups one after another, then a second launch).
constexpr int kRedBlock = 1024;
constexpr int kRedWaves = kRedBlock / 64;
// pairwise_small: up to 16 level-1 groups per wave, so one block takes
// count <= 16 * 16 * 64 = 2^14 values through every level.
constexpr int kSmallGroups = 16;
constexpr uint64_t kSmallMax = (uint64_t)kRedWaves * kSmallGroups * 64u;

// Two 64-way levels in one launch: block b folds level-1 groups
// [64 b, 64 b + 64) (each group = 64 inputs, zero past `count`, folded by one
// wave's butterfly) and then those 64 group sums (zero past the last group):
// out[b] is two consecutive 64-way levels of the tree.
__global__ __launch_bounds__(kRedBlock) void pairwise4096_pass(const double* __restrict__ in, uint64_t count,
                                                               double* __restrict__ out, uint64_t groups1,
                                                               unsigned int* reset, unsigned int* flag, unsigned seq) {
  constexpr int kPer = 64 / kRedWaves;  // level-1 groups per wave
  __shared__ double g1[64];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  if (reset && blockIdx.x == 0 && threadIdx.x == 0) *reset = 0u;
  const uint64_t base = (uint64_t)blockIdx.x * 64u;
  double v[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {  // every load first
    const uint64_t g = base + w + (uint64_t)k * kRedWaves, i = g * 64u + lane;
    v[k] = (g < groups1 && i < count) ? in[i] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const uint32_t j = w + (uint32_t)k * kRedWaves;
    const double s = (base + j < groups1) ? wave_sum(v[k]) : 0.0;
    if (lane == 0) g1[j] = s;
  }
  __syncthreads();
  if (w == 0) {
    const double s = wave_sum(g1[lane]);
    if (lane == 0) {
      out[blockIdx.x] = s;
      if (flag) {  // the last pass (one block)
        __threadfence_system();
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// Every remaining level of count <= kSmallMax values (count >= 2) in one block:
// level 1 (64-way groups, zero past `count`), then each next level of
// 64-way group sums (zero past the level's end) until one value is left —
// bit-identical to the passes launch_pairwise_reduce ran before round 6.
__global__ __launch_bounds__(kRedBlock) void pairwise_small(const double* __restrict__ in, uint64_t count,
                                                            double* __restrict__ out, unsigned int* reset,
                                                            unsigned int* flag, unsigned seq) {
  __shared__ double lv[kRedWaves * kSmallGroups];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  if (reset && threadIdx.x == 0) *reset = 0u;
  uint32_t cnt = (uint32_t)((count + 63u) / 64u);  // level-1 groups
  double v[kSmallGroups];
#pragma unroll
  for (int k = 0; k < kSmallGroups; ++k) {  // every load first
    const uint64_t i = (uint64_t)(w + (uint32_t)k * kRedWaves) * 64u + lane;
    v[k] = i < count ? in[i] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < kSmallGroups; ++k) {
    const uint32_t g = w + (uint32_t)k * kRedWaves;
    if (g < cnt) {  // wave-uniform
      const double s = wave_sum(v[k]);
      if (lane == 0) lv[g] = s;
    }
  }
  __syncthreads();
  while (cnt > 1) {  // the next levels: at most 256 -> 4 -> 1 (block-uniform)
    const uint32_t groups = (cnt + 63u) / 64u;
    double s = 0.0;
    if (w < groups) {
      const uint32_t i = w * 64u + lane;
      s = wave_sum(i < cnt ? lv[i] : 0.0);
    }
    __syncthreads();  // every read of this level before any write
    if (w < groups && lane == 0) lv[w] = s;
    __syncthreads();
    cnt = groups;
  }
  if (threadIdx.x == 0) {
    out[0] = lv[0];
    if (flag) {
      __threadfence_system();
      __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

uint64_t pairwise_scratch_size(uint64_t count) {
  uint64_t total = 0;
  while (count > 1) {
    count = (count + 63) / 64;
    total += count;
  }
  return total + 1;
}

hipError_t launch_pairwise_reduce(const double* in, uint64_t count, double* scratch, double* out,
                                  hipStream_t s, unsigned int* reset_counter, unsigned int* flag, unsigned seq) {
  if (count == 0) return hipMemsetAsync(out, 0, sizeof(double), s);
  if (count == 1) return hipMemcpyAsync(out, in, sizeof(double), hipMemcpyDeviceToDevice, s);
  const double* src = in;
  double* dst = scratch;
  unsigned int* reset = reset_counter;  // zeroed by the first pass
  while (count > kSmallMax) {  // two levels per launch; leaves > 2^14 / 4096 >= 5 values
    const uint64_t groups = (count + 63) / 64, groups2 = (groups + 63) / 64;
    hipLaunchKernelGGL(pairwise4096_pass, dim3((unsigned)groups2), dim3(kRedBlock), 0, s, src, count, dst, groups,
                       reset, nullptr, seq);
    reset = nullptr;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    src = dst;
    dst += groups2;
    count = groups2;
  }
  hipLaunchKernelGGL(pairwise_small, dim3(1), dim3(kRedBlock), 0, s, src, count, out, reset, flag, seq);
  return hipGetLastError();
}

hipError_t launch_pairwise_reduce_seg(const double* in, uint64_t count, uint64_t nseg, double* scratch, double* out,
                                      hipStream_t s) {
  if (nseg == 0) return hipSuccess;
  if (count == 0) return hipMemsetAsync(out, 0, nseg * sizeof(double), s);
  if (count == 1) return hipMemcpyAsync(out, in, nseg * sizeof(double), hipMemcpyDeviceToDevice, s);
  const double* src = in;
  double* dst = scratch;
  while (count > 1) {
    const uint64_t groups = (count + 63) / 64;
    const uint64_t blocks = (groups * nseg + kWavesPerBlock - 1) / kWavesPerBlock;
    double* target = (groups == 1) ? out : dst;
    hipLaunchKernelGGL(pairwise64_pass_seg, dim3((unsigned)blocks), dim3(kBlock), 0, s, src, count, target, groups,
                       nseg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    src = target;
    dst = target + groups * nseg;
    count = groups;
  }
  return hipSuccess;
}

// Sum of `count` per-chunk visited-state counts into *out (zeroed by the
// caller): integer adds, exact in any order.  Replaces a count x 4-byte D2H
// copy summed on the host (config 5 -p8: 4 MiB, ~0.25 ms per call).
__global__ __launch_bounds__(kBlock) void sum_visited(const unsigned* __restrict__ in, uint64_t count,
                                                      unsigned long long* out) {
  __shared__ unsigned long long part[kWavesPerBlock];
  unsigned long long v = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < count; i += (uint64_t)gridDim.x * kBlock)
    v += in[i];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) t += part[w];
    atomicAdd(out, t);
  }
}

hipError_t launch_sum_visited(const unsigned* in, uint64_t count, unsigned long long* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess || count == 0) return e;
  const uint64_t blocks = std::min<uint64_t>(1024, (count + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(sum_visited, dim3((unsigned)blocks), dim3(kBlock), 0, s, in, count, out);
  return hipGetLastError();
}

#define SUP_DISPATCH(KIND, FN, ...)                 \
  if (n <= 16) return FN##_##KIND##_1(__VA_ARGS__);   \
  if (n <= 32) return FN##_##KIND##_17(__VA_ARGS__);  \
  if (n <= 48) return FN##_##KIND##_33(__VA_ARGS__);  \
  return FN##_##KIND##_49(__VA_ARGS__);

hipError_t launch_walk(WalkKind kind, int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  switch (kind) {
    case kWalkDense: { SUP_DISPATCH(dense, launch, n, p, grid, s) }
    case kWalkSparse: { SUP_DISPATCH(sparse, launch, n, p, grid, s) }
    case kWalkSkip: { SUP_DISPATCH(skip, launch, n, p, grid, s) }
    case kWalkSeg: break;  // run-time specialised: jit_launch (jit.cpp)
  }
  return hipErrorInvalidValue;
}

hipError_t walk_occupancy(WalkKind kind, int n, int* blocks_per_cu) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  switch (kind) {
    case kWalkDense: { SUP_DISPATCH(dense, occupancy, n, blocks_per_cu) }
    case kWalkSparse: { SUP_DISPATCH(sparse, occupancy, n, blocks_per_cu) }
    case kWalkSkip: { SUP_DISPATCH(skip, occupancy, n, blocks_per_cu) }
    case kWalkSeg: break;  // jit_occupancy (jit.cpp)
  }
  return hipErrorInvalidValue;
}

hipError_t launch_walk_batch(WalkKind kind, int n, const WalkParams& p, const LeafBatch& b, int grid, hipStream_t s) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  switch (kind) {
    case kWalkDense: { SUP_DISPATCH(dense, launch_batch, n, p, b, grid, s) }
    case kWalkSparse: { SUP_DISPATCH(sparse, launch_batch, n, p, b, grid, s) }
    default: break;
  }
  return hipErrorInvalidValue;
}

hipError_t walk_batch_occupancy(WalkKind kind, int n, int* blocks_per_cu) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  switch (kind) {
    case kWalkDense: { SUP_DISPATCH(dense, occupancy_batch, n, blocks_per_cu) }
    case kWalkSparse: { SUP_DISPATCH(sparse, occupancy_batch, n, blocks_per_cu) }
    default: break;
  }
  return hipErrorInvalidValue;
}

hipError_t launch_lds(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  SUP_DISPATCH(lds, launch, n, p, grid, s)
}

hipError_t lds_occupancy(int n, int m, int* blocks_per_cu) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  SUP_DISPATCH(lds, occupancy, n, m, blocks_per_cu)
}

hipError_t launch_exact(int n, int g, const WalkParams& p, const ExactParams& e, int grid, hipStream_t s) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  SUP_DISPATCH(exact, launch, n, g, p, e, grid, s)
}

hipError_t launch_dd(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  SUP_DISPATCH(dd, launch, n, p, grid, s)
}

hipError_t dd_occupancy(int n, int* blocks_per_cu) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  SUP_DISPATCH(dd, occupancy, n, blocks_per_cu)
}

hipError_t launch_dd_blocked(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  SUP_DISPATCH(ddblocked, launch, n, p, grid, s)
}

hipError_t dd_blocked_occupancy(int n, int* blocks_per_cu) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  SUP_DISPATCH(ddblocked, occupancy, n, blocks_per_cu)
}

hipError_t exact_occupancy(int n, int g, int* blocks_per_cu) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  SUP_DISPATCH(exact, occupancy, n, g, blocks_per_cu)
}

}  // namespace sup
