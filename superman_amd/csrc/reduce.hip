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

__global__ __launch_bounds__(kBlock) void pairwise64_pass(const double* __restrict__ in, uint64_t count,
                                                          double* __restrict__ out, uint64_t groups,
                                                          unsigned int* reset, unsigned int* flag, unsigned seq) {
  const uint64_t g = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (reset && blockIdx.x == 0 && threadIdx.x == 0) *reset = 0u;  // the walk before this pass is done with it
  if (g >= groups) return;  // whole wave exits together (g is wave-uniform)
  const uint64_t i = g * 64u + lane;
  const double v = (i < count) ? in[i] : 0.0;
  const double s = wave_sum(v);
  if (lane == 0) {
    out[g] = s;
    if (flag) {  // the last pass (one group): the call's result, then its sequence number
      __threadfence_system();
      __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// One 64-way pass over each of nseg segments of `count` values: group g of
// segment i reads that segment's values [64 g, 64 g + 64) (zero past its
// end), the groups of one call to pairwise64_pass on the segment alone.
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

// Two 64-way levels in one launch: block b folds level-1 groups
// [64 b, 64 b + 64) (each group = 64 inputs, zero past `count`, folded by one
// wave as pairwise64_pass folds it) and then those 64 group sums (zero past
// the last group) as the next pairwise64_pass would: out[b] is bit-identical
// to two consecutive pairwise64_pass launches (round 4: half the launches).
__global__ __launch_bounds__(kBlock) void pairwise4096_pass(const double* __restrict__ in, uint64_t count,
                                                            double* __restrict__ out, uint64_t groups1,
                                                            unsigned int* reset, unsigned int* flag, unsigned seq) {
  __shared__ double g1[64];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  if (reset && blockIdx.x == 0 && threadIdx.x == 0) *reset = 0u;
  const uint64_t base = (uint64_t)blockIdx.x * 64u;
  for (uint32_t k = w; k < 64u; k += kWavesPerBlock) {
    const uint64_t g = base + k;  // level-1 group
    double v = 0.0;
    if (g < groups1) {
      const uint64_t i = g * 64u + lane;
      v = wave_sum((i < count) ? in[i] : 0.0);
    }
    if (lane == 0) g1[k] = v;
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
  while (count > 1) {
    const uint64_t groups = (count + 63) / 64;
    if (groups > 1) {  // two levels at once
      const uint64_t groups2 = (groups + 63) / 64;
      double* target = (groups2 == 1) ? out : dst;
      hipLaunchKernelGGL(pairwise4096_pass, dim3((unsigned)groups2), dim3(kBlock), 0, s, src, count, target, groups,
                         reset, groups2 == 1 ? flag : nullptr, seq);
      reset = nullptr;
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      src = target;
      dst = target + groups2;
      count = groups2;
      continue;
    }
    const uint64_t blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
    double* target = (groups == 1) ? out : dst;
    hipLaunchKernelGGL(pairwise64_pass, dim3((unsigned)blocks), dim3(kBlock), 0, s, src, count, target, groups, reset,
                       groups == 1 ? flag : nullptr, seq);
    reset = nullptr;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    src = target;
    dst = target + groups;
    count = groups;
  }
  return hipSuccess;
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
