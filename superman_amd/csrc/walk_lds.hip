// walk_lds.hip — the north star's LDS-staged form of the dense Gray walk, kept
// as a measured alternative to walk_dense.hip.
//
// As the reference kernel_xshared_coalescing_mshared (gpu_exact_dense.cu:
// 329-399): the per-thread X vector lives in LDS in the coalesced
// thread-strided layout xs[j * kLdsBlock + t], and the walk bits' signed
// columns are staged in LDS and read as broadcasts.  Each Gray step reads,
// updates and writes back all n entries of X and forms the product on the
// way.  The arithmetic (x_j + col_j, the 4-way strided product tree of
// prod4, the alternating accumulate, the per-chunk lane sum) is walk_dense's,
// operation for operation, so the result is bit-identical to the plain dense
// walk (tests/test_gpu_parity.py) and the comparison measures only where X
// lives.  One 64-thread wave per block keeps the LDS footprint at n * 512 B +
// the columns, so ~7 blocks fit a CU's 160 KiB at n = 40.
#include "kernels.hpp"
#include "walk_common.hpp"

namespace sup {

constexpr int kLdsBlock = 64;

template <int N>
__global__ __launch_bounds__(kLdsBlock) void walk_lds(WalkParams p) {
  constexpr int NP = pad8(N);
  extern __shared__ double smem[];
  double* xs = smem;                  // [N][kLdsBlock]
  double* cs = smem + N * kLdsBlock;  // [2 m][NP]: walk bit k, sign neg at (2k + neg) NP
  const uint32_t lane = threadIdx.x;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const int ncol = 2 * p.m * NP;
  for (int i = (int)lane; i < ncol; i += kLdsBlock) cs[i] = p.cols[2 * p.L * NP + i];
  __syncthreads();

  // one Gray step: X += col (LDS read-modify-write), product as prod4
  auto step = [&](const double* col) {
    double q[4] = {1.0, 1.0, 1.0, 1.0};
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double v = xs[j * kLdsBlock + lane] + col[j];
      xs[j * kLdsBlock + lane] = v;
      q[j & 3] = (j < 4) ? v : q[j & 3] * v;
    }
    return (q[0] * q[1]) * (q[2] * q[3]);
  };

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {
    double keep = 0.0;
    for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {
      const uint64_t a = (uint64_t)g * p.group + j;
      if (a >= p.chunk_count) break;
      const uint64_t ga = p.chunk_begin + a;
      double acc;
      {
        double x[N];
        chunk_start<N>(x, p, ga, lane);
#pragma unroll
        for (int r = 0; r < N; ++r) xs[r * kLdsBlock + lane] = x[r];
        acc = prod4<N>(x);  // t = 0
      }
      uint32_t t = 1;
      for (; t + 1 < T; t += 2) {
        acc -= step(cs + ((t >> 1) & 1u) * NP);
        const uint32_t u = t + 1;
        const uint32_t k = (uint32_t)__builtin_ctz(u);
        const uint32_t neg = (u >> (k + 1)) & 1u;
        acc += step(cs + (2u * k + neg) * NP);
      }
      if (t < T) acc -= step(cs + ((t >> 1) & 1u) * NP);
      if (((uint32_t)ga ^ lane_par) & 1u) acc = -acc;
      const double part = wave_sum(lane_valid ? acc : 0.0);
      keep = (lane == j) ? part : keep;
    }
    const uint64_t a = (uint64_t)g * p.group + lane;
    if (lane < (uint32_t)p.group && a < p.chunk_count) p.chunk_out[a] = keep;
  }
}

template <int N>
static size_t lds_bytes(int m) {
  return sizeof(double) * ((size_t)N * kLdsBlock + 2 * (size_t)m * pad8(N));
}

template <int N, int HI>
static hipError_t launch_rec(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_lds<N>, dim3(grid), dim3(kLdsBlock), lds_bytes<N>(p.m), s, p);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_rec<N + 1, HI>(n, p, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_rec(int n, int m, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_lds<N>, kLdsBlock, lds_bytes<N>(m));
  if constexpr (N < HI) return occ_rec<N + 1, HI>(n, m, blocks_per_cu);
  return hipErrorInvalidValue;
}

#define SUP_CAT2(a, b) a##b
#define SUP_CAT(a, b) SUP_CAT2(a, b)

hipError_t SUP_CAT(launch_lds_, SUP_N_LO)(int n, const WalkParams& p, int grid, hipStream_t s) {
  return launch_rec<SUP_N_LO, SUP_N_HI>(n, p, grid, s);
}
hipError_t SUP_CAT(occupancy_lds_, SUP_N_LO)(int n, int m, int* blocks_per_cu) {
  return occ_rec<SUP_N_LO, SUP_N_HI>(n, m, blocks_per_cu);
}

}  // namespace sup
