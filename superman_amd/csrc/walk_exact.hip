// walk_exact.hip — exact permanent of an integer matrix: the dense Ryser /
// Gray-code walk in residue arithmetic, for gfx950.
//
// Same enumeration as walk_dense.hip (wave-uniform Gray walk, X in VGPRs, the
// flipped column as SGPR operands; reference kernel gpu_exact_dense.cu:329-399)
// on the doubled matrix 2A, so every row value is an integer:
//   X_j(S) = 2 x_j(S) = sum_c (+-) a_jc,   |X_j| <= rowabs_j = sum_c |a_jc|,
// held exactly in fp64.  Only the products leave the integers' range; each
// term prod_j X_j is formed modulo up to kMaxPrimes primes p < 2^42 (exact
// fp64 residue arithmetic, red() below), summed with its Gray sign, and the
// host joins the residues by CRT into the exact integer
//   T = sum_i (-1)^i prod_j X_j(gray(i)) = 2^(n-1) perm / (2 - 4(n&1)).
// The reference computes the same sum in fp64 (its -b / int path); this path
// is exact, so it equals every exact reference result bit for bit.
#include "kernels.hpp"
#include "walk_common.hpp"

namespace sup {

// t - rint(t / p) * p for |t| < 2^53: the fma is exact (the true result is a
// small integer), rint(t * pinv) may be off by one, so the result lies in
// (-1.5 p, 1.5 p) — still a residue of t.
__device__ __forceinline__ double red(double t, double p, double pinv) {
  return __builtin_fma(-__builtin_rint(t * pinv), p, t);
}

// prod_j X_j mod p as a chain r <- red(r * X_j): |r| < 1.5 p and |X_j| <=
// maxX with 1.5 p maxX < 2^53 (host picks p), so every product is exact.
template <int N>
__device__ __forceinline__ double chain_mod(const double (&x)[N], double p, double pinv) {
  double r = x[0];
#pragma unroll
  for (int j = 1; j < N; ++j) r = red(r * x[j], p, pinv);
  return r;
}

template <int N>
__global__ __launch_bounds__(kBlock) void walk_exact(WalkParams p, ExactParams e) {
  constexpr int NP = pad8(N);
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * NP * 8u;  // engine bit L = walk bit 0

  double tot[kMaxPrimes];  // this lane's share of the wave's chunks, per prime
#pragma unroll
  for (int q = 0; q < kMaxPrimes; ++q) tot[q] = 0.0;

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g < p.chunk_count; g = next_chunk(p.counter)) {
    const uint64_t ga = p.chunk_begin + g;
    double x[N];
    chunk_start<N>(x, p, ga, lane);
    double acc[kMaxPrimes];
#pragma unroll
    for (int q = 0; q < kMaxPrimes; ++q)
      if (q < e.nprimes) acc[q] = chain_mod<N>(x, e.prime[q], e.pinv[q]);
    for (uint32_t t = 1; t < T; ++t) {
      const uint32_t k = (uint32_t)__builtin_ctz(t);
      const uint32_t neg = (t >> (k + 1)) & 1u;
      add_col<N>(x, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u));
      const bool odd = t & 1u;
#pragma unroll
      for (int q = 0; q < kMaxPrimes; ++q)
        if (q < e.nprimes) {
          const double r = chain_mod<N>(x, e.prime[q], e.pinv[q]);
          acc[q] = odd ? acc[q] - r : acc[q] + r;
          // |acc| grows by < 1.5 p per step: fold it every 256 steps
          if ((t & 255u) == 0u) acc[q] = red(acc[q], e.prime[q], e.pinv[q]);
        }
    }
    // subset parity = parity(gray(ga)) ^ parity(lane) ^ parity(g(t)), the
    // last folded into the alternating signs above
    const bool flip = ((uint32_t)ga ^ lane_par) & 1u;
#pragma unroll
    for (int q = 0; q < kMaxPrimes; ++q)
      if (q < e.nprimes) {
        const double a = red(acc[q], e.prime[q], e.pinv[q]);
        tot[q] = red(tot[q] + (lane_valid ? (flip ? -a : a) : 0.0), e.prime[q], e.pinv[q]);
      }
  }
  // 64 lanes, |tot| < 1.5 p each: the plain sum is exact; store it in [0, p)
  const uint32_t wave = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
#pragma unroll
  for (int q = 0; q < kMaxPrimes; ++q)
    if (q < e.nprimes) {
      double v = tot[q];
#pragma unroll
      for (int off = 1; off <= 32; off <<= 1) v += __shfl_xor(v, off, 64);
      double r = red(v, e.prime[q], e.pinv[q]);
      if (r < 0.0) r += e.prime[q];
      if (r < 0.0) r += e.prime[q];
      if (r >= e.prime[q]) r -= e.prime[q];
      if (lane == 0) e.wave_out[(uint64_t)wave * kMaxPrimes + q] = r;
    }
}

template <int N, int HI>
static hipError_t launch_rec(int n, const WalkParams& p, const ExactParams& e, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_exact<N>, dim3(grid), dim3(kBlock), 0, s, p, e);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_rec<N + 1, HI>(n, p, e, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_rec(int n, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_exact<N>, kBlock, 0);
  if constexpr (N < HI) return occ_rec<N + 1, HI>(n, blocks_per_cu);
  return hipErrorInvalidValue;
}

#define SUP_CAT2(a, b) a##b
#define SUP_CAT(a, b) SUP_CAT2(a, b)

hipError_t SUP_CAT(launch_exact_, SUP_N_LO)(int n, const WalkParams& p, const ExactParams& e, int grid,
                                            hipStream_t s) {
  return launch_rec<SUP_N_LO, SUP_N_HI>(n, p, e, grid, s);
}
hipError_t SUP_CAT(occupancy_exact_, SUP_N_LO)(int n, int* blocks_per_cu) {
  return occ_rec<SUP_N_LO, SUP_N_HI>(n, blocks_per_cu);
}

}  // namespace sup
