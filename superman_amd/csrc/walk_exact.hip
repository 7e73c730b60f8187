// walk_exact.hip — exact permanent of an integer matrix: the dense Ryser /
// Gray-code walk in residue arithmetic, for gfx950.
//
// Same enumeration as walk_dense.hip (wave-uniform Gray walk, X in VGPRs, the
// flipped column as SGPR operands; reference kernel gpu_exact_dense.cu:329-399)
// on the doubled matrix 2A, so every row value is an integer:
//   X_j(S) = 2 x_j(S) = sum_c (+-) a_jc,   |X_j| <= rowabs_j = sum_c |a_jc|,
// held exactly in fp64.  Only the products leave the integers' range; each
// term prod_j X_j is formed modulo up to kMaxPrimes primes p < 2^42 (exact
// fp64 residue arithmetic, red() below; rows multiplied in exact groups of
// G = 1, 2 or 4 first), summed with its Gray sign, and the
// host joins the residues by CRT into the exact integer
//   T = sum_i (-1)^i prod_j X_j(gray(i)) = 2^(n-1) perm / (2 - 4(n&1)).
// The reference computes the same sum in fp64 (its -b / int path); this path
// is exact, so it equals every exact reference result bit for bit.
// Chunk ends (round 5): X holds exact integers, so a lane-uniform row that no
// walk column touches (WalkParams::umask, exact.cpp's column order chosen to
// leave many) and is exactly zero at a chunk's first state makes every term of
// the chunk zero; the chunk is not walked (walk_sparse.hip's check).
#include "kernels.hpp"
#include "walk_common.hpp"
#include "walk_zero.hpp"

namespace sup {

// t - rint(t / p) * p for |t| < 2^53: the fma is exact (the true result is a
// small integer), rint(t * pinv) may be off by one, so the result lies in
// (-1.5 p, 1.5 p) — still a residue of t.
__device__ __forceinline__ double red(double t, double p, double pinv) {
  return __builtin_fma(-__builtin_rint(t * pinv), p, t);
}

// Rows in groups of G: y_k = prod of X over group k, exact (|y_k| <= maxX^G,
// the host keeps G log2(maxX) + log2(1.5 p) < 53), formed once per step and
// shared by every prime.
template <int N, int G>
struct Groups {
  static constexpr int K = (N + G - 1) / G;
};
template <int N, int G>
__device__ __forceinline__ void group_products(const double (&x)[N], double (&y)[Groups<N, G>::K]) {
#pragma unroll
  for (int k = 0; k < Groups<N, G>::K; ++k) {
    double v = x[k * G];
#pragma unroll
    for (int i = 1; i < G; ++i)
      if (k * G + i < N) v *= x[(k * G + i < N) ? k * G + i : 0];
    y[k] = v;
  }
}

// prod_k y_k mod p as a chain r <- red(r * y_k), starting from red(y_0):
// |r| < 1.5 p, so every product is exact.
template <int K>
__device__ __forceinline__ double chain_mod(const double (&y)[K], double p, double pinv) {
  double r = red(y[0], p, pinv);
#pragma unroll
  for (int k = 1; k < K; ++k) r = red(r * y[k], p, pinv);
  return r;
}

template <int N, int G>
__global__ __launch_bounds__(kBlock) void walk_exact(WalkParams p, ExactParams e) {
  constexpr int K = Groups<N, G>::K;
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
    if (zero_rows<N>(x) & SUP_KARG(umask)) continue;  // chunk end: every term exactly zero
    double acc[kMaxPrimes], y[K];
    group_products<N, G>(x, y);
#pragma unroll
    for (int q = 0; q < kMaxPrimes; ++q)
      if (q < e.nprimes) acc[q] = chain_mod<K>(y, e.prime[q], e.pinv[q]);
    for (uint32_t t = 1; t < T; ++t) {
      const uint32_t k = (uint32_t)__builtin_ctz(t);
      const uint32_t neg = (t >> (k + 1)) & 1u;
      add_col<N>(x, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u));
      const bool odd = t & 1u;
      group_products<N, G>(x, y);
#pragma unroll
      for (int q = 0; q < kMaxPrimes; ++q)
        if (q < e.nprimes) {
          const double r = chain_mod<K>(y, e.prime[q], e.pinv[q]);
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

// Prefix-blocked form (round 5; walk_sparse.hip's structure in residues): rows
// in first-touch order over the walk columns (make_plan, kind kWalkSparse), so
// flipping walk column k changes only the nblk[k] leading 8-row blocks.  Per
// prime, R[b] = prod of the rows of blocks >= b mod p (R[NB] = 1), re-formed
// for the changed blocks only, top block first: R[b] = chain of block b's
// exact group products starting from R[b + 1].  Every value is an exact
// residue, so the sums equal the dense walk's residue for residue.
template <int N, int G>
__device__ __forceinline__ double block_chain(const double (&x)[N], int b, double r, double p, double pinv) {
  // block b's rows in groups of G (exact products), each folded into r
#pragma unroll
  for (int j0 = 0; j0 < 8; j0 += G) {
    const int r0 = 8 * b + j0;
    if (r0 < N) {
      double y = x[r0];
#pragma unroll
      for (int i = 1; i < G; ++i)
        if (r0 + i < N && j0 + i < 8) y *= x[(r0 + i < N) ? r0 + i : 0];
      r = red(r * y, p, pinv);
    }
  }
  return r;
}

template <int N, int G>
__global__ __launch_bounds__(kBlock) void walk_exact_blocked(WalkParams p, ExactParams e) {
  constexpr int NP = pad8(N);
  constexpr int NB = Blocks<N>::NB;
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * NP * 8u;

  double tot[kMaxPrimes];
#pragma unroll
  for (int q = 0; q < kMaxPrimes; ++q) tot[q] = 0.0;

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g < p.chunk_count; g = next_chunk(p.counter)) {
    const uint64_t ga = p.chunk_begin + g;
    double x[N];
    chunk_start<N>(x, p, ga, lane);
    if (zero_rows<N>(x) & SUP_KARG(umask)) continue;  // chunk end: every term exactly zero
    double R[kMaxPrimes][NB + 1], acc[kMaxPrimes];
#pragma unroll
    for (int q = 0; q < kMaxPrimes; ++q)
      if (q < e.nprimes) {
        R[q][NB] = 1.0;
#pragma unroll
        for (int b = NB - 1; b >= 0; --b) R[q][b] = block_chain<N, G>(x, b, R[q][b + 1], e.prime[q], e.pinv[q]);
        acc[q] = R[q][0];
      }
    for (uint32_t t = 1; t < T; ++t) {
      const uint32_t k = (uint32_t)__builtin_ctz(t);
      const uint32_t neg = (t >> (k + 1)) & 1u;
      const int nb = nb_of(p, k);
      cdbl* col = opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u);
#pragma unroll
      for (int b = NB - 1; b >= 0; --b)
        if (b < nb) {
#pragma unroll
          for (int j = 8 * b; j < 8 * b + 8 && j < N; ++j) x[j] += col[j];
        }
      const bool odd = t & 1u;
#pragma unroll
      for (int q = 0; q < kMaxPrimes; ++q)
        if (q < e.nprimes) {
#pragma unroll
          for (int b = NB - 1; b >= 0; --b)
            if (b < nb) R[q][b] = block_chain<N, G>(x, b, R[q][b + 1], e.prime[q], e.pinv[q]);
          acc[q] = odd ? acc[q] - R[q][0] : acc[q] + R[q][0];
          if ((t & 255u) == 0u) acc[q] = red(acc[q], e.prime[q], e.pinv[q]);
        }
    }
    const bool flip = ((uint32_t)ga ^ lane_par) & 1u;
#pragma unroll
    for (int q = 0; q < kMaxPrimes; ++q)
      if (q < e.nprimes) {
        const double a = red(acc[q], e.prime[q], e.pinv[q]);
        tot[q] = red(tot[q] + (lane_valid ? (flip ? -a : a) : 0.0), e.prime[q], e.pinv[q]);
      }
  }
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

// g = 1, 2, 4: the dense walk with groups of g; 8 + g: the prefix-blocked walk
template <int N, int HI>
static hipError_t launch_rec(int n, int g, const WalkParams& p, const ExactParams& e, int grid, hipStream_t s) {
  if (n == N) {
    switch (g) {
      case 4: hipLaunchKernelGGL((walk_exact<N, 4>), dim3(grid), dim3(kBlock), 0, s, p, e); break;
      case 2: hipLaunchKernelGGL((walk_exact<N, 2>), dim3(grid), dim3(kBlock), 0, s, p, e); break;
      case 1: hipLaunchKernelGGL((walk_exact<N, 1>), dim3(grid), dim3(kBlock), 0, s, p, e); break;
      case 12: hipLaunchKernelGGL((walk_exact_blocked<N, 4>), dim3(grid), dim3(kBlock), 0, s, p, e); break;
      case 10: hipLaunchKernelGGL((walk_exact_blocked<N, 2>), dim3(grid), dim3(kBlock), 0, s, p, e); break;
      case 9: hipLaunchKernelGGL((walk_exact_blocked<N, 1>), dim3(grid), dim3(kBlock), 0, s, p, e); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_rec<N + 1, HI>(n, g, p, e, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_rec(int n, int g, int* blocks_per_cu) {
  if (n == N) {
    switch (g) {
      case 4: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_exact<N, 4>, kBlock, 0);
      case 2: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_exact<N, 2>, kBlock, 0);
      case 1: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_exact<N, 1>, kBlock, 0);
      case 12: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_exact_blocked<N, 4>, kBlock, 0);
      case 10: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_exact_blocked<N, 2>, kBlock, 0);
      case 9: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_exact_blocked<N, 1>, kBlock, 0);
      default: return hipErrorInvalidValue;
    }
  }
  if constexpr (N < HI) return occ_rec<N + 1, HI>(n, g, blocks_per_cu);
  return hipErrorInvalidValue;
}

#define SUP_CAT2(a, b) a##b
#define SUP_CAT(a, b) SUP_CAT2(a, b)

hipError_t SUP_CAT(launch_exact_, SUP_N_LO)(int n, int g, const WalkParams& p, const ExactParams& e, int grid,
                                            hipStream_t s) {
  return launch_rec<SUP_N_LO, SUP_N_HI>(n, g, p, e, grid, s);
}
hipError_t SUP_CAT(occupancy_exact_, SUP_N_LO)(int n, int g, int* blocks_per_cu) {
  return occ_rec<SUP_N_LO, SUP_N_HI>(n, g, blocks_per_cu);
}

}  // namespace sup
