// walk_dd.hip — the dense Ryser / Gray-code walk in double-double for gfx950:
// the MI355X counterpart of the reference's quad-precision calculation
// (revised_perman/main.cpp:141-142, `-q`: parallel_perman64<__float128,S>,
// cpu_algos.hpp:761-873, a CPU-only OpenMP loop).
//
// Enumeration, lane layout and wave-chunk queue are walk_dense.hip's
// (walk_common.hpp); every value of the walk is a double-double (dd.hpp):
//   x_j(S) = x0_j + sum_{c in S} a_jc   (dd_add_d, the column as SGPR operands)
//   term   = prod_j x_j                 (4 strided dd partial products)
//   acc   += (-1)^t term                (dd_add)
// x0 comes from the host in double-double (the Nijenhuis-Wilf start vector,
// exact up to 2^-106), so the walk carries ~106 bits where the fp64 walks carry
// 53.  Per Gray step and lane: 9n + 7(n-1) + 20 fp64 VALU ops (~8x the fp64
// walk).  Each wave-chunk's partial leaves as (hi, lo); the host adds the
// partials in a fixed pairwise order (quad.cpp), and quad.cpp's host twin runs
// the same dd.hpp operations in the same order: results are bit-identical on
// the GPU, on any device count and on host threads.
// Chunk ends (round 5, walk_sparse.hip's check): a lane-uniform row that no
// walk column touches (WalkParams::umask; quad.cpp orders the columns to leave
// many) and is exactly zero at a chunk's first state makes every term of the
// chunk zero; the chunk's part is (0, 0) without walking it.
#include "dd.hpp"
#include "kernels.hpp"
#include "walk_common.hpp"
#include "walk_zero.hpp"

namespace sup {

template <int N, int LO, int HI>
__device__ __forceinline__ void dd_add_rows(dd (&x)[N], cdbl* col) {
#pragma unroll
  for (int j = LO; j < HI; ++j) x[j] = dd_add_d(x[j], col[j]);
}

// Full-column update, in two SGPR pieces above 32 rows (as add_col).
template <int N>
__device__ __forceinline__ void dd_add_col(dd (&x)[N], cdbl* col) {
  if constexpr (N <= 32) {
    dd_add_rows<N, 0, N>(x, col);
  } else {
    dd_add_rows<N, 0, 32>(x, col);
    __builtin_amdgcn_sched_barrier(0);
    dd_add_rows<N, 32, N>(x, col);
  }
}

// Four strided partial products, combined as (p0 p1)(p2 p3) — prod4's shape.
template <int N>
__device__ __forceinline__ dd dd_prod4(const dd (&x)[N]) {
  const dd one{1.0, 0.0};
  dd p0 = x[0];
  dd p1 = N > 1 ? x[1 < N ? 1 : 0] : one;
  dd p2 = N > 2 ? x[2 < N ? 2 : 0] : one;
  dd p3 = N > 3 ? x[3 < N ? 3 : 0] : one;
#pragma unroll
  for (int j = 4; j < N; j += 4) {
    p0 = dd_mul(p0, x[j]);
    if (j + 1 < N) p1 = dd_mul(p1, x[j + 1 < N ? j + 1 : 0]);
    if (j + 2 < N) p2 = dd_mul(p2, x[j + 2 < N ? j + 2 : 0]);
    if (j + 3 < N) p3 = dd_mul(p3, x[j + 3 < N ? j + 3 : 0]);
  }
  if (N == 1) return p0;
  if (N == 2) return dd_mul(p0, p1);
  if (N == 3) return dd_mul(dd_mul(p0, p1), p2);
  return dd_mul(dd_mul(p0, p1), dd_mul(p2, p3));
}

// 64-lane pairwise dd sum (ascending xor offsets; dd_add is commutative, so
// every lane ends with the same value).
__device__ __forceinline__ dd dd_wave_sum(dd v) {
#pragma unroll
  for (int off = 1; off <= 32; off <<= 1) {
    const dd o{__shfl_xor(v.hi, off, 64), __shfl_xor(v.lo, off, 64)};
    v = dd_add(v, o);
  }
  return v;
}

// p.x0: 2 NP doubles (hi block, then lo block); p.chunk_out: 2 doubles per
// wave-chunk (hi, lo).
// Occupancy: 4n VGPRs hold x.  Up to n = 40 the kernel is asked for 2 waves
// per SIMD (256 VGPRs): without the request LLVM allocates 266-282 VGPRs at
// n = 26-29 and 258 at n = 40, i.e. 1 wave; with it 173-191 and 256 (2 spilled
// VGPRs at n = 40).  Above 40 the request would spill 8-580 VGPRs: 1 wave.
template <int N>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(N <= 40 ? 2 : 1))) void walk_dd(WalkParams p) {
  constexpr int NP = pad8(N);
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * NP * 8u;  // engine bit L = walk bit 0

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {
    dd keep{0.0, 0.0};  // lane j keeps the partial of chunk g*p.group + j
    for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {
      const uint64_t a = (uint64_t)g * p.group + j;
      if (a >= p.chunk_count) break;
      const uint64_t ga = p.chunk_begin + a;
      // chunk start (chunk_start's order: x0, high bits ascending, lane bits ascending)
      dd x[N];
      {
        cdbl* x0 = opaque_c(p.x0, 0);
#pragma unroll
        for (int r = 0; r < N; ++r) x[r] = dd{x0[r], x0[NP + r]};
        uint64_t h = ga ^ (ga >> 1);
        const uint32_t hb = (uint32_t)(p.L + p.m);
        while (h) {
          const uint32_t b = (uint32_t)__builtin_ctzll(h);
          h &= h - 1;
          dd_add_col<N>(x, opaque_c(p.cols, (2u * (hb + b)) * NP * 8u));
        }
        for (int e = 0; e < p.L; ++e) {
          cdbl* col = opaque_c(p.cols, (2u * e) * NP * 8u);
          const bool on = (lane >> e) & 1u;
#pragma unroll
          for (int r = 0; r < N; ++r) x[r] = dd_add_d(x[r], on ? col[r] : 0.0);
        }
      }
      {
        double h[N];  // a normalised double-double is zero iff its high part is
#pragma unroll
        for (int r = 0; r < N; ++r) h[r] = x[r].hi;
        if (zero_rows<N>(h) & SUP_KARG(umask)) {  // chunk end: every term exactly zero
          if (lane == j) keep = dd{0.0, 0.0};
          continue;
        }
      }
      dd acc = dd_prod4<N>(x);  // t = 0
      uint32_t t = 1;
      // odd t flips walk bit 0 (term sign -), even t walk bit ctz(t) (sign +)
      for (; t + 1 < T; t += 2) {
        dd_add_col<N>(x, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u));
        acc = dd_add(acc, dd_neg(dd_prod4<N>(x)));
        const uint32_t u = t + 1;
        const uint32_t k = (uint32_t)__builtin_ctz(u);
        const uint32_t neg = (u >> (k + 1)) & 1u;
        dd_add_col<N>(x, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u));
        acc = dd_add(acc, dd_prod4<N>(x));
      }
      if (t < T) {
        dd_add_col<N>(x, opaque_c(p.cols, offL + ((t >> 1) & 1u) * NP * 8u));
        acc = dd_add(acc, dd_neg(dd_prod4<N>(x)));
      }
      if (((uint32_t)ga ^ lane_par) & 1u) acc = dd_neg(acc);
      const dd part = dd_wave_sum(lane_valid ? acc : dd{0.0, 0.0});
      if (lane == j) keep = part;
    }
    const uint64_t a = (uint64_t)g * p.group + lane;
    if (lane < (uint32_t)p.group && a < p.chunk_count) {
      p.chunk_out[2 * a] = keep.hi;
      p.chunk_out[2 * a + 1] = keep.lo;
    }
  }
}

// Prefix-blocked form (round 5; walk_sparse.hip's structure in
// double-double): rows in first-touch order over the walk columns (make_plan,
// kind kWalkSparse), x in 8-row blocks with suffix products U[b] = prod of the
// rows of blocks >= b (U[NB] = 1); flipping walk column k adds it to the
// nblk[k] leading blocks and re-forms their U top block first, block b as
// ((x0 x1)(x2 x3))((x4 x5)(x6 x7)) times U[b + 1].  quad.cpp's host twin runs
// the same operations in the same order.
template <int N, int B>
__device__ __forceinline__ dd dd_bprod8(const dd (&x)[N]) {
  const dd one{1.0, 0.0};
  auto v = [&](int i) -> dd { return (8 * B + i < N) ? x[(8 * B + i < N) ? 8 * B + i : 0] : one; };
  return dd_mul(dd_mul(dd_mul(v(0), v(1)), dd_mul(v(2), v(3))), dd_mul(dd_mul(v(4), v(5)), dd_mul(v(6), v(7))));
}

template <int N, int B>
__device__ __forceinline__ void dd_blk_step(dd (&x)[N], dd (&U)[Blocks<N>::NB + 1], cdbl* col, int nb) {
  constexpr int NB = Blocks<N>::NB;
  if constexpr (B < NB) {
    if (nb > B) {
      dd_blk_step<N, B + 1>(x, U, col, nb);  // deeper blocks first: U[B + 1] is current below
#pragma unroll
      for (int j = 8 * B; j < 8 * B + 8 && j < N; ++j) x[j] = dd_add_d(x[j], col[j]);
      U[B] = dd_mul(dd_bprod8<N, B>(x), U[B + 1]);
    }
  }
}

template <int N, int B>
__device__ __forceinline__ void dd_suffix_all(const dd (&x)[N], dd (&U)[Blocks<N>::NB + 1]) {
  if constexpr (B >= 0) {
    U[B] = dd_mul(dd_bprod8<N, B>(x), U[B + 1]);
    dd_suffix_all<N, B - 1>(x, U);
  }
}

template <int N>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(N <= 28 ? 2 : 1))) void walk_dd_blocked(
    WalkParams p) {
  constexpr int NP = pad8(N);
  constexpr int NB = Blocks<N>::NB;
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * NP * 8u;

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {
    dd keep{0.0, 0.0};
    for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {
      const uint64_t a = (uint64_t)g * p.group + j;
      if (a >= p.chunk_count) break;
      const uint64_t ga = p.chunk_begin + a;
      dd x[N];
      {
        cdbl* x0 = opaque_c(p.x0, 0);
#pragma unroll
        for (int r = 0; r < N; ++r) x[r] = dd{x0[r], x0[NP + r]};
        uint64_t h = ga ^ (ga >> 1);
        const uint32_t hb = (uint32_t)(p.L + p.m);
        while (h) {
          const uint32_t b = (uint32_t)__builtin_ctzll(h);
          h &= h - 1;
          dd_add_col<N>(x, opaque_c(p.cols, (2u * (hb + b)) * NP * 8u));
        }
        for (int e = 0; e < p.L; ++e) {
          cdbl* col = opaque_c(p.cols, (2u * e) * NP * 8u);
          const bool on = (lane >> e) & 1u;
#pragma unroll
          for (int r = 0; r < N; ++r) x[r] = dd_add_d(x[r], on ? col[r] : 0.0);
        }
      }
      {
        double h[N];
#pragma unroll
        for (int r = 0; r < N; ++r) h[r] = x[r].hi;
        if (zero_rows<N>(h) & SUP_KARG(umask)) {  // chunk end: every term exactly zero
          if (lane == j) keep = dd{0.0, 0.0};
          continue;
        }
      }
      dd U[NB + 1];
      U[NB] = dd{1.0, 0.0};
      dd_suffix_all<N, NB - 1>(x, U);
      dd acc = U[0];  // t = 0
      for (uint32_t t = 1; t < T; ++t) {
        const uint32_t k = (uint32_t)__builtin_ctz(t);
        const uint32_t neg = (t >> (k + 1)) & 1u;
        dd_blk_step<N, 0>(x, U, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u), nb_of(p, k));
        acc = dd_add(acc, (t & 1u) ? dd_neg(U[0]) : U[0]);
      }
      if (((uint32_t)ga ^ lane_par) & 1u) acc = dd_neg(acc);
      const dd part = dd_wave_sum(lane_valid ? acc : dd{0.0, 0.0});
      if (lane == j) keep = part;
    }
    const uint64_t a = (uint64_t)g * p.group + lane;
    if (lane < (uint32_t)p.group && a < p.chunk_count) {
      p.chunk_out[2 * a] = keep.hi;
      p.chunk_out[2 * a + 1] = keep.lo;
    }
  }
}

template <int N, int HI>
static hipError_t launch_rec(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_dd<N>, dim3(grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_rec<N + 1, HI>(n, p, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_rec(int n, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_dd<N>, kBlock, 0);
  if constexpr (N < HI) return occ_rec<N + 1, HI>(n, blocks_per_cu);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t launch_blocked_rec(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_dd_blocked<N>, dim3(grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_blocked_rec<N + 1, HI>(n, p, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_blocked_rec(int n, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_dd_blocked<N>, kBlock, 0);
  if constexpr (N < HI) return occ_blocked_rec<N + 1, HI>(n, blocks_per_cu);
  return hipErrorInvalidValue;
}

#define SUP_CAT2(a, b) a##b
#define SUP_CAT(a, b) SUP_CAT2(a, b)

hipError_t SUP_CAT(launch_ddblocked_, SUP_N_LO)(int n, const WalkParams& p, int grid, hipStream_t s) {
  return launch_blocked_rec<SUP_N_LO, SUP_N_HI>(n, p, grid, s);
}
hipError_t SUP_CAT(occupancy_ddblocked_, SUP_N_LO)(int n, int* blocks_per_cu) {
  return occ_blocked_rec<SUP_N_LO, SUP_N_HI>(n, blocks_per_cu);
}

hipError_t SUP_CAT(launch_dd_, SUP_N_LO)(int n, const WalkParams& p, int grid, hipStream_t s) {
  return launch_rec<SUP_N_LO, SUP_N_HI>(n, p, grid, s);
}
hipError_t SUP_CAT(occupancy_dd_, SUP_N_LO)(int n, int* blocks_per_cu) {
  return occ_rec<SUP_N_LO, SUP_N_HI>(n, blocks_per_cu);
}

}  // namespace sup
