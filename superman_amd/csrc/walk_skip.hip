// walk_skip.hip — SkipPer walk for gfx950 (wave-uniform zero-row skipping).
//
// Replaces kernel_xshared_coalescing_mshared_skipper (reference
// gpu_exact_sparse.cu:555-670; CPU form revised_perman/cpu_algos.hpp:1035-1213).
// The reference lets every GPU thread jump independently: when x_r == 0 for the
// last zero row r, the term stays 0 until a column of row r flips, so it jumps
// i to the next toggle of any such column (gpu_exact_sparse.cu:648-666).
// Independent per-thread jumps diverge on a 64-wide SIMD.  Here the jump is
// taken by the whole wave, and only on rows whose value is the same on every
// lane ("lane-uniform" rows: rows no lane column touches — SkipOrder puts the
// sparsest columns on the lane bits, so most rows qualify):
//   * a step's products are checked with one ballot; only if all 64 lanes are
//     zero are the lane-uniform rows scanned for an exact zero;
//   * the wave jumps to the LATEST next-toggle over all zero uniform rows
//     (the product is zero until every one of them has changed), which is at
//     least the reference's jump (it uses only the last zero row);
//   * skipped terms are exactly zero (x_r stays exactly 0 until a column of
//     row r flips), so the sum is unchanged.
// Rows are prefix-blocked exactly as in walk_sparse.hip.
#include "walk_common.hpp"
#include "kernels.hpp"

namespace sup {

// Next walk index t' > t at which walk bit k toggles (ctz(t') == k).
__device__ __forceinline__ uint32_t next_toggle(uint32_t t, uint32_t k) {
  uint32_t c = ((t >> (k + 1)) << (k + 1)) + (1u << k);
  if (c <= t) c += 2u << k;
  return c;
}

// x[rows of blocks < nb] += col (jump path: adds only, products refreshed once)
template <int N, int B>
__device__ __forceinline__ void add_nest(double (&x)[N], cdbl* col, int nb) {
  if constexpr (B < Blocks<N>::NB) {
    if (nb > B) {
#pragma unroll
      for (int j = 8 * B; j < 8 * B + 8 && j < N; ++j) x[j] += col[j];
      add_nest<N, B + 1>(x, col, nb);
    }
  }
}

template <int N>
__global__ __launch_bounds__(kBlock) void walk_skip(WalkParams p) {
  constexpr int NP = pad8(N);
  constexpr int NB = Blocks<N>::NB;
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const uint32_t offL = 2u * (uint32_t)p.L * NP * 8u;
  const uint64_t umask = p.umask;  // lane-uniform rows

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {
    double keep = 0.0;
    uint32_t vkeep = 0;
    for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {
      const uint64_t a = (uint64_t)g * p.group + j;
      if (a >= p.chunk_count) break;
      const uint64_t ga = p.chunk_begin + a;
      double x[N];
      chunk_start<N>(x, p, ga, lane);
      double U[NB + 1];
      suffix_all<N>(x, U);
      double acc = 0.0;
      uint32_t visited = 0;
      uint32_t t = 0;
      // Zero check after visiting state t (X valid for t, term added): if
      // every lane's term is zero and some lane-uniform row is exactly zero,
      // returns the index to continue from (X moved there), else t + 1 with
      // X untouched (the caller takes the ordinary single-bit step).
      auto jump = [&](uint32_t t) -> uint32_t {
        // v_cmp straight into an SGPR mask per row (no VGPR temporaries);
        // lane-uniform rows hold the same value on every lane, so lane 0 decides
        uint64_t zm = 0;
#pragma unroll
        for (int r = 0; r < N; ++r) zm |= (__builtin_amdgcn_ballot_w64(x[r] == 0.0) & 1ull) << r;
        zm &= umask;
        if (!zm) return t + 1;
        // each zero row r stays zero until one of its walk columns toggles (or
        // for the rest of the chunk if it has none); the product is zero until
        // the last of those toggles
        uint32_t target = t + 1;
        while (zm) {
          const uint32_t r = (uint32_t)__builtin_ctzll(zm);
          zm &= zm - 1;
          uint64_t mm = ((const __attribute__((address_space(4))) uint64_t*)p.rowmask)[r];
          uint32_t tr = T;
          while (mm) {
            const uint32_t k = (uint32_t)__builtin_ctzll(mm);
            mm &= mm - 1;
            const uint32_t c = next_toggle(t, k);
            tr = c < tr ? c : tr;
          }
          target = tr > target ? tr : target;
        }
        if (target == t + 1 || target >= T) return target;
        // Gray move t -> target: add the differing walk columns in ascending
        // bit order (each to its nblk leading blocks), then refresh all suffix
        // products once.  Bit-identical to one sparse_step per bit: block b's
        // x is final after the last bit with nblk > b, and that step formed
        // U[b] from it and the final U[b+1] — the same expression suffix_all
        // evaluates on the final x.
        const uint32_t gn = target ^ (target >> 1);
        uint32_t diff = (t ^ (t >> 1)) ^ gn;
        do {
          const uint32_t k = (uint32_t)__builtin_ctz(diff);
          diff &= diff - 1;
          const uint32_t neg = ((gn >> k) & 1u) ^ 1u;
          add_nest<N, 0>(x, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u), nb_of(p, k));
        } while (diff);
        suffix_all<N>(x, U);
        return target | 0x80000000u;  // flag: X already moved
      };
      for (;;) {
        // visit state t.  acc +/- term as one fma with an exact +-1 factor
        // (bit-identical to the add/sub, no per-lane select)
        ++visited;
        acc = __builtin_fma((t & 1u) ? -1.0 : 1.0, U[0], acc);
        if (__builtin_amdgcn_ballot_w64(U[0] != 0.0) == 0) {
          const uint32_t nx = jump(t);
          if (nx & 0x80000000u) {
            t = nx & 0x7fffffffu;
            continue;
          }
          if (nx >= T) break;
        }
        if (++t >= T) break;
        // ordinary single-bit Gray step to t
        const uint32_t k = (uint32_t)__builtin_ctz(t);
        const uint32_t neg = (t >> (k + 1)) & 1u;
        sparse_step<N>(x, U, opaque_c(p.cols, offL + (2u * k + neg) * NP * 8u), nb_of(p, k));
      }
      if (((uint32_t)ga ^ lane_par) & 1u) acc = -acc;
      const double part = wave_sum(lane_valid ? acc : 0.0);
      keep = (lane == j) ? part : keep;
      vkeep = (lane == j) ? visited : vkeep;
    }
    const uint64_t a = (uint64_t)g * p.group + lane;
    if (lane < (uint32_t)p.group && a < p.chunk_count) {
      p.chunk_out[a] = keep;
      if (p.visited) p.visited[a] = vkeep;
    }
  }
}

template <int N, int HI>
static hipError_t launch_rec(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n == N) {
    hipLaunchKernelGGL(walk_skip<N>, dim3(grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_rec<N + 1, HI>(n, p, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_rec(int n, int* blocks_per_cu) {
  if (n == N) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, walk_skip<N>, kBlock, 0);
  if constexpr (N < HI) return occ_rec<N + 1, HI>(n, blocks_per_cu);
  return hipErrorInvalidValue;
}

#define SUP_CAT2(a, b) a##b
#define SUP_CAT(a, b) SUP_CAT2(a, b)

hipError_t SUP_CAT(launch_skip_, SUP_N_LO)(int n, const WalkParams& p, int grid, hipStream_t s) {
  return launch_rec<SUP_N_LO, SUP_N_HI>(n, p, grid, s);
}
hipError_t SUP_CAT(occupancy_skip_, SUP_N_LO)(int n, int* blocks_per_cu) {
  return occ_rec<SUP_N_LO, SUP_N_HI>(n, blocks_per_cu);
}

}  // namespace sup
