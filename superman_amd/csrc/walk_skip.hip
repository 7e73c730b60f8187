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
#include <cstdlib>

#include "walk_common.hpp"
#include "walk_zero.hpp"
#include "kernels.hpp"

namespace sup {

// Next walk index t' > t at which walk bit k toggles (ctz(t') == k).
__device__ __forceinline__ uint32_t next_toggle(uint32_t t, uint32_t k) {
  uint32_t c = ((t >> (k + 1)) << (k + 1)) + (1u << k);
  if (c <= t) c += 2u << k;
  return c;
}

// x[rows of blocks < nb] += col (jump path: adds only, products re-formed once)
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

// nblk of walk bit k read from the kernel arguments where it is used (a
// scalar load beside the column's): held in SGPRs across the walk, the two
// packed words were spilled and reloaded with v_readlane on every segment.
__device__ __forceinline__ int nb_at(uint32_t k) {
  const uint64_t w = k < 16 ? SUP_KARG(nb_lo) : SUP_KARG(nb_hi);
  return (int)((w >> ((k & 15u) * 4u)) & 15u);
}

// LOW = 3 (below): the 15 steps inside an aligned 16-step segment, state
// t + S flipping walk bit k = ctz(S) with a compile-time block count (one
// block for walk bits 0-2, two for bit 3: at least each bit's own count, and
// re-forming a block a column does not touch gives the same values, so the
// sum is bit-identical) and its sign bit (t + S) >> (k + 1): the position's
// for k < 3, bit 4 of t (ng3) for k = 3.  Straight-line: no branch, no
// per-step scalar arithmetic.
template <int N, int S = 1>
__device__ __forceinline__ void seg15(double (&x)[N], double (&U)[Blocks<N>::NB + 1], const double* colw,
                                      uint32_t ng3, double& acc) {
  if constexpr (S < 16) {
    constexpr int NP = pad8(N);
    constexpr uint32_t k = (uint32_t)__builtin_ctz(S);
    constexpr int nbs = k < 3 ? 1 : 2;
    const uint32_t neg = k < 3 ? (((uint32_t)S >> (k + 1)) & 1u) : ng3;
    sparse_step_static<N, (nbs < Blocks<N>::NB ? nbs : Blocks<N>::NB)>(x, U, opaque_c(colw, (2u * k + neg) * NP * 8u));
    if constexpr (S & 1) acc -= U[0];
    else acc += U[0];
    seg15<N, S + 1>(x, U, colw, ng3, acc);
  }
}

// Round 5.  Round 4's kernel checked every visited
// state for an all-zero product and jumped from there: 56 scalar against 37
// vector instructions per visited wave-state (counters,
// profiles/r4/pmc_skip44_*.csv) — the scalar unit the four SIMDs of a CU
// share was the bound, and per-state bookkeeping was its load (the check, the
// sign, the loop's exits, the move).  A leaner per-state form of the same
// policy still measured 59 scalar instructions (profiles/r5).  This kernel
// changes the policy instead: it skips whole segments of 2^kSkipSegBits Gray
// steps (aligned), and walks the others with walk_sparse's paired loop, whose
// scalar work per step is a fraction of a checked step's:
//   * at a segment start t (and only there) with every lane's term zero, the
//     lane-uniform rows that are exactly zero and that no walk bit below
//     kSkipSegBits touches are zero for the whole segment, and until one of
//     their walk columns toggles: the wave moves to the last of those toggles
//     (a segment start).  Skipped terms are exactly zero, so the sum is the
//     per-state walk's (the skips are fewer: the simulation on config 5
//     visits 27.6 % of the states instead of 21.8 %, tools/probes/skip_sim);
//   * elsewhere the pair (walk bit 0 with its block count in an SGPR, then
//     walk bit ctz) steps and accumulates as walk_sparse does;
//   * the move adds the differing walk columns block-wise and re-forms the
//     suffix products once (bit-identical to one step per bit, see there);
//   * the arguments only the zero scan and the chunk end read are loaded
//     where they are used; U is kept out of LLVM's alloca-to-vector
//     promotion (Makefile: promoted, the jump and step paths disagreed on its
//     register layout, 8 v_mov_b64 per visited state).
// The host twin (engine_cpu.cpp) and the oracle's mirror follow the same
// segments, so results and visited counts agree bit for bit.
//
// Round 6: round 5's pair loop spent 21.1 scalar
// instructions per visited wave-state on each step's bit, sign, block count
// and column offset — the CU's one scalar unit as busy as its four SIMDs'
// VALU (issue 0.60).  The low walk bits flip in a fixed pattern, and their
// block counts are the launch's, so the walk is now specialised by form (the
// host picks the most specialised one the plan's block counts allow,
// skip_form):
//   LOW 3  the 15 steps inside an aligned 16-step segment are straight-line
//          code with compile-time block counts, offsets and signs (seg15);
//          only the step into the next segment has a run-time bit;
//   LOW 2  eight steps per iteration, walk bits 0-2 on one block;
//   LOW 1  four steps per iteration, walk bits 0-1 on one block;
//   LOW 0  four steps per iteration, every block count at run time.
// Config 5 (--jit -1, form 3): 779 -> 537 ms, scalar instructions per
// visited wave-state 21.1 -> 4.9, the same 19.8 fp64 (profiles/r6/
// probe_skip_forms.log, pmc_skip44_forms.csv; issue 0.87); every form gives
// the same bits and visited counts (tests/test_gpu_skip_forms.py).  On the
// way (profiles/r6/probe_skip_*.log): quad loop 685 ms, + one-block low bits
// 636, + octet 575, + segment 531.  Measured and dropped: an octet loop with
// run-time block counts (SGPR spills 72 -> 140, 811 ms), the whole segment
// straight-line with run-time counts (200 SGPR spills and phi copies that
// doubled the VALU, 1138 ms), block 0 kept as two half products (133 VGPRs:
// 1070 ms at 3 waves, 970 ms at 4 with scratch).
template <int N, int LOW>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void walk_skip(WalkParams p) {
  constexpr bool ONE = LOW >= 1;
  constexpr int NP = pad8(N);
  const uint32_t lane = threadIdx.x & 63u;
  const bool lane_valid = lane < (1u << p.L);
  const uint32_t lane_par = __builtin_popcount(lane) & 1u;
  const uint32_t T = 1u << p.m;
  const int nb0 = nb_of(p, 0), nb1 = nb_of(p, 1);

  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {
    double keep = 0.0;
    uint32_t vkeep = 0;
    for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {
      const uint64_t a = (uint64_t)g * p.group + j;
      if (a >= p.chunk_count) break;
      const uint64_t ga = p.chunk_begin + a;
      double x[N];
      chunk_start<N>(x, p, ga, lane);
      double U[Blocks<N>::NB + 1];
      suffix_all<N>(x, U);
      const double* colw = p.cols + 2 * p.L * NP;  // walk bit k, sign s: colw + (2k + s) NP
      double acc = U[0];  // state 0
      uint32_t visited = 1;
      uint32_t u = 1;
      // state 0 opens a segment: the zero check before its walk (T = 1: state 0 is the chunk)
      bool check = true;
      for (; T > 1;) {
        if (check && __builtin_amdgcn_ballot_w64(U[0] != 0.0) == 0) {
          // Every lane's term at the segment start t = u - 1 is zero.  A
          // lane-uniform row that is exactly zero and that no walk bit below
          // kSkipSegBits touches stays zero for the whole segment and until one of its
          // walk columns toggles (for the rest of the chunk if it has none):
          // the product is zero until the last of those toggles over all such
          // rows, a segment start.  Skipped terms are exactly zero.
          const uint32_t t = u - 1;
          uint64_t zm = zero_rows<N>(x) & SUP_KARG(umask);
          const __attribute__((address_space(4))) uint64_t* rmask =
              (const __attribute__((address_space(4))) uint64_t*)SUP_KARG(rowmask);
          uint32_t nx = t;
          while (zm) {
            const uint32_t r = (uint32_t)__builtin_ctzll(zm);
            zm &= zm - 1;
            uint64_t mm = rmask[r];
            if (mm & kSkipSegMask) continue;
            uint32_t tr = T;
            while (mm) {
              const uint32_t k = (uint32_t)__builtin_ctzll(mm);
              mm &= mm - 1;
              const uint32_t c = next_toggle(t, k);
              tr = c < tr ? c : tr;
            }
            nx = tr > nx ? tr : nx;
          }
          if (nx >= T) break;
          if (nx > t) {
            // Gray move t -> nx: add the differing walk columns in ascending
            // bit order (each to its nblk leading blocks), then re-form every
            // suffix product once.  Bit-identical to one step per bit: block
            // b's x is final after the last bit with nblk > b, and that step
            // formed U[b] from it and the final U[b + 1] — the expression
            // suffix_all evaluates on the final x (oracle: e_sparse_step per bit).
            const uint32_t gn = nx ^ (nx >> 1);
            uint32_t diff = (t ^ (t >> 1)) ^ gn;
            do {
              const uint32_t k = (uint32_t)__builtin_ctz(diff);
              diff &= diff - 1;
              const uint32_t neg = ((gn >> k) & 1u) ^ 1u;
              add_nest<N, 0>(x, opaque_c(colw, (2u * k + neg) * NP * 8u), nb_at(k));
            } while (diff);
            suffix_all<N>(x, U);
            u = nx + 1;
            ++visited;
            acc += U[0];  // nx is a segment start: even
            continue;  // check the new segment start
          }
        }
        // the quad u (walk bit 0, +), u + 1 (walk bit 1), u + 2 (bit 0, -),
        // u + 3 (walk bit ctz(u + 3) >= 2); u = 1 mod 4 here (segment starts
        // are multiples of 16), so walk bit 0's sign is + then - and walk bit
        // 1's is bit 2 of u + 1; the same steps in the same order as the pairs
        if constexpr (LOW == 3) {  // u = t + 1, t a segment start
          seg15<N>(x, U, colw, (u >> 4) & 1u, acc);
          visited += 15u;
          if (u + 15u >= T) break;
          const uint32_t v = u + 15u;
          const uint32_t k = (uint32_t)__builtin_ctz(v);
          const uint32_t neg = (v >> (k + 1)) & 1u;
          sparse_step<N>(x, U, opaque_c(colw, (2u * k + neg) * NP * 8u), nb_at(k));
          acc += U[0];
          ++visited;
          u += 16u;
          check = true;  // v opens a segment
          continue;
        }
        // ONE (walk bits 0 and 1 touch row block 0 only, as on every sparse
        // matrix measured): their steps are straight-line, one block
#define SUP_SKIP_LOW(NBV, OFF)                                                        \
  if constexpr (ONE) {                                                              \
    sparse_step_static<N, 1>(x, U, opaque_c(colw, (OFF) * NP * 8u));                \
  } else {                                                                          \
    int nbo = (NBV);                                                                \
    asm volatile("" : "+s"(nbo));                                                   \
    sparse_step<N>(x, U, opaque_c(colw, (OFF) * NP * 8u), nbo);                     \
  }
        SUP_SKIP_LOW(nb0, 0u)
        acc -= U[0];
        if (u + 1 >= T) {  // T = 2: the chunk's last state
          ++visited;
          break;
        }
        SUP_SKIP_LOW(nb1, 2u + (((u + 1) >> 2) & 1u))
        acc += U[0];
        SUP_SKIP_LOW(nb0, 1u)
        acc -= U[0];
#undef SUP_SKIP_LOW
        if constexpr (LOW == 2) {
          // walk bit 2 on block 0 too: the octet u .. u + 7 (u = 1 mod 8 here)
          if (u + 3 < T) {
            sparse_step_static<N, 1>(x, U, opaque_c(colw, (4u + (((u + 3) >> 3) & 1u)) * NP * 8u));
            acc += U[0];
            sparse_step_static<N, 1>(x, U, opaque_c(colw, 0u));
            acc -= U[0];
            sparse_step_static<N, 1>(x, U, opaque_c(colw, 3u * NP * 8u));
            acc += U[0];
            sparse_step_static<N, 1>(x, U, opaque_c(colw, NP * 8u));
            acc -= U[0];
            visited += (u + 7 < T) ? 8u : 7u;
            if (u + 7 >= T) break;
            const uint32_t v = u + 7;
            const uint32_t k = (uint32_t)__builtin_ctz(v);
            const uint32_t neg = (v >> (k + 1)) & 1u;
            sparse_step<N>(x, U, opaque_c(colw, (2u * k + neg) * NP * 8u), nb_at(k));
            acc += U[0];
            u += 8;
            check = (v & kSkipSegMask) == 0;  // v opens a segment
            continue;
          }
        }
        visited += (u + 3 < T) ? 4u : 3u;
        if (u + 3 >= T) break;
        const uint32_t v = u + 3;
        const uint32_t k = (uint32_t)__builtin_ctz(v);
        const uint32_t neg = (v >> (k + 1)) & 1u;
        sparse_step<N>(x, U, opaque_c(colw, (2u * k + neg) * NP * 8u), nb_at(k));
        acc += U[0];
        u += 4;
        check = (v & kSkipSegMask) == 0;  // v opens a segment
      }
      if (((uint32_t)ga ^ lane_par) & 1u) acc = -acc;
      const double part = wave_sum(lane_valid ? acc : 0.0);
      keep = (lane == j) ? part : keep;
      vkeep = (lane == j) ? visited : vkeep;
    }
    chunk_store((uint64_t)g * SUP_KARG(group), SUP_KARG(group), keep, vkeep);
  }
}

// The form a launch takes: the most specialised one whose static block
// counts cover the walk's own (LOW 3: bits 0-2 one block, bit 3 two; LOW 2:
// bits 0-2 one; LOW 1: bits 0-1 one; LOW 0: every count at run time).
// SUP_SKIP_FORM caps it (tests run every form on one matrix: same bits).
static int skip_form(const WalkParams& p) {
  static const int cap = [] {
    const char* e = std::getenv("SUP_SKIP_FORM");
    return e ? std::atoi(e) : 3;
  }();
  auto nbk = [&](int k) { return (int)((p.nb_lo >> (4 * k)) & 15ull); };
  int form = 0;
  if (p.m >= 4 && nbk(0) <= 1 && nbk(1) <= 1 && nbk(2) <= 1 && nbk(3) <= 2) form = 3;
  else if (p.m >= 3 && nbk(0) <= 1 && nbk(1) <= 1 && nbk(2) <= 1) form = 2;
  else if (p.m >= 2 && nbk(0) <= 1 && nbk(1) <= 1) form = 1;
  return form < cap ? form : (cap < 0 ? 0 : cap);
}

template <int N, int HI>
static hipError_t launch_rec(int n, const WalkParams& p, int grid, hipStream_t s) {
  if (n == N) {
    switch (skip_form(p)) {
      case 3: hipLaunchKernelGGL((walk_skip<N, 3>), dim3(grid), dim3(kBlock), 0, s, p); break;
      case 2: hipLaunchKernelGGL((walk_skip<N, 2>), dim3(grid), dim3(kBlock), 0, s, p); break;
      case 1: hipLaunchKernelGGL((walk_skip<N, 1>), dim3(grid), dim3(kBlock), 0, s, p); break;
      default: hipLaunchKernelGGL((walk_skip<N, 0>), dim3(grid), dim3(kBlock), 0, s, p); break;
    }
    return hipGetLastError();
  }
  if constexpr (N < HI) return launch_rec<N + 1, HI>(n, p, grid, s);
  return hipErrorInvalidValue;
}

template <int N, int HI>
static hipError_t occ_rec(int n, int* blocks_per_cu) {
  if (n == N) {  // the smaller residency of the two forms (the launch picks one by the block counts)
    int occ[4] = {0, 0, 0, 0};
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[0], walk_skip<N, 0>, kBlock, 0);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[1], walk_skip<N, 1>, kBlock, 0);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[2], walk_skip<N, 2>, kBlock, 0);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[3], walk_skip<N, 3>, kBlock, 0);
    *blocks_per_cu = occ[0];
    for (int v : occ) *blocks_per_cu = v < *blocks_per_cu ? v : *blocks_per_cu;
    return e;
  }
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
