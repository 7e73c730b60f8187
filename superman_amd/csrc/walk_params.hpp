// walk_params.hpp — launch parameters shared by host and the gfx950 walk kernels.
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#else
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#endif

namespace sup {

constexpr int kBlock = 256;  // threads per workgroup (4 waves)
constexpr int kWavesPerBlock = kBlock / 64;

// Pad n up to a multiple of 8 doubles (64 B) so every column starts on an
// s_load_dwordx16 boundary.
constexpr int pad8(int n) { return (n + 7) & ~7; }

struct WalkParams {
  const double* cols;              // signed column table: entry (2*e + neg) * NP + j, e = engine bit
  const double* x0;                // NP doubles: Nijenhuis-Wilf start vector (rows in engine order)
  const int* nblk;                 // sparse kernels: per engine bit, # of 8-row blocks the prefix touches
  const uint64_t* rowmask;         // skipper: per row, walk-bit mask of the columns touching the row
  unsigned long long chunk_begin;  // first wave-chunk (global index)
  unsigned long long chunk_count;  // wave-chunks in this launch
  int L;                           // lane bits (<= 6)
  int m;                           // walk bits
  int n;                           // matrix order (runtime copy, for tables)
  int pad_;
  unsigned long long umask;        // skipper: bit r set <=> row r is lane-uniform (no lane column touches it)
  double* chunk_out;               // [chunk_count] per-wave-chunk partial sums
  unsigned int* counter;           // dynamic wave-chunk queue head (zeroed before launch)
  unsigned int* visited;           // optional [chunk_count]: product evaluations per chunk (skipper)
  // sparse kernels: nblk of walk bit k packed as 4-bit fields, k < 16 in nb_lo,
  // k >= 16 in nb_hi (kept in SGPRs: no memory round trip per step)
  unsigned long long nb_lo, nb_hi;
  // wave-chunks are dequeued in groups of `group` (1, 2, 4, ..., 64)
  // consecutive chunks; the group's partials leave the wave as one store of
  // 8*group bytes.
  // The host picks the largest group that still leaves >= 32 groups per
  // resident wave (tail balance beats write coalescing).
  unsigned int group;
  // segmented walk: the queue's tail phase.  Tickets below tail_begin / group
  // hand out `group` chunks each; the chunks from tail_begin on go out in
  // groups of tail_group (< group), so the waves finish within a smaller group
  // of each other (tail_group 0: no tail phase).
  unsigned int tail_group;
  unsigned int tail_ticket;        // = tail_begin / group (0xffffffff: no tail phase)
  unsigned int pad3_;
  unsigned long long tail_begin;
  // segmented walk (jit.cpp): per walk bit, the values of the rows its column
  // touches, packed (+ block, then - block, each padded to 8 doubles)
  const double* jtab;
  // diagnostics (SUP_JIT_TRACE): per wave 8 u64 — realtime and shader-clock
  // stamps at entry and exit, chunks walked, shader cycles spent in chunk
  // starts; nullptr (and never written) otherwise
  unsigned long long* trace;
  // The fused fold (walk_common.hpp chunk_store; fold_cnt == nullptr: the
  // partials go to chunk_out and launch_pairwise_reduce folds them after the
  // walk).  fold_cnt: one arrival counter per 64-group of every level, zero
  // between launches (the group's last arriver resets it); fold_lv: the
  // level values; fold_out: [0] the result, [2] the visited sum (u64);
  // fold_vis: the visited accumulator (zero between launches) or nullptr;
  // fold_reset: the next launch's queue head, zeroed by the final fold;
  // fold_flag: fold_seq is stored there (system scope) after the result.
  unsigned int* fold_cnt;
  double* fold_lv;
  double* fold_out;
  unsigned long long* fold_vis;
  unsigned int* fold_reset;
  unsigned int* fold_flag;
  unsigned int fold_seq;
  // 1: the final fold publishes the result (and the visited sum before it)
  // with system-scope stores and no flag: the host waits for the result slot
  // to leave the sentinel it wrote (run_range); 0: result, fence, flag
  unsigned int fold_sys;
  // segmented walk with a start table (Plan::start_tab): chunk ga's start
  // state without the lane columns at start_tab[ga * NP], or nullptr
  const double* start_tab;
};

// Exact path (walk_exact.hip): residues of the walk's terms modulo up to
// kMaxPrimes primes (p < 2^42, held in fp64; pinv = 1 / p rounded).
constexpr int kMaxPrimes = 8;
struct ExactParams {
  double prime[kMaxPrimes];
  double pinv[kMaxPrimes];
  int nprimes;
  int pad_;
  double* wave_out;  // [grid waves][kMaxPrimes]: each wave's residue sum, in [0, p)
};

}  // namespace sup
