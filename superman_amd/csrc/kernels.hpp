// kernels.hpp — host-visible launch entry points of the gfx950 walk kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "walk_batch.hpp"
#include "walk_params.hpp"

namespace sup {

// SkipPer (walk_skip.hip, its host twin engine_cpu.cpp; oracle/oracle.c
// restates it): zero checks and jumps at the starts of aligned segments of
// 2^kSkipSegBits Gray steps.
#ifndef SUP_SKIP_SEG_BITS
#define SUP_SKIP_SEG_BITS 4  // (other values: experiments; oracle/oracle.c must agree)
#endif
constexpr int kSkipSegBits = SUP_SKIP_SEG_BITS;
constexpr uint32_t kSkipSegMask = (1u << kSkipSegBits) - 1u;

// Per-N-range launchers (one translation unit per range, see Makefile).
#define SUP_DECL_RANGE(KIND, LO)                                                      \
  hipError_t launch_##KIND##_##LO(int n, const WalkParams& p, int grid, hipStream_t s); \
  hipError_t occupancy_##KIND##_##LO(int n, int* blocks_per_cu);
SUP_DECL_RANGE(dense, 1)
SUP_DECL_RANGE(dense, 17)
SUP_DECL_RANGE(dense, 33)
SUP_DECL_RANGE(dense, 49)
SUP_DECL_RANGE(sparse, 1)
SUP_DECL_RANGE(sparse, 17)
SUP_DECL_RANGE(sparse, 33)
SUP_DECL_RANGE(sparse, 49)
SUP_DECL_RANGE(skip, 1)
SUP_DECL_RANGE(skip, 17)
SUP_DECL_RANGE(skip, 33)
SUP_DECL_RANGE(skip, 49)
#undef SUP_DECL_RANGE
#define SUP_DECL_BATCH(KIND, LO)                                                                       \
  hipError_t launch_batch_##KIND##_##LO(int n, const WalkParams& p, const LeafBatch& b, int grid, hipStream_t s); \
  hipError_t occupancy_batch_##KIND##_##LO(int n, int* blocks_per_cu);
SUP_DECL_BATCH(dense, 1)
SUP_DECL_BATCH(dense, 17)
SUP_DECL_BATCH(dense, 33)
SUP_DECL_BATCH(dense, 49)
SUP_DECL_BATCH(sparse, 1)
SUP_DECL_BATCH(sparse, 17)
SUP_DECL_BATCH(sparse, 33)
SUP_DECL_BATCH(sparse, 49)
#undef SUP_DECL_BATCH
#define SUP_DECL_EXACT(LO)                                                                                  \
  hipError_t launch_exact_##LO(int n, int g, const WalkParams& p, const ExactParams& e, int grid,        \
                               hipStream_t s);                                                        \
  hipError_t occupancy_exact_##LO(int n, int g, int* blocks_per_cu);
SUP_DECL_EXACT(1)
SUP_DECL_EXACT(17)
SUP_DECL_EXACT(33)
SUP_DECL_EXACT(49)
#undef SUP_DECL_EXACT
#define SUP_DECL_DD(LO)                                                               \
  hipError_t launch_dd_##LO(int n, const WalkParams& p, int grid, hipStream_t s);    \
  hipError_t occupancy_dd_##LO(int n, int* blocks_per_cu);
SUP_DECL_DD(1)
SUP_DECL_DD(17)
SUP_DECL_DD(33)
SUP_DECL_DD(49)
#undef SUP_DECL_DD
#define SUP_DECL_DDB(LO)                                                                  \
  hipError_t launch_ddblocked_##LO(int n, const WalkParams& p, int grid, hipStream_t s);  \
  hipError_t occupancy_ddblocked_##LO(int n, int* blocks_per_cu);
SUP_DECL_DDB(1)
SUP_DECL_DDB(17)
SUP_DECL_DDB(33)
SUP_DECL_DDB(49)
#undef SUP_DECL_DDB
#define SUP_DECL_LDS(LO)                                                                   \
  hipError_t launch_lds_##LO(int n, const WalkParams& p, int grid, hipStream_t s);        \
  hipError_t occupancy_lds_##LO(int n, int m, int* blocks_per_cu);
SUP_DECL_LDS(1)
SUP_DECL_LDS(17)
SUP_DECL_LDS(33)
SUP_DECL_LDS(49)
#undef SUP_DECL_LDS

// kWalkSeg: the pattern-specialised segmented walk (jit.cpp), compiled at run
// time with hiprtc for one matrix pattern; launched through hipModule APIs.
enum WalkKind { kWalkDense = 0, kWalkSparse = 1, kWalkSkip = 2, kWalkSeg = 3 };

// Launch the walk kernel of `kind` for matrix order n (1..64).
hipError_t launch_walk(WalkKind kind, int n, const WalkParams& p, int grid, hipStream_t s);
// Resident 256-thread blocks per CU for that kernel (occupancy API).
hipError_t walk_occupancy(WalkKind kind, int n, int* blocks_per_cu);

// A batch of leaves of one order and layout in one launch (walk_batch.hpp;
// kWalkDense / kWalkSparse), and its occupancy.
hipError_t launch_walk_batch(WalkKind kind, int n, const WalkParams& p, const LeafBatch& b, int grid, hipStream_t s);
hipError_t walk_batch_occupancy(WalkKind kind, int n, int* blocks_per_cu);

// LDS-staged dense walk (walk_lds.hip; 64-thread blocks, X in LDS).
hipError_t launch_lds(int n, const WalkParams& p, int grid, hipStream_t s);
hipError_t lds_occupancy(int n, int m, int* blocks_per_cu);

// Exact residue walk (walk_exact.hip) for matrix order n (1..64), rows
// multiplied in exact groups of g (1, 2 or 4) before the residue chain.
hipError_t launch_exact(int n, int g, const WalkParams& p, const ExactParams& e, int grid, hipStream_t s);
hipError_t exact_occupancy(int n, int g, int* blocks_per_cu);

// Double-double dense walk (walk_dd.hip): p.x0 = 2 NP doubles (hi, lo),
// p.chunk_out = 2 doubles (hi, lo) per wave-chunk.
hipError_t launch_dd(int n, const WalkParams& p, int grid, hipStream_t s);
hipError_t dd_occupancy(int n, int* blocks_per_cu);
// Its prefix-blocked form (walk_dd_blocked, a kWalkSparse plan: p.nb_lo / nb_hi).
hipError_t launch_dd_blocked(int n, const WalkParams& p, int grid, hipStream_t s);
hipError_t dd_blocked_occupancy(int n, int* blocks_per_cu);

// Fixed-order pairwise reduction of `count` doubles into *out (64-way passes,
// zero padded; mirrored by oracle/oracle.c orc_pairwise_reduce).  `scratch`
// must hold ceil(count/64) + ceil(count/4096) + ... doubles.
// reset_counter (optional): zeroed by the first pass, which runs after the
// walk that used it (the next launch's queue then needs no memset).
// flag (optional, count > 1): the last pass stores `seq` there after *out,
// system-scope ordered (mapped host memory: the host waits on it).
hipError_t launch_pairwise_reduce(const double* in, uint64_t count, double* scratch, double* out,
                                  hipStream_t s, unsigned int* reset_counter = nullptr, unsigned int* flag = nullptr,
                                  unsigned seq = 0);
uint64_t pairwise_scratch_size(uint64_t count);
// *out = sum of `count` unsigned values (zeroed first, on stream s).
hipError_t launch_sum_visited(const unsigned* in, uint64_t count, unsigned long long* out, hipStream_t s);
// The same tree over each of `nseg` consecutive segments of `count` doubles
// (a leaf batch's chunk partials): out[i] is bit-identical to
// launch_pairwise_reduce over segment i alone.  `scratch` holds nseg times
// pairwise_scratch_size(count).
hipError_t launch_pairwise_reduce_seg(const double* in, uint64_t count, uint64_t nseg, double* scratch, double* out,
                                      hipStream_t s);

}  // namespace sup
