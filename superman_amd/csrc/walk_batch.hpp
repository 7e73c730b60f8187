// walk_batch.hpp — several independent permanents of one order in one launch
// (the -o / -u leaves: sup_perman_reduced).  Not part of the segmented walk's
// embedded headers (jit.cpp), so its plan keys do not depend on it.
//
// A batch of K leaves with the same order and layout (lane bits L, walk bits
// m, 2^h wave-chunks each) is one wave-chunk queue of K 2^h chunks: global
// chunk a is chunk a mod 2^h of leaf a >> h, walked exactly as the one-leaf
// kernel walks it (same device code, that leaf's tables), and its partial
// lands in chunk_out[a].  Each leaf's 2^h partials are then folded by the
// one-leaf pairwise tree (launch_pairwise_reduce_seg), so every leaf's result
// is bit-identical to its own launch.
#pragma once
#include "walk_params.hpp"

namespace sup {

struct LeafDesc {
  const double* cols;       // the leaf's signed column table (2 (n-1) x NP)
  const double* x0;         // its start vector (NP)
  unsigned long long nb_lo;  // prefix-blocked walk: packed nblk (WalkParams::nb_lo / nb_hi)
  unsigned long long nb_hi;
  unsigned long long ends;   // prefix-blocked walk: chunk-end rows (walk_sparse.hip; WalkParams::umask there)
};

struct LeafBatch {
  const LeafDesc* leaves;  // [K], device memory
  unsigned int leaf_bits;  // h: chunks per leaf = 2^h
  unsigned int pad_;
};

}  // namespace sup
