// engine.hpp — host side of the MI355X permanent engine: plans, device
// contexts, schedulers.  Replaces the reference's per-call wrappers
// (gpu_exact_dense.cu:401-990, gpu_exact_sparse.cu:673-1408), which recompute
// x0/transpose, cudaMalloc, launch, D2H 2-4 MiB of per-thread partials and sum
// on the host on every call.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/superman.h"
#include "kernels.hpp"

namespace sup {

// Thread-local error channel behind sup_last_error().
void set_error(const std::string& msg);
const char* last_error();

// Convert the caller's T matrix (int/float/double) to fp64 (exact for all three).
int to_double(const void* mat, sup_dtype t, int n, std::vector<double>& out);

// Nijenhuis–Wilf start vector, reference order of operations
// (gpu_exact_dense.cu:642-652): rs = sum_k a[j][k] (ascending k, starting 0.0),
// x0[j] = a[j][n-1] - rs/2, p0 = prod_j x0[j] (ascending j, starting 1.0).
void nw_start(const double* A, int n, double* x0, double* p0);

// Walk layout for an n x n problem (depends on n only, so results are
// bit-reproducible across grids and device counts).
struct Layout {
  int L;          // lane bits = min(6, n-1)
  int m;          // walk bits
  int h;          // high (wave-chunk) bits = n-1-L-m
  uint64_t chunks() const { return 1ull << h; }
};
Layout default_layout(int n);

struct Plan {
  int n = 0;
  int NP = 0;
  WalkKind kind = kWalkDense;
  Layout lay{};
  std::vector<int> rowperm;        // engine row j = matrix row rowperm[j]
  std::vector<int> colmap;         // engine bit e = matrix column colmap[e] (e < n-1)
  std::vector<double> cols;        // (2*(n-1)) x NP signed column table (engine order)
  std::vector<double> x0;          // NP, engine row order
  std::vector<int> nblk;           // n-1: prefix row-block count per engine bit
  std::vector<uint64_t> rowmask;   // n: walk-bit mask of each engine row
  uint64_t umask = 0;              // lane-uniform engine rows
};

// Build a plan.  identity_map keeps engine bit e = column e (needed when a
// chunk range must match reference Gray indices: sup_partial); otherwise the
// SpaRyser walk takes its walk columns in greedy_walk_order.
int make_plan(const double* A, int n, WalkKind kind, bool identity_map, const Layout& lay, Plan& P);

// Walk-column order minimising the prefix-block cost (first `count` columns).
std::vector<int> greedy_walk_order(const double* A, int n, int count);

// Estimated fp64 VALU ops per Gray step of a plan (dense: 2n+1; prefix kernels:
// sum_k 2^-(k+1) (16 nblk_k + 1)).
double walk_cost(const Plan& P);

// The plan sup_perman / sup_perman_shard run for this request: for
// SUP_KERNEL_DENSE the engine takes the prefix-blocked walk whenever its cost
// model is lower (same sum, structural zeros skipped); SUP_KERNEL_DENSE_PLAIN
// forces the plain dense walk.
int plan_for(const double* A, int n, sup_kernel kernel, const Layout& lay, Plan& P);

struct RangeResult {
  double partial = 0.0;     // pairwise sum over the range's wave-chunks
  double kernel_ms = 0.0;   // walk kernel device time (hipEvents on the launch stream)
  uint64_t visited = 0;     // evaluated products (lanes * steps), skipper only
  int grid = 0;
};

// Walk wave-chunks [c0, c1) of plan P on device `dev` (synchronous).
int run_range(int dev, const Plan& P, uint64_t c0, uint64_t c1, bool want_visited, RangeResult& r);

// Combine partials with the same pairwise tree the device reduction uses.
double pairwise_host(const std::vector<double>& v);

int device_count(int* n);

// Schedulers (one host thread per device).
struct SchedResult {
  double total = 0.0;       // sum over all wave-chunks (includes the p0 term)
  double kernel_ms = 0.0;   // max over devices of summed walk-kernel time
  uint64_t visited = 0;
  int devices = 0;
  int grid = 0;
  int cpu_items = 0;
  std::vector<double> dev_partials;
};
int schedule(const Plan& P, sup_sched sched, const sup_opts& o, uint64_t c0, uint64_t c1,
             SchedResult& out);

// All-reduce (sum, fp64) over RCCL, in one process, of per-device vectors with
// disjoint supports (exact in any order); merged = the slot-wise sum.
int rccl_allreduce_partials(const std::vector<int>& devs, const std::vector<std::vector<double>>& contrib,
                            std::vector<double>& merged);

// CPU worker: the same wave-chunk walk on host threads (used for `-c` and for
// the hybrid `-c -g` chunk queue).  Bit-identical to the dense/sparse kernels.
double cpu_walk_range(const Plan& P, uint64_t c0, uint64_t c1, int threads);

}  // namespace sup
