// engine.hpp — host side of the MI355X permanent engine: plans, device
// contexts, schedulers.  Replaces the reference's per-call wrappers
// (gpu_exact_dense.cu:401-990, gpu_exact_sparse.cu:673-1408), which recompute
// x0/transpose, cudaMalloc, launch, D2H 2-4 MiB of per-thread partials and sum
// on the host on every call.
#pragma once
#include <stdint.h>
#include <cstdio>
#include <memory>
#include <mutex>
#include <functional>
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

// Cached walk bits (Plan::seg_cc) at most (the host twin and the oracle size
// their per-state arrays for 2^4 states).
constexpr int kMaxCachedBits = 4;

// Walk layout for an n x n problem (depends on n only, so results are
// bit-reproducible across grids and device counts).
struct Layout {
  int L;          // lane bits = min(6, n-1)
  int m;          // walk bits
  int h;          // high (wave-chunk) bits = n-1-L-m
  bool fixed = false;  // m asked for by the caller (sup_opts::walk_log2): plans keep it
  int cc_cap = kMaxCachedBits;  // segmented walk: cached walk bits at most (make_seg_plan)
  uint64_t chunks() const { return 1ull << h; }
};
Layout default_layout(int n);

// Product tree of the segmented walk (jit.cpp make_tree).  Items are engine
// rows (item_row[t] = row) and, when tail_hi > tail_lo, one constant item
// (item_row = -1): the halving-tree product of rows [tail_lo, tail_hi), which
// no walk bit >= 1 touches.  Node i = value(a[i]) * value(b[i]), where id <
// items() names item id and id = items() + i' names node i' < i.  sig = the
// step classes that make a node dirty: bit c < seg_b for walk bit c + 1, bit
// seg_b for the shared step of walk bits > seg_b.  A step of class c re-forms
// exactly the nodes with bit c, in index order.
struct ProdTree {
  std::vector<int> item_row;
  std::vector<uint32_t> item_sig;
  int tail_lo = 0, tail_hi = 0;
  std::vector<int> a, b;
  std::vector<uint32_t> sig;
  // storage plan (segmented walk, jit.cpp seg_fit), per item and per node:
  // bit 0 = its copies over x are kept live, bit 1 = its copies over y (inner
  // tree); otherwise they are formed on demand inside the nearest live
  // ancestor (the value is the same either way)
  std::vector<uint8_t> item_live, node_live;
  int items() const { return (int)item_row.size(); }
  int K() const { return (int)a.size(); }
  int root() const { return K() ? items() + K() - 1 : (items() ? 0 : -1); }
  uint32_t root_sig() const { return K() ? sig.back() : (items() ? item_sig[0] : 0u); }
};

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
  uint64_t chunk_ends = 0;         // prefix-blocked walk: lane-uniform rows no walk column touches (walk_sparse.hip)
  // ---- segmented walk (kind kWalkSeg, jit.cpp) ----
  // Engine rows [0, R) are the rows some walk column touches, in first-touch
  // order; segment i = rows [seg_start[i], seg_start[i+1]) are the rows walk
  // bit k_i touched first; rows [seg_start.back(), n) ("rest") no walk column
  // touches.  touched[k] = engine rows with a nonzero in walk bit k.
  std::vector<int> seg_start;
  std::vector<std::vector<int>> touched;
  std::vector<int> sub_start;      // sub-segments of segment 0 (first touch by walk bits >= 1);
                                   // rows [sub_start.back(), seg_start[1]) are constant per chunk
  int seg_b = 0;                   // pair bits [0, seg_b) have specialised steps (seg_static_bits)
  std::vector<int> dyn_rows;       // rows touched by walk bits > seg_b (their shared step)
  ProdTree outer_tree;             // rows outside segment 0 (over x)
  ProdTree inner_tree;             // segment 0's rows (once over x, once over y)
  bool lds = false;                // kWalkDense run by the LDS-staged kernel (walk_lds.hip; same bits)
  bool integral = false;           // every entry an integer (the segmented walk may then skip chunks)
  int seg_cc = 0;                  // cached step classes: walk bits 1..seg_cc held in every state
  double seg_ops = 0.0;            // fp64 VALU ops per Gray step of the generated kernel
  double seg_skip = 0.0;           // sampled fraction of wave-chunks the kernel skips (integer matrices)
  int seg_regs = 0;                // values live across steps (doubles), estimate
  int seg_budget = 0;              // live-value budget the storage plan was fitted to
  std::vector<int> jofs;           // [m] offset (doubles) of walk bit k's + block in jtab
  std::vector<double> jtab;        // packed touched values: + block, - block (each padded to 8); then,
                                   // from seg_cbase, the row-copy constants (jit.cpp Gen::tail)
  size_t seg_cbase = 0;
  // Segmented walk: every wave-chunk's start state without the lane columns
  // (x0 + the chunk bits' columns, added on the host in chunk_start's order:
  // the same values), read by the kernel instead of formed (walk_common.hpp
  // chunk_start_tab) when the table is at most kStartTabMaxBytes.
  bool start_tab_on = false;
  std::vector<double> start_tab;   // chunks x NP
  int seg_kp = 4;                  // SGPR pieces (8 doubles) pinned per step region of the generated code
  std::string jit_src;             // generated HIP source of the specialised kernel
  uint64_t jit_key = 0;            // hash of jit_src + compile options
  uint64_t uid = 0;                // plan-cache identity (0: uncached); a device that holds
                                   // this plan's tables skips their upload (run_range)
  std::vector<int> seg_order;      // segmented walk: the m walk + L lane columns its search chose
  bool seg_loop_scratch = false;   // build_seg's check of a short walk's kernel found scratch in its loop
};

// The choices a segmented-walk plan is rebuilt from without searching: walk +
// lane column order, specialised pair bits, live-value budget (persisted on
// disk by make_seg_plan, so a later process skips the walk-order search and
// the compiler check).
struct SegChoice {
  std::vector<int> order;
  int b = 0;
  int budget = 0;
  int cc_cap = kMaxCachedBits;
};

// Build a plan.  identity_map keeps engine bit e = column e (needed when a
// chunk range must match reference Gray indices: sup_partial); otherwise the
// SpaRyser walk takes its walk columns in greedy_walk_order.
// `choice` (segmented walk only): rebuild from recorded choices instead of
// searching (SegChoice).
int make_plan(const double* A, int n, WalkKind kind, bool identity_map, const Layout& lay, Plan& P,
              const SegChoice* choice = nullptr);

// Walk-column order minimising the prefix-block cost (first `count` columns).
std::vector<int> greedy_walk_order(const double* A, int n, int count);
// SkipPer walk + lane columns (walk first) chosen for the chunks its first-state
// zero check ends (integer matrices); false: keep SkipOrder's map (engine.cpp).
// baseline (m + L columns; NULL: SkipOrder's map) is kept unless the search beats
// its ops x chunks walked by `factor`.
bool skip_walk_order(const double* A, int n, const Layout& lay, std::vector<int>& out,
                     const std::vector<int>* baseline, double factor);
// A long prefix-blocked plan of an integer matrix, its columns searched for
// chunk ends (engine.cpp; exact.cpp and quad.cpp use it too).
int improve_sparse_plan(const double* A, int n, const Layout& lay, Plan& P);
// Host threads the planners' searches use (jit.cpp).
int plan_threads();

// ---- segmented walk (jit.cpp) ----
// Walk-column order for the segmented walk: greedy starts from every column,
// then pairwise-swap descent on seg_cost (first `count` columns returned).
// *b_out = the specialised pair bits the order was chosen for (seg_b).
std::vector<int> seg_walk_order(const double* A, int n, int m, int count, int* b_out, int cc_cap = kMaxCachedBits);
// Sampled fraction of wave-chunks the segmented kernel skips (walk-untouched
// rows exactly zero in every lane) for an extended walk order (m walk
// columns, then the lane columns); integer matrices.
double seg_skip_estimate(const double* A, int n, const std::vector<int>& order, int m, int samples);
// The same for a built segmented plan (engine row and column order).
double seg_skip_fraction_plan(const Plan& P, int samples);
// Engine row order of the segmented walk for walk columns `walk`: rows in
// first-touch order, segment 0 (the rows of walk[0]) internally ordered by
// first touch among walk[1..], its rows no other walk column touches last.
std::vector<int> seg_row_order(const double* A, int n, const std::vector<int>& walk);
// Fill the segment structure, packed table and generated source of a plan
// whose rows are already in first-touch order (make_plan, kind kWalkSeg).
// fixed_budget > 0: fit the storage plan to that live-value budget, no
// compiler check (a recorded choice).
int build_seg(Plan& P, int fixed_budget = 0);
// Disk cache of segmented-walk choices (next to the code objects): key ->
// (walk bits m, SegChoice).  jit_toolchain_hash() covers what the choices
// were priced with (generated-code headers, compile options, hiprtc).
bool seg_choice_load(uint64_t key, int* m, SegChoice* c);
bool seg_choice_exists(uint64_t key);
// Cold segmented-plan cost (walk-order search + the compiler check's
// compiles) predicted for order n on this host: seg_cold_model (a GPU box's
// 16 threads, scaled to this host's plan threads) times this host's recorded
// speed (the last cold plan's measured / modelled cost; 1 when none).
double seg_cold_model(int n);
double seg_cold_predict(int n);
// Record a cold plan of order n that took `seconds` (the host's speed ratio).
void seg_cost_store(int n, double seconds);
double seg_cost_ratio_load();  // recorded measured / modelled ratio, -1 if none
void seg_choice_store(uint64_t key, int m, const SegChoice& c);
// Auto mode's (jit = 0) first decision for a matrix and request, recorded next
// to the plan choices: 1 segmented walk, 0 ahead-of-time walk, -1 none yet.
int auto_decision_load(uint64_t key);
// Records `seg` only if no decision is on disk yet (created exclusively: two
// processes deciding at once cannot both win) and returns the decision on
// disk afterwards, which the caller follows; `seg` when there is no cache.
int auto_decision_store(uint64_t key, int seg);
uint64_t jit_toolchain_hash();
// Default specialised pair bits, min(m - 1, 5) (the walk loop is unrolled by
// 2^b pair steps; walk bits > b share one straight-line step).  Plans choose
// b in 5..8 by the op count (seg_walk_order / build_seg).
int seg_static_bits(int m);
// Row-copy constants of the segmented walk (x^S_r = x^0_r + seg_cx(P, r, S),
// y^S_r = x^0_r + seg_cy(P, r, S); S = cached state masked to the walk bits
// 1..seg_cc that touch row r, nonzero for seg_cx).
double seg_cx(const Plan& P, int r, uint32_t S);
double seg_cy(const Plan& P, int r, uint32_t S);
// fp64 VALU ops per Gray step and lane of the segmented walk.
double seg_walk_cost(const Plan& P);
// Resolve (compile or fetch from cache) the specialised kernel of P for the
// current device `dev`, then launch it / query its occupancy.
int jit_occupancy(int dev, const Plan& P, int* blocks_per_cu, double* compile_ms);
int jit_launch(int dev, const Plan& P, const WalkParams& p, int grid, hipStream_t s);
// Compile (or find in the caches) the specialised kernel of P without loading it.
int jit_compile_only(const Plan& P, double* compile_ms);
// What a compiled kernel does with registers and scratch (codescan.cpp):
// metadata counts, and the scratch instructions inside its walk loop (the
// natural loop with the most fp64 VALU work that holds no inner loop with half
// of it), found by disassembling the code object.
struct CodeScan {
  int vgprs = -1, vgpr_spills = -1, scratch_bytes = -1;  // .vgpr_count, .vgpr_spill_count, private segment
  int insts = 0, scratch_insts = 0, loops = 0;           // whole kernel
  int loop_scratch = -1, loop_f64 = 0, loop_insts = 0;   // the walk loop (-1: none found)
  int loop_readlane = 0;                                 // its v_readlane (SGPR spill reloads)
};
int scan_code_object(const std::vector<char>& code, const char* kernel, CodeScan* out);
// Compile (or fetch) P's kernel and scan it.
int jit_code_scan(const Plan& P, CodeScan* out);
// Milliseconds this thread spent compiling specialised kernels (hiprtc; a batch
// compiled on helper threads counts its wall time here).  Per thread, so
// concurrent callers do not count each other's compiles.
double jit_compile_ms_thread();

// Estimated fp64 VALU ops per Gray step of a plan (dense: 2n+1; prefix kernels:
// sum_k 2^-(k+1) (16 nblk_k + 1)).
double walk_cost(const Plan& P);

// The plan sup_perman / sup_perman_shard run for this request: for
// SUP_KERNEL_DENSE the engine takes the prefix-blocked walk whenever its cost
// model is lower (same sum, structural zeros skipped); SUP_KERNEL_DENSE_PLAIN
// forces the plain dense walk.
// jit: sup_opts.jit (-1 never, 0 auto, 1 whenever the segmented walk's cost
// model wins); ndev: devices the walk is spread over (auto mode's estimate).
// dev: the device a SkipPer request on an integer matrix samples its visited
// fraction on (the decision itself does not depend on it).
int plan_for(const double* A, int n, sup_kernel kernel, const Layout& lay, Plan& P, int jit = -1, int ndev = 1,
             int dev = 0);
// The same, sharing the cached plan instead of copying it (the per-call path
// of sup_perman / sup_perman_shard).
int plan_for_shared(const double* A, int n, sup_kernel kernel, const Layout& lay, std::shared_ptr<const Plan>& P,
                    int jit = -1, int ndev = 1, int dev = 0, bool keep = true);

struct RangeResult {
  double partial = 0.0;     // pairwise sum over the range's wave-chunks
  double kernel_ms = 0.0;   // walk kernel device time (hipEvents on the launch stream)
  uint64_t visited = 0;     // evaluated products (lanes * steps), skipper only
  int grid = 0;
  double compile_ms = 0.0;  // segmented walk: hiprtc compile time spent by this call
};

// Walk wave-chunks [c0, c1) of plan P on device `dev` (synchronous).
// The dynamic item queue shared by -p6/-p8, the exact path and the
// estimators: `takers` host threads (one per device, plus the hybrid CPU
// worker) pull item indices 0..nitems-1 from one atomic counter until they run
// out or a taker fails; take(taker, item) writes only its own outputs
// (item-indexed slots, per-taker accumulators), so the combined result never
// depends on who took which item.  Returns SUP_OK or the first failure (with
// its message).
int run_item_queue(uint64_t nitems, int takers, const std::function<int(int, uint64_t)>& take);
// slot (optional): a device pointer on `dev`; the range's partial is also
// copied there on the device (the -R combine all-reduces those slots).
int run_range(int dev, const Plan& P, uint64_t c0, uint64_t c1, bool want_visited, RangeResult& r,
              double* slot = nullptr);
// Leaf batches (sup_perman_reduced's leaves): up to kMaxBatchLeaves plans of
// one order, walk kind (plain / prefix-blocked) and layout in one launch on
// device `dev`; partial[i] is bit-identical to run_range over plan i's whole
// range.  batchable(): whether two plans can share a launch.
constexpr int kMaxBatchLeaves = 32;
// The batch kernels index chunks with 32 bits (walk_sparse_batch): batchable()
// caps a leaf at 2^kMaxBatchLeafChunkBits chunks, so a batch stays below 2^32.
constexpr int kMaxBatchLeafChunkBits = 26;
static_assert((uint64_t)kMaxBatchLeaves << kMaxBatchLeafChunkBits <= (1ull << 32),
              "leaf batches must fit 32-bit chunk indices");
bool batchable(const Plan& a, const Plan& b);
int run_range_batch(int dev, const std::vector<const Plan*>& plans, std::vector<double>& partial, double* kernel_ms);

// Combine partials with the same pairwise tree the device reduction uses.
double pairwise_host(const std::vector<double>& v);

int device_count(int* n);
// Context lanes: up to kCtxLanes device contexts per logical device; a host
// thread picks its lane with set_ctx_lane (default 0) and the schedulers'
// threads inherit the caller's.
constexpr int kCtxLanes = 8;
void set_ctx_lane(int lane);
int ctx_lane();
// Deferred walk timing for the calling thread (sup_opts.timing = 0): run_range
// records the walk's events without waiting for them; kernel_time reads them.
void set_defer_timing(bool on);
int kernel_time(int dev, double* total_ms, uint64_t* launches);
int phys_device(int dev);  // logical -> physical (SUP_DEVICE_MAP; identity when unset)
// Select logical device `dev` (physical phys_device(dev)) on this thread:
// hipSetDevice plus a thread-local note of the logical id, which
// check_device compares.
hipError_t select_device(int dev);
// SUP_CHECK_DEVICE=1 (tests): before every allocation,
// module load and launch of a device thread, the thread's HIP device must be
// the physical device behind the logical device whose context it uses, and
// the logical device it last selected must be that one (on a one-GPU box with
// SUP_DEVICE_MAP=0,0,... the physical ids agree, the logical ones do not).  A
// mismatch returns SUP_EHIP.  Off: one branch.
int check_device(int dev, const char* what);
uint64_t device_checks_passed();
// A HIP call whose failure returns SUP_EHIP with the call's text and HIP's message.
#ifndef SUP_HIP
#define SUP_HIP(call)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      set_error(std::string(#call) + ": " + hipGetErrorString(e_));                    \
      return SUP_EHIP;                                                                 \
    }                                                                                  \
  } while (0)
#endif

#define SUP_ON_DEVICE(dev, what)                 \
  do {                                           \
    const int rc_ = check_device((dev), (what)); \
    if (rc_) return rc_;                         \
  } while (0)
// HIP init, contexts of devices [first, first + count) and the AOT walks of order n (sup_device_warmup)
int warm_devices(int first, int count, int n);
// physical devices of the RCCL combine over logical `devs`; SUP_ERCCL if two share a GPU
int rccl_physical_devices(const std::vector<int>& devs, std::vector<int>& phys);

// Schedulers (one host thread per device).
struct SchedResult {
  double total = 0.0;       // sum over all wave-chunks (includes the p0 term)
  double kernel_ms = 0.0;   // max over devices of summed walk-kernel time
  uint64_t visited = 0;
  int devices = 0;
  int grid = 0;
  int cpu_items = 0;
  double compile_ms = 0.0;  // summed over devices
  int items_resumed = 0;    // queue items taken from the checkpoint file (sup_opts::checkpoint)
  std::vector<double> dev_partials;
};
int schedule(const Plan& P, sup_sched sched, const sup_opts& o, uint64_t c0, uint64_t c1,
             SchedResult& out);
// Checkpoint file of the chunk queue (sup_opts::checkpoint; engine.cpp):
// ckpt_open loads the items a file with header `head` records (marking them
// in `done`, their partials in `ipart`) and leaves it open for appending;
// ckpt_record appends one finished item (thread-safe, flushed and fsynced).
struct Checkpoint {
  FILE* f = nullptr;
  std::mutex mu;
  ~Checkpoint() {
    if (f) std::fclose(f);
  }
};
int ckpt_open(const char* path, const char* head, uint64_t nitems, std::vector<double>& ipart,
              std::vector<char>& done, uint64_t& vis, int& resumed, Checkpoint& ck);
int ckpt_record(Checkpoint& ck, uint64_t it, double part, uint64_t visited);

// 64-bit fingerprint of everything that decides a plan's sum and its rounding
// (sup_plan_key; the checkpoint file's header)
uint64_t plan_fingerprint(const Plan& P);

// CPU worker: the same wave-chunk walk on host threads (used for `-c` and for
// the hybrid `-c -g` chunk queue).  Bit-identical to the dense/sparse kernels.
double cpu_walk_range(const Plan& P, uint64_t c0, uint64_t c1, int threads);

// ---- exact path (exact.cpp, walk_exact.hip) ----
// Per prime, sum over wave-chunks [c0, c1) of the terms of the dense identity
// plan P (of 2A) modulo that prime, in [0, p): on device `dev` (rows
// multiplied in exact groups of `group` = 1, 2 or 4 first), or on host
// threads (same residues: every operation is exact).
int run_range_exact(int dev, const Plan& P, int group, uint64_t c0, uint64_t c1, const std::vector<double>& primes,
                    std::vector<uint64_t>& res, double* kernel_ms);
void cpu_exact_range(const Plan& P, uint64_t c0, uint64_t c1, const std::vector<double>& primes, int threads,
                     std::vector<uint64_t>& res);
// Exact permanent of integer-valued A as a decimal string (sup_perman_exact).
// Several devices or o.cpu_worker: a queue of chunk items; *cpu_items = items
// the CPU worker took.
int exact_perman(const double* A, int n, const sup_opts& o, bool on_cpu, std::string& out, double* kernel_ms,
                 int* devices_used, int* cpu_items = nullptr);
// The same after the -o reductions (sup_perman_reduced_exact): exact leaves, big-integer sum.
int exact_perman_reduced(const double* A, int n, const sup_opts& o, bool on_cpu, const sup_reduce_opts& r,
                         std::string& out, double* kernel_ms, int* leaves);

// ---- double-double walk (quad.cpp, walk_dd.hip) ----
// Wave-chunk partials (hi, lo) of chunks [c0, c1) of the dense identity plan
// P with the double-double start vector x0dd (2 NP: hi block, lo block) into
// parts[2 (c - c0) + {0, 1}]: on device `dev`, or on host threads (bit-identical).
int run_range_dd(int dev, const Plan& P, const std::vector<double>& x0dd, uint64_t c0, uint64_t c1,
                 double* parts, double* kernel_ms);
void cpu_dd_range(const Plan& P, const std::vector<double>& x0dd, uint64_t c0, uint64_t c1, int threads,
                  double* parts);
struct dd;
// -o / -u with leaves computed concurrently (sup_perman_reduced,
// sup_perman_reduced_exact; decompose_dd_batched: double-double leaves and
// combine, sup_perman_reduced_quad): leaf(worker, a, n, &value) is called from
// `workers` host threads as the decomposition produces leaves; the combine is
// folded afterwards in the recursive order, so the result equals the
// sequential fold's bit for bit.
// memo: a leaf equal to an earlier one takes its value without a call (off
// when the callback must see every leaf, e.g. to sum exact values itself).
int decompose_batched(const double* A, int n, const sup_reduce_opts& r, int workers,
                      const std::function<int(int, const double*, int, double*)>& leaf, double* out, int* n_leaves,
                      bool memo = true);
// The same with leaves handed out in batches (a worker takes up to
// `batch_max` queued leaves of one order at once), in two stages:
// staged(worker, mats, n, values, walk) plans a batch
// on the host and returns its device part in `walk`, which the worker's own
// walker thread runs while the worker plans the next batch (channel depth 2).
typedef std::function<int(int, const std::vector<const double*>&, int, const std::vector<double*>&,
                          std::function<int()>&)>
    LeafBatchStagedFn;
int decompose_batched_staged(const double* A, int n, const sup_reduce_opts& r, int workers, int batch_max,
                             const LeafBatchStagedFn& staged, double* out, int* n_leaves);
int decompose_dd_batched(const double* A, int n, const sup_reduce_opts& r, int workers,
                         const std::function<int(int, const double*, int, dd*)>& leaf, dd* out, int* n_leaves);
// Permanent in double-double (sup_perman_quad): *hi + *lo.
int quad_perman(const double* A, int n, const sup_opts& o, bool on_cpu, double* hi, double* lo, double* kernel_ms,
                int* devices_used);

}  // namespace sup
