// jit.cpp — the segmented walk: a Gray walk kernel specialised at run time for
// one matrix pattern, compiled for gfx950 with hiprtc.
//
// Why.  The reference SpaRyser step touches only the CSC rows of the flipped
// column but keeps the product incrementally with an fp64 divide
// (gpu_exact_sparse.cu:503-549).  The ahead-of-time prefix-blocked walk
// (walk_sparse.hip) avoids the divide by keeping suffix products of 8-row
// blocks, but it must add the whole block (zeros included) and re-multiply
// every block of the prefix.  When the kernel is generated for the pattern at
// hand, every walk step is straight-line code that
//   * adds the flipped column only to the rows it touches (values packed
//     contiguously, one s_load_dwordx16 per 8 of them, SGPR operands of
//     v_add_f64), and
//   * re-forms only the product-tree nodes above those rows (make_tree: rows
//     that change on the same steps share a node).
//
// Paired form.  Gray steps 2j and 2j+1 differ in walk bit 0 only.  Segment 0
// (the rows walk bit 0 touches) is held twice, x (bit 0 clear) and
// y = x + a_0 (bit 0 set), and the pair contributes
//   (-1)^j (prod_seg0 x - prod_seg0 y) * U1,    U1 = product of all other rows,
// accumulated with one fma.  The walk is then a Gray walk over walk bits
// 1..m-1 at half the step count; a step touching segment 0 updates both copies
// and re-forms both products.  The loop is unrolled by 2^b pair steps
// (b chosen per plan, 5..8): pair bits below b get straight-line steps with
// compile-time table offsets (the top one with sign q&1), and every higher
// bit shares one straight-line step over the union of their rows (full signed
// column, zeros included) — a switch over per-bit steps would make LLVM
// carry copies of x across its arms (measured: 120 -> 242 VGPRs).
//
// Cached walk bits.  Walk bits 1..cc (cc <= 3, seg_best) are held in every
// state: each node that depends on them has one copy per state of those
// bits, so their pair steps only accumulate (the state is a compile-time
// constant inside the unrolled block) and the other steps update every copy.
// Only x^0 (walk bits 0..cc clear) is walked; row copies are x^0 + constants
// (seg_cx, seg_cy), and every row or node copy is kept live or formed on
// demand inside its consumer (seg_fit's storage plan) — the same values
// either way.  cc, the storage plan and b are chosen on the exact op count
// within a live-value budget.
//
// D = prod_x - prod_y of segment 0 fuses the x root's product with the
// subtraction into one fma (dexpr).
//
// Measured on MI355X (profiles/r2): n=40 d=0.5 bench matrix 11.6 VALU
// instructions per Gray step (cost model 11.4; round 1 18.2; the prefix-
// blocked AOT walk executes 46.6, the plain dense walk 81), VALU 93% busy at 2
// waves/SIMD, 3.08e12 steps/s.  Everything else (chunk start, lane layout,
// wave-chunk queue, reduction order) is walk_common.hpp's, shared with the
// ahead-of-time kernels, and the arithmetic is mirrored bit for bit by
// engine_cpu.cpp (tree_*, seg_*) and oracle/oracle.c (kind 3).
//
// Lane sum.  Two levels: acc takes the pair terms of one 2^b-pair block and
// folds into a running total after each shared step (8.0e-12 against 2.4e-11
// for one long fma chain on the n = 40 bench matrix, same speed).
//
// Chunk skip.  Rows no walk bit touches (the outer tree's tail) are constant
// over a wave-chunk; when their product is an exact zero in every valid lane
// the chunk's walk is skipped (integer matrices; the planner weighs it:
// config 5 skips 87% of its chunks).
//
// Compiled code objects are cached in memory (per process, per device) and on
// disk: $SUP_JIT_CACHE_DIR, else $XDG_CACHE_HOME/superman_amd, else
// ~/.cache/superman_amd (SUP_JIT_CACHE_DIR="" disables the disk cache).
// Debugging / experiment knobs: SUP_JIT_DUMP=<dir> keeps the generated source,
// SUP_JIT_VERBOSE prints the plan's op count, live values and cached bits;
// SUP_JIT_CC / _B / _STORAGE / _BUDGET / _STARTS / _POLISH / _REGMAX / _KP /
// _PF / _XSTEP / _WAVES / _LDS force cached bits, pair bits, storage budget,
// live-value budget (no compiler check), search starts, skip polish, register
// budget, SGPR pieces per region, prefetch, cross-step regions, occupancy,
// dynamic LDS.
#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sched.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <iterator>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <queue>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <sstream>
#include <tuple>
#include <string_view>
#include <thread>

#include "engine.hpp"
#include "jit_internal.hpp"

namespace sup {

// hiprtc time spent by this thread (and the wall time of compile batches it
// ran on helper threads or processes): per call, not process-wide, so
// concurrent callers do not count each other's compiles (jit_internal.hpp)
thread_local double t_compile_ms = 0.0;
// Set when hiprtc fails on a segmented walk (jit_internal.hpp).
std::atomic<bool> g_jit_failed{false};

namespace {
#include "jit_headers.inc"  // kWalkCommonSrc, kWalkParamsSrc (generated from the headers by the Makefile)

// A kernel with no scratch at all is preferred over one whose spills stay in
// the chunk start unless that one saves more than this fraction of the ops.
constexpr double kScratchTolerance = 0.01;

// ---------------------------------------------------------------- planning --

// Step class of walk bit k >= 1: k - 1 for the specialised pair bits, seg_b
// for the shared step of the walk bits above them.
int step_class(int k, int b) { return k <= b ? k - 1 : b; }

// Copies of a value whose step classes are `sig`: one per state of the cached
// classes (the lowest cc classes) it depends on.
inline int copies(uint32_t sig, int cc) { return 1 << __builtin_popcount(sig & ((1u << cc) - 1u)); }

// Dirty weight of a step-class set: how often (x 2^b per pair step) a value
// with these classes is re-formed, times its copies.  Cached classes never
// re-form anything; class c < b flips on 2^-(c+1) of the pair steps, the
// shared class on ~2^-b.
struct ClassWeights {
  uint64_t w[512];  // classes 0..b, b <= 8
  ClassWeights(int b, int cc) {
    for (uint32_t s = 0; s < 512; ++s) {
      uint64_t v = 0;
      for (int c = cc; c <= b && c < 9; ++c)
        if ((s >> c) & 1u) v += c < b ? (1ull << (b - 1 - c)) : 1ull;
      w[s] = v * (uint64_t)copies(s, cc);
    }
  }
};

// Greedy product tree over the item rows `rows` (+ one constant item for the
// rows [tail_lo, tail_hi), which no walk bit >= 1 touches): repeatedly join the
// two clusters whose union is cheapest to keep, i.e. minimise W(sig_i | sig_j)
// (ClassWeights); ties -> the first pair (i < j) in list order; the joined
// cluster goes to the end.  Rows that change together end up under one node,
// so a step re-forms only the nodes above the rows it touches.
ProdTree make_tree(const std::vector<int>& rows, const std::vector<uint32_t>& rsig, int tail_lo, int tail_hi,
                   const ClassWeights& W) {
  ProdTree t;
  t.tail_lo = tail_lo, t.tail_hi = tail_hi;
  for (int r : rows) t.item_row.push_back(r), t.item_sig.push_back(rsig[r]);
  if (tail_hi > tail_lo) t.item_row.push_back(-1), t.item_sig.push_back(0u);
  std::vector<int> id;
  std::vector<uint32_t> sg;
  for (int i = 0; i < t.items(); ++i) id.push_back(i), sg.push_back(t.item_sig[i]);
  while (id.size() > 1) {
    size_t bi = 0, bj = 1;
    uint64_t bw = UINT64_MAX;
    for (size_t i = 0; i < id.size(); ++i)
      for (size_t j = i + 1; j < id.size(); ++j) {
        const uint64_t w = W.w[(sg[i] | sg[j]) & 511u];
        if (w < bw) bw = w, bi = i, bj = j;
      }
    const uint32_t ns = sg[bi] | sg[bj];
    t.a.push_back(id[bi]), t.b.push_back(id[bj]), t.sig.push_back(ns);
    id.erase(id.begin() + bj), sg.erase(sg.begin() + bj);
    id.erase(id.begin() + bi), sg.erase(sg.begin() + bi);
    id.push_back(t.items() + t.K() - 1), sg.push_back(ns);
  }
  return t;
}

// The segmented walk's structure in engine rows (rows in seg_row_order):
// touched[k] = rows walk bit k touches; segment 0 = rows [0, len0) (walk bit
// 0's rows; [0, s_end) touched by some walk bit >= 1, [s_end, len0) not);
// other rows [len0, r_end) touched by some walk bit >= 1, [r_end, n) by none.
struct SegRows {
  int n = 0, m = 0, b = 0, len0 = 0, s_end = 0, r_end = 0;
  std::vector<std::vector<int>> touched;
  std::vector<int> dyn_rows;      // rows of walk bits > b (the shared step)
  std::vector<uint32_t> rsig;     // step classes of each row
};

void seg_rows_finish(SegRows& R, int b) {
  R.b = b;
  R.rsig.assign(R.n, 0u);
  std::vector<char> dyn(R.n, 0);
  for (int k = 1; k < R.m; ++k)
    for (int r : R.touched[k]) {
      R.rsig[r] |= 1u << step_class(k, R.b);
      if (k > R.b) dyn[r] = 1;
    }
  R.dyn_rows.clear();
  for (int r = 0; r < R.n; ++r)
    if (dyn[r]) R.dyn_rows.push_back(r);
}

struct SegFit {
  int cc = 0;
  double ops = 1e300;   // fp64 VALU ops per Gray step (the generated code, exactly)
  int regs = 0;         // values live across steps (doubles), estimate
  ProdTree outer, inner;
};

// Pair-step frequency (x 2^b) of a value re-formed on the step classes `s`:
// class c < b flips on 2^-(c+1) of the pair steps, the shared class b on
// ~2^-b; cached classes (c < cc) never re-form anything.
inline uint64_t freq(uint32_t s, int b, int cc) {
  uint64_t v = 0;
  for (int c = cc; c <= b && c < 9; ++c)
    if ((s >> c) & 1u) v += c < b ? (1ull << (b - 1 - c)) : 1ull;
  return v;
}

// Live-value budgets (seg_fit's estimate, doubles): <= kRegs3 fits 3 waves
// per SIMD (168 VGPRs), <= kRegsMax fits 2 (256 VGPRs) without spills in the
// walk loop.  The estimate runs above what the compiler allocates (round 1:
// 102 -> 188 VGPRs, 142 -> 246 VGPRs no spill, 205 -> 175 spilled VGPRs).
// Occupancy 2 costs ~2% against 3 on this walk (measured, n = 40), 1 ~35%.
constexpr int kRegs3 = 90;
// The default; long walks check it against the compiler (build_seg: larger
// or smaller budgets by the code object's VGPR spill count).  SUP_JIT_REGMAX
// fixes it (experiments).
static const int kRegsMax = std::getenv("SUP_JIT_REGMAX") ? std::atoi(std::getenv("SUP_JIT_REGMAX")) : 170;
constexpr double kOcc2Penalty = 1.02;

// Trees, cost, live values and the storage plan of every value, with cc
// cached classes, fitted to `budget` live values.
//
// Values.  Only x^0 (the lane state with walk bits 0..cc clear) is walked;
// every other value is a pure function of it: the copy of row r for cached
// state S is x^S_r = x^0_r + cx_r[S] (x^0_r when no bit of S touches r), its
// walk-bit-0 twin y^S_r = x^0_r + cy_r[S] (seg_cx / seg_cy), and a tree node
// copy is the product of its children's copies.  Each row copy and node copy
// set (per tree and variant x / y) is either live — formed on the steps of
// its own classes and kept — or formed on demand inside its nearest live
// ancestor (D for segment 0's roots).  The choice changes no value (the same
// operations on the same operands), only ops and registers: starting from all
// live (segment 0's roots excepted: D reads them once), values are dropped
// greedily by ops added per register freed — first every one that adds
// nothing (a parent formed exactly when the child is: the tree joins equal
// step classes first), then the cheapest until the live values fit `budget`.
SegFit seg_fit(const SegRows& R, int cc, int budget, int budget_hi = -1, SegFit* fit_hi = nullptr) {
  SegFit f;
  f.cc = cc;
  const ClassWeights W(R.b, cc);
  std::vector<int> orow, irow;
  for (int r = R.len0; r < R.r_end; ++r) orow.push_back(r);
  for (int r = 0; r < R.s_end; ++r) irow.push_back(r);
  f.outer = make_tree(orow, R.rsig, R.r_end, R.n, W);
  f.inner = make_tree(irow, R.rsig, R.s_end, R.len0, W);
  struct Val {
    int parent = -1;            // parent value (-1: a root)
    int kids[2] = {-1, -1};
    double fr = 0;              // formations per 2^b pair steps
    int cop = 1;                // copies
    double own = 0;             // own ops to form all copies
    int store = 0;              // registers if live
    bool live = true, fixed = false;
    double F = 0;               // ops to form all copies, non-live descendants included
  };
  std::vector<Val> V;
  // values of tree t over x (yv = false) or y; returns the index of item 0
  auto add_tree = [&](const ProdTree& t, bool yv, bool outer) {
    const int base = (int)V.size();
    for (int id = 0; id < t.items() + t.K(); ++id) {
      Val v;
      uint32_t sig;
      if (id < t.items()) {
        const int r = t.item_row[id];
        sig = r < 0 ? 0u : R.rsig[r];
        v.cop = copies(sig, cc);
        v.store = r < 0 ? 0 : (yv ? v.cop : v.cop - 1);  // x^0 itself needs no copy
        v.own = v.store;
        v.fixed = v.store == 0;
      } else {
        const int i = id - t.items();
        sig = t.sig[i];
        v.cop = copies(sig, cc);
        v.own = v.store = v.cop;
        v.kids[0] = base + t.a[i], v.kids[1] = base + t.b[i];
      }
      v.fr = (double)freq(sig, R.b, cc);
      V.push_back(v);
    }
    for (int i = 0; i < t.K(); ++i) V[base + t.a[i]].parent = V[base + t.b[i]].parent = base + t.items() + i;
    if (t.root() >= 0) {
      Val& rt = V[base + t.root()];
      if (outer) rt.fixed = true;           // the outer root: read by every accumulate
      else if (!rt.fixed) rt.live = false;  // segment 0's roots: read by D only
    }
    return base;
  };
  const int bo = add_tree(f.outer, false, true), bx = add_tree(f.inner, false, false),
            by = add_tree(f.inner, true, false);
  const uint32_t dsig = f.inner.root() >= 0 ? f.inner.root_sig() : 0u;
  const double fD = (double)freq(dsig, R.b, cc);
  const int cD = copies(dsig, cc);
  double xadds = 0;
  for (int r = 0; r < R.n; ++r) xadds += (double)freq(R.rsig[r], R.b, cc);
  auto total = [&](int* regs) {
    for (auto& v : V) {  // children precede parents
      v.F = v.own;
      for (int k : v.kids)
        if (k >= 0 && !V[k].live) v.F += (double)v.cop / V[k].cop * V[k].F;
    }
    double ops = xadds;
    int rg = 6 + R.n;  // x^0, acc, tot, loop state
    for (auto& v : V)
      if (v.live) ops += v.fr * v.F, rg += v.store;
    if (f.inner.root() >= 0) {  // D per copy: the sub (fused with a root node's mul) and its non-live tops
      ops += f.inner.K() ? 0.0 : fD * cD;
      for (int rt : {bx + f.inner.root(), by + f.inner.root()})
        if (!V[rt].live) ops += fD * (double)cD / V[rt].cop * V[rt].F;
      rg += cD;
    }
    *regs = rg;
    return ops;
  };
  // values formed exactly as often as their parent (same step classes, same
  // copies) cost nothing on demand: all at once (a chain of them keeps the
  // property up to its nearest live ancestor)
  for (auto& v : V)
    if (v.live && !v.fixed && v.parent >= 0 && V[v.parent].fr * V[v.parent].cop == v.fr * v.cop) v.live = false;
  for (const int rt : {bx + f.inner.root(), by + f.inner.root()})
    if (f.inner.root() >= 0)
      for (int k : V[rt].kids)  // children of segment 0's roots: consumer D
        if (k >= 0 && V[k].live && !V[k].fixed && fD * cD == V[k].fr * V[k].cop) V[k].live = false;
  int regs = 0;
  double ops = total(&regs);
  // the decisions: bit 0 over x, bit 1 over y
  auto out = [&](SegFit& g, double ops_now, int regs_now) {
    g.cc = cc;
    g.outer = f.outer, g.inner = f.inner;
    auto put = [&](ProdTree& t, int base, int bit) {
      t.item_live.assign(t.items(), 0);
      t.node_live.assign(t.K(), 0);
      for (int j = 0; j < t.items(); ++j)
        if (V[base + j].live && !V[base + j].fixed) t.item_live[j] |= (uint8_t)(1u << bit);
      for (int i = 0; i < t.K(); ++i)
        if (V[base + t.items() + i].live) t.node_live[i] |= (uint8_t)(1u << bit);
    };
    put(g.outer, bo, 0);
    put(g.inner, bx, 0);
    for (int j = 0; j < g.inner.items(); ++j)
      if (V[by + j].live && !V[by + j].fixed) g.inner.item_live[j] |= 2u;
    for (int i = 0; i < g.inner.K(); ++i)
      if (V[by + g.inner.items() + i].live) g.inner.node_live[i] |= 2u;
    g.ops = (ops_now / (double)(1u << R.b) + 1.0) / 2.0;  // + the accumulate fma; pair -> Gray steps
    g.regs = regs_now;
  };
  bool took_hi = fit_hi == nullptr;
  // Greedy with a lazy heap: removing V changes only the F of its ancestors
  // up to its nearest live ancestor A (A's own entry) and the consumer of the
  // live values nearest below V (now A): only those entries are renewed.
  auto nearest_live = [&](int i) {
    int a = V[i].parent;
    while (a >= 0 && !V[a].live) a = V[a].parent;
    return a;
  };
  auto delta = [&](int i) {
    const int a = nearest_live(i);
    const double fa = a >= 0 ? V[a].fr : fD, ca = a >= 0 ? V[a].cop : cD;
    return V[i].F * (fa * ca / V[i].cop - V[i].fr);
  };
  typedef std::tuple<double, int, int> Entry;  // (ops added per register, value, version)
  std::priority_queue<Entry, std::vector<Entry>, std::greater<Entry>> heap;
  std::vector<int> ver(V.size(), 0);
  std::vector<double> dlt(V.size(), 0.0);
  auto push = [&](int i) {
    if (!V[i].live || V[i].fixed) return;
    dlt[i] = delta(i);
    heap.push(Entry{dlt[i] / V[i].store, i, ++ver[i]});
  };
  for (int i = 0; i < (int)V.size(); ++i) push(i);
  std::vector<int> stack;
  for (;;) {
    while (!heap.empty() && std::get<2>(heap.top()) != ver[std::get<1>(heap.top())]) heap.pop();  // stale
    const int best = heap.empty() ? -1 : std::get<1>(heap.top());
    const double bd = best < 0 ? 0.0 : dlt[best];
    // the larger budget's plan is the state where its greedy would stop
    if (!took_hi && (best < 0 || (bd > 1e-9 && regs <= budget_hi))) out(*fit_hi, ops, regs), took_hi = true;
    if (best < 0 || (bd > 1e-9 && regs <= budget)) break;
    heap.pop();
    V[best].live = false;
    ++ver[best];
    ops += bd, regs -= V[best].store;
    for (int p = V[best].parent; p >= 0; p = V[p].parent) {  // F up to the nearest live ancestor
      V[p].F += (double)V[p].cop / V[best].cop * V[best].F;
      if (V[p].live) {
        push(p);
        break;
      }
    }
    stack.assign(1, best);  // live values nearest below: new consumer
    while (!stack.empty()) {
      const int u = stack.back();
      stack.pop_back();
      for (int k : V[u].kids)
        if (k >= 0) {
          if (V[k].live) push(k);
          else stack.push_back(k);
        }
    }
  }
  if (!took_hi) out(*fit_hi, ops, regs);
  out(f, ops, regs);
  return f;
}

// Best number of cached classes (0 .. min(kMaxCachedBits, b-1)) within the
// register budget.
std::atomic<long> g_fit_calls{0};  // planning effort (SUP_JIT_VERBOSE)
// Live-value budget the walk-order search prices orders at (SUP_JIT_SEARCH_BUDGET
// for experiments; the compiler check then refits the chosen order).
int search_budget() {
  static const int b = std::getenv("SUP_JIT_SEARCH_BUDGET") ? std::atoi(std::getenv("SUP_JIT_SEARCH_BUDGET")) : kRegsMax;
  return b;
}

// Cap on the cached walk bits the planner tries: kMaxCachedBits, or lower with
// SUP_JIT_MAXCC (experiments: A/B against fewer cached bits with the budget
// check still on).
int max_cached() {
  const char* e = std::getenv("SUP_JIT_MAXCC");
  return e ? std::max(0, std::min(kMaxCachedBits, std::atoi(e))) : kMaxCachedBits;
}

SegFit seg_best(const SegRows& R, int cc_max, int regs_max = kRegsMax) {
  ++g_fit_calls;
  SegFit best;
  double bscore = 1e300;
  for (int cc = 0; cc <= std::min(cc_max, std::max(0, R.b - 1)); ++cc) {
    SegFit hi;
    SegFit lo = seg_fit(R, cc, kRegs3, regs_max, &hi);  // one greedy: both budgets' plans
    for (SegFit* f : {&lo, &hi}) {
      if (f->regs > regs_max && cc > 0) continue;
      const double score = f->ops * (f->regs <= kRegs3 ? 1.0 : kOcc2Penalty) * (f->regs > regs_max ? 2.0 : 1.0);
      if (score < bscore) bscore = score, best = std::move(*f);
    }
  }
  return best;
}

// SegRows of walk columns `walk` in the engine row order make_plan uses,
// with b specialised pair bits.
SegRows seg_rows_of(const double* A, int n, const std::vector<int>& walk, int b) {
  SegRows R;
  R.n = n, R.m = (int)walk.size();
  const std::vector<int> order = seg_row_order(A, n, walk);
  auto nz = [&](int row, int c) { return A[(size_t)row * n + c] != 0.0; };
  R.touched.assign(R.m, {});
  std::vector<char> any1(n, 0);
  for (int k = 0; k < R.m; ++k)
    for (int j = 0; j < n; ++j)
      if (nz(order[j], walk[k])) {
        R.touched[k].push_back(j);
        if (k >= 1) any1[j] = 1;
      }
  R.len0 = (int)R.touched[0].size();
  R.s_end = 0;
  while (R.s_end < R.len0 && any1[R.s_end]) ++R.s_end;
  R.r_end = R.len0;
  while (R.r_end < n && any1[R.r_end]) ++R.r_end;
  seg_rows_finish(R, b);
  return R;
}

// Score of a fit: ops per Gray step, 2% more when it needs the 2-wave budget.
double seg_score(const SegFit& f) { return f.ops * (f.regs <= kRegs3 ? 1.0 : kOcc2Penalty); }

// Instruction bytes of the unrolled 2^b-pair block (the loop body), estimated
// from the op count: 2 * ops per Gray step per pair step, 8 B per fp64 VOP3
// instruction, +25% for the scalar loads, branches and sched barriers.  The
// block must stay well inside the 64 KB instruction cache two CUs share.
constexpr double kMaxBlockBytes = 40.0 * 1024.0;
double seg_block_bytes(const SegFit& f, int b) { return 1.25 * 8.0 * 2.0 * f.ops * (double)(1u << b); }

// Candidate specialised pair-bit counts for m walk bits: SUP_JIT_B forces one
// (experiments), else 5..8 (fewer when the walk is shorter).  More pair bits
// make the shared step of the higher walk bits rarer (it adds the full column
// to the union of their rows) and let more rows keep a class of their own, at
// 2x the code per bit (measured on MI355X, profiles/r2/probe_b.log: the n = 40
// d = 0.5 bench matrix 2.06e12 Gray steps/s at b = 5, 2.14e12 at 6, 2.05e12 at
// 7, each as its op count predicts; config 5 3.57e13 / 3.95e13 / 5.13e13).
std::vector<int> seg_b_candidates(int m) {
  std::vector<int> v;
  if (const char* e = std::getenv("SUP_JIT_B")) {
    v.push_back(std::min(m - 1, std::max(3, std::min(8, std::atoi(e)))));
    return v;
  }
  for (int b = 5; b <= 8; ++b) {
    const int bb = std::min(m - 1, b);
    if (v.empty() || v.back() != bb) v.push_back(bb);
  }
  return v;
}

}  // namespace

// Default specialised pair bits when no choice was made (SUP_JIT_B forces, 3..8)
int seg_static_bits(int m) {
  int b = 5;
  if (const char* e = std::getenv("SUP_JIT_B")) b = std::max(3, std::min(8, std::atoi(e)));
  return std::min(m - 1, b);
}

double seg_walk_cost(const Plan& P) { return P.seg_ops; }

// Greedy starts the walk-order descent runs from (SUP_JIT_STARTS overrides):
// 32 when the plain walk would take a second or more on one MI355X (2n + 1 ops
// per Gray step at 3.7e13 lane-ops/s: n >= 40), else 3.  More starts find
// cheaper walks (n = 40 bench matrix: 13.05 ops per step from 3 starts, 12.66
// from 8 before the fused D; after it 12.16 from 8 or 16, 11.93 from 32 or
// 64); the descents run on plan_threads() host threads (32 starts: 1.7 s on 8).
// Host threads for the plan's searches: the machine's, at most OMP_NUM_THREADS
// (the GPU box's CPU share) and 16.
int plan_threads() {
  int t = (int)std::max(1u, std::thread::hardware_concurrency());
  if (const char* e = std::getenv("OMP_NUM_THREADS")) t = std::min(t, std::max(1, std::atoi(e)));
  return std::min(t, 16);
}

// Run fn(0..count-1) on up to plan_threads() host threads (the caller's
// included); results are gathered by index, so they do not depend on timing.
void parallel_tasks(size_t count, const std::function<void(size_t)>& fn, int max_threads = 1 << 20) {
  std::atomic<size_t> next{0};
  auto worker = [&]() {
    for (size_t i = next++; i < count; i = next++) fn(i);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < std::min({plan_threads(), (int)count, max_threads}); ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
}

int seg_search_starts(int n) {
  if (const char* e = std::getenv("SUP_JIT_STARTS")) return std::max(1, std::atoi(e));
  return std::ldexp(1.0, n - 1) * (2.0 * n + 1.0) / 3.7e13 >= 1.0 ? 32 : 3;
}

std::vector<int> seg_walk_order(const double* A, int n, int m, int count, int* b_out, int cc_cap) {
  cc_cap = std::min(cc_cap, max_cached());
  const int nb = n - 1;
  m = std::min(m, nb);
  count = std::min(std::max(count, m), nb);
  std::vector<int> nnz(n, 0);
  for (int c = 0; c < nb; ++c)
    for (int i = 0; i < n; ++i) nnz[c] += A[(size_t)i * n + c] != 0.0;
  // greedy continuation: fewest newly touched rows, then fewest nonzeros, then lowest index
  auto extend = [&](std::vector<int> order, int upto) {
    std::vector<char> used(n, 0), placed(n, 0);
    for (int c : order) {
      used[c] = 1;
      for (int i = 0; i < n; ++i) placed[i] |= A[(size_t)i * n + c] != 0.0;
    }
    while ((int)order.size() < upto) {
      int best = -1, bnew = 1 << 30;
      for (int c = 0; c < nb; ++c) {
        if (used[c]) continue;
        int nw = 0;
        for (int i = 0; i < n; ++i) nw += !placed[i] && A[(size_t)i * n + c] != 0.0;
        if (nw < bnew || (nw == bnew && nnz[c] < nnz[best])) best = c, bnew = nw;
      }
      used[best] = 1;
      order.push_back(best);
      for (int i = 0; i < n; ++i) placed[i] |= A[(size_t)i * n + best] != 0.0;
    }
    return order;
  };
  // the exact op count of the generated code (best cached-class count within
  // the register budget); walk bit 0 defines segment 0 (the paired rows) and
  // must touch a row
  auto cost = [&](const std::vector<int>& o, int b) {
    if (nnz[o[0]] == 0) return 1e300;
    if (m < 3) return 0.0;
    const SegFit f = seg_best(seg_rows_of(A, n, std::vector<int>(o.begin(), o.begin() + m), b), cc_cap,
                              search_budget());
    return seg_block_bytes(f, b) > kMaxBlockBytes ? 1e300 : seg_score(f);
  };
  if (m == 0) {
    if (b_out) *b_out = 0;
    return extend({}, count);
  }
  // one search per candidate b (the best order differs with b), each on its
  // own host thread; the cheapest (order, b) wins, ties -> the smaller b
  const std::vector<int> cands = seg_b_candidates(m);
  std::vector<std::vector<int>> bests(cands.size());
  std::vector<std::vector<std::pair<double, std::vector<int>>>> finals(cands.size());
  std::vector<double> bcosts(cands.size(), 1e300);
  // phase 1, one host thread per b: greedy continuations from every first
  // column, ranked by cost
  std::vector<std::vector<std::pair<double, std::vector<int>>>> starts(cands.size());
  auto rank_starts = [&](size_t ci) {
    const int b = cands[ci];
    for (int f = 0; f < nb; ++f) {
      std::vector<int> o = extend({f}, m);
      starts[ci].push_back({cost(o, b), std::move(o)});
    }
    std::stable_sort(starts[ci].begin(), starts[ci].end(),
                     [](const std::pair<double, std::vector<int>>& x, const std::pair<double, std::vector<int>>& y) {
                       return x.first < y.first;
                     });
  };
  {
    std::vector<std::thread> th;
    for (size_t ci = 1; ci < cands.size(); ++ci) th.emplace_back(rank_starts, ci);
    rank_starts(0);
    for (auto& t : th) t.join();
  }
  // phase 2: a descent from each of the seg_search_starts(n) cheapest starts
  // of every b — swap a walk position with another walk position or an unused
  // column while the cost drops (positions whose weight 2^-(k+1) is visible) —
  // as independent tasks on a pool of host threads; every result is a final
  // candidate (deterministic: gathered in (b, start) order)
  const int hot = std::min(m, 12);
  const size_t nstart = std::min((size_t)nb, (size_t)seg_search_starts(n));
  std::vector<std::pair<size_t, size_t>> tasks;
  for (size_t si = 0; si < nstart; ++si)
    for (size_t ci = 0; ci < cands.size(); ++ci) tasks.push_back({ci, si});
  std::vector<std::pair<double, std::vector<int>>> results(tasks.size());
  auto descend = [&](size_t ti) {
    const size_t ci = tasks[ti].first, si = tasks[ti].second;
    const int b = cands[ci];
    std::vector<int> cur = starts[ci][si].second;
    double ccost = starts[ci][si].first;
    for (int pass = 0; pass < 8 && ccost < 1e300; ++pass) {
      bool improved = false;
      for (int a = 0; a < hot; ++a) {
        for (int c = 0; c < nb; ++c) {
          if (c == cur[a]) continue;
          std::vector<int> o = cur;
          auto it = std::find(o.begin(), o.end(), c);
          if (it != o.end()) std::swap(o[a], *it);
          else o[a] = c;
          const double v = cost(o, b);
          if (v < ccost - 1e-12) ccost = v, cur = o, improved = true;
        }
      }
      if (!improved) break;
    }
    results[ti] = {ccost, std::move(cur)};
  };
  {
    std::atomic<size_t> next{0};
    auto worker = [&]() {
      for (size_t ti = next++; ti < tasks.size(); ti = next++) descend(ti);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < std::min<int>(plan_threads(), (int)tasks.size()); ++t) th.emplace_back(worker);
    worker();
    for (auto& t : th) t.join();
  }
  for (size_t ci = 0; ci < cands.size(); ++ci) finals[ci].clear();
  for (size_t ti = 0; ti < tasks.size(); ++ti) {
    const size_t ci = tasks[ti].first;
    if (bests[ci].empty() || results[ti].first < bcosts[ci] - 1e-12) bcosts[ci] = results[ti].first, bests[ci] = results[ti].second;
    finals[ci].push_back(results[ti]);
  }
  size_t gi = 0;
  for (size_t ci = 1; ci < cands.size(); ++ci)
    if (bcosts[ci] < bcosts[gi] - 1e-12) gi = ci;
  // Integer matrices: the kernel skips wave-chunks whose walk-untouched rows
  // hold an exact zero in every lane, which the op count does not see; the
  // final candidates are compared on ops x (1 - sampled skip fraction).
  bool integral = true;
  for (size_t i = 0; i < (size_t)n * n && integral; ++i) integral = A[i] == std::floor(A[i]);
  // swap descent of order `bo` (b = bb) on ops x (1 - skip), kPolishSamples
  // sampled chunks per trial (the same chunks for every trial); returns the
  // final eff and leaves the order in bo.  512 samples overfit: on config 5
  // the descent's best at 512 (0.176 ops per nominal step) measured 0.216.
  constexpr int kPolishSamples = 8192;
  constexpr int kPolishEvals = 48;
  // Shard balance: make_plan puts the high columns that touch no
  // walk-untouched row (they never change a skip) on the top chunk bits, so
  // contiguous shards of 2, 4, 8 GPUs see the same skips only when there are
  // at least 3 of them (min(3, high bits)).  Orders with fewer are not taken
  // (config 5 with 16 polish starts: the best order had fewer, and 4 of 8
  // shards walked nothing).
  const int need_free = std::min(3, std::max(0, nb - count));
  auto balanced = [&](const std::vector<int>& full) {
    std::vector<char> wrow(n, 0), used(n, 0);
    for (int k = 0; k < m; ++k)
      for (int i = 0; i < n; ++i) wrow[i] |= A[(size_t)i * n + full[k]] != 0.0;
    for (int c : full) used[c] = 1;
    int free_cols = 0;
    for (int c = 0; c < nb; ++c) {
      if (used[c]) continue;
      bool f = true;
      for (int i = 0; i < n && f; ++i) f = wrow[i] || A[(size_t)i * n + c] == 0.0;
      free_cols += f;
    }
    return free_cols >= need_free;
  };
  auto polish = [&](std::vector<int>& bo, int bb, double beff) {
    if (!balanced(extend(bo, count))) beff = 1e300;  // any balanced order improves on it
    const int npos = std::min(count, m + std::min(6, nb - m));
    std::vector<int> cur(bo.begin(), bo.begin() + npos);
    double cur_ops = cost(std::vector<int>(cur.begin(), cur.begin() + m), bb);
    // best-improvement passes: every swap's skip first (2048 samples), then
    // for the kPolishEvals most promising by the optimistic bound 0.85 x ops
    // x (1 - skip) (one swap rarely cuts the ops by 15 %) the op count (a
    // storage fit) and the skip on all samples
    for (int pass = 0; pass < 16; ++pass) {
      std::vector<std::tuple<double, bool, std::vector<int>>> trials;  // (1 - skip, walk unchanged, order)
      for (int a = 0; a < npos; ++a)
        for (int c = 0; c < nb; ++c) {
          if (c == cur[a]) continue;
          std::vector<int> o = cur;
          auto it = std::find(o.begin(), o.end(), c);
          const bool walk_same = a >= m && (it == o.end() || it - o.begin() >= m);
          if (it != o.end()) std::swap(o[a], *it);
          else o[a] = c;
          trials.emplace_back(1.0 - seg_skip_estimate(A, n, extend(o, count), m, kPolishSamples / 4), walk_same,
                              std::move(o));
        }
      std::stable_sort(trials.begin(), trials.end(),
                       [](const auto& x, const auto& y) { return std::get<0>(x) < std::get<0>(y); });
      double best = beff;
      int bi = -1;
      double bops = cur_ops;
      for (size_t t = 0; t < trials.size() && (int)t < kPolishEvals; ++t) {
        if (cur_ops * 0.85 * std::get<0>(trials[t]) >= best) break;
        const std::vector<int>& o = std::get<2>(trials[t]);
        if (!balanced(extend(o, count))) continue;
        const double keep = 1.0 - seg_skip_estimate(A, n, extend(o, count), m, kPolishSamples);
        const double ops = std::get<1>(trials[t]) ? cur_ops : cost(std::vector<int>(o.begin(), o.begin() + m), bb);
        if (ops < 1e300 && ops * keep < best - 1e-12) best = ops * keep, bi = (int)t, bops = ops;
      }
      if (bi < 0) break;
      beff = best, cur = std::get<2>(trials[bi]), cur_ops = bops;
    }
    bo = extend(cur, count);
    return beff;
  };
  if (integral && count >= m + std::min(6, nb - m)) {
    double beff = 1e300;
    std::vector<int> bo;
    int bb = cands[gi];
    std::vector<std::tuple<double, int, std::vector<int>>> ranked;  // (eff, b, order)
    for (size_t ci = 0; ci < cands.size(); ++ci)
      for (const auto& fc : finals[ci]) {
        if (fc.first >= 1e300) continue;
        const std::vector<int> full = extend(fc.second, count);
        const double eff = balanced(full) ? fc.first * (1.0 - seg_skip_estimate(A, n, full, m, kPolishSamples)) : 1e300;
        if (std::getenv("SUP_JIT_VERBOSE"))
          std::fprintf(stderr, "  candidate b=%d ops=%.4f skip=%.3f eff=%.4f\n", cands[ci], fc.first,
                       1.0 - eff / fc.first, eff);
        ranked.emplace_back(eff, cands[ci], full);
        if (eff < beff - 1e-12) beff = eff, bo = full, bb = cands[ci];
      }
    if (!bo.empty()) {
      // polish: swap descent on ops x (1 - skip) (SUP_JIT_POLISH=0 skips
      // it) of the kPolish best distinct candidates (16; SUP_JIT_NPOLISH), one
      // host thread each; the best result wins.  The descent is local and its
      // end varies a lot with the start: on config 5 (n = 44 d = 0.15 int,
      // up to 4 cached bits) the 16 starts end at 0.15-0.42 ops per nominal
      // step, the 4 best-ranked ones all at 0.36-0.37 (planning 5.8 s with 4
      // starts, 7.5 s with 16 on 8 host threads).
      // Every walk position and the lane columns (positions m .. m+L-1) are
      // polished: the lanes cost no ops, and with the walk columns they
      // decide which rows stay untouched (config 5: 0.205 -> 0.201 against
      // the first 12 walk positions only).
      const char* pe = std::getenv("SUP_JIT_POLISH");
      if (!pe || std::atoi(pe) != 0) {
        const int kPolish = std::getenv("SUP_JIT_NPOLISH") ? std::max(1, std::atoi(std::getenv("SUP_JIT_NPOLISH"))) : 16;
        std::stable_sort(ranked.begin(), ranked.end(),
                         [](const auto& x, const auto& y) { return std::get<0>(x) < std::get<0>(y); });
        std::vector<std::tuple<double, int, std::vector<int>>> starts;
        for (const auto& r : ranked) {
          bool dup = false;
          for (const auto& q : starts) dup |= std::get<1>(q) == std::get<1>(r) && std::get<2>(q) == std::get<2>(r);
          if (!dup) starts.push_back(r);
          if ((int)starts.size() == kPolish) break;
        }
        std::vector<double> effs(starts.size());
        std::vector<std::thread> th;
        for (size_t i = 0; i < starts.size(); ++i)
          th.emplace_back([&, i] { effs[i] = polish(std::get<2>(starts[i]), std::get<1>(starts[i]), std::get<0>(starts[i])); });
        for (auto& t : th) t.join();
        if (std::getenv("SUP_JIT_VERBOSE"))
          for (size_t i = 0; i < starts.size(); ++i) {
            const std::vector<int>& o = std::get<2>(starts[i]);
            const double ops = cost(std::vector<int>(o.begin(), o.begin() + m), std::get<1>(starts[i]));
            std::fprintf(stderr, "  polished #%zu b=%d eff=%.4f ops=%.4f eff@16384=%.4f\n", i, std::get<1>(starts[i]),
                         effs[i], ops, ops * (1.0 - seg_skip_estimate(A, n, o, m, 16384)));
          }
        size_t bi = 0;
        for (size_t i = 1; i < starts.size(); ++i)
          if (effs[i] < effs[bi] - 1e-12) bi = i;
        beff = effs[bi], bb = std::get<1>(starts[bi]), bo = std::get<2>(starts[bi]);
        if (std::getenv("SUP_JIT_VERBOSE")) std::fprintf(stderr, "  polished eff=%.4f\n", beff);
      }
      if (b_out) *b_out = bb;
      return bo;
    }
  }
  if (b_out) *b_out = cands[gi];
  return extend(bests[gi], count);
}

double seg_skip_fraction_plan(const Plan& P, int samples) {
  const int n = P.n, L = P.lay.L, m = P.lay.m, nb = n - 1;
  const int tail_lo = P.seg_start.empty() ? n : P.seg_start.back();
  if (tail_lo >= n) return 0.0;
  for (const double v : P.cols)
    if (v != std::floor(v)) return 0.0;  // exact zeros need integer entries
  const int h = nb - L - m;
  int skipped = 0;
  std::vector<double> base(n - tail_lo);
  for (int s = 0; s < samples; ++s) {
    const uint64_t a = h > 0 ? ((uint64_t)s * 0x9E3779B97F4A7C15ull) >> (64 - std::min(h, 63)) : 0;
    const uint64_t g = a ^ (a >> 1);
    for (int r = tail_lo; r < n; ++r) {
      double v = P.x0[r];
      for (int k = 0; k < h; ++k)
        if ((g >> k) & 1u) v += P.cols[(size_t)(2 * (L + m + k)) * P.NP + r];
      base[r - tail_lo] = v;
    }
    bool all = true;
    for (unsigned lane = 0; lane < (1u << L) && all; ++lane) {
      bool zero = false;
      for (int r = tail_lo; r < n && !zero; ++r) {
        double v = base[r - tail_lo];
        for (int e = 0; e < L; ++e)
          if ((lane >> e) & 1u) v += P.cols[(size_t)(2 * e) * P.NP + r];
        zero = v == 0.0;
      }
      all = zero;
    }
    skipped += all;
  }
  return (double)skipped / samples;
}

double seg_skip_estimate(const double* A, int n, const std::vector<int>& order, int m, int samples) {
  const int nb = n - 1, L = std::min(6, nb - m);
  if ((int)order.size() < m + L) return 0.0;
  std::vector<char> walk(n, 0), used(n, 0);
  for (int k = 0; k < m; ++k) walk[order[k]] = used[order[k]] = 1;
  for (int e = 0; e < L; ++e) used[order[m + e]] = 1;
  std::vector<int> high;  // high (chunk) bits: the unused columns in matrix order (make_plan)
  for (int c = 0; c < nb; ++c)
    if (!used[c]) high.push_back(c);
  std::vector<int> tail;  // rows no walk column touches
  for (int r = 0; r < n; ++r) {
    bool t = true;
    for (int c = 0; c < nb && t; ++c) t = !(walk[c] && A[(size_t)r * n + c] != 0.0);
    if (t) tail.push_back(r);
  }
  if (tail.empty()) return 0.0;
  std::vector<double> x0(n);
  double p0;
  nw_start(A, n, x0.data(), &p0);
  const int h = (int)high.size();
  // Integer entries (x0 half-integers): every sum below is exact, so tail row
  // r is zero in lane l iff its chunk value == -(its lane columns' sum over
  // l).  Per row: its nonzero high-column entries and the distinct lane sums
  // with the mask of lanes holding each; a chunk is skipped when the rows'
  // zero-lane masks cover every lane.
  struct Row {
    double x0;
    std::vector<std::pair<int, double>> hi;         // (chunk bit, entry)
    std::vector<std::pair<double, uint64_t>> lane;  // (-lane sum, lanes)
  };
  const uint64_t all_lanes = L >= 6 ? ~0ull : (1ull << (1u << L)) - 1ull;
  std::vector<Row> rows(tail.size());
  for (size_t i = 0; i < tail.size(); ++i) {
    const double* a = A + (size_t)tail[i] * n;
    rows[i].x0 = x0[tail[i]];
    for (int k = 0; k < h; ++k)
      if (a[high[k]] != 0.0) rows[i].hi.push_back({k, a[high[k]]});
    for (unsigned l = 0; l < (1u << L); ++l) {
      double v = 0.0;
      for (int e = 0; e < L; ++e)
        if ((l >> e) & 1u) v += a[order[m + e]];
      auto it = std::find_if(rows[i].lane.begin(), rows[i].lane.end(), [&](const auto& q) { return q.first == -v; });
      if (it == rows[i].lane.end()) rows[i].lane.push_back({-v, 1ull << l});
      else it->second |= 1ull << l;
    }
  }
  int skipped = 0;
  for (int s = 0; s < samples; ++s) {
    const uint64_t a = h ? ((uint64_t)s * 0x9E3779B97F4A7C15ull) >> (64 - std::min(h, 63)) : 0;
    const uint64_t g = a ^ (a >> 1);
    uint64_t zero = 0;
    for (size_t i = 0; i < rows.size() && zero != all_lanes; ++i) {
      double v = rows[i].x0;
      for (const auto& q : rows[i].hi)
        if ((g >> q.first) & 1u) v += q.second;
      for (const auto& q : rows[i].lane)
        if (v == q.first) zero |= q.second;
    }
    skipped += zero == all_lanes;
  }
  return (double)skipped / samples;
}

std::vector<int> seg_row_order(const double* A, int n, const std::vector<int>& walk) {
  std::vector<int> order;
  std::vector<char> placed(n, 0), in0(n, 0);
  for (int i = 0; i < n; ++i) in0[i] = !walk.empty() && A[(size_t)i * n + walk[0]] != 0.0;
  for (size_t k = 1; k < walk.size(); ++k)  // segment 0, by first touch among walk[1..]
    for (int i = 0; i < n; ++i)
      if (in0[i] && !placed[i] && A[(size_t)i * n + walk[k]] != 0.0) placed[i] = 1, order.push_back(i);
  for (int i = 0; i < n; ++i)
    if (in0[i] && !placed[i]) placed[i] = 1, order.push_back(i);
  for (size_t k = 1; k < walk.size(); ++k)  // the other segments
    for (int i = 0; i < n; ++i)
      if (!placed[i] && A[(size_t)i * n + walk[k]] != 0.0) placed[i] = 1, order.push_back(i);
  for (int i = 0; i < n; ++i)
    if (!placed[i]) order.push_back(i);
  return order;
}

// ----------------------------------------------------------------- codegen --

// Constants of the row copies (seg_fit): a_k(r) = the + column of walk bit k
// at engine row r; cx_r[S] = a_{k(low)}(r) (+ cx_r[S \ low]) for the lowest
// set bit low of S (walk bit k(low) = ctz(low) + 1), cy_r[S] = a_0(r) (+ cx_r[S]).
double seg_cx(const Plan& P, int r, uint32_t S) {
  const uint32_t low = S & (0u - S), rest = S ^ low;
  const int k = __builtin_ctz(low) + 1;
  const double a = P.cols[(size_t)(2 * (P.lay.L + k)) * P.NP + r];
  return rest ? seg_cx(P, r, rest) + a : a;
}
double seg_cy(const Plan& P, int r, uint32_t S) {
  const double a0 = P.cols[(size_t)(2 * P.lay.L) * P.NP + r];
  return S ? a0 + seg_cx(P, r, S) : a0;
}

namespace {

std::string tree(int lo, int hi, const char* v = "x") {
  if (hi - lo == 1) return std::string(v) + "[" + std::to_string(lo) + "]";
  const int mid = lo + (hi - lo + 1) / 2;
  return "(" + tree(lo, mid, v) + " * " + tree(mid, hi, v) + ")";
}

// submasks of m in increasing order (0 included)
std::vector<uint32_t> submasks(uint32_t m) {
  std::vector<uint32_t> v;
  for (uint32_t s = 0; s <= m; ++s)
    if ((s & ~m) == 0) v.push_back(s);
  return v;
}

// A statement of a step whose operands may read constants of the step's
// constant stream: "@<i>@" in `text` stands for the stream's i-th value.
struct Stmt {
  std::string text;
};

// Generated kernel (paired segmented walk).  Gray steps 2j and 2j+1 differ in
// walk bit 0 only, so they are evaluated together: segment 0 (the rows walk
// bit 0 touches) is held twice, x (bit 0 clear) and y = x + a_0 (bit 0 set),
// and the pair contributes (-1)^j (prod_seg0 x - prod_seg0 y) * U1, U1 being
// the product of every other row.  The pair walk is a Gray walk over walk
// bits 1..m-1 (pair bit p = walk bit p+1).  Both products are product trees
// (make_tree): a step re-forms the nodes above the rows it touches.
// Cached classes (walk bits 1..cc): every node that depends on them is held
// in each of their states, so their pair steps only accumulate (the state is
// known at compile time inside the unrolled block) and every other step
// updates all copies.  Only x[r] (x^0) is walked; the row copies x^S, y^S are
// x[r] + a constant (seg_cx / seg_cy), kept live or formed on demand inside
// the node that reads them (ProdTree::item_live).
//
// Names: x[r] = x^0_r; live copies x<r>_<S> (S != 0) and y[r] / y<r>_<S>;
// node i of a tree <N><i>_<copy>, copy = state masked to the node's classes;
// constant items (tails) <T>; D<S> = top_x - top_y of segment 0.
struct Gen {
  const Plan& P;
  int len0;
  uint32_t ccm;
  std::vector<uint32_t> rsig;
  std::ostringstream o;
  // constant directory (init): (row, S, variant) -> index into the jtab tail
  std::map<std::tuple<int, uint32_t, int>, int> cdir;
  std::vector<double> ctab;          // appended to P.jtab at cbase
  size_t cbase = 0;
  std::vector<int> kofs;             // per step class: offset (doubles, from cbase) of its stream
  // per step class: position (doubles, from cbase) of its idx-th constant —
  // kofs[c] + idx, or a place in another class's stream that holds the same
  // value (share_streams: a class whose constants another stream already
  // holds, in an order that costs no extra pieces, emits no stream of its own)
  std::vector<std::vector<int>> cpos;
  std::vector<char> own_stream;
  std::vector<std::vector<Stmt>> cls_stmts;
  std::vector<std::vector<double>> cls_consts;
  // which tree item holds row r: (tree 0 outer / 1 inner, item)
  std::vector<std::pair<int, int>> item_of;

  explicit Gen(const Plan& p) : P(p), len0(p.seg_start[1]), ccm((1u << p.seg_cc) - 1u), rsig(p.n, 0u) {
    for (int k = 1; k < p.lay.m; ++k)
      for (int r : p.touched[k]) rsig[r] |= 1u << step_class(k, p.seg_b);
    item_of.assign(p.n, {-1, -1});
    for (int ti = 0; ti < 2; ++ti) {
      const ProdTree& t = ti ? p.inner_tree : p.outer_tree;
      for (int j = 0; j < t.items(); ++j)
        if (t.item_row[j] >= 0) item_of[t.item_row[j]] = {ti, j};
    }
  }
  const ProdTree& tr(int ti) const { return ti ? P.inner_tree : P.outer_tree; }
  uint32_t rs(int r) const { return rsig[r] & ccm; }
  bool live(int r, int v) const {  // v: 0 copies over x, 1 over y
    const auto it = item_of[r];
    return it.first >= 0 && (tr(it.first).item_live[it.second] >> v) & 1u;
  }
  double cval(int r, uint32_t S, int v) const { return v ? seg_cy(P, r, S) : seg_cx(P, r, S); }
  // name of a row copy (S already masked to the row's cached classes)
  std::string cname(int r, uint32_t S, int v) const {
    if (v == 0) return S ? "x" + std::to_string(r) + "_" + std::to_string(S) : "x[" + std::to_string(r) + "]";
    return S ? "y" + std::to_string(r) + "_" + std::to_string(S) : "y[" + std::to_string(r) + "]";
  }
  int dir(int r, uint32_t S, int v) {
    auto key = std::make_tuple(r, S, v);
    auto it = cdir.find(key);
    if (it != cdir.end()) return it->second;
    const int i = (int)ctab.size();
    ctab.push_back(cval(r, S, v));
    cdir[key] = i;
    return i;
  }
  // init-time constant: one scalar load of the directory entry
  std::string kinit(int r, uint32_t S, int v) {
    return "opaque_c(p.jtab, " + std::to_string((cbase + dir(r, S, v)) * 8) + "u)[0]";
  }

  // tree operand id in state S: `step` = inside a step (on-demand copies read
  // the stream `ks`), else init (every copy is a named variable)
  std::string opnd(int ti, int v, int id, uint32_t S, std::vector<double>* ks) const {
    const ProdTree& t = tr(ti);
    if (id < t.items()) {
      const int r = t.item_row[id];
      if (r < 0) return ti == 0 ? "Ro" : (v ? "Cy" : "Cx");
      const uint32_t s = S & rs(r);
      if (v == 0 && s == 0) return "x[" + std::to_string(r) + "]";
      if (!ks || live(r, v)) return cname(r, s, v);
      ks->push_back(cval(r, s, v));
      return "(x[" + std::to_string(r) + "] + @" + std::to_string(ks->size() - 1) + "@)";
    }
    const int i = id - t.items();
    if (ks && !nlive(ti, v, i)) return "(" + node(ti, v, i, S, ks) + ")";  // formed on demand
    const char* N = ti == 0 ? "o" : (v ? "py" : "px");
    return N + std::to_string(i) + "_" + std::to_string(S & t.sig[i] & ccm);
  }
  bool nlive(int ti, int v, int i) const { return (tr(ti).node_live[i] >> v) & 1u; }
  // node i's variable name for copy S (chunk start and live nodes)
  std::string nname(int ti, int v, int i, uint32_t S) const {
    const char* N = ti == 0 ? "o" : (v ? "py" : "px");
    return N + std::to_string(i) + "_" + std::to_string(S & tr(ti).sig[i] & ccm);
  }
  uint32_t csig(int ti, int id) const {
    const ProdTree& t = tr(ti);
    return (id < t.items() ? t.item_sig[id] : t.sig[id - t.items()]) & ccm;
  }
  // operand at the chunk start: live values by name, the rest inline (row
  // copies read their constant with one scalar load), so only live values are
  // held while the trees are formed
  std::string iopnd(int ti, int v, int id, uint32_t S) {
    const ProdTree& t = tr(ti);
    if (id < t.items()) {
      const int r = t.item_row[id];
      if (r < 0) return ti == 0 ? "Ro" : (v ? "Cy" : "Cx");
      const uint32_t s = S & rs(r);
      if (s == 0) return v ? "y[" + std::to_string(r) + "]" : "x[" + std::to_string(r) + "]";
      if (live(r, v)) return cname(r, s, v);
      return "(x[" + std::to_string(r) + "] + " + kinit(r, s, v) + ")";
    }
    const int i = id - t.items();
    if (nlive(ti, v, i)) return nname(ti, v, i, S);
    return "(" + iopnd(ti, v, t.a[i], S) + " * " + iopnd(ti, v, t.b[i], S) + ")";
  }
  std::string top(int ti, int v, uint32_t S) const {
    const ProdTree& t = tr(ti);
    return t.root() < 0 ? std::string() : opnd(ti, v, t.root(), S, nullptr);
  }
  std::string node(int ti, int v, int i, uint32_t S, std::vector<double>* ks) const {
    const ProdTree& t = tr(ti);
    return opnd(ti, v, t.a[i], S, ks) + " * " + opnd(ti, v, t.b[i], S, ks);
  }
  uint32_t inner_root_csig() const { return P.inner_tree.root() < 0 ? 0u : csig(1, P.inner_tree.root()); }
  // D = top_x - top_y of segment 0's tree; with a root node, the x root's
  // product fuses with the subtraction: fma(x_a, x_b, -top_y) (one rounding;
  // engine_cpu.cpp seg_D, oracle.c e_seg_D)
  template <class Op>
  std::string dexpr(Op op) const {
    const ProdTree& t = P.inner_tree;
    const int rt = t.root();
    if (rt < t.items()) return op(0, rt) + " - " + op(1, rt);
    const int i = rt - t.items();
    return "__builtin_fma(" + op(0, t.a[i]) + ", " + op(0, t.b[i]) + ", -" + op(1, rt) + ")";
  }
  std::string dname(uint32_t s) const { return "D" + std::to_string(s & inner_root_csig()); }

  // statements of a step of class c after its x^0 adds (same for every
  // occurrence of the class): live copies of the rows it touches, the dirty
  // nodes of every copy, D
  void build_class(int c) {
    std::vector<Stmt>& st = cls_stmts[c];
    std::vector<double>& ks = cls_consts[c];
    const std::vector<int>& rows = c < P.seg_b ? P.touched[c + 1] : P.dyn_rows;
    for (int r : rows)
      for (int v = 0; v < (r < len0 ? 2 : 1); ++v)
        if (live(r, v))
          for (uint32_t S : submasks(rs(r))) {
            if (v == 0 && S == 0) continue;
            ks.push_back(cval(r, S, v));
            st.push_back({cname(r, S, v) + " = x[" + std::to_string(r) + "] + @" + std::to_string(ks.size() - 1) +
                          "@;"});
          }
    auto upd = [&](int ti, int v) {
      const ProdTree& t = tr(ti);
      for (int i = 0; i < t.K(); ++i)
        if (((t.sig[i] >> c) & 1u) && nlive(ti, v, i))
          for (uint32_t S : submasks(t.sig[i] & ccm))
            st.push_back({nname(ti, v, i, S) + " = " + node(ti, v, i, S, &ks) + ";"});
    };
    upd(0, 0);
    if ((P.inner_tree.root_sig() >> c) & 1u) {
      upd(1, 0);
      upd(1, 1);
      for (uint32_t S : submasks(inner_root_csig()))
        st.push_back({dname(S) + " = " +
                      dexpr([&](int v, int id) { return opnd(1, v, id, S, &ks); }) + ";"});
    }
  }

  // ---- straight-line code as a stream of items over SGPR pieces ----
  // An item is one statement; its operands are wave-uniform dbl8 pieces
  // (column values, row-copy constants) loaded with s_load_dwordx16.  `$i:e$`
  // in an item's text is element e of piece i (pieces[i] = its load
  // expression).  emit_items cuts the stream into regions of at most seg_kp
  // distinct pieces, each region's pieces pinned to SGPRs at its start and a
  // scheduling barrier after it; a region may span several pair steps (a
  // sparse step needs one or two pieces, so the waits are shared).  With
  // prefetch the pieces of region r+1 are requested at the start of region r.
  // The budget (Plan::seg_kp, 4) was measured on the n = 40 bench matrix:
  // 2.33e12 Gray steps/s against 2.27e12 at 2 and 2.04e12 at 1; compile()
  // regenerates with a smaller one if the register allocator runs out.
  // SUP_JIT_PF overrides prefetch (experiments).
  struct Item {
    std::string text;
    std::vector<int> pieces;
    int step = -1;  // pair step the item belongs to (-1: none)
  };
  std::vector<std::string> pieces;
  std::map<std::string, int> piece_id;
  int next_step_id = 0;
  int piece(const std::string& load_expr) {
    auto it = piece_id.find(load_expr);
    if (it != piece_id.end()) return it->second;
    pieces.push_back(load_expr);
    return piece_id[load_expr] = (int)pieces.size() - 1;
  }
  static std::string pref(int pc, int e) { return "$" + std::to_string(pc) + ":" + std::to_string(e) + "$"; }

  // Items of one pair step of class c: the x^0 adds of `rows` (value i of the
  // table at byte offset expression `off` from `base` for rows[i], or value
  // rows[i] of a full column, `full`), then the class's statements (row-copy
  // constants from its stream in jtab).
  void step_items(std::vector<Item>& out, const std::string& base, const std::string& off,
                  const std::vector<int>& rows, bool full, int c) {
    auto col_piece = [&](int pc) {
      return piece("((cjdbl8*)(" + base + " + " + off + "))[" + std::to_string(pc) + "]");
    };
    const int sid = next_step_id++;
    for (size_t i = 0; i < rows.size(); ++i) {
      const int vi = full ? rows[i] : (int)i, pc = col_piece(vi / 8);
      out.push_back({"x[" + std::to_string(rows[i]) + "] += " + pref(pc, vi % 8) + ";", {pc}, sid});
    }
    if (c < P.seg_cc) return;
    for (const Stmt& st : cls_stmts[c]) {
      Item it;
      it.step = sid;
      const std::string& t = st.text;
      for (size_t q = 0; q < t.size(); ++q) {
        if (t[q] != '@') {
          it.text += t[q];
          continue;
        }
        const size_t e = t.find('@', q + 1);
        const int idx = std::atoi(t.substr(q + 1, e - q - 1).c_str());
        const int pos = cpos[c][idx];
        // a class reading another class's stream loads each piece through a
        // fresh opaque base: otherwise LLVM merges the two steps' loads of the
        // same piece and keeps them live across the block (SGPR spills)
        const bool fresh = std::getenv("SUP_JIT_FRESHBASE") && std::atoi(std::getenv("SUP_JIT_FRESHBASE"));
        const std::string jb = own_stream[c] && !fresh ? "jt" : "(const char*)opaque_c(p.jtab, 0u)";
        const int pc = piece("((cjdbl8*)(" + jb + " + " + std::to_string((cbase + pos - pos % 8) * 8) + "u))[0]");
        it.text += pref(pc, pos % 8);
        if (std::find(it.pieces.begin(), it.pieces.end(), pc) == it.pieces.end()) it.pieces.push_back(pc);
        q = e;
      }
      out.push_back(std::move(it));
    }
  }

  void emit_items(const std::vector<Item>& items, const char* ind) {
    const int kp = P.seg_kp;
    const bool pf = std::getenv("SUP_JIT_PF") ? std::atoi(std::getenv("SUP_JIT_PF")) != 0 : true;
    if (items.empty()) return;
    std::vector<std::pair<size_t, size_t>> reg;
    std::vector<std::vector<int>> rp;
    // a region takes a following pair step only whole (small sparse steps
    // share a region; a large step starts its own: measured, n = 40 bench
    // matrix 2.33e12 per-step against 2.21e12 with regions cut anywhere)
    auto step_pieces = [&](size_t j, std::vector<int> need) {
      for (size_t k = j; k < items.size() && (items[k].step == items[j].step || items[k].step < 0); ++k)
        for (int pc : items[k].pieces)
          if (std::find(need.begin(), need.end(), pc) == need.end()) need.push_back(pc);
      return need;
    };
    const bool xstep = std::getenv("SUP_JIT_XSTEP") ? std::atoi(std::getenv("SUP_JIT_XSTEP")) != 0 : true;
    for (size_t i = 0; i < items.size();) {
      std::vector<int> pcs;
      size_t j = i;
      for (; j < items.size(); ++j) {
        if (j > i && items[j].step >= 0 && items[j].step != items[j - 1].step &&
            (!xstep || (int)step_pieces(j, pcs).size() > kp))
          break;
        std::vector<int> need = pcs;
        for (int pc : items[j].pieces)
          if (std::find(need.begin(), need.end(), pc) == need.end()) need.push_back(pc);
        if ((int)need.size() > kp && j > i) break;
        pcs = need;
      }
      reg.push_back({i, j});
      rp.push_back(pcs);
      i = j;
    }
    // Accumulates (no pieces) that close a region float into the next one:
    // their fma chain on acc is serial, and there the scheduler can interleave
    // it with the next step's independent adds (same statements, same order
    // of the chain: the bits do not change).  SUP_JIT_ACCFLOAT=0 disables.
    const bool accfloat = std::getenv("SUP_JIT_ACCFLOAT") ? std::atoi(std::getenv("SUP_JIT_ACCFLOAT")) != 0 : true;
    std::vector<std::vector<size_t>> order(reg.size());
    for (size_t r = 0; r < reg.size(); ++r)
      for (size_t i = reg[r].first; i < reg[r].second; ++i) order[r].push_back(i);
    if (accfloat)
      for (size_t r = 0; r + 1 < reg.size(); ++r) {
        std::vector<size_t> tail;
        while (!order[r].empty() && items[order[r].back()].step < 0 && items[order[r].back()].pieces.empty() &&
               order[r].size() > 1) {
          tail.insert(tail.begin(), order[r].back());
          order[r].pop_back();
        }
        if (tail.empty()) continue;
        // spread the chain over the next region's leading x^0 adds (they
        // write no value an accumulate reads: D and the outer root are
        // re-formed after them), one accumulate after every `gap` of them
        size_t lead = 0;
        while (lead < order[r + 1].size() && items[order[r + 1][lead]].text.compare(0, 2, "x[") == 0) ++lead;
        if (lead == 0) {  // nothing to interleave with: keep them where they were
          order[r].insert(order[r].end(), tail.begin(), tail.end());
          continue;
        }
        std::vector<size_t> nx;
        const size_t gap = std::max<size_t>(1, lead / (tail.size() + 1));
        size_t t = 0;
        for (size_t i = 0; i < order[r + 1].size(); ++i) {
          if (i == lead)
            while (t < tail.size()) nx.push_back(tail[t++]);
          nx.push_back(order[r + 1][i]);
          if (i < lead && t < tail.size() && (i + 1) % gap == 0) nx.push_back(tail[t++]);
        }
        while (t < tail.size()) nx.push_back(tail[t++]);
        order[r + 1] = nx;
      }
    auto pname = [&](size_t r, int pc) { return "s" + std::to_string(pc) + "_" + std::to_string(r); };
    auto load = [&](size_t r) {
      for (int pc : rp[r]) o << ind << "  jdbl8 " << pname(r, pc) << " = " << pieces[pc] << ";\n";
    };
    // Pin at most kp pieces: a region holds one item that needs more (a
    // near-dense D product reads up to 8 pieces, 128 SGPRs) — pinning all of
    // them, beside the next region's prefetched pieces, asks for more SGPRs
    // than a wave has ("inline assembly requires more registers than
    // available", dense d = 0.9 at n >= 46).  The rest load unpinned; the
    // operations and their order do not change.
    auto pin = [&](size_t r) {
      if (rp[r].empty()) return;
      o << ind << "  asm volatile(\"\" :";
      const size_t np = std::min(rp[r].size(), (size_t)std::max(1, kp));
      for (size_t q = 0; q < np; ++q) o << (q ? ", " : " ") << "\"+s\"(" << pname(r, rp[r][q]) << ")";
      o << ");\n";
    };
    o << ind << "{\n";
    load(0);
    pin(0);
    for (size_t r = 0; r < reg.size(); ++r) {
      if (pf && r + 1 < reg.size()) load(r + 1);
      for (size_t i : order[r]) {
        const std::string& t = items[i].text;
        std::string out;
        for (size_t q = 0; q < t.size(); ++q) {
          if (t[q] != '$') {
            out += t[q];
            continue;
          }
          const size_t colon = t.find(':', q + 1), e = t.find('$', q + 1);
          const int pc = std::atoi(t.substr(q + 1, colon - q - 1).c_str());
          out += pname(r, pc) + "[" + t.substr(colon + 1, e - colon - 1) + "]";
          q = e;
        }
        o << ind << "  " << out << "\n";
      }
      if (r + 1 < reg.size()) {
        if (pf) pin(r + 1);
        o << ind << "  __builtin_amdgcn_sched_barrier(0);\n";
        if (!pf) {
          load(r + 1);
          pin(r + 1);
        }
      }
    }
    o << ind << "}\n";
  }

  // accumulate pair term with cached state S
  std::string accumulate_text(bool neg, uint32_t S) const {
    const std::string D = dname(S), U = top(0, 0, S);
    if (U.empty()) return std::string("acc ") + (neg ? "-= " : "+= ") + D + ";";
    return "acc = __builtin_fma(" + std::string(neg ? "-" : "") + D + ", " + U + ", acc);";
  }

  std::string off_const(int k, int neg) const {
    const int blk = (((int)P.touched[k].size() + 7) & ~7);
    return std::to_string((P.jofs[k] + neg * blk) * 8) + "u";
  }
  std::string off_dyn(int k, const char* negv) const {
    const int blk = (((int)P.touched[k].size() + 7) & ~7);
    return std::to_string(P.jofs[k] * 8) + "u + " + negv + " * " + std::to_string(blk * 8) + "u";
  }

  // cached state (walk bits 1..cc) at pair index j with j mod B = st:
  // gray bit i = bit i ^ bit i+1 of st (i + 1 < b)
  uint32_t state(unsigned st) const {
    uint32_t S = 0;
    for (int i = 0; i < P.seg_cc; ++i) S |= (((st >> i) ^ (st >> (i + 1))) & 1u) << i;
    return S;
  }

  // the constant tail appended to P.jtab (directory for the chunk start, then
  // one stream per step class, each 8-double aligned)
  std::vector<double> tail() const {
    std::vector<double> t = ctab;
    t.resize((t.size() + 7) & ~(size_t)7, 0.0);
    for (size_t c = 0; c < cls_consts.size(); ++c) {
      if (!own_stream[c]) continue;
      t.insert(t.end(), cls_consts[c].begin(), cls_consts[c].end());
      t.resize((t.size() + 7) & ~(size_t)7, 0.0);
    }
    return t;
  }

  // Positions in `pool` of the constants of `need`, in order: each is matched
  // to the first occurrence of its value at or after the previous match
  // (wrapping to the first occurrence), so a sequence that follows the pool's
  // order reads it front to back.  Empty if some value is missing.  Matching
  // by value is exact: the operand is that double either way.
  static std::vector<int> match_stream(const std::vector<double>& need, const std::vector<double>& pool) {
    std::map<uint64_t, std::vector<int>> where;
    for (size_t i = 0; i < pool.size(); ++i) {
      uint64_t k;
      std::memcpy(&k, &pool[i], 8);
      where[k].push_back((int)i);
    }
    std::vector<int> at;
    int prev = -1;
    for (double v : need) {
      uint64_t k;
      std::memcpy(&k, &v, 8);
      auto it = where.find(k);
      if (it == where.end()) return {};
      const std::vector<int>& w = it->second;
      auto nx = std::upper_bound(w.begin(), w.end(), prev);
      prev = nx != w.end() ? *nx : w.front();
      at.push_back(prev);
    }
    return at;
  }
  // Distinct 8-double pieces a run of positions touches, counted per run of
  // consecutive equal pieces (what the step regions load).
  static int piece_runs(const std::vector<int>& pos) {
    int runs = 0, last = -1;
    for (int p : pos)
      if (p / 8 != last) ++runs, last = p / 8;
    return runs;
  }
  // Stream sharing (round 4): a step class whose every constant another
  // class's stream holds — near-dense walks re-form almost every copy on the
  // top specialised step and on the shared step, the same constants in nearly
  // the same order (double/40_0.90_0: 716 of them, 5.7 KB) — reads that
  // stream instead of its own when that costs at most 1/8 more piece loads.
  // The hot constant set then fits the 16 KB scalar cache better.  Same
  // values, same operations: the results do not change.
  void share_streams(std::vector<int>& host) const {
    const int b = P.seg_b;
    std::vector<int> order;
    for (int c = 0; c <= b; ++c)
      if (!cls_consts[c].empty()) order.push_back(c);
    // larger streams host smaller ones
    std::stable_sort(order.begin(), order.end(),
                     [&](int x, int y) { return cls_consts[x].size() > cls_consts[y].size(); });
    for (size_t i = 1; i < order.size(); ++i) {
      const int c = order[i];
      for (size_t j = 0; j < i; ++j) {
        const int h = order[j];
        if (host[h] >= 0) continue;  // hosts keep their own stream
        const std::vector<int> at = match_stream(cls_consts[c], cls_consts[h]);
        if (at.empty()) continue;
        std::vector<int> own(cls_consts[c].size());
        for (size_t q = 0; q < own.size(); ++q) own[q] = (int)q;
        // the host's pieces must be read front to back: a piece read again
        // after others is one load to LLVM (same address, constant memory),
        // held in SGPRs across the step (measured: 730 v_readlane spill
        // reloads in the d = 0.9 walk loop when it was allowed)
        bool forward = true;
        for (size_t q = 1; q < at.size() && forward; ++q) forward = at[q] / 8 >= at[q - 1] / 8;
        if (forward && 8 * piece_runs(at) <= 9 * piece_runs(own)) {
          host[c] = h;
          break;
        }
      }
    }
  }

  std::string source() {
    const int n = P.n, L = P.lay.L, m = P.lay.m, b = P.seg_b, cc = P.seg_cc;
    const unsigned B = 1u << b, Q = 1u << (m - 1 - b);
    cbase = P.seg_cbase;
    // the chunk start's directory first (its size fixes the streams' offsets)
    for (int r = 0; r < n; ++r)
      for (int v = 0; v < (r < len0 ? 2 : 1); ++v)
        for (uint32_t S : submasks(rs(r)))
          if (v == 1 || S != 0) dir(r, S, v);
    cls_stmts.assign(b + 1, {});
    cls_consts.assign(b + 1, {});
    for (int c = cc; c <= b; ++c) build_class(c);
    kofs.assign(b + 1, 0);
    own_stream.assign(b + 1, 1);
    std::vector<int> host(b + 1, -1);  // class whose stream class c reads (-1: its own)
    if (!std::getenv("SUP_JIT_NOSHARE")) share_streams(host);
    {
      size_t off = (ctab.size() + 7) & ~(size_t)7;
      for (int c = 0; c <= b; ++c) {
        if (host[c] >= 0) {
          own_stream[c] = 0;
          continue;
        }
        kofs[c] = (int)off;
        off = (off + cls_consts[c].size() + 7) & ~(size_t)7;
      }
    }
    cpos.assign(b + 1, {});
    for (int c = 0; c <= b; ++c) {
      if (host[c] < 0) {
        for (size_t i = 0; i < cls_consts[c].size(); ++i) cpos[c].push_back(kofs[c] + (int)i);
      } else {
        const std::vector<int> at = match_stream(cls_consts[c], cls_consts[host[c]]);
        for (int i : at) cpos[c].push_back(kofs[host[c]] + i);
      }
    }
    if (std::getenv("SUP_JIT_VERBOSE")) {
      std::fprintf(stderr, "  constant streams (doubles): directory %zu", ctab.size());
      for (int c = 0; c <= b; ++c) {
        int same = -1;
        for (int c2 = 0; c2 < c && same < 0; ++c2)
          if (!cls_consts[c].empty() && cls_consts[c2] == cls_consts[c]) same = c2;
        std::vector<double> u = cls_consts[c];
        std::sort(u.begin(), u.end());
        const size_t nd = (size_t)(std::unique(u.begin(), u.end()) - u.begin());
        size_t shared = 0;  // constants an earlier class's stream also holds
        for (double v : cls_consts[c]) {
          bool f = false;
          for (int c2 = 0; c2 < c && !f; ++c2)
            f = std::find(cls_consts[c2].begin(), cls_consts[c2].end(), v) != cls_consts[c2].end();
          shared += f;
        }
        std::fprintf(stderr, ", class %d: %zu (%zu distinct, %zu in earlier streams)%s%s", c, cls_consts[c].size(), nd,
                     shared, same >= 0 ? " (= earlier)" : "", own_stream[c] ? "" : " [reads another class's stream]");
      }
      std::fprintf(stderr, "\n");
    }
    int nlive = 0;
    for (int r = 0; r < n; ++r)
      for (int v = 0; v < 2; ++v) nlive += live(r, v);
    o << "// generated by superman_amd jit.cpp: paired segmented Gray walk, n=" << n << " L=" << L << " m=" << m
      << " segment0=" << len0 << " (" << P.inner_tree.K() << " tree nodes) outer tree nodes=" << P.outer_tree.K()
      << " pair bits specialised=" << b << " cached=" << cc << " live values~" << P.seg_regs
      << " live row-copy sets=" << nlive << "\n";
    o << "#include \"walk_common.hpp\"\n";
    o << "namespace sup {\n";
    o << "typedef double jdbl8 __attribute__((ext_vector_type(8)));\n";
    o << "typedef const __attribute__((address_space(4))) jdbl8 cjdbl8;\n";
    // occupancy target from the values live across the walk loop (seg_fit's
    // estimate): 3 waves per SIMD when they fit 168 VGPRs, else 2 (~2% slower
    // on this walk; the compiler's own choice may trade occupancy for
    // scheduling freedom).  SUP_JIT_WAVES overrides (experiments).
    int waves = P.seg_regs <= 64 ? 4 : (P.seg_regs <= kRegs3 ? 3 : 2);
    if (const char* e = std::getenv("SUP_JIT_WAVES")) waves = std::max(1, std::min(8, std::atoi(e)));
    o << "extern \"C\" __global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(" << waves
      << "))) void sup_walk_seg(WalkParams p) {\n";
    o << "  constexpr int N = " << n << ";\n";
    // The lane id is re-read (v_mbcnt, asm volatile: not hoisted) where a
    // chunk starts and where it ends, instead of one value live across the
    // walk loop; the wave's slot in the block is an SGPR.
    o << "#define SUP_LANE() ({ uint32_t l_; asm volatile(\"v_mbcnt_lo_u32_b32 %0, -1, 0\\n\\tv_mbcnt_hi_u32_b32 %0, -1, %0\" : \"=v\"(l_)); l_; })\n";
    // experiment (SUP_JIT_PHASE=k): odd workgroups start 64 k cycles late, so
    // the two waves sharing a SIMD (one per workgroup) are out of phase
    if (const char* e = std::getenv("SUP_JIT_PHASE"))
      if (std::atoi(e) > 0)
        o << "  if (blockIdx.x & 1u) __builtin_amdgcn_s_sleep(" << std::min(127, std::atoi(e)) << ");\n";
    // experiment (SUP_JIT_PRIO=1): static issue priority for the odd
    // workgroups' waves, so each SIMD's two waves (one per workgroup) stop
    // trading VALU slots by age (MI355X_MICROARCH.md, two waves per SIMD, item 4)
    if (const char* e = std::getenv("SUP_JIT_PRIO"))
      if (std::atoi(e) > 0) o << "  if (blockIdx.x & 1u) __builtin_amdgcn_s_setprio(" << std::min(3, std::atoi(e)) << ");\n";
    // A group's chunk partials (and walked-step counts) wait in LDS, not in
    // registers held across the walk loop: two fewer VGPR values live in the
    // loop (LDS is otherwise unused; 3 KB per block).
    o << "  __shared__ double s_keep[" << kBlock / 64 << "][64];\n";
    o << "  __shared__ uint32_t s_vkeep[" << kBlock / 64 << "][64];\n";
    o << "  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n";
    // SUP_JIT_TRACE (diagnostics; a knob, so a fresh plan and kernel): each
    // wave stamps its entry / exit and sums the shader cycles of its chunk
    // starts (the start state, row copies and trees: everything before the walk
    // loop), for the launch ramp / queue tail / chunk-start split
    const bool trace = std::getenv("SUP_JIT_TRACE") != nullptr;
    if (trace)
      o << "  const uint64_t tr_r0 = __builtin_amdgcn_s_memrealtime(), tr_c0 = __builtin_amdgcn_s_memtime();\n"
        << "  uint64_t tr_n = 0, tr_sc = 0;\n";
    // ticket t -> chunks [base, base + len): groups of p.group, then (from
    // p.tail_begin) groups of p.tail_group
    // (p.tail_ticket = p.tail_begin / p.group from the host: all of it
    // wave-uniform scalar arithmetic)
    // (every ticket from the atomic counter: dealing the head of the queue
    // out statically, one atomic per wave and round, measured 9 % slower on
    // the bench matrix even with equal work per chunk — waves do not progress
    // evenly; profiles/r3/probe_ab_static.log)
    o << "  for (uint32_t t = next_chunk(p.counter);; t = next_chunk(p.counter)) {\n";
    o << "    const bool head = t < p.tail_ticket;\n";
    o << "    const uint64_t base = head ? (uint64_t)t * p.group\n";
    o << "                               : p.tail_begin + (uint64_t)(t - p.tail_ticket) * p.tail_group;\n";
    o << "    const uint32_t len = head ? p.group : p.tail_group;\n";
    o << "    if (base >= p.chunk_count) break;\n";
    o << "    for (uint32_t j = 0; j < len; ++j) {\n";
    o << "      const uint64_t a = base + j;\n";
    o << "      if (a >= p.chunk_count) break;\n";
    o << "      const uint64_t ga = p.chunk_begin + a;\n";
    o << "      double x[N], y[" << len0 << "];\n";
    if (trace) o << "      const uint64_t tr_s = __builtin_amdgcn_s_memtime();\n";
    o << "      chunk_start" << (P.start_tab_on ? "_tab" : "") << "<N>(x, p, ga, SUP_LANE());\n";
    o << "      {\n";  // y = x + a_0 on segment 0 (the + block of walk bit 0) = y^0
    o << "        cjdbl8* cv = (cjdbl8*)opaque_c(p.jtab, " << off_const(0, 0) << ");\n";
    for (int r = 0; r < len0; ++r) o << "        y[" << r << "] = x[" << r << "] + cv[" << r / 8 << "][" << r % 8 << "];\n";
    o << "      }\n";
    // the live row copies for the cached states (y copy 0 is y[r])
    for (int r = 0; r < n; ++r)
      for (int v = 0; v < (r < len0 ? 2 : 1); ++v)
        if (live(r, v))
          for (uint32_t S : submasks(rs(r))) {
            if (S == 0) continue;
            o << "      double " << cname(r, S, v) << " = x[" << r << "] + " << kinit(r, S, v) << ";\n";
          }
    // constant items (tails) and the live node copies (on-demand ones inline)
    auto tree_init = [&](int ti, int v) {
      const ProdTree& t = tr(ti);
      if (t.tail_hi > t.tail_lo)
        o << "      const double " << (ti == 0 ? "Ro" : (v ? "Cy" : "Cx")) << " = "
          << tree(t.tail_lo, t.tail_hi, v ? "y" : "x") << ";\n";
      for (int i = 0; i < t.K(); ++i)
        if (this->nlive(ti, v, i))
          for (uint32_t S : submasks(t.sig[i] & ccm))
            o << "      double " << nname(ti, v, i, S) << " = " << iopnd(ti, v, t.a[i], S) << " * "
              << iopnd(ti, v, t.b[i], S) << ";\n";
    };
    tree_init(0, 0);
    // Rows no walk bit touches (the outer tree's tail, Ro) are constant over the
    // chunk: when Ro is an exact zero in every valid lane (integer matrices),
    // every product of the chunk is zero and the walk is skipped (part = +0).
    o << "      double acc = 0.0;\n";
    o << "      uint32_t vis = 0;\n";
    if (P.outer_tree.tail_hi > P.outer_tree.tail_lo)
      o << "      if (__builtin_amdgcn_ballot_w64(SUP_LANE() < " << (1u << L) << "u && Ro != 0.0) != 0) {\n";
    else
      o << "      {\n";
    o << "      vis = " << (1u << m) << "u;\n";
    tree_init(1, 0);
    tree_init(1, 1);
    if (P.inner_tree.root() >= 0)
      for (uint32_t S : submasks(inner_root_csig()))
        o << "      double " << dname(S) << " = " << dexpr([&](int v, int id) { return iopnd(1, v, id, S); })
          << ";\n";
    else
      o << "      double D0 = 0.0;\n";
    {
      const std::string U = top(0, 0, 0);
      o << "      acc = " << (U.empty() ? dname(0) : dname(0) + " * " + U) << ";\n";
    }
    // two-level lane sum: acc folds into tot after each shared dyn step, so
    // no sequential sum runs longer than 2^b pairs (error growth, HISTORY.md §3.3 "Lane sum")
    o << "      double tot = 0.0;\n";
    if (trace) o << "      asm volatile(\"\" : \"+v\"(acc));\n      tr_sc += __builtin_amdgcn_s_memtime() - tr_s;\n      ++tr_n;\n";
    o << "      for (uint32_t q = 0; q < " << Q << "u; ++q) {\n";
    const char* ind = "        ";
    // pair index j = B*q + s, s = 1 .. B-1: pair bit p = ctz(s) (walk bit p+1);
    // neg = (j >> (p+1)) & 1 = bit p+1 of s for p < b-1, bit 0 of q for p = b-1
    // the 2^b - 1 pair steps of the block as one item stream (regions may
    // span steps); the top specialised bit's sign is bit 0 of q
    // one opaque base per iteration: the pieces' loads cannot leave the loop,
    // and their constant offsets fold into the s_load immediates
    o << ind << "const char* jt = (const char*)opaque_c(p.jtab, 0u);\n";
    o << ind << "const uint32_t ng = q & 1u;\n";
    {
      std::vector<Item> items;
      for (unsigned st = 1; st < B; ++st) {
        const int pb = __builtin_ctz(st), k = pb + 1;
        if (pb >= cc && !P.touched[k].empty())  // cached walk bits: their state's copies are already there
          step_items(items, "jt", pb < b - 1 ? off_const(k, (st >> (pb + 1)) & 1u) : off_dyn(k, "ng"),
                     P.touched[k], false, step_class(k, b));
        items.push_back({accumulate_text(st & 1u, state(st)), {}});
      }
      emit_items(items, ind);
    }
    if (Q > 1) {
      // j = B(q+1): pair bit b + ctz(q+1) (walk bit b+1+ctz(q+1)), neg =
      // ((q+1) >> (ctz(q+1)+1)) & 1.  One straight-line step for all of them
      // (no per-bit branches): the full signed column is added to every row
      // some walk bit > b touches (zeros elsewhere) and every node above such
      // a row is re-formed.  Cached state 0.
      o << ind << "if (q + 1u < " << Q << "u) {\n";
      o << ind << "  const uint32_t kk = (uint32_t)__builtin_ctz(q + 1u);\n";
      o << ind << "  const uint32_t ngd = ((q + 1u) >> (kk + 1u)) & 1u;\n";
      {
        std::vector<Item> items;
        step_items(items, "(const char*)opaque_c(p.cols, 0u)",
                   "(2u * (" + std::to_string(L + b + 1) + "u + kk) + ngd) * " + std::to_string(P.NP * 8) + "u",
                   P.dyn_rows, true, P.seg_b);
        items.push_back({accumulate_text(false, 0u), {}});
        emit_items(items, "          ");
      }
      o << ind << "  tot += acc;\n" << ind << "  acc = 0.0;\n";
      o << ind << "}\n";
    }
    o << "      }\n";
    o << "      acc = tot + acc;\n";
    o << "      if (((uint32_t)ga ^ (uint32_t)__builtin_popcount(SUP_LANE())) & 1u) acc = -acc;\n";
    o << "      }\n";
    o << "      const uint32_t lane = SUP_LANE();\n";
    o << "      const double part = wave_sum(lane < " << (1u << L) << "u ? acc : 0.0);\n";
    o << "      if (lane == j) s_keep[wv][j] = part, s_vkeep[wv][j] = vis;\n";
    o << "    }\n";
    o << "    __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");\n";
    o << "    __builtin_amdgcn_wave_barrier();\n";
    o << "    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");\n";
    o << "    const uint32_t lane = SUP_LANE();\n";
    o << "    chunk_store(base, len, s_keep[wv][lane], s_vkeep[wv][lane]);\n";
    o << "    __builtin_amdgcn_wave_barrier();\n";
    o << "  }\n";
    if (trace)
      o << "  if (p.trace && SUP_LANE() == 0) {\n"
        << "    unsigned long long* t = p.trace + 8ull * (blockIdx.x * " << kBlock / 64 << "u + wv);\n"
        << "    t[0] = tr_r0; t[1] = __builtin_amdgcn_s_memrealtime(); t[2] = tr_c0;\n"
        << "    t[3] = __builtin_amdgcn_s_memtime(); t[4] = tr_n; t[5] = tr_sc;\n"
        << "  }\n";
    o << "}\n";
    o << "}  // namespace sup\n";
    return o.str();
  }
};

const char* const kJitOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off"};
constexpr int kJitNopts = 4;

// hiprtc options: kJitOpts, plus the LLVM machine scheduler strategy
// SUP_JIT_SCHED names (experiments: max-ilp, max-memory-clause, ...).
}  // namespace

std::vector<std::string> jit_opts() {
  std::vector<std::string> v(kJitOpts, kJitOpts + kJitNopts);
  if (const char* e = std::getenv("SUP_JIT_SCHED"))
    if (*e) v.push_back("-mllvm"), v.push_back(std::string("-amdgpu-sched-strategy=") + e);
  if (const char* e = std::getenv("SUP_JIT_OPAQUE_R2"))
    if (std::atoi(e)) v.push_back("-DSUP_OPAQUE_BEFORE_OFFSET=1");
  return v;
}

namespace {

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

// The compiler: hiprtc's version and the library file it runs from (name,
// size, content hash) — part of the code-object key and the plan-choice key, so a
// disk cache written by another ROCm release is not reused.  The file matters
// within one release number: a process that imports torch first resolves
// hiprtc (and comgr) to torch's bundled copies, which report the same version
// as /opt/rocm's but generate different code (the n = 40 bench matrix: the
// budget check picks 214 live values with one, 206 with the other).
std::string hiprtc_version() {
  static const std::string v = [] {
    int major = 0, minor = 0;
    if (hiprtcVersion(&major, &minor) != HIPRTC_SUCCESS) return std::string("hiprtc ?");
    std::string r = "hiprtc " + std::to_string(major) + "." + std::to_string(minor) + " hip " + std::to_string(HIP_VERSION);
    Dl_info di;
    if (dladdr(reinterpret_cast<void*>(&hiprtcCreateProgram), &di) && di.dli_fname) {
      // the file's name and a hash of its bytes (~1 MB, ~1 ms): the same
      // library on another machine of the same image gives the same key (its
      // path may differ by symlinks, its mtime by how the image was unpacked)
      const char* slash = std::strrchr(di.dli_fname, '/');
      r += std::string(" ") + (slash ? slash + 1 : di.dli_fname);
      std::ifstream f(di.dli_fname, std::ios::binary);
      if (f) {
        std::string bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        char hx[40];
        std::snprintf(hx, sizeof hx, " %zu %016llx", bytes.size(), (unsigned long long)fnv1a(bytes));
        r += hx;
      }
    }
    return r;
  }();
  return v;
}

}  // namespace

uint64_t toolchain_hash_impl() {
  std::string key;
  for (const std::string& opt : jit_opts()) key += "\n//" + opt;
  key += std::string("\n//") + kWalkCommonSrc + kWalkParamsSrc;
  key += "\n//" + hiprtc_version();
  return fnv1a(key);
}

namespace {

// Code-object key of a generated source: the source, the compile options, the
// embedded headers and the compiler's version.
uint64_t jit_source_key(const std::string& src) {
  std::string key = src;
  for (const std::string& opt : jit_opts()) key += "\n//" + opt;
  key += std::string("\n//") + kWalkCommonSrc + kWalkParamsSrc;
  key += "\n//" + hiprtc_version();
  return fnv1a(key);
}

}  // namespace

// Start tables up to this size (bytes): config 2's 2^14 chunks x 32 rows are
// 4 MB, the n = 40 bench matrix's 2^20 chunks would be 335 MB (formed on the
// device instead).  Measured on config 2: the chunk starts without their
// chunk-bit column adds take 2.2 % off the walk (an upper bound: the table
// row's scalar loads remain).
constexpr size_t kStartTabMaxBytes = 16u << 20;
// ... and for short chunks only: the chunk-bit adds are ~1.6 % of a 2^11-step
// chunk's ops (config 2: the walk 2 % faster), 0.5 % at 2^15 (config 3: no
// measurable gain for 5 MB more reads per launch).
constexpr int kStartTabMaxWalkBits = 12;

// Plan::start_tab: chunk ga's start state without the lane columns — x0, then
// the columns of the set bits of gray(ga) in ascending order, each added to
// rows [0, n): chunk_start's own additions in its order (IEEE adds, so the
// same values the device would form).
static void seg_start_table(Plan& P) {
  const int n = P.n, NP = P.NP;
  const uint64_t C = P.lay.chunks();
  const unsigned hb = (unsigned)(P.lay.L + P.lay.m);
  P.start_tab.assign((size_t)C * NP, 0.0);
  const size_t blocks = (size_t)std::min<uint64_t>(C, 64);
  parallel_tasks(blocks, [&](size_t b) {
    for (uint64_t ga = C * b / blocks; ga < C * (b + 1) / blocks; ++ga) {
      double* x = P.start_tab.data() + (size_t)ga * NP;
      for (int j = 0; j < NP; ++j) x[j] = P.x0[j];
      for (uint64_t h = ga ^ (ga >> 1); h; h &= h - 1) {
        const double* col = P.cols.data() + (size_t)(2u * (hb + (unsigned)__builtin_ctzll(h))) * NP;
        for (int j = 0; j < n; ++j) x[j] += col[j];
      }
    }
  });
}

int build_seg(Plan& P, int fixed_budget) {
  const int n = P.n, L = P.lay.L, m = P.lay.m;
  if (m < 3) {
    set_error("segmented walk needs >= 3 walk bits");
    return SUP_EINVAL;
  }
  if (P.cols.empty()) return SUP_EINVAL;
  // the start table (chunk_start_tab): decided before any source is generated,
  // built once the plan is chosen (the ladder's candidates are copies of P)
  P.start_tab.clear();
  P.start_tab_on = !std::getenv("SUP_JIT_NO_START_TAB") && P.lay.m <= kStartTabMaxWalkBits &&
                   (double)P.lay.chunks() * P.NP * sizeof(double) <= (double)kStartTabMaxBytes;
  // rows are in first-touch order already: rebuild the shape in engine rows
  P.touched.assign(m, {});
  P.seg_start.assign(1, 0);
  std::vector<char> seen(n, 0);
  int R = 0;
  for (int k = 0; k < m; ++k) {
    const double* col = P.cols.data() + (size_t)(2 * (L + k)) * P.NP;
    for (int j = 0; j < n; ++j)
      if (col[j] != 0.0) {
        P.touched[k].push_back(j);
        if (!seen[j]) seen[j] = 1, ++R;
      }
    if (R > P.seg_start.back()) P.seg_start.push_back(R);
  }
  for (int j = 0; j < R; ++j)
    if (!seen[j]) {
      set_error("segmented walk: rows are not in first-touch order");
      return SUP_EINVAL;
    }
  if (P.touched[0].empty()) {
    set_error("segmented walk: walk column 0 has no nonzero");
    return SUP_EINVAL;
  }
  // sub-segments of segment 0: rows in first-touch order by walk bits >= 1
  // (make_plan orders them so, seg_row_order), constant rows last
  {
    const int len0 = P.seg_start[1];
    std::vector<char> got(len0, 0);
    int cnt = 0;
    P.sub_start.assign(1, 0);
    for (int k = 1; k < m; ++k) {
      for (int r : P.touched[k])
        if (r < len0 && !got[r]) {
          if (r != cnt) {
            set_error("segmented walk: segment 0 rows are not in sub-segment order");
            return SUP_EINVAL;
          }
          got[r] = 1, ++cnt;
        }
      if (cnt > P.sub_start.back()) P.sub_start.push_back(cnt);
    }
  }
  // specialised pair bits: the walk-order search's choice (make_plan), else
  // the candidate with the cheapest fit on these rows
  if (P.seg_b < 1 || P.seg_b > m - 1) {
    P.seg_b = seg_static_bits(m);
    if (!std::getenv("SUP_JIT_B")) {
      double best = 1e300;
      for (const int cb : seg_b_candidates(m)) {
        SegRows R;
        R.n = n, R.m = m, R.touched = P.touched;
        R.len0 = P.seg_start[1], R.s_end = P.sub_start.back(), R.r_end = P.seg_start.back();
        seg_rows_finish(R, cb);
        const SegFit f = seg_best(R, std::min(max_cached(), P.lay.cc_cap));
        const double sc = seg_block_bytes(f, cb) > kMaxBlockBytes ? 1e300 : seg_score(f);
        if (sc < best - 1e-12) best = sc, P.seg_b = cb;
      }
    }
  }
  P.dyn_rows.clear();
  {
    std::vector<char> in(n, 0);
    for (int k = P.seg_b + 1; k < m; ++k)
      for (int r : P.touched[k]) in[r] = 1;
    for (int j = 0; j < n; ++j)
      if (in[j]) P.dyn_rows.push_back(j);
  }
  // product trees, cached classes and storage plan for a live-value budget,
  // then the tables and the generated source
  SegRows SR;
  SR.n = n, SR.m = m, SR.touched = P.touched;
  SR.len0 = P.seg_start[1], SR.s_end = P.sub_start.back(), SR.r_end = P.seg_start.back();
  seg_rows_finish(SR, P.seg_b);
  // trees, cached classes and storage plan for live-value budget `budget`,
  // then the tables and the generated source (Q starts as a copy of P)
  const int cc_cap = std::min(max_cached(), P.lay.cc_cap);
  auto finish = [&SR, &cc_cap, n, L, m](Plan& Q, int budget) {
    SegFit f;
    // experiments / tests: SUP_JIT_CC forces cc; SUP_JIT_STORAGE forces the
    // storage budget of the chosen plan (same walk order and trees, other
    // live/on-demand choices: the same values, so bit-identical results)
    if (const char* e = std::getenv("SUP_JIT_CC"))
      f = seg_fit(SR, std::max(0, std::min({std::atoi(e), SR.b - 1, kMaxCachedBits})), budget);
    else f = seg_best(SR, cc_cap, budget);
    if (const char* e = std::getenv("SUP_JIT_STORAGE")) f = seg_fit(SR, f.cc, std::max(0, std::atoi(e)));
    Q.outer_tree = std::move(f.outer);
    Q.inner_tree = std::move(f.inner);
    Q.seg_cc = f.cc;
    Q.seg_ops = f.ops;
    Q.seg_regs = f.regs;
    Q.seg_budget = budget;
    Q.jofs.assign(m, 0);
    Q.jtab.clear();
    for (int k = 0; k < m; ++k) {
      const std::vector<int>& t = Q.touched[k];
      const size_t blk = (t.size() + 7) & ~(size_t)7;
      Q.jofs[k] = (int)Q.jtab.size();
      Q.jtab.resize(Q.jtab.size() + 2 * std::max<size_t>(blk, 8), 0.0);
      for (size_t i = 0; i < t.size(); ++i) {
        Q.jtab[Q.jofs[k] + i] = Q.cols[(size_t)(2 * (L + k)) * Q.NP + t[i]];
        Q.jtab[Q.jofs[k] + blk + i] = Q.cols[(size_t)(2 * (L + k) + 1) * Q.NP + t[i]];
      }
    }
    Q.seg_cbase = Q.jtab.size();
    Q.seg_kp = 4;
    if (const char* e = std::getenv("SUP_JIT_KP")) Q.seg_kp = std::max(1, std::atoi(e));
    Gen g(Q);
    Q.jit_src = g.source();
    {
      const std::vector<double> t = g.tail();
      Q.jtab.insert(Q.jtab.end(), t.begin(), t.end());
    }
    Q.jit_key = jit_source_key(Q.jit_src);
    (void)n;
  };
  // SUP_JIT_BUDGET (experiments) or a recorded choice: this budget, no
  // compiler check
  const char* env_budget = std::getenv("SUP_JIT_BUDGET");
  if (env_budget) fixed_budget = std::max(1, std::atoi(env_budget));
  finish(P, fixed_budget > 0 ? fixed_budget : kRegsMax);
  // The live-value budget against the compiler (walks of 10 ms or more).  The
  // estimate is rough: on the n = 40 bench matrix budgets up to 192 compile
  // without a spill, 194-216 spill 5-13 VGPRs, 218+ 17-27; denser or larger
  // matrices spill inside the walk loop at the default.  So a ladder of
  // budgets is planned (host threads), the distinct kernels are compiled as
  // a bisection for the largest budget whose loop stays clean (below), and
  // each code object is disassembled (codescan.cpp): the one
  // with the fewest ops whose walk loop touches no scratch wins, a kernel with
  // no scratch at all preferred unless the other saves more than
  // kScratchTolerance of the ops (spills in the chunk start cost HBM writes
  // and next to no time).  Where every kernel the compiler accepts scratches
  // inside the walk loop, or hiprtc's register allocator gives up (some dense
  // n >= 46 patterns), there is no segmented plan and the engine runs the
  // ahead-of-time walk.
  const bool fixed = fixed_budget > 0 || std::getenv("SUP_JIT_REGMAX") || std::getenv("SUP_JIT_STORAGE") ||
                     std::getenv("SUP_JIT_CC") || std::getenv("SUP_JIT_NOVERIFY");
  const double walk_s = std::ldexp(1.0, n - 1) * P.seg_ops / 3.7e13;
  if (fixed && std::getenv("SUP_JIT_VERBOSE")) {  // experiments: what the compiler made of the fixed plan
    CodeScan s;
    const int rc = jit_code_scan(P, &s);
    std::fprintf(stderr, "  fixed budget %d: ops %.4f rc %d vgprs %d spills %d scratch %dB (loop %d of %d insts)\n",
                 P.seg_budget, P.seg_ops, rc, s.vgprs, s.vgpr_spills, s.scratch_bytes, s.loop_scratch, s.loop_insts);
  }
  // Short walks skip the ladder (its compiles would cost more than they save),
  // but 16 cached states need many registers: the kernel that would run is
  // compiled (it is needed anyway; cached by its key) and checked, and if its
  // walk loop touches scratch make_seg_plan plans again with 3 cached bits (on
  // the 0.6 ms n = 32 config 2 walk, 4 cached bits spill 21 VGPRs inside the
  // loop: 0.665 ms against 0.588 ms with 3).
  if (!fixed && walk_s < 0.01 && P.seg_cc > 3) {
    CodeScan s;
    P.seg_loop_scratch = jit_code_scan(P, &s) != SUP_OK || s.loop_scratch != 0;
  }
  if (!fixed && walk_s >= 0.01 && P.seg_regs > kRegs3) {
    // the ladder of budgets, one candidate plan per budget (host threads)
    std::vector<int> budgets;
    for (int b2 = kRegs3 + 20; b2 <= kRegsMax + 60; b2 += 8) budgets.push_back(b2);
    std::vector<Plan> cand(budgets.size(), P);
    parallel_tasks(budgets.size(), [&](size_t i) { finish(cand[i], budgets[i]); });
    // distinct kernels in budget order
    std::vector<size_t> idx;
    for (size_t i = 0; i < cand.size(); ++i) {
      bool dup = false;
      for (size_t j : idx) dup = dup || cand[j].jit_key == cand[i].jit_key;
      if (!dup) idx.push_back(i);
    }
    std::vector<CodeScan> scans(cand.size());
    std::vector<int> src(cand.size(), SUP_EHIP);
    std::vector<char> done(cand.size(), 0);
    auto compile_one = [&](size_t i) {
      if (done[i]) return;
      const auto t0 = std::chrono::steady_clock::now();
      const double own = t_compile_ms;  // wall time (the compile's own count stays out)
      src[i] = jit_code_scan(cand[i], &scans[i]);
      t_compile_ms = own + std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      done[i] = 1;
    };
    auto clean = [&](size_t i) { return done[i] && src[i] == SUP_OK && scans[i].loop_scratch == 0; };
    // Probe: the default budget's kernel, first.  hiprtc's register allocator
    // gives up on some dense n >= 46 patterns ("maximum depth for
    // recoloring"): a pattern that fails here has no segmented plan.
    size_t pp = 0;
    for (size_t k = 0; k < idx.size(); ++k)
      if (budgets[idx[k]] <= kRegsMax) pp = k;
    // The search, as a replay over the outcomes known so far (0 = not compiled
    // yet): the candidate it needs next, kLadderDone, or kLadderFail.  From the
    // probe: the largest clean budget, bisected over idx positions (above the
    // probe when the probe is clean, else below it; lo clean, hi not), then a
    // kernel with no scratch at all within kScratchTolerance of its ops (the
    // largest such budget below it).  One compile at a time in this process —
    // hiprtc compiles in one process do not overlap (8 threads compiling 8
    // kernels take 0.8 of the time of 8 sequential compiles; the comgr action
    // is serialised), hence a bisection (5 compiles instead of 8 on the n = 40
    // bench matrix; the same choice wherever "clean" and "no scratch at all"
    // are monotone in the budget, as on every matrix measured).
    enum { kUnknown = 0, kFail, kDirty, kCleanScratch, kClean0 };
    constexpr long kLadderDone = -1, kLadderFail = -2;
    auto next_needed = [&](const std::vector<int>& o) -> long {
      const size_t probe = idx[pp];
      if (o[probe] == kUnknown) return (long)probe;
      if (o[probe] == kFail) return kLadderFail;
      auto cl = [&](size_t i) { return o[i] >= kCleanScratch; };
      size_t c_pos;
      if (cl(probe)) {
        size_t lo = pp, hi = idx.size();
        while (hi - lo > 1) {
          const size_t mid = lo + (hi - lo) / 2;
          if (o[idx[mid]] == kUnknown) return (long)idx[mid];
          (cl(idx[mid]) ? lo : hi) = mid;
        }
        c_pos = lo;
      } else {
        long lo = -1, hi = (long)pp;
        while (hi - lo > 1) {
          const long mid = lo + (hi - lo) / 2;
          if (o[idx[mid]] == kUnknown) return (long)idx[mid];
          (cl(idx[mid]) ? lo : hi) = mid;
        }
        if (lo < 0) return kLadderFail;
        c_pos = (size_t)lo;
      }
      if (o[idx[c_pos]] != kClean0)
        for (size_t k = c_pos; k-- > 0;) {
          if (cand[idx[k]].seg_ops > cand[idx[c_pos]].seg_ops * (1.0 + kScratchTolerance)) break;
          if (o[idx[k]] == kUnknown) return (long)idx[k];
          if (o[idx[k]] == kClean0) break;
        }
      return kLadderDone;
    };
    std::vector<int> outcome(cand.size(), kUnknown);
    const size_t procs = rtc_procs();
    for (;;) {
      const long k = next_needed(outcome);
      if (k < 0) break;
      if (procs > 1 && !jit_code_cached(cand[k])) {
        // Ahead of the search: the candidates its next steps could need, over
        // every outcome of the compiles still ahead (breadth first, up to one
        // per host core), compiled at once by helper processes
        // (prefetch_compiles).  The search then runs as above on the cached
        // code objects: the same decisions, the same plan.
        std::vector<const Plan*> batch;
        std::vector<char> queued(cand.size(), 0);
        std::queue<std::vector<int>> q;
        q.push(outcome);
        for (size_t visits = 0; !q.empty() && batch.size() < procs && visits < 4096; ++visits) {
          std::vector<int> h = std::move(q.front());
          q.pop();
          const long s = next_needed(h);
          if (s < 0) continue;
          if (!queued[s] && !jit_code_cached(cand[s])) queued[s] = 1, batch.push_back(&cand[s]);
          for (int r : {kDirty, kCleanScratch, kClean0}) {
            std::vector<int> h2 = h;
            h2[s] = r;
            q.push(std::move(h2));
          }
        }
        const auto t0 = std::chrono::steady_clock::now();
        prefetch_compiles(batch, procs);
        t_compile_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      }
      compile_one((size_t)k);
      outcome[k] = src[k] != SUP_OK         ? kFail
                   : scans[k].loop_scratch  ? kDirty
                   : scans[k].scratch_bytes ? kCleanScratch
                                            : kClean0;
    }
    if (outcome[idx[pp]] == kFail) return SUP_EHIP;  // the probe's compile error is set
    auto pick = [&]() {
      int c = -1, bare = -1;
      for (size_t i : idx) {
        if (!clean(i)) continue;
        if (c < 0 || cand[i].seg_ops < cand[c].seg_ops) c = (int)i;
        if (scans[i].scratch_bytes == 0 && (bare < 0 || cand[i].seg_ops < cand[bare].seg_ops)) bare = (int)i;
      }
      return (bare >= 0 && c >= 0 && cand[bare].seg_ops <= cand[c].seg_ops * (1.0 + kScratchTolerance)) ? bare : c;
    };
    const int best = pick();
    if (std::getenv("SUP_JIT_VERBOSE"))
      for (size_t i : idx)
        if (done[i])
          std::fprintf(stderr, "  budget %d: ops %.4f rc %d vgprs %d spills %d scratch %dB (loop %d of %d insts, %d readlane)%s\n",
                       budgets[i], cand[i].seg_ops, src[i], scans[i].vgprs, scans[i].vgpr_spills,
                       scans[i].scratch_bytes, scans[i].loop_scratch, scans[i].loop_insts, scans[i].loop_readlane,
                       (int)i == best ? "  <- chosen" : "");
    if (best < 0) {
      set_error("segmented walk: every budget's kernel touches scratch inside its walk loop (or fails to compile)");
      return SUP_EHIP;
    }
    P = std::move(cand[best]);
  }
  P.seg_skip = seg_skip_fraction_plan(P, 2048);
  if (P.start_tab_on) seg_start_table(P);
  if (std::getenv("SUP_JIT_VERBOSE"))
    std::fprintf(stderr, "seg plan n=%d m=%d b=%d ops/step=%.4f regs=%d cc=%d table=%zu B (columns %zu B) key=%016llx "
                 "(storage plans evaluated: %ld)\n", n, m, P.seg_b, P.seg_ops, P.seg_regs, P.seg_cc,
                 P.jtab.size() * sizeof(double), P.seg_cbase * sizeof(double), (unsigned long long)P.jit_key,
                 g_fit_calls.load());
  return SUP_OK;
}

// The generated kernel source of plan P with `kp` SGPR pieces per step region
// (jit_internal.hpp: the compile's register retry regenerates with fewer).
std::string seg_source(const Plan& P, int kp) {
  Plan Q = P;
  Q.seg_kp = kp;
  return Gen(Q).source();
}

}  // namespace sup
