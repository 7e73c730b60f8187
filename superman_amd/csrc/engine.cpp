// engine.cpp — plans, per-device contexts, single/static/chunked schedulers.
#include "engine.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>

#include <elf.h>
#include <link.h>  // dl_iterate_phdr: the library build id (checkpoint header)
#include <unistd.h>  // environ

namespace sup {

// ---------------------------------------------------------------- errors --
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* last_error() { return g_err.c_str(); }


// -------------------------------------------------------------- matrices --
int to_double(const void* mat, sup_dtype t, int n, std::vector<double>& out) {
  if (!mat || n < 1 || n > SUP_MAX_N) {
    set_error("matrix pointer is null or n is outside [1, 64]");
    return SUP_EINVAL;
  }
  const size_t nn = (size_t)n * n;
  out.resize(nn);
  switch (t) {
    case SUP_INT32: {
      const int32_t* a = (const int32_t*)mat;
      for (size_t i = 0; i < nn; ++i) out[i] = (double)a[i];
      return SUP_OK;
    }
    case SUP_FLOAT32: {
      const float* a = (const float*)mat;
      for (size_t i = 0; i < nn; ++i) out[i] = (double)a[i];
      return SUP_OK;
    }
    case SUP_FLOAT64:
      std::memcpy(out.data(), mat, nn * sizeof(double));
      return SUP_OK;
  }
  set_error("unknown sup_dtype");
  return SUP_EINVAL;
}

void nw_start(const double* A, int n, double* x0, double* p0) {
  double p = 1.0;
  for (int j = 0; j < n; ++j) {
    double rs = 0.0;
    for (int k = 0; k < n; ++k) rs += A[(size_t)j * n + k];
    x0[j] = A[(size_t)j * n + (n - 1)] - rs / 2;
    p *= x0[j];
  }
  *p0 = p;
}

Layout default_layout(int n) {
  Layout l;
  const int nb = n - 1;
  l.L = nb < 6 ? nb : 6;
  const int rest = nb - l.L;
  // >= 2^10 walk steps per wave-chunk when possible, and at most 2^20
  // wave-chunks (8 MiB of partials) — fine-grained enough that the dynamic
  // chunk queue balances a whole MI355X (~5k resident waves) to < 1 %.
  // Small n (rest < 23): the walk shortens (down to 2^6 steps) until there are
  // 2^13 wave-chunks, so the whole chip walks instead of a few waves.
  int m = rest < 10 ? rest : 10;
  if (rest - m < 13) m = std::max(std::min(rest, 6), rest - 13);
  if (rest - 20 > m) m = rest - 20;
  if (m > 31) m = 31;  // 32-bit walk index in the kernels (n > 58 only)
  l.m = m;
  l.h = rest - m;
  return l;
}

// Walk-column order that keeps the row prefixes small: the first column is
// tried exhaustively, the rest is greedy (fewest newly covered rows, then
// fewest nonzeros, then lowest index); the order with the lowest prefix cost
// (VALU ops per Gray step, DESIGN.md §3.2: walk bit k flips with frequency
// 2^-(k+1) and costs 8*nblk adds, 8*nblk muls and one accumulate)
// wins.  Column n-1 (Nijenhuis-Wilf) is never a walk column.
std::vector<int> greedy_walk_order(const double* A, int n, int count) {
  const int nb = n - 1;
  count = std::min(count, nb);
  // column c's rows as a bit set (n <= 64): a candidate's new rows are one
  // popcount (the -o leaves plan a new matrix each: 0.3-0.7 ms -> ~0.05 ms)
  std::vector<uint64_t> cm(nb, 0);
  std::vector<int> nnz(n, 0);
  for (int c = 0; c < nb; ++c) {
    for (int i = 0; i < n; ++i)
      if (A[(size_t)i * n + c] != 0.0) cm[c] |= 1ull << i;
    nnz[c] = __builtin_popcountll(cm[c]);
  }
  auto greedy_from = [&](int first) {
    std::vector<int> order{first};
    std::vector<char> used(n, 0);
    used[first] = 1;
    uint64_t placed = cm[first];
    while ((int)order.size() < count) {
      int best = -1, bnew = 1 << 30;
      for (int c = 0; c < nb; ++c) {
        if (used[c]) continue;
        const int nw = __builtin_popcountll(cm[c] & ~placed);
        if (nw < bnew || (nw == bnew && nnz[c] < nnz[best])) best = c, bnew = nw;
      }
      used[best] = 1;
      order.push_back(best);
      placed |= cm[best];
    }
    return order;
  };
  // prefix_cost over the bit sets (the same row counts, so the same cost)
  auto cost_of = [&cm](const std::vector<int>& walk) {
    uint64_t placed = 0;
    double cost = 0.0, w = 0.5;
    for (int c : walk) {
      placed |= cm[c];
      cost += w * (16.0 * ((__builtin_popcountll(placed) + 7) / 8) + 1.0);
      w *= 0.5;
    }
    return cost;
  };
  std::vector<int> best;
  double bcost = 1e300;
  for (int f = 0; f < nb && count > 0; ++f) {
    std::vector<int> o = greedy_from(f);
    const double c = cost_of(o);
    if (c < bcost) bcost = c, best = o;
  }
  return best;
}

// ---- SkipPer column order (round 5) ----------------------------------------
// The SkipPer kernel's zero check at a wave-chunk's first state ends the chunk
// when a row that no walk and no lane column touches ("uniform tail" row) is
// exactly zero: its value is fixed for the whole chunk (x0 plus the chunk
// bits' columns).  Which rows those are is decided by the set of walk + lane
// columns, so the column map decides how many chunks SkipPer walks at all.
// SkipOrder's own map (identity) walks 25.7 % of config 5's states
// (profiles/r5); a map chosen for these chunk ends walks 10.6 % at a lower
// prefix cost (tools/probes/skip_sim.c).
namespace {
struct SkipOrderEval {
  const double* A;
  int n, m, L;
  std::vector<uint64_t> cm;  // column -> rows (bit set)
  std::vector<double> x0;
  // prefix-block cost of the first m columns (walk_cost's terms)
  double prefix_cost(const std::vector<int>& o) const {
    uint64_t placed = 0;
    double cost = 0.0, w = 0.5;
    for (int k = 0; k < m; ++k) {
      placed |= cm[o[k]];
      cost += w * (16.0 * ((__builtin_popcountll(placed) + 7) / 8) + 1.0);
      w *= 0.5;
    }
    return cost + w * 16.0 * ((n + 7) / 8);
  }
  // sampled fraction of wave-chunks whose first state has an exactly zero
  // uniform tail row (integer matrices: every sum here is exact); chunk
  // indices drawn as in seg_skip_estimate (jit.cpp)
  double kill(const std::vector<int>& o, int samples) const {
    const int nb = n - 1;
    uint64_t wl = 0;  // rows touched by a walk or lane column
    std::vector<char> used(nb, 0);
    for (int k = 0; k < m + L; ++k) wl |= cm[o[k]], used[o[k]] = 1;
    std::vector<int> high;
    for (int c = 0; c < nb; ++c)
      if (!used[c]) high.push_back(c);
    struct Row {
      double x0;
      std::vector<std::pair<int, double>> hi;
    };
    std::vector<Row> rows;
    for (int r = 0; r < n; ++r) {
      if ((wl >> r) & 1u) continue;
      Row q{x0[r], {}};
      for (int k = 0; k < (int)high.size(); ++k)
        if (A[(size_t)r * n + high[k]] != 0.0) q.hi.push_back({k, A[(size_t)r * n + high[k]]});
      rows.push_back(std::move(q));
    }
    if (rows.empty()) return 0.0;
    const int h = (int)high.size();
    int killed = 0;
    for (int s = 0; s < samples; ++s) {
      const uint64_t a = h ? ((uint64_t)s * 0x9E3779B97F4A7C15ull) >> (64 - std::min(h, 63)) : 0;
      const uint64_t g = a ^ (a >> 1);
      for (const Row& q : rows) {
        double v = q.x0;
        for (const auto& e : q.hi)
          if ((g >> e.first) & 1u) v += e.second;
        if (v == 0.0) {
          ++killed;
          break;
        }
      }
    }
    return (double)killed / samples;
  }
  double eff(const std::vector<int>& o, int samples) const { return prefix_cost(o) * (1.0 - kill(o, samples)); }
};
}  // namespace

// Walk + lane columns (m + L of them, walk first) for the SkipPer walk of an
// integer matrix, chosen on ops per nominal step x the fraction of chunks not
// ended at their first state; false when SkipOrder's own map (columns
// L..L+m-1 walk, 0..L-1 lanes) is not clearly worse (the estimate does not see
// the jumps inside a chunk, which favour SkipOrder's map: it must be beaten
// by 2x).  Deterministic (fixed seeds, results gathered in start order), so
// every process and host plans the same walk.  Random-restart local search:
// starts = the greedy prefix order, SkipOrder's map and random column sets;
// each start takes kRounds random moves (swap a walk or lane column with an
// unused one, or a walk with a lane column), keeping improvements on a
// 512-sample estimate; the best end on 8192 samples wins.
bool skip_walk_order(const double* A, int n, const Layout& lay, std::vector<int>& out,
                     const std::vector<int>* baseline, double factor) {
  const int nb = n - 1, m = lay.m, L = lay.L;
  if (m < 3 || m + L >= nb) return false;
  SkipOrderEval E{A, n, m, L, std::vector<uint64_t>(nb, 0), std::vector<double>(n)};
  for (int c = 0; c < nb; ++c)
    for (int i = 0; i < n; ++i)
      if (A[(size_t)i * n + c] != 0.0) E.cm[c] |= 1ull << i;
  double p0;
  nw_start(A, n, E.x0.data(), &p0);
  std::vector<int> ident;
  for (int k = 0; k < m; ++k) ident.push_back(L + k);
  for (int e = 0; e < L; ++e) ident.push_back(e);
  constexpr int kStarts = 16, kRounds = 1500, kScreen = 512, kFinal = 8192;
  std::vector<std::vector<int>> starts;
  {
    std::vector<int> g = greedy_walk_order(A, n, m + L);
    starts.push_back(g);
    starts.push_back(ident);
    uint64_t z = 0x5EED5C1Bull;
    auto rnd = [&z]() {  // splitmix64
      uint64_t x = (z += 0x9E3779B97F4A7C15ull);
      x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
      x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
      return x ^ (x >> 31);
    };
    while ((int)starts.size() < kStarts) {
      std::vector<int> cols(nb);
      for (int c = 0; c < nb; ++c) cols[c] = c;
      for (int i = nb - 1; i > 0; --i) std::swap(cols[i], cols[rnd() % (uint64_t)(i + 1)]);
      cols.resize(m + L);
      starts.push_back(cols);
    }
  }
  std::vector<std::vector<int>> ends(starts.size());
  std::vector<double> effs(starts.size());
  auto search = [&](size_t si) {
    uint64_t z = 0xC0FFEEull + 7919ull * si;
    auto rnd = [&z]() {
      uint64_t x = (z += 0x9E3779B97F4A7C15ull);
      x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
      x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
      return x ^ (x >> 31);
    };
    std::vector<int> cur = starts[si];
    double cv = E.eff(cur, kScreen);
    std::vector<char> in(nb, 0);
    for (int c : cur) in[c] = 1;
    for (int it = 0; it < kRounds; ++it) {
      std::vector<int> t = cur;
      const int a = (int)(rnd() % (uint64_t)(m + L));
      // the other side of the move: an unused column, or (walk <-> lane) a
      // position on the other side
      const int n_out = nb - (m + L), n_other = a < m ? L : m;
      const int pick = (int)(rnd() % (uint64_t)(n_out + n_other));
      int incoming = -1;
      if (pick < n_out) {
        int k = pick;
        for (int c = 0; c < nb; ++c)
          if (!in[c] && k-- == 0) {
            incoming = c;
            break;
          }
        t[a] = incoming;
      } else {
        const int b = a < m ? m + (pick - n_out) : pick - n_out;
        std::swap(t[a], t[b]);
      }
      const double v = E.eff(t, kScreen);
      if (v < cv) {
        if (incoming >= 0) in[cur[a]] = 0, in[incoming] = 1;
        cur = std::move(t), cv = v;
      }
    }
    ends[si] = cur;
    effs[si] = E.eff(cur, kFinal);
  };
  {
    std::atomic<size_t> next{0};
    auto worker = [&]() {
      for (size_t i = next++; i < starts.size(); i = next++) search(i);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < std::min<int>(plan_threads(), (int)starts.size()); ++t) th.emplace_back(worker);
    worker();
    for (auto& t : th) t.join();
  }
  size_t bi = 0;
  for (size_t i = 1; i < ends.size(); ++i)
    if (effs[i] < effs[bi] - 1e-12) bi = i;
  const std::vector<int>& base = baseline && (int)baseline->size() == m + L ? *baseline : ident;
  const double e_base = E.eff(base, kFinal);
  if (std::getenv("SUP_JIT_VERBOSE"))
    std::fprintf(stderr, "chunk-end column search n=%d: best eff %.4f (cost %.3f, kill %.3f) vs the baseline's %.4f\n",
                 n, effs[bi], E.prefix_cost(ends[bi]), E.kill(ends[bi], kFinal), e_base);
  if (!(effs[bi] < factor * e_base)) return false;
  out = ends[bi];
  return true;
}

// A prefix-blocked plan of an integer matrix whose walk is predicted to take
// >= kChunkEndSearchSec (every state, walk_cost's ops): its walk + lane columns
// searched for chunk ends (skip_walk_order against its greedy order; taken when
// it cuts ops x chunks walked by 10 %).  Deterministic, from the matrix alone.
static constexpr double kChunkEndSearchSec = 4.0;
// fp64 VALU lane-ops per second of one MI355X on the walk kernels (measured:
// 46.6 ops/step at 7.98e11 steps/s on the n=40 bench), for the planners' time
// predictions (this search, SkipPer's, jit's auto mode).
static constexpr double kLaneOpsPerSec = 3.7e13;
int improve_sparse_plan(const double* A, int n, const Layout& lay, Plan& P) {
  if (P.kind != kWalkSparse || !P.integral || lay.m < 3 ||
      std::ldexp(1.0, n - 1) * walk_cost(P) / kLaneOpsPerSec < kChunkEndSearchSec)
    return SUP_OK;
  std::vector<int> base;
  for (int k = 0; k < lay.m; ++k) base.push_back(P.colmap[lay.L + k]);
  for (int e = 0; e < lay.L; ++e) base.push_back(P.colmap[e]);
  SegChoice c;
  if (!skip_walk_order(A, n, lay, c.order, &base, 0.9)) return SUP_OK;
  Plan Q;
  const int rc = make_plan(A, n, kWalkSparse, false, lay, Q, &c);
  if (rc == SUP_OK) P = std::move(Q);
  return rc;
}

double walk_cost(const Plan& P) {
  if (P.kind == kWalkDense) return 2.0 * P.n + 1.0;
  if (P.kind == kWalkSeg) return seg_walk_cost(P);
  double cost = 0.0, w = 0.5;
  for (int k = 0; k < P.lay.m; ++k, w *= 0.5) cost += w * (16.0 * P.nblk[P.lay.L + k] + 1.0);
  return cost + w * 16.0 * ((P.n + 7) / 8);  // tail: the rest of the walk bits, bounded
}

// ops per nominal Gray step, chunks the walk skips discounted: what the
// planner compares walks on (the reported cost model stays per walked step)
static double walk_cost_eff(const Plan& P) {
  return P.kind == kWalkSeg ? walk_cost(P) * (1.0 - P.seg_skip) : walk_cost(P);
}

// SUP_NO_CHUNK_ENDS=1 (experiments, A/B): no chunk ends in the prefix-blocked
// and exact walks (walk_sparse.hip); the sums are the same, the ended chunks'
// terms being exact zeros.
static bool no_chunk_ends() {
  static const bool off = [] {
    const char* e = std::getenv("SUP_NO_CHUNK_ENDS");
    return e && std::atoi(e) != 0;
  }();
  return off;
}

int make_plan(const double* A, int n, WalkKind kind, bool identity_map, const Layout& lay, Plan& P,
              const SegChoice* choice) {
  if (n < 1 || n > SUP_MAX_N) {
    set_error("n must be in [1, 64]");
    return SUP_EINVAL;
  }
  P = Plan();
  P.n = n;
  P.NP = pad8(n);
  P.kind = kind;
  P.lay = lay;
  P.integral = true;
  for (size_t i = 0; i < (size_t)n * n && P.integral; ++i) P.integral = A[i] == std::floor(A[i]);
  const int nb = n - 1;  // flippable columns (column n-1 is the Nijenhuis-Wilf column)
  const int L = lay.L, m = lay.m;

  // ---- engine bit -> matrix column
  P.colmap.resize(nb);
  for (int e = 0; e < nb; ++e) P.colmap[e] = e;
  // a caller-chosen walk + lane order: a map searched for chunk ends
  // (skip_walk_order: SkipPer, and long prefix-blocked / exact / double-double
  // walks of integer matrices), or the exact walk's greedy order (exact.cpp)
  const bool given_order = (kind == kWalkSkip || kind == kWalkDense || kind == kWalkSparse) && choice && m > 0;
  if (!identity_map && (kind == kWalkSparse || kind == kWalkSeg || given_order) && m > 0) {
    // walk bits get the greedy prefix order (greedy_walk_order; the segmented
    // walk: seg_walk_order), lane bits the next L columns of that order, high
    // bits the rest in matrix order.
    int segb = 0;
    std::vector<int> order;
    // a recorded order (plan choices on disk) is taken only when it is a set of
    // m + L distinct flippable columns: a corrupted or foreign record would
    // index past the matrix or give a column map that is not a permutation
    auto valid_order = [&](const std::vector<int>& o) {
      if ((int)o.size() != m + L) return false;
      std::vector<char> seen(nb, 0);
      for (int v : o) {
        if (v < 0 || v >= nb || seen[v]) return false;
        seen[v] = 1;
      }
      return true;
    };
    if (given_order) {
      if (!valid_order(choice->order)) {
        set_error("walk column order: not m + L distinct flippable columns");
        return SUP_EINVAL;
      }
      order = choice->order;
    } else if (kind == kWalkSeg && choice && valid_order(choice->order) && choice->b >= 0 && choice->b <= m) {
      order = choice->order;
      segb = choice->b;
    } else {
      order = kind == kWalkSeg ? seg_walk_order(A, n, m, m + L, &segb, lay.cc_cap) : greedy_walk_order(A, n, m + L);
    }
    P.seg_b = segb;
    if (kind == kWalkSeg) P.seg_order.assign(order.begin(), order.begin() + (m + L));
    std::vector<char> used(n, 0);
    for (int k = 0; k < m; ++k) P.colmap[L + k] = order[k], used[order[k]] = 1;
    for (int e = 0; e < L; ++e) P.colmap[e] = order[m + e], used[order[m + e]] = 1;
    int e = L + m;
    // High bits (the wave-chunk index).  The segmented walk on an integer
    // matrix skips the wave-chunks whose rows untouched by the walk columns are
    // exactly zero in every lane; a high column with no nonzero in those rows
    // never changes that, so those columns take the top bits: contiguous
    // shards (sup_perman_shard, -p5) then see the same skip pattern.  (Config
    // 5 before: the top chunk bit alone decided skipping, half the shards had
    // nothing to walk at 2, 4 and 8 GPUs.)  Otherwise matrix order.
    std::vector<char> top(n, 0);
    if (kind == kWalkSeg || given_order) {
      bool integral = true;
      for (size_t i = 0; i < (size_t)n * n && integral; ++i) integral = A[i] == std::floor(A[i]);
      // (SkipPer ends a chunk on a row no walk and no lane column touches)
      std::vector<char> wrow(n, 0);
      for (int k = 0; k < (given_order ? m + L : m); ++k)
        for (int i = 0; i < n; ++i) wrow[i] |= A[(size_t)i * n + order[k]] != 0.0;
      for (int c = 0; c < nb && integral; ++c) {
        top[c] = 1;
        for (int i = 0; i < n; ++i)
          if (!wrow[i] && A[(size_t)i * n + c] != 0.0) top[c] = 0;
      }
    }
    for (int pass = 0; pass < 2; ++pass)
      for (int c = 0; c < nb; ++c)
        if (!used[c] && top[c] == pass) P.colmap[e++] = c;
  }

  // ---- engine row order
  P.rowperm.resize(n);
  for (int j = 0; j < n; ++j) P.rowperm[j] = j;
  P.nblk.assign(std::max(nb, 1), 0);
  P.rowmask.assign(n, 0);
  if (kind != kWalkDense) {
    // rows in first-touch order over the walk columns (walk order), then the rest
    std::vector<char> placed(n, 0);
    std::vector<int> order;
    order.reserve(n);
    for (int k = 0; k < m; ++k) {
      const int c = P.colmap[L + k];
      for (int i = 0; i < n; ++i)
        if (!placed[i] && A[(size_t)i * n + c] != 0.0) {
          placed[i] = 1;
          order.push_back(i);
        }
      P.nblk[L + k] = ((int)order.size() + 7) / 8;
    }
    for (int i = 0; i < n; ++i)
      if (!placed[i]) order.push_back(i);
    P.rowperm = order;
    if (kind == kWalkSeg) {  // segment 0 sub-ordered (jit.cpp)
      std::vector<int> walk(m);
      for (int k = 0; k < m; ++k) walk[k] = P.colmap[L + k];
      P.rowperm = seg_row_order(A, n, walk);
    }
    // a walk column may touch no new row: nblk must still cover its own rows,
    // which are all inside the prefix, so the prefix count above is correct.
  }
  for (int e = 0; e < nb; ++e)
    if (e < L || e >= L + m) P.nblk[e] = (n + 7) / 8;  // not used by the walk; keep sane

  // ---- tables
  P.cols.assign((size_t)2 * std::max(nb, 1) * P.NP, 0.0);
  for (int e = 0; e < nb; ++e) {
    const int c = P.colmap[e];
    for (int j = 0; j < n; ++j) {
      const double v = A[(size_t)P.rowperm[j] * n + c];
      P.cols[(size_t)(2 * e) * P.NP + j] = v;
      P.cols[(size_t)(2 * e + 1) * P.NP + j] = -v;
    }
  }
  std::vector<double> x0(n);
  double p0;
  nw_start(A, n, x0.data(), &p0);
  P.x0.assign(P.NP, 0.0);
  for (int j = 0; j < n; ++j) P.x0[j] = x0[P.rowperm[j]];

  // ---- skipper metadata
  P.umask = 0;
  for (int j = 0; j < n; ++j) {
    const int i = P.rowperm[j];
    bool lane_touched = false;
    for (int e = 0; e < L; ++e)
      if (A[(size_t)i * n + P.colmap[e]] != 0.0) lane_touched = true;
    if (!lane_touched) P.umask |= 1ull << j;
    uint64_t rm = 0;
    for (int k = 0; k < m; ++k)
      if (A[(size_t)i * n + P.colmap[L + k]] != 0.0) rm |= 1ull << k;
    P.rowmask[j] = rm;
    // a lane-uniform row no walk column touches is constant over a wave-chunk:
    // exactly zero at the chunk's first state, the chunk ends there (walk_sparse)
    if ((kind == kWalkSparse || kind == kWalkDense) && !lane_touched && rm == 0 && !no_chunk_ends())
      P.chunk_ends |= 1ull << j;
  }
  if (kind == kWalkSeg) return build_seg(P, choice ? choice->budget : 0);
  return SUP_OK;
}

// Auto mode's bar where nothing bounds the saving (orders below
// kJitWarmMinN; jit != 0 never asks): no walk that short repays a plan.
static constexpr double kJitMinSavingSec = 3.0;
// Auto mode (jit = 0) decides once per matrix and request, and every later
// run follows that decision (AutoRecord): the plan (walk-order search +
// compiles, seg_cold_predict: ~1.6 s at n = 40 on a GPU box, cold) is paid
// once, the walk time it saves on every run.  So a plan is started when the
// walk time it can save over kAutoRuns runs would repay it — the bench
// matrix, a 0.5 s saving per run on one MI355X, specialises on a fresh host;
// a matrix walked once loses at most the plan's cost.  Once the search and
// the compiler check have run their cost is spent, and the segmented walk is
// taken when it saves kJitWarmSavingSec per run.
static constexpr double kAutoRuns = 4.0;
// When an earlier process recorded this matrix's segmented-walk choices (disk
// cache, make_seg_plan), the plan is rebuilt in ~5-50 ms and its code object
// loads from disk: auto mode specialises whenever the walk saves more than this.
static constexpr double kJitWarmSavingSec = 0.1;
// Below this order no walk lasts kJitWarmSavingSec (2^29 steps at ~3e12/s):
// auto mode does not look at the disk cache.
static constexpr int kJitWarmMinN = 30;

static int plan_for_uncached(const double* A, int n, sup_kernel kernel, const Layout& lay, Plan& P, int jit,
                             int ndev, int dev, double min_saving);
static double auto_min_saving(const double* A, int n, const Layout& lay, int jit);

// Chunk start of the segmented walk (start index's column sums, row copies,
// trees of every cached state), in VALU ops per lane: ~750 fitted from config
// 3's kernel time against its walk length, ~1700 from the d = 0.2 companion's
// (profiles/r2/probe_walklen.log).
static constexpr double kSegStartOps = 2048.0;

// The segmented walk on the default layout, or on longer wave-chunks where its
// steps are cheap: a chunk's walk (2^m steps) should be >= 32 chunk starts.
// Both walks are planned and the one with fewer ops per nominal step, chunk
// start and chunk skip included, wins.  At least 2^14 chunks remain (8 per
// resident wave of one GPU, one per wave of each of 8 GPUs).  Round 6 lowered
// this from 2^15: config 2 (n = 32) then walks m = 11 instead of 10, 0.555
// against 0.580 ms (chunk starts 13.5 -> 10.2 % of the wave cycles, queue tail
// 3.4 -> 7 %; profiles/r6/cfg2_knobs.log), config 3 m = 15 instead of 14
// (1.905 against 1.92-1.94 ms, profiles/r6/cfg3_m.log).  The layout depends
// only on the matrix, so every GPU count sums the same chunks (bit-identical
// results).
static constexpr int kSegMinChunkBits = 14;
static uint64_t knob_hash_env();

// Disk key of a segmented-walk plan: what its choices depend on, the layout
// request, experiment knobs and the toolchain the choices were priced with.
// For a non-integer matrix the choices (walk-order search, trees, budget, the
// generated source) depend on the zero pattern only, so the key is the
// pattern: matrices that differ only in their nonzero values (a rescaled row,
// another draw of the same pattern) share one record and one kernel.  Integer
// matrices add their values (the chunk-skip estimate and the column order of
// the chunk bits look at exact zeros of row sums).
static uint64_t seg_disk_key(const double* A, int n, const Layout& lay) {
  uint64_t h = 0x5eed5e9a11ull ^ jit_toolchain_hash();
  auto mix = [&h](const void* p, size_t bytes) {
    const unsigned char* c = (const unsigned char*)p;
    for (size_t i = 0; i < bytes; ++i) h = (h ^ c[i]) * 1099511628211ull;
  };
  const size_t nn = (size_t)n * n;
  bool integral = true;
  for (size_t i = 0; i < nn && integral; ++i) integral = A[i] == std::floor(A[i]);
  const int32_t head[] = {6 /* format: bump when the planner changes */, n, lay.L, lay.m, (int32_t)lay.fixed, (int32_t)integral};
  mix(head, sizeof head);
  if (integral) {
    mix(A, nn * sizeof(double));
  } else {
    std::vector<unsigned char> pat((nn + 7) / 8, 0);
    for (size_t i = 0; i < nn; ++i)
      if (A[i] != 0.0) pat[i / 8] |= (unsigned char)(1u << (i % 8));
    mix(pat.data(), pat.size());
  }
  const uint64_t k = knob_hash_env();
  mix(&k, sizeof k);
  return h;
}

static int make_seg_plan(const double* A, int n, const Layout& lay, Plan& P) {
  // a later process rebuilds the plan from its recorded choices (no search,
  // no compiler check: ~0.1 s instead of seconds)
  const uint64_t dkey = seg_disk_key(A, n, lay);
  {
    int m2 = 0;
    SegChoice c;
    if (seg_choice_load(dkey, &m2, &c) && m2 >= 3 && m2 <= lay.m + lay.h && (!lay.fixed || m2 == lay.m)) {
      Layout l2 = lay;
      l2.m = m2;
      l2.h = lay.m + lay.h - m2;
      l2.cc_cap = c.cc_cap;
      if (make_plan(A, n, kWalkSeg, false, l2, P, &c) == SUP_OK) return SUP_OK;
    }
  }
  const auto t_cold = std::chrono::steady_clock::now();
  // a short walk whose 4-cached-bit kernel touches scratch in its loop
  // (build_seg's check) is planned again with 3 cached bits
  auto plan = [A, n](const Layout& l, Plan& Q) {
    int r = make_plan(A, n, kWalkSeg, false, l, Q);
    if (r == SUP_OK && Q.seg_loop_scratch && l.cc_cap > 3) {
      Layout l3 = l;
      l3.cc_cap = 3;
      r = make_plan(A, n, kWalkSeg, false, l3, Q);
    }
    return r;
  };
  int rc = plan(lay, P);
  if (rc) return rc;
  if (!lay.fixed) {
    const int mmax = std::min(lay.m + lay.h - kSegMinChunkBits, 31);
    int m2 = lay.m;
    while (m2 < mmax && std::ldexp(walk_cost(P), m2) < 32.0 * kSegStartOps) ++m2;
    if (m2 != lay.m) {
      Layout l2 = lay;
      l2.m = m2;
      l2.h = lay.m + lay.h - m2;
      Plan s2;
      if (plan(l2, s2) == SUP_OK) {
        auto eff = [](const Plan& q) {
          return (1.0 - q.seg_skip) * (walk_cost(q) + std::ldexp(kSegStartOps, -q.lay.m));
        };
        if (eff(s2) < eff(P)) P = std::move(s2);
      }
    }
  }
  SegChoice c;
  c.order = P.seg_order;
  c.b = P.seg_b;
  c.budget = P.seg_budget;
  c.cc_cap = P.lay.cc_cap;
  seg_choice_store(dkey, P.lay.m, c);
  // what this cold plan cost (search + the compiler check's compiles): auto
  // mode's cold bar on this host (plan_for)
  const double cold_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_cold).count();
  seg_cost_store(n, cold_s);
  if (std::getenv("SUP_JIT_VERBOSE"))
    std::fprintf(stderr, "cold segmented plan n=%d: %.3f s (compiles %.3f s wall on this thread)\n", n, cold_s,
                 jit_compile_ms_thread() * 1e-3);
  return SUP_OK;
}

// Plans are pure functions of (matrix, request, layout): repeated calls on the
// same matrix (the bench's steps, a shard per rank, -p6 items, reductions
// revisiting a leaf) reuse the plan instead of re-running the walk-order
// search (~5-15 ms at n = 40, comparable to an 8-GPU shard's walk).
namespace {
struct PlanKey {
  uint64_t hash;
  int n, kernel, L, m, jit, ndev;
  bool fixed;      // walk length asked for (sup_opts::walk_log2): make_seg_plan keeps it
  uint64_t knobs;  // SUP_JIT_* experiment settings the planner and code generator read
  // Not in the key: auto mode's bar (auto_min_saving), which moves with the
  // disk cache (this matrix's choices recorded, this host's cold plan cost) —
  // possibly written meanwhile by another rank or thread.  The first auto-mode
  // decision for a matrix and request is kept for the process, so a call after
  // sup_prepare / sup_plan_key (the bench's plan-agreement check) walks the
  // plan that was checked.
  bool operator<(const PlanKey& o) const {
    return std::tie(hash, n, kernel, L, m, jit, ndev, fixed, knobs) <
           std::tie(o.hash, o.n, o.kernel, o.L, o.m, o.jit, o.ndev, o.fixed, o.knobs);
  }
};
std::mutex g_plan_mu;
// cached plans are shared, not copied: a cached call takes a reference (the
// segmented plan's source, tables and trees are ~200 KB at n = 40)
std::map<PlanKey, std::pair<std::vector<double>, std::shared_ptr<const Plan>>> g_plans;
constexpr size_t kPlanCacheMax = 32;

// Hash of every SUP_JIT_* variable that shapes a plan or its generated source
// (experiment knobs), so a process that changes one gets a fresh plan; the
// cache location, source dumps and log verbosity do not change a plan.
uint64_t knob_hash() {
  uint64_t h = 1469598103934665603ull;
  for (char** e = environ; e && *e; ++e) {
    const char* v = *e;
    if (std::strncmp(v, "SUP_JIT_", 8) != 0 || !std::strncmp(v, "SUP_JIT_CACHE_DIR=", 18) ||
        !std::strncmp(v, "SUP_JIT_DUMP=", 13) || !std::strncmp(v, "SUP_JIT_VERBOSE=", 16) ||
        !std::strncmp(v, "SUP_JIT_COLD_RATIO=", 19))
      continue;
    for (const char* c = v; *c; ++c) h = (h ^ (unsigned char)*c) * 1099511628211ull;
    h = (h ^ 0xffu) * 1099511628211ull;
  }
  return h;
}
}  // namespace

static uint64_t knob_hash_env() { return knob_hash(); }

int plan_for_shared(const double* A, int n, sup_kernel kernel, const Layout& lay, std::shared_ptr<const Plan>& out,
                    int jit, int ndev, int dev, bool keep) {
  const size_t nn = (size_t)n * n;
  // in-process cache key only (the entry also keeps the matrix and compares
  // it): four independent FNV-style lanes, so the multiply chain is a quarter
  // as long (n = 32: 1.7 -> ~0.5 us per call)
  uint64_t l[4] = {1469598103934665603ull, 0x9e3779b97f4a7c15ull, 0xc2b2ae3d27d4eb4full, 0x165667b19e3779f9ull};
  size_t i = 0;
  for (; i + 4 <= nn; i += 4)
    for (int k = 0; k < 4; ++k) {
      uint64_t b;
      std::memcpy(&b, A + i + k, 8);
      l[k] = (l[k] ^ b) * 1099511628211ull;
    }
  for (; i < nn; ++i) {
    uint64_t b;
    std::memcpy(&b, A + i, 8);
    l[0] = (l[0] ^ b) * 1099511628211ull;
  }
  uint64_t h = l[0];
  for (int k = 1; k < 4; ++k) h = (h ^ l[k]) * 1099511628211ull;
  // ndev only feeds auto mode's compile-or-not decision
  const PlanKey key{h, n, (int)kernel, lay.L, lay.m, jit, jit == 0 ? ndev : 0, lay.fixed, knob_hash()};
  {
    std::lock_guard<std::mutex> g(g_plan_mu);
    auto it = g_plans.find(key);
    if (it != g_plans.end() && std::equal(A, A + nn, it->second.first.begin())) {
      out = it->second.second;
      return SUP_OK;
    }
  }
  auto P = std::make_shared<Plan>();
  const int rc = plan_for_uncached(A, n, kernel, lay, *P, jit, ndev, dev, auto_min_saving(A, n, lay, jit));
  if (rc) return rc;
  if (!keep) {  // a plan walked once (a batch's leaf): the cache keeps the caller's plans
    out = P;
    return SUP_OK;
  }
  std::lock_guard<std::mutex> g(g_plan_mu);
  {
    auto it = g_plans.find(key);  // another thread planned the same request meanwhile: its plan stands
    if (it != g_plans.end() && std::equal(A, A + nn, it->second.first.begin())) {
      out = it->second.second;
      return SUP_OK;
    }
  }
  if (g_plans.size() >= kPlanCacheMax) g_plans.clear();
  static uint64_t next_uid = 0;
  P->uid = ++next_uid;
  out = P;
  g_plans[key] = {std::vector<double>(A, A + nn), out};
  return SUP_OK;
}

int plan_for(const double* A, int n, sup_kernel kernel, const Layout& lay, Plan& P, int jit, int ndev, int dev) {
  std::shared_ptr<const Plan> sp;
  const int rc = plan_for_shared(A, n, kernel, lay, sp, jit, ndev, dev);
  if (rc == SUP_OK) P = *sp;
  return rc;
}

// SkipPer evaluates only the states its zero checks cannot rule out; its
// checks and jumps cost it efficiency per evaluated state.  Round 5's kernel
// (segment-start checks, walk_sparse's paired steps elsewhere) with the
// searched column map (skip_walk_order) on config 5 int: 19.3 modelled ops per
// visited state, 10.6 % visited, 0.779 s — 2.31e13 ops/s against the plain
// walks' 3.7e13 (profiles/r5/probe_skip_searched_map.log; SkipOrder's map:
// 0.69, round 4's per-state kernel: 0.37).  Round 6's kernel forms
// (walk_skip.hip: straight-line segments) walk the same states in 0.537 s,
// 3.35e13 ops/s: 0.90 — the price SkipPer is weighed at; the column search's
// threshold below keeps round 5's rate, so the plans (and bits) it picks are
// unchanged.
static constexpr double kSkipEfficiency = 0.62;
static constexpr double kSkipPriceEfficiency = 0.90;
// SkipPer walks predicted (every state, SkipOrder's map, at kSkipEfficiency)
// to take at least this long search their column map for chunk ends
// (~0.2-0.6 s of host time; config 5: 9.5 s predicted, 0.54 s walked after
// the search).
static constexpr double kSkipSearchMinSec = 4.0;

// Fraction of the states the SkipPer plan P evaluates, measured on a fixed
// sample of its wave-chunks (8 evenly spaced ranges, ~1/64 of the walk) on
// device `dev`; -1 without a device.  Deterministic: visited counts depend only
// on the matrix and the chunks, not on timing.
static double skip_visited_fraction(const Plan& P, int dev) {
  int nd = 0;
  if (device_count(&nd) != SUP_OK || nd < 1) return -1.0;
  if (dev < 0 || dev >= nd) dev = 0;
  const uint64_t C = P.lay.chunks(), len = std::max<uint64_t>(1, C / 512);
  uint64_t vis = 0, tot = 0;
  for (uint64_t i = 0; i < 8; ++i) {
    uint64_t c0 = (2 * i + 1) * C / 16;
    if (c0 + len > C) c0 = C - len;
    RangeResult r;
    if (run_range(dev, P, c0, c0 + len, true, r) != SUP_OK) return -1.0;
    vis += r.visited;
    tot += len << (P.lay.L + P.lay.m);
  }
  return tot ? (double)vis / (double)tot : 1.0;
}

// Auto mode's bar for starting a segmented plan: the walk time it can save
// per run must exceed the predicted cold plan cost (seg_cold_predict: n, this
// host's plan threads and its recorded speed) over kAutoRuns runs; ~0 (the
// warm bar) when an earlier process left this matrix's plan choices and
// kernel in the disk cache.
static double auto_min_saving(const double* A, int n, const Layout& lay, int jit) {
  if (jit != 0 || n < kJitWarmMinN) return kJitMinSavingSec;  // below: no walk lasts even the lowest bar
  if (seg_choice_exists(seg_disk_key(A, n, lay))) return kJitWarmSavingSec;
  return std::max(kJitWarmSavingSec, seg_cold_predict(n) / kAutoRuns);
}

// Auto mode's first decision per matrix and request, on disk (round 4).  The
// bar above moves with the cache: a cold run keeps the ahead-of-time walk
// where the search + compile would cost more than they save, and once a plan's
// choices are recorded (a --jit 1 run, another rank) the same command would
// specialise — a different operation order, so different last bits of an fp64
// result between two runs of one command.  So auto mode records what it
// decided the first time and later processes follow it (cold and warm runs
// print the same bits; --jit 1 / -1 pick a walk explicitly).  Recorded only
// where the decision can depend on the cache: auto mode (jit = 0) and a walk
// long enough to save the warm bar (n >= 37 dense: the -o leaves never write).
struct AutoRecord {
  uint64_t key = 0;
  int recorded = -1;  // -1: none (or not recordable), 0 / 1 as recorded
  bool active = false;
  AutoRecord(const double* A, int n, const Layout& lay, sup_kernel kernel, int ndev, int jit, double walk_s) {
    active = jit == 0 && n >= kJitWarmMinN && walk_s >= kJitWarmSavingSec;
    if (!active) return;
    key = seg_disk_key(A, n, lay) ^ (0x9e3779b97f4a7c15ull * (uint64_t)(1 + (int)kernel)) ^
          ((uint64_t)std::max(ndev, 1) << 48);
    recorded = auto_decision_load(key);
  }
  // records seg unless a decision is on disk; returns the decision to follow
  // (another process that decided first wins)
  bool store(bool seg) const {
    if (active && recorded < 0) return auto_decision_store(key, seg ? 1 : 0) == 1;
    return seg;
  }
};

static int plan_for_uncached(const double* A, int n, sup_kernel kernel, const Layout& lay, Plan& P, int jit,
                             int ndev, int dev, double min_saving) {
  // candidates in preference order; the cheapest by walk_cost wins
  std::vector<WalkKind> kinds;
  auto make_seg = [&](Plan& s) { return make_seg_plan(A, n, lay, s); };
  switch (kernel) {
    case SUP_KERNEL_SKIPPER: {
      // SkipPer only gains where some x_j(S) is exactly zero.  With a
      // non-integer entry that is a measure-zero coincidence, so SkipPer
      // evaluates every state; with integer entries the fraction it
      // evaluates is measured on a sample of its chunks (GPU; without a
      // device the request keeps SkipPer).  The segmented walk (same sum,
      // every state) runs instead when that is cheaper.
      int rc = make_plan(A, n, kWalkSkip, false, lay, P);
      if (rc) return rc;
      bool integral = true;
      for (size_t i = 0; i < (size_t)n * n && integral; ++i) integral = A[i] == std::floor(A[i]);
      // an integer matrix whose SkipPer walk is long: the column map chosen
      // for the chunks SkipPer ends at their first state (skip_walk_order;
      // decided from the matrix alone, so every device count and host plans
      // the same walk)
      if (integral && n >= 10 &&
          std::ldexp(1.0, n - 1) * walk_cost(P) / (kSkipEfficiency * kLaneOpsPerSec) >= kSkipSearchMinSec) {
        SegChoice c;
        Plan Q;
        if (skip_walk_order(A, n, lay, c.order, nullptr, 0.5) && make_plan(A, n, kWalkSkip, false, lay, Q, &c) == SUP_OK)
          P = std::move(Q);
      }
      if (jit < 0 || n < 10 || lay.m < 3) return SUP_OK;
      const double steps = std::ldexp(1.0, n - 1) / std::max(ndev, 1);
      double skip_cost = walk_cost(P) / (integral ? kSkipPriceEfficiency : 1.0);  // f <= 1
      const AutoRecord rec(A, n, lay, kernel, ndev, jit, steps * skip_cost / kLaneOpsPerSec);
      if (rec.recorded == 0) return SUP_OK;
      Plan s;
      if (rec.recorded == 1) {  // the recorded decision: the segmented walk (choices on disk)
        if (make_seg(s) == SUP_OK) P = std::move(s);
        return SUP_OK;
      }
      auto decide = [&]() -> bool {
        // auto mode: no segmented plan (its search takes ~0.1-1 s) where even a
        // free walk could not save the compile
        if (jit < 1 && steps * skip_cost / kLaneOpsPerSec < min_saving) return false;
        if (make_seg(s) != SUP_OK) return false;
        if (walk_cost_eff(s) >= skip_cost) return false;
        // the plan is paid for now: the segmented walk when it saves the warm bar
        const double bar = std::min(min_saving, kJitWarmSavingSec);
        if (jit < 1 && steps * (skip_cost - walk_cost_eff(s)) / kLaneOpsPerSec < bar) return false;
        if (integral) {
          const double f = skip_visited_fraction(P, dev);
          if (f < 0.0) return false;
          skip_cost *= f;
        }
        const double saved = steps * (skip_cost - walk_cost_eff(s)) / kLaneOpsPerSec;
        return walk_cost_eff(s) < skip_cost && (jit >= 1 || saved >= bar);
      };
      const bool seg = decide();
      if (rec.store(seg)) {
        if (seg) P = std::move(s);
        else if (make_seg(s) == SUP_OK) P = std::move(s);  // another process decided first
      }
      return SUP_OK;
    }
    case SUP_KERNEL_DENSE_PLAIN: return make_plan(A, n, kWalkDense, false, lay, P);
    case SUP_KERNEL_DENSE_LDS: {
      int rc = make_plan(A, n, kWalkDense, false, lay, P);
      P.lds = true;
      return rc;
    }
    case SUP_KERNEL_SEGMENTED:
      if (n < 10 || lay.m < 3) {
        set_error("the segmented walk needs n >= 10 (>= 3 walk bits)");
        return SUP_EUNSUPPORTED;
      }
      return make_seg(P);
    case SUP_KERNEL_SPARYSER: kinds = {kWalkSparse}; break;
    case SUP_KERNEL_DENSE: kinds = {kWalkDense}; if (n >= 8) kinds.push_back(kWalkSparse); break;
    default: set_error("unknown sup_kernel"); return SUP_EINVAL;
  }
  Plan best;
  int rc = make_plan(A, n, kinds[0], false, lay, best);
  if (rc == SUP_OK && kinds[0] == kWalkSparse) rc = improve_sparse_plan(A, n, lay, best);
  if (rc) return rc;
  for (size_t i = 1; i < kinds.size(); ++i) {
    Plan c;
    if (make_plan(A, n, kinds[i], false, lay, c) == SUP_OK && walk_cost(c) < walk_cost(best) &&
        (kinds[i] != kWalkSparse || improve_sparse_plan(A, n, lay, c) == SUP_OK))
      best = std::move(c);
  }
  const double best_s = std::ldexp(1.0, n - 1) / std::max(ndev, 1) * walk_cost(best) / kLaneOpsPerSec;
  const bool may_save = best_s >= min_saving;  // auto mode: skip the segmented plan's search where it cannot pay
  if (jit >= 0 && n >= 8 && lay.m >= 3) {
    const AutoRecord rec(A, n, lay, kernel, ndev, jit, best_s);
    Plan s;
    if (rec.recorded == 1) {  // the recorded decision: the segmented walk (choices on disk)
      if (make_seg(s) == SUP_OK) best = std::move(s);
    } else if (rec.recorded < 0 && (jit >= 1 || may_save)) {
      bool seg = false;
      const bool planned = make_seg(s) == SUP_OK;
      if (planned && walk_cost_eff(s) < walk_cost(best)) {
        // the search and the compiler check are paid now: the segmented walk
        // when it saves the warm bar per run
        const double steps = std::ldexp(1.0, n - 1) / std::max(ndev, 1);
        const double saved = steps * (walk_cost(best) - walk_cost_eff(s)) / kLaneOpsPerSec;
        seg = jit >= 1 || saved >= std::min(min_saving, kJitWarmSavingSec);
      }
      if (rec.store(seg) && planned) best = std::move(s);
    } else if (rec.recorded < 0) {
      if (rec.store(false) && make_seg(s) == SUP_OK) best = std::move(s);  // another process decided first
    }
  }
  P = std::move(best);
  return SUP_OK;
}

uint64_t plan_fingerprint(const Plan& P) {
  // everything that decides which wave-chunk sums which subsets, in what
  // order and with which operations: walk kind, layout, column map, the
  // signed column table, the segmented walk's choices and its kernel source
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](const void* p, size_t bytes) {
    const unsigned char* c = (const unsigned char*)p;
    for (size_t i = 0; i < bytes; ++i) h = (h ^ c[i]) * 1099511628211ull;
  };
  const int32_t head[] = {P.n, (int32_t)P.kind, (int32_t)P.lds, P.lay.L, P.lay.m, P.lay.h, P.seg_cc, P.seg_b,
                          P.seg_budget, P.seg_kp};
  mix(head, sizeof head);
  mix(P.colmap.data(), P.colmap.size() * sizeof(int));
  mix(P.cols.data(), P.cols.size() * sizeof(double));
  mix(P.x0.data(), P.x0.size() * sizeof(double));
  mix(&P.jit_key, sizeof P.jit_key);
  mix(P.jtab.data(), P.jtab.size() * sizeof(double));
  return h;
}

double pairwise_host(const std::vector<double>& v) {
  if (v.empty()) return 0.0;
  size_t p = 1;
  while (p < v.size()) p <<= 1;
  std::vector<double> a(p, 0.0);
  std::copy(v.begin(), v.end(), a.begin());
  while (p > 1) {
    p >>= 1;
    for (size_t i = 0; i < p; ++i) a[i] = a[2 * i] + a[2 * i + 1];
  }
  return a[0];
}

// -------------------------------------------------------- device contexts --
struct DeviceCtx {
  int dev = 0;   // logical id (the API's)
  int phys = 0;  // the HIP device it runs on (phys_device)
  int cus = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // deferred walk timing (set_defer_timing): event pairs recorded around walks
  // whose times are read later (kernel_time), and the pairs free for reuse
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending, ev_free;
  double deferred_ms = 0.0;
  uint64_t deferred_n = 0;
  double* d_cols = nullptr;
  size_t cols_cap = 0;
  double* d_jtab = nullptr;
  size_t jtab_cap = 0;
  double* d_start = nullptr;  // the segmented walk's start table (Plan::start_tab)
  size_t start_cap = 0;
  double* d_x0 = nullptr;
  int* d_nblk = nullptr;
  uint64_t* d_rowmask = nullptr;
  double* d_chunk = nullptr;
  size_t chunk_cap = 0;
  double* d_scratch = nullptr;
  size_t scratch_cap = 0;
  unsigned* d_visited = nullptr;
  double* d_wave = nullptr;   // exact path: per-wave residues
  size_t wave_cap = 0;
  double* d_x0dd = nullptr;   // double-double walk: start vector (hi, lo)
  size_t x0dd_cap = 0;
  size_t visited_cap = 0;
  // queue heads and the fused fold's visited accumulator: head 0 at [0], head 1
  // at [16] (own 64-byte lines), the accumulator (u64) at byte 128
  unsigned* d_counter = nullptr;
  bool head_zero[2] = {false, false};  // head known to be 0 (zeroed by the last run_range's reduction)
  int head = 0;                        // run_range's head for the next fused-fold walk
  unsigned* d_foldcnt = nullptr;       // the fused fold's arrival counters (zero between launches)
  size_t foldcnt_cap = 0;
  double* d_result = nullptr;
  double* h_result = nullptr;  // pinned host slot (mapped): the reduction writes the result here
  double* m_result = nullptr;  // its device address (nullptr: copy from d_result instead)
  unsigned* h_flag = nullptr;  // beside h_result: the sequence number of the last call whose result is there
  unsigned* m_flag = nullptr;
  unsigned flag_seq = 0;
  // leaf batches (run_range_batch): packed tables, descriptors, results
  double* d_batch = nullptr;
  size_t batch_cap = 0;
  LeafDesc* d_desc = nullptr;
  size_t desc_cap = 0;
  double* d_bres = nullptr;
  size_t bres_cap = 0;
  double* h_bres = nullptr;  // pinned, kMaxBatchLeaves doubles
  int occ_batch[2][SUP_MAX_N + 1] = {};
  uint64_t tables_uid = 0;  // Plan::uid whose cols / x0 / nblk / rowmask / jtab the device holds
  std::mutex mu;
  int occ[3][SUP_MAX_N + 1] = {};  // AOT kernels; segmented walk: jit_occupancy
};

static std::mutex g_ctx_mu;
static std::vector<std::unique_ptr<DeviceCtx>> g_ctx;  // [logical device * kCtxLanes + lane]

// Context lane of the calling thread (set_ctx_lane): host threads that run
// independent permanents at once on one device (the -o leaves, engine_leaf)
// each take their own lane — own stream, buffers and queue counter — so their
// launches, copies and syncs overlap instead of queueing on one context.
static thread_local int t_ctx_lane = 0;
void set_ctx_lane(int lane) { t_ctx_lane = std::max(0, std::min(kCtxLanes - 1, lane)); }
int ctx_lane() { return t_ctx_lane; }

// Deferred walk timing (sup_opts.timing = 0, sup_perman_shard): run_range
// records its walk's HIP events as usual but does not wait for the end event
// — the call returns once its result is there, while the kernel's last waves
// may still be exiting — and kernel_time reads the deferred pairs later.
static thread_local bool t_defer_timing = false;
void set_defer_timing(bool on) { t_defer_timing = on; }

// Logical devices.  Every device id of the API (sup_opts::device_id, the
// devices of a multi-device schedule) is a logical id; SUP_DEVICE_MAP (a
// comma list of physical ids, e.g. "0,0,0,0") puts several logical devices on
// one physical GPU, each with its own context (stream, buffers, queue), so the
// multi-device schedulers' per-device threads, combines and item queues run —
// concurrently — on a one-GPU machine.  Unset: logical = physical.  RCCL needs
// distinct physical devices (rccl_allreduce_slots refuses a duplicated map).
static std::vector<int> device_map() {
  std::vector<int> m;
  const char* e = std::getenv("SUP_DEVICE_MAP");
  if (!e || !*e) return m;
  for (const char* p = e; *p;) {
    char* end = nullptr;
    const long v = std::strtol(p, &end, 10);
    if (end == p || v < 0 || v > 1023) return {-1};  // malformed: device_count reports it
    m.push_back((int)v);
    p = *end == ',' ? end + 1 : end;
    if (*end && *end != ',') return {-1};
  }
  return m;
}

int phys_device(int dev) {
  const std::vector<int> m = device_map();
  return (m.empty() || dev < 0 || dev >= (int)m.size()) ? dev : m[dev];
}

static thread_local int t_logical = -1;  // the logical device this thread last selected

hipError_t select_device(int dev) {
  const hipError_t e = hipSetDevice(phys_device(dev));
  t_logical = e == hipSuccess ? dev : -1;
  return e;
}

static bool check_device_on() {
  static const bool on = [] {
    const char* e = std::getenv("SUP_CHECK_DEVICE");
    return e && std::atoi(e) != 0;
  }();
  return on;
}
static std::atomic<uint64_t> g_device_checks{0};

int check_device(int dev, const char* what) {
  if (!check_device_on()) return SUP_OK;
  int cur = -1;
  const int want = phys_device(dev);
  if (hipGetDevice(&cur) != hipSuccess || cur != want || t_logical != dev) {
    set_error(std::string("SUP_CHECK_DEVICE: ") + what + " for logical device " + std::to_string(dev) +
              " (physical " + std::to_string(want) + ") on a thread whose HIP device is " + std::to_string(cur) +
              " and whose last selected logical device is " + std::to_string(t_logical));
    return SUP_EHIP;
  }
  g_device_checks.fetch_add(1, std::memory_order_relaxed);
  return SUP_OK;
}

uint64_t device_checks_passed() { return g_device_checks.load(); }

int device_count(int* n) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    set_error(std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    return SUP_ENODEV;
  }
  const std::vector<int> m = device_map();
  if (!m.empty() && c > 0) {
    for (int p : m)
      if (p < 0 || p >= c) {
        *n = 0;
        set_error("SUP_DEVICE_MAP must be a comma list of existing physical device ids (" + std::to_string(c) +
                  " visible)");
        return SUP_ENODEV;
      }
    c = (int)m.size();
  }
  *n = c;
  return SUP_OK;
}

static int get_ctx(int dev, DeviceCtx** out) {
  int cnt = 0;
  int rc = device_count(&cnt);
  if (rc) return rc;
  if (cnt == 0) {
    set_error("no HIP device available (the engine has no CPU fallback for GPU algorithms)");
    return SUP_ENODEV;
  }
  if (dev < 0 || dev >= cnt) {
    set_error("device id " + std::to_string(dev) + " out of range (" + std::to_string(cnt) + " devices)");
    return SUP_ENODEV;
  }
  const int pd = phys_device(dev);
  const size_t slot = (size_t)dev * kCtxLanes + (size_t)t_ctx_lane;
  std::lock_guard<std::mutex> g(g_ctx_mu);
  if (g_ctx.size() < (size_t)cnt * kCtxLanes) g_ctx.resize((size_t)cnt * kCtxLanes);
  if (g_ctx[slot] && g_ctx[slot]->phys != pd) {
    set_error("logical device " + std::to_string(dev) + " moved to another physical device (SUP_DEVICE_MAP "
              "changed after first use)");
    return SUP_EINVAL;
  }
  if (!g_ctx[slot]) {
    auto c = std::make_unique<DeviceCtx>();
    c->dev = dev;
    c->phys = pd;
    SUP_HIP(select_device(dev));
    SUP_ON_DEVICE(dev, "context allocations");
    hipDeviceProp_t prop;
    SUP_HIP(hipGetDeviceProperties(&prop, pd));
    c->cus = prop.multiProcessorCount;
    SUP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    SUP_HIP(hipEventCreate(&c->ev0));
    SUP_HIP(hipEventCreate(&c->ev1));
    SUP_HIP(hipMalloc(&c->d_x0, SUP_MAX_N * sizeof(double)));
    SUP_HIP(hipMalloc(&c->d_nblk, SUP_MAX_N * sizeof(int)));
    SUP_HIP(hipMalloc(&c->d_rowmask, SUP_MAX_N * sizeof(uint64_t)));
    SUP_HIP(hipMalloc(&c->d_counter, 256));
    // zeroed on the context's own stream: a null-stream hipMemset is not ordered
    // with this non-blocking stream and could land after the first walk began
    SUP_HIP(hipMemsetAsync(c->d_counter, 0, 256, c->stream));
    SUP_HIP(hipStreamSynchronize(c->stream));
    SUP_HIP(hipMalloc(&c->d_result, 64));
    // the result slot is host memory the device writes directly (mapped,
    // coherent): the reduction's last pass stores the partial there, so no
    // D2H copy is queued per call; d_result stays for the -R slot copy
    SUP_HIP(hipHostMalloc(&c->h_result, 64, hipHostMallocMapped | hipHostMallocCoherent));
    if (hipHostGetDevicePointer((void**)&c->m_result, c->h_result, 0) != hipSuccess) c->m_result = nullptr;
    c->h_flag = reinterpret_cast<unsigned*>(c->h_result + 1);
    *c->h_flag = 0u;
    c->m_flag = c->m_result ? reinterpret_cast<unsigned*>(c->m_result + 1) : nullptr;
    g_ctx[slot] = std::move(c);
  }
  *out = g_ctx[slot].get();
  return SUP_OK;
}

// Device warm-up (sup_device_warmup): the HIP runtime's initialisation,
// each device's context (stream, events, buffers) and the ahead-of-time walk
// code objects of order n, so a caller can overlap them with its host-side
// planning instead of paying them after it.
int warm_devices(int first, int count, int n) {
  for (int d = first; d < first + count; ++d) {
    DeviceCtx* c = nullptr;
    if (int rc = get_ctx(d, &c)) return rc;
    std::lock_guard<std::mutex> g(c->mu);
    SUP_HIP(select_device(c->dev));
    if (n >= 1 && n <= SUP_MAX_N)
      for (WalkKind k : {kWalkDense, kWalkSparse}) {
        int b = 0;
        SUP_HIP(walk_occupancy(k, n, &b));
      }
  }
  return SUP_OK;
}

// The deferred walk times of the calling thread's context on logical device
// `dev` since the last read: waits for their end events, returns their sum
// and count, and starts a new tally.
int kernel_time(int dev, double* total_ms, uint64_t* launches) {
  DeviceCtx* c = nullptr;
  if (int rc = get_ctx(dev, &c)) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  SUP_HIP(select_device(c->dev));
  for (auto& ev : c->ev_pending) {
    SUP_HIP(hipEventSynchronize(ev.second));
    float m = 0.f;
    SUP_HIP(hipEventElapsedTime(&m, ev.first, ev.second));
    c->deferred_ms += m;
    ++c->deferred_n;
    c->ev_free.push_back(ev);
  }
  c->ev_pending.clear();
  if (total_ms) *total_ms = c->deferred_ms;
  if (launches) *launches = c->deferred_n;
  c->deferred_ms = 0.0;
  c->deferred_n = 0;
  return SUP_OK;
}

// Per-call completion (round 4, tools/probe_launch.hip, profiles/r4/probe_launch_b.log):
// around a 500 us kernel, marker events + one more launch + hipStreamSynchronize
// cost 18.9 us beyond the kernel; waiting instead for a sequence number the
// last kernel stores in mapped host memory, 11.9 us.  (Events carried by the
// launch itself, hipExtModuleLaunchKernel, measured worse: 23.7 / 15.5 us.)
// So a call whose result lands in mapped host memory waits for the sequence
// number the reduction's last pass stores after it; SUP_FLAG_WAIT=0 restores
// the stream sync (A/B).
static bool result_flag_wait() {
  static const bool on = [] {
    const char* e = std::getenv("SUP_FLAG_WAIT");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}
// The fused fold (run_range; walk_common.hpp chunk_store) is the default;
// SUP_FOLD=0 restores the reduction launches after the walk (A/B: the same
// tree, the same bits).
static bool fold_fused() {
  static const bool on = [] {
    const char* e = std::getenv("SUP_FOLD");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}
// Spin on the flag for up to 2 ms (a short walk's wait); false: not seen yet
// (a long walk, or a fault that stopped the stream) — the caller then blocks
// in hipStreamSynchronize, which also reports the stream's error.
static constexpr double kFlagSpinMs = 2.0;
// The fused fold's result slot before a walk whose final fold publishes the
// result itself (WalkParams::fold_sys): a signalling-NaN pattern no fold
// produces in practice (a result that equals it only costs the spin window).
static constexpr uint64_t kResultSentinel = 0x7ff4dead5eedbeefull;
static bool result_sys() {
  static const bool on = [] {
    const char* e = std::getenv("SUP_RESULT_SYS");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}
static bool wait_result(const double* slot) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t* w = reinterpret_cast<const uint64_t*>(slot);
  for (unsigned i = 1;; ++i) {
    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) != kResultSentinel) return true;
    __builtin_ia32_pause();
    if ((i & 255u) == 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::microseconds((long)(kFlagSpinMs * 1000.0)))
      return false;
  }
}
static bool wait_flag(const unsigned* flag, unsigned seq) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 1;; ++i) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return true;
    __builtin_ia32_pause();
    if ((i & 255u) == 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::microseconds((long)(kFlagSpinMs * 1000.0)))
      return false;
  }
}

template <class T>
static int ensure(T*& p, size_t& cap, size_t need) {
  if (need <= cap) return SUP_OK;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  hipError_t e = hipMalloc(&p, need * sizeof(T));
  if (e != hipSuccess) {
    set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return SUP_ENOMEM;
  }
  cap = need;
  return SUP_OK;
}

int run_range(int dev, const Plan& P, uint64_t c0, uint64_t c1, bool want_visited, RangeResult& r, double* slot) {
  r = RangeResult();
  if (c1 <= c0) return SUP_OK;  // empty range: partial 0
  if (c1 > P.lay.chunks()) {
    set_error("wave-chunk range exceeds the plan");
    return SUP_EINVAL;
  }
  DeviceCtx* c = nullptr;
  int rc = get_ctx(dev, &c);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  SUP_HIP(select_device(c->dev));
  SUP_ON_DEVICE(c->dev, "device buffers");
  const uint64_t count = c1 - c0;
  const double* cols_before = c->d_cols;
  const double* jtab_before = c->d_jtab;
  if ((rc = ensure(c->d_cols, c->cols_cap, P.cols.size()))) return rc;
  if ((rc = ensure(c->d_chunk, c->chunk_cap, (size_t)count))) return rc;
  if ((rc = ensure(c->d_scratch, c->scratch_cap, (size_t)pairwise_scratch_size(count)))) return rc;
  // walked states per chunk: SkipPer's jumps, the segmented walk's chunk skip
  // (only where the walk leaves rows untouched)
  const bool visited = want_visited && (P.kind == kWalkSkip || (P.kind == kWalkSeg && P.outer_tree.tail_hi >
                                                                                           P.outer_tree.tail_lo));
  if (visited && (rc = ensure(c->d_visited, c->visited_cap, (size_t)count))) return rc;

  const bool seg = P.kind == kWalkSeg;
  if (seg && (rc = ensure(c->d_jtab, c->jtab_cap, P.jtab.size()))) return rc;
  const bool stab = seg && !P.start_tab.empty();
  const double* start_before = c->d_start;
  if (stab && (rc = ensure(c->d_start, c->start_cap, P.start_tab.size()))) return rc;

  hipStream_t s = c->stream;
  // the plan's tables: uploaded unless this device already holds them (same
  // cached plan, buffers not reallocated) — repeated calls on one matrix
  // (bench steps, -p6 items, reduction leaves) skip five H2D copies
  if (P.uid == 0 || P.uid != c->tables_uid || c->d_cols != cols_before || c->d_jtab != jtab_before ||
      c->d_start != start_before) {
    if (seg)
      SUP_HIP(hipMemcpyAsync(c->d_jtab, P.jtab.data(), P.jtab.size() * sizeof(double), hipMemcpyHostToDevice, s));
    if (stab)
      SUP_HIP(hipMemcpyAsync(c->d_start, P.start_tab.data(), P.start_tab.size() * sizeof(double),
                             hipMemcpyHostToDevice, s));
    SUP_HIP(hipMemcpyAsync(c->d_cols, P.cols.data(), P.cols.size() * sizeof(double), hipMemcpyHostToDevice, s));
    SUP_HIP(hipMemcpyAsync(c->d_x0, P.x0.data(), P.x0.size() * sizeof(double), hipMemcpyHostToDevice, s));
    SUP_HIP(hipMemcpyAsync(c->d_nblk, P.nblk.data(), P.nblk.size() * sizeof(int), hipMemcpyHostToDevice, s));
    SUP_HIP(hipMemcpyAsync(c->d_rowmask, P.rowmask.data(), P.rowmask.size() * sizeof(uint64_t),
                           hipMemcpyHostToDevice, s));
    c->tables_uid = P.uid;
  }
  // The fused fold (walk_common.hpp chunk_store): the walk folds its own
  // partials, so no reduction launch follows it; its final fold zeroes the
  // other queue head, which the next such walk takes (the heads alternate: a
  // wave may still take its last, empty ticket after the fold completes).
  const bool fused = fold_fused() && !P.lds &&
                     (P.kind == kWalkSeg || P.kind == kWalkDense || P.kind == kWalkSparse || P.kind == kWalkSkip);
  if (fused) {
    // a grown buffer starts at zero (compare capacities: a reallocation may
    // return the same address, with stale contents)
    const size_t cap_before = c->foldcnt_cap;
    if ((rc = ensure(c->d_foldcnt, c->foldcnt_cap, (size_t)pairwise_scratch_size(count)))) return rc;
    if (c->foldcnt_cap != cap_before) SUP_HIP(hipMemsetAsync(c->d_foldcnt, 0, c->foldcnt_cap * sizeof(unsigned), s));
  }
  const int qh = fused ? c->head : 0;
  unsigned* head = c->d_counter + 16 * qh;
  // the queue head: zeroed by the previous run_range's reduction, else here
  if (!c->head_zero[qh]) SUP_HIP(hipMemsetAsync(head, 0, sizeof(unsigned), s));
  c->head_zero[qh] = false;

  int occ_seg = 0, occ_lds = 0;
  if (seg) SUP_ON_DEVICE(c->dev, "segmented-walk module load");
  if (seg && (rc = jit_occupancy(c->phys, P, &occ_seg, &r.compile_ms))) return rc;
  if (P.lds) {  // LDS-staged dense walk: one wave per block, LDS-limited residency
    SUP_HIP(lds_occupancy(P.n, P.lay.m, &occ_lds));
    if (occ_lds < 1) occ_lds = 1;
  }
  int& occ = seg ? occ_seg : (P.lds ? occ_lds : c->occ[P.kind][P.n]);
  if (occ == 0) {
    int b = 0;
    SUP_HIP(walk_occupancy(P.kind, P.n, &b));
    occ = b > 0 ? b : 1;
  }
  const uint64_t wpb = P.lds ? 1 : kWavesPerBlock;  // waves per block
  const uint64_t resident = (uint64_t)c->cus * (uint64_t)occ;  // resident blocks
  const uint64_t res_waves = resident * wpb;
  // chunk groups of up to 64 (one lane per partial: a 512-byte store); the
  // largest that leaves >= 32 groups per resident wave (tail balance).  n = 40
  // on one MI355X: 16 chunks, 128-byte stores (8 chunks: 64-byte partial-line
  // stores, 2.5x the partials' bytes in WRITE_SIZE)
  unsigned group = 64;
  while (group > 1 && count / ((uint64_t)group * res_waves) < 32) group >>= 1;
  if (const char* e = std::getenv("SUP_WALK_GROUP"))  // experiments: force the chunk group (power of two <= 64)
    group = std::max(1u, std::min(64u, 1u << (31 - __builtin_clz((unsigned)std::max(1, std::atoi(e))))));
  // Segmented walk: the last chunks go out in quarter groups, so the waves
  // finish within a quarter group of each other (a group of 16 n = 40 chunks
  // is ~5 ms of one wave's time).  Smaller tail groups measured 0.25 % faster
  // on the headline (tail groups of 4 174.7-174.9 ms, of 2 174.4-174.5, of 1
  // 174.3-174.5, profiles/r6/probe_tail_group.log) but each tail chunk then
  // costs its own ticket, publish and fold reads: 11.7 -> 16.8 MB of HBM
  // traffic per launch (profiles/r6/tail1_hbm_d050.json), so quarter groups stay.
  // The tail phase holds ~2 groups per resident wave, rounded to whole groups.
  unsigned tail_group = 0;
  uint64_t tail_begin = count;
  if (seg && group >= 2) {
    tail_group = std::max(1u, group / 4);
    if (const char* e = std::getenv("SUP_WALK_TAIL"))  // experiments: tail group (0 = no tail phase)
      tail_group = std::min(group, (unsigned)std::max(0, std::atoi(e)));
    if (tail_group) {
      tail_group = 1u << (31 - __builtin_clz(tail_group));  // a power of two
      const uint64_t tail = 2 * res_waves * group;
      // on a multiple of 64 (so of the group): no 64-group of the fused fold
      // mixes group sizes (walk_common.hpp chunk_store)
      tail_begin = count > tail ? (count - tail) / 64 * 64 : 0;
    }
  }
  const uint64_t waves_needed = (count + group - 1) / group;  // one chunk group per wave at a time
  uint64_t grid = (waves_needed + wpb - 1) / wpb;
  if (grid > resident) grid = resident;
  if (grid < 1) grid = 1;

  WalkParams p{};
  p.cols = c->d_cols;
  p.x0 = c->d_x0;
  p.nblk = c->d_nblk;
  p.rowmask = c->d_rowmask;
  p.chunk_begin = c0;
  p.chunk_count = count;
  p.L = P.lay.L;
  p.m = P.lay.m;
  p.n = P.n;
  p.umask = P.kind == kWalkSparse ? P.chunk_ends : P.umask;  // walk_sparse: its chunk-end rows
  p.chunk_out = c->d_chunk;
  p.counter = head;
  p.visited = visited && !fused ? c->d_visited : nullptr;
  p.group = group;
  p.tail_group = tail_group;
  p.tail_begin = tail_begin;
  p.tail_ticket = tail_group ? (unsigned)(tail_begin / group) : 0xffffffffu;
  p.jtab = seg ? c->d_jtab : nullptr;
  p.start_tab = stab ? c->d_start : nullptr;
  p.nb_lo = p.nb_hi = 0;
  for (int k = 0; k < P.lay.m && k < 32; ++k) {
    const uint64_t v = (uint64_t)(P.nblk[P.lay.L + k] & 15);
    if (k < 16) p.nb_lo |= v << (4 * k);
    else p.nb_hi |= v << (4 * (k - 16));
  }

  // SUP_JIT_TRACE=<file>: the segmented walk's per-wave stamps (diagnostics)
  const char* trace_path = seg ? std::getenv("SUP_JIT_TRACE") : nullptr;
  unsigned long long* d_trace = nullptr;
  if (trace_path && *trace_path) {
    SUP_HIP(hipMalloc(&d_trace, grid * kWavesPerBlock * 8 * sizeof(unsigned long long)));
    SUP_HIP(hipMemsetAsync(d_trace, 0, grid * kWavesPerBlock * 8 * sizeof(unsigned long long), s));
    p.trace = d_trace;
  }

  // where the result goes: mapped host memory (no D2H copy; with a sequence
  // number the host can wait on) unless an -R slot copy takes it from d_result
  const bool to_host = c->m_result && !slot;
  const bool direct = to_host && (fused || count > 1);  // (old path: one chunk is a copy, not a pass)
  const bool flagged = direct && (fused || !visited) && result_flag_wait();
  const unsigned seq = ++c->flag_seq;
  if (fused) {
    p.fold_cnt = c->d_foldcnt;
    p.fold_lv = c->d_scratch;
    p.fold_out = to_host ? c->m_result : c->d_result;
    p.fold_vis = visited ? reinterpret_cast<unsigned long long*>(c->d_counter + 32) : nullptr;
    p.fold_reset = c->d_counter + 16 * (qh ^ 1);
    p.fold_flag = flagged ? c->m_flag : nullptr;
    p.fold_seq = seq;
    if (flagged && result_sys()) {  // the result slot itself is the signal
      p.fold_flag = nullptr;
      p.fold_sys = 1;
      __atomic_store_n(reinterpret_cast<uint64_t*>(c->h_result), kResultSentinel, __ATOMIC_RELEASE);
    }
  }

  hipEvent_t e0 = c->ev0, e1 = c->ev1;
  const bool defer = t_defer_timing;
  if (defer) {
    if (c->ev_free.empty()) {
      std::pair<hipEvent_t, hipEvent_t> ev;
      SUP_HIP(hipEventCreate(&ev.first));
      SUP_HIP(hipEventCreate(&ev.second));
      c->ev_free.push_back(ev);
    }
    std::tie(e0, e1) = c->ev_free.back();
    c->ev_free.pop_back();
    c->ev_pending.emplace_back(e0, e1);
  }
  SUP_ON_DEVICE(c->dev, "walk launch");
  SUP_HIP(hipEventRecord(e0, s));
  if (seg) {
    if ((rc = jit_launch(c->phys, P, p, (int)grid, s))) return rc;
  } else if (P.lds) {
    SUP_HIP(launch_lds(P.n, p, (int)grid, s));
  } else {
    SUP_HIP(launch_walk(P.kind, P.n, p, (int)grid, s));
  }
  SUP_HIP(hipEventRecord(e1, s));
  unsigned long long* vsum = reinterpret_cast<unsigned long long*>(c->h_result + 2);
  if (fused) {
    if (!to_host) {
      SUP_HIP(hipMemcpyAsync(c->h_result, c->d_result, sizeof(double), hipMemcpyDeviceToHost, s));
      if (visited) SUP_HIP(hipMemcpyAsync(vsum, c->d_result + 2, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    }
  } else {
    // (the -R combine copies d_result into its slot on the device; one chunk is a copy, not a pass)
    SUP_ON_DEVICE(c->dev, "reduction launch");
    SUP_HIP(launch_pairwise_reduce(c->d_chunk, count, c->d_scratch, direct ? c->m_result : c->d_result, s, head,
                                   flagged ? c->m_flag : nullptr, seq));
    if (!direct) SUP_HIP(hipMemcpyAsync(c->h_result, c->d_result, sizeof(double), hipMemcpyDeviceToHost, s));
    // visited states: summed on the device, 8 bytes back (beside the result in
    // the mapped slot: h_result[2])
    if (visited) {
      SUP_HIP(launch_sum_visited(c->d_visited, count, reinterpret_cast<unsigned long long*>(c->d_result + 2), s));
      SUP_HIP(hipMemcpyAsync(vsum, c->d_result + 2, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    }
  }
  if (slot) SUP_HIP(hipMemcpyAsync(slot, c->d_result, sizeof(double), hipMemcpyDeviceToDevice, s));
  // spin on the flag only where the walk is predicted to end within the spin
  // window (cost model on this device's CUs; a longer walk blocks in the
  // stream sync at once instead of holding a host core for 2 ms)
  const double predicted_ms = std::ldexp((double)count, P.lay.L + P.lay.m) * walk_cost_eff(P) / kLaneOpsPerSec *
                              1e3 * (256.0 / std::max(1, c->cus));
  const bool seen = flagged && predicted_ms <= kFlagSpinMs &&
                    (p.fold_sys ? wait_result(c->h_result) : wait_flag(c->h_flag, seq));
  if (!seen) SUP_HIP(hipStreamSynchronize(s));
  if (fused) {  // the final fold zeroed the other head
    c->head_zero[qh ^ 1] = true;
    c->head = qh ^ 1;
    if (std::getenv("SUP_FOLD_CHECK")) {  // debugging: every arrival counter back at zero
      SUP_HIP(hipStreamSynchronize(s));
      std::vector<unsigned> cc(c->foldcnt_cap);
      SUP_HIP(hipMemcpy(cc.data(), c->d_foldcnt, cc.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
      unsigned hd[64];
      SUP_HIP(hipMemcpy(hd, c->d_counter, 256, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < cc.size(); ++i)
        if (cc[i]) {
          std::fprintf(stderr, "SUP_FOLD_CHECK: counter %zu = %u after a fused walk (kind %d n %d count %llu group %u tail %u/%llu)\n",
                       i, cc[i], (int)P.kind, P.n, (unsigned long long)count, group, tail_group, (unsigned long long)tail_begin);
          break;
        }
      std::fprintf(stderr, "SUP_FOLD_CHECK: kind %d n %d count %llu grid %llu heads %u %u vis %llu result %.17g\n", (int)P.kind,
                   P.n, (unsigned long long)count, (unsigned long long)grid, hd[0], hd[16],
                   *reinterpret_cast<unsigned long long*>(hd + 32), *c->h_result);
    }
  } else {
    c->head_zero[0] = count > 1;  // the reduction's first pass zeroed it (one chunk: a copy, no pass)
  }

  float ms = 0.f;
  // (after a flag wait the walk's result is there, but its end event may not
  // be: waiting for it costs ~8 us per call on config 2 — deferred timing
  // leaves it for kernel_time)
  hipError_t ee = defer ? hipSuccess : hipEventElapsedTime(&ms, e0, e1);
  if (ee == hipErrorNotReady) {
    SUP_HIP(hipEventSynchronize(e1));
    ee = hipEventElapsedTime(&ms, e0, e1);
  }
  if (defer && c->ev_pending.size() >= 256) {  // bound the pending pairs: read the finished ones
    size_t k = 0;
    for (; k < c->ev_pending.size() && hipEventQuery(c->ev_pending[k].second) == hipSuccess; ++k) {
      float m = 0.f;
      SUP_HIP(hipEventElapsedTime(&m, c->ev_pending[k].first, c->ev_pending[k].second));
      c->deferred_ms += m;
      ++c->deferred_n;
      c->ev_free.push_back(c->ev_pending[k]);
    }
    c->ev_pending.erase(c->ev_pending.begin(), c->ev_pending.begin() + (long)k);
  }
  if (ee != hipSuccess) {
    set_error(std::string("hipEventElapsedTime: ") + hipGetErrorString(ee));
    return SUP_EHIP;
  }
  r.partial = *c->h_result;
  r.kernel_ms = ms;
  r.grid = (int)grid;
  if (d_trace) {
    std::vector<unsigned long long> tr(grid * kWavesPerBlock * 8);
    SUP_HIP(hipMemcpy(tr.data(), d_trace, tr.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    SUP_HIP(hipFree(d_trace));
    if (FILE* f = std::fopen(trace_path, "a")) {
      std::fprintf(f, "# launch chunks %llu grid %llu waves_resident %llu group %u tail_group %u kernel_ms %.4f\n",
                   (unsigned long long)count, (unsigned long long)grid, (unsigned long long)res_waves, group,
                   tail_group, ms);
      for (size_t w = 0; w < tr.size() / 8; ++w)
        std::fprintf(f, "%zu %llu %llu %llu %llu %llu %llu\n", w, tr[8 * w], tr[8 * w + 1], tr[8 * w + 2],
                     tr[8 * w + 3], tr[8 * w + 4], tr[8 * w + 5]);
      std::fclose(f);
    }
  }
  if (visited) {
    r.visited = (uint64_t)*vsum * (uint64_t)(1ull << P.lay.L);
  } else {
    r.visited = count << (P.lay.L + P.lay.m);
  }
  return SUP_OK;
}

// Several leaves (the -o / -u reduction's permanents) in one launch: plans of
// one order, walk kind (plain or prefix-blocked) and layout.  Their tables are
// packed into one device buffer, the batch kernel walks the K 2^h wave-chunks
// as one queue (walk_batch.hpp), and each leaf's partials are folded by the
// one-leaf pairwise tree: partial[i] is bit-identical to run_range over plan
// i's whole range (tests/test_gpu_reduce_workers.py).  One launch instead of
// K removes K - 1 launch tails, syncs and result copies.
bool batchable(const Plan& a, const Plan& b) {
  return (a.kind == kWalkDense || a.kind == kWalkSparse) && a.kind == b.kind && !a.lds && !b.lds && a.n == b.n &&
         a.lay.L == b.lay.L && a.lay.m == b.lay.m && a.lay.h == b.lay.h && a.cols.size() == b.cols.size() &&
         a.x0.size() == b.x0.size() && a.lay.chunks() >= 1 &&
         a.lay.chunks() <= (1ull << kMaxBatchLeafChunkBits);  // 32-bit chunk ids (engine.hpp)
}

int run_range_batch(int dev, const std::vector<const Plan*>& plans, std::vector<double>& partial, double* kernel_ms) {
  const size_t K = plans.size();
  partial.assign(K, 0.0);
  if (kernel_ms) *kernel_ms = 0.0;
  if (K == 0) return SUP_OK;
  if (K > (size_t)kMaxBatchLeaves) {
    set_error("leaf batch larger than kMaxBatchLeaves");
    return SUP_EINVAL;
  }
  const Plan& P0 = *plans[0];
  for (const Plan* q : plans)
    if (!batchable(P0, *q)) {
      set_error("leaf batch: plans of different order, walk or layout");
      return SUP_EINVAL;
    }
  DeviceCtx* c = nullptr;
  int rc = get_ctx(dev, &c);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  SUP_HIP(select_device(c->dev));
  SUP_ON_DEVICE(c->dev, "device buffers");
  const uint64_t C = P0.lay.chunks(), count = C * K;
  const size_t colsz = P0.cols.size(), stride = colsz + P0.x0.size();
  if ((rc = ensure(c->d_batch, c->batch_cap, K * stride))) return rc;
  if ((rc = ensure(c->d_desc, c->desc_cap, K))) return rc;
  if ((rc = ensure(c->d_chunk, c->chunk_cap, (size_t)count))) return rc;
  if ((rc = ensure(c->d_scratch, c->scratch_cap, (size_t)(K * pairwise_scratch_size(C))))) return rc;
  if ((rc = ensure(c->d_bres, c->bres_cap, K))) return rc;
  if (!c->h_bres) SUP_HIP(hipHostMalloc(&c->h_bres, kMaxBatchLeaves * sizeof(double), hipHostMallocDefault));
  std::vector<double> tab(K * stride);
  std::vector<LeafDesc> desc(K);
  for (size_t i = 0; i < K; ++i) {
    const Plan& P = *plans[i];
    std::copy(P.cols.begin(), P.cols.end(), tab.begin() + i * stride);
    std::copy(P.x0.begin(), P.x0.end(), tab.begin() + i * stride + colsz);
    desc[i].cols = c->d_batch + i * stride;
    desc[i].x0 = c->d_batch + i * stride + colsz;
    desc[i].nb_lo = desc[i].nb_hi = 0;
    desc[i].ends = P.kind == kWalkSparse ? P.chunk_ends : 0;
    for (int k = 0; k < P.lay.m && k < 32 && P.kind == kWalkSparse; ++k) {
      const uint64_t v = (uint64_t)(P.nblk[P.lay.L + k] & 15);
      if (k < 16) desc[i].nb_lo |= v << (4 * k);
      else desc[i].nb_hi |= v << (4 * (k - 16));
    }
  }
  hipStream_t s = c->stream;
  SUP_HIP(hipMemcpyAsync(c->d_batch, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice, s));
  SUP_HIP(hipMemcpyAsync(c->d_desc, desc.data(), K * sizeof(LeafDesc), hipMemcpyHostToDevice, s));
  SUP_HIP(hipMemsetAsync(c->d_counter, 0, sizeof(unsigned), s));
  c->head_zero[0] = false;  // this walk leaves queue head 0 nonzero
  int& occ = c->occ_batch[P0.kind == kWalkSparse][P0.n];
  if (occ == 0) {
    int b = 0;
    SUP_HIP(walk_batch_occupancy(P0.kind, P0.n, &b));
    occ = b > 0 ? b : 1;
  }
  const uint64_t res_waves = (uint64_t)c->cus * (uint64_t)occ * kWavesPerBlock;
  // groups as run_range picks them, and never larger than one leaf's chunks
  unsigned group = 64;
  while (group > 1 && (count / ((uint64_t)group * res_waves) < 32 || group > C)) group >>= 1;
  const uint64_t waves_needed = (count + group - 1) / group;
  uint64_t grid = (waves_needed + kWavesPerBlock - 1) / kWavesPerBlock;
  grid = std::max<uint64_t>(1, std::min<uint64_t>(grid, (uint64_t)c->cus * (uint64_t)occ));
  WalkParams p{};
  p.cols = desc[0].cols;
  p.x0 = desc[0].x0;
  p.chunk_begin = 0;
  p.chunk_count = count;
  p.L = P0.lay.L;
  p.m = P0.lay.m;
  p.n = P0.n;
  p.chunk_out = c->d_chunk;
  p.counter = c->d_counter;
  p.group = group;
  p.tail_ticket = 0xffffffffu;
  LeafBatch lb{c->d_desc, (unsigned)P0.lay.h, 0};
  SUP_HIP(hipEventRecord(c->ev0, s));
  SUP_ON_DEVICE(c->dev, "batch walk launch");
  SUP_HIP(launch_walk_batch(P0.kind, P0.n, p, lb, (int)grid, s));
  SUP_HIP(hipEventRecord(c->ev1, s));
  SUP_HIP(launch_pairwise_reduce_seg(c->d_chunk, C, K, c->d_scratch, c->d_bres, s));
  SUP_HIP(hipMemcpyAsync(c->h_bres, c->d_bres, K * sizeof(double), hipMemcpyDeviceToHost, s));
  SUP_HIP(hipStreamSynchronize(s));
  float ms = 0.f;
  SUP_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  for (size_t i = 0; i < K; ++i) partial[i] = c->h_bres[i];
  if (kernel_ms) *kernel_ms = ms;
  return SUP_OK;
}

// Exact residue walk (walk_exact.hip) over wave-chunks [c0, c1) of a dense
// identity-map plan of 2A: per prime, the sum of the terms mod p (in [0, p)).
// Residue sums are exact, so neither the wave a chunk lands on nor the order
// of the per-wave sums changes the result.
int run_range_exact(int dev, const Plan& P, int group, uint64_t c0, uint64_t c1, const std::vector<double>& primes,
                    std::vector<uint64_t>& res, double* kernel_ms) {
  const int np = (int)primes.size();
  res.assign(np, 0);
  if (kernel_ms) *kernel_ms = 0.0;
  if (c1 <= c0) return SUP_OK;
  // group 1, 2, 4: the dense kernel on a dense plan; 8 + g: the prefix-blocked
  // kernel on a prefix-blocked plan (walk_exact.hip)
  const bool blocked = (group & 8) != 0;
  if (np < 1 || np > kMaxPrimes || P.kind != (blocked ? kWalkSparse : kWalkDense) || c1 > P.lay.chunks()) {
    set_error("run_range_exact: bad request");
    return SUP_EINVAL;
  }
  DeviceCtx* c = nullptr;
  int rc = get_ctx(dev, &c);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  SUP_HIP(select_device(c->dev));
  SUP_ON_DEVICE(c->dev, "device buffers");
  int occ = 0;
  SUP_HIP(exact_occupancy(P.n, group, &occ));
  if (occ < 1) occ = 1;
  const uint64_t count = c1 - c0;
  uint64_t grid = (uint64_t)c->cus * (uint64_t)occ;
  const uint64_t need_blocks = (count + kWavesPerBlock - 1) / kWavesPerBlock;
  if (grid > need_blocks) grid = need_blocks;
  if (grid < 1) grid = 1;
  const size_t waves = (size_t)grid * kWavesPerBlock;
  if ((rc = ensure(c->d_cols, c->cols_cap, P.cols.size()))) return rc;
  if ((rc = ensure(c->d_wave, c->wave_cap, waves * kMaxPrimes))) return rc;
  hipStream_t s = c->stream;
  c->tables_uid = 0;  // the exact walk's own tables replace the cached plan's
  SUP_HIP(hipMemcpyAsync(c->d_cols, P.cols.data(), P.cols.size() * sizeof(double), hipMemcpyHostToDevice, s));
  SUP_HIP(hipMemcpyAsync(c->d_x0, P.x0.data(), P.x0.size() * sizeof(double), hipMemcpyHostToDevice, s));
  SUP_HIP(hipMemsetAsync(c->d_counter, 0, sizeof(unsigned), s));
  c->head_zero[0] = false;  // this walk leaves queue head 0 nonzero
  WalkParams p{};
  p.cols = c->d_cols;
  p.x0 = c->d_x0;
  p.chunk_begin = c0;
  p.chunk_count = count;
  p.L = P.lay.L;
  p.m = P.lay.m;
  p.n = P.n;
  p.counter = c->d_counter;
  p.group = 1;
  p.umask = P.chunk_ends;  // walk_exact: its chunk-end rows (walk_sparse.hip's check)
  p.nb_lo = p.nb_hi = 0;
  for (int k = 0; blocked && k < P.lay.m && k < 32; ++k) {  // walk_exact_blocked: nblk of walk bit k
    const uint64_t v = (uint64_t)(P.nblk[P.lay.L + k] & 15);
    if (k < 16) p.nb_lo |= v << (4 * k);
    else p.nb_hi |= v << (4 * (k - 16));
  }
  ExactParams e{};
  for (int q = 0; q < np; ++q) e.prime[q] = primes[q], e.pinv[q] = 1.0 / primes[q];
  e.nprimes = np;
  e.wave_out = c->d_wave;
  SUP_HIP(hipEventRecord(c->ev0, s));
  SUP_ON_DEVICE(c->dev, "exact walk launch");
  SUP_HIP(launch_exact(P.n, group, p, e, (int)grid, s));
  SUP_HIP(hipEventRecord(c->ev1, s));
  std::vector<double> w(waves * kMaxPrimes);
  SUP_HIP(hipMemcpyAsync(w.data(), c->d_wave, w.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  SUP_HIP(hipStreamSynchronize(s));
  float ms = 0.f;
  SUP_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  if (kernel_ms) *kernel_ms = ms;
  for (int q = 0; q < np; ++q) {
    const uint64_t pq = (uint64_t)primes[q];
    uint64_t acc = 0;  // waves x p < 2^64
    for (size_t i = 0; i < waves; ++i) acc = (acc + (uint64_t)w[i * kMaxPrimes + q]) % pq;
    res[q] = acc;
  }
  return SUP_OK;
}

int run_range_dd(int dev, const Plan& P, const std::vector<double>& x0dd, uint64_t c0, uint64_t c1,
                 double* parts, double* kernel_ms) {
  if (kernel_ms) *kernel_ms = 0.0;
  if (c1 <= c0) return SUP_OK;
  const bool blocked = P.kind == kWalkSparse;  // walk_dd_blocked; else the dense walk_dd
  if ((P.kind != kWalkDense && !blocked) || c1 > P.lay.chunks() || x0dd.size() != 2 * (size_t)P.NP) {
    set_error("run_range_dd: bad request");
    return SUP_EINVAL;
  }
  DeviceCtx* c = nullptr;
  int rc = get_ctx(dev, &c);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  SUP_HIP(select_device(c->dev));
  SUP_ON_DEVICE(c->dev, "device buffers");
  int occ = 0;
  SUP_HIP(blocked ? dd_blocked_occupancy(P.n, &occ) : dd_occupancy(P.n, &occ));
  if (occ < 1) occ = 1;
  const uint64_t count = c1 - c0;
  uint64_t grid = (uint64_t)c->cus * (uint64_t)occ;
  const uint64_t need_blocks = (count + kWavesPerBlock - 1) / kWavesPerBlock;
  if (grid > need_blocks) grid = need_blocks;
  if (grid < 1) grid = 1;
  if ((rc = ensure(c->d_cols, c->cols_cap, P.cols.size()))) return rc;
  if ((rc = ensure(c->d_x0dd, c->x0dd_cap, x0dd.size()))) return rc;
  if ((rc = ensure(c->d_chunk, c->chunk_cap, (size_t)(2 * count)))) return rc;
  hipStream_t s = c->stream;
  c->tables_uid = 0;  // the walk's own tables replace the cached plan's
  SUP_HIP(hipMemcpyAsync(c->d_cols, P.cols.data(), P.cols.size() * sizeof(double), hipMemcpyHostToDevice, s));
  SUP_HIP(hipMemcpyAsync(c->d_x0dd, x0dd.data(), x0dd.size() * sizeof(double), hipMemcpyHostToDevice, s));
  SUP_HIP(hipMemsetAsync(c->d_counter, 0, sizeof(unsigned), s));
  c->head_zero[0] = false;  // this walk leaves queue head 0 nonzero
  WalkParams p{};
  p.cols = c->d_cols;
  p.x0 = c->d_x0dd;
  p.umask = P.chunk_ends;  // walk_dd: its chunk-end rows
  p.chunk_begin = c0;
  p.chunk_count = count;
  p.L = P.lay.L;
  p.m = P.lay.m;
  p.n = P.n;
  p.chunk_out = c->d_chunk;
  p.counter = c->d_counter;
  p.group = 1;
  p.nb_lo = p.nb_hi = 0;
  for (int k = 0; blocked && k < P.lay.m && k < 32; ++k) {  // walk_dd_blocked: nblk of walk bit k
    const uint64_t v = (uint64_t)(P.nblk[P.lay.L + k] & 15);
    if (k < 16) p.nb_lo |= v << (4 * k);
    else p.nb_hi |= v << (4 * (k - 16));
  }
  SUP_HIP(hipEventRecord(c->ev0, s));
  SUP_ON_DEVICE(c->dev, "double-double walk launch");
  SUP_HIP(blocked ? launch_dd_blocked(P.n, p, (int)grid, s) : launch_dd(P.n, p, (int)grid, s));
  SUP_HIP(hipEventRecord(c->ev1, s));
  SUP_HIP(hipMemcpyAsync(parts, c->d_chunk, 2 * count * sizeof(double), hipMemcpyDeviceToHost, s));
  SUP_HIP(hipStreamSynchronize(s));
  float ms = 0.f;
  SUP_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  if (kernel_ms) *kernel_ms = ms;
  return SUP_OK;
}

}  // namespace sup
