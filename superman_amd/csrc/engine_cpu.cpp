// engine_cpu.cpp — the wave-chunk walk on host threads.
//
// Used for the CLI's explicit CPU algorithm (`-c`, reference RunAlgo cpu
// branch main.cu:186-238) and as the hybrid CPU worker of the chunk queue
// (`-c -g -p6`, reference gpu_exact_dense.cu:822-845).  It is never a
// fallback for a GPU request: GPU entry points fail with SUP_ENODEV when no
// device is present.  It simulates the 64 lanes of a wave and performs the
// same fp64 operations in the same order as walk_{dense,sparse,skip}.hip, so
// a chunk range gives bit-identical partials on CPU and GPU.
#include <algorithm>
#include <cmath>
#include <thread>

#include "engine.hpp"

namespace sup {

namespace {

struct Lane {
  double x[SUP_MAX_N];
  double U[SUP_MAX_N / 8 + 2];
};

inline double prod4(const double* x, int n) {
  double p0 = x[0];
  double p1 = n > 1 ? x[1] : 1.0;
  double p2 = n > 2 ? x[2] : 1.0;
  double p3 = n > 3 ? x[3] : 1.0;
  for (int j = 4; j < n; j += 4) {
    p0 *= x[j];
    if (j + 1 < n) p1 *= x[j + 1];
    if (j + 2 < n) p2 *= x[j + 2];
    if (j + 3 < n) p3 *= x[j + 3];
  }
  return (p0 * p1) * (p2 * p3);
}

inline double bprod8(const double* x, int n, int b) {
  double v[8];
  for (int i = 0; i < 8; ++i) v[i] = (8 * b + i < n) ? x[8 * b + i] : 1.0;
  return ((v[0] * v[1]) * (v[2] * v[3])) * ((v[4] * v[5]) * (v[6] * v[7]));
}

inline void suffix_all(Lane& s, int n) {
  const int NB = (n + 7) / 8;
  s.U[NB] = 1.0;
  for (int b = NB - 1; b >= 0; --b) s.U[b] = bprod8(s.x, n, b) * s.U[b + 1];
}

inline void sparse_step(Lane& s, int n, const double* col, int nb) {
  const int NB = (n + 7) / 8;
  for (int b = 0; b < NB && b < nb; ++b) {
    const int hi = std::min(8 * b + 8, n);
    for (int j = 8 * b; j < hi; ++j) s.x[j] += col[j];
  }
  for (int b = NB - 1; b >= 0; --b)
    if (b < nb) s.U[b] = bprod8(s.x, n, b) * s.U[b + 1];
}

inline const double* col_of(const Plan& P, int e, int neg) {
  return P.cols.data() + (size_t)(2 * e + neg) * P.NP;
}

void chunk_start(const Plan& P, uint64_t ga, unsigned lane, Lane& s) {
  const int n = P.n, L = P.lay.L, m = P.lay.m;
  for (int j = 0; j < n; ++j) s.x[j] = P.x0[j];
  uint64_t h = ga ^ (ga >> 1);
  while (h) {
    const int b = __builtin_ctzll(h);
    h &= h - 1;
    const double* c = col_of(P, L + m + b, 0);
    for (int j = 0; j < n; ++j) s.x[j] += c[j];
  }
  for (int e = 0; e < L; ++e) {
    const double sel = ((lane >> e) & 1u) ? 1.0 : 0.0;
    const double* c = col_of(P, e, 0);
    for (int j = 0; j < n; ++j) s.x[j] = std::fma(sel, c[j], s.x[j]);
  }
}

double pairwise64(double* v) {
  for (int w = 64; w > 1; w >>= 1)
    for (int i = 0; i < w / 2; ++i) v[i] = v[2 * i] + v[2 * i + 1];
  return v[0];
}

inline uint32_t next_toggle(uint32_t t, uint32_t k) {
  uint32_t c = ((t >> (k + 1)) << (k + 1)) + (1u << k);
  if (c <= t) c += 2u << k;
  return c;
}

// ---- segmented walk (jit.cpp's generated kernel, same operations) --------
double seg_tree(const double* x, int lo, int hi) {
  if (hi - lo == 1) return x[lo];
  const int mid = lo + (hi - lo + 1) / 2;
  return seg_tree(x, lo, mid) * seg_tree(x, mid, hi);
}

// Product tree values (Plan::outer_tree / inner_tree, jit.cpp make_tree):
// constant item T = halving tree over the tail rows, node i = value(a[i]) *
// value(b[i]).
struct TreeVal {
  double N[2 * SUP_MAX_N], T;
};
inline double tree_id(const ProdTree& t, const double* a, const TreeVal& v, int id) {
  if (id < t.items()) return t.item_row[id] < 0 ? v.T : a[t.item_row[id]];
  return v.N[id - t.items()];
}
void tree_init(const ProdTree& t, const double* a, TreeVal& v) {
  v.T = t.tail_hi > t.tail_lo ? seg_tree(a, t.tail_lo, t.tail_hi) : 1.0;
  for (int i = 0; i < t.K(); ++i) v.N[i] = tree_id(t, a, v, t.a[i]) * tree_id(t, a, v, t.b[i]);
}
// re-form the nodes of step class c (index order)
inline void tree_update(const ProdTree& t, const double* a, TreeVal& v, int c) {
  for (int i = 0; i < t.K(); ++i)
    if ((t.sig[i] >> c) & 1u) v.N[i] = tree_id(t, a, v, t.a[i]) * tree_id(t, a, v, t.b[i]);
}
// the tree's product: its root, else none (1: fma(D, 1, acc) == acc + D)
inline double tree_top(const ProdTree& t, const double* a, const TreeVal& v) {
  return t.root() < 0 ? 1.0 : tree_id(t, a, v, t.root());
}

// D = top_x - top_y of segment 0's tree; a root node's product fuses with
// the subtraction, fma(x_a, x_b, -top_y), as in the kernel (jit.cpp dexpr)
inline double seg_D(const ProdTree& t, const double* x, const TreeVal& vx, const double* y, const TreeVal& vy) {
  if (t.K() == 0) return tree_top(t, x, vx) - tree_top(t, y, vy);
  const int i = t.K() - 1;
  return std::fma(tree_id(t, x, vx, t.a[i]), tree_id(t, x, vx, t.b[i]), -vy.N[i]);
}

// Paired form: Gray steps 2j, 2j+1 differ in walk bit 0 only; segment 0 (the
// rows walk bit 0 touches) is kept as x (bit 0 clear) and y = x + a_0, and the
// pair adds (-1)^j (prod_seg0 x - prod_seg0 y) * U1 (U1 = outer tree over the
// other rows; segment 0's products are its tree over x and over y).
// Pair step j flips walk bit k = ctz(j) + 1; walk bits k <= seg_b use their
// own touched rows, bits > seg_b one shared step over dyn_rows (the generated
// kernel's straight-line step for those bits).
// Cached walk bits 1..seg_cc: the kernel holds every node that depends on
// them once per state of those bits and their steps only accumulate.  Only
// x^0 (walk bits 0..cc clear) is walked; every row copy is a pure function of
// it, x^S_r = x^0_r + seg_cx(r, S) (x^0_r when no bit of S touches r) and
// y^S_r = x^0_r + seg_cy(r, S), whether the kernel keeps it live or forms it
// on demand.  Restated here as one full lane state per cached state S, its
// rows re-derived from x^0 whenever x^0_r changes; every non-cached step then
// re-forms every state's dirty nodes, and pair j accumulates with the state
// of its Gray bits.
constexpr int kMaxCached = kMaxCachedBits;
struct SegLane {
  double x0[SUP_MAX_N];
  double x[1 << kMaxCached][SUP_MAX_N], y[1 << kMaxCached][SUP_MAX_N], D[1 << kMaxCached];
  TreeVal o[1 << kMaxCached], ix[1 << kMaxCached], iy[1 << kMaxCached];
};
// Row-copy constants of a plan: cached part of each row's classes and
// cx[r][S], cy[r][S] (seg_cx / seg_cy) for S within it.
struct SegConsts {
  uint32_t rs[SUP_MAX_N];
  double cx[SUP_MAX_N][1 << kMaxCached], cy[SUP_MAX_N][1 << kMaxCached];
  explicit SegConsts(const Plan& P) {
    const uint32_t ccm = (1u << P.seg_cc) - 1u;
    for (int r = 0; r < P.n; ++r) rs[r] = 0;
    for (int k = 1; k <= P.seg_cc && k < P.lay.m; ++k)
      for (int r : P.touched[k]) rs[r] |= 1u << (k - 1);
    for (int r = 0; r < P.n; ++r) {
      rs[r] &= ccm;
      for (uint32_t S = 0; S < (1u << P.seg_cc); ++S) {
        if (S & ~rs[r]) continue;
        cx[r][S] = S ? seg_cx(P, r, S) : 0.0;
        cy[r][S] = r < P.seg_start[1] ? seg_cy(P, r, S) : 0.0;
      }
    }
  }
};

inline void seg_derive(SegLane& g, const Plan& P, const SegConsts& K, int r) {
  const int len0 = P.seg_start[1];
  for (uint32_t S = 0; S < (1u << P.seg_cc); ++S) {
    const uint32_t s = S & K.rs[r];
    g.x[S][r] = s ? g.x0[r] + K.cx[r][s] : g.x0[r];
    if (r < len0) g.y[S][r] = g.x0[r] + K.cy[r][s];
  }
}

void seg_init(const Lane& s, SegLane& g, const Plan& P, const SegConsts& K) {
  const int NS = 1 << P.seg_cc;
  std::copy(s.x, s.x + P.n, g.x0);
  for (int r = 0; r < P.n; ++r) seg_derive(g, P, K, r);
  for (int S = 0; S < NS; ++S) {
    tree_init(P.outer_tree, g.x[S], g.o[S]);
    tree_init(P.inner_tree, g.x[S], g.ix[S]);
    tree_init(P.inner_tree, g.y[S], g.iy[S]);
    g.D[S] = seg_D(P.inner_tree, g.x[S], g.ix[S], g.y[S], g.iy[S]);
  }
}

void seg_step(SegLane& g, const Plan& P, const SegConsts& K, int k, int neg) {
  const int c = k <= P.seg_b ? k - 1 : P.seg_b;
  if (c < P.seg_cc) return;  // cached walk bit: nothing changes
  if (k > P.seg_b) {  // shared step: full signed column over dyn_rows (zeros included)
    if (P.dyn_rows.empty()) return;
    const double* col = col_of(P, P.lay.L + k, neg);
    for (int r : P.dyn_rows) g.x0[r] += col[r], seg_derive(g, P, K, r);
  } else {
    const std::vector<int>& t = P.touched[k];
    if (t.empty()) return;
    const size_t blk = (t.size() + 7) & ~(size_t)7;
    const double* v = P.jtab.data() + P.jofs[k] + (neg ? blk : 0);
    for (size_t i = 0; i < t.size(); ++i) g.x0[t[i]] += v[i], seg_derive(g, P, K, t[i]);
  }
  for (int S = 0; S < (1 << P.seg_cc); ++S) {
    tree_update(P.outer_tree, g.x[S], g.o[S], c);
    if ((P.inner_tree.root_sig() >> c) & 1u) {
      tree_update(P.inner_tree, g.x[S], g.ix[S], c);
      tree_update(P.inner_tree, g.y[S], g.iy[S], c);
      g.D[S] = seg_D(P.inner_tree, g.x[S], g.ix[S], g.y[S], g.iy[S]);
    }
  }
}

// cached state at pair index j: Gray bits 1..cc of the walk (pair bits 0..cc-1)
inline int seg_state(uint32_t j, int cc) {
  int S = 0;
  for (int i = 0; i < cc; ++i) S |= (int)(((j >> i) ^ (j >> (i + 1))) & 1u) << i;
  return S;
}

// One wave-chunk: returns the wave's pairwise lane sum.
double chunk_partial(const Plan& P, uint64_t ga) {
  const int n = P.n, L = P.lay.L, m = P.lay.m;
  const uint32_t T = 1u << m;
  double lane_val[64];
  if (P.kind == kWalkSeg) {
    // the kernel's chunk skip: the outer tree's tail (rows no walk bit touches)
    // is an exact zero in every valid lane -> the chunk's part is +0
    const ProdTree& ot = P.outer_tree;
    if (ot.tail_hi > ot.tail_lo) {
      bool live = false;
      for (unsigned l = 0; l < (1u << L) && !live; ++l) {
        Lane s;
        chunk_start(P, ga, l, s);
        live = seg_tree(s.x, ot.tail_lo, ot.tail_hi) != 0.0;
      }
      if (!live) return 0.0;
    }
    const SegConsts K(P);
    for (unsigned l = 0; l < 64; ++l) {
      if (l >= (1u << L)) {
        lane_val[l] = 0.0;
        continue;
      }
      Lane s;
      chunk_start(P, ga, l, s);
      static thread_local SegLane g;
      seg_init(s, g, P, K);
      double acc = g.D[0] * tree_top(P.outer_tree, g.x[0], g.o[0]);
      // two-level lane sum (the kernel's): acc folds into tot after each shared
      // dyn step's pair j = 2^seg_b (q + 1), so no sequential sum runs longer
      // than 2^seg_b pairs
      double tot = 0.0;
      const uint32_t qmask = (1u << P.seg_b) - 1u;
      for (uint32_t j = 1; j < T / 2; ++j) {  // pair steps: walk bit ctz(j) + 1
        const uint32_t pb = __builtin_ctz(j);
        seg_step(g, P, K, (int)pb + 1, (j >> (pb + 1)) & 1u);
        const int S = seg_state(j, P.seg_cc);
        acc = std::fma((j & 1u) ? -g.D[S] : g.D[S], tree_top(P.outer_tree, g.x[S], g.o[S]), acc);
        if ((j & qmask) == 0u) tot += acc, acc = 0.0;
      }
      acc = tot + acc;
      const unsigned par = (unsigned)__builtin_popcount(l) & 1u;
      if ((((unsigned)ga) ^ par) & 1u) acc = -acc;
      lane_val[l] = acc;
    }
    return pairwise64(lane_val);
  }
  if (P.kind != kWalkSkip) {
    if (P.kind == kWalkSparse && P.chunk_ends) {
      // the kernel's chunk end: a chunk-end row (lane-uniform, no walk column)
      // exactly zero at the first state -> the chunk's part is +0
      Lane s;
      chunk_start(P, ga, 0, s);
      for (int j = 0; j < n; ++j)
        if (((P.chunk_ends >> j) & 1u) && s.x[j] == 0.0) return 0.0;
    }
    for (unsigned l = 0; l < 64; ++l) {
      if (l >= (1u << L)) {
        lane_val[l] = 0.0;
        continue;
      }
      Lane s;
      chunk_start(P, ga, l, s);
      double acc;
      if (P.kind == kWalkDense) {
        acc = prod4(s.x, n);
        for (uint32_t t = 1; t < T; ++t) {
          const uint32_t k = __builtin_ctz(t);
          const int neg = (t >> (k + 1)) & 1u;
          const double* c = col_of(P, L + k, neg);
          for (int j = 0; j < n; ++j) s.x[j] += c[j];
          const double pr = prod4(s.x, n);
          acc = (t & 1u) ? acc - pr : acc + pr;
        }
      } else {
        suffix_all(s, n);
        acc = s.U[0];
        for (uint32_t t = 1; t < T; ++t) {
          const uint32_t k = __builtin_ctz(t);
          const int neg = (t >> (k + 1)) & 1u;
          sparse_step(s, n, col_of(P, L + k, neg), P.nblk[L + k]);
          acc = (t & 1u) ? acc - s.U[0] : acc + s.U[0];
        }
      }
      const unsigned par = (unsigned)__builtin_popcount(l) & 1u;
      if ((((unsigned)ga) ^ par) & 1u) acc = -acc;
      lane_val[l] = acc;
    }
    return pairwise64(lane_val);
  }
  // SkipPer: all 64 lanes in lock-step, wave-uniform jumps at segment
  // starts (walk_skip.hip: segments of 2^kSkipSegBits Gray steps).
  static thread_local Lane S[64];
  double acc[64];
  for (unsigned l = 0; l < 64; ++l) {
    chunk_start(P, ga, l, S[l]);
    suffix_all(S[l], n);
    acc[l] = S[l].U[0];  // state 0
  }
  auto all_zero = [&]() {
    for (unsigned l = 0; l < 64; ++l)
      if (S[l].U[0] != 0.0) return false;
    return true;
  };
  auto step = [&](uint32_t k, int neg) {
    for (unsigned l = 0; l < 64; ++l) sparse_step(S[l], n, col_of(P, L + k, neg), P.nblk[L + k]);
  };
  uint32_t u = 1;
  bool check = true;
  for (; T > 1;) {  // T = 1: state 0 is the chunk
    if (check && all_zero()) {
      const uint32_t t = u - 1;
      uint64_t zm = 0;
      for (int r = 0; r < n; ++r)
        if (S[0].x[r] == 0.0) zm |= 1ull << r;
      zm &= P.umask;
      uint32_t nx = t;
      while (zm) {
        const int r = __builtin_ctzll(zm);
        zm &= zm - 1;
        uint64_t mm = P.rowmask[r];
        if (mm & kSkipSegMask) continue;
        uint32_t tr = T;
        while (mm) {
          const uint32_t k = __builtin_ctzll(mm);
          mm &= mm - 1;
          const uint32_t c = next_toggle(t, k);
          tr = c < tr ? c : tr;
        }
        nx = tr > nx ? tr : nx;
      }
      if (nx >= T) break;
      if (nx > t) {
        const uint32_t gn = nx ^ (nx >> 1);
        uint32_t diff = (t ^ (t >> 1)) ^ gn;
        do {
          const uint32_t k = __builtin_ctz(diff);
          diff &= diff - 1;
          step(k, ((gn >> k) & 1u) ^ 1u);
        } while (diff);
        for (unsigned l = 0; l < 64; ++l) acc[l] += S[l].U[0];  // nx: a segment start, even
        u = nx + 1;
        continue;
      }
    }
    step(0, (u >> 1) & 1u);
    for (unsigned l = 0; l < 64; ++l) acc[l] -= S[l].U[0];
    if (u + 1 >= T) break;
    const uint32_t v = u + 1, k = __builtin_ctz(v);
    step(k, (v >> (k + 1)) & 1u);
    for (unsigned l = 0; l < 64; ++l) acc[l] += S[l].U[0];
    u += 2;
    check = (v & kSkipSegMask) == 0;
  }
  for (unsigned l = 0; l < 64; ++l) {
    const unsigned par = (unsigned)__builtin_popcount(l) & 1u;
    double a = acc[l];
    if ((((unsigned)ga) ^ par) & 1u) a = -a;
    lane_val[l] = (l < (1u << L)) ? a : 0.0;
  }
  return pairwise64(lane_val);
}

}  // namespace

double cpu_walk_range(const Plan& P, uint64_t c0, uint64_t c1, int threads) {
  if (c1 <= c0) return 0.0;
  const uint64_t count = c1 - c0;
  std::vector<double> part(count, 0.0);
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(threads, 1), count));
  std::vector<std::thread> th;
  for (int w = 0; w < T; ++w)
    th.emplace_back([&, w]() {
      for (uint64_t a = w; a < count; a += (uint64_t)T) part[a] = chunk_partial(P, c0 + a);
    });
  for (auto& t : th) t.join();
  // same 64-way zero-padded pairwise passes as launch_pairwise_reduce
  while (part.size() > 1) {
    const size_t groups = (part.size() + 63) / 64;
    std::vector<double> nxt(groups);
    for (size_t g = 0; g < groups; ++g) {
      double v[64];
      for (int l = 0; l < 64; ++l) {
        const size_t i = g * 64 + l;
        v[l] = i < part.size() ? part[i] : 0.0;
      }
      nxt[g] = pairwise64(v);
    }
    part.swap(nxt);
  }
  return part[0];
}

// ---- exact path: walk_exact.hip's residue arithmetic on host threads ----
namespace {
inline double red(double t, double p, double pinv) { return std::fma(-std::rint(t * pinv), p, t); }
inline double chain_mod(const double* x, int n, double p, double pinv) {
  double r = red(x[0], p, pinv);  // |r| < 1.5 p before the first product
  for (int j = 1; j < n; ++j) r = red(r * x[j], p, pinv);
  return r;
}
inline uint64_t to_res(double v, uint64_t p) {  // |v| < 2^53, integer-valued
  const int64_t i = (int64_t)v % (int64_t)p;
  return (uint64_t)(i < 0 ? i + (int64_t)p : i);
}
}  // namespace

void cpu_exact_range(const Plan& P, uint64_t c0, uint64_t c1, const std::vector<double>& primes, int threads,
                     std::vector<uint64_t>& res) {
  const int np = (int)primes.size(), n = P.n, L = P.lay.L, m = P.lay.m;
  res.assign(np, 0);
  if (c1 <= c0) return;
  const uint64_t count = c1 - c0;
  const int TH = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(threads, 1), count));
  std::vector<std::vector<uint64_t>> part(TH, std::vector<uint64_t>(np, 0));
  std::vector<std::thread> th;
  for (int w = 0; w < TH; ++w)
    th.emplace_back([&, w]() {
      std::vector<double> pinv(np), acc(np);
      for (int q = 0; q < np; ++q) pinv[q] = 1.0 / primes[q];
      for (uint64_t a = w; a < count; a += (uint64_t)TH) {
        const uint64_t ga = c0 + a;
        if (P.chunk_ends) {  // walk_exact's chunk end: a zero chunk-end row, every term zero
          Lane s;
          chunk_start(P, ga, 0, s);
          bool end = false;
          for (int j = 0; j < n && !end; ++j) end = ((P.chunk_ends >> j) & 1u) && s.x[j] == 0.0;
          if (end) continue;
        }
        for (unsigned l = 0; l < (1u << L); ++l) {
          Lane s;
          chunk_start(P, ga, l, s);
          for (int q = 0; q < np; ++q) acc[q] = chain_mod(s.x, n, primes[q], pinv[q]);
          for (uint32_t t = 1; t < (1u << m); ++t) {
            const uint32_t k = __builtin_ctz(t);
            const double* c = col_of(P, L + (int)k, (t >> (k + 1)) & 1u);
            for (int j = 0; j < n; ++j) s.x[j] += c[j];
            for (int q = 0; q < np; ++q) {
              const double r = chain_mod(s.x, n, primes[q], pinv[q]);
              acc[q] = (t & 1u) ? acc[q] - r : acc[q] + r;
              if ((t & 255u) == 0u) acc[q] = red(acc[q], primes[q], pinv[q]);
            }
          }
          const bool flip = (((unsigned)ga ^ (unsigned)__builtin_popcount(l)) & 1u) != 0;
          for (int q = 0; q < np; ++q) {
            const uint64_t pq = (uint64_t)primes[q];
            const uint64_t v = to_res(red(acc[q], primes[q], pinv[q]), pq);
            part[w][q] = (part[w][q] + (flip ? (pq - v) % pq : v)) % pq;
          }
        }
      }
    });
  for (auto& t : th) t.join();
  for (int q = 0; q < np; ++q) {
    const uint64_t pq = (uint64_t)primes[q];
    for (int w = 0; w < TH; ++w) res[q] = (res[q] + part[w][q]) % pq;
  }
}

}  // namespace sup
