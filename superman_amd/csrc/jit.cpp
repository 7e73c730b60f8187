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
//   * re-multiplies only the segments that contain a touched row, then the
//     suffix chain U_i = S_i * U_{i+1} down to U_0, the term.
// Segments are the first-touch groups of the walk columns (rows walk bit k
// touched first), so a step of walk bit k never goes deeper than segment k.
//
// Paired form.  Gray steps 2j and 2j+1 differ in walk bit 0 only.  Segment 0
// (the rows walk bit 0 touches) is held twice, x (bit 0 clear) and
// y = x + a_0 (bit 0 set), and the pair contributes
//   (-1)^j (prod_seg0 x - prod_seg0 y) * U1,    U1 = product of all other rows,
// accumulated with one fma.  The walk is then a Gray walk over walk bits
// 1..m-1 at half the step count; a step touching segment 0 updates both copies
// and re-forms both products.  The loop is unrolled by 2^b pair steps
// (b = seg_static_bits): pair bits below b get straight-line steps with
// compile-time table offsets (the top one with sign q&1), and every higher
// bit shares one straight-line step over the union of their rows (full signed
// column, zeros included) — a switch over per-bit steps would make LLVM
// carry copies of x across its arms (measured: 120 -> 242 VGPRs).
//
// Measured on MI355X (profiles/r1): n=40 d=0.5 bench matrix 29.4 VALU
// instructions per Gray step (cost model 32.7; the prefix-blocked AOT walk
// executes 46.6, the plain dense walk 81), VALU 99% busy, 1.26e12 steps/s.
// Everything else (chunk start, lane layout, wave-chunk queue, reduction
// order) is walk_common.hpp's, shared with the ahead-of-time kernels, and
// the arithmetic is mirrored bit for bit by engine_cpu.cpp (seg_*) and
// oracle/oracle.c (kind 3).
//
// Compiled code objects are cached in memory (per process, per device) and on
// disk: $SUP_JIT_CACHE_DIR, else $XDG_CACHE_HOME/superman_amd, else
// ~/.cache/superman_amd (SUP_JIT_CACHE_DIR="" disables the disk cache).
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>

#include "engine.hpp"

namespace sup {

namespace {
#include "jit_headers.inc"  // kWalkCommonSrc, kWalkParamsSrc (generated from the headers by the Makefile)

// ---------------------------------------------------------------- planning --

struct SegShape {
  std::vector<int> seg_start;               // boundaries, rows in first-touch order
  std::vector<std::vector<int>> touched;    // per walk bit, engine rows
};

// Segment structure of walk columns `walk` (matrix columns, in walk-bit order):
// rows are numbered in first-touch order.
SegShape seg_shape(const double* A, int n, const std::vector<int>& walk) {
  SegShape s;
  std::vector<int> pos(n, -1);
  int R = 0;
  s.seg_start.push_back(0);
  for (int c : walk) {
    for (int i = 0; i < n; ++i)
      if (pos[i] < 0 && A[(size_t)i * n + c] != 0.0) pos[i] = R++;
    if (R > s.seg_start.back()) s.seg_start.push_back(R);
  }
  for (int c : walk) {
    std::vector<int> t;
    for (int i = 0; i < n; ++i)
      if (A[(size_t)i * n + c] != 0.0) t.push_back(pos[i]);
    std::sort(t.begin(), t.end());
    s.touched.push_back(std::move(t));
  }
  return s;
}

int seg_index(const std::vector<int>& seg_start, int row) {
  return (int)(std::upper_bound(seg_start.begin(), seg_start.end(), row) - seg_start.begin()) - 1;
}

// Segment 0 is split the same way as the whole matrix: its rows are ordered
// by the first walk bit >= 1 that touches them (sub-segments), rows no such
// bit touches last (constant within a wave-chunk).  Sub-segment of each
// segment-0 row, -1 for the constant ones; *nsub, *srest = counts.
std::vector<int> sub_of(const std::vector<int>& seg_start, const std::vector<std::vector<int>>& touched, int* nsub,
                        int* srest) {
  const int len0 = seg_start[1];
  std::vector<int> sub(len0, -1);
  int cnt = 0, ns = 0;
  for (size_t k = 1; k < touched.size(); ++k) {
    bool grew = false;
    for (int r : touched[k])
      if (r < len0 && sub[r] < 0) sub[r] = ns, ++cnt, grew = true;
    if (grew) ++ns;
  }
  *nsub = ns;
  *srest = len0 - cnt;
  return sub;
}

// Ops of one chain update (segments of sizes len[], constant tail present or
// not) for dirty segments `dirty` up to `smax`: (len - 1) muls per dirty
// segment of the tree, one chain mul per segment (none for the last one
// without a tail).
double chain_ops(const std::vector<int>& len, bool tail, const std::vector<char>& dirty, int smax) {
  double ops = 0.0;
  const int ns = (int)len.size();
  for (int i = 0; i <= smax; ++i) {
    if (dirty[i]) ops += len[i] - 1;
    if (i < ns - 1 || tail) ops += 1.0;
  }
  return ops;
}

// VALU ops of one pair step flipping a walk bit k >= 1 that touches rows t
// (the generated code, exactly): |t| adds, plus one more per touched row of
// segment 0 (its bit-0-set copy y); the outer chain over segments >= 1; when
// segment 0 is touched, its sub-segment chains for x and for y and their
// difference D; one fma into the accumulator.
double step_ops(const std::vector<int>& seg_start, int n, const std::vector<int>& t, const std::vector<int>& sub,
                int nsub, int srest) {
  if (t.empty()) return 1.0;
  const int nseg = (int)seg_start.size() - 1, len0 = seg_start[1];
  std::vector<int> olen;
  for (int i = 1; i < nseg; ++i) olen.push_back(seg_start[i + 1] - seg_start[i]);
  std::vector<int> slen(nsub, 0);
  for (int r = 0; r < len0; ++r)
    if (sub[r] >= 0) ++slen[sub[r]];
  std::vector<char> od(std::max(nseg - 1, 1), 0), sd(std::max(nsub, 1), 0);
  int omax = -1, smax = -1;
  double ops = (double)t.size() + 1.0;
  for (int r : t) {
    if (r < len0) {
      ops += 1.0;
      sd[sub[r]] = 1;
      smax = std::max(smax, sub[r]);
    } else {
      const int i = seg_index(seg_start, r) - 1;
      od[i] = 1;
      omax = std::max(omax, i);
    }
  }
  if (omax >= 0) ops += chain_ops(olen, seg_start.back() < n, od, omax);
  if (smax >= 0) ops += 2.0 * chain_ops(slen, srest > 0, sd, smax) + 1.0;
  return ops;
}

// Gray steps come in pairs that differ in walk bit 0 only, so a pair step
// flips walk bit k >= 1 (pair bit k-1); pair bits p < b get a specialised
// step each, bits p >= b (1/2^b of the pair steps) share one step over the
// union of their rows.  Ops per Gray step = ops per pair step / 2.
double cost_of(const std::vector<int>& seg_start, int n, const std::vector<std::vector<int>>& touched) {
  const int m = (int)touched.size(), b = seg_static_bits(m);
  int nsub = 0, srest = 0;
  const std::vector<int> sub = sub_of(seg_start, touched, &nsub, &srest);
  std::vector<char> in(n, 0);
  for (int k = b + 1; k < m; ++k)
    for (int r : touched[k]) in[r] = 1;
  std::vector<int> dyn;
  for (int j = 0; j < n; ++j)
    if (in[j]) dyn.push_back(j);
  const double dyn_ops = step_ops(seg_start, n, dyn, sub, nsub, srest);
  double c = 0.0, w = 0.5;
  for (int p = 0; p + 1 < m; ++p, w *= 0.5)
    c += w * (p < b ? step_ops(seg_start, n, touched[p + 1], sub, nsub, srest) : dyn_ops);
  return c / 2.0;
}

double shape_cost(const SegShape& s, int n) { return cost_of(s.seg_start, n, s.touched); }

// Step class of walk bit k >= 1: k - 1 for the specialised pair bits, seg_b
// for the shared step of the walk bits above them.
int step_class(int k, int b) { return k <= b ? k - 1 : b; }

// Greedy product tree over rows [lo, tail_lo) (+ the constant item for rows
// [tail_lo, tail_hi)): repeatedly join the two clusters whose union is dirty
// least often, i.e. minimise w(sig_i | sig_j) with w(class c) = 2^(b-1-c) (walk
// bit c+1 flips on 2^-(c+1) of the pair steps) and w(shared) = 1; ties -> the
// first pair (i < j) in list order; the joined cluster goes to the end.  Rows
// that always change together end up under one node, so a step re-forms only
// the nodes above the rows it touches (the first-touch chain it replaces had
// to re-form whole segments and every link above them).
ProdTree make_tree(const std::vector<uint32_t>& rsig, int lo, int tail_lo, int tail_hi, int b) {
  ProdTree t;
  t.tail_lo = tail_lo, t.tail_hi = tail_hi;
  for (int r = lo; r < tail_lo; ++r) t.item_row.push_back(r), t.item_sig.push_back(rsig[r]);
  if (tail_hi > tail_lo) t.item_row.push_back(-1), t.item_sig.push_back(0u);
  auto weight = [b](uint32_t s) {
    uint64_t w = 0;
    for (int c = 0; c <= b; ++c)
      if ((s >> c) & 1u) w += c < b ? (1ull << (b - 1 - c)) : 1ull;
    return w;
  };
  std::vector<int> id;
  std::vector<uint32_t> sg;
  for (int i = 0; i < t.items(); ++i) id.push_back(i), sg.push_back(t.item_sig[i]);
  while (id.size() > 1) {
    size_t bi = 0, bj = 1;
    uint64_t bw = UINT64_MAX;
    for (size_t i = 0; i < id.size(); ++i)
      for (size_t j = i + 1; j < id.size(); ++j) {
        const uint64_t w = weight(sg[i] | sg[j]);
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

int nodes_with(const ProdTree& t, int c) {
  int k = 0;
  for (uint32_t s : t.sig) k += (s >> c) & 1u;
  return k;
}

}  // namespace

int seg_static_bits(int m) { return std::min(m - 1, 5); }

// Ops per Gray step of the generated kernel, exactly: per pair step of class
// c, the adds of its rows (twice on segment 0), the dirty outer nodes, the
// dirty inner nodes over x and over y, D when segment 0 changed, the fma.
double seg_walk_cost(const Plan& P) {
  const int m = P.lay.m, b = P.seg_b, len0 = P.seg_start[1];
  double c = 0.0, w = 0.5;
  for (int p = 0; p + 1 < m; ++p, w *= 0.5) {
    const int k = p + 1, cl = step_class(k, b);
    const std::vector<int>& t = k <= b ? P.touched[k] : P.dyn_rows;
    double ops = 1.0 + (double)t.size();
    for (int r : t) ops += r < len0;
    ops += nodes_with(P.outer_tree, cl) + 2.0 * nodes_with(P.inner_tree, cl);
    ops += (P.inner_tree.root_sig() >> cl) & 1u;
    c += w * ops;
  }
  return c / 2.0;
}

std::vector<int> seg_walk_order(const double* A, int n, int m, int count) {
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
  // walk bit 0 defines segment 0 (the paired rows): it must touch a row
  auto cost = [&](const std::vector<int>& o) {
    if (nnz[o[0]] == 0) return 1e300;
    return shape_cost(seg_shape(A, n, std::vector<int>(o.begin(), o.begin() + m)), n);
  };
  std::vector<int> best;
  double bcost = 1e300;
  for (int f = 0; f < nb && m > 0; ++f) {
    std::vector<int> o = extend({f}, m);
    const double c = cost(o);
    if (c < bcost) bcost = c, best = o;
  }
  if (m == 0) return extend({}, count);
  // descent: swap a walk position with another walk position or an unused
  // column while the cost drops (positions whose weight 2^-(k+1) is visible)
  const int hot = std::min(m, 12);
  for (int pass = 0; pass < 8; ++pass) {
    bool improved = false;
    for (int a = 0; a < hot; ++a) {
      for (int c = 0; c < nb; ++c) {
        if (c == best[a]) continue;
        std::vector<int> o = best;
        auto it = std::find(o.begin(), o.end(), c);
        if (it != o.end()) std::swap(o[a], *it);
        else o[a] = c;
        const double v = cost(o);
        if (v < bcost - 1e-12) bcost = v, best = o, improved = true;
      }
    }
    if (!improved) break;
  }
  return extend(best, count);
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
namespace {

std::string tree(int lo, int hi, const char* v = "x") {
  if (hi - lo == 1) return std::string(v) + "[" + std::to_string(lo) + "]";
  const int mid = lo + (hi - lo + 1) / 2;
  return "(" + tree(lo, mid, v) + " * " + tree(mid, hi, v) + ")";
}

// Signature of node i's parent (-1 for the root): a node dirty exactly when
// its parent is need not stay live between steps.
int parent_sig(const ProdTree& t, int i) {
  const int id = t.items() + i;
  for (int j = i + 1; j < t.K(); ++j)
    if (t.a[j] == id || t.b[j] == id) return (int)t.sig[j];
  return -1;
}

// Names of one product tree's values in the generated code: items are the
// row array `arr` and the constant item `T`; node i is `N<i>`.
struct TreeNames {
  const ProdTree* t;
  std::string arr, N, T;
  std::string id(int i) const {
    if (i < t->items()) return t->item_row[i] < 0 ? T : arr + "[" + std::to_string(t->item_row[i]) + "]";
    return N + std::to_string(i - t->items());
  }
  std::string top() const { return t->root() < 0 ? std::string() : id(t->root()); }
  std::string node(int i) const { return id(t->a[i]) + " * " + id(t->b[i]); }
};

// Generated kernel (paired segmented walk).  Gray steps 2j and 2j+1 differ in
// walk bit 0 only, so they are evaluated together: segment 0 (the rows walk
// bit 0 touches) is held twice, x (bit 0 clear) and y = x + a_0 (bit 0 set),
// and the pair contributes (-1)^j (prod_seg0 x - prod_seg0 y) * U1, U1 being
// the product of every other row.  The pair walk is a Gray walk over walk
// bits 1..m-1 (pair bit p = walk bit p+1).  Both products are product trees
// (make_tree): a step re-forms the nodes above the rows it touches.
struct Gen {
  const Plan& P;
  int len0;
  TreeNames outer, inx, iny;
  std::ostringstream o;
  explicit Gen(const Plan& p) : P(p), len0(p.seg_start[1]) {
    outer = {&p.outer_tree, "x", "o", "Ro"};
    inx = {&p.inner_tree, "x", "px", "Cx"};
    iny = {&p.inner_tree, "y", "py", "Cy"};
  }

  void tree_init(const TreeNames& t, const char* ind) {
    if (t.t->tail_hi > t.t->tail_lo)
      o << ind << "const double " << t.T << " = " << tree(t.t->tail_lo, t.t->tail_hi, t.arr.c_str()) << ";\n";
    for (int i = 0; i < t.t->K(); ++i) o << ind << "double " << t.N << i << " = " << t.node(i) << ";\n";
  }
  // re-form the nodes of step class c; returns whether the root changed
  bool tree_update(const TreeNames& t, int c, const char* ind) {
    for (int i = 0; i < t.t->K(); ++i)
      if ((t.t->sig[i] >> c) & 1u) o << ind << "  " << t.N << i << " = " << t.node(i) << ";\n";
    return (t.t->root_sig() >> c) & 1u;
  }
  std::string dexpr() const { return inx.top() + " - " + iny.top(); }
  void accumulate(bool neg, const char* ind) {
    if (outer.top().empty()) o << ind << (neg ? "acc -= D;\n" : "acc += D;\n");
    else o << ind << "acc = __builtin_fma(" << (neg ? "-D" : "D") << ", " << outer.top() << ", acc);\n";
  }

  // Add the values at table pointer `cv` (dbl8 pieces) to rows `rows` (and
  // to their y copies in segment 0): value i of the block belongs to row
  // rows[i] (packed table), or value rows[i] of the block (full column,
  // `full`).  At most 2 pieces (32 SGPRs) are pinned at a time.
  void adds(const std::vector<int>& rows, bool full, const char* ind) {
    std::vector<std::pair<int, int>> vr;  // (value index, row)
    for (size_t i = 0; i < rows.size(); ++i) vr.push_back({full ? rows[i] : (int)i, rows[i]});
    std::vector<int> pieces;
    for (auto& e : vr)
      if (pieces.empty() || pieces.back() != e.first / 8) pieces.push_back(e.first / 8);
    for (size_t g = 0; g < pieces.size(); g += 2) {
      const size_t ge = std::min(pieces.size(), g + 2);
      for (size_t q = g; q < ge; ++q) o << ind << "  jdbl8 v" << pieces[q] << " = cv[" << pieces[q] << "];\n";
      o << ind << "  asm volatile(\"\" :";
      for (size_t q = g; q < ge; ++q) o << (q > g ? ", " : " ") << "\"+s\"(v" << pieces[q] << ")";
      o << ");\n";
      for (auto& e : vr)
        if (e.first / 8 >= pieces[g] && e.first / 8 <= pieces[ge - 1]) {
          const std::string v = "v" + std::to_string(e.first / 8) + "[" + std::to_string(e.first % 8) + "]";
          o << ind << "  x[" << e.second << "] += " << v << ";\n";
          if (e.second < len0) o << ind << "  y[" << e.second << "] += " << v << ";\n";
        }
      if (ge < pieces.size()) o << ind << "  __builtin_amdgcn_sched_barrier(0);\n";
    }
  }

  void products(int c, const char* ind) {
    tree_update(outer, c, ind);
    if (tree_update(inx, c, ind)) {
      tree_update(iny, c, ind);
      o << ind << "  D = " << dexpr() << ";\n";
    }
  }

  // pair step flipping walk bit k <= seg_b: packed touched values; `off` = byte offset expression
  void step(int k, const std::string& off, const char* ind) {
    const std::vector<int>& t = P.touched[k];
    if (t.empty()) return;
    o << ind << "{\n";
    o << ind << "  cjdbl8* cv = (cjdbl8*)opaque_c(p.jtab, " << off << ");\n";
    adds(t, false, ind);
    products(step_class(k, P.seg_b), ind);
    o << ind << "}\n";
  }

  std::string off_const(int k, int neg) const {
    const int blk = (((int)P.touched[k].size() + 7) & ~7);
    return std::to_string((P.jofs[k] + neg * blk) * 8) + "u";
  }
  std::string off_dyn(int k, const char* negv) const {
    const int blk = (((int)P.touched[k].size() + 7) & ~7);
    return std::to_string(P.jofs[k] * 8) + "u + " + negv + " * " + std::to_string(blk * 8) + "u";
  }

  std::string source() {
    const int n = P.n, L = P.lay.L, m = P.lay.m, b = P.seg_b;
    const unsigned B = 1u << b, Q = 1u << (m - 1 - b);
    o << "// generated by superman_amd jit.cpp: paired segmented Gray walk, n=" << n << " L=" << L << " m=" << m
      << " segment0=" << len0 << " (" << P.inner_tree.K() << " tree nodes) outer tree nodes=" << P.outer_tree.K()
      << " pair bits specialised=" << b << "\n";
    o << "#include \"walk_common.hpp\"\n";
    o << "namespace sup {\n";
    o << "typedef double jdbl8 __attribute__((ext_vector_type(8)));\n";
    o << "typedef const __attribute__((address_space(4))) jdbl8 cjdbl8;\n";
    // occupancy target from the values live across the walk loop (x, y,
    // chain values, D, acc, loop state; 2 VGPRs each): the compiler's own
    // choice trades occupancy 2 for scheduling freedom, which costs more
    // latency hiding than it buys.  SUP_JIT_WAVES overrides (experiments).
    int vals = n + len0 + 4;
    for (const TreeNames* t : {&outer, &inx, &iny}) {  // nodes kept across steps
      vals += t->t->tail_hi > t->t->tail_lo;
      for (int i = 0; i < t->t->K(); ++i) {
        const int par = parent_sig(*t->t, i);
        vals += par < 0 || (uint32_t)par != t->t->sig[i];
      }
    }
    int waves = 2 * vals <= 116 ? 4 : 3;  // (occupancy 2 is never worth it: measured)
    if (const char* e = std::getenv("SUP_JIT_WAVES")) waves = std::max(1, std::min(8, std::atoi(e)));
    o << "extern \"C\" __global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(" << waves
      << "))) void sup_walk_seg(WalkParams p) {\n";
    o << "  constexpr int N = " << n << ";\n";
    o << "  const uint32_t lane = threadIdx.x & 63u;\n";
    o << "  const bool lane_valid = lane < " << (1u << L) << "u;\n";
    o << "  const uint32_t lane_par = __builtin_popcount(lane) & 1u;\n";
    o << "  for (uint32_t g = next_chunk(p.counter); (uint64_t)g * p.group < p.chunk_count; g = next_chunk(p.counter)) {\n";
    o << "    double keep = 0.0;\n";
    o << "    for (uint32_t j = 0; j < (uint32_t)p.group; ++j) {\n";
    o << "      const uint64_t a = (uint64_t)g * p.group + j;\n";
    o << "      if (a >= p.chunk_count) break;\n";
    o << "      const uint64_t ga = p.chunk_begin + a;\n";
    o << "      double x[N], y[" << len0 << "];\n";
    o << "      chunk_start<N>(x, p, ga, lane);\n";
    o << "      {\n";  // y = x + a_0 on segment 0 (the + block of walk bit 0)
    o << "        cjdbl8* cv = (cjdbl8*)opaque_c(p.jtab, " << off_const(0, 0) << ");\n";
    for (int r = 0; r < len0; ++r) o << "        y[" << r << "] = x[" << r << "] + cv[" << r / 8 << "][" << r % 8 << "];\n";
    o << "      }\n";
    tree_init(outer, "      ");
    tree_init(inx, "      ");
    tree_init(iny, "      ");
    o << "      double D = " << dexpr() << ";\n";
    o << "      double acc = " << (outer.top().empty() ? std::string("D") : "D * " + outer.top()) << ";\n";
    o << "      for (uint32_t q = 0; q < " << Q << "u; ++q) {\n";
    const char* ind = "        ";
    // pair index j = B*q + s, s = 1 .. B-1: pair bit p = ctz(s) (walk bit p+1);
    // neg = (j >> (p+1)) & 1 = bit p+1 of s for p < b-1, bit 0 of q for p = b-1
    for (unsigned st = 1; st < B; ++st) {
      const int pb = __builtin_ctz(st);
      if (pb < b - 1) {
        step(pb + 1, off_const(pb + 1, (st >> (pb + 1)) & 1u), ind);
      } else {
        o << ind << "{\n" << ind << "  const uint32_t ng = q & 1u;\n";
        step(pb + 1, off_dyn(pb + 1, "ng"), "          ");
        o << ind << "}\n";
      }
      accumulate(st & 1u, ind);
    }
    if (Q > 1) {
      // j = B(q+1): pair bit b + ctz(q+1) (walk bit b+1+ctz(q+1)), neg =
      // ((q+1) >> (ctz(q+1)+1)) & 1.  One straight-line step for all of them
      // (no per-bit branches): the full signed column is added to every row
      // some walk bit > b touches (zeros elsewhere) and every segment such a
      // row lies in is re-multiplied.
      o << ind << "if (q + 1u < " << Q << "u) {\n";
      o << ind << "  const uint32_t kk = (uint32_t)__builtin_ctz(q + 1u);\n";
      o << ind << "  const uint32_t ng = ((q + 1u) >> (kk + 1u)) & 1u;\n";
      o << ind << "  cjdbl8* cv = (cjdbl8*)opaque_c(p.cols, (2u * (" << (L + b + 1) << "u + kk) + ng) * "
        << P.NP * 8 << "u);\n";
      adds(P.dyn_rows, true, ind);
      products(P.seg_b, ind);
      accumulate(false, "          ");
      o << ind << "}\n";
    }
    o << "      }\n";
    o << "      if (((uint32_t)ga ^ lane_par) & 1u) acc = -acc;\n";
    o << "      const double part = wave_sum(lane_valid ? acc : 0.0);\n";
    o << "      keep = (lane == j) ? part : keep;\n";
    o << "    }\n";
    o << "    const uint64_t a = (uint64_t)g * p.group + lane;\n";
    o << "    if (lane < (uint32_t)p.group && a < p.chunk_count) p.chunk_out[a] = keep;\n";
    o << "  }\n";
    o << "}\n";
    o << "}  // namespace sup\n";
    return o.str();
  }
};

const char* const kJitOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off"};
constexpr int kJitNopts = 4;

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

}  // namespace

int build_seg(Plan& P) {
  const int n = P.n, L = P.lay.L, m = P.lay.m;
  if (m < 3) {
    set_error("segmented walk needs >= 3 walk bits");
    return SUP_EINVAL;
  }
  if (P.cols.empty()) return SUP_EINVAL;
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
  P.seg_b = seg_static_bits(m);
  P.dyn_rows.clear();
  {
    std::vector<char> in(n, 0);
    for (int k = P.seg_b + 1; k < m; ++k)
      for (int r : P.touched[k]) in[r] = 1;
    for (int j = 0; j < n; ++j)
      if (in[j]) P.dyn_rows.push_back(j);
  }
  {  // product trees: rows outside segment 0 and segment 0's rows, by step class
    std::vector<uint32_t> rsig(n, 0u);
    for (int k = 1; k < m; ++k)
      for (int r : P.touched[k]) rsig[r] |= 1u << step_class(k, P.seg_b);
    const int len0 = P.seg_start[1];
    P.outer_tree = make_tree(rsig, len0, P.seg_start.back(), n, P.seg_b);
    P.inner_tree = make_tree(rsig, 0, P.sub_start.back(), len0, P.seg_b);
  }
  P.jofs.assign(m, 0);
  P.jtab.clear();
  for (int k = 0; k < m; ++k) {
    const std::vector<int>& t = P.touched[k];
    const size_t blk = (t.size() + 7) & ~(size_t)7;
    P.jofs[k] = (int)P.jtab.size();
    P.jtab.resize(P.jtab.size() + 2 * std::max<size_t>(blk, 8), 0.0);
    for (size_t i = 0; i < t.size(); ++i) {
      P.jtab[P.jofs[k] + i] = P.cols[(size_t)(2 * (L + k)) * P.NP + t[i]];
      P.jtab[P.jofs[k] + blk + i] = P.cols[(size_t)(2 * (L + k) + 1) * P.NP + t[i]];
    }
  }
  Gen g(P);
  P.jit_src = g.source();
  std::string key = P.jit_src;
  for (int i = 0; i < kJitNopts; ++i) key += std::string("\n//") + kJitOpts[i];
  key += std::string("\n//") + kWalkCommonSrc + kWalkParamsSrc;
  P.jit_key = fnv1a(key);
  return SUP_OK;
}

// ------------------------------------------------------ compile and cache --
namespace {

std::mutex g_jit_mu;
std::map<uint64_t, std::shared_ptr<std::vector<char>>> g_code;        // key -> code object
std::map<std::pair<int, uint64_t>, hipFunction_t> g_fn;               // (device, key) -> kernel
std::map<std::pair<int, uint64_t>, int> g_occ;
double g_compile_ms = 0.0;

std::string cache_dir() {
  const char* e = std::getenv("SUP_JIT_CACHE_DIR");
  if (e) return e;  // "" disables
  if (const char* x = std::getenv("XDG_CACHE_HOME")) return std::string(x) + "/superman_amd";
  if (const char* h = std::getenv("HOME")) return std::string(h) + "/.cache/superman_amd";
  return "";
}

std::string key_hex(uint64_t k) {
  char b[32];
  std::snprintf(b, sizeof b, "%016llx", (unsigned long long)k);
  return b;
}

bool read_file(const std::string& path, std::vector<char>& out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(sz > 0 ? (size_t)sz : 0);
  const bool ok = sz > 0 && std::fread(out.data(), 1, out.size(), f) == out.size();
  std::fclose(f);
  return ok;
}

void write_file_atomic(const std::string& dir, const std::string& name, const std::vector<char>& data) {
  std::string cur;
  for (size_t i = 1; i <= dir.size(); ++i)  // mkdir -p
    if (i == dir.size() || dir[i] == '/') {
      cur = dir.substr(0, i);
      ::mkdir(cur.c_str(), 0755);
    }
  const std::string tmp = dir + "/." + name + "." + std::to_string(::getpid());
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;  // cache is best effort
  const bool ok = std::fwrite(data.data(), 1, data.size(), f) == data.size();
  std::fclose(f);
  if (ok) std::rename(tmp.c_str(), (dir + "/" + name).c_str());
  else std::remove(tmp.c_str());
}

int compile(const Plan& P, std::shared_ptr<std::vector<char>>& code) {
  auto it = g_code.find(P.jit_key);
  if (it != g_code.end()) {
    code = it->second;
    return SUP_OK;
  }
  const std::string dir = cache_dir();
  const std::string name = "seg_" + key_hex(P.jit_key) + ".co";
  auto co = std::make_shared<std::vector<char>>();
  if (!dir.empty() && read_file(dir + "/" + name, *co)) {
    g_code[P.jit_key] = co;
    code = co;
    return SUP_OK;
  }
  if (const char* d = std::getenv("SUP_JIT_DUMP")) {  // debugging: keep the generated source
    FILE* f = std::fopen((std::string(d) + "/seg_" + key_hex(P.jit_key) + ".hip").c_str(), "w");
    if (f) std::fputs(P.jit_src.c_str(), f), std::fclose(f);
  }
  auto t0 = std::chrono::steady_clock::now();
  hiprtcProgram prog;
  const char* hdr[] = {kWalkCommonSrc, kWalkParamsSrc};
  const char* names[] = {"walk_common.hpp", "walk_params.hpp"};
  if (hiprtcCreateProgram(&prog, P.jit_src.c_str(), "sup_walk_seg.hip", 2, hdr, names) != HIPRTC_SUCCESS) {
    set_error("hiprtcCreateProgram failed");
    return SUP_EHIP;
  }
  const hiprtcResult cr = hiprtcCompileProgram(prog, kJitNopts, kJitOpts);
  if (cr != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    set_error(std::string("hiprtc compile of the segmented walk failed: ") + hiprtcGetErrorString(cr) + "\n" +
              log.substr(0, 2000));
    return SUP_EHIP;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  co->resize(cs);
  hiprtcGetCode(prog, co->data());
  hiprtcDestroyProgram(&prog);
  g_compile_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (!dir.empty()) write_file_atomic(dir, name, *co);
  g_code[P.jit_key] = co;
  code = co;
  return SUP_OK;
}

int resolve(int dev, const Plan& P, hipFunction_t* fn) {
  if (P.kind != kWalkSeg || P.jit_src.empty()) {
    set_error("plan has no segmented-walk kernel");
    return SUP_EINVAL;
  }
  std::lock_guard<std::mutex> g(g_jit_mu);
  auto k = std::make_pair(dev, P.jit_key);
  auto it = g_fn.find(k);
  if (it != g_fn.end()) {
    *fn = it->second;
    return SUP_OK;
  }
  std::shared_ptr<std::vector<char>> code;
  int rc = compile(P, code);
  if (rc) return rc;
  hipModule_t mod;
  hipError_t e = hipModuleLoadData(&mod, code->data());
  if (e != hipSuccess) {
    set_error(std::string("hipModuleLoadData (segmented walk): ") + hipGetErrorString(e));
    return SUP_EHIP;
  }
  if ((e = hipModuleGetFunction(fn, mod, "sup_walk_seg")) != hipSuccess) {
    set_error(std::string("hipModuleGetFunction (segmented walk): ") + hipGetErrorString(e));
    return SUP_EHIP;
  }
  g_fn[k] = *fn;  // modules live for the process (one per pattern and device)
  return SUP_OK;
}

}  // namespace

int jit_compile_only(const Plan& P, double* compile_ms) {
  if (P.kind != kWalkSeg || P.jit_src.empty()) {
    set_error("plan has no segmented-walk kernel");
    return SUP_EINVAL;
  }
  const double before = jit_compile_ms_total();
  std::shared_ptr<std::vector<char>> code;
  int rc;
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    rc = compile(P, code);
  }
  if (compile_ms) *compile_ms = jit_compile_ms_total() - before;
  return rc;
}

int jit_occupancy(int dev, const Plan& P, int* blocks_per_cu, double* compile_ms) {
  const double before = jit_compile_ms_total();
  hipFunction_t fn;
  int rc = resolve(dev, P, &fn);
  if (rc) return rc;
  if (compile_ms) *compile_ms = jit_compile_ms_total() - before;
  std::lock_guard<std::mutex> g(g_jit_mu);
  auto k = std::make_pair(dev, P.jit_key);
  auto it = g_occ.find(k);
  if (it != g_occ.end()) {
    *blocks_per_cu = it->second;
    return SUP_OK;
  }
  int b = 0;
  hipError_t e = hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&b, fn, kBlock, 0);
  if (e != hipSuccess) {
    set_error(std::string("occupancy query (segmented walk): ") + hipGetErrorString(e));
    return SUP_EHIP;
  }
  g_occ[k] = b > 0 ? b : 1;
  *blocks_per_cu = g_occ[k];
  return SUP_OK;
}

int jit_launch(int dev, const Plan& P, const WalkParams& p, int grid, hipStream_t s) {
  hipFunction_t fn;
  int rc = resolve(dev, P, &fn);
  if (rc) return rc;
  WalkParams arg = p;
  void* args[] = {&arg};
  hipError_t e = hipModuleLaunchKernel(fn, (unsigned)grid, 1, 1, kBlock, 1, 1, 0, s, args, nullptr);
  if (e != hipSuccess) {
    set_error(std::string("hipModuleLaunchKernel (segmented walk): ") + hipGetErrorString(e));
    return SUP_EHIP;
  }
  return SUP_OK;
}

double jit_compile_ms_total() {
  std::lock_guard<std::mutex> g(g_jit_mu);
  return g_compile_ms;
}

}  // namespace sup
