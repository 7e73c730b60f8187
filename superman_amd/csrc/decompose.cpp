// decompose.cpp — matrix reductions in front of the Gray-code engine: degree-1/2
// compression, the d1/d2/d34 expansion recursion and the scaling wrapper.
//
// Replaces the reference's v2 host driver (revised_perman/main.cpp:993-1264:
// compress_and_calculate_recursive, compress_singleton_and_then_recurse,
// scale_and_calculate) and its helpers (revised_perman/util.h:1138-1407
// getRowNnz/getColNnz/checkEmpty/getMinNnz/d1compress/d2compress/d34compress,
// util.h:1445-1593 scalesk/scaleMatrix).  Each leaf is one exact permanent
// computed by a caller-supplied function (the GPU engine in
// sup_perman_reduced, anything in tests); the tree is combined on the host in
// the reference's order (left child + right child, scale factors divided out
// column vector first, then row vector).
//
// Deliberate differences from the reference (HISTORY.md §7):
//   * the nonzero test is != 0 (the reference's getRowNnz uses > 0 and skips
//     negative entries), as everywhere else in this engine;
//   * all reductions run in fp64 (the reference runs them in the storage type:
//     int for integer / pattern files — identical while values stay below
//     2^53);
//   * every leaf is preprocessed (-r) and scaled from its own entries (the
//     reference hands the first d34 child its parent's stale CSR/CSC,
//     main.cpp:1036-1045, and reorders intermediate matrices in place);
//   * an empty row/column after singleton removal returns 0 (the reference
//     prints "Perman is 0" and exits, main.cpp:1089-1093).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <type_traits>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "dd.hpp"
#include "engine.hpp"

namespace sup {
namespace {

struct Mat {
  int n = 0;
  std::vector<double> a;  // row-major n x n
  double& at(int i, int j) { return a[(size_t)i * n + j]; }
  double at(int i, int j) const { return a[(size_t)i * n + j]; }
};

int row_nnz(const Mat& m, int i) {  // util.h:1138-1149 (!= 0)
  int c = 0;
  for (int j = 0; j < m.n; ++j) c += m.at(i, j) != 0.0;
  return c;
}
int col_nnz(const Mat& m, int j) {  // util.h:1151-1162 (!= 0)
  int c = 0;
  for (int i = 0; i < m.n; ++i) c += m.at(i, j) != 0.0;
  return c;
}
bool has_empty(const Mat& m) {  // util.h:1164-1178 checkEmpty
  for (int i = 0; i < m.n; ++i)
    if (row_nnz(m, i) == 0 || col_nnz(m, i) == 0) return true;
  return false;
}
int min_deg(const Mat& m) {  // util.h:1180-1197 getMinNnz
  int d = m.n;
  for (int i = 0; i < m.n; ++i) d = std::min(d, std::min(row_nnz(m, i), col_nnz(m, i)));
  return d;
}

// Remove row r and column c.
Mat minor_of(const Mat& m, int r, int c) {
  Mat o;
  o.n = m.n - 1;
  o.a.resize((size_t)o.n * o.n);
  for (int i = 0, ii = 0; i < m.n; ++i) {
    if (i == r) continue;
    for (int j = 0, jj = 0; j < m.n; ++j) {
      if (j == c) continue;
      o.at(ii, jj++) = m.at(i, j);
    }
    ++ii;
  }
  return o;
}

// util.h:1199-1249 d1compress: the LAST degree-1 row (else the last degree-1
// column) is expanded: perm(A) = v * perm(A - row - col); v is folded into
// the first row of the minor.
bool d1(Mat& m) {
  int r = -1, c = -1;
  for (int i = 0; i < m.n; ++i) {
    if (row_nnz(m, i) == 1) r = i;
    if (col_nnz(m, i) == 1) c = i;
  }
  if (r < 0 && c < 0) return false;
  double v = 0.0;
  if (r >= 0) {
    for (int j = 0; j < m.n; ++j)
      if (m.at(r, j) != 0.0) {
        v = m.at(r, j);
        c = j;
        break;
      }
  } else {
    for (int i = 0; i < m.n; ++i)
      if (m.at(i, c) != 0.0) {
        v = m.at(i, c);
        r = i;
        break;
      }
  }
  m = minor_of(m, r, c);
  for (int j = 0; j < m.n; ++j) m.at(0, j) *= v;
  return true;
}

// util.h:1251-1319 d2compress: the first index i whose row (preferred) or
// column has two nonzeros k1 < k2.  Row case: drop the row and column k2,
// column k1 := a[r][k2]*A[:,k1] + a[r][k1]*A[:,k2] (perm is linear in a column).
bool d2(Mat& m) {
  int r = -1, c = -1;
  for (int i = 0; i < m.n; ++i) {
    if (row_nnz(m, i) == 2) r = i;
    if (col_nnz(m, i) == 2) c = i;
    if (r >= 0 || c >= 0) break;
  }
  if (r < 0 && c < 0) return false;
  int k1 = -1, k2 = -1;
  for (int j = 0; j < m.n; ++j) {
    const double v = (r >= 0) ? m.at(r, j) : m.at(j, c);
    if (v != 0.0) {
      if (k1 < 0) {
        k1 = j;
      } else {
        k2 = j;
        break;
      }
    }
  }
  Mat o;
  if (r >= 0) {
    o = minor_of(m, r, k2);
    const int jj = k1;  // k1 < k2: its index survives
    for (int i = 0, ii = 0; i < m.n; ++i) {
      if (i == r) continue;
      o.at(ii++, jj) = (m.at(i, k1) * m.at(r, k2)) + (m.at(i, k2) * m.at(r, k1));
    }
  } else {
    o = minor_of(m, k2, c);
    const int ii = k1;
    for (int j = 0, jj = 0; j < m.n; ++j) {
      if (j == c) continue;
      o.at(ii, jj++) = (m.at(k1, j) * m.at(k2, c)) + (m.at(k2, j) * m.at(k1, c));
    }
  }
  m = std::move(o);
  return true;
}

// util.h:1321-1407 d34compress: a row (or, transposed, a column) of degree
// 3 or 4 is split into two pairs {n0,n1}, {n2,n3} (n3 = the last zero column
// for degree 3), each merged as in d2: perm(A) = perm(m) + perm(m2).
void d34(Mat& m, Mat& m2, int deg) {
  int r = -1, c = -1;
  for (int i = 0; i < m.n; ++i) {
    if (row_nnz(m, i) == deg) r = i;
    if (col_nnz(m, i) == deg) c = i;
    if (r >= 0 || c >= 0) break;
  }
  Mat t = m;
  if (r < 0) {  // transpose: perm(A) = perm(A^T)
    for (int i = 0; i < m.n; ++i)
      for (int j = 0; j < m.n; ++j) t.at(j, i) = m.at(i, j);
    r = c;
  }
  int nb[4] = {-1, -1, -1, -1}, idx = 0, zero = -1;
  for (int j = 0; j < t.n; ++j) {
    if (t.at(r, j) != 0.0) {
      if (idx < 4) nb[idx++] = j;
    } else {
      zero = j;
    }
  }
  if (nb[3] == -1) nb[3] = zero;
  auto merged = [&](int keep, int drop) {
    Mat o = minor_of(t, r, drop);
    const int jj = keep < drop ? keep : keep - 1;
    for (int i = 0, ii = 0; i < t.n; ++i) {
      if (i == r) continue;
      o.at(ii++, jj) = (t.at(r, keep) * t.at(i, drop)) + (t.at(r, drop) * t.at(i, keep));
    }
    return o;
  };
  m2 = merged(nb[2], nb[3]);
  m = merged(nb[0], nb[1]);
}

// util.h:1445-1567 scalesk: alternate column / row passes setting every
// column (row) sum of the scaled matrix to `thr` until the mean row and
// column sums are within 10 of it.  Sums in CSC (rows ascending) / CSR
// (columns ascending) order, product left to right as in the reference.
int scalesk(const Mat& m, double thr, std::vector<double>& rv, std::vector<double>& cv) {
  const int n = m.n;
  rv.assign(n, 1.0);
  cv.assign(n, 1.0);
  double max_error = 100.0;
  for (int it = 0; max_error > 10.0; ++it) {
    if (it == 1000) {
      set_error("scaling did not converge in 1000 passes");
      return SUP_EINVAL;
    }
    for (int j = 0; j < n; ++j) {
      if (col_nnz(m, j) == 0) continue;
      double sum = 0.0;
      for (int i = 0; i < n; ++i)
        if (m.at(i, j) != 0.0) sum += m.at(i, j) * cv[j] * rv[i];
      cv[j] = thr / sum;
    }
    for (int i = 0; i < n; ++i) {
      if (row_nnz(m, i) == 0) continue;
      double sum = 0.0;
      for (int j = 0; j < n; ++j)
        if (m.at(i, j) != 0.0) sum += m.at(i, j) * rv[i] * cv[j];
      rv[i] = thr / sum;
    }
    double colsum = 0.0, rowsum = 0.0;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i)
        if (m.at(i, j) != 0.0) colsum += m.at(i, j) * cv[j] * rv[i];
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        if (m.at(i, j) != 0.0) rowsum += m.at(i, j) * rv[i] * cv[j];
    max_error = std::max(std::fabs(thr - colsum / n), std::fabs(thr - rowsum / n));
  }
  return SUP_OK;
}

// util.h:1569-1593 scaleMatrix: rows by rv, then columns by cv.
Mat scaled(const Mat& m, const std::vector<double>& rv, const std::vector<double>& cv) {
  Mat o = m;
  for (int i = 0; i < m.n; ++i)
    for (int j = 0; j < m.n; ++j) o.at(i, j) *= rv[i];
  for (int j = 0; j < m.n; ++j)
    for (int i = 0; i < m.n; ++i) o.at(i, j) *= cv[j];
  return o;
}

// Leaf values and their combine: fp64 (sup_decompose's callback) or
// double-double (decompose_dd_batched: -o / -u with -q leaves).
struct DblOps {
  typedef double V;
  static V zero() { return 0.0; }
  static V add(V a, V b) { return a + b; }
  static V div(V a, double d) { return a / d; }
};
struct DdOps {
  typedef dd V;
  static V zero() { return dd{0.0, 0.0}; }
  static V add(V a, V b) { return dd_add(a, b); }
  static V div(V a, double d) { return dd_div_d(a, d); }
};

// Deferred combine (decompose_batched): the decomposition records the fold it
// would perform — zero, leaf i, a + b, a / d — as nodes in creation order, and
// hands each leaf matrix to a worker as soon as it appears; once every leaf
// value is in, the nodes are evaluated in creation order (children before
// parents), which is the recursive fold's order of fp64 operations on the same
// operands: the result equals DblOps's bit for bit.
struct ENode {
  int32_t op;  // 0 zero, 1 leaf a, 2 add(a, b), 3 div(a, d)
  int32_t a, b;
  double d;
};
struct ExprOps {
  typedef int32_t V;
  static thread_local std::vector<ENode>* T;
  static V push(const ENode& e) {
    T->push_back(e);
    return (V)(T->size() - 1);
  }
  static V zero() { return push({0, 0, 0, 0.0}); }
  static V add(V a, V b) { return push({2, a, b, 0.0}); }
  static V div(V a, double d) { return push({3, a, 0, d}); }
};
thread_local std::vector<ENode>* ExprOps::T = nullptr;

template <class Ops>
struct Decomposer {
  typedef typename Ops::V V;
  sup_reduce_opts r;
  std::function<int(const double*, int, V*)> fn;
  int leaves = 0;
  int rc = SUP_OK;

  V leaf(const Mat& m) {
    if (rc) return Ops::zero();
    if (m.n > SUP_MAX_N) {
      set_error("a leaf of order " + std::to_string(m.n) + " remains after the reductions (the engine takes n <= " +
                std::to_string(SUP_MAX_N) + "; try -o)");
      rc = SUP_EUNSUPPORTED;
      return Ops::zero();
    }
    ++leaves;
    V v = Ops::zero();
    const int e = fn(m.a.data(), m.n, &v);
    if (e) {
      rc = e;
      if (std::string(sup_last_error()).empty()) set_error("leaf permanent failed");
    }
    return v;
  }

  // main.cpp:1127-1259 scale_and_calculate: perm(A) = perm(D_r A D_c) / prod(cv) / prod(rv).
  V scale_then(const Mat& m, bool then_compress) {
    std::vector<double> rv, cv;
    if (rc) return Ops::zero();
    if ((rc = scalesk(m, r.scale_threshold, rv, cv))) return Ops::zero();
    Mat s = scaled(m, rv, cv);
    V v = then_compress ? singletons(s) : leaf(s);
    for (int i = 0; i < m.n; ++i) v = Ops::div(v, cv[i]);
    for (int i = 0; i < m.n; ++i) v = Ops::div(v, rv[i]);
    return v;
  }

  // main.cpp:993-1063 compress_and_calculate_recursive
  V recurse(Mat& m) {
    if (rc) return Ops::zero();
    const int md = min_deg(m);
    if (md < r.max_deg && m.n > r.min_n) {
      if (md == 0) return Ops::zero();  // an empty row or column
      if (md == 1) {
        d1(m);
        return recurse(m);
      }
      if (md == 2) {
        d2(m);
        return recurse(m);
      }
      Mat m2;
      d34(m, m2, md);
      const V left = recurse(m);
      return Ops::add(left, recurse(m2));
    }
    return r.scale_threshold > 0.0 ? scale_then(m, false) : leaf(m);
  }

  // main.cpp:1065-1100 compress_singleton_and_then_recurse
  V singletons(Mat& m) {
    bool comp = true;
    while (comp && m.n > 1) {
      comp = d1(m) || d2(m);
      if (comp && has_empty(m)) return Ops::zero();  // rank deficient: perm = 0
    }
    return recurse(m);
  }

  // the whole request: main.cpp:1640-1660 (-u scales the whole matrix first,
  // then -o compresses it and scales each leaf again; -o alone compresses;
  // neither = one leaf)
  V run(Mat& m) { return r.scale_threshold > 0.0 ? scale_then(m, r.compress != 0) : r.compress ? singletons(m) : leaf(m); }
};

// d34 splits a row of degree 3 or 4 (main.cpp:1007 hard-codes minDeg < 5), and
// needs a zero column and two surviving merges (order >= 5): larger max_deg
// would split a degree-5+ row on its first four nonzeros, a smaller min_n
// would recurse into n = 0 leaves
int check_reduce_opts(const sup_reduce_opts& r, const char* who) {
  if (r.max_deg < 1 || r.max_deg > 5 || r.min_n < 4) {
    set_error(std::string(who) + ": need 1 <= max_deg <= 5 and min_n >= 4 (got max_deg " + std::to_string(r.max_deg) +
              ", min_n " + std::to_string(r.min_n) + ")");
    return SUP_EINVAL;
  }
  return SUP_OK;
}

}  // namespace

namespace {
struct PairHash {
  size_t operator()(const std::pair<uint64_t, uint64_t>& p) const { return (size_t)(p.first ^ (p.second * 31)); }
};

// Two independent 64-bit hashes (FNV-1a, and a multiply-xorshift mix) of a
// leaf's order and entries' bit patterns.
std::pair<uint64_t, uint64_t> leaf_key(const double* a, int k) {
  uint64_t h1 = 1469598103934665603ull ^ (uint64_t)k, h2 = 0x9e3779b97f4a7c15ull * (uint64_t)(k + 1);
  for (size_t i = 0; i < (size_t)k * k; ++i) {
    uint64_t b;
    std::memcpy(&b, a + i, sizeof b);
    for (int s = 0; s < 64; s += 8) h1 = (h1 ^ ((b >> s) & 0xff)) * 1099511628211ull;
    h2 ^= b + 0x9e3779b97f4a7c15ull + (h2 << 6) + (h2 >> 2);
    h2 *= 0xff51afd7ed558ccdull;
    h2 ^= h2 >> 33;
  }
  return {h1, h2};
}

template <class Ops>
int batched(const double* A, int n, const sup_reduce_opts& r, int workers,
            const std::function<int(int, const double*, int, typename Ops::V*)>& leaf, typename Ops::V* out,
            int* n_leaves, const char* who, bool memo, int batch_max = 1,
            const std::function<int(int, const std::vector<const double*>&, int,
                                    const std::vector<typename Ops::V*>&)>* leaves = nullptr,
            const LeafBatchStagedFn* staged = nullptr) {
  typedef typename Ops::V V;
  set_error("");
  if (int rc = check_reduce_opts(r, who)) return rc;
  workers = std::max(1, workers);
  struct Job {
    std::vector<double> a;
    int n;
    V* slot;
  };
  std::mutex mu;
  std::condition_variable cv_put, cv_get;
  std::deque<Job> q;
  std::deque<V> vals;  // leaf values by leaf id (references stay valid as it grows)
  bool closed = false, failed = false;
  int frc = SUP_OK;
  std::string ferr;
  batch_max = leaves || staged ? std::max(1, batch_max) : 1;
  const size_t cap = (size_t)workers * 4 * (size_t)batch_max;
  // Two-stage batches (staged): each worker plans its batch on the host and
  // hands the device part to its own walker thread through a channel of
  // depth 2, so the next batch is planned while this one walks (one worker:
  // the GPU no longer idles while the host plans).  Batches of one worker walk
  // in the order it planned them; values land in their slots either way.
  struct Chan {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<int()>> q;
    bool closed = false;
  };
  std::vector<std::unique_ptr<Chan>> chans;
  std::vector<std::thread> walkers;
  auto fail = [&](int e) {
    std::lock_guard<std::mutex> lk(mu);
    if (!failed) failed = true, frc = e, ferr = sup_last_error();
    cv_put.notify_all();
  };
  if (staged) {
    for (int w = 0; w < workers; ++w) chans.emplace_back(new Chan);
    for (int w = 0; w < workers; ++w)
      walkers.emplace_back([&, w]() {
        Chan& ch = *chans[w];
        for (;;) {
          std::function<int()> job;
          {
            std::unique_lock<std::mutex> lk(ch.mu);
            ch.cv.wait(lk, [&] { return !ch.q.empty() || ch.closed; });
            if (ch.q.empty()) return;
            job = std::move(ch.q.front());
            ch.q.pop_front();
          }
          ch.cv.notify_all();
          bool skip;
          {
            std::lock_guard<std::mutex> lk(mu);
            skip = failed;
          }
          if (!skip)
            if (const int e = job()) fail(e);
        }
      });
  }
  auto work = [&](int w) {
    for (;;) {
      std::vector<Job> js;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_get.wait(lk, [&] { return !q.empty() || closed; });
        if (q.empty()) return;
        // up to batch_max queued leaves of the first one's order (no waiting for more)
        js.push_back(std::move(q.front()));
        q.pop_front();
        while ((int)js.size() < batch_max && !q.empty() && q.front().n == js[0].n) {
          js.push_back(std::move(q.front()));
          q.pop_front();
        }
      }
      cv_put.notify_all();
      {
        std::lock_guard<std::mutex> lk(mu);
        if (failed) continue;  // drain without computing
      }
      int e = SUP_OK;
      if (staged) {
        std::vector<const double*> mats;
        std::vector<V*> slots;
        for (const Job& j : js) mats.push_back(j.a.data()), slots.push_back(j.slot);
        std::function<int()> walk;
        if constexpr (std::is_same<V, double>::value) e = (*staged)(w, mats, js[0].n, slots, walk);
        if (!e) {
          Chan& ch = *chans[w];
          std::unique_lock<std::mutex> lk(ch.mu);
          ch.cv.wait(lk, [&] { return ch.q.size() < 2; });
          ch.q.push_back(std::move(walk));
          lk.unlock();
          ch.cv.notify_all();
        }
      } else if (leaves) {
        std::vector<const double*> mats;
        std::vector<V*> slots;
        for (const Job& j : js) mats.push_back(j.a.data()), slots.push_back(j.slot);
        e = (*leaves)(w, mats, js[0].n, slots);
      } else {
        e = leaf(w, js[0].a.data(), js[0].n, js[0].slot);
      }
      if (e) fail(e);
    }
  };
  std::vector<std::thread> th;
  for (int w = 0; w < workers; ++w) th.emplace_back(work, w);
  std::vector<ENode> nodes;
  ExprOps::T = &nodes;
  // A leaf equal to an earlier one (d34 expansions repeat matrices: 7 % of
  // dwt_59's 145,798 leaves, 26 % of chesapeake's 231) takes that leaf's value:
  // matrices are keyed by two independent 64-bit hashes of their bytes and order
  std::unordered_map<std::pair<uint64_t, uint64_t>, int32_t, PairHash> seen;
  Decomposer<ExprOps> d;
  d.r = r;
  d.fn = [&](const double* a, int k, int32_t* v) {
    const std::pair<uint64_t, uint64_t> key = leaf_key(a, k);
    const auto hit = memo ? seen.find(key) : seen.end();
    if (hit != seen.end()) {
      *v = ExprOps::push({1, hit->second, 0, 0.0});
      return SUP_OK;
    }
    std::unique_lock<std::mutex> lk(mu);
    cv_put.wait(lk, [&] { return q.size() < cap || failed; });
    if (failed) {
      set_error(ferr);
      return frc;
    }
    const int32_t id = (int32_t)vals.size();
    if (memo) seen.emplace(key, id);
    vals.push_back(Ops::zero());
    q.push_back(Job{std::vector<double>(a, a + (size_t)k * k), k, &vals.back()});
    lk.unlock();
    cv_get.notify_one();
    *v = ExprOps::push({1, id, 0, 0.0});
    return SUP_OK;
  };
  Mat m;
  m.n = n;
  m.a.assign(A, A + (size_t)n * n);
  const int32_t root = d.run(m);
  ExprOps::T = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu);
    closed = true;
  }
  cv_get.notify_all();
  for (auto& t : th) t.join();
  for (auto& ch : chans) {  // the planners are done: let the walkers drain their channels
    {
      std::lock_guard<std::mutex> lk(ch->mu);
      ch->closed = true;
    }
    ch->cv.notify_all();
  }
  for (auto& t : walkers) t.join();
  if (failed) {
    set_error(ferr);
    return frc;
  }
  if (d.rc) return d.rc;
  std::vector<V> val(nodes.size(), Ops::zero());
  for (size_t i = 0; i < nodes.size(); ++i) {
    const ENode& e = nodes[i];
    val[i] = e.op == 1 ? vals[e.a] : e.op == 2 ? Ops::add(val[e.a], val[e.b]) : e.op == 3 ? Ops::div(val[e.a], e.d)
                                                                                           : Ops::zero();
  }
  *out = val[root];
  if (n_leaves) *n_leaves = d.leaves;
  return SUP_OK;
}
}  // namespace

int decompose_batched(const double* A, int n, const sup_reduce_opts& r, int workers,
                      const std::function<int(int, const double*, int, double*)>& leaf, double* out, int* n_leaves,
                      bool memo) {
  return batched<DblOps>(A, n, r, workers, leaf, out, n_leaves, "sup_perman_reduced", memo);
}

int decompose_batched_staged(const double* A, int n, const sup_reduce_opts& r, int workers, int batch_max,
                             const LeafBatchStagedFn& staged, double* out, int* n_leaves) {
  const std::function<int(int, const double*, int, double*)> one = [&](int w, const double* a, int k, double* v) {
    std::function<int()> walk;
    const int e = staged(w, std::vector<const double*>{a}, k, std::vector<double*>{v}, walk);
    return e ? e : walk();
  };
  return batched<DblOps>(A, n, r, workers, one, out, n_leaves, "sup_perman_reduced", true, batch_max, nullptr,
                         &staged);
}

int decompose_dd_batched(const double* A, int n, const sup_reduce_opts& r, int workers,
                         const std::function<int(int, const double*, int, dd*)>& leaf, dd* out, int* n_leaves) {
  return batched<DdOps>(A, n, r, workers, leaf, out, n_leaves, "sup_perman_reduced_quad", true);
}

}  // namespace sup

using namespace sup;

extern "C" {

void sup_reduce_opts_init(sup_reduce_opts* r) {
  if (!r) return;
  r->compress = 0;
  r->scale_threshold = 0.0;
  r->min_n = 30;   // main.cpp:1007 (nov > 30)
  r->max_deg = 5;  // main.cpp:1007 (minDeg < 5)
  r->preprocessing = 0;
}

int sup_decompose(const void* mat, sup_dtype t, int n, const sup_reduce_opts* r_in, sup_leaf_fn fn, void* user,
                  double* out, int* n_leaves) {
  if (!mat || !fn || !out || n < 1 || n > SUP_MAX_READ_N) {
    set_error("sup_decompose: bad argument");
    return SUP_EINVAL;
  }
  set_error("");
  Decomposer<DblOps> d;
  if (r_in) d.r = *r_in;
  else sup_reduce_opts_init(&d.r);
  if (int rc = check_reduce_opts(d.r, "sup_decompose")) return rc;
  d.fn = [fn, user](const double* a, int k, double* v) { return fn(a, k, user, v); };
  Mat m;
  m.n = n;
  m.a.resize((size_t)n * n);
  for (size_t i = 0; i < m.a.size(); ++i)
    m.a[i] = t == SUP_INT32 ? (double)((const int32_t*)mat)[i]
             : t == SUP_FLOAT32 ? (double)((const float*)mat)[i] : ((const double*)mat)[i];
  const double v = d.run(m);
  if (d.rc) return d.rc;
  *out = v;
  if (n_leaves) *n_leaves = d.leaves;
  return SUP_OK;
}

}  // extern "C"
