// exact.cpp — exact permanent of an integer matrix (sup_perman_exact).
//
// The reference computes the permanent of int and -b (binary) inputs in fp64
// (gpu_exact_dense.cu:329-399 with T = int; parallel_perman64,
// rev/cpu_algos.hpp:761-873), so beyond 2^53 its result is rounded.  Here the
// same Ryser / Gray-code sum is evaluated exactly:
//   * the walk runs on 2A, whose row values X_j = 2 x_j are integers with
//     |X_j| <= rowabs_j, exact in fp64 (walk_exact.hip, host twin
//     cpu_exact_range);
//   * each term prod_j X_j is reduced modulo k primes p < 2^42 (exact fp64
//     residue arithmetic), summed with its Gray sign;
//   * the residues of T = sum_i (-1)^i prod_j X_j(gray(i)) are joined by CRT
//     (Garner) into the exact integer T, |T| <= 2^(n-1) prod_j rowabs_j <
//     (prod p) / 2, and perm = (4(n&1) - 2) T / 2^n.  T must be divisible by
//     2^(n-1): that is checked, a free self-test of the whole computation.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <atomic>
#include <mutex>
#include <thread>

#include "engine.hpp"

namespace sup {
namespace {

typedef unsigned __int128 u128;

uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)((u128)a * b % m); }
uint64_t powmod(uint64_t a, uint64_t e, uint64_t m) {
  uint64_t r = 1 % m;
  for (a %= m; e; e >>= 1, a = mulmod(a, a, m))
    if (e & 1) r = mulmod(r, a, m);
  return r;
}
// deterministic Miller-Rabin for n < 3.3e24
bool is_prime(uint64_t n) {
  if (n < 2) return false;
  for (uint64_t p : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull})
    if (n % p == 0) return n == p;
  uint64_t d = n - 1;
  int s = 0;
  while (!(d & 1)) d >>= 1, ++s;
  for (uint64_t a : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull}) {
    uint64_t x = powmod(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool comp = true;
    for (int i = 1; i < s && comp; ++i) {
      x = mulmod(x, x, n);
      if (x == n - 1) comp = false;
    }
    if (comp) return false;
  }
  return true;
}

// Unsigned big integer, 32-bit limbs, little-endian.
struct Big {
  std::vector<uint32_t> d;
  bool zero() const { return d.empty(); }
  void trim() {
    while (!d.empty() && d.back() == 0) d.pop_back();
  }
  void mul_add(uint64_t m, uint64_t a) {  // *this = *this * m + a
    u128 carry = a;
    for (auto& limb : d) {
      const u128 v = (u128)limb * m + carry;
      limb = (uint32_t)v;
      carry = v >> 32;
    }
    while (carry) d.push_back((uint32_t)carry), carry >>= 32;
    trim();
  }
  void add(const Big& o) {  // *this += o
    u128 carry = 0;
    if (d.size() < o.d.size()) d.resize(o.d.size(), 0u);
    for (size_t i = 0; i < d.size(); ++i) {
      const u128 v = (u128)d[i] + (i < o.d.size() ? o.d[i] : 0u) + carry;
      d[i] = (uint32_t)v;
      carry = v >> 32;
    }
    if (carry) d.push_back((uint32_t)carry);
    trim();
  }
  static Big from_dec(const std::string& s) {
    Big b;
    for (char c : s)
      if (c >= '0' && c <= '9') b.mul_add(10, (uint64_t)(c - '0'));
    return b;
  }
  int cmp(const Big& o) const {
    if (d.size() != o.d.size()) return d.size() < o.d.size() ? -1 : 1;
    for (size_t i = d.size(); i-- > 0;)
      if (d[i] != o.d[i]) return d[i] < o.d[i] ? -1 : 1;
    return 0;
  }
  void sub(const Big& o) {  // *this -= o, requires *this >= o
    int64_t borrow = 0;
    for (size_t i = 0; i < d.size(); ++i) {
      int64_t v = (int64_t)d[i] - borrow - (i < o.d.size() ? (int64_t)o.d[i] : 0);
      borrow = v < 0;
      d[i] = (uint32_t)(v + (borrow << 32));
    }
    trim();
  }
  uint32_t divmod(uint32_t m) {  // *this /= m, returns the remainder
    uint64_t r = 0;
    for (size_t i = d.size(); i-- > 0;) {
      const uint64_t v = (r << 32) | d[i];
      d[i] = (uint32_t)(v / m);
      r = v % m;
    }
    trim();
    return (uint32_t)r;
  }
  bool low_bits_zero(int k) const {  // *this divisible by 2^k
    for (int i = 0; i < k; ++i)
      if (i / 32 < (int)d.size() && ((d[i / 32] >> (i % 32)) & 1u)) return false;
    return true;
  }
  void shr(int k) {
    const int w = k / 32, b = k % 32;
    if (w >= (int)d.size()) {
      d.clear();
      return;
    }
    d.erase(d.begin(), d.begin() + w);
    if (b) {
      for (size_t i = 0; i < d.size(); ++i) d[i] = (d[i] >> b) | (i + 1 < d.size() ? d[i + 1] << (32 - b) : 0u);
    }
    trim();
  }
  std::string dec() const {
    if (d.empty()) return "0";
    Big t = *this;
    std::string s;
    while (!t.zero()) {
      uint32_t r = t.divmod(1000000000u);
      for (int i = 0; i < 9; ++i) s.push_back((char)('0' + r % 10)), r /= 10;
    }
    while (s.size() > 1 && s.back() == '0') s.pop_back();
    std::reverse(s.begin(), s.end());
    return s;
  }
};

}  // namespace

int exact_perman(const double* A, int n, const sup_opts& o, bool on_cpu, std::string& out, double* kernel_ms,
                 int* devices_used, int* cpu_items) {
  // integrality and size
  double maxrow = 0.0, logT = n - 1;
  for (int j = 0; j < n; ++j) {
    double ra = 0.0;
    for (int c = 0; c < n; ++c) {
      const double v = A[(size_t)j * n + c];
      if (v != std::floor(v) || std::fabs(v) >= 2147483648.0) {
        set_error("sup_perman_exact: entries must be integers with |a| < 2^31");
        return SUP_EINVAL;
      }
      ra += std::fabs(v);
    }
    if (ra == 0.0) {  // a zero row: the permanent is 0
      out = "0";
      if (kernel_ms) *kernel_ms = 0.0;
      if (devices_used) *devices_used = 0;
      if (cpu_items) *cpu_items = 0;
      return SUP_OK;
    }
    maxrow = std::max(maxrow, ra);
    logT += std::log2(ra);
  }
  // |X_j| <= maxrow.  The GPU multiplies rows in exact groups of G (|y| <=
  // maxrow^G < 2^(G xbits)) before the residue chain, whose |r| < 1.5 p, so
  // 1.5 p 2^(G xbits) < 2^53 keeps every product exact; p < 2^42 also bounds
  // the 256-step accumulation (< 2^51).  G trades shared group products
  // (n (1 - 1/G) per step) against chain length (4 n / G per prime) and
  // smaller primes (more of them).
  const int xbits = (int)std::ceil(std::log2(maxrow + 1.0));
  int group = 0, pbits = 0;
  double best = 1e300;
  for (int G : {1, 2, 4}) {
    const int pb = std::min(42, 52 - G * xbits - 1);
    if (pb < 20) continue;
    const double primes_needed = std::ceil((logT + 3.0) / (pb - 0.5));
    const double ops = n * (1.0 - 1.0 / G) + primes_needed * (4.0 * std::ceil((double)n / G) + 3.0);
    if (ops < best) best = ops, group = G, pbits = pb;
  }
  if (group == 0) {
    set_error("sup_perman_exact: row sums of |a| must stay below 2^31 for the residue walk");
    return SUP_EUNSUPPORTED;
  }
  // primes: the largest below 2^pbits, until their product exceeds 2 |T| (+ margin)
  std::vector<double> primes;
  double bits = 0.0;
  for (uint64_t c = (1ull << pbits) - 1; bits < logT + 2.0 + 1.0; c -= 2)
    if (is_prime(c)) primes.push_back((double)c), bits += std::log2((double)c);
  const int np = (int)primes.size();

  Plan P;
  std::vector<double> A2((size_t)n * n);
  for (size_t i = 0; i < A2.size(); ++i) A2[i] = 2.0 * A[i];
  // The prefix-blocked walk (walk_exact_blocked: rows in first-touch order,
  // only the flipped column's leading 8-row blocks re-formed) when its cost
  // model beats the dense walk's, as plan_for decides for the fp64 walks;
  // else the dense walk with its walk + lane columns in the greedy prefix
  // order.  Either way the rows no walk or lane column touches end the chunks
  // where they are exactly zero (walk_exact.hip), and any column order gives
  // the same exact sum.
  const Layout lay = default_layout(n);
  int rc = SUP_OK;
  if (lay.m > 0 && (rc = make_plan(A2.data(), n, kWalkSparse, false, lay, P)) == SUP_OK &&
      walk_cost(P) < 2.0 * n + 1.0 && (rc = improve_sparse_plan(A2.data(), n, lay, P)) == SUP_OK) {
    group |= 8;  // run_range_exact / walk_exact.hip: the blocked kernel
  } else {
    SegChoice order;
    order.order = greedy_walk_order(A2.data(), n, lay.m + lay.L);
    rc = make_plan(A2.data(), n, kWalkDense, false, lay, P, lay.m > 0 ? &order : nullptr);
  }
  if (rc) return rc;
  const uint64_t C = P.lay.chunks();

  // residues of T, per prime.  One device: its whole range, kMaxPrimes per
  // launch.  Several devices, or the CPU worker (-c with -g): a queue of
  // power-of-two items of wave-chunks (o.chunk_log2, else ~16 per taker) that
  // one host thread per device, and the CPU worker on o.threads host threads,
  // take in turn (as the fp64 -p6 queue, gpu_exact_dense.cu:776-904).  Residue
  // sums are exact, so who took which item never changes the result.
  std::vector<uint64_t> res(np, 0);
  double kms = 0.0;
  int used = 0, cpu_done = 0;
  if (on_cpu) {
    cpu_exact_range(P, 0, C, primes, std::max(o.threads, 1), res);
  } else {
    int ndev = 0;
    if ((rc = device_count(&ndev))) return rc;
    if (o.device_id < 0 || o.device_id >= ndev) {
      set_error("sup_perman_exact: device_id out of range");
      return SUP_EINVAL;
    }
    const int G = std::max(1, std::min(o.gpu_num, ndev - o.device_id));
    const bool cpu = o.cpu_worker != 0;
    const int takers = G + (cpu ? 1 : 0);
    uint64_t item = C;
    if (takers > 1) {
      if (o.chunk_log2 > 0) {
        item = std::min<uint64_t>(C, 1ull << std::min(o.chunk_log2, 62));
      } else {
        item = 1;
        while (item * 2 <= C && C / (item * 2) >= (uint64_t)takers * 16) item <<= 1;
      }
    }
    const uint64_t nitems = (C + item - 1) / item;
    std::vector<std::vector<uint64_t>> dres(takers, std::vector<uint64_t>(np, 0));
    std::vector<double> dms(takers, 0.0);
    std::vector<int> dtook(takers, 0);
    auto add = [&](int g, const std::vector<uint64_t>& r, int q0) {
      for (size_t i = 0; i < r.size(); ++i) dres[g][q0 + i] = (dres[g][q0 + i] + r[i]) % (uint64_t)primes[q0 + i];
    };
    auto take = [&](int g, uint64_t it) -> int {
      const uint64_t a = it * item, b = std::min(C, a + item);
      if (g == G) {  // the CPU worker: every prime in one pass
        std::vector<uint64_t> r;
        cpu_exact_range(P, a, b, primes, std::max(o.threads, 1), r);
        add(g, r, 0);
      } else {
        for (int q0 = 0; q0 < np; q0 += kMaxPrimes) {
          const std::vector<double> pr(primes.begin() + q0, primes.begin() + std::min(np, q0 + kMaxPrimes));
          std::vector<uint64_t> r;
          double ms = 0.0;
          const int e = run_range_exact(o.device_id + g, P, group, a, b, pr, r, &ms);
          if (e) return e;
          add(g, r, q0);
          dms[g] += ms;
        }
      }
      ++dtook[g];
      return SUP_OK;
    };
    if ((rc = run_item_queue(nitems, takers, take))) return rc;
    for (int q = 0; q < np; ++q)
      for (int g = 0; g < takers; ++g) res[q] = (res[q] + dres[g][q]) % (uint64_t)primes[q];
    kms = *std::max_element(dms.begin(), dms.begin() + G);
    used = G;
    cpu_done = cpu ? dtook[G] : 0;
  }

  // Garner: mixed-radix digits v_i, then T = sum v_i prod_{j<i} p_j in [0, M)
  std::vector<uint64_t> p(np), v(np);
  for (int i = 0; i < np; ++i) p[i] = (uint64_t)primes[i];
  for (int i = 0; i < np; ++i) {
    uint64_t x = res[i] % p[i], prod = 1 % p[i], acc = 0;  // acc = value of digits < i mod p_i
    for (int j = 0; j < i; ++j) {
      acc = (acc + mulmod(v[j] % p[i], prod, p[i])) % p[i];
      prod = mulmod(prod, p[j] % p[i], p[i]);
    }
    const uint64_t diff = (x + p[i] - acc) % p[i];
    v[i] = mulmod(diff, powmod(prod, p[i] - 2, p[i]), p[i]);
  }
  // Horner: T = (...(v_{k-1} p_{k-2} + v_{k-2}) p_{k-3} + ...) p_0 + v_0
  Big T, M, half;
  T.mul_add(1, v[np - 1]);
  for (int i = np - 2; i >= 0; --i) T.mul_add(p[i], v[i]);
  M.d.assign(1, 1u);
  for (int i = 0; i < np; ++i) M.mul_add(p[i], 0);
  // signed: T > M/2 stands for T - M
  half = M;
  half.divmod(2);
  bool neg = false;
  if (T.cmp(half) > 0) {
    Big t = M;
    t.sub(T);
    T = t;
    neg = true;
  }
  // perm = (4(n&1) - 2) T / 2^n = (n odd ? 1 : -1) T / 2^(n-1)
  if (!T.low_bits_zero(n - 1)) {
    set_error("sup_perman_exact: self-check failed (T not divisible by 2^(n-1))");
    return SUP_EHIP;
  }
  T.shr(n - 1);
  if (!(n & 1)) neg = !neg;
  out = (neg && !T.zero() ? "-" : "") + T.dec();
  if (kernel_ms) *kernel_ms = kms;
  if (devices_used) *devices_used = used;
  if (cpu_items) *cpu_items = cpu_done;
  return SUP_OK;
}

// -o reductions with exact leaves: without scaling the d1/d2/d34 tree folds
// every coefficient into its leaf matrices (integers stay integers), so
// perm(A) = sum of the leaf permanents; each leaf is computed exactly and the
// sum is a big integer (the fp64 combine of the same tree loses every digit on
// chesapeake).
namespace {
struct ReducedExact {
  const sup_opts* o;
  bool on_cpu;
  Big pos, neg;
  double kms = 0.0;
};
}  // namespace

int exact_perman_reduced(const double* A, int n, const sup_opts& o, bool on_cpu, const sup_reduce_opts& r,
                         std::string& out, double* kernel_ms, int* leaves) {
  if (r.scale_threshold > 0.0) {
    set_error("sup_perman_reduced_exact: scaling (-u) is not exact");
    return SUP_EUNSUPPORTED;
  }
  ReducedExact R;
  R.o = &o;
  R.on_cpu = on_cpu;
  sup_reduce_opts rr = r;
  rr.compress = 1;
  double approx = 0.0;
  int nl = 0;
  // GPU leaves several at a time, each worker on its own context lane (as
  // sup_perman_reduced); the exact sum does not depend on the order
  std::mutex mu;
  const char* lw = std::getenv("SUP_LEAF_WORKERS");
  const int workers = on_cpu ? 1 : lw ? std::max(1, std::min(kCtxLanes, std::atoi(lw))) : kCtxLanes;
  const int rc = decompose_batched(A, n, rr, workers, [&](int w, const double* a, int k, double* v) {
    set_ctx_lane(w);
    std::string s;
    double kms = 0.0;
    int used = 0;
    const int e = exact_perman(a, k, *R.o, R.on_cpu, s, &kms, &used);
    if (e) return e;
    const bool negative = !s.empty() && s[0] == '-';
    Big b = Big::from_dec(s);
    *v = std::strtod(s.c_str(), nullptr);
    std::lock_guard<std::mutex> g(mu);
    R.kms += kms;
    (negative ? R.neg : R.pos).add(b);
    return SUP_OK;
  }, &approx, &nl, false);  // every leaf (repeats included) adds its exact value
  if (rc) return rc;
  if (R.pos.cmp(R.neg) >= 0) {
    R.pos.sub(R.neg);
    out = R.pos.dec();
  } else {
    R.neg.sub(R.pos);
    out = "-" + R.neg.dec();
  }
  if (kernel_ms) *kernel_ms = R.kms;
  if (leaves) *leaves = nl;
  return SUP_OK;
}

}  // namespace sup
