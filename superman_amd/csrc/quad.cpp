// quad.cpp — the permanent in double-double (~106 bits): sup_perman_quad, the
// MI355X counterpart of the reference's quad-precision calculation
// (revised_perman/main.cpp:141-142 `-q`: parallel_perman64<__float128,S>,
// cpu_algos.hpp:761-873).
//
// Plan: the dense identity plan (default layout; the fp64 engine's wave-chunk
// enumeration).  Start vector: x0_j = a_j,n-1 - rowsum_j / 2 with the row sum
// accumulated in double-double (gpu_exact_dense.cu:642-652 in ~106 bits).
// Walk: walk_dd.hip on o.gpu_num devices (static contiguous split of the
// wave-chunks, one host thread per device), or cpu_dd_range below on host
// threads — the same dd.hpp operations in the same order, so the chunk
// partials are bit-identical.  They are combined on the host in one fixed
// pairwise tree over the global chunk index, so the result does not depend on
// the device count, the split or the host thread count.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <string>
#include <thread>

#include "dd.hpp"
#include "engine.hpp"

namespace sup {

namespace {

// Start state of wave-chunk ga, lane `lane` (walk_dd.hip's chunk start).
void dd_start(const Plan& P, const std::vector<double>& x0dd, uint64_t ga, uint32_t lane, dd* x) {
  const int n = P.n, NP = P.NP, L = P.lay.L;
  for (int r = 0; r < n; ++r) x[r] = dd{x0dd[r], x0dd[NP + r]};
  uint64_t h = ga ^ (ga >> 1);
  const int hb = L + P.lay.m;
  while (h) {
    const int b = __builtin_ctzll(h);
    h &= h - 1;
    const double* col = P.cols.data() + (size_t)(2 * (hb + b)) * NP;
    for (int r = 0; r < n; ++r) x[r] = dd_add_d(x[r], col[r]);
  }
  for (int e = 0; e < L; ++e) {
    const double* col = P.cols.data() + (size_t)(2 * e) * NP;
    const bool on = (lane >> e) & 1u;
    for (int r = 0; r < n; ++r) x[r] = dd_add_d(x[r], on ? col[r] : 0.0);
  }
}

// dd_prod4 (walk_dd.hip): strided partials p_{j mod 4}, then (p0 p1)(p2 p3).
dd dd_prod(const dd* x, int n) {
  dd p[4] = {x[0], n > 1 ? x[1] : dd{1.0, 0.0}, n > 2 ? x[2] : dd{1.0, 0.0}, n > 3 ? x[3] : dd{1.0, 0.0}};
  for (int j = 4; j < n; ++j) p[j & 3] = dd_mul(p[j & 3], x[j]);
  if (n == 1) return p[0];
  if (n == 2) return dd_mul(p[0], p[1]);
  if (n == 3) return dd_mul(dd_mul(p[0], p[1]), p[2]);
  return dd_mul(dd_mul(p[0], p[1]), dd_mul(p[2], p[3]));
}

void dd_add_colv(dd* x, const double* col, int n) {
  for (int r = 0; r < n; ++r) x[r] = dd_add_d(x[r], col[r]);
}

// walk_dd_blocked's block product: ((x0 x1)(x2 x3))((x4 x5)(x6 x7)), rows
// past n = 1.
dd dd_bprod8(const dd* x, int n, int b) {
  auto v = [&](int i) { return 8 * b + i < n ? x[8 * b + i] : dd{1.0, 0.0}; };
  return dd_mul(dd_mul(dd_mul(v(0), v(1)), dd_mul(v(2), v(3))), dd_mul(dd_mul(v(4), v(5)), dd_mul(v(6), v(7))));
}

// One wave-chunk, every lane, then the 64-lane xor butterfly (dd_wave_sum).
dd dd_chunk(const Plan& P, const std::vector<double>& x0dd, uint64_t ga) {
  const int n = P.n, NP = P.NP, L = P.lay.L;
  const uint32_t T = 1u << P.lay.m;
  const double* colL = P.cols.data() + (size_t)(2 * L) * NP;  // walk bit 0, + and - columns follow
  dd v[64];
  std::vector<dd> x(n);
  if (P.chunk_ends) {  // walk_dd's chunk end: a zero chunk-end row, every term zero
    dd_start(P, x0dd, ga, 0, x.data());
    for (int r = 0; r < n; ++r)
      if (((P.chunk_ends >> r) & 1u) && x[r].hi == 0.0) return dd{0.0, 0.0};
  }
  for (uint32_t lane = 0; lane < 64; ++lane) {
    if (lane >= (1u << L)) {
      v[lane] = dd{0.0, 0.0};
      continue;
    }
    dd_start(P, x0dd, ga, lane, x.data());
    if (P.kind == kWalkSparse) {  // walk_dd_blocked: suffix products of 8-row blocks
      const int NB = (n + 7) / 8;
      std::vector<dd> U(NB + 1);
      U[NB] = dd{1.0, 0.0};
      for (int b = NB - 1; b >= 0; --b) U[b] = dd_mul(dd_bprod8(x.data(), n, b), U[b + 1]);
      dd acc = U[0];
      for (uint32_t t = 1; t < T; ++t) {
        const uint32_t k = (uint32_t)__builtin_ctz(t);
        const uint32_t neg = (t >> (k + 1)) & 1u;
        const double* col = colL + (size_t)(2u * k + neg) * NP;
        const int nb = P.nblk[L + k];
        for (int b = nb - 1; b >= 0; --b) {  // top block first (deeper blocks' U current)
          for (int j = 8 * b; j < 8 * b + 8 && j < n; ++j) x[j] = dd_add_d(x[j], col[j]);
          U[b] = dd_mul(dd_bprod8(x.data(), n, b), U[b + 1]);
        }
        acc = dd_add(acc, (t & 1u) ? dd_neg(U[0]) : U[0]);
      }
      const uint32_t lane_par = __builtin_popcount(lane) & 1u;
      if (((uint32_t)ga ^ lane_par) & 1u) acc = dd_neg(acc);
      v[lane] = acc;
      continue;
    }
    dd acc = dd_prod(x.data(), n);
    uint32_t t = 1;
    for (; t + 1 < T; t += 2) {
      dd_add_colv(x.data(), colL + (size_t)((t >> 1) & 1u) * NP, n);
      acc = dd_add(acc, dd_neg(dd_prod(x.data(), n)));
      const uint32_t u = t + 1;
      const uint32_t k = (uint32_t)__builtin_ctz(u);
      const uint32_t neg = (u >> (k + 1)) & 1u;
      dd_add_colv(x.data(), colL + (size_t)(2u * k + neg) * NP, n);
      acc = dd_add(acc, dd_prod(x.data(), n));
    }
    if (t < T) {
      dd_add_colv(x.data(), colL + (size_t)((t >> 1) & 1u) * NP, n);
      acc = dd_add(acc, dd_neg(dd_prod(x.data(), n)));
    }
    const uint32_t lane_par = __builtin_popcount(lane) & 1u;
    if (((uint32_t)ga ^ lane_par) & 1u) acc = dd_neg(acc);
    v[lane] = acc;
  }
  for (int off = 1; off <= 32; off <<= 1) {
    dd w[64];
    for (int l = 0; l < 64; ++l) w[l] = dd_add(v[l], v[l ^ off]);
    std::copy(w, w + 64, v);
  }
  return v[0];
}

// Pairwise tree over the chunk index (zero padded to a power of two).
dd dd_pairwise(std::vector<dd> v) {
  if (v.empty()) return dd{0.0, 0.0};
  while (v.size() > 1) {
    std::vector<dd> w((v.size() + 1) / 2);
    for (size_t i = 0; i < w.size(); ++i) w[i] = 2 * i + 1 < v.size() ? dd_add(v[2 * i], v[2 * i + 1]) : v[2 * i];
    v.swap(w);
  }
  return v[0];
}

}  // namespace

void cpu_dd_range(const Plan& P, const std::vector<double>& x0dd, uint64_t c0, uint64_t c1, int threads,
                  double* parts) {
  if (c1 <= c0) return;
  const uint64_t count = c1 - c0;
  const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(threads, 1), count));
  std::vector<std::thread> th;
  for (int w = 0; w < nt; ++w)
    th.emplace_back([&, w]() {
      for (uint64_t a = (uint64_t)w; a < count; a += (uint64_t)nt) {
        const dd v = dd_chunk(P, x0dd, c0 + a);
        parts[2 * a] = v.hi, parts[2 * a + 1] = v.lo;
      }
    });
  for (auto& t : th) t.join();
}

int quad_perman(const double* A, int n, const sup_opts& o, bool on_cpu, double* hi, double* lo, double* kernel_ms,
                int* devices_used) {
  Plan P;
  // The prefix-blocked walk (walk_dd_blocked) when its cost model beats the
  // dense walk's, else the dense walk with its walk + lane columns in the
  // greedy prefix order; the rows none of them touches end the chunks where
  // they are exactly zero.  Above n = 28 the blocked kernel's suffix products
  // do not fit two waves per SIMD (1 wave: 268 VGPRs at n = 30), so it must
  // save more: measured (profiles/r5/probe_quad_blocked.log) the bench matrix
  // (n = 40, modelled 45.5 against 81 ops) ran 12.0 s blocked against 9.9 s
  // dense, d = 0.2 and dwt_59's n = 30 leaves (~0.25-0.3 of the dense ops)
  // faster blocked.
  const Layout lay = default_layout(n);
  const double bar = (n <= 28 ? 1.0 : 0.4) * (2.0 * n + 1.0);
  int rc = SUP_OK;
  if (!(lay.m > 0 && (rc = make_plan(A, n, kWalkSparse, false, lay, P)) == SUP_OK && walk_cost(P) < bar &&
        (rc = improve_sparse_plan(A, n, lay, P)) == SUP_OK)) {
    SegChoice order;
    order.order = greedy_walk_order(A, n, lay.m + lay.L);
    rc = make_plan(A, n, kWalkDense, false, lay, P, lay.m > 0 ? &order : nullptr);
  }
  if (rc) return rc;
  // Nijenhuis-Wilf start vector in double-double (rows in engine order)
  std::vector<double> x0dd(2 * (size_t)P.NP, 0.0);
  for (int j = 0; j < n; ++j) {
    const int i = P.rowperm[j];
    dd rs{0.0, 0.0};
    for (int c = 0; c < n; ++c) rs = dd_add_d(rs, A[(size_t)i * n + c]);
    const dd x = dd_add_d(dd{-0.5 * rs.hi, -0.5 * rs.lo}, A[(size_t)i * n + n - 1]);
    x0dd[j] = x.hi, x0dd[P.NP + j] = x.lo;
  }
  const uint64_t C = P.lay.chunks();
  std::vector<double> parts(2 * C, 0.0);
  double kms = 0.0;
  int used = 0;
  if (on_cpu) {
    cpu_dd_range(P, x0dd, 0, C, std::max(o.threads, 1), parts.data());
  } else {
    int ndev = 0;
    if ((rc = device_count(&ndev))) return rc;
    if (ndev == 0) {
      set_error("no HIP device available (sup_perman_quad has no CPU fallback; on_cpu = 1 runs host threads)");
      return SUP_ENODEV;
    }
    if (o.device_id < 0 || o.device_id >= ndev) {
      set_error("sup_perman_quad: device_id out of range");
      return SUP_EINVAL;
    }
    const int G = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, std::min(o.gpu_num, ndev - o.device_id)), C));
    std::vector<int> drc(G, SUP_OK);
    std::vector<double> dms(G, 0.0);
    std::vector<std::string> derr(G);  // g_err is thread_local: carry worker messages back
    auto work = [&](int g) {
      const uint64_t a = C * (uint64_t)g / (uint64_t)G, b = C * (uint64_t)(g + 1) / (uint64_t)G;
      drc[g] = run_range_dd(o.device_id + g, P, x0dd, a, b, parts.data() + 2 * a, &dms[g]);
      if (drc[g]) derr[g] = last_error();
    };
    std::vector<std::thread> th;
    for (int g = 1; g < G; ++g) th.emplace_back(work, g);
    work(0);
    for (auto& t : th) t.join();
    for (int g = 0; g < G; ++g)
      if (drc[g]) {
        set_error(derr[g]);
        return drc[g];
      }
    kms = *std::max_element(dms.begin(), dms.end());
    used = G;
  }
  std::vector<dd> v(C);
  for (uint64_t a = 0; a < C; ++a) v[a] = dd{parts[2 * a], parts[2 * a + 1]};
  dd total = dd_pairwise(std::move(v));
  // perm = (4(n&1) - 2) * total: a power-of-two scale, exact
  const double f = 4.0 * (n & 1) - 2.0;
  *hi = f * total.hi;
  *lo = f * total.lo;
  if (kernel_ms) *kernel_ms = kms;
  if (devices_used) *devices_used = used;
  return SUP_OK;
}

}  // namespace sup
