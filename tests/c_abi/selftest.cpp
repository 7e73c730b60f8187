// selftest.cpp — host-code self test for the sanitizer builds
// (make -C superman_amd/csrc sanitize: AddressSanitizer + UndefinedBehavior-
// Sanitizer, and ThreadSanitizer).  No GPU is needed: it drives every host
// path that runs without a device, with the thread counts that make the
// threaded code race if it can, and checks results are identical across
// thread counts (the engine's results never depend on timing):
//   - the dynamic item queue (run_item_queue) that -p6/-p8, the exact path and
//     the estimators share, with several takers, one of them the real CPU
//     walk (cpu_walk_range, itself threaded) as the hybrid worker runs it;
//   - planning: the walk-order search's thread pool, the segmented walk's
//     budget ladder and its concurrent hiprtc compiles + code scans;
//   - the host walks of every kernel family (sup_perman_cpu), the exact
//     residue walk, the double-double walk and the estimators on host threads;
//   - the readers, CSR/CSC, SortOrder/SkipOrder, the -o/-u reductions.
// Usage: selftest <repo root>
#include <atomic>
#include <functional>
#include <memory>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../include/superman.h"
#include "../../superman_amd/csrc/engine.hpp"

static int failures = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s (%s)\n", __FILE__,     \
                   __LINE__, #c, sup_last_error());                       \
      ++failures;                                                         \
    }                                                                     \
  } while (0)

static std::vector<double> random_matrix(int n, double d, unsigned seed, bool integer) {
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<double> a((size_t)n * n, 0.0);
  for (auto& v : a)
    if (u(g) < d) v = integer ? (double)(1 + (int)(u(g) * 5)) : u(g) * 5.0;
  for (int i = 0; i < n; ++i) a[(size_t)i * n + (i * 7 + 3) % n] = 1.0;  // no empty row / column
  return a;
}

static void test_queue() {
  // fake device takers write item slots and their own accumulators; one
  // taker walks real wave-chunks on host threads, as the hybrid worker does
  const int n = 20;
  std::vector<double> A = random_matrix(n, 0.5, 7, false);
  sup::Plan P;
  CHECK(sup::make_plan(A.data(), n, sup::kWalkDense, true, sup::default_layout(n), P) == SUP_OK);
  const uint64_t C = P.lay.chunks();
  for (int takers : {1, 3, 5}) {
    std::vector<double> slot(C, 0.0);
    std::vector<uint64_t> took(takers, 0);
    std::atomic<int> cpu{0};
    const int rc = sup::run_item_queue(C, takers, [&](int t, uint64_t it) {
      if (t == takers - 1) {
        slot[it] = sup::cpu_walk_range(P, it, it + 1, 3);
        cpu.fetch_add(1);
      } else {
        slot[it] = sup::cpu_walk_range(P, it, it + 1, 1);
      }
      ++took[t];
      return SUP_OK;
    });
    CHECK(rc == SUP_OK);
    uint64_t sum = 0;
    for (uint64_t v : took) sum += v;
    CHECK(sum == C);
    CHECK(sup::pairwise_host(slot) == sup::cpu_walk_range(P, 0, C, 4));
  }
  // a failing taker stops the queue and its message survives the thread
  const int rc = sup::run_item_queue(1000, 4, [&](int, uint64_t it) {
    if (it == 500) {
      sup::set_error("item 500 failed on purpose");
      return SUP_EHIP;
    }
    return SUP_OK;
  });
  CHECK(rc == SUP_EHIP);
  CHECK(std::strcmp(sup_last_error(), "item 500 failed on purpose") == 0);
}

// Checkpoint file of the chunk queue: concurrent appends, reload, a torn last
// line dropped, a foreign header refused (engine.cpp ckpt_open / ckpt_record).
static void test_checkpoint() {
  char path[] = "/tmp/sup_selftest_ckpt_XXXXXX";
  const int fd = mkstemp(path);
  CHECK(fd >= 0);
  close(fd);
  const char* head = "supckpt 2 0123456789abcdef 0 0 0 4096 64 64\n";
  const uint64_t N = 64;
  std::vector<double> want(N);
  for (uint64_t i = 0; i < N; ++i) want[i] = std::ldexp((double)(i * 2654435761u % 1000003u), -(int)(i % 50)) - 7.5;
  {
    std::vector<double> ip(N, 0.0);
    std::vector<char> done(N, 0);
    uint64_t vis = 0;
    int resumed = -1;
    sup::Checkpoint ck;
    CHECK(sup::ckpt_open(path, head, N, ip, done, vis, resumed, ck) == SUP_OK);  // empty file: fresh
    CHECK(resumed == 0);
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&, t] {
        for (uint64_t i = t; i < N; i += 8) CHECK(sup::ckpt_record(ck, i, want[i], 100 + i) == SUP_OK);
      });
    for (auto& x : th) x.join();
  }
  {
    FILE* f = std::fopen(path, "a");  // an interrupted append
    std::fputs("7 3ff00000", f);
    std::fclose(f);
  }
  std::vector<double> ip(N, 0.0);
  std::vector<char> done(N, 0);
  uint64_t vis = 0;
  int resumed = 0;
  {
    sup::Checkpoint ck;
    CHECK(sup::ckpt_open(path, head, N, ip, done, vis, resumed, ck) == SUP_OK);
  }
  CHECK(resumed == (int)N);
  CHECK(std::memcmp(ip.data(), want.data(), N * sizeof(double)) == 0);
  CHECK(vis == 100 * N + N * (N - 1) / 2);
  {
    std::vector<double> ip2(N, 0.0);
    std::vector<char> done2(N, 0);
    uint64_t vis2 = 0;
    int resumed2 = 0;
    sup::Checkpoint ck;
    CHECK(sup::ckpt_open(path, "supckpt 2 fedcba9876543210 0 0 0 4096 64 64\n", N, ip2, done2, vis2, resumed2, ck) ==
          SUP_EINVAL);
  }
  std::remove(path);
}

static void test_host_walks() {
  for (int n : {12, 17, 22}) {
    std::vector<double> A = random_matrix(n, 0.45, 100 + n, true);
    for (sup_kernel k : {SUP_KERNEL_DENSE, SUP_KERNEL_SPARYSER, SUP_KERNEL_SKIPPER, SUP_KERNEL_SEGMENTED}) {
      std::vector<double> M = A;
      std::vector<int> rp(n), cp(n);
      if (k == SUP_KERNEL_SKIPPER) CHECK(sup_skip_order(M.data(), SUP_FLOAT64, n, rp.data(), cp.data()) == SUP_OK);
      double p1 = 0, p8 = 0;
      CHECK(sup_perman_cpu(M.data(), SUP_FLOAT64, n, k, 1, &p1, nullptr) == SUP_OK);
      CHECK(sup_perman_cpu(M.data(), SUP_FLOAT64, n, k, 8, &p8, nullptr) == SUP_OK);
      CHECK(p1 == p8);
    }
    // exact integer on host threads, two thread counts, and against fp64
    sup_opts o;
    sup_opts_init(&o);
    char e1[600], e4[600];
    o.threads = 1;
    CHECK(sup_perman_exact(A.data(), SUP_FLOAT64, n, &o, 1, e1, sizeof e1, nullptr) == SUP_OK);
    o.threads = 4;
    CHECK(sup_perman_exact(A.data(), SUP_FLOAT64, n, &o, 1, e4, sizeof e4, nullptr) == SUP_OK);
    CHECK(std::strcmp(e1, e4) == 0);
    double pd = 0;
    CHECK(sup_perman_cpu(A.data(), SUP_FLOAT64, n, SUP_KERNEL_DENSE, 4, &pd, nullptr) == SUP_OK);
    CHECK(std::fabs(pd - std::strtod(e1, nullptr)) <= 1e-9 * std::fabs(pd));
    // double-double on host threads
    double h1 = 0, l1 = 0, h4 = 0, l4 = 0;
    o.threads = 1;
    CHECK(sup_perman_quad(A.data(), SUP_FLOAT64, n, &o, 1, &h1, &l1, nullptr) == SUP_OK);
    o.threads = 4;
    CHECK(sup_perman_quad(A.data(), SUP_FLOAT64, n, &o, 1, &h4, &l4, nullptr) == SUP_OK);
    CHECK(h1 == h4 && l1 == l4);
  }
}

static void test_planning(const std::string& root) {
  // n = 32 (BASELINE config 2): walk-order search pool, budget ladder,
  // concurrent compiles and code scans (hiprtc runs without a device)
  void* mat = nullptr;
  sup_dtype t;
  int n = 0, nnz = 0;
  CHECK(sup_read_matrix((root + "/tests/fixtures/double__32_0.50_0").c_str(), 0, &mat, &t, &n, &nnz) == SUP_OK);
  if (!mat) return;
  sup_opts o;
  sup_opts_init(&o);
  o.jit = 1;
  int kind = -1, L = 0, m = 0, cc = 0, pb = 0;
  double ops = 0, ms = 0;
  std::vector<int> colmap(n);
  CHECK(sup_prepare(mat, t, n, SUP_KERNEL_DENSE, &o, &kind, &ms) == SUP_OK);
  CHECK(kind == 3);
  CHECK(sup_plan_info(mat, t, n, SUP_KERNEL_DENSE, &o, &kind, colmap.data(), &L, &m, &cc, &pb, &ops) == SUP_OK);
  uint64_t k1 = 0, k2 = 0;
  CHECK(sup_plan_key(mat, t, n, SUP_KERNEL_DENSE, &o, &k1) == SUP_OK);
  CHECK(sup_plan_key(mat, t, n, SUP_KERNEL_DENSE, &o, &k2) == SUP_OK);
  CHECK(k1 == k2 && k1 != 0);
  // the host twin of the segmented walk on the same plan, two thread counts
  double s1 = 0, s8 = 0;
  CHECK(sup_perman_cpu(mat, t, 22 < n ? 22 : n, SUP_KERNEL_SEGMENTED, 1, &s1, nullptr) == SUP_OK);
  CHECK(sup_perman_cpu(mat, t, 22 < n ? 22 : n, SUP_KERNEL_SEGMENTED, 8, &s8, nullptr) == SUP_OK);
  CHECK(s1 == s8);
  sup_free(mat);
  // config 5 (n = 44 integer, SkipOrder): the SkipPer, SpaRyser and exact
  // plans search their columns for chunk ends on host threads (round 5)
  CHECK(sup_read_matrix((root + "/tests/fixtures/synth44_0.15_int").c_str(), 0, &mat, &t, &n, &nnz) == SUP_OK);
  if (!mat) return;
  std::vector<double> A5(n * n);
  for (int i = 0; i < n * n; ++i) A5[i] = t == SUP_INT32 ? ((const int*)mat)[i] : ((const double*)mat)[i];
  std::vector<int> rp(n), cp(n);
  CHECK(sup_skip_order(A5.data(), SUP_FLOAT64, n, rp.data(), cp.data()) == SUP_OK);
  o.jit = -1;
  std::vector<int> cm1(n), cm2(n);
  CHECK(sup_plan_info(A5.data(), SUP_FLOAT64, n, SUP_KERNEL_SKIPPER, &o, &kind, cm1.data(), &L, &m, &cc, &pb, &ops) ==
        SUP_OK);
  CHECK(kind == 2 && ops < 25.5);
  CHECK(sup_plan_info(A5.data(), SUP_FLOAT64, n, SUP_KERNEL_SPARYSER, &o, &kind, cm2.data(), &L, &m, &cc, &pb, &ops) ==
        SUP_OK);
  CHECK(kind == 1 && cm1 == cm2);  // the same search, the same columns
  sup_free(mat);
}

static void test_io_and_reductions(const std::string& root) {
  void* mat = nullptr;
  sup_dtype t;
  int n = 0, nnz = 0;
  CHECK(sup_read_mtx((root + "/tests/fixtures/mtx/chesapeake.mtx").c_str(), 0, &mat, &t, &n, &nnz) == SUP_OK);
  if (mat) {
    int cnt = 0;
    CHECK(sup_count_nnz(mat, t, n, &cnt) == SUP_OK);
    sup_free(mat);
  }
  {
    // -o reductions down to small leaves (min_n 12), exact leaves on host
    // threads, against the direct exact walk of the same matrix
    const int m = 24;
    std::vector<double> R = random_matrix(m, 0.15, 11, true);
    sup_reduce_opts r;
    sup_reduce_opts_init(&r);
    r.compress = 1;
    r.min_n = 12;
    sup_opts o;
    sup_opts_init(&o);
    o.threads = 4;
    char red[600], dir[600];
    CHECK(sup_perman_reduced_exact(R.data(), SUP_FLOAT64, m, &o, 1, &r, red, sizeof red, nullptr) == SUP_OK);
    CHECK(sup_perman_exact(R.data(), SUP_FLOAT64, m, &o, 1, dir, sizeof dir, nullptr) == SUP_OK);
    CHECK(std::strcmp(red, dir) == 0);
    // the deferred combine with concurrent leaf workers (sup_perman_reduced's
    // GPU form) against the sequential callback fold: the same bits
    auto leaf = [](const double* a, int k, double* v) {
      return sup_perman_cpu(a, SUP_FLOAT64, k, SUP_KERNEL_DENSE, 2, v, nullptr);
    };
    double seq = 0.0, par = 0.0;
    int ls = 0, lp = 0;
    CHECK(sup_decompose(R.data(), SUP_FLOAT64, m, &r,
                        [](const double* a, int k, void*, double* v) {
                          return sup_perman_cpu(a, SUP_FLOAT64, k, SUP_KERNEL_DENSE, 2, v, nullptr);
                        },
                        nullptr, &seq, &ls) == SUP_OK);
    CHECK(sup::decompose_batched(R.data(), m, r, 6, [&](int, const double* a, int k, double* v) { return leaf(a, k, v); },
                                 &par, &lp) == SUP_OK);
    CHECK(ls == lp && ls > 4 && std::memcmp(&seq, &par, sizeof seq) == 0);
    // two-stage batches (sup_perman_reduced's batched GPU form): planners hand
    // each batch's walk to their walker threads; 1 and 3 workers, batches of
    // up to 4 leaves, the walk on host threads here: the same bits
    for (int workers : {1, 3}) {
      double stg = 0.0;
      int lst = 0;
      const sup::LeafBatchStagedFn staged = [&](int, const std::vector<const double*>& as, int k,
                                                const std::vector<double*>& vs, std::function<int()>& walk) {
        auto mats = std::make_shared<std::vector<std::vector<double>>>();
        for (const double* a : as) mats->emplace_back(a, a + (size_t)k * k);
        walk = [mats, vs, k, &leaf]() {
          for (size_t i = 0; i < mats->size(); ++i)
            if (const int e = leaf((*mats)[i].data(), k, vs[i])) return e;
          return SUP_OK;
        };
        return SUP_OK;
      };
      CHECK(sup::decompose_batched_staged(R.data(), m, r, workers, 4, staged, &stg, &lst) == SUP_OK);
      CHECK(lst == ls && std::memcmp(&seq, &stg, sizeof seq) == 0);
    }
    // a failing walk stops the staged decomposition and its message survives the walker thread
    {
      std::atomic<int> walks{0};
      double stg = 0.0;
      const sup::LeafBatchStagedFn staged = [&](int, const std::vector<const double*>&, int,
                                                const std::vector<double*>&, std::function<int()>& walk) {
        walk = [&walks]() {
          if (walks.fetch_add(1) == 1) {
            sup::set_error("walk 1 failed on purpose");
            return SUP_EHIP;
          }
          return SUP_OK;
        };
        return SUP_OK;
      };
      CHECK(sup::decompose_batched_staged(R.data(), m, r, 2, 2, staged, &stg, &lp) == SUP_EHIP);
      CHECK(std::strcmp(sup_last_error(), "walk 1 failed on purpose") == 0);
    }
    // a failing leaf stops the decomposition and its message survives the worker thread
    std::atomic<int> calls{0};
    CHECK(sup::decompose_batched(R.data(), m, r, 4,
                                 [&](int, const double*, int, double*) {
                                   if (calls.fetch_add(1) == 2) {
                                     sup::set_error("leaf 2 failed on purpose");
                                     return SUP_EHIP;
                                   }
                                   return SUP_OK;
                                 },
                                 &par, &lp) == SUP_EHIP);
    CHECK(std::strcmp(sup_last_error(), "leaf 2 failed on purpose") == 0);
  }
  std::vector<double> A = random_matrix(24, 0.3, 5, false);
  int cnt = 0;
  CHECK(sup_count_nnz(A.data(), SUP_FLOAT64, 24, &cnt) == SUP_OK);
  std::vector<int> cptrs(25), rows(cnt), rptrs(25), cols(cnt);
  std::vector<double> cv(cnt), rv(cnt);
  CHECK(sup_compress(A.data(), SUP_FLOAT64, 24, cptrs.data(), rows.data(), cv.data(), rptrs.data(), cols.data(),
                     rv.data()) == SUP_OK);
  std::vector<int> rp(24), cp(24);
  std::vector<double> B = A;
  CHECK(sup_sort_order(B.data(), SUP_FLOAT64, 24, cp.data()) == SUP_OK);
  B = A;
  CHECK(sup_skip_order(B.data(), SUP_FLOAT64, 24, rp.data(), cp.data()) == SUP_OK);
  // estimators on host threads: the estimate depends on (matrix, samples, seed) only
  int* g = nullptr;
  int nov = 0;
  CHECK(sup_grid_graph(6, 6, &g, &nov) == SUP_OK);
  sup_opts o;
  sup_opts_init(&o);
  sup_approx_result a1, a4;
  o.threads = 1;
  CHECK(sup_approx(g, SUP_INT32, nov, 1, 64 * 200, 4, 5, 9, &o, 1, &a1) == SUP_OK);
  o.threads = 4;
  CHECK(sup_approx(g, SUP_INT32, nov, 1, 64 * 200, 4, 5, 9, &o, 1, &a4) == SUP_OK);
  CHECK(a1.mean == a4.mean);
  sup_free(g);
  // argument errors come back as codes, never crashes
  double out = 0;
  CHECK(sup_perman_cpu(nullptr, SUP_FLOAT64, 4, SUP_KERNEL_DENSE, 1, &out, nullptr) == SUP_EINVAL);
  CHECK(sup_perman_cpu(A.data(), SUP_FLOAT64, 65, SUP_KERNEL_DENSE, 1, &out, nullptr) == SUP_EINVAL);
}

int main(int argc, char** argv) {
  const std::string root = argc > 1 ? argv[1] : ".";
  test_queue();
  test_checkpoint();
  test_host_walks();
  test_planning(root);
  test_io_and_reductions(root);
  std::printf("selftest: %s (%d failed checks)\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
