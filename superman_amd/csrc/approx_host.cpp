// approx_host.cpp — host side of the randomized estimators: C ABI sup_approx
// (GPU kernels or host threads), the multi-device sample-block queue, and the
// grid-graph generator of the reference's -i mode.
//
// Replaces the drivers gpu_perman64_rasmussen / _approximation (+ their
// _multigpucpu_chunks forms, gpu_approximation_dense.cu:373-700,
// gpu_approximation_sparse.cu:455-790), the CPU estimators rasmussen /
// approximation_perman64 (+ _sparse, algo.h:172-560) and gridGraph2compressed
// (util.h:403-520).
//
// Samples are grouped in blocks of 64; a run covers ceil(samples / 64) blocks,
// cut into power-of-two items of blocks that devices (and, with cpu_worker,
// one host thread) take from a queue.  Each item's three block sums are folded
// by the same 64-way pairwise passes on either side and the items by the host
// pairwise tree, so the estimate is bit-identical for any device count and
// for CPU vs GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "approx.hpp"
#include "approx_core.hpp"
#include "engine.hpp"

namespace sup {
namespace {

struct Pattern {
  int n = 0, W = 1;
  std::vector<uint64_t> row, col;  // n x W each
};

int words_for(int n) {
  const int w = (n + 63) / 64;
  int p = 1;
  while (p < w) p <<= 1;
  return p;
}

Pattern make_pattern(const std::vector<double>& a, int n) {
  Pattern P;
  P.n = n;
  P.W = words_for(n);
  P.row.assign((size_t)n * P.W, 0);
  P.col.assign((size_t)n * P.W, 0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      if (a[(size_t)i * n + j] != 0.0) {
        P.row[(size_t)i * P.W + (j >> 6)] |= 1ull << (j & 63);
        P.col[(size_t)j * P.W + (i >> 6)] |= 1ull << (i & 63);
      }
  return P;
}

double pairwise64v(double* v) {
  for (int w = 64; w > 1; w >>= 1)
    for (int i = 0; i < w / 2; ++i) v[i] = v[2 * i] + v[2 * i + 1];
  return v[0];
}

// The device's launch_pairwise_reduce on the host: 64-way zero-padded passes.
double fold64(std::vector<double> part) {
  if (part.empty()) return 0.0;
  while (part.size() > 1) {
    const size_t groups = (part.size() + 63) / 64;
    std::vector<double> nxt(groups);
    for (size_t g = 0; g < groups; ++g) {
      double v[64];
      for (int l = 0; l < 64; ++l) {
        const size_t i = g * 64 + l;
        v[l] = i < part.size() ? part[i] : 0.0;
      }
      nxt[g] = pairwise64v(v);
    }
    part.swap(nxt);
  }
  return part[0];
}

struct Job {
  const Pattern* P;
  int method, intervals, times;
  uint64_t seed;
};

template <int W>
double one_sample(const Job& J, uint64_t s, std::vector<float>& dr, std::vector<float>& dc, bool& zero) {
  if (J.method == 0) return rasmussen_sample<W>(J.P->row.data(), J.P->n, J.seed, s, zero);
  return scaling_sample<W>(J.P->row.data(), J.P->col.data(), J.P->n, J.intervals, J.times, J.seed, s, dr.data(),
                           dc.data(), 1u, zero);
}

// Blocks [b0, b1) on `threads` host threads -> the item's (sum, sq, zeros).
void cpu_item(const Job& J, uint64_t b0, uint64_t b1, int threads, double out[3]) {
  const uint64_t nb = b1 - b0;
  std::vector<double> ps(nb), pq(nb), pz(nb);
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, threads), nb));
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t]() {
      std::vector<float> dr(J.P->n), dc(J.P->n);
      for (uint64_t b = t; b < nb; b += (uint64_t)T) {
        double e[64], q[64], z[64];
        for (int l = 0; l < 64; ++l) {
          bool zero = false;
          const uint64_t s = (b0 + b) * 64 + l;
          double v;
          switch (J.P->W) {
            case 1: v = one_sample<1>(J, s, dr, dc, zero); break;
            case 2: v = one_sample<2>(J, s, dr, dc, zero); break;
            case 4: v = one_sample<4>(J, s, dr, dc, zero); break;
            case 8: v = one_sample<8>(J, s, dr, dc, zero); break;
            default: v = one_sample<16>(J, s, dr, dc, zero); break;
          }
          e[l] = v;
          q[l] = v * v;
          z[l] = zero ? 1.0 : 0.0;
        }
        ps[b] = pairwise64v(e);
        pq[b] = pairwise64v(q);
        pz[b] = pairwise64v(z);
      }
    });
  for (auto& t : th) t.join();
  out[0] = fold64(std::move(ps));
  out[1] = fold64(std::move(pq));
  out[2] = fold64(std::move(pz));
}

#define AHIP(call)                                                                    \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) {                                                           \
      set_error(std::string(#call) + ": " + hipGetErrorString(e_));                   \
      return SUP_EHIP;                                                                \
    }                                                                                 \
  } while (0)

// One device: its own buffers, items taken from the shared queue.
struct DevWorker {
  int dev = 0, cus = 0, grid = 0;
  bool coop = false;  // one wave per sample (approx.hip approx_coop), same bits
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  uint64_t *d_row = nullptr, *d_col = nullptr;
  double *d_part = nullptr, *d_scr = nullptr, *d_out = nullptr;
  float* d_dr = nullptr;
  unsigned* d_cnt = nullptr;
  double kernel_ms = 0.0;

  int init(int device, const Job& J, uint64_t item) {
    dev = device;
    AHIP(select_device(dev));
    hipDeviceProp_t prop;
    AHIP(hipGetDeviceProperties(&prop, phys_device(dev)));
    cus = prop.multiProcessorCount;
    // The cooperative form for large n (tools/probes/probe_approx_coop.py,
    // profiles/r2/probe_approx_coop.log): the scaling estimator from n > 96
    // (its per-lane factors live in an HBM scratch: 0.81x at n = 72, 2.5x at
    // 128, 110x at 288 and 648), Rasmussen from n > 128 (0.35x at 128, 4.6x at
    // 288, 5x at 648); SUP_APPROX_COOP=0/1 forces the form (same bits).
    coop = (J.method == 1 && J.P->n > 96) || J.P->n > 128;
    if (const char* e = std::getenv("SUP_APPROX_COOP")) coop = std::atoi(e) != 0;
    int occ = 1;
    if (coop) AHIP(approx_coop_occupancy(J.P->W, J.method, J.P->n, &occ));
    else AHIP(approx_occupancy(J.P->W, J.method, &occ));
    grid = std::max(1, cus * std::max(1, occ));
    grid = (int)std::min<uint64_t>((uint64_t)grid, (item + 3) / 4);
    SUP_ON_DEVICE(dev, "estimator buffers");
    AHIP(hipStreamCreate(&st));
    AHIP(hipEventCreate(&e0));
    AHIP(hipEventCreate(&e1));
    const size_t pw = J.P->row.size() * sizeof(uint64_t);
    AHIP(hipMalloc(&d_row, pw));
    AHIP(hipMalloc(&d_col, pw));
    AHIP(hipMemcpy(d_row, J.P->row.data(), pw, hipMemcpyHostToDevice));
    AHIP(hipMemcpy(d_col, J.P->col.data(), pw, hipMemcpyHostToDevice));
    AHIP(hipMalloc(&d_part, 3 * item * sizeof(double)));
    AHIP(hipMalloc(&d_scr, (pairwise_scratch_size(item) + 1) * sizeof(double)));
    AHIP(hipMalloc(&d_out, 3 * sizeof(double)));
    AHIP(hipMalloc(&d_cnt, sizeof(unsigned)));
    if (J.method == 1 && !coop) AHIP(hipMalloc(&d_dr, 2ull * J.P->n * (size_t)grid * kBlock * sizeof(float)));
    return SUP_OK;
  }
  int run(const Job& J, uint64_t b0, uint64_t nb, double out[3]) {
    AHIP(select_device(dev));
    ApproxParams p{};
    p.rowpat = d_row;
    p.colpat = d_col;
    p.part = d_part;
    p.scratch = d_dr;
    p.counter = d_cnt;
    p.seed = J.seed;
    p.block0 = b0;
    p.nblocks = nb;
    p.n = J.P->n;
    p.method = J.method;
    p.intervals = J.intervals;
    p.times = J.times;
    p.lanes_total = (uint32_t)grid * kBlock;
    AHIP(hipMemsetAsync(d_cnt, 0, sizeof(unsigned), st));
    SUP_ON_DEVICE(dev, "estimator launch");
    AHIP(hipEventRecord(e0, st));
    if (coop) AHIP(launch_approx_coop(J.P->W, p, grid, st));
    else AHIP(launch_approx(J.P->W, p, grid, st));
    AHIP(hipEventRecord(e1, st));
    for (int k = 0; k < 3; ++k) AHIP(launch_pairwise_reduce(d_part + k * nb, nb, d_scr, d_out + k, st));
    AHIP(hipMemcpyAsync(out, d_out, 3 * sizeof(double), hipMemcpyDeviceToHost, st));
    AHIP(hipStreamSynchronize(st));
    float ms = 0.f;
    AHIP(hipEventElapsedTime(&ms, e0, e1));
    kernel_ms += ms;
    return SUP_OK;
  }
  ~DevWorker() {
    if (!st) return;
    (void)hipSetDevice(phys_device(dev));
    (void)hipFree(d_row);
    (void)hipFree(d_col);
    (void)hipFree(d_part);
    (void)hipFree(d_scr);
    (void)hipFree(d_out);
    (void)hipFree(d_cnt);
    if (d_dr) (void)hipFree(d_dr);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(st);
  }
};

}  // namespace
}  // namespace sup

using namespace sup;

extern "C" {

int sup_approx(const void* mat, sup_dtype t, int n, int method, uint64_t samples, int scale_intervals,
               int scale_times, uint64_t seed, const sup_opts* o_in, int on_cpu, sup_approx_result* res) {
  auto t0 = std::chrono::steady_clock::now();
  if (!mat || !res || n < 1 || n > 1024 || (method != 0 && method != 1) || samples == 0) {
    set_error("sup_approx: bad argument (n in [1, 1024], method 0 or 1, samples > 0)");
    return SUP_EINVAL;
  }
  if (method == 1 && (scale_intervals < 1 || scale_times < 0)) {
    set_error("sup_approx: scale_intervals must be >= 1 and scale_times >= 0");
    return SUP_EINVAL;
  }
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  std::vector<double> a((size_t)n * n);
  for (size_t i = 0; i < a.size(); ++i)
    a[i] = t == SUP_INT32 ? (double)((const int32_t*)mat)[i]
           : t == SUP_FLOAT32 ? (double)((const float*)mat)[i] : ((const double*)mat)[i];
  const Pattern P = make_pattern(a, n);
  const Job J{&P, method, scale_intervals, scale_times, seed};
  const uint64_t nblocks = (samples + 63) / 64;
  // items: a power of two of blocks, chosen from nblocks alone (>= 16 items when possible)
  uint64_t item = 1;
  while (item * 2 * 16 <= nblocks) item <<= 1;
  const uint64_t nitems = (nblocks + item - 1) / item;
  std::vector<double> is(nitems), iq(nitems), iz(nitems);
  std::memset(res, 0, sizeof(*res));
  int rc = SUP_OK;
  if (on_cpu) {
    for (uint64_t it = 0; it < nitems; ++it) {
      double r[3];
      cpu_item(J, it * item, std::min(nblocks, (it + 1) * item), std::max(1, o.threads), r);
      is[it] = r[0], iq[it] = r[1], iz[it] = r[2];
    }
    res->cpu_blocks = (int64_t)nblocks;
  } else {
    int cnt = 0;
    if (device_count(&cnt) != SUP_OK || cnt == 0) {
      set_error("no HIP device available (GPU estimators have no CPU fallback; use on_cpu)");
      return SUP_ENODEV;
    }
    const int G = std::max(1, o.gpu_num);
    if (o.device_id < 0 || o.device_id + G > cnt) {
      set_error("device range out of bounds");
      return SUP_ENODEV;
    }
    std::vector<DevWorker> dw(G);
    for (int g = 0; g < G && rc == SUP_OK; ++g) rc = dw[g].init(o.device_id + g, J, item);
    if (rc) return rc;
    std::atomic<int64_t> cpu_blocks{0};
    // takers 0..G-1: one host thread per device; taker G: the hybrid CPU
    // worker (-c with -g), the reference's cpu_chunk
    auto take = [&](int g, uint64_t it) -> int {
      const uint64_t b0 = it * item, b1 = std::min(nblocks, b0 + item);
      double r[3];
      if (g == G) {
        cpu_item(J, b0, b1, std::max(1, o.threads), r);
        cpu_blocks += (int64_t)(b1 - b0);
      } else {
        const int e = dw[g].run(J, b0, b1 - b0, r);
        if (e) return e;
      }
      is[it] = r[0], iq[it] = r[1], iz[it] = r[2];
      return SUP_OK;
    };
    if ((rc = run_item_queue(nitems, G + (o.cpu_worker ? 1 : 0), take))) return rc;
    for (int g = 0; g < G; ++g) res->kernel_ms = std::max(res->kernel_ms, dw[g].kernel_ms);
    res->devices = G;
    res->cpu_blocks = cpu_blocks.load();
  }
  const double N = (double)(nblocks * 64);
  const double s = pairwise_host(is), q = pairwise_host(iq), z = pairwise_host(iz);
  res->samples = nblocks * 64;
  res->mean = s / N;
  const double var = std::max(0.0, q / N - res->mean * res->mean) * N / std::max(1.0, N - 1.0);
  res->std_error = std::sqrt(var / N);
  res->zero_fraction = z / N;
  res->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SUP_OK;
}

// util.h:403-520 gridGraph2compressed: the m x n grid graph (one dimension
// even) as the bipartite adjacency of its two colour classes, nov = m*n/2;
// its permanent counts the domino tilings of the m x n board.
int sup_grid_graph(int m, int n, int** mat, int* nov) {
  if (!mat || !nov || m < 1 || n < 1) {
    set_error("sup_grid_graph: bad argument");
    return SUP_EINVAL;
  }
  if (m % 2 == 1 && n % 2 == 1) {
    set_error("one of the grid dimensions should be even");
    return SUP_EINVAL;
  }
  const int N = m * n / 2;
  if (N > 1024) {
    set_error("grid graph larger than 1024 x 1024");
    return SUP_EINVAL;
  }
  int rows, cols;
  if (m % 2 == 0) {
    rows = n;
    cols = m;
  } else {
    rows = m;
    cols = n;
  }
  std::vector<std::pair<int, int>> e1, e2;  // (vertex of colour class 1 / 2, neighbour)
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) {
      const bool c1 = (i % 2 == 0 && j % 2 == 0) || (i % 2 == 1 && j % 2 == 1);
      auto& e = c1 ? e1 : e2;
      const int x = i * (cols / 2) + j / 2;
      if (x - cols / 2 >= 0) e.push_back({x, x - cols / 2});
      if (x + cols / 2 < N) e.push_back({x, x + cols / 2});
      if (j % 2 == 0) {
        if (j != 0) e.push_back({x, x - 1});
        e.push_back({x, x});
      } else {
        e.push_back({x, x});
        if (j != cols - 1) e.push_back({x, x + 1});
      }
    }
  int* a = (int*)std::calloc((size_t)N * N, sizeof(int));
  if (!a) {
    set_error("out of host memory");
    return SUP_ENOMEM;
  }
  for (auto& p : e1) a[(size_t)p.first * N + p.second] = 1;
  for (auto& p : e2) a[(size_t)p.second * N + p.first] = 1;  // util.h:484-486
  *mat = a;
  *nov = N;
  return SUP_OK;
}

}  // extern "C"
