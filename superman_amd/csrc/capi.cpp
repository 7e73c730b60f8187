// capi.cpp — extern "C" boundary (include/superman.h).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "dd.hpp"
#include "engine.hpp"

using namespace sup;

namespace {

int check_common(const void* mat, int n, double* out) {
  if (!mat || !out) {
    set_error("null matrix or output pointer");
    return SUP_EINVAL;
  }
  if (n < 1 || n > SUP_MAX_N) {
    set_error("n = " + std::to_string(n) + " outside [1, 64] (64-bit Gray index)");
    return SUP_EINVAL;
  }
  return SUP_OK;
}

// The kernels index the walk with 32 bits (T = 1u << m) and pack the walk
// bits' block counts into two 64-bit words (k < 32), as default_layout
// assumes; an item of the chunk queue is 2^chunk_log2 wave-chunks (< 2^64).
int check_walk_opts(const sup_opts& o) {
  if (o.walk_log2 < 0 || o.walk_log2 > 31) {
    set_error("walk_log2 = " + std::to_string(o.walk_log2) + " outside [0, 31] (0 = default layout)");
    return SUP_EINVAL;
  }
  if (o.chunk_log2 < 0 || o.chunk_log2 > 62) {
    set_error("chunk_log2 = " + std::to_string(o.chunk_log2) + " outside [0, 62] (0 = automatic item size)");
    return SUP_EINVAL;
  }
  return SUP_OK;
}

WalkKind kind_of(sup_kernel k) {
  switch (k) {
    case SUP_KERNEL_SPARYSER: return kWalkSparse;
    case SUP_KERNEL_SKIPPER: return kWalkSkip;
    case SUP_KERNEL_SEGMENTED: return kWalkSeg;
    default: return kWalkDense;
  }
}

void fill_stats(sup_stats* st, const Plan& P, const SchedResult& r, double wall_ms, uint64_t gray) {
  if (!st) return;
  std::memset(st, 0, sizeof(*st));
  st->kernel_ms = r.kernel_ms;
  st->wall_ms = wall_ms;
  st->gray_steps = gray;
  st->visited_steps = r.visited;
  st->devices_used = r.devices;
  st->lane_bits = P.lay.L;
  st->walk_bits = P.lay.m;
  st->grid = r.grid;
  st->chunks_done_cpu = r.cpu_items;
  for (size_t i = 0; i < r.dev_partials.size() && i < 16; ++i) st->partials[i] = r.dev_partials[i];
  st->walk_kind = P.lds ? 4 : (int)P.kind;
  st->leaves = 1;
  st->est_ops_per_step = walk_cost(P);
  st->jit_ms = r.compile_ms;
  st->items_resumed = r.items_resumed;
  if (P.kind == kWalkSeg) {
    st->seg_cached_bits = (int16_t)P.seg_cc;
    st->seg_pair_bits = (int16_t)P.seg_b;
  }
}

}  // namespace

extern "C" {

void sup_opts_init(sup_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->gpu_num = 1;
  o->device_id = 0;
  o->threads = 16;  // main.cu:333
  o->block_dim = 256;
  o->timing = 1;
}

int sup_abi_version(void) { return SUP_ABI_VERSION; }
const char* sup_last_error(void) { return last_error(); }
int sup_device_count(int* count) {
  if (!count) return SUP_EINVAL;
  return device_count(count);
}
uint64_t sup_device_checks(void) { return device_checks_passed(); }
int sup_device_warmup(int device_id, int gpu_num, int n) {
  if (device_id < 0 || gpu_num < 1) return SUP_EINVAL;
  return warm_devices(device_id, gpu_num, n);
}
int sup_kernel_time(int device_id, double* total_ms, uint64_t* launches) {
  if (device_id < 0) return SUP_EINVAL;
  return kernel_time(device_id, total_ms, launches);
}
int sup_rccl_devices(int ndev, int* phys) {
  if (ndev < 1 || ndev > 1024 || !phys) return SUP_EINVAL;
  std::vector<int> devs(ndev), p;
  for (int g = 0; g < ndev; ++g) devs[g] = g;
  if (int rc = rccl_physical_devices(devs, p)) return rc;
  std::copy(p.begin(), p.end(), phys);
  return SUP_OK;
}

int sup_nw_start(const void* mat, sup_dtype t, int n, double* x0, double* p0) {
  if (!x0 || !p0) {
    set_error("null output pointer");
    return SUP_EINVAL;
  }
  std::vector<double> A;
  int rc = to_double(mat, t, n, A);
  if (rc) return rc;
  nw_start(A.data(), n, x0, p0);
  return SUP_OK;
}

// The default layout, or the walk length (m walk bits) sup_opts::walk_log2 asks for.
static Layout layout_for(int n, const sup_opts& o) {
  Layout lay = default_layout(n);
  if (o.walk_log2 > 0) {
    const int rest = n - 1 - lay.L;
    lay.m = std::min(o.walk_log2, rest);
    lay.h = rest - lay.m;
    lay.fixed = true;
  }
  return lay;
}

int sup_perman(const void* mat, sup_dtype t, int n, sup_kernel kernel, sup_sched sched, const sup_opts* o_in,
               double* out, sup_stats* st) {
  auto t0 = std::chrono::steady_clock::now();
  int rc = check_common(mat, n, out);
  if (rc) return rc;
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  std::vector<double> A;
  if ((rc = to_double(mat, t, n, A))) return rc;
  if ((rc = check_walk_opts(o))) return rc;
  const Layout lay = layout_for(n, o);
  std::shared_ptr<const Plan> sp;
  if ((rc = plan_for_shared(A.data(), n, kernel, lay, sp, o.jit, sched == SUP_SCHED_SINGLE ? 1 : o.gpu_num,
                            o.device_id)))
    return rc;
  const Plan& P = *sp;
  SchedResult r;
  if ((rc = schedule(P, sched, o, 0, P.lay.chunks(), r))) return rc;
  *out = (double)(4 * (n & 1) - 2) * r.total;  // gpu_exact_dense.cu:698
  const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fill_stats(st, P, r, wall, 1ull << (n - 1));
  return SUP_OK;
}

int sup_partial(const void* mat, sup_dtype t, int n, sup_kernel kernel, uint64_t start, uint64_t end,
                const sup_opts* o_in, double* out, sup_stats* st) {
  auto t0 = std::chrono::steady_clock::now();
  int rc = check_common(mat, n, out);
  if (rc) return rc;
  const uint64_t space = 1ull << (n - 1);
  if (start > end || end > space) {
    set_error("range [start, end) must satisfy start <= end <= 2^(n-1)");
    return SUP_EINVAL;
  }
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  if ((rc = check_walk_opts(o))) return rc;
  // Largest layout whose wave-chunk (2^(L+m) Gray indices) divides both ends.
  Layout lay = default_layout(n);
  const int nb = n - 1;
  auto align_of = [&](uint64_t v) -> int { return v == 0 || v == space ? nb : __builtin_ctzll(v); };
  const int al = std::min(align_of(start), align_of(end));
  if (al < lay.L) {
    set_error("range ends must be multiples of 2^" + std::to_string(lay.L) + " (one wave of Gray indices)");
    return SUP_EINVAL;
  }
  if (lay.L + lay.m > al) {
    lay.m = al - lay.L;
    lay.h = nb - lay.L - lay.m;
  }
  if (o.walk_log2 > 0 && o.walk_log2 < lay.m) {
    lay.m = o.walk_log2;
    lay.h = nb - lay.L - lay.m;
  }
  std::vector<double> A;
  if ((rc = to_double(mat, t, n, A))) return rc;
  Plan P;
  if ((rc = make_plan(A.data(), n, kind_of(kernel), true, lay, P))) return rc;
  P.lds = kernel == SUP_KERNEL_DENSE_LDS;
  const int cb = lay.L + lay.m;
  SchedResult r;
  if ((rc = schedule(P, o.gpu_num > 1 ? SUP_SCHED_STATIC : SUP_SCHED_SINGLE, o, start >> cb, end >> cb, r)))
    return rc;
  *out = r.total;
  const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fill_stats(st, P, r, wall, end - start);
  return SUP_OK;
}

int sup_perman_cpu(const void* mat, sup_dtype t, int n, sup_kernel kernel, int threads, double* out,
                   sup_stats* st) {
  auto t0 = std::chrono::steady_clock::now();
  int rc = check_common(mat, n, out);
  if (rc) return rc;
  std::vector<double> A;
  if ((rc = to_double(mat, t, n, A))) return rc;
  Plan P;
  if ((rc = plan_for(A.data(), n, kernel, default_layout(n), P))) return rc;
  SchedResult r;
  r.total = cpu_walk_range(P, 0, P.lay.chunks(), threads < 1 ? 1 : threads);
  r.visited = 1ull << (n - 1);
  *out = (double)(4 * (n & 1) - 2) * r.total;
  const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fill_stats(st, P, r, wall, 1ull << (n - 1));
  return SUP_OK;
}

int sup_perman_shard(const void* mat, sup_dtype t, int n, sup_kernel kernel, int shard, int nshards,
                     const sup_opts* o_in, double* out, sup_stats* st) {
  auto t0 = std::chrono::steady_clock::now();
  int rc = check_common(mat, n, out);
  if (rc) return rc;
  if (nshards < 1 || shard < 0 || shard >= nshards) {
    set_error("shard index out of range");
    return SUP_EINVAL;
  }
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  if ((rc = check_walk_opts(o))) return rc;
  std::vector<double> A;
  if ((rc = to_double(mat, t, n, A))) return rc;
  std::shared_ptr<const Plan> sp;
  if ((rc = plan_for_shared(A.data(), n, kernel, layout_for(n, o), sp, o.jit, nshards, o.device_id))) return rc;
  const Plan& P = *sp;
  const uint64_t C = P.lay.chunks();
  const uint64_t c0 = C * (uint64_t)shard / (uint64_t)nshards, c1 = C * (uint64_t)(shard + 1) / (uint64_t)nshards;
  SchedResult r;
  struct DeferTiming {  // sup_opts.timing = 0: this call's walk time is read by sup_kernel_time
    explicit DeferTiming(bool on) { set_defer_timing(on); }
    ~DeferTiming() { set_defer_timing(false); }
  } defer(o.timing == 0);
  if ((rc = schedule(P, SUP_SCHED_SINGLE, o, c0, c1, r))) return rc;
  *out = r.total;
  const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fill_stats(st, P, r, wall, (c1 - c0) << (P.lay.L + P.lay.m));
  return SUP_OK;
}

int sup_perman_exact(const void* mat, sup_dtype t, int n, const sup_opts* o_in, int on_cpu, char* out,
                     size_t out_len, sup_stats* st) {
  auto t0 = std::chrono::steady_clock::now();
  if (!out || out_len < 2) {
    set_error("sup_perman_exact: output buffer missing or too small");
    return SUP_EINVAL;
  }
  std::vector<double> A;
  int rc = to_double(mat, t, n, A);
  if (rc) return rc;
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  std::string s;
  double kms = 0.0;
  int used = 0, cpu_items = 0;
  if ((rc = exact_perman(A.data(), n, o, on_cpu != 0, s, &kms, &used, &cpu_items))) return rc;
  if (s.size() + 1 > out_len) {
    set_error("sup_perman_exact: output buffer too small");
    return SUP_EINVAL;
  }
  std::memcpy(out, s.c_str(), s.size() + 1);
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->kernel_ms = kms;
    st->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    st->gray_steps = 1ull << (n - 1);
    st->visited_steps = st->gray_steps;
    st->devices_used = used;
    st->chunks_done_cpu = cpu_items;
    st->walk_kind = (int)kWalkDense;
    st->leaves = 1;
  }
  return SUP_OK;
}

int sup_perman_quad(const void* mat, sup_dtype t, int n, const sup_opts* o_in, int on_cpu, double* out_hi,
                    double* out_lo, sup_stats* st) {
  auto t0 = std::chrono::steady_clock::now();
  if (!out_hi) {
    set_error("sup_perman_quad: out_hi missing");
    return SUP_EINVAL;
  }
  std::vector<double> A;
  int rc = to_double(mat, t, n, A);
  if (rc) return rc;
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  double hi = 0.0, lo = 0.0, kms = 0.0;
  int used = 0;
  if ((rc = quad_perman(A.data(), n, o, on_cpu != 0, &hi, &lo, &kms, &used))) return rc;
  *out_hi = hi;
  if (out_lo) *out_lo = lo;
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->kernel_ms = kms;
    st->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    st->gray_steps = 1ull << (n - 1);
    st->visited_steps = st->gray_steps;
    st->devices_used = used;
    st->walk_kind = (int)kWalkDense;
    st->leaves = 1;
    st->est_ops_per_step = 16.0 * n + 13.0;
  }
  return SUP_OK;
}

int sup_perman_reduced_exact(const void* mat, sup_dtype t, int n, const sup_opts* o_in, int on_cpu,
                             const sup_reduce_opts* r_in, char* out, size_t out_len, sup_stats* st) {
  auto t0 = std::chrono::steady_clock::now();
  if (!mat || !out || out_len < 2 || n < 1 || n > SUP_MAX_READ_N) {
    set_error("sup_perman_reduced_exact: bad argument");
    return SUP_EINVAL;
  }
  const size_t nn = (size_t)n * n;
  std::vector<double> A(nn);
  for (size_t i = 0; i < nn; ++i)
    A[i] = t == SUP_INT32 ? (double)((const int32_t*)mat)[i]
           : t == SUP_FLOAT32 ? (double)((const float*)mat)[i] : ((const double*)mat)[i];
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  sup_reduce_opts r;
  if (r_in) r = *r_in;
  else sup_reduce_opts_init(&r);
  std::string s;
  double kms = 0.0;
  int leaves = 0, rc;
  if ((rc = exact_perman_reduced(A.data(), n, o, on_cpu != 0, r, s, &kms, &leaves))) return rc;
  if (s.size() + 1 > out_len) {
    set_error("sup_perman_reduced_exact: output buffer too small");
    return SUP_EINVAL;
  }
  std::memcpy(out, s.c_str(), s.size() + 1);
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->kernel_ms = kms;
    st->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    st->leaves = leaves;
    st->walk_kind = (int)kWalkDense;
  }
  return SUP_OK;
}

int sup_plan_info(const void* mat, sup_dtype t, int n, sup_kernel kernel, const sup_opts* o_in, int* walk_kind,
                  int* colmap, int* L, int* m, int* cached_bits, int* pair_bits, double* est_ops_per_step) {
  std::vector<double> A;
  int rc = to_double(mat, t, n, A);
  if (rc) return rc;
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  Plan P;
  if ((rc = check_walk_opts(o))) return rc;
  if ((rc = plan_for(A.data(), n, kernel, layout_for(n, o), P, o.jit, o.gpu_num, o.device_id))) return rc;
  if (walk_kind) *walk_kind = P.lds ? 4 : (int)P.kind;
  if (cached_bits) *cached_bits = P.kind == kWalkSeg ? P.seg_cc : 0;
  if (pair_bits) *pair_bits = P.kind == kWalkSeg ? P.seg_b : 0;
  if (est_ops_per_step) *est_ops_per_step = walk_cost(P);
  if (colmap)
    for (int e = 0; e < n - 1; ++e) colmap[e] = P.colmap[e];
  if (L) *L = P.lay.L;
  if (m) *m = P.lay.m;
  return SUP_OK;
}

int sup_plan_key(const void* mat, sup_dtype t, int n, sup_kernel kernel, const sup_opts* o_in, uint64_t* key) {
  if (!key) {
    set_error("sup_plan_key: key pointer missing");
    return SUP_EINVAL;
  }
  std::vector<double> A;
  int rc = to_double(mat, t, n, A);
  if (rc) return rc;
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  Plan P;
  if ((rc = check_walk_opts(o))) return rc;
  if ((rc = plan_for(A.data(), n, kernel, layout_for(n, o), P, o.jit, o.gpu_num, o.device_id))) return rc;
  *key = plan_fingerprint(P);
  return SUP_OK;
}

int sup_prepare(const void* mat, sup_dtype t, int n, sup_kernel kernel, const sup_opts* o_in, int* walk_kind,
                double* compile_ms) {
  std::vector<double> A;
  int rc = to_double(mat, t, n, A);
  if (rc) return rc;
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  Plan P;
  if ((rc = check_walk_opts(o))) return rc;
  // compiles may already happen while planning (the live-value budget is
  // checked against the compiler), so the time is taken around both
  const double before = jit_compile_ms_thread();
  if ((rc = plan_for(A.data(), n, kernel, layout_for(n, o), P, o.jit, o.gpu_num, o.device_id))) return rc;
  if (walk_kind) *walk_kind = P.lds ? 4 : (int)P.kind;
  if (P.kind == kWalkSeg && (rc = jit_compile_only(P, nullptr))) return rc;
  if (compile_ms) *compile_ms = jit_compile_ms_thread() - before;
  return SUP_OK;
}

// ---- reference-signature wrappers ------------------------------------------
// The reference's sparse wrappers take the caller's CSC (cptrs, rows, cvals)
// and, for SkipPer, CSR (rptrs, cols) next to the dense matrix (built by
// matrix2compressed*, util.h:522-551).  The engine derives its own structure
// from `mat` (touched rows per column, SkipOrder masks), so these arrays must
// describe exactly mat's nonzeros: each column's rows ascending with their
// values, each row's columns ascending.  They are checked, never silently
// ignored: an array built with the reference's `> 0` test (util.h:537,542),
// which drops negative entries, is refused with SUP_EINVAL.
static double entry(const void* mat, sup_dtype t, size_t i) {
  return t == SUP_INT32 ? (double)((const int32_t*)mat)[i]
         : t == SUP_FLOAT32 ? (double)((const float*)mat)[i] : ((const double*)mat)[i];
}

static int check_compressed(const void* mat, sup_dtype t, int n, const int* cptrs, const int* rows,
                            const void* cvals, const int* rptrs, const int* cols) {
  if (!mat || n < 1 || n > SUP_MAX_N) {
    set_error("reference wrapper: null matrix or n outside [1, 64]");
    return SUP_EINVAL;
  }
  if (!cptrs || !rows || !cvals) {
    set_error("reference wrapper: CSC arrays (cptrs, rows, cvals) missing");
    return SUP_EINVAL;
  }
  auto bad = [](const std::string& m) {
    set_error("reference wrapper: " + m + " (build CSR/CSC with sup_compress: nonzero test != 0)");
    return SUP_EINVAL;
  };
  if (cptrs[0] != 0) return bad("cptrs[0] != 0");
  for (int c = 0; c < n; ++c) {
    if (cptrs[c + 1] < cptrs[c]) return bad("cptrs not ascending");
    int want = 0;
    for (int r = 0; r < n; ++r) want += entry(mat, t, (size_t)r * n + c) != 0.0;
    if (cptrs[c + 1] - cptrs[c] != want)
      return bad("column " + std::to_string(c) + " lists " + std::to_string(cptrs[c + 1] - cptrs[c]) +
                 " entries, the matrix has " + std::to_string(want) + " nonzeros");
    for (int k = cptrs[c]; k < cptrs[c + 1]; ++k) {
      const int r = rows[k];
      if (r < 0 || r >= n || (k > cptrs[c] && r <= rows[k - 1])) return bad("CSC rows out of range or order");
      const double v = entry(mat, t, (size_t)r * n + c);
      if (v == 0.0 || entry(cvals, t, (size_t)k) != v)
        return bad("CSC value at (" + std::to_string(r) + ", " + std::to_string(c) + ") differs from the matrix");
    }
  }
  if (rptrs || cols) {
    if (!rptrs || !cols) return bad("CSR arrays incomplete");
    if (rptrs[0] != 0) return bad("rptrs[0] != 0");
    for (int r = 0; r < n; ++r) {
      if (rptrs[r + 1] < rptrs[r]) return bad("rptrs not ascending");
      int want = 0;
      for (int c = 0; c < n; ++c) want += entry(mat, t, (size_t)r * n + c) != 0.0;
      if (rptrs[r + 1] - rptrs[r] != want) return bad("row " + std::to_string(r) + " nonzero count differs");
      for (int k = rptrs[r]; k < rptrs[r + 1]; ++k) {
        const int c = cols[k];
        if (c < 0 || c >= n || (k > rptrs[r] && c <= cols[k - 1]) || entry(mat, t, (size_t)r * n + c) == 0.0)
          return bad("CSR columns out of range, order or pattern");
      }
    }
  }
  return SUP_OK;
}

static int run_ref(const void* mat, sup_dtype t, int nov, sup_kernel k, sup_sched s, int gpu_num, int cpu,
                   int threads, double* out) {
  sup_opts o;
  sup_opts_init(&o);
  o.gpu_num = gpu_num < 1 ? 1 : gpu_num;
  o.cpu_worker = cpu;
  o.threads = threads;
  return sup_perman(mat, t, nov, k, s, &o, out, nullptr);
}

int sup_gpu_perman64_xshared_coalescing_mshared(const void* mat, sup_dtype t, int nov, int, int, double* out) {
  return run_ref(mat, t, nov, SUP_KERNEL_DENSE, SUP_SCHED_SINGLE, 1, 0, 16, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_multigpu(const void* mat, sup_dtype t, int nov, int gpu_num, int,
                                                         int, double* out) {
  return run_ref(mat, t, nov, SUP_KERNEL_DENSE, SUP_SCHED_STATIC, gpu_num, 0, 16, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks(const void* mat, sup_dtype t, int nov,
                                                                   int gpu_num, int cpu, int threads, int, int,
                                                                   double* out) {
  return run_ref(mat, t, nov, SUP_KERNEL_DENSE, SUP_SCHED_CHUNKS, gpu_num, cpu, threads, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_multigpu_manual_distribution(const void* mat, sup_dtype t, int nov,
                                                                             int gpu_num, int, int, double* out) {
  return run_ref(mat, t, nov, SUP_KERNEL_DENSE, SUP_SCHED_MANUAL, gpu_num, 0, 16, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_sparse(const void* mat, const int* cptrs, const int* rows,
                                                       const void* cvals, sup_dtype t, int nov, int, int,
                                                       double* out) {
  int rc = check_compressed(mat, t, nov, cptrs, rows, cvals, nullptr, nullptr);
  return rc ? rc : run_ref(mat, t, nov, SUP_KERNEL_SPARYSER, SUP_SCHED_SINGLE, 1, 0, 16, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_multigpu_sparse(const void* mat, const int* cptrs, const int* rows,
                                                                const void* cvals, sup_dtype t, int nov, int gpu_num,
                                                                int, int, double* out) {
  int rc = check_compressed(mat, t, nov, cptrs, rows, cvals, nullptr, nullptr);
  return rc ? rc : run_ref(mat, t, nov, SUP_KERNEL_SPARYSER, SUP_SCHED_STATIC, gpu_num, 0, 16, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_sparse(const void* mat, const int* cptrs,
                                                                          const int* rows, const void* cvals,
                                                                          sup_dtype t, int nov, int gpu_num, int cpu,
                                                                          int threads, int, int, double* out) {
  int rc = check_compressed(mat, t, nov, cptrs, rows, cvals, nullptr, nullptr);
  return rc ? rc : run_ref(mat, t, nov, SUP_KERNEL_SPARYSER, SUP_SCHED_CHUNKS, gpu_num, cpu, threads, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_multigpu_sparse_manual_distribution(const void* mat, const int* cptrs,
                                                                                    const int* rows, const void* cvals,
                                                                                    sup_dtype t, int nov, int gpu_num,
                                                                                    int, int, double* out) {
  int rc = check_compressed(mat, t, nov, cptrs, rows, cvals, nullptr, nullptr);
  return rc ? rc : run_ref(mat, t, nov, SUP_KERNEL_SPARYSER, SUP_SCHED_MANUAL, gpu_num, 0, 16, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_skipper(const void* mat, const int* rptrs, const int* cols,
                                                        const int* cptrs, const int* rows, const void* cvals,
                                                        sup_dtype t, int nov, int, int, double* out) {
  int rc = check_compressed(mat, t, nov, cptrs, rows, cvals, rptrs, cols);
  return rc ? rc : run_ref(mat, t, nov, SUP_KERNEL_SKIPPER, SUP_SCHED_SINGLE, 1, 0, 16, out);
}
int sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_skipper(const void* mat, const int* rptrs,
                                                                           const int* cols, const int* cptrs,
                                                                           const int* rows, const void* cvals,
                                                                           sup_dtype t, int nov, int gpu_num, int cpu,
                                                                           int threads, int, int, double* out) {
  int rc = check_compressed(mat, t, nov, cptrs, rows, cvals, rptrs, cols);
  return rc ? rc : run_ref(mat, t, nov, SUP_KERNEL_SKIPPER, SUP_SCHED_CHUNKS, gpu_num, cpu, threads, out);
}


// ---- reductions + engine (sup_decompose with engine leaves) ----------------
namespace {
struct LeafCtx {
  sup_kernel kernel;
  sup_sched sched;
  sup_opts o;
  int on_cpu;
  int preprocessing;
  sup_stats acc;
  bool first = true;
};

int leaf_compute(const LeafCtx& c, const double* a, int n, double* out, sup_stats* st) {
  std::vector<double> m(a, a + (size_t)n * n);
  std::vector<int> rp(n), cp(n);
  int rc = SUP_OK;
  // main.cpp:983-988: every leaf's CSR/CSC is built with the -r order
  if (c.preprocessing == 1) rc = sup_sort_order(m.data(), SUP_FLOAT64, n, cp.data());
  else if (c.preprocessing == 2) rc = sup_skip_order(m.data(), SUP_FLOAT64, n, rp.data(), cp.data());
  if (rc) return rc;
  return c.on_cpu ? sup_perman_cpu(m.data(), SUP_FLOAT64, n, c.kernel, c.o.threads, out, st)
                  : sup_perman(m.data(), SUP_FLOAT64, n, c.kernel, c.sched, &c.o, out, st);
}

// Whether the leaves of this request may share launches (run_range_batch):
// one device, the single-device schedule, a kernel request the batch kernels
// serve, and no checkpoint.  Leaves whose plan turns out otherwise (a
// segmented or SkipPer plan) still go one at a time.
int leaf_workers();
int leaf_batch_max();
bool leaf_batching(const LeafCtx& c) {
  if (leaf_batch_max() <= 1) return false;
  return !c.on_cpu && c.sched == SUP_SCHED_SINGLE && c.o.use_rccl <= 0 && !(c.o.checkpoint && *c.o.checkpoint) &&
         (c.kernel == SUP_KERNEL_DENSE || c.kernel == SUP_KERNEL_SPARYSER || c.kernel == SUP_KERNEL_DENSE_PLAIN);
}
// Default: batches of 16.  Measured on dwt_59 (145,798 n = 30 leaves, one
// MI355X): round 4, one worker 65.2 s -> 46.7 s with batches of 16, but with 8
// workers the concurrent one-leaf launches filled the GPU (37.8 s against
// 39.6 s batched), so batches were for one worker only.  Since round 5 the
// prefix-blocked walk ends ~64 % of these leaves' chunks at their first state
// (walk_sparse.hip): the leaves are short, launches and host planning weigh
// more, and batches win at every worker count — 8 workers 17.9 s one leaf per
// launch, 12.7 s batched; one worker 48.1 s / 16.8 s
// (profiles/r5/probe_reduce_chunk_ends.log).
int leaf_batch_max() {
  const char* e = std::getenv("SUP_LEAF_BATCH");
  if (e) return std::max(1, std::min(kMaxBatchLeaves, std::atoi(e)));
  return 16;
}

// Several leaves of order n: each planned as sup_perman plans it (the same
// plan, so the same bits), the batchable ones walked in one launch, the rest
// one at a time through sup_perman.
// A batch of leaves planned on the host (leaf_plan_batch), walked later
// (leaf_walk_batch), so a worker can plan the next batch while this one walks
// (decompose_batched_staged).  Each leaf is planned as sup_perman plans it
// (the same plan, so the same bits); the batchable ones walk in one launch,
// the rest one at a time through sup_perman.
struct LeafBatchState {
  int n = 0;
  std::vector<std::vector<double>> ms;
  std::vector<std::shared_ptr<const Plan>> plans;
  std::vector<double*> outs;
  std::chrono::steady_clock::time_point t0;
};

int leaf_plan_batch(const LeafCtx& c, const std::vector<const double*>& mats, int n, const std::vector<double*>& outs,
                    LeafBatchState& b) {
  b.t0 = std::chrono::steady_clock::now();
  const size_t K = mats.size();
  b.n = n;
  b.outs = outs;
  b.ms.assign(K, {});
  b.plans.assign(K, nullptr);
  const Layout lay = layout_for(n, c.o);
  int rc = check_walk_opts(c.o);
  if (rc) return rc;
  for (size_t i = 0; i < K; ++i) {
    b.ms[i].assign(mats[i], mats[i] + (size_t)n * n);
    std::vector<int> rp(n), cp(n);
    if (c.preprocessing == 1) rc = sup_sort_order(b.ms[i].data(), SUP_FLOAT64, n, cp.data());
    else if (c.preprocessing == 2) rc = sup_skip_order(b.ms[i].data(), SUP_FLOAT64, n, rp.data(), cp.data());
    if (rc) return rc;
    // batch leaves stay out of the process plan cache (32 entries): two batches of 16 would evict the
    // caller's plans; a repeated leaf is served by the reduction's leaf memo
    if ((rc = plan_for_shared(b.ms[i].data(), n, c.kernel, lay, b.plans[i], c.o.jit, 1, c.o.device_id, false)))
      return rc;
  }
  return SUP_OK;
}

int leaf_walk_batch(const LeafCtx& c, const LeafBatchState& b, sup_stats* st) {
  const size_t K = b.ms.size();
  const int n = b.n;
  const auto& ms = b.ms;
  const auto& plans = b.plans;
  const auto& outs = b.outs;
  const auto t0 = b.t0;
  int rc = SUP_OK;
  std::memset(st, 0, sizeof(*st));
  const double sign = (double)(4 * (n & 1) - 2);  // gpu_exact_dense.cu:698
  std::vector<const Plan*> group;
  std::vector<size_t> gi;
  double kms = 0.0;
  uint64_t steps = 0;
  for (size_t i = 0; i < K; ++i) {
    if (K > 1 && batchable(*plans[i], *plans[i])) {
      if (group.empty() || batchable(*group[0], *plans[i])) {
        group.push_back(plans[i].get());
        gi.push_back(i);
        continue;
      }
    }
    sup_stats one;  // not batchable with the group: on its own, as before
    if ((rc = sup_perman(ms[i].data(), SUP_FLOAT64, n, c.kernel, c.sched, &c.o, outs[i], &one))) return rc;
    kms += one.kernel_ms;
    steps += one.gray_steps;
    st->walk_kind = one.walk_kind;
  }
  if (!group.empty()) {
    std::vector<double> part;
    double ms_b = 0.0;
    if ((rc = run_range_batch(c.o.device_id, group, part, &ms_b))) return rc;
    for (size_t q = 0; q < gi.size(); ++q) *outs[gi[q]] = sign * part[q];
    kms += ms_b;
    steps += (uint64_t)gi.size() << (n - 1);
    st->walk_kind = (int)group[0]->kind;
    st->lane_bits = group[0]->lay.L;
    st->walk_bits = group[0]->lay.m;
    st->est_ops_per_step = walk_cost(*group[0]);
  }
  st->kernel_ms = kms;
  st->gray_steps = steps;
  st->visited_steps = steps;
  st->devices_used = 1;
  st->leaves = (int)K;
  st->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SUP_OK;
}


void leaf_accumulate(LeafCtx& c, const sup_stats& st) {
  if (c.first) {
    c.acc = st;
    c.first = false;
  } else {
    const sup_stats prev = c.acc;
    c.acc = st;
    c.acc.kernel_ms += prev.kernel_ms;
    c.acc.wall_ms += prev.wall_ms;
    c.acc.gray_steps += prev.gray_steps;
    c.acc.visited_steps += prev.visited_steps;
    c.acc.leaves += prev.leaves;
  }
}

// Concurrent GPU leaves of sup_perman_reduced: one per context lane (8; dwt_59's
// 145,798 n = 30 leaves: 85 s one at a time, 41 s with 4, 39 s with 8,
// profiles/r3/probe_reduce_memo.log).  SUP_LEAF_WORKERS overrides; 1 = one leaf
// at a time, as the reference's RunAlgo per leaf.
int leaf_workers() {
  const char* e = std::getenv("SUP_LEAF_WORKERS");
  return e ? std::max(1, std::min(kCtxLanes, std::atoi(e))) : kCtxLanes;
}

}  // namespace

int sup_perman_reduced_quad(const void* mat, sup_dtype t, int n, const sup_opts* o_in, int on_cpu,
                            const sup_reduce_opts* r_in, double* out_hi, double* out_lo, sup_stats* st) {
  auto t0 = std::chrono::steady_clock::now();
  if (!mat || !out_hi || n < 1 || n > SUP_MAX_READ_N) {
    set_error("sup_perman_reduced_quad: bad argument");
    return SUP_EINVAL;
  }
  std::vector<double> A((size_t)n * n);
  for (size_t i = 0; i < A.size(); ++i)
    A[i] = t == SUP_INT32 ? (double)((const int32_t*)mat)[i]
           : t == SUP_FLOAT32 ? (double)((const float*)mat)[i] : ((const double*)mat)[i];
  sup_opts o;
  if (o_in) o = *o_in;
  else sup_opts_init(&o);
  sup_reduce_opts r;
  if (r_in) r = *r_in;
  else sup_reduce_opts_init(&r);
  double kms = 0.0;
  int used = 0;
  std::mutex mu;
  // GPU leaves several at a time on their own context lanes (as sup_perman_reduced)
  auto leaf = [&](int w, const double* a, int k, dd* v) {
    set_ctx_lane(w);
    double ms = 0.0;
    int u = 0;
    const int rc = quad_perman(a, k, o, on_cpu != 0, &v->hi, &v->lo, &ms, &u);
    std::lock_guard<std::mutex> g(mu);
    kms += ms;
    used = std::max(used, u);
    return rc;
  };
  dd v{0.0, 0.0};
  int leaves = 0;
  const int rc = decompose_dd_batched(A.data(), n, r, on_cpu ? 1 : leaf_workers(), leaf, &v, &leaves);
  if (rc) return rc;
  *out_hi = v.hi;
  if (out_lo) *out_lo = v.lo;
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->kernel_ms = kms;
    st->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    st->devices_used = used;
    st->walk_kind = (int)kWalkDense;
    st->leaves = leaves;
  }
  return SUP_OK;
}

int sup_perman_reduced(const void* mat, sup_dtype t, int n, sup_kernel kernel, sup_sched sched, const sup_opts* o_in,
                       int on_cpu, const sup_reduce_opts* r_in, double* out, sup_stats* st) {
  LeafCtx c;
  c.kernel = kernel;
  c.sched = sched;
  if (o_in) c.o = *o_in;
  else sup_opts_init(&c.o);
  if (c.o.checkpoint && *c.o.checkpoint) {  // one file per computation; a reduction runs many
    set_error("sup_perman_reduced: checkpoint files are for one permanent (sup_perman with SUP_SCHED_CHUNKS)");
    return SUP_EUNSUPPORTED;
  }
  c.on_cpu = on_cpu;
  sup_reduce_opts r;
  if (r_in) r = *r_in;
  else sup_reduce_opts_init(&r);
  c.preprocessing = r.preprocessing;
  std::memset(&c.acc, 0, sizeof(c.acc));
  int leaves = 0;
  // GPU leaves: leaf_workers() host threads, each on its own context lane of
  // the devices (stream, buffers), so one leaf's planning, uploads, launch
  // gaps and sync overlap the others' walks; host leaves (-c) one at a time
  // (each uses the -t threads).  Same result bits either way: the combine is
  // folded in the sequential order (decompose_batched).
  if (!mat || !out || n < 1 || n > SUP_MAX_READ_N) {
    set_error("sup_perman_reduced: bad argument");
    return SUP_EINVAL;
  }
  std::vector<double> A((size_t)n * n);
  for (size_t i = 0; i < A.size(); ++i)
    A[i] = t == SUP_INT32 ? (double)((const int32_t*)mat)[i]
           : t == SUP_FLOAT32 ? (double)((const float*)mat)[i] : ((const double*)mat)[i];
  std::mutex smu;
  // leaves in batches of up to leaf_batch_max() per launch (run_range_batch),
  // else one at a time; either way the same bits
  const int rc =
      leaf_batching(c)
          // two stages: a worker plans its next batch while its walker thread walks this one
          ? decompose_batched_staged(
                A.data(), n, r, leaf_workers(), leaf_batch_max(),
                [&c, &smu](int w, const std::vector<const double*>& as, int k, const std::vector<double*>& vs,
                           std::function<int()>& walk) {
                  set_ctx_lane(w);
                  auto b = std::make_shared<LeafBatchState>();
                  if (const int e = leaf_plan_batch(c, as, k, vs, *b)) return e;
                  walk = [&c, &smu, b, w]() {
                    set_ctx_lane(w);
                    sup_stats st;
                    if (const int e = leaf_walk_batch(c, *b, &st)) return e;
                    std::lock_guard<std::mutex> g(smu);
                    leaf_accumulate(c, st);
                    return SUP_OK;
                  };
                  return SUP_OK;
                },
                out, &leaves)
          : decompose_batched(A.data(), n, r, c.on_cpu ? 1 : leaf_workers(),
                              [&c, &smu](int w, const double* a, int k, double* v) {
                                set_ctx_lane(w);
                                sup_stats st;
                                const int e = leaf_compute(c, a, k, v, &st);
                                if (e) return e;
                                std::lock_guard<std::mutex> g(smu);
                                leaf_accumulate(c, st);
                                return SUP_OK;
                              },
                              out, &leaves);
  if (rc) return rc;
  if (st) {
    *st = c.acc;
    st->leaves = leaves;
  }
  return SUP_OK;
}

}  // extern "C"
