// perman_main.cpp — the `perman` command line, a drop-in for the reference's
// v1 CLI (main.cu:325-600): same short/long options, same algorithm ids, same
// "Result: <name> <perm> in <sec>" line (cout default precision), plus a
// full-precision "Permanent: %.17e" line (the legacy line has ~6 digits).
//
// Extensions (v2 semantics, revised_perman/main.cpp:1298-1476): -l <dev>
// first device, -k <reps> repetitions, -o compression (d1/d2 singletons, then
// the d1/d2/d34 expansion while n > 30), -u <t> scaling; MatrixMarket input
// (detected by its banner, read as main.cpp:1515-1615).  Own additions: -R
// insist on the RCCL combine of multi-GPU partials (by default it runs
// whenever the -d devices are distinct GPUs, else the host pairwise tree); -v per-kernel / per-chunk timing;
// --seed (-S) the estimators' Philox seed (-a / -i; the reference seeds with
// time(0), so its estimates are not reproducible); --jit (-J) <-1|0|1> the
// pattern-specialised segmented walk (sup_opts.jit: never / auto / whenever
// its cost model wins); --exact (-E) the exact integer permanent of an int /
// -b (binary) matrix (sup_perman_exact: residue walk + CRT; the reference's
// int path is fp64): on -g with -p5/-p6 it uses -d devices, with -c alone
// the -t host threads.  -q (v2's quad calculation, main.cpp:141-142): the
// dense walk in double-double (sup_perman_quad), -d devices with -p5/-p6,
// -t host threads with -c; with -o / -u every leaf and the combine in
// double-double (sup_perman_reduced_quad); prints hi and the hi + lo pair.
#include <getopt.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/superman.h"

namespace {

struct Cli {
  bool generic = true, dense = true, approximation = false, gpu = false, cpu = false, grid_graph = false;
  bool rccl = false, verbose = false, compression = false, exact = false, quad = false;
  bool half_calc = false, half_store = false;
  int gpu_num = 2, threads = 16, perman_algo = 1, preprocessing = 0, device = 0, reps = 1;
  double scaling = -1.0;
  long number_of_times = 100000;  // main.cu:338-344 defaults
  int scale_intervals = 4, scale_times = 5, gridm = 36, gridn = 36;
  unsigned long long seed = 1;
  int jit = 0;
  std::string filename, checkpoint;
};

int fail(const char* what) {
  std::fprintf(stderr, "perman: %s: %s\n", what, sup_last_error());
  return 1;
}

void report(const std::string& name, double perm, double sec) {
  std::cout << "Result: " << name << " " << perm << " in " << sec << std::endl;
  std::printf("Permanent: %.17e\n", perm);
  std::fflush(stdout);
}

// main.cu:77-103, 156-183 (GPU) and 193-243 (CPU) approximation dispatch;
// main.cu:250-320 RunPermanForGridGraphs (sparse names, -i -m -n).
int run_approx(const Cli& c) {
  void* mat = nullptr;
  sup_dtype t = SUP_INT32;
  int n = 0, nnz = 0;
  if (c.grid_graph) {
    int* g = nullptr;
    if (sup_grid_graph(c.gridm, c.gridn, &g, &n) != SUP_OK) return fail("grid graph");
    mat = g;
  } else if (sup_read_matrix(c.filename.c_str(), c.generic ? 0 : 1, &mat, &t, &n, &nnz) != SUP_OK) {
    return fail("reading matrix");
  }
  const bool sparse = c.grid_graph || !c.dense;
  const int a = c.perman_algo;
  std::string name;
  int method = 0;
  bool multi = false;
  if (c.gpu) {
    static const char* dn[] = {"", "gpu_perman64_rasmussen", "gpu_perman64_approximation",
                               "gpu_perman64_rasmussen_multigpucpu_chunks",
                               "gpu_perman64_approximation_multigpucpu_chunks"};
    if (a < 1 || a > 4) {
      std::cout << "Unknown Algorithm ID" << std::endl;
      sup_free(mat);
      return 0;
    }
    name = std::string(dn[a]) + (sparse ? "_sparse" : "");
    method = (a == 2 || a == 4) ? 1 : 0;
    multi = a >= 3;
  } else {
    if (a != 1 && a != 2) {
      std::cout << "Unknown Algorithm ID" << std::endl;
      sup_free(mat);
      return 0;
    }
    name = std::string(a == 1 ? "rasmussen" : "approximation_perman64") + (sparse ? "_sparse" : "");
    method = a - 1;
  }
  sup_opts o;
  sup_opts_init(&o);
  o.gpu_num = multi ? c.gpu_num : 1;
  o.device_id = c.device;
  o.threads = c.threads;
  o.cpu_worker = (multi && c.cpu) ? 1 : 0;
  for (int r = 0; r < c.reps; ++r) {
    sup_approx_result res;
    auto t0 = std::chrono::steady_clock::now();
    const int rc = sup_approx(mat, t, n, method, (uint64_t)std::max(1L, c.number_of_times), c.scale_intervals,
                              c.scale_times, c.seed + (unsigned long long)r, &o, c.gpu ? 0 : 1, &res);
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc != SUP_OK) {
      sup_free(mat);
      return fail(name.c_str());
    }
    const char* tag = c.grid_graph ? "Try" : "Result";
    std::printf("Result: %s %2lf in %lf\n", name.c_str(), res.mean, sec);
    std::cout << tag << ": " << name << " " << res.mean << " in " << sec << std::endl;
    std::printf("Permanent: %.17e\nStdError: %.6e samples %llu zeros %.4f\n", res.mean, res.std_error,
                (unsigned long long)res.samples, res.zero_fraction);
    std::fflush(stdout);
  }
  sup_free(mat);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  Cli c;
  const char* const short_options = "bsr:t:f:gd:cap:x:y:z:im:n:l:k:Rvou:S:J:Eqhwe:";
  const struct option long_options[] = {{"binary", 0, NULL, 'b'},       {"sparse", 0, NULL, 's'},
                                        {"preprocessing", 1, NULL, 'r'}, {"threads", 1, NULL, 't'},
                                        {"file", 1, NULL, 'f'},          {"gpu", 0, NULL, 'g'},
                                        {"device", 1, NULL, 'd'},        {"cpu", 0, NULL, 'c'},
                                        {"approximation", 0, NULL, 'a'}, {"perman", 1, NULL, 'p'},
                                        {"numOfTimes", 1, NULL, 'x'},    {"scaleIntervals", 1, NULL, 'y'},
                                        {"scaleTimes", 1, NULL, 'z'},    {"grid", 0, NULL, 'i'},
                                        {"gridm", 1, NULL, 'm'},         {"gridn", 1, NULL, 'n'},
                                        {"gpu-id", 1, NULL, 'l'},        {"reps", 1, NULL, 'k'},
                                        {"rccl", 0, NULL, 'R'},          {"verbose", 0, NULL, 'v'},
                                        {"compression", 0, NULL, 'o'},   {"scaling", 1, NULL, 'u'},
                                        {"seed", 1, NULL, 'S'},          {"jit", 1, NULL, 'J'},
                                        {"exact", 0, NULL, 'E'},         {"quad", 0, NULL, 'q'},
                                        {"halfCalc", 0, NULL, 'h'},      {"halfStore", 0, NULL, 'w'},
                                        {"gridMultip", 1, NULL, 'e'},    {"checkpoint", 1, NULL, 'C'},
                                        {NULL, 0, NULL, 0}};
  int opt;
  auto need_arg = [&](char o) -> bool {
    if (optarg[0] == '-') {
      std::fprintf(stderr, "Option -%c requires an argument.\n", o);
      return false;
    }
    return true;
  };
  while ((opt = getopt_long(argc, argv, short_options, long_options, NULL)) != -1) {
    switch (opt) {
      case 'b': c.generic = false; break;
      case 's': c.dense = false; break;
      case 'r': if (!need_arg('t')) return 1; c.preprocessing = std::atoi(optarg); break;
      case 't': if (!need_arg('t')) return 1; c.threads = std::atoi(optarg); break;
      case 'f': if (!need_arg('f')) return 1; c.filename = optarg; break;
      case 'a': c.approximation = true; break;
      case 'g': c.gpu = true; break;
      case 'd': if (!need_arg('d')) return 1; c.gpu_num = std::atoi(optarg); break;
      case 'c': c.cpu = true; break;
      case 'p': if (!need_arg('p')) return 1; c.perman_algo = std::atoi(optarg); break;
      case 'x': if (!need_arg('x')) return 1; c.number_of_times = std::atol(optarg); break;
      case 'y': if (!need_arg('y')) return 1; c.scale_intervals = std::atoi(optarg); break;
      case 'z': if (!need_arg('z')) return 1; c.scale_times = std::atoi(optarg); break;
      case 'm': if (!need_arg('m')) return 1; c.gridm = std::atoi(optarg); break;
      case 'n': if (!need_arg('n')) return 1; c.gridn = std::atoi(optarg); break;
      case 'S': if (!need_arg('S')) return 1; c.seed = std::strtoull(optarg, nullptr, 10); break;
      case 'J': c.jit = std::atoi(optarg); break;  // may be negative: no need_arg
      case 'C': if (!need_arg('C')) return 1; c.checkpoint = optarg; break;  // -p6 / -p8: resumable
      case 'i': c.grid_graph = true; break;
      case 'l': if (!need_arg('l')) return 1; c.device = std::atoi(optarg); break;
      case 'k': if (!need_arg('k')) return 1; c.reps = std::max(1, std::atoi(optarg)); break;
      case 'R': c.rccl = true; break;
      case 'E': c.exact = true; break;
      case 'q': c.quad = true; break;
      case 'v': c.verbose = true; break;
      // v2 flags (revised_perman/main.cpp:1431-1460): -w stores the matrix in
      // single precision (the permanent of the float-rounded entries); -h asks
      // for single-precision calculation, which this engine does not provide
      // (float X loses every digit at n >= 30): computed in fp64,
      // with a note; -e <multiplier> scales the reference's launch grid, which
      // the engine sizes from the occupancy itself: accepted, no effect.  (v2's
      // -v, quad storage, is this CLI's verbose flag: fp64 storage rounds an
      // entry by at most 2^-53 relative, below the walk's own rounding.)
      case 'h': c.half_calc = true; break;
      case 'w': c.half_store = true; break;
      case 'e': if (!need_arg('e')) return 1; break;
      case 'o': c.compression = true; break;  // revised_perman/main.cpp:1462
      case 'u':                                // main.cpp:1465 (atoi)
        if (!need_arg('u')) return 1;
        c.scaling = (double)std::atoi(optarg);
        break;
      case '?': return 1;
      default: std::abort();
    }
  }
  if (!c.grid_graph && c.filename.empty()) {
    std::fprintf(stderr, "Option -f is a required argument.\n");
    return 1;
  }
  for (int i = optind; i < argc; ++i) std::printf("Non-option argument %s\n", argv[i]);
  if (!c.cpu && !c.gpu) c.gpu = true;  // main.cu:482-484
  if (c.grid_graph || c.approximation) return run_approx(c);

  void* mat = nullptr;
  sup_dtype t;
  int n = 0, nnz = 0;
  if (sup_read_matrix(c.filename.c_str(), c.generic ? 0 : 1, &mat, &t, &n, &nnz) != SUP_OK)
    return fail("reading matrix");
  if (c.half_store && t == SUP_FLOAT64) {  // v2 -w: single-precision storage
    double* d = (double*)mat;
    float* f = (float*)std::malloc(sizeof(float) * (size_t)n * n);
    if (!f) return fail("allocating the single-precision matrix");
    for (size_t i = 0; i < (size_t)n * n; ++i) f[i] = (float)d[i];
    sup_free(mat);
    mat = f;
    t = SUP_FLOAT32;
  }
  if (c.half_calc)
    std::fprintf(stderr, "perman: -h (single-precision calculation) is computed in fp64 by this engine\n");
  // main.cu:512-518 / 544-550 / 577-583: preprocessing rewrites mat (with
  // -o / -u it is applied to every leaf of the reductions instead).
  const bool reduce = c.compression || c.scaling > 0.0;
  sup_reduce_opts ro;
  sup_reduce_opts_init(&ro);
  ro.compress = c.compression ? 1 : 0;
  ro.scale_threshold = c.scaling > 0.0 ? c.scaling : 0.0;
  ro.preprocessing = c.preprocessing;
  std::vector<int> rp(n), cp(n);
  if (!reduce && c.preprocessing == 1) {
    if (sup_sort_order(mat, t, n, cp.data()) != SUP_OK) return fail("SortOrder");
  } else if (!reduce && c.preprocessing == 2) {
    if (sup_skip_order(mat, t, n, rp.data(), cp.data()) != SUP_OK) return fail("SkipOrder");
  }

  sup_opts o;
  sup_opts_init(&o);
  o.gpu_num = c.gpu_num;
  o.device_id = c.device;
  o.threads = c.threads;
  o.cpu_worker = (c.gpu && c.cpu) ? 1 : 0;
  // multi-device partials: RCCL whenever the devices are distinct GPUs (-1),
  // -R insists on it (an error when SUP_DEVICE_MAP shares a GPU)
  o.use_rccl = c.rccl ? 1 : -1;
  o.verbose = c.verbose ? 1 : 0;
  o.jit = c.jit;
  o.checkpoint = c.checkpoint.empty() ? nullptr : c.checkpoint.c_str();

  if (c.exact) {  // exact integer permanent (any -p: the sum does not depend on the kernel)
    if (c.scaling > 0.0) {
      std::fprintf(stderr, "perman: --exact does not combine with -u (scaling is not exact)\n");
      sup_free(mat);
      return 1;
    }
    if (c.gpu && c.perman_algo != 5 && c.perman_algo != 6 && c.perman_algo != 8) o.gpu_num = 1;
    if (c.perman_algo != 6 && c.perman_algo != 8) o.cpu_worker = 0;  // the hybrid worker joins the queues only
    static char buf[1 << 16];
    sup_stats st;
    int rc = SUP_OK;
    const auto t0 = std::chrono::steady_clock::now();
    for (int rep = 0; rep < c.reps && rc == SUP_OK; ++rep)
      rc = reduce ? sup_perman_reduced_exact(mat, t, n, &o, c.gpu ? 0 : 1, &ro, buf, sizeof buf, &st)
                  : sup_perman_exact(mat, t, n, &o, c.gpu ? 0 : 1, buf, sizeof buf, &st);
    const double sec =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / (double)c.reps;
    sup_free(mat);
    if (rc != SUP_OK) return fail("exact permanent");
    std::cout << "Result: " << (c.gpu ? "gpu_perman64_exact_residue" : "cpu_perman64_exact_residue") << " " << buf
              << " in " << sec << std::endl;
    std::printf("Permanent: %s\n", buf);
    if (c.verbose)
      std::printf("Stats: devices %d kernel_ms %.3f wall_ms %.3f cpu_items %d\n", st.devices_used, st.kernel_ms,
                  st.wall_ms, st.chunks_done_cpu);
    return 0;
  }

  if (c.quad) {  // double-double dense walk (any -p: the sum does not depend on the kernel)
    if (c.gpu && c.perman_algo != 5 && c.perman_algo != 6 && c.perman_algo != 8) o.gpu_num = 1;
    double hi = 0.0, lo = 0.0;
    sup_stats st;
    int rc = SUP_OK;
    const auto t0 = std::chrono::steady_clock::now();
    for (int rep = 0; rep < c.reps && rc == SUP_OK; ++rep)
      rc = reduce ? sup_perman_reduced_quad(mat, t, n, &o, c.gpu ? 0 : 1, &ro, &hi, &lo, &st)
                  : sup_perman_quad(mat, t, n, &o, c.gpu ? 0 : 1, &hi, &lo, &st);
    const double sec =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / (double)c.reps;
    sup_free(mat);
    if (rc != SUP_OK) return fail("double-double permanent");
    std::cout << "Result: " << (c.gpu ? "gpu_perman64_quad" : "cpu_perman64_quad") << " " << hi << " in " << sec
              << std::endl;
    std::printf("Permanent: %.17e\n", hi);
    std::printf("Permanent (double-double): %.17e %+.17e\n", hi, lo);
    if (c.verbose)
      std::printf("Stats: devices %d kernel_ms %.3f wall_ms %.3f\n", st.devices_used, st.kernel_ms, st.wall_ms);
    return 0;
  }

  std::string name;
  sup_kernel kern = SUP_KERNEL_DENSE;
  sup_sched sched = SUP_SCHED_SINGLE;
  bool on_gpu = c.gpu;
  const int a = c.perman_algo;
  if (on_gpu) {
    // main.cu:30-143 GPU exact dispatch
    if (c.dense) {
      static const char* names[] = {"gpu_perman64_xglobal", "gpu_perman64_xlocal", "gpu_perman64_xshared",
                                    "gpu_perman64_xshared_coalescing",
                                    "gpu_perman64_xshared_coalescing_mshared"};
      if (a >= 0 && a <= 4) {
        name = names[a];
      } else if (a == 5) {
        name = "gpu_perman64_xshared_coalescing_mshared_multigpu";
        sched = SUP_SCHED_STATIC;
      } else if (a == 6) {
        name = "gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks";
        sched = SUP_SCHED_CHUNKS;
      } else if (a == 66) {
        name = "gpu_perman64_xshared_coalescing_mshared_multigpu_manual_distribution";
        sched = SUP_SCHED_MANUAL;
        o.gpu_num = 4;  // main.cu:75 hard-codes 4 devices
      } else {
        std::cout << "Unknown Algorithm ID" << std::endl;
        sup_free(mat);
        return 0;
      }
    } else {
      static const char* names[] = {"", "gpu_perman64_xlocal_sparse", "gpu_perman64_xshared_sparse",
                                    "gpu_perman64_xshared_coalescing_sparse",
                                    "gpu_perman64_xshared_coalescing_mshared_sparse"};
      kern = SUP_KERNEL_SPARYSER;
      if (a >= 1 && a <= 4) {
        name = names[a];
      } else if (a == 5) {
        name = "gpu_perman64_xshared_coalescing_mshared_multigpu_sparse";
        sched = SUP_SCHED_STATIC;
      } else if (a == 6) {
        name = "gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_sparse";
        sched = SUP_SCHED_CHUNKS;
      } else if (a == 7) {
        name = "gpu_perman64_xshared_coalescing_mshared_skipper";
        kern = SUP_KERNEL_SKIPPER;
      } else if (a == 8) {
        name = "gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_skipper";
        kern = SUP_KERNEL_SKIPPER;
        sched = SUP_SCHED_CHUNKS;
      } else if (a == 66) {
        name = "gpu_perman64_xshared_coalescing_mshared_multigpu_sparse_manual_distribution";
        sched = SUP_SCHED_MANUAL;
        o.gpu_num = 4;
      } else {
        std::cout << "Unknown Algorithm ID" << std::endl;
        sup_free(mat);
        return 0;
      }
    }
    if (sched == SUP_SCHED_SINGLE) o.gpu_num = 1;
  } else {
    // main.cu:186-238 CPU exact dispatch (dense ignores -p, main.cu:188)
    if (c.dense) {
      name = "parallel_perman64";
    } else if (a == 1) {
      name = "parallel_perman64_sparse";
      kern = SUP_KERNEL_SPARYSER;
    } else if (a == 2 || a == 3) {
      name = a == 2 ? "parallel_skip_perman64_w" : "parallel_skip_perman64_w_balanced";
      kern = SUP_KERNEL_SKIPPER;
    } else {
      sup_free(mat);
      return 0;  // the reference prints nothing for other sparse CPU ids
    }
  }

  // HIP initialisation, the device contexts and the walk code objects on a
  // thread beside the planning sup_perman does first on the host (a cold
  // segmented plan is ~1 s of search and compiles): the walk then starts on a
  // warm runtime.  Its errors surface again in the call itself.
  std::thread warm;
  if (on_gpu) warm = std::thread([&o, n] { (void)sup_device_warmup(o.device_id, o.gpu_num, n); });
  struct Join {
    std::thread& t;
    ~Join() {
      if (t.joinable()) t.join();
    }
  } join_warm{warm};
  for (int r = 0; r < c.reps; ++r) {
    double perm = 0.0;
    sup_stats st;
    auto t0 = std::chrono::steady_clock::now();
    int rc = reduce   ? sup_perman_reduced(mat, t, n, kern, sched, &o, on_gpu ? 0 : 1, &ro, &perm, &st)
             : on_gpu ? sup_perman(mat, t, n, kern, sched, &o, &perm, &st)
                      : sup_perman_cpu(mat, t, n, kern, c.threads, &perm, &st);
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc != SUP_OK) {
      sup_free(mat);
      return fail(name.c_str());
    }
    report(name, perm, sec);
    if (c.verbose)
      std::printf("Stats: kernel_ms %.3f gray_steps %llu visited %llu devices %d lanes %d walk %d grid %d leaves %d "
                  "walk_kind %d ops_per_step %.1f jit_ms %.1f cpu_items %d device_checks %llu\n",
                  st.kernel_ms, (unsigned long long)st.gray_steps, (unsigned long long)st.visited_steps,
                  st.devices_used, st.lane_bits, st.walk_bits, st.grid, st.leaves, st.walk_kind, st.est_ops_per_step,
                  st.jit_ms, st.chunks_done_cpu, (unsigned long long)sup_device_checks());
  }
  sup_free(mat);
  return 0;
}
