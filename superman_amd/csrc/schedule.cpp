// schedule.cpp — the multi-device schedulers of the engine (reference
// gpu_perman64_*_multigpu / _multigpucpu_chunks / _manual_distribution,
// gpu_exact_dense.cu:701-990, gpu_exact_sparse.cu:916-1121, 1192-1400): the
// static split, the dynamic chunk queue with the hybrid CPU worker, the manual
// distribution; the RCCL combine of device partials; checkpoint / resume of
// the queue.  The reference sums device partials on the host after OpenMP
// threads (gpu_exact_dense.cu:847-901).
#include "engine.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <future>
#include <map>
#include <mutex>
#include <thread>

#include <elf.h>
#include <link.h>  // dl_iterate_phdr: the library build id (checkpoint header)
#include <unistd.h>

namespace sup {

// ------------------------------------------------------------------ RCCL --
// Combine per-device partials over RCCL without giving up the fixed reduction
// order: every device owns a `len`-slot buffer, zero outside the slots it
// filled (its own partial, or the chunk items it dequeued) — each walk writes
// its partial into its slot on the device, after the pairwise reduce.  Every
// slot then has one nonzero addend, so the all-reduce SUM is exact whatever
// ring order RCCL uses; one D2H of the merged buffer follows, and the caller
// folds it with the same pairwise tree as the host path: -R results are
// bit-identical to the host combine.  Communicators are created once per
// device set and kept for the process (ncclCommInitAll is the slow part).
struct RcclSlots {
  std::vector<int> devs;
  std::vector<double*> buf;
  std::vector<hipStream_t> st;
  size_t len = 0;
  ~RcclSlots() {
    for (size_t g = 0; g < devs.size(); ++g) {
      (void)hipSetDevice(devs[g]);
      if (buf[g]) (void)hipFree(buf[g]);
      if (st[g]) (void)hipStreamDestroy(st[g]);
    }
  }
};

// The physical device of each logical device in `devs` (RCCL ranks are
// physical devices); a map that puts two of them on one GPU is refused.
int rccl_physical_devices(const std::vector<int>& devs, std::vector<int>& phys) {
  phys.clear();
  for (int d : devs) phys.push_back(phys_device(d));
  std::vector<int> uniq = phys;
  std::sort(uniq.begin(), uniq.end());
  if (std::adjacent_find(uniq.begin(), uniq.end()) != uniq.end()) {
    phys.clear();
    set_error("RCCL combine (-R) needs distinct physical devices; SUP_DEVICE_MAP puts several logical devices on "
              "one (use the host combine)");
    return SUP_ERCCL;
  }
  return SUP_OK;
}

static int rccl_slots_init(const std::vector<int>& devs, size_t len, RcclSlots& r) {
  r.buf.assign(devs.size(), nullptr);
  r.st.assign(devs.size(), nullptr);
  if (int rc = rccl_physical_devices(devs, r.devs)) {
    r.buf.clear();
    r.st.clear();
    return rc;
  }
  r.len = len;
  // buffers and streams on the communicator's (physical) device: r.devs, not
  // the logical ids, which a permuted SUP_DEVICE_MAP ("1,0") maps elsewhere
  for (size_t g = 0; g < r.devs.size(); ++g) {
    SUP_HIP(hipSetDevice(r.devs[g]));
    SUP_HIP(hipMalloc(&r.buf[g], std::max<size_t>(len, 1) * sizeof(double)));
    SUP_HIP(hipStreamCreateWithFlags(&r.st[g], hipStreamNonBlocking));
    SUP_HIP(hipMemsetAsync(r.buf[g], 0, std::max<size_t>(len, 1) * sizeof(double), r.st[g]));
    SUP_HIP(hipStreamSynchronize(r.st[g]));
  }
  return SUP_OK;
}

static std::mutex g_comm_mu;
static std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;

// Whether the logical devices `devs` sit on distinct physical GPUs (the auto
// combine's test; no error is set).
static bool distinct_physical(const std::vector<int>& devs) {
  std::vector<int> p;
  for (int d : devs) p.push_back(phys_device(d));
  std::sort(p.begin(), p.end());
  return std::adjacent_find(p.begin(), p.end()) == p.end();
}

// The communicators of the physical device set `phys`, created on first use
// (ncclCommInitAll) and kept for the process.  Thread-safe; the error message
// is returned in `err` as well, since g_err is thread-local and the caller may
// run this on a helper thread to overlap it with the walk.
static int rccl_comms(const std::vector<int>& phys, std::vector<ncclComm_t>** out, std::string& err) {
  std::lock_guard<std::mutex> lk(g_comm_mu);
  auto it = g_comms.find(phys);
  if (it == g_comms.end()) {
    std::vector<ncclComm_t> comms(phys.size());
    const ncclResult_t nr = ncclCommInitAll(comms.data(), (int)phys.size(), phys.data());
    if (nr != ncclSuccess) {
      err = std::string("ncclCommInitAll: ") + ncclGetErrorString(nr);
      set_error(err);
      return SUP_ERCCL;
    }
    it = g_comms.emplace(phys, std::move(comms)).first;
  }
  *out = &it->second;
  return SUP_OK;
}

static int rccl_allreduce_slots(RcclSlots& r, std::vector<double>& merged) {
  const int G = (int)r.devs.size();
  std::vector<ncclComm_t>* comms = nullptr;
  std::string err;
  if (int rc = rccl_comms(r.devs, &comms, err)) return rc;
  std::lock_guard<std::mutex> lk(g_comm_mu);  // one collective per communicator at a time
  ncclResult_t nr = ncclGroupStart();
  for (int g = 0; g < G && nr == ncclSuccess; ++g)
    nr = ncclAllReduce(r.buf[g], r.buf[g], r.len, ncclFloat64, ncclSum, (*comms)[g], r.st[g]);
  const ncclResult_t ge = ncclGroupEnd();
  if (nr != ncclSuccess || ge != ncclSuccess) {
    set_error(std::string("ncclAllReduce: ") + ncclGetErrorString(nr != ncclSuccess ? nr : ge));
    return SUP_ERCCL;
  }
  merged.assign(r.len, 0.0);
  for (int g = 0; g < G; ++g) {
    SUP_HIP(hipSetDevice(r.devs[g]));
    SUP_HIP(hipStreamSynchronize(r.st[g]));
  }
  SUP_HIP(hipSetDevice(r.devs[0]));
  SUP_HIP(hipMemcpy(merged.data(), r.buf[0], r.len * sizeof(double), hipMemcpyDeviceToHost));
  return SUP_OK;
}

// The communicators' creation (ncclCommInitAll: hundreds of ms on a fresh
// 8-GPU process) started on a helper thread as soon as the schedule knows it
// will combine over RCCL, so it overlaps the walk instead of following it.
struct CommWarmup {
  std::future<std::pair<int, std::string>> f;
  void start(const std::vector<int>& phys) {
    f = std::async(std::launch::async, [phys] {
      std::vector<ncclComm_t>* c = nullptr;
      std::string err;
      const int rc = rccl_comms(phys, &c, err);
      return std::make_pair(rc, err);
    });
  }
  int join() {  // before the all-reduce (and on every exit path, by the destructor)
    if (!f.valid()) return SUP_OK;
    auto r = f.get();
    if (r.first) set_error(r.second);
    return r.first;
  }
  ~CommWarmup() {
    if (f.valid()) f.wait();
  }
};

// ------------------------------------------------------------ checkpoint --
// sup_opts::checkpoint: a text file, header "supckpt 2 <plan fingerprint>
// <library build id> <toolchain hash> <c0> <c1> <item> <nitems>", then one line "<item> <partial bits> <visited>"
// per finished queue item, appended and flushed (fsync) as items finish.  On
// open, an existing file with the same header lends its items (a torn last
// line from an interrupted write is dropped) and is rewritten clean; another
// header is refused.  Item partials are exact fp64 bit patterns and the items
// are folded by the same pairwise tree, so a resumed run returns the
// uninterrupted run's bits.
// Identity of this library build: the ELF build-id note (--build-id=sha1, a
// hash of the linked object: host code and every gfx950 code object in it)
// of the shared object holding this function, folded to 64 bits; 0 if absent.
static int build_id_cb(struct dl_phdr_info* info, size_t, void* data) {
  auto* io = static_cast<std::pair<uintptr_t, uint64_t>*>(data);
  bool mine = false;
  for (int i = 0; i < info->dlpi_phnum && !mine; ++i) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[i];
    const uintptr_t lo = info->dlpi_addr + ph.p_vaddr;
    mine = ph.p_type == PT_LOAD && io->first >= lo && io->first < lo + ph.p_memsz;
  }
  if (!mine) return 0;
  for (int i = 0; i < info->dlpi_phnum; ++i) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[i];
    if (ph.p_type != PT_NOTE) continue;
    const char* p = (const char*)(info->dlpi_addr + ph.p_vaddr);
    const char* end = p + ph.p_memsz;
    while (p + sizeof(ElfW(Nhdr)) <= end) {
      const ElfW(Nhdr)* nh = (const ElfW(Nhdr)*)p;
      const char* name = p + sizeof(ElfW(Nhdr));
      const char* desc = name + ((nh->n_namesz + 3) & ~3u);
      if (nh->n_type == NT_GNU_BUILD_ID && nh->n_namesz == 4 && std::memcmp(name, "GNU", 4) == 0) {
        uint64_t h = 0xcbf29ce484222325ull;
        for (unsigned k = 0; k < nh->n_descsz; ++k) h = (h ^ (unsigned char)desc[k]) * 1099511628211ull;
        io->second = h;
        return 1;
      }
      p = desc + ((nh->n_descsz + 3) & ~3u);
    }
  }
  return 1;
}

uint64_t library_build_id() {
  static const uint64_t id = [] {
    std::pair<uintptr_t, uint64_t> io{(uintptr_t)(void*)&build_id_cb, 0};
    dl_iterate_phdr(build_id_cb, &io);
    return io.second;
  }();
  return id;
}

int ckpt_open(const char* path, const char* head, uint64_t nitems, std::vector<double>& ipart,
                     std::vector<char>& done, uint64_t& vis, int& resumed, Checkpoint& ck) {
  vis = 0;
  resumed = 0;
  std::string body = head;
  if (FILE* in = std::fopen(path, "r")) {
    char line[256];
    const bool empty = !std::fgets(line, sizeof line, in);  // an empty file starts afresh
    const bool same = empty || std::strcmp(line, head) == 0;
    while (same && !empty && std::fgets(line, sizeof line, in)) {
      const size_t len = std::strlen(line);
      unsigned long long i = 0, bits = 0, v = 0;
      char tail = 0;
      if (len == 0 || line[len - 1] != '\n' || std::sscanf(line, "%llu %llx %llu%c", &i, &bits, &v, &tail) != 4 ||
          i >= nitems)
        break;  // torn or foreign line: stop at it
      if (done[i]) continue;
      done[i] = 1;
      std::memcpy(&ipart[i], &bits, sizeof bits);
      vis += v;
      ++resumed;
      body += line;
    }
    std::fclose(in);
    if (!same) {
      set_error(std::string("checkpoint ") + path + " belongs to another computation (plan, chunk range or item "
                "size differ); remove it or pass another file");
      return SUP_EINVAL;
    }
  }
  // rewrite header + the lines kept, then append from there
  const std::string tmp = std::string(path) + ".tmp" + std::to_string(::getpid());
  FILE* w = std::fopen(tmp.c_str(), "w");
  if (!w || std::fwrite(body.data(), 1, body.size(), w) != body.size() || std::fflush(w) != 0 ||
      ::fsync(fileno(w)) != 0 || std::fclose(w) != 0 || std::rename(tmp.c_str(), path) != 0) {
    set_error(std::string("checkpoint ") + path + ": cannot write it");
    return SUP_EIO;
  }
  if (!(ck.f = std::fopen(path, "a"))) {
    set_error(std::string("checkpoint ") + path + ": cannot append to it");
    return SUP_EIO;
  }
  return SUP_OK;
}

int ckpt_record(Checkpoint& ck, uint64_t it, double part, uint64_t visited) {
  if (!ck.f) return SUP_OK;
  uint64_t bits;
  std::memcpy(&bits, &part, sizeof bits);
  std::lock_guard<std::mutex> g(ck.mu);
  if (std::fprintf(ck.f, "%llu %016llx %llu\n", (unsigned long long)it, (unsigned long long)bits,
                   (unsigned long long)visited) < 0 ||
      std::fflush(ck.f) != 0 || ::fsync(fileno(ck.f)) != 0) {
    set_error("checkpoint: write failed");
    return SUP_EIO;
  }
  return SUP_OK;
}

// ------------------------------------------------------------ schedulers --
int run_item_queue(uint64_t nitems, int takers, const std::function<int(int, uint64_t)>& take) {
  std::atomic<uint64_t> next{0};
  std::atomic<bool> failed{false};
  std::vector<int> rcs(takers, SUP_OK);
  std::vector<std::string> errs(takers);  // g_err is thread_local: carry worker messages back
  const int lane = ctx_lane();            // so is the context lane: the takers keep the caller's
  auto worker = [&](int t) {
    set_ctx_lane(lane);
    while (!failed.load()) {
      const uint64_t it = next.fetch_add(1);
      if (it >= nitems) return;
      if ((rcs[t] = take(t, it)) != SUP_OK) {
        errs[t] = last_error();
        failed.store(true);
        return;
      }
    }
  };
  if (takers == 1) {
    worker(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < takers; ++t) th.emplace_back(worker, t);
    for (auto& x : th) x.join();
  }
  for (int t = 0; t < takers; ++t)
    if (rcs[t]) {
      set_error(errs[t]);
      return rcs[t];
    }
  return SUP_OK;
}

int schedule(const Plan& P, sup_sched sched, const sup_opts& o, uint64_t c0, uint64_t c1,
             SchedResult& out) {
  out = SchedResult();
  // hiprtc time spent while this schedule ran: on the calling thread, or the
  // most any device worker thread spent (they compile concurrently)
  double worker_jit_ms = 0.0;
  struct JitClock {
    SchedResult& o;
    const double& workers;
    double t0 = jit_compile_ms_thread();
    ~JitClock() { o.compile_ms = std::max(jit_compile_ms_thread() - t0, workers); }
  } jit_clock{out, worker_jit_ms};
  int ndev = 0;
  int rc = device_count(&ndev);
  if (rc) return rc;
  if (ndev == 0) {
    set_error("no HIP device available (the engine has no CPU fallback for GPU algorithms)");
    return SUP_ENODEV;
  }
  int G = (sched == SUP_SCHED_SINGLE) ? 1 : std::max(1, o.gpu_num);
  if (o.device_id < 0 || o.device_id + G > ndev) {
    set_error("requested devices [" + std::to_string(o.device_id) + ", " + std::to_string(o.device_id + G) +
              ") but only " + std::to_string(ndev) + " are visible");
    return SUP_ENODEV;
  }
  std::vector<int> devs(G);
  for (int g = 0; g < G; ++g) devs[g] = o.device_id + g;
  const uint64_t total = c1 - c0;
  const bool want_visited = true;

  // Combine of the device partials: use_rccl 2 forces RCCL (even on one
  // device: exercises it), 1 asks for it (SUP_ERCCL when the devices share a
  // GPU), -1 (the CLI default) takes it whenever the G > 1 devices are
  // distinct physical GPUs and keeps the host pairwise tree otherwise; 0: host.
  bool rccl = (G > 1 && o.use_rccl > 0) || o.use_rccl == 2;
  if (G > 1 && o.use_rccl < 0) rccl = distinct_physical(devs);
  auto say_combine = [&](bool used, const char* why) {
    if (o.verbose)
      std::printf("Combine: %s over %d device%s%s\n", used ? "RCCL all-reduce (slot buffers)" : "host pairwise tree",
                  G, G == 1 ? "" : "s", why);
  };
  CommWarmup warm;
  if (sched != SUP_SCHED_CHUNKS && o.checkpoint && *o.checkpoint) {
    set_error("a checkpoint file needs the chunk queue (-p6 / -p8, SUP_SCHED_CHUNKS)");
    return SUP_EUNSUPPORTED;
  }
  if (sched != SUP_SCHED_CHUNKS) {
    // Single device, a static contiguous split (-p5: G equal pieces, piece g
    // on device g), or the reference's manual distribution (-p66,
    // gpu_exact_dense.cu:913-990 / gpu_exact_sparse.cu:1328-1400: 3/8, 3/8,
    // 1/8, 1/8 of the space on 4 devices, for unequal GPUs) as eight equal
    // pieces owned {0,0,0,1,1,1,2,3} (mod G).  Piece partials are folded by
    // the pairwise tree in piece order; equal power-of-two pieces are subtrees
    // of the one-device tree, so -p5 on 2/4/8 devices and -p66 on any give the
    // one-device result bit for bit.
    const bool manual = sched == SUP_SCHED_MANUAL;
    const int npieces = manual ? 8 : G;
    std::vector<int> owner(npieces);
    for (int q = 0; q < npieces; ++q) owner[q] = manual ? (q < 3 ? 0 : q < 6 ? 1 : q == 6 ? 2 : 3) % G : q;
    RcclSlots slots;
    if (rccl && (rc = rccl_slots_init(devs, npieces, slots))) return rc;
    if (rccl) warm.start(slots.devs);
    std::vector<RangeResult> rr(npieces);
    std::vector<int> rcs(G, SUP_OK);
    std::vector<std::string> errs(G);  // g_err is thread_local: carry worker messages back
    const int lane = ctx_lane();
    auto work = [&](int g) {
      set_ctx_lane(lane);
      auto t0 = std::chrono::steady_clock::now();
      for (int q = 0; q < npieces && !rcs[g]; ++q) {
        if (owner[q] != g) continue;
        const uint64_t a = c0 + total * (uint64_t)q / (uint64_t)npieces;
        const uint64_t b = c0 + total * (uint64_t)(q + 1) / (uint64_t)npieces;
        rcs[g] = run_range(devs[g], P, a, b, want_visited, rr[q], rccl ? slots.buf[g] + q : nullptr);
      }
      if (rcs[g]) errs[g] = last_error();
      if (o.verbose) {
        double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("kernel%d in %f\n", devs[g], s);
      }
    };
    if (G == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (int g = 0; g < G; ++g) th.emplace_back(work, g);
      for (auto& t : th) t.join();
    }
    for (int g = 0; g < G; ++g)
      if (rcs[g]) {
        set_error(errs[g]);
        return rcs[g];
      }
    out.dev_partials.assign(G, 0.0);
    std::vector<double> piece(npieces), dev_ms(G, 0.0), dev_jit(G, 0.0);
    for (int q = 0; q < npieces; ++q) {
      const int g = owner[q];
      piece[q] = rr[q].partial;
      out.dev_partials[g] += rr[q].partial;
      dev_ms[g] += rr[q].kernel_ms;
      dev_jit[g] += rr[q].compile_ms;
      out.visited += rr[q].visited;
      out.grid = std::max(out.grid, rr[q].grid);
    }
    for (int g = 0; g < G; ++g) {
      out.kernel_ms = std::max(out.kernel_ms, dev_ms[g]);
      worker_jit_ms = std::max(worker_jit_ms, dev_jit[g]);
    }
    out.devices = G;
    if (rccl) {
      std::vector<double> merged;
      if ((rc = warm.join()) || (rc = rccl_allreduce_slots(slots, merged))) return rc;
      out.total = pairwise_host(merged);
    } else {
      out.total = pairwise_host(piece);
    }
    say_combine(rccl, rccl || G == 1 ? "" : o.use_rccl < 0 ? " (devices share a GPU)" : "");
    return SUP_OK;
  }

  // Dynamic chunk queue (-p6 / -p8): power-of-two aligned items of wave-chunks,
  // taken by one host thread per device (and optionally a CPU worker).  Item
  // partials are combined in item order by the same pairwise tree, so the
  // result does not depend on which device took which item.
  uint64_t item = 1;
  if (o.chunk_log2 > 0) {
    item = 1ull << o.chunk_log2;
  } else {
    // 16 items per taker; one device with nothing to balance against (no CPU
    // worker) and no checkpoint to resume from walks its range as one item —
    // the same subtree sums, without 15 more launches and launch tails
    // (config 5 -p8: 0.39 ms of a 48.9 ms step)
    const bool alone = G == 1 && !o.cpu_worker && !(o.checkpoint && *o.checkpoint);
    const uint64_t target_items = alone ? 1 : (uint64_t)G * 16;
    while (item * 2 <= total && total / (item * 2) >= target_items) item <<= 1;
  }
  const uint64_t nitems = (total + item - 1) / item;
  std::vector<double> ipart(nitems, 0.0);
  // items an earlier, interrupted call recorded (sup_opts::checkpoint)
  std::vector<char> done(nitems, 0);
  uint64_t resumed_vis = 0;
  Checkpoint ck;
  const bool ckpt = o.checkpoint && *o.checkpoint;
  if (ckpt) {
    // the plan's fingerprint, the library build (every ahead-of-time kernel's
    // code object) and the hiprtc toolchain: partials from another binary are
    // not mixed into a resumed run
    char head[240];
    std::snprintf(head, sizeof head, "supckpt 2 %016llx %016llx %016llx %llu %llu %llu %llu\n",
                  (unsigned long long)plan_fingerprint(P), (unsigned long long)library_build_id(),
                  (unsigned long long)jit_toolchain_hash(), (unsigned long long)c0, (unsigned long long)c1,
                  (unsigned long long)item, (unsigned long long)nitems);
    if ((rc = ckpt_open(o.checkpoint, head, nitems, ipart, done, resumed_vis, out.items_resumed, ck))) return rc;
    if (o.verbose)
      std::printf("Checkpoint %s: %d of %llu items resumed\n", o.checkpoint, out.items_resumed,
                  (unsigned long long)nitems);
  }
  std::vector<uint64_t> pending;
  for (uint64_t it = 0; it < nitems; ++it)
    if (!done[it]) pending.push_back(it);
  // -R: device g writes the partial of every item it takes into slot `item`
  // of its own buffer (the CPU worker's items, and items resumed from a
  // checkpoint, have no device: host combine)
  const bool rccl_items = rccl && !o.cpu_worker && !ckpt;
  RcclSlots slots;
  if (rccl_items && (rc = rccl_slots_init(devs, nitems, slots))) return rc;
  if (rccl_items) warm.start(slots.devs);
  std::vector<double> dev_ms(G + 1, 0.0), dev_jit(G, 0.0);
  std::vector<uint64_t> dev_vis(G + 1, 0);
  std::vector<int> dev_grid(G + 1, 0);
  std::vector<double> dev_sum(G, 0.0);
  std::atomic<int> cpu_items{0};
  // takers 0..G-1: one host thread per device; taker G: the CPU worker
  auto take = [&](int g, uint64_t it) -> int {
    const uint64_t a = c0 + it * item;
    const uint64_t b = std::min(c1, a + item);
    auto t0 = std::chrono::steady_clock::now();
    uint64_t vis = 0;
    if (g == G) {
      ipart[it] = cpu_walk_range(P, a, b, std::max(1, o.threads));
      vis = (b - a) << (P.lay.L + P.lay.m);
      dev_vis[G] += vis;
      cpu_items.fetch_add(1);
    } else {
      RangeResult r;
      const int e = run_range(devs[g], P, a, b, want_visited, r, rccl_items ? slots.buf[g] + it : nullptr);
      if (e) return e;
      ipart[it] = r.partial;
      vis = r.visited;
      dev_sum[g] += r.partial;
      dev_ms[g] += r.kernel_ms;
      dev_jit[g] += r.compile_ms;
      dev_vis[g] += r.visited;
      dev_grid[g] = std::max(dev_grid[g], r.grid);
    }
    if (const int e = ckpt_record(ck, it, ipart[it], vis)) return e;
    if (o.verbose) {
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (g == G) std::printf("ChunkID %llu is DONE by CPU in %f\n", (unsigned long long)it, sec);
      else std::printf("ChunkID %llu is DONE by kernel%d in %f\n", (unsigned long long)it, devs[g], sec);
    }
    return SUP_OK;
  };
  if ((rc = run_item_queue(pending.size(), G + (o.cpu_worker ? 1 : 0),
                          [&](int g, uint64_t q) { return take(g, pending[q]); })))
    return rc;
  out.devices = G;
  out.cpu_items = cpu_items.load();
  out.visited = resumed_vis;
  for (int g = 0; g < G; ++g) worker_jit_ms = std::max(worker_jit_ms, dev_jit[g]);
  for (int g = 0; g <= G; ++g) {
    out.kernel_ms = std::max(out.kernel_ms, dev_ms[g]);
    out.visited += dev_vis[g];
    out.grid = std::max(out.grid, dev_grid[g]);
  }
  out.dev_partials = dev_sum;
  if (rccl_items) {
    std::vector<double> merged;
    if ((rc = warm.join()) || (rc = rccl_allreduce_slots(slots, merged))) return rc;
    out.total = pairwise_host(merged);
  } else {
    out.total = pairwise_host(ipart);
  }
  say_combine(rccl_items, rccl_items || G == 1 ? ""
                          : o.cpu_worker  ? " (the CPU worker's items have no device slot)"
                          : ckpt          ? " (checkpointed items)"
                          : o.use_rccl < 0 ? " (devices share a GPU)" : "");
  return SUP_OK;
}

}  // namespace sup
