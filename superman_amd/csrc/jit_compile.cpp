// jit_compile.cpp — compiling and caching the segmented walk's generated
// kernels (jit.cpp): hiprtc for gfx950, the memory and disk caches of code
// objects, the helper processes that compile a budget ladder's candidates in
// parallel, module loads and launches, and the small records auto mode keeps
// on disk (plan choices, first decisions, this host's cold plan cost).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <sched.h>
#include <signal.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>

#include "engine.hpp"
#include "jit_internal.hpp"

namespace sup {

namespace {
#include "jit_headers.inc"  // kWalkCommonSrc, kWalkParamsSrc (the in-memory headers hiprtc compiles against)

// Budget candidates compiled at once (host threads) by the compiler check.
constexpr size_t kMaxParallelCompiles = 8;
// Process-wide gate on hiprtcCompileProgram: at most kMaxParallelCompiles
// compiles run at once across every caller (budget ladders, -o leaf workers,
// per-device threads of a multi-device schedule), and only one at a time once
// any compile has failed — the batch limit alone did not bound compiles that
// several callers start concurrently.
class CompileGate {
 public:
  void enter() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return busy_ < (g_jit_failed.load() ? 1u : (unsigned)kMaxParallelCompiles); });
    ++busy_;
  }
  void leave() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      --busy_;
    }
    cv_.notify_all();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  unsigned busy_ = 0;
};
CompileGate g_compile_gate;
}  // namespace

CompileSlot::CompileSlot() { g_compile_gate.enter(); }
CompileSlot::~CompileSlot() { g_compile_gate.leave(); }

// ------------------------------------------------------ compile and cache --
namespace {

std::mutex g_jit_mu;
std::map<uint64_t, std::shared_ptr<std::vector<char>>> g_code;        // key -> code object
std::map<std::pair<int, uint64_t>, hipFunction_t> g_fn;               // (device, key) -> kernel
std::map<std::pair<int, uint64_t>, int> g_occ;
// SUP_JIT_LDS (experiments): dynamic LDS bytes per block, to cap residency
// and measure the walk's sensitivity to occupancy.
unsigned jit_lds_bytes() {
  const char* e = std::getenv("SUP_JIT_LDS");
  return e ? (unsigned)std::strtoul(e, nullptr, 10) : 0u;
}

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
  // one temporary per process and thread (threads of one process may write the same entry at once)
  const std::string tmp = dir + "/." + name + "." + std::to_string(::getpid()) + "." +
                          std::to_string(std::hash<std::thread::id>()(std::this_thread::get_id()));
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;  // cache is best effort
  const bool ok = std::fwrite(data.data(), 1, data.size(), f) == data.size();
  std::fclose(f);
  if (ok) std::rename(tmp.c_str(), (dir + "/" + name).c_str());
  else std::remove(tmp.c_str());
}

// Code object of P's kernel: from memory, the disk cache, or hiprtc.  Safe to
// call from several threads at once (the budget check compiles its candidates
// concurrently); g_jit_mu guards the maps only, not the compile.
int compile(const Plan& P, std::shared_ptr<std::vector<char>>& code) {
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    auto it = g_code.find(P.jit_key);
    if (it != g_code.end()) {
      code = it->second;
      return SUP_OK;
    }
  }
  const std::string dir = cache_dir();
  const std::string name = "seg_" + key_hex(P.jit_key) + ".co";
  auto co = std::make_shared<std::vector<char>>();
  auto publish = [&]() {
    std::lock_guard<std::mutex> g(g_jit_mu);
    auto ins = g_code.emplace(P.jit_key, co);  // a concurrent compile of the same key may have won
    code = ins.first->second;
    return SUP_OK;
  };
  if (!dir.empty() && read_file(dir + "/" + name, *co)) return publish();
  if (const char* d = std::getenv("SUP_JIT_DUMP")) {  // debugging: keep the generated source
    FILE* f = std::fopen((std::string(d) + "/seg_" + key_hex(P.jit_key) + ".hip").c_str(), "w");
    if (f) std::fputs(P.jit_src.c_str(), f), std::fclose(f);
  }
  if (const char* e = std::getenv("SUP_JIT_FAIL"))  // tests: a compile hiprtc refuses (the fallback paths)
    if (std::atoi(e)) {
      g_jit_failed.store(true);
      set_error("hiprtc compile of the segmented walk failed: refused on request (SUP_JIT_FAIL)");
      return SUP_EHIP;
    }
  auto t0 = std::chrono::steady_clock::now();
  hiprtcProgram prog;
  const char* hdr[] = {kWalkCommonSrc, kWalkParamsSrc};
  const char* names[] = {"walk_common.hpp", "walk_params.hpp"};
  // A step region's pinned pieces can exceed the SGPRs the allocator has left
  // ("ran out of registers"); the source is then regenerated with half the
  // piece budget (the same operations in the same order: bit-identical
  // results, same tables), down to one piece.
  std::string src = P.jit_src;
  for (int kp = P.seg_kp;; kp /= 2) {
    if (hiprtcCreateProgram(&prog, src.c_str(), "sup_walk_seg.hip", 2, hdr, names) != HIPRTC_SUCCESS) {
      set_error("hiprtcCreateProgram failed");
      return SUP_EHIP;
    }
    const std::vector<std::string> opts = jit_opts();
    std::vector<const char*> optp;
    for (const std::string& x : opts) optp.push_back(x.c_str());
    hiprtcResult cr;
    std::string log;
    {
      CompileSlot slot;  // process-wide limit on concurrent compiles (CompileGate)
      cr = hiprtcCompileProgram(prog, (int)optp.size(), optp.data());
      if (cr != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(prog, &ls);
        log.assign(ls, '\0');
        if (ls) hiprtcGetProgramLog(prog, &log[0]);
        // a failure other than the register retry below: serialise from here on,
        // set before this slot frees so no further compile starts beside it
        if (kp <= 1 || log.find("ran out of registers") == std::string::npos) g_jit_failed.store(true);
      }
    }
    if (cr == HIPRTC_SUCCESS) break;
    hiprtcDestroyProgram(&prog);
    if (kp > 1 && log.find("ran out of registers") != std::string::npos) {
      src = seg_source(P, kp / 2);
      continue;
    }
    g_jit_failed.store(true);
    set_error(std::string("hiprtc compile of the segmented walk failed: ") + hiprtcGetErrorString(cr) + "\n" +
              log.substr(0, 2000));
    return SUP_EHIP;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  co->resize(cs);
  hiprtcGetCode(prog, co->data());
  hiprtcDestroyProgram(&prog);
  t_compile_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (!dir.empty()) write_file_atomic(dir, name, *co);
  return publish();
}

}  // namespace

// ------------------------------------------------- out-of-process compiles --
// hiprtc compiles in one process are serialised, so a batch of candidate
// kernels (the budget ladder's next steps) is compiled by helper processes,
// one per host core: superman_amd/bin/sup_rtc (sup_rtc.cpp) loads the same
// hiprtc library as this process and writes the code object, which enters the
// memory and disk caches exactly as an in-process compile's would.  Best
// effort: a candidate whose helper fails is compiled in process when the
// search reaches it (with the register retry and the error message).
// SUP_RTC_PROCS caps the helpers (0 or 1: none); SUP_RTC_HELPER names the
// helper binary.

bool jit_code_cached(const Plan& P) {
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    if (g_code.count(P.jit_key)) return true;
  }
  const std::string dir = cache_dir();
  struct stat st;
  return !dir.empty() && ::stat((dir + "/seg_" + key_hex(P.jit_key) + ".co").c_str(), &st) == 0 && st.st_size > 0;
}

namespace {

std::string rtc_helper() {
  if (const char* e = std::getenv("SUP_RTC_HELPER")) return e;
  Dl_info info;
  if (!dladdr((void*)&rtc_helper, &info) || !info.dli_fname) return "";
  std::string lib = info.dli_fname;  // .../superman_amd/lib/libsuperman_hip.so
  const size_t s = lib.rfind('/');
  return (s == std::string::npos ? std::string(".") : lib.substr(0, s)) + "/../bin/sup_rtc";
}

std::string hiprtc_library() {
  Dl_info info;
  if (!dladdr((void*)&hiprtcCompileProgram, &info) || !info.dli_fname) return "";
  return info.dli_fname;
}

}  // namespace

// A helper compile that runs longer than this is abandoned (a candidate's
// compile takes 0.2-2.5 s on the bench matrices).
constexpr int kHelperLimitS = 300;

size_t rtc_procs() {
  if (const char* e = std::getenv("SUP_RTC_PROCS")) return (size_t)std::max(0, std::atoi(e));
  if (g_jit_failed.load() || std::getenv("SUP_JIT_FAIL")) return 0;
  cpu_set_t set;
  size_t cpus = std::max(1u, std::thread::hardware_concurrency());
  if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = (size_t)CPU_COUNT(&set);
  return std::min<size_t>(16, cpus);
}

void prefetch_compiles(const std::vector<const Plan*>& plans, size_t procs) {
  std::vector<const Plan*> todo;
  for (const Plan* p : plans)
    if (!jit_code_cached(*p)) todo.push_back(p);
  if (todo.size() < 2 || procs < 2 || g_jit_failed.load()) return;  // one compile: in process, as fast
  const std::string helper = rtc_helper(), lib = hiprtc_library();
  if (helper.empty() || lib.empty() || ::access(helper.c_str(), X_OK) != 0) return;
  const char* tmpdir = std::getenv("TMPDIR");
  std::string dir = std::string(tmpdir && *tmpdir ? tmpdir : "/tmp") + "/sup_rtc_XXXXXX";
  if (!::mkdtemp(&dir[0])) return;
  auto put = [&](const std::string& name, const std::string& text) {
    std::ofstream f(dir + "/" + name, std::ios::binary);
    f << text;
    return (bool)f;
  };
  std::vector<std::string> made;
  if (put("walk_common.hpp", kWalkCommonSrc) && put("walk_params.hpp", kWalkParamsSrc)) {
    made = {"walk_common.hpp", "walk_params.hpp"};
    const std::vector<std::string> opts = jit_opts();
    std::atomic<size_t> next{0};
    std::mutex mu;
    auto worker = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < todo.size();) {
        const Plan& P = *todo[i];
        const std::string name = "seg_" + key_hex(P.jit_key);
        {
          std::lock_guard<std::mutex> g(mu);
          for (const char* ext : {".hip", ".co", ".co.part", ".log", ".log.part"}) made.push_back(name + ext);
        }
        if (!put(name + ".hip", P.jit_src)) continue;
        std::vector<std::string> args = {helper, lib, dir, name};
        args.insert(args.end(), opts.begin(), opts.end());
        std::vector<char*> argv;
        for (std::string& a : args) argv.push_back(&a[0]);
        argv.push_back(nullptr);
        pid_t pid = 0;
        if (posix_spawn(&pid, helper.c_str(), nullptr, nullptr, argv.data(), environ) != 0) continue;
        // a helper that has not finished in kHelperLimitS is killed: its
        // candidate is then compiled in process if the search reaches it
        int status = 0;
        const auto t_spawn = std::chrono::steady_clock::now();
        bool done = false;
        for (;;) {
          const pid_t w = ::waitpid(pid, &status, WNOHANG);
          if (w == pid) {
            done = true;
            break;
          }
          if (w < 0 && errno != EINTR) break;
          if (std::chrono::steady_clock::now() - t_spawn > std::chrono::seconds(kHelperLimitS)) {
            ::kill(pid, SIGKILL);
            while (::waitpid(pid, &status, 0) < 0 && errno == EINTR) {
            }
            break;
          }
          ::usleep(1000);
        }
        if (!done || !WIFEXITED(status) || WEXITSTATUS(status) != 0) continue;
        auto co = std::make_shared<std::vector<char>>();
        if (!read_file(dir + "/" + name + ".co", *co)) continue;
        {
          std::lock_guard<std::mutex> g(g_jit_mu);
          g_code.emplace(P.jit_key, co);
        }
        const std::string cdir = cache_dir();
        if (!cdir.empty()) write_file_atomic(cdir, name + ".co", *co);
      }
    };
    std::vector<std::thread> th;
    for (size_t t = 0; t < std::min(procs, todo.size()); ++t) th.emplace_back(worker);
    for (auto& t : th) t.join();
  }
  for (const std::string& f : made) ::unlink((dir + "/" + f).c_str());
  ::rmdir(dir.c_str());
}

namespace {

int resolve(int dev, const Plan& P, hipFunction_t* fn) {
  if (P.kind != kWalkSeg || P.jit_src.empty()) {
    set_error("plan has no segmented-walk kernel");
    return SUP_EINVAL;
  }
  auto k = std::make_pair(dev, P.jit_key);
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    auto it = g_fn.find(k);
    if (it != g_fn.end()) {
      *fn = it->second;
      return SUP_OK;
    }
  }
  std::shared_ptr<std::vector<char>> code;
  int rc = compile(P, code);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(g_jit_mu);
  auto it = g_fn.find(k);
  if (it != g_fn.end()) {
    *fn = it->second;
    return SUP_OK;
  }
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
  const double before = jit_compile_ms_thread();
  std::shared_ptr<std::vector<char>> code;
  const int rc = compile(P, code);
  if (compile_ms) *compile_ms = jit_compile_ms_thread() - before;
  return rc;
}

int jit_code_scan(const Plan& P, CodeScan* out) {
  std::shared_ptr<std::vector<char>> code;
  const int rc = compile(P, code);
  if (rc) return rc;
  return scan_code_object(*code, "sup_walk_seg", out);
}

int jit_occupancy(int dev, const Plan& P, int* blocks_per_cu, double* compile_ms) {
  const double before = jit_compile_ms_thread();
  hipFunction_t fn;
  int rc = resolve(dev, P, &fn);
  if (rc) return rc;
  if (compile_ms) *compile_ms = jit_compile_ms_thread() - before;
  std::lock_guard<std::mutex> g(g_jit_mu);
  auto k = std::make_pair(dev, P.jit_key);
  auto it = g_occ.find(k);
  if (it != g_occ.end()) {
    *blocks_per_cu = it->second;
    return SUP_OK;
  }
  int b = 0;
  hipError_t e = hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&b, fn, kBlock, jit_lds_bytes());
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
  hipError_t e = hipModuleLaunchKernel(fn, (unsigned)grid, 1, 1, kBlock, 1, 1, jit_lds_bytes(), s, args, nullptr);
  if (e != hipSuccess) {
    set_error(std::string("hipModuleLaunchKernel (segmented walk): ") + hipGetErrorString(e));
    return SUP_EHIP;
  }
  return SUP_OK;
}

double jit_compile_ms_thread() { return t_compile_ms; }

uint64_t jit_toolchain_hash() {
  static const uint64_t h = toolchain_hash_impl();
  return h;
}

// Recorded segmented-walk choices: a small text file next to the code objects,
// "supseg 3 <m> <b> <budget> <cc cap> <count> <order...>".
bool seg_choice_load(uint64_t key, int* m, SegChoice* c) {
  const std::string dir = cache_dir();
  if (dir.empty()) return false;
  std::vector<char> buf;
  if (!read_file(dir + "/plan_" + key_hex(key) + ".txt", buf)) return false;
  buf.push_back('\0');
  std::istringstream in(buf.data());
  std::string tag;
  int ver = 0, cnt = 0;
  if (!(in >> tag >> ver >> *m >> c->b >> c->budget >> c->cc_cap >> cnt) || tag != "supseg" || ver != 3 || cnt < 1 ||
      cnt > 64 || c->cc_cap < 0 || c->cc_cap > kMaxCachedBits)
    return false;
  c->order.resize(cnt);
  for (int& v : c->order)
    if (!(in >> v) || v < 0 || v > 63) return false;
  return true;
}

bool seg_choice_exists(uint64_t key) {
  const std::string dir = cache_dir();
  struct stat sb;
  return !dir.empty() && ::stat((dir + "/plan_" + key_hex(key) + ".txt").c_str(), &sb) == 0;
}

void seg_choice_store(uint64_t key, int m, const SegChoice& c) {
  const std::string dir = cache_dir();
  if (dir.empty() || c.order.empty()) return;
  std::ostringstream o;
  o << "supseg 3 " << m << ' ' << c.b << ' ' << c.budget << ' ' << c.cc_cap << ' ' << c.order.size();
  for (int v : c.order) o << ' ' << v;
  o << '\n';
  const std::string str = o.str();
  write_file_atomic(dir, "plan_" + key_hex(key) + ".txt", std::vector<char>(str.begin(), str.end()));
}

// Auto mode's decision: "supauto 1 <0|1>" in auto_<key>.txt.  Its bar moves
// with the cache (a recorded plan makes specialising cheap), so the first
// decision is kept: later processes running the same command walk the same
// plan and print the same bits.
int auto_decision_load(uint64_t key) {
  const std::string dir = cache_dir();
  if (dir.empty()) return -1;
  std::vector<char> buf;
  if (!read_file(dir + "/auto_" + key_hex(key) + ".txt", buf)) return -1;
  buf.push_back('\0');
  std::istringstream in(buf.data());
  std::string tag;
  int ver = 0, v = -1;
  if (!(in >> tag >> ver >> v) || tag != "supauto" || ver != 1 || (v != 0 && v != 1)) return -1;
  return v;
}

int auto_decision_store(uint64_t key, int seg) {
  const std::string dir = cache_dir();
  if (dir.empty()) return seg;
  const std::string name = "auto_" + key_hex(key) + ".txt";
  const std::string str = std::string("supauto 1 ") + (seg ? "1" : "0") + "\n";
  // write a private temporary, then link() it to the final name: link fails
  // when the name exists, so the first process to decide wins and every other
  // follows what it recorded (write_file_atomic's rename would overwrite)
  const std::string mine = "." + name + ".new" + std::to_string(::getpid()) + "." +
                           std::to_string(std::hash<std::thread::id>()(std::this_thread::get_id()));
  write_file_atomic(dir, mine, std::vector<char>(str.begin(), str.end()));
  (void)::link((dir + "/" + mine).c_str(), (dir + "/" + name).c_str());
  std::remove((dir + "/" + mine).c_str());
  const int on_disk = auto_decision_load(key);
  return on_disk >= 0 ? on_disk : seg;
}

// What a cold segmented plan (walk-order search + the compiler check's
// compiles) costs.  Measured on a GPU box with an empty plan cache and an
// empty comgr cache (tools/probe_cold.sh, profiles/r5/probe_cold.log), 16
// threads: the search 0.13 s at n = 32, 0.16 s at 36, 0.39 s at 40, 0.64 s at
// 44 (8 threads: 0.67 s at 40, 1.17 s at 44); the compiler check's kernels
// ~0.25 s each, one after another (hiprtc compiles in one process do not
// overlap), 5 of them for the bisected budget ladder at n = 40 (1.25 s).
double seg_cold_model(int n) {
  const double search = 0.39 * std::exp2((n - 40) / 6.5) * std::pow(16.0 / plan_threads(), 0.8);
  return search + 1.25;
}

// This host's recorded speed: "supcost 2 <measured / modelled>", one file per
// toolchain next to the code objects, written by every cold plan.
static std::string seg_cost_name() { return "cost_" + key_hex(jit_toolchain_hash()) + ".txt"; }

double seg_cost_ratio_load() {
  const std::string dir = cache_dir();
  if (dir.empty()) return -1.0;
  std::vector<char> buf;
  if (!read_file(dir + "/" + seg_cost_name(), buf)) return -1.0;
  buf.push_back('\0');
  std::istringstream in(buf.data());
  std::string tag;
  int ver = 0;
  double r = -1.0;
  if (!(in >> tag >> ver >> r) || tag != "supcost" || ver != 2 || !(r > 0.0) || r > 1000.0) return -1.0;
  return r;
}

double seg_cold_predict(int n) {
  // SUP_JIT_COLD_RATIO (tests, experiments): this host's speed ratio, in place
  // of the recorded one (not a plan knob: knob_hash leaves it out)
  const char* e = std::getenv("SUP_JIT_COLD_RATIO");
  const double r = e ? std::atof(e) : seg_cost_ratio_load();
  return seg_cold_model(n) * (r > 0.0 ? std::min(8.0, std::max(0.25, r)) : 1.0);
}

void seg_cost_store(int n, double seconds) {
  const std::string dir = cache_dir();
  if (dir.empty() || !(seconds > 0.0)) return;
  char b[64];
  std::snprintf(b, sizeof b, "supcost 2 %.4f\n", seconds / seg_cold_model(n));
  const std::string str = b;
  write_file_atomic(dir, seg_cost_name(), std::vector<char>(str.begin(), str.end()));
}

}  // namespace sup
