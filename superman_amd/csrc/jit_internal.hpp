// jit_internal.hpp — what the segmented walk's planner and code generator
// (jit.cpp) share with its compiler and caches (jit_compile.cpp).  Internal to
// the library.
#pragma once
#include <atomic>
#include <string>
#include <vector>

#include "engine.hpp"

namespace sup {

// hiprtc time spent by this thread (and the wall time of compile batches it
// ran on helper threads or processes): per call, not process-wide.
extern thread_local double t_compile_ms;
// Set when hiprtc fails on a segmented walk (an error, or a register allocator
// that gives up, "maximum depth for recoloring").  Such a failure next to
// concurrent compiles has crashed the process (LLVM's error path is not
// thread-safe), so from then on this process compiles one kernel at a time.
extern std::atomic<bool> g_jit_failed;

// A slot of the process-wide gate on hiprtcCompileProgram (at most 8 compiles
// at once, one once any compile has failed), held for one compile.
struct CompileSlot {
  CompileSlot();
  ~CompileSlot();
  CompileSlot(const CompileSlot&) = delete;
  CompileSlot& operator=(const CompileSlot&) = delete;
};

// hiprtc options of every segmented-walk compile (part of every cache key).
std::vector<std::string> jit_opts();
// Hash of the generated-code headers, compile options and hiprtc library.
uint64_t toolchain_hash_impl();
// The generated kernel source of plan P with `kp` SGPR pieces per step region.
std::string seg_source(const Plan& P, int kp);

// Out-of-process compiles (sup_rtc helpers): whether P's code object is in the
// memory or disk cache; how many helpers run at once; compile a batch ahead.
bool jit_code_cached(const Plan& P);
size_t rtc_procs();
void prefetch_compiles(const std::vector<const Plan*>& plans, size_t procs);

}  // namespace sup
