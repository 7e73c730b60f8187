// sup_rtc — one hiprtc compile of a generated segmented-walk kernel, in its
// own process.  hiprtc compiles inside one process are serialised (the comgr
// action behind hiprtcCompileProgram holds a process-wide lock: 8 threads
// compiling 8 kernels take 0.8x the time of 8 sequential compiles), so the
// budget ladder's candidates (jit.cpp build_seg) are compiled ahead of the
// bisection by a pool of these helpers, one per host core, and the code
// objects land in the engine's code cache.  The helper loads the very hiprtc
// library the parent process uses (path from dladdr in the parent: torch's
// bundled copy in a torch process, /opt/rocm's otherwise), so the code object
// is the one an in-process compile would have produced, byte for byte.
//
//   sup_rtc <libhiprtc.so> <dir> <name> <option>...
// reads <dir>/walk_common.hpp, <dir>/walk_params.hpp and <dir>/<name>.hip;
// writes <dir>/<name>.co (exit 0), or the compile log to <dir>/<name>.log
// (exit 1).  Any failure leaves the compile to the parent, in process.
#include <dlfcn.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

typedef struct _hiprtcProgram* Prog;
typedef int (*CreateFn)(Prog*, const char*, const char*, int, const char* const*, const char* const*);
typedef int (*CompileFn)(Prog, int, const char* const*);
typedef int (*SizeFn)(Prog, size_t*);
typedef int (*GetFn)(Prog, char*);
typedef int (*DestroyFn)(Prog*);

bool slurp(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream s;
  s << f.rdbuf();
  out = s.str();
  return true;
}

bool spill(const std::string& path, const char* data, size_t size) {
  const std::string part = path + ".part";
  FILE* f = std::fopen(part.c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(data, 1, size, f) == size;
  if (std::fclose(f) != 0 || !ok) {
    std::remove(part.c_str());
    return false;
  }
  return std::rename(part.c_str(), path.c_str()) == 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: sup_rtc <libhiprtc.so> <dir> <name> <option>...\n");
    return 2;
  }
  const std::string dir = argv[2], name = argv[3];
  const std::string logp = dir + "/" + name + ".log";
  auto fail = [&](const std::string& why) {
    spill(logp, why.data(), why.size());
    return 1;
  };
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail(std::string("dlopen: ") + dlerror());
  auto create = (CreateFn)dlsym(h, "hiprtcCreateProgram");
  auto compile = (CompileFn)dlsym(h, "hiprtcCompileProgram");
  auto code_size = (SizeFn)dlsym(h, "hiprtcGetCodeSize");
  auto code = (GetFn)dlsym(h, "hiprtcGetCode");
  auto log_size = (SizeFn)dlsym(h, "hiprtcGetProgramLogSize");
  auto log = (GetFn)dlsym(h, "hiprtcGetProgramLog");
  auto destroy = (DestroyFn)dlsym(h, "hiprtcDestroyProgram");
  if (!create || !compile || !code_size || !code || !log_size || !log || !destroy)
    return fail("hiprtc entry points missing");
  std::string src, common, params;
  if (!slurp(dir + "/" + name + ".hip", src) || !slurp(dir + "/walk_common.hpp", common) ||
      !slurp(dir + "/walk_params.hpp", params))
    return fail("request files missing");
  const char* hdr[] = {common.c_str(), params.c_str()};
  const char* names[] = {"walk_common.hpp", "walk_params.hpp"};
  Prog prog = nullptr;
  if (create(&prog, src.c_str(), "sup_walk_seg.hip", 2, hdr, names) != 0) return fail("hiprtcCreateProgram failed");
  std::vector<const char*> opts(argv + 4, argv + argc);
  if (compile(prog, (int)opts.size(), opts.data()) != 0) {
    size_t ls = 0;
    log_size(prog, &ls);
    std::string text(ls, '\0');
    if (ls) log(prog, &text[0]);
    destroy(&prog);
    return fail("hiprtc: " + text);
  }
  size_t cs = 0;
  code_size(prog, &cs);
  std::vector<char> co(cs);
  code(prog, co.data());
  destroy(&prog);
  if (cs == 0 || !spill(dir + "/" + name + ".co", co.data(), co.size())) return fail("writing the code object");
  return 0;
}
