// probe_launch.hip — what one small call's HIP API sequence costs on this box
// (the per-call host cost of HISTORY.md §3.4): launch + sync round trips of tiny
// kernels with and without timing events, the same sequence as a graph, and
// waiting by polling mapped host memory instead of hipStreamSynchronize.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/probes/probe_launch tools/probes/probe_launch.hip
//   tools/probes/probe_launch [spin]      (spin: hipDeviceScheduleSpin before the context exists)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void tiny(double* out, double v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = v;
}

// the last kernel of a call: writes the result and then a flag (both to mapped
// host memory), system-scope release so the host sees the value before the flag
__global__ void tiny_flag(double* out, volatile unsigned* flag, unsigned seq, double v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = v;
    __threadfence_system();
    flag[0] = seq;
  }
}

// a walk-sized kernel: every wave busy for `ticks` of the 100 MHz constant clock
__global__ void busy(double* out, long long ticks) {
  const long long t0 = wall_clock64();
  double a = threadIdx.x;
  while (wall_clock64() - t0 < ticks) a = a * 1.0000001 + 1e-9;
  if (a == 12345.0) out[1] = a;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const bool spin = argc > 1 && std::strcmp(argv[1], "spin") == 0;
  if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  double* d;
  CK(hipMalloc(&d, 64));
  double* h;
  CK(hipHostMalloc((void**)&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
  double* m;
  CK(hipHostGetDevicePointer((void**)&m, h, 0));
  unsigned* hf;
  CK(hipHostMalloc((void**)&hf, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned* mf;
  CK(hipHostGetDevicePointer((void**)&mf, hf, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 2000;

  auto run = [&](const char* name, auto body) {
    for (int i = 0; i < 200; ++i) body(i);
    const double t0 = now_us();
    for (int i = 0; i < R; ++i) body(i);
    const double t = (now_us() - t0) / R;
    std::printf("%-58s %7.2f us per call%s\n", name, t, spin ? " (spin)" : "");
  };

  // the engine's sequence around a 500 us kernel on the whole chip: wall - event time
  // is what a call costs beyond its walk
  for (int poll = 0; poll < 2; ++poll) {
    double wall = 0, kern = 0;
    const int RB = 400;
    for (int i = 0; i < RB + 20; ++i) {
      const double t0 = now_us();
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(busy, dim3(2048), dim3(256), 0, s, d, 50000LL);
      CK(hipEventRecord(e1, s));
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
      if (poll) {
        hipError_t q;
        while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
        }
        CK(q);
      } else {
        CK(hipStreamSynchronize(s));
      }
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double t1 = now_us();
      if (i >= 20) wall += t1 - t0, kern += ms * 1000.0;
    }
    std::printf("500 us kernel + ev pair + 1 launch, %s: wall %.2f us, kernel %.2f us, outside %.2f us%s\n",
                poll ? "poll hipStreamQuery" : "hipStreamSynchronize", wall / RB, kern / RB, (wall - kern) / RB,
                spin ? " (spin)" : "");
  }
  // the same with the events carried by the launch itself (hipExtLaunchKernel:
  // the dispatch's own timestamps, no marker packets), waiting by sync or by
  // polling a flag the last kernel writes to mapped host memory
  unsigned fseq = 1000000;
  for (int mode = 0; mode < 3; ++mode) {
    double wall = 0, kern = 0;
    const int RB = 400;
    for (int i = 0; i < RB + 20; ++i) {
      const double t0 = now_us();
      if (mode == 2) {
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(busy, dim3(2048), dim3(256), 0, s, d, 50000LL);
        CK(hipEventRecord(e1, s));
      } else {
        hipExtLaunchKernelGGL(busy, dim3(2048), dim3(256), 0, s, e0, e1, 0, d, 50000LL);
      }
      ++fseq;
      hipLaunchKernelGGL(tiny_flag, dim3(1), dim3(64), 0, s, m, mf, fseq, 1.0);
      if (mode >= 1) {
        while (__atomic_load_n(hf, __ATOMIC_ACQUIRE) != fseq) {
        }
        CK(hipEventSynchronize(e1));
      } else {
        CK(hipStreamSynchronize(s));
      }
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double t1 = now_us();
      if (i >= 20) wall += t1 - t0, kern += ms * 1000.0;
    }
    const char* names[] = {"ext launch(events) + flag kernel, hipStreamSynchronize",
                           "ext launch(events) + flag kernel, poll flag",
                           "ev + launch + ev + flag kernel, poll flag"};
    std::printf("500 us kernel, %s: wall %.2f us, kernel %.2f us, outside %.2f us%s\n", names[mode], wall / RB,
                kern / RB, (wall - kern) / RB, spin ? " (spin)" : "");
  }
  run("ext launch(events) + 2 launches + sync + elapsed", [&](int) {
    hipExtLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, e0, e1, 0, d, 1.0);
    for (int k = 0; k < 2; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
  });
  run("launch + sync", [&](int) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipStreamSynchronize(s));
  });
  run("3 launches + sync", [&](int) {
    for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipStreamSynchronize(s));
  });
  run("3 launches (no sync) [host issue cost]", [&](int i) {
    for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    if (i % 64 == 63) CK(hipStreamSynchronize(s));
  });
  run("memset + ev + launch + ev + 2 launches + sync + elapsed", [&](int) {
    CK(hipMemsetAsync(d + 4, 0, 4, s));
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipEventRecord(e1, s));
    for (int k = 0; k < 2; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
  });
  run("ev + launch + ev + 2 launches + sync + elapsed [engine]", [&](int) {
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipEventRecord(e1, s));
    for (int k = 0; k < 2; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
  });
  run("ev + launch + ev + 2 launches + poll hipStreamQuery + elapsed", [&](int) {
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipEventRecord(e1, s));
    for (int k = 0; k < 2; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    hipError_t q;
    while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    CK(q);
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
  });
  run("launch + poll hipStreamQuery", [&](int) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    hipError_t q;
    while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    CK(q);
  });
  run("hipEventRecord alone [host cost]", [&](int i) {
    CK(hipEventRecord(e0, s));
    if (i % 64 == 63) CK(hipStreamSynchronize(s));
  });
  unsigned seq = 0;
  run("ev + launch + ev + launch + flag launch, poll flag + ev sync", [&](int) {
    ++seq;
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    CK(hipEventRecord(e1, s));
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    hipLaunchKernelGGL(tiny_flag, dim3(1), dim3(64), 0, s, m, mf, seq, 1.0);
    while (__atomic_load_n(hf, __ATOMIC_ACQUIRE) != seq) {
    }
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
  });
  run("launch + 2 launches + flag poll (no events)", [&](int) {
    ++seq;
    for (int k = 0; k < 2; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
    hipLaunchKernelGGL(tiny_flag, dim3(1), dim3(64), 0, s, m, mf, seq, 1.0);
    while (__atomic_load_n(hf, __ATOMIC_ACQUIRE) != seq) {
    }
  });

  // the engine's sequence as a graph (captured once, launched per call)
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  CK(hipEventRecord(e0, s));
  hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
  CK(hipEventRecord(e1, s));
  for (int k = 0; k < 2; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  run("graph(ev + launch + ev + 2 launches) + sync + elapsed", [&](int) {
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
  });
  hipGraph_t g2;
  hipGraphExec_t ge2;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, 1.0);
  CK(hipStreamEndCapture(s, &g2));
  CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
  run("graph(3 launches) + sync", [&](int) {
    CK(hipGraphLaunch(ge2, s));
    CK(hipStreamSynchronize(s));
  });
  std::printf("result %g\n", h[0]);
  return 0;
}
