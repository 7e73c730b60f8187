// Probe: can the fp64 matrix core add throughput beside the fp64 VALU on gfx950?
// Modes: 0 VALU fma chains only, 1 MFMA f64 16x16x4 chains only, 2 both in every
// wave (R MFMAs per 8 FMAs), 3 split by wave (even waves VALU, odd waves MFMA).
// Prints achieved fp64 TFLOP/s per mode. Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE, int R>
__global__ __launch_bounds__(256) void probe(double* out, int iters, double a, double b) {
  double x0 = threadIdx.x * 1e-9, x1 = x0 + 1e-9, x2 = x0 + 2e-9, x3 = x0 + 3e-9;
  double x4 = x0 + 4e-9, x5 = x0 + 5e-9, x6 = x0 + 6e-9, x7 = x0 + 7e-9;
  d4 m0 = {0, 0, 0, 0}, m1 = m0, m2 = m0, m3 = m0;
  const int wave = threadIdx.x >> 6;
  const bool do_valu = MODE == 0 || MODE == 2 || (MODE == 3 && (wave & 1) == 0);
  const bool do_mfma = MODE == 1 || MODE == 2 || (MODE == 3 && (wave & 1) == 1);
  for (int i = 0; i < iters; ++i) {
    if (do_valu) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b);
        x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
        x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b);
        x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
      }
    }
    if (do_mfma) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        m0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, m0, 0, 0, 0);
        m1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, m1, 0, 0, 0);
        m2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, m2, 0, 0, 0);
        m3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, m3, 0, 0, 0);
      }
    }
  }
  double s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  d4 m = m0 + m1 + m2 + m3;
  out[blockIdx.x * 256 + threadIdx.x] = s + m[0] + m[1] + m[2] + m[3];
}

template <int MODE, int R>
static void run(const char* name, double* d, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<MODE, R><<<blocks, 256>>>(d, 16, 0.999999, 1e-7);  // warm
  hipEventRecord(e0);
  probe<MODE, R><<<blocks, 256>>>(d, iters, 0.999999, 1e-7);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double waves = blocks * 4.0;
  double valu_waves = 0, mfma_waves = 0;
  if (MODE == 0) valu_waves = waves;
  if (MODE == 1) mfma_waves = waves;
  if (MODE == 2) valu_waves = mfma_waves = waves;
  if (MODE == 3) valu_waves = mfma_waves = waves / 2;
  const double fv = valu_waves * iters * 32.0 * 64 * 2;    // 32 FMAs x 64 lanes
  const double fm = mfma_waves * iters * 4.0 * R * 2048;   // 16x16x4 x 2 flops
  printf("%-28s %8.3f ms  valu %6.2f TF  mfma %6.2f TF  total %6.2f TF\n", name, ms,
         fv / ms * 1e-9, fm / ms * 1e-9, (fv + fm) / ms * 1e-9);
}

int main(int argc, char** argv) {
  int blocks = argc > 1 ? atoi(argv[1]) : 2048;
  int iters = argc > 2 ? atoi(argv[2]) : 20000;
  double* d;
  hipMalloc(&d, sizeof(double) * blocks * 256);
  run<0, 1>("valu only", d, blocks, iters);
  run<1, 1>("mfma only (R=1)", d, blocks, iters);
  run<1, 2>("mfma only (R=2)", d, blocks, iters);
  run<2, 1>("same wave R=1", d, blocks, iters);
  run<2, 2>("same wave R=2", d, blocks, iters);
  run<3, 1>("split waves R=1", d, blocks, iters);
  run<3, 2>("split waves R=2", d, blocks, iters);
  run<3, 4>("split waves R=4", d, blocks, iters);
  hipFree(d);
  return 0;
}
