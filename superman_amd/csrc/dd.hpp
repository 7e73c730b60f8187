// dd.hpp — double-double arithmetic (~106-bit significand) shared by the
// gfx950 quad-class walk (walk_dd.hip) and its host twin (quad.cpp), so both
// run the same operations in the same order and agree bit for bit.
//
// The reference's v2 `-q` mode computes Ryser in __float128
// (revised_perman/main.cpp:141-142 -> parallel_perman64<__float128,S>,
// cpu_algos.hpp:761-873; CPU only, ~3e6 Gray steps/s on 8 cores here).
// gfx950 has no quad arithmetic; a value hi + lo with |lo| <= ulp(hi)/2 held
// in two fp64 registers, formed with error-free transformations (two_sum,
// fma-based two_prod), carries ~106 bits at 8-17 fp64 VALU ops per operation.
// Built with -ffp-contract=off (host and device): the only fmas are the
// explicit ones below.
#pragma once

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define SUP_DD_FN __host__ __device__ __forceinline__
#else
#define SUP_DD_FN inline
#endif

namespace sup {

struct dd {
  double hi, lo;
};

// s + e = a + b exactly (Knuth); any magnitudes.
SUP_DD_FN dd dd_two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  const double e = (a - (s - bb)) + (b - bb);
  return dd{s, e};
}

// s + e = a + b exactly when |a| >= |b| (or a == 0) (Dekker).
SUP_DD_FN dd dd_fast_two_sum(double a, double b) {
  const double s = a + b;
  return dd{s, b - (s - a)};
}

// x + c, c a double (the walk's column add): 9 ops.
SUP_DD_FN dd dd_add_d(dd x, double c) {
  const dd s = dd_two_sum(x.hi, c);
  return dd_fast_two_sum(s.hi, s.lo + x.lo);
}

// a + b, both double-double ("accurate" sum: both parts two_sum'ed): 20 ops.
SUP_DD_FN dd dd_add(dd a, dd b) {
  dd s = dd_two_sum(a.hi, b.hi);
  const dd t = dd_two_sum(a.lo, b.lo);
  s = dd_fast_two_sum(s.hi, s.lo + t.hi);
  return dd_fast_two_sum(s.hi, s.lo + t.lo);
}

SUP_DD_FN dd dd_neg(dd a) { return dd{-a.hi, -a.lo}; }

// a * b (a.lo * b.lo dropped, below the format's precision): 7 ops.
SUP_DD_FN dd dd_mul(dd a, dd b) {
  const double p = a.hi * b.hi;
  double e = __builtin_fma(a.hi, b.hi, -p);
  e = __builtin_fma(a.hi, b.lo, e);
  e = __builtin_fma(a.lo, b.hi, e);
  return dd_fast_two_sum(p, e);
}

// a / d, d a double: quotient, exact remainder by fma, corrected quotient.
SUP_DD_FN dd dd_div_d(dd a, double d) {
  const double q1 = a.hi / d;
  const double p = q1 * d;
  const double e = __builtin_fma(q1, d, -p);
  const double rem = ((a.hi - p) - e) + a.lo;
  return dd_fast_two_sum(q1, rem / d);
}

}  // namespace sup
